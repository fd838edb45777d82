#!/bin/bash
# decode QuantLinear kernel: parity tests, then rocprof kernel durations per Llama shape for the
# default (LDS-DMA) kernel and the register-staged stream kernel
set -o pipefail
mkdir -p gpurun_out/ql
export PYTHONPATH=$PWD:$PWD/tensorrt-model-optimizer_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qlinear.py > gpurun_out/ql/tests.log 2>&1 || { tail -30 gpurun_out/ql/tests.log; exit 1; }
tail -2 gpurun_out/ql/tests.log
bash scripts/gpu_r02_qlprof.sh "$@"
