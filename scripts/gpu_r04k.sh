#!/bin/bash
# r04 iteration k: the calibration-bookkeeping kernels (fill / fold / check / MoE row mask) --
# their GPU tests and the calibration suites that run through them, then C2 (kernel diff + the
# ptq_llama wall-clock) and the C5 per-batch split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04k}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_amax_bookkeeping.py tests/test_gpu_mtq.py tests/test_gpu_moe_nvfp4_once.py tests/test_gpu_dp.py tests/test_gpu_dp_devices.py tests/test_gpu_reference_suite.py tests/test_gpu_awq_b128.py tests/test_gpu_awq_gemm.py tests/test_gpu_c4.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 10; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u scripts/prof_c2_diff.py 6 > gpurun_out/${TAG}_c2diff.txt 2> gpurun_out/${TAG}_c2diff.err || { tail -20 gpurun_out/${TAG}_c2diff.err; exit 11; }
head -8 gpurun_out/${TAG}_c2diff.txt
timeout -k 10 300 python -u scripts/ptq_llama.py > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || { tail -20 gpurun_out/${TAG}_c2.err; exit 12; }
tail -1 gpurun_out/${TAG}_c2.json
bash scripts/gpu_c5prof.sh ${TAG} || exit 13
