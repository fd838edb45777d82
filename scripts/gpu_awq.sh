#!/bin/bash
# AWQ-lite search GEMM: parity tests, then the one-process A/B bench (scripts/bench_awq_gemm.py).  Usage (on the GPU box): bash scripts/gpu_awq.sh [TAG]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-awq}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_awq_gemm.py tests/test_gpu_awq_b128.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 10; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 500 python -u scripts/bench_awq_gemm.py 8192 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 11; }
cat gpurun_out/${TAG}_bench.err
