#!/bin/bash
# AWQ search GEMM: parity tests (both modes), then the per-linear bench (fused vs unfused).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for mode in 0 1; do
  MTQ_AMD_AWQ_GEMM_MODE=$mode timeout -k 10 300 python -u -m pytest tests/test_gpu_awq_gemm.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/awq_tests_m$mode.log 2>&1 || { tail -40 gpurun_out/awq_tests_m$mode.log; exit 10; }
  tail -1 gpurun_out/awq_tests_m$mode.log
done
for mode in 0 1; do
  MTQ_AMD_AWQ_GEMM_MODE=$mode timeout -k 10 300 python -u scripts/bench_awq_gemm.py ${M:-8192} > gpurun_out/awq_bench_m$mode.json 2> gpurun_out/awq_bench_m$mode.err || { tail -20 gpurun_out/awq_bench_m$mode.err; exit 11; }
  echo "mode $mode"; grep -v amdgpu.ids gpurun_out/awq_bench_m$mode.err
done
MTQ_AMD_AWQ_GEMM_PROBE=1 timeout -k 10 300 python -u scripts/bench_awq_gemm.py ${M:-8192} > gpurun_out/awq_bench_p1.json 2> gpurun_out/awq_bench_p1.err || exit 12
echo "probe 1 (mode 0)"; grep -o "'search_gemm_tflops': [0-9.]*" gpurun_out/awq_bench_p1.err
