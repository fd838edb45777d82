#!/bin/bash
# AWQ tests, then C3 512 x 512 wall-clock and a 128-sample kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_awq_gemm.py tests/test_gpu_mtq.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/awq_tests.log 2>&1 || { tail -30 gpurun_out/awq_tests.log; exit 10; }
tail -1 gpurun_out/awq_tests.log
timeout -k 10 400 python -u scripts/ptq_llama.py --config INT4_AWQ_CFG --no-baseline > gpurun_out/c3_512.json 2> gpurun_out/c3_512.err || { tail -20 gpurun_out/c3_512.err; exit 11; }
tail -1 gpurun_out/c3_512.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c3" -o trace --output-format csv -- python3 "$R/scripts/ptq_llama.py" --config INT4_AWQ_CFG --no-baseline --samples 128 > "$R/gpurun_out/c3_128_prof.json" 2> "$R/gpurun_out/c3_128_prof.err" || exit 12
find "$R/gpurun_out/prof_c3" -name "*kernel_trace.csv" -delete
cat "$R/gpurun_out/c3_128_prof.json"
echo ok
