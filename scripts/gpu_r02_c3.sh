#!/bin/bash
# GPU tests, then C3 (Llama-3-8B INT4_AWQ_CFG, 512 x 512) wall-clock and a 128-sample kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 10; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u scripts/ptq_llama.py --config INT4_AWQ_CFG --no-baseline > gpurun_out/c3_512.json 2> gpurun_out/c3_512.err || { tail -20 gpurun_out/c3_512.err; exit 11; }
tail -1 gpurun_out/c3_512.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c3" -o trace --output-format csv -- python3 "$R/scripts/ptq_llama.py" --config INT4_AWQ_CFG --no-baseline --samples 128 > "$R/gpurun_out/c3_128_prof.json" 2> "$R/gpurun_out/c3_128_prof.err" || exit 12
echo ok
