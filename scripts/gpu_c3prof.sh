#!/bin/bash
# C3 (Llama-3-8B INT4_AWQ_CFG, 512 x 512 calibration) wall-clock, then a rocprofv3 kernel trace +
# stats of the same run (GPU time per kernel; sum of kernel time vs wall = host / idle gaps).
# Usage (on the GPU box): bash scripts/gpu_c3prof.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${1:-c3prof}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/ptq_llama.py --config INT4_AWQ_CFG --no-baseline > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 31; }
cat gpurun_out/${TAG}_c3.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_trace" -o trace --output-format csv -- python3 "$R/benchmarks/ptq_llama.py" --config INT4_AWQ_CFG --no-baseline > "$R/gpurun_out/${TAG}_c3_traced.json" 2> "$R/gpurun_out/${TAG}_trace.err" || { tail -20 "$R/gpurun_out/${TAG}_trace.err"; exit 32; }
cd "$R"
python3 scripts/trace_gaps.py gpurun_out/${TAG}_trace/trace_kernel_trace.csv gpurun_out/${TAG}_gaps.json > /dev/null || true
find gpurun_out/${TAG}_trace -type f ! -name "*stats.csv" -delete
head -30 gpurun_out/${TAG}_trace/*/trace_kernel_stats.csv 2>/dev/null | cut -c1-200 || true
echo ok
