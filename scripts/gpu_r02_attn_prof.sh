#!/bin/bash
# attention kernel: error stats vs the reference goldens, bench, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/attn
timeout -k 10 300 python -u scripts/attn_err_stats.py > gpurun_out/attn/err_stats.json 2> gpurun_out/attn/err.log || { tail -20 gpurun_out/attn/err.log; exit 11; }
timeout -k 10 300 python -u scripts/bench_attention.py --out gpurun_out/attn/bench.json > gpurun_out/attn/bench.log 2>&1 || { tail -20 gpurun_out/attn/bench.log; exit 12; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/attn/prof" -o trace --output-format csv -- python3 "$R/scripts/bench_attention.py" --iters 10 > "$R/gpurun_out/attn/prof.log" 2>&1 || exit 13
find "$R/gpurun_out/attn/prof" -name "*kernel_trace.csv" -delete
cat "$R/gpurun_out/attn/err_stats.json" "$R/gpurun_out/attn/bench.json"
