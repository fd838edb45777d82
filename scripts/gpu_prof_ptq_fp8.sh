#!/bin/bash
# GPU job: kernel-level profile of the Llama-3-8B FP8 PTQ run (GEMM vs quantizer vs other kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ptq_fp8" -o run --output-format csv -- python3 "$R/benchmarks/ptq_llama.py" --no-baseline > "$R/gpurun_out/prof_ptq_fp8.json" 2> "$R/gpurun_out/prof_ptq_fp8.err" || exit 21
find "$R/gpurun_out/prof_ptq_fp8" -type f ! -name "*stats.csv" -delete
find "$R/gpurun_out/prof_ptq_fp8" -name "*stats.csv"
