#!/bin/bash
# r02 round check: bench.py (default: kernels + FP8 PTQ + C3 AWQ PTQ + CPU baseline), rocprofv3
# kernel stats of the bench kernels, PMC traffic passes, AWQ search bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r02b}
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 11; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python -u scripts/bench_awq_gemm.py > gpurun_out/awq_bench_$TAG.json 2> gpurun_out/awq_bench_$TAG.err || { tail -20 gpurun_out/awq_bench_$TAG.err; exit 12; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o trace --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu --no-ptq > "$R/gpurun_out/bench_prof_$TAG.json" 2> "$R/gpurun_out/prof_$TAG.err" || exit 13
find "$R/gpurun_out/prof_$TAG" -name "*kernel_trace.csv" -delete
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch_$TAG" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 20 > "$R/gpurun_out/pmc_fetch_$TAG.log" 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write_$TAG" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 20 > "$R/gpurun_out/pmc_write_$TAG.log" 2>&1 || exit 15
echo ok
