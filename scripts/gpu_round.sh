#!/bin/bash
# Round check: full GPU tests, bench.py (default), rocprofv3 kernel stats, PMC traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 10; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 11; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o trace --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu --no-ptq > "$R/gpurun_out/bench_prof_$TAG.json" 2> "$R/gpurun_out/prof_$TAG.err" || exit 12
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch_$TAG" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 20 > "$R/gpurun_out/pmc_fetch_$TAG.log" 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write_$TAG" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 20 > "$R/gpurun_out/pmc_write_$TAG.log" 2>&1 || exit 14
cat "$R/gpurun_out/bench_$TAG.json"
echo ok
