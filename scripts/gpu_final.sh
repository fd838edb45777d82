#!/bin/bash
# Round-end check on one MI355X: the whole -m gpu suite (one process), the default bench.py line,
# a rocprofv3 kernel trace + stats of the SAME bench.py command (the exact tree), and the PMC
# FETCH_SIZE / WRITE_SIZE passes of the bench's dominant kernel (roofline.traffic).
# Usage (on the GPU box): bash scripts/gpu_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${1:-final}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 10; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 11; }
tail -c 400 gpurun_out/${TAG}_bench.json
cd /tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_trace" -o trace --output-format csv -- python3 "$R/bench.py" > "$R/gpurun_out/${TAG}_bench_traced.json" 2> "$R/gpurun_out/${TAG}_trace.err" || exit 12
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_pmc_fetch" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 20 > "$R/gpurun_out/${TAG}_pmc_fetch.log" 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_pmc_write" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 20 > "$R/gpurun_out/${TAG}_pmc_write.log" 2>&1 || exit 14
cd "$R"
find gpurun_out/${TAG}_trace gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write -type f ! -name "*stats.csv" ! -name "*counter_collection.csv" -delete
echo ok
