#!/bin/bash
# AWQ search GEMM (gate shape): counter list + L2 hit / TA counters for the default pp kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${1:-awq}
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/${TAG}_counters.txt" 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/gpurun_out/${TAG}_l2" -o p --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 14336 4096 > "$R/gpurun_out/${TAG}_l2.log" 2>&1 || exit 22
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum --kernel-trace -d "$R/gpurun_out/${TAG}_ta" -o p --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 14336 4096 > "$R/gpurun_out/${TAG}_ta.log" 2>&1 || echo "ta pass failed"
cd "$R"
for p in l2 ta; do python3 scripts/pmc_csv_summary.py gpurun_out/${TAG}_$p awq_search_pp > gpurun_out/${TAG}_$p.json || true; done
find gpurun_out/${TAG}_l2 gpurun_out/${TAG}_ta -type f ! -name "*.json" -delete 2>/dev/null
cat gpurun_out/${TAG}_l2.json gpurun_out/${TAG}_ta.json
grep -c "" gpurun_out/${TAG}_counters.txt
