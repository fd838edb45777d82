#!/bin/bash
# MXFP4 export packer on the bench input: per-launch trace (min / max / stddev), the effective clock
# from GRBM_GUI_ACTIVE over each dispatch, and FETCH_SIZE / WRITE_SIZE (separate passes).
# Usage (on the GPU box): bash scripts/gpu_export_pmc.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${1:-xp}
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_trace" -o trace --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel export_mxfp4 --iters 40 > "$R/gpurun_out/${TAG}_trace.log" 2>&1 || exit 20
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$R/gpurun_out/${TAG}_grbm" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel export_mxfp4 --iters 40 > "$R/gpurun_out/${TAG}_grbm.log" 2>&1 || exit 21
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_fetch" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel export_mxfp4 --iters 40 > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || exit 22
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_write" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel export_mxfp4 --iters 40 > "$R/gpurun_out/${TAG}_write.log" 2>&1 || exit 23
cd "$R"
find gpurun_out/${TAG}_trace gpurun_out/${TAG}_grbm gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write -type f ! -name "*stats.csv" ! -name "*counter_collection.csv" ! -name "*kernel_trace.csv" -delete
echo ok
