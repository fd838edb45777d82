#!/bin/bash
# Export packers + histogram on the bench input: rocprofv3 kernel trace with per-dispatch stats
# (min / max / stddev of every launch), then PMC passes for the MXFP4 packer (effective clock from
# GRBM_GUI_ACTIVE, VALU / wait counters, FETCH and WRITE bytes).  Usage: bash scripts/gpu_prof_export.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${1:-pexp}
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
for k in export_mxfp4 export_nvfp4 export_int4 hist; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_trace_$k" -o trace --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel $k --iters 50 > "$R/gpurun_out/${TAG}_trace_$k.log" 2>&1 || exit 31
done
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d "$R/gpurun_out/${TAG}_pmc1" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel export_mxfp4 --iters 20 > "$R/gpurun_out/${TAG}_pmc1.log" 2>&1 || exit 32
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_pmc2" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel export_mxfp4 --iters 20 > "$R/gpurun_out/${TAG}_pmc2.log" 2>&1 || exit 33
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --kernel-trace -d "$R/gpurun_out/${TAG}_pmc3" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --kernel export_mxfp4 --iters 20 > "$R/gpurun_out/${TAG}_pmc3.log" 2>&1 || exit 34
cd "$R"
find gpurun_out/${TAG}_* -type f -name "*.csv" ! -name "*stats.csv" ! -name "*counter_collection.csv" -delete
ls -R gpurun_out/${TAG}_* | head -40
