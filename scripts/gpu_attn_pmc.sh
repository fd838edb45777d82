#!/bin/bash
# Fused attention (bench shape): kernel trace + two PMC passes per P mode.
# Usage: bash scripts/gpu_attn_pmc.sh TAG [modes...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${1:-attn}
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in "$@"; do
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-trace -d "$R/gpurun_out/${TAG}_${m}_p1" -o p --output-format csv -- python3 "$R/scripts/prof_attn.py" $m 5 > "$R/gpurun_out/${TAG}_${m}_p1.log" 2>&1 || exit 31
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_LDS --kernel-trace -d "$R/gpurun_out/${TAG}_${m}_p2" -o p --output-format csv -- python3 "$R/scripts/prof_attn.py" $m 5 > "$R/gpurun_out/${TAG}_${m}_p2.log" 2>&1 || exit 32
  cd "$R"
  for p in p1 p2; do python3 scripts/pmc_csv_summary.py gpurun_out/${TAG}_${m}_$p attn_fwd > gpurun_out/${TAG}_${m}_$p.json || exit 33; done
  find gpurun_out/${TAG}_${m}_p1 gpurun_out/${TAG}_${m}_p2 -type f ! -name "*.json" -delete
done
