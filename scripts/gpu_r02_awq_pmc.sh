#!/bin/bash
# PMC passes (one counter group per run) on the AWQ search GEMM.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/awq_pmc
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$R/gpurun_out/awq_pmc/p$i" -o pmc --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" > "$R/gpurun_out/awq_pmc/p$i.log" 2>&1 || { tail -5 "$R/gpurun_out/awq_pmc/p$i.log"; exit 20; }
done
python3 "$R/scripts/pmc_csv_summary.py" "$R/gpurun_out/awq_pmc" awq_search_gemm > "$R/gpurun_out/awq_pmc/summary.txt" 2>&1 || true
cat "$R/gpurun_out/awq_pmc/summary.txt"
find "$R/gpurun_out/awq_pmc" -name "*kernel_trace.csv" -delete
