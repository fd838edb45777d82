#!/bin/bash
# AWQ search GEMM (gate_proj shape, 8192 tokens, 11 alphas): rocprofv3 kernel stats + PMC passes
# (one counter group per run, each under its own time limit).  Usage: bash scripts/gpu_awq_pmc.sh TAG [N K]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=${1:-awq}
N=${2:-14336}
K=${3:-4096}
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_trace" -o t --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 $N $K > "$R/gpurun_out/${TAG}_trace.log" 2>&1 || exit 21
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d "$R/gpurun_out/${TAG}_pmc1" -o p --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 $N $K > "$R/gpurun_out/${TAG}_pmc1.log" 2>&1 || exit 22
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$R/gpurun_out/${TAG}_pmc2" -o p --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 $N $K > "$R/gpurun_out/${TAG}_pmc2.log" 2>&1 || exit 23
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_pmc3" -o p --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 $N $K > "$R/gpurun_out/${TAG}_pmc3.log" 2>&1 || exit 24
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/gpurun_out/${TAG}_pmc4" -o p --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 $N $K > "$R/gpurun_out/${TAG}_pmc4.log" 2>&1 || exit 24
cd "$R"
for p in pmc1 pmc2 pmc3 pmc4; do python3 scripts/pmc_csv_summary.py gpurun_out/${TAG}_$p ${KSUB:-awq_search_w4} > gpurun_out/${TAG}_$p.json || exit 25; done
find gpurun_out/${TAG}_trace gpurun_out/${TAG}_pmc1 gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_pmc3 gpurun_out/${TAG}_pmc4 -type f ! -name "*stats.csv" ! -name "*.json" -delete
cat gpurun_out/${TAG}_pmc1.json gpurun_out/${TAG}_pmc2.json gpurun_out/${TAG}_pmc3.json gpurun_out/${TAG}_pmc4.json
find gpurun_out/${TAG}_trace -name "*kernel_stats.csv" -exec cat {} \;
# the hipBLASLt GEMMs of the same batch: clock and MFMA duty for comparison
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d "$R/gpurun_out/${TAG}_blt1" -o p --output-format csv -- python3 "$R/scripts/prof_hipblaslt.py" 8192 $N $K > "$R/gpurun_out/${TAG}_blt1.log" 2>&1 || exit 26
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$R/gpurun_out/${TAG}_blt2" -o p --output-format csv -- python3 "$R/scripts/prof_hipblaslt.py" 8192 $N $K > "$R/gpurun_out/${TAG}_blt2.log" 2>&1 || exit 27
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_blt3" -o p --output-format csv -- python3 "$R/scripts/prof_hipblaslt.py" 8192 $N $K > "$R/gpurun_out/${TAG}_blt3.log" 2>&1 || exit 27
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/gpurun_out/${TAG}_blt4" -o p --output-format csv -- python3 "$R/scripts/prof_hipblaslt.py" 8192 $N $K > "$R/gpurun_out/${TAG}_blt4.log" 2>&1 || exit 27
cd "$R"
for p in blt1 blt2 blt3 blt4; do python3 scripts/pmc_csv_summary.py gpurun_out/${TAG}_$p Cijk > gpurun_out/${TAG}_$p.json || exit 28; done
find gpurun_out/${TAG}_blt1 gpurun_out/${TAG}_blt2 gpurun_out/${TAG}_blt3 gpurun_out/${TAG}_blt4 -type f ! -name "*.json" -delete
cat gpurun_out/${TAG}_blt1.json gpurun_out/${TAG}_blt2.json gpurun_out/${TAG}_blt3.json gpurun_out/${TAG}_blt4.json
