#!/bin/bash
# attention kernel A/B: stage 32 vs 64 keys per barrier pair, + LDS counters of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/attn
for st in 32 64; do
  MTQ_AMD_ATTN_STAGE=$st timeout -k 10 300 python scripts/bench_attention.py --iters 30 > gpurun_out/attn/ab_$st.json 2>&1 || exit 11
  echo "stage $st"; python -c "import json;d=json.load(open('gpurun_out/attn/ab_$st.json'));print({k:v['ms'] for k,v in d['modes'].items()})"
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY --kernel-trace -d "$R/gpurun_out/attn/pmc" -o pmc --output-format csv -- python3 "$R/scripts/bench_attention.py" --iters 3 > "$R/gpurun_out/attn/pmc.log" 2>&1 || exit 12
python3 "$R/scripts/pmc_csv_summary.py" "$R/gpurun_out/attn/pmc" Li128ELi0ELi32 2>&1 | head -40 || true
