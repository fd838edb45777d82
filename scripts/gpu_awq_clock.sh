#!/bin/bash
# MFMA duty and effective clock of AWQ search kernel variants (gate shape): one PMC pass each
# (SQ_VALU_MFMA_BUSY_CYCLES per SIMD vs GRBM_GUI_ACTIVE per XCD).  Usage: gpu_awq_clock.sh TAG "ENV1" "ENV2" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
TAG=$1
shift
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for envs in "$@"; do
  i=$((i+1))
  cd /tmp
  env $envs timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d "$R/gpurun_out/${TAG}_c$i" -o p --output-format csv -- python3 "$R/scripts/prof_awq_gemm.py" 8192 14336 4096 > "$R/gpurun_out/${TAG}_c$i.log" 2>&1 || exit 20
  cd "$R"
  python3 scripts/pmc_csv_summary.py gpurun_out/${TAG}_c$i awq_search_pp > gpurun_out/${TAG}_c$i.json || exit 21
  python3 - "$R/gpurun_out/${TAG}_c$i" "$envs" <<'PY'
import csv, json, sys
from pathlib import Path
d = json.load(open(sys.argv[1] + ".json"))
durs = []
for f in Path(sys.argv[1]).rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        if "awq_search_pp" in r["Kernel_Name"]:
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
ns = min(durs)
gui = d["GRBM_GUI_ACTIVE"]["mean"] / 8
mfma = d["SQ_VALU_MFMA_BUSY_CYCLES"]["mean"] / 1024
w = d["SQ_WAVE_CYCLES"]["mean"]
print(json.dumps({"env": sys.argv[2], "min_kernel_ms": ns / 1e6, "clock_ghz_est": round(gui / (sum(durs) / len(durs)), 3),
                  "mfma_duty": round(mfma / gui, 3), "wait_any": round(d["SQ_WAIT_ANY"]["mean"] / w, 3),
                  "wait_inst": round(d["SQ_WAIT_INST_ANY"]["mean"] / w, 3), "active": round(d["SQ_ACTIVE_INST_ANY"]["mean"] / w, 3)}))
PY
  find gpurun_out/${TAG}_c$i -type f ! -name "*.json" -delete
done
