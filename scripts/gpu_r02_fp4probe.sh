#!/bin/bash
# FP4 convert semantics probe + VALU/LDS PMC of the MX / NVFP4 / histogram kernels.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./scripts/probe_fp4_cvt > gpurun_out/fp4probe.txt 2>&1 || { cat gpurun_out/fp4probe.txt; exit 10; }
cat gpurun_out/fp4probe.txt
for k in mxfp4 nvfp4 hist; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d gpurun_out/r02b_${k}_pmc1 -o run -- python3 scripts/prof_kernel.py --kernel $k --iters 8 > gpurun_out/r02b_${k}_pmc1.log 2>&1 || exit 12
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS -d gpurun_out/r02b_${k}_pmc2 -o run -- python3 scripts/prof_kernel.py --kernel $k --iters 8 > gpurun_out/r02b_${k}_pmc2.log 2>&1 || exit 13
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02b_trace -o run -- python3 scripts/prof_kernel.py --kernel hist --iters 20 > gpurun_out/r02b_trace.log 2>&1 || exit 14
echo done
