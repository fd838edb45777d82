#!/bin/bash
# r02 first call: full GPU suite, then LDS/VALU PMC passes on the histogram kernel.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r02a_tests.log 2>&1 || { tail -30 gpurun_out/r02a_tests.log; exit 10; }
tail -3 gpurun_out/r02a_tests.log
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/r02a_hist_trace -o run -- python3 scripts/prof_kernel.py --kernel hist --iters 20 > gpurun_out/r02a_hist_trace.log 2>&1 || exit 11
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r02a_hist_pmc1 -o run -- python3 scripts/prof_kernel.py --kernel hist --iters 8 > gpurun_out/r02a_hist_pmc1.log 2>&1 || exit 12
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r02a_fp8_pmc1 -o run -- python3 scripts/prof_kernel.py --kernel fp8_block128 --iters 8 > gpurun_out/r02a_fp8_pmc1.log 2>&1 || exit 13
echo done
