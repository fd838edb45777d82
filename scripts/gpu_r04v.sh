#!/bin/bash
# r04v: the AWQ W4R search-kernel experiment (variants 1, 2), the MXFP4 export store-kind
# experiment (variants 5-10), then the round-end check (scripts/gpu_final.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/exp/bench_awq_w4r.py 1,2 5 > gpurun_out/r04v_w4r.json 2> gpurun_out/r04v_w4r.err
rc=$?; tail -5 gpurun_out/r04v_w4r.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/exp/bench_export_exp.py 5,6,7,8,9,10 7 > gpurun_out/r04v_export.json 2> gpurun_out/r04v_export.err
rc=$?; cat gpurun_out/r04v_export.json; tail -3 gpurun_out/r04v_export.err; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_final.sh r04v
