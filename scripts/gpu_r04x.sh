#!/bin/bash
# r04x: MXFP4 export packer at U = 4 in the product -- export / compress parity tests, the packer
# A/B (product vs variant 11), then the FP8 per-tensor / NVFP4 packers at U = 4 vs 2, then the
# wide-linear AWQ search orderings (scripts/exp/bench_awq_mall.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "export or compress or mx or golden" > gpurun_out/r04x_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04x_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/exp/bench_export_exp.py 11 7 > gpurun_out/r04x_export.json 2> gpurun_out/r04x_export.err
rc=$?; cat gpurun_out/r04x_export.json; tail -3 gpurun_out/r04x_export.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/exp/bench_export_exp2.py 7 > gpurun_out/r04x_export2.json 2> gpurun_out/r04x_export2.err
rc=$?; cat gpurun_out/r04x_export2.json; tail -3 gpurun_out/r04x_export2.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp/bench_awq_mall.py 5 > gpurun_out/r04x_mall.json 2> gpurun_out/r04x_mall.err
rc=$?; tail -5 gpurun_out/r04x_mall.err; exit $rc
