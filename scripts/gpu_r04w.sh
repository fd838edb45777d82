#!/bin/bash
# r04w: MXFP4 export packer with the LDS-gathered scale line in the product -- the export / compress
# parity tests, then the packer A/B (product vs variants 8, 11, 12, 13); then the AWQ search GEMMs
# under TunableOp's solution vs the default heuristic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "export or compress or mx or golden" > gpurun_out/r04w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04w_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/exp/bench_export_exp.py 8,11,12,13 7 > gpurun_out/r04w_export.json 2> gpurun_out/r04w_export.err
rc=$?; cat gpurun_out/r04w_export.json; tail -3 gpurun_out/r04w_export.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/exp/bench_tunableop.py 5 > gpurun_out/r04w_tunableop.json 2> gpurun_out/r04w_tunableop.err
rc=$?; tail -5 gpurun_out/r04w_tunableop.err; exit $rc
