#!/bin/bash
# GPU check of the calibration-search kernels (MSE sweeps, AWQ-clip).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_search.py -q -x -p no:cacheprovider > gpurun_out/search_tests.log 2>&1
st=$?
tail -40 gpurun_out/search_tests.log
exit $st
