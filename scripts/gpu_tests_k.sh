#!/bin/bash
# Run a subset of the GPU tests: scripts/gpu_tests_k.sh "<pytest -k expr or file list>"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest $1 -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_k.log 2>&1
rc=$?
tail -40 gpurun_out/tests_k.log
exit $rc
