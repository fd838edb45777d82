#!/bin/bash
# Full GPU test suite (one pytest process), then the KV/search diagnostics.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
st=$?
tail -40 gpurun_out/gpu_tests.log
exit $st
