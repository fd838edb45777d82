#!/bin/bash
# The whole -m gpu suite (one process), then another GPU script -- unless the suite ended by a
# time limit, an abort or a crash (124 / 137 / 134 / 139 or a signal), in which case nothing
# further touches the GPU.  Usage (on the GPU box): bash scripts/gpu_tests_then.sh TAG [script args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-t}
shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_gpu_tests.log
echo "gpu tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $# -gt 0 ]; then bash "$@" || exit $?; fi
exit $rc
