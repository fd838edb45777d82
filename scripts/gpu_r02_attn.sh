#!/bin/bash
# fused flash attention with P qdq: GPU tests (one process), log under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py ${EXTRA_TESTS} -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_attn.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_attn.log | tail -60
exit $rc
