#!/bin/bash
# GPU kernel tests for the reduction launches, then the variant sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_it6.log 2>&1 || { tail -40 gpurun_out/gpu_tests_it6.log; exit 10; }
tail -3 gpurun_out/gpu_tests_it6.log
timeout -k 10 400 python -u scripts/sweep_reduce.py > gpurun_out/sweep_reduce2.log 2>&1 || { tail -30 gpurun_out/sweep_reduce2.log; exit 11; }
grep -v "^ \|^{\|^}" gpurun_out/sweep_reduce2.log
