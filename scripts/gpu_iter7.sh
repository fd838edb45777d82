#!/bin/bash
# GPU tests, histogram variant sweep, PTQ breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_it7.log 2>&1 || { tail -40 gpurun_out/gpu_tests_it7.log; exit 10; }
tail -2 gpurun_out/gpu_tests_it7.log
timeout -k 10 300 python -u scripts/sweep_reduce.py hist > gpurun_out/sweep_hist.log 2>&1 || { tail -30 gpurun_out/sweep_hist.log; exit 11; }
grep -v "^ \|^{\|^}" gpurun_out/sweep_hist.log
timeout -k 10 300 python -u scripts/ptq_breakdown.py > gpurun_out/ptq_breakdown3.json 2> gpurun_out/ptq_breakdown3.err || { tail -30 gpurun_out/ptq_breakdown3.err; exit 12; }
cat gpurun_out/ptq_breakdown3.json
