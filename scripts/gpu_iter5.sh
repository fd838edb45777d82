#!/bin/bash
# Reduction-kernel variant sweep + PTQ phase breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/sweep_reduce.py > gpurun_out/sweep_reduce.log 2>&1 || { tail -30 gpurun_out/sweep_reduce.log; exit 10; }
grep -v "^ \|^{\|^}" gpurun_out/sweep_reduce.log
timeout -k 10 300 python -u scripts/ptq_breakdown.py > gpurun_out/ptq_breakdown2.json 2> gpurun_out/ptq_breakdown2.err || { tail -30 gpurun_out/ptq_breakdown2.err; exit 11; }
cat gpurun_out/ptq_breakdown2.json
