#!/bin/bash
# Sweep the fused QuantLinear launch variants (MTQ_AMD_QLINEAR_VARIANT), per-linear timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARS:-0 1 2 3 4 5}; do
  MTQ_AMD_QLINEAR_VARIANT=$v timeout -k 10 120 python -u scripts/bench_qlinear.py --per-linear-only --iters 30 > gpurun_out/ql_v$v.json 2> gpurun_out/ql_v$v.err || { tail -5 gpurun_out/ql_v$v.err; exit 10; }
  echo "v$v $(head -1 gpurun_out/ql_v$v.json)"
done
