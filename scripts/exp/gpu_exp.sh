#!/bin/bash
# Experiment A/B runs on the GPU box (measurement only; scripts/exp/*.so built in the container).
# Usage: bash scripts/exp/gpu_exp.sh TAG [hist|awq|export]...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-exp}
shift
mkdir -p gpurun_out
for w in "$@"; do
  case $w in
    hist) timeout -k 10 300 python -u scripts/exp/bench_hist_exp.py > gpurun_out/${TAG}_hist.json 2> gpurun_out/${TAG}_hist.err || { tail -20 gpurun_out/${TAG}_hist.err; exit 21; }
          cat gpurun_out/${TAG}_hist.json ;;
    awq) timeout -k 10 400 python -u scripts/exp/bench_awq_exp.py > gpurun_out/${TAG}_awq.json 2> gpurun_out/${TAG}_awq.err || { tail -20 gpurun_out/${TAG}_awq.err; exit 22; }
          cat gpurun_out/${TAG}_awq.json ;;
    export) timeout -k 10 300 python -u scripts/exp/bench_export_exp.py > gpurun_out/${TAG}_export.json 2> gpurun_out/${TAG}_export.err || { tail -20 gpurun_out/${TAG}_export.err; exit 23; }
          cat gpurun_out/${TAG}_export.json ;;
  esac
done
