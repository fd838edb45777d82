#!/bin/bash
# C5 (Mixtral-8x7B FP8, 512 x 512) wall-clock split per batch (scripts/prof_c5_batches.py).
# Usage (on the GPU box): bash scripts/gpu_c5prof.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c5p}
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/prof_c5_batches.py > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 41; }
cat gpurun_out/${TAG}_c5.json
