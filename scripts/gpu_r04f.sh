#!/bin/bash
# r04 iteration f: MXFP4 export packer variants (scripts/exp), C2 (Llama-3-8B FP8) phase breakdown, C5 (Mixtral-8x7B FP8) per-batch split,
# C3 with the act-scale sharing (auto routing).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04f}
mkdir -p gpurun_out
bash scripts/exp/gpu_exp.sh ${TAG}x export || exit 40
timeout -k 10 300 python -u scripts/ptq_breakdown.py > gpurun_out/${TAG}_c2split.json 2> gpurun_out/${TAG}_c2split.err || { tail -20 gpurun_out/${TAG}_c2split.err; exit 41; }
cat gpurun_out/${TAG}_c2split.json
bash scripts/gpu_c5prof.sh ${TAG} || exit 42
bash scripts/gpu_c3ab.sh ${TAG}_c3 auto || exit 43
