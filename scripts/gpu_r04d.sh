#!/bin/bash
# r04 iteration d: the ring-buffered AWQ experiment (v50/v53 beside v31/v33), PMC passes of the
# product AWQ search kernel vs hipBLASLt on gate_proj (FETCH after the r04 unit raster), then the
# bench.py --gpus 2 self-launch rehearsal (two gloo ranks sharing the card).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04d}
mkdir -p gpurun_out
bash scripts/exp/gpu_exp.sh ${TAG}x awq || exit 51
bash scripts/gpu_awq_pmc.sh ${TAG}_awq || exit 52
MTQ_AMD_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --no-suite --no-cpu --no-ptq > gpurun_out/${TAG}_n2.json 2> gpurun_out/${TAG}_n2.err || { tail -20 gpurun_out/${TAG}_n2.err; exit 53; }
cat gpurun_out/${TAG}_n2.json
