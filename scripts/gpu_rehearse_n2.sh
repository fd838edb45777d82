#!/bin/bash
# Rehearse bench.py's N>1 path (torchrun, 2 ranks) on a single GPU with the gloo backend: the
# headline kernel per rank, C2 data-parallel with the packed amax exchange, and C4 through the
# layer-sharded pipeline (40 Llama-3-70B layers per rank, P2P hand-off + packed all_reduce(MAX)).
# C3 is left out (two AWQ weight caches sized for a whole GPU each would not share one card).
# Usage (on the GPU box): bash scripts/gpu_rehearse_n2.sh TAG
set -euo pipefail
TAG=${1:-n2}
mkdir -p gpurun_out
export MTQ_AMD_DIST_BACKEND=gloo
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-c3 --no-suite \
  > gpurun_out/${TAG}_n2.json 2> gpurun_out/${TAG}_n2.err
tail -c 3000 gpurun_out/${TAG}_n2.json
