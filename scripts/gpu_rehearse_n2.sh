#!/bin/bash
# Rehearse bench.py's N>1 path (torchrun, 2 ranks) on a single GPU with the gloo backend.
set -euo pipefail
mkdir -p gpurun_out
export MTQ_AMD_DIST_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/rehearse_n2.log 2>&1
tail -c 3000 gpurun_out/rehearse_n2.log
