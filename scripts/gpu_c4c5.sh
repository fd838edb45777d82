#!/bin/bash
# Full-size C5 (Mixtral-8x7B FP8) and C4 (Llama-3-70B MXFP4 W+A) PTQ wall-clock beside the bf16
# forward, r03 kernels.  Usage: bash scripts/gpu_c4c5.sh TAG [c5|c4|c4n2]...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c45}
shift
mkdir -p gpurun_out
for what in "$@"; do
  case $what in
    c5) timeout -k 10 900 python -u benchmarks/ptq_llama.py --model mixtral-8x7b > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 21; }
        cat gpurun_out/${TAG}_c5.json ;;
    c4) timeout -k 10 900 python -u scripts/ptq_sharded.py > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || { tail -20 gpurun_out/${TAG}_c4.err; exit 22; }
        cat gpurun_out/${TAG}_c4.json ;;
    c4n2) timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 scripts/ptq_sharded.py --one-gpu --backend gloo > gpurun_out/${TAG}_c4n2.json 2> gpurun_out/${TAG}_c4n2.err || { tail -30 gpurun_out/${TAG}_c4n2.err; exit 23; }
        cat gpurun_out/${TAG}_c4n2.json ;;
  esac
done
