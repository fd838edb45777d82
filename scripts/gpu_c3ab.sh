#!/bin/bash
# C3 (Llama-3-8B INT4_AWQ_CFG, 512 x 512 calibration) wall-clock with the AWQ search routed
# through each path: MTQ_AMD_AWQ_FUSED=auto (fused kernel for N <= 2048, hipBLASLt batched above),
# always (fused kernel everywhere).  Usage: bash scripts/gpu_c3ab.sh TAG [auto|always|never]...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3ab}
shift
mkdir -p gpurun_out
for m in "$@"; do
  MTQ_AMD_AWQ_FUSED=$m timeout -k 10 300 python -u benchmarks/ptq_llama.py --config INT4_AWQ_CFG --no-baseline > gpurun_out/${TAG}_$m.json 2> gpurun_out/${TAG}_$m.err || { tail -20 gpurun_out/${TAG}_$m.err; exit 31; }
  echo "$m $(cat gpurun_out/${TAG}_$m.json)"
done
