#!/bin/bash
# Attention stage-size A/B (MTQ_AMD_ATTN_STAGE 64 vs 32, the 32-key stage runs 3 waves / SIMD for
# 16-bit none / FP8 P), interleaved, plus the attention tests under the 32-key stage.
# Usage: bash scripts/gpu_attn_ab.sh TAG
set -o pipefail
TAG=${1:-attnab}
mkdir -p gpurun_out
MTQ_AMD_ATTN_STAGE=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests32.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests32.log; exit 10; }
tail -1 gpurun_out/${TAG}_tests32.log
for r in 1 2; do
  for st in 64 32; do
    MTQ_AMD_ATTN_STAGE=$st timeout -k 10 200 python -u benchmarks/attention.py --iters 50 --out gpurun_out/${TAG}_s${st}_r$r.json > gpurun_out/${TAG}_s${st}_r$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_s${st}_r$r.log; exit 11; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_s${st}_r$r.json'));print('stage $st round $r',{k:v['ms'] for k,v in d['modes'].items()})"
  done
done
