#!/bin/bash
# Attention A/B of an environment switch, interleaved twice, plus the attention tests under each
# value.  Usage: bash scripts/gpu_attn_env_ab.sh TAG ENVVAR v1 v2 ...
set -o pipefail
TAG=$1; VAR=$2; shift 2
mkdir -p gpurun_out
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests_$v.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests_$v.log; exit 10; }
  echo "$VAR=$v $(tail -1 gpurun_out/${TAG}_tests_$v.log)"
done
for r in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python -u benchmarks/attention.py --iters 50 --out gpurun_out/${TAG}_${v}_r$r.json > gpurun_out/${TAG}_${v}_r$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_${v}_r$r.log; exit 11; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_r$r.json'));print('$VAR=$v round $r',{k:v['ms'] for k,v in d['modes'].items()})"
  done
done
