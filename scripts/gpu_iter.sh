#!/bin/bash
# Iteration check on one MI355X: the attention + export GPU tests, the attention bench and the
# kernel table of bench.py (no CPU baseline, no PTQ).  Usage: bash scripts/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_export.py tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 10; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u benchmarks/attention.py --iters 50 --out gpurun_out/${TAG}_attn.json > gpurun_out/${TAG}_attn.log 2>&1 || { tail -20 gpurun_out/${TAG}_attn.log; exit 11; }
tail -5 gpurun_out/${TAG}_attn.log
timeout -k 10 300 python -u bench.py --no-cpu --no-ptq > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 12; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['roofline']['frac']);[print(' ',k,v['frac'],v['ms']) for k,v in d['kernels'].items()]"
