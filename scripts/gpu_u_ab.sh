#!/bin/bash
# Kernel-table A/B of a vectors-per-lane switch: the kernel GPU tests, then bench.py (no CPU
# baseline, no PTQ) once per value.  Usage: bash scripts/gpu_u_ab.sh TAG ENVVAR v1 v2 ...
set -o pipefail
TAG=$1; VAR=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_reference_suite.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 10; }
tail -1 gpurun_out/${TAG}_tests.log
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu --no-ptq > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { tail -20 gpurun_out/${TAG}_$v.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$v.json'));print('$VAR=$v',{k:v['frac'] for k,v in d['kernels'].items() if 'dynamic' in k or 'static' in k})"
done
