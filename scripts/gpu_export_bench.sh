#!/bin/bash
# Export packing kernels: parity tests, then the bench kernel table at MTQ_AMD_EXPORT_U = 1, 2, 4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_export.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "export" > gpurun_out/gx_tests.log 2>&1 || { tail -30 gpurun_out/gx_tests.log; exit 10; }
tail -2 gpurun_out/gx_tests.log
for u in 1 2 4; do
  MTQ_AMD_EXPORT_U=$u timeout -k 10 300 python bench.py --no-cpu --no-ptq > gpurun_out/gx_bench_u$u.json 2> gpurun_out/gx_bench_u$u.err || { tail -20 gpurun_out/gx_bench_u$u.err; exit 11; }
  echo "U=$u"
  python -c "import json;d=json.load(open('gpurun_out/gx_bench_u$u.json'));[print(' ',k,v) for k,v in d['kernels'].items() if 'export' in k]"
done
