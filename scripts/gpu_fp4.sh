#!/bin/bash
# Native FP4 converts: MX / NVFP4 parity, then bench lines native vs emulated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "mx or nvfp4 or fused or MX or export" > gpurun_out/fp4_tests.log 2>&1 || { tail -40 gpurun_out/fp4_tests.log; exit 10; }
tail -2 gpurun_out/fp4_tests.log
for v in 0 1; do
  MTQ_AMD_FP4_EMULATE=$v timeout -k 10 300 python bench.py --no-cpu --no-ptq --steps 20 > gpurun_out/fp4_bench_e$v.json 2> gpurun_out/fp4_bench_e$v.err || { tail -20 gpurun_out/fp4_bench_e$v.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/fp4_bench_e$v.json'));k=d['kernels'];print('emulate=$v', 'mxfp4', k['mxfp4_block32_dynamic'], 'nvfp4', k['nvfp4_block16_dynamic'], 'hist', k['histogram_2048_abs'])"
done
