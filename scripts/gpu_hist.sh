#!/bin/bash
# Histogram variants: parity (histc) tests, then the bench line per MTQ_AMD_HIST_VARIANT
# (0 = pattern U4 prefetch, 20 = U4, 21 = U2 prefetch, 22 = U8 prefetch; 10 = r01 division kernel).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "hist or Hist or calib or entropy or percentile" > gpurun_out/gh_tests.log 2>&1 || { tail -30 gpurun_out/gh_tests.log; exit 10; }
tail -2 gpurun_out/gh_tests.log
for v in 21 23 24 21 23 24; do
  MTQ_AMD_HIST_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu --no-ptq --steps 20 > gpurun_out/gh_bench_v$v.json 2> gpurun_out/gh_bench_v$v.err || { tail -20 gpurun_out/gh_bench_v$v.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/gh_bench_v$v.json'));print('v$v', d['kernels']['histogram_2048_abs'])"
done
