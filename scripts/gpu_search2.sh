#!/bin/bash
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_search.py -q -x -p no:cacheprovider > gpurun_out/search_tests.log 2>&1 || { tail -30 gpurun_out/search_tests.log; exit 1; }
tail -2 gpurun_out/search_tests.log
timeout -k 10 600 python scripts/bench_search.py --cpu --out gpurun_out/search.json > /dev/null && cat gpurun_out/search.json
