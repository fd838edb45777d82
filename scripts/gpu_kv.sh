#!/bin/bash
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kv.py tests/test_gpu_export.py -q -x -p no:cacheprovider > gpurun_out/kv_tests.log 2>&1 || { tail -40 gpurun_out/kv_tests.log; exit 1; }
tail -2 gpurun_out/kv_tests.log
timeout -k 10 900 python scripts/ptq_llama.py --kv FP8_KV_CFG > gpurun_out/ptq_fp8_kv.json && cat gpurun_out/ptq_fp8_kv.json
timeout -k 10 900 python scripts/ptq_llama.py --config NVFP4_DEFAULT_CFG --kv NVFP4_KV_CFG --no-baseline > gpurun_out/ptq_nvfp4_kv.json && cat gpurun_out/ptq_nvfp4_kv.json
