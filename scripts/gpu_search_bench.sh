#!/bin/bash
# Search-kernel throughput + rocprof trace/PMC + Llama-3-8B PTQ wall-clock with mse / awq_full.
set -uo pipefail
mkdir -p gpurun_out profiles/r01
export TMPDIR=/tmp
run() { "$@"; st=$?; if [ $st -ne 0 ]; then echo "FAILED($st): $*"; exit $st; fi; }
run timeout -k 10 600 python scripts/bench_search.py --cpu --out gpurun_out/search.json
run timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_search -o run -- python3 scripts/bench_search.py --iters 5
run timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/pmc_search -o run -- python3 scripts/bench_search.py --iters 2
run timeout -k 10 900 python benchmarks/ptq_llama.py --config NVFP4_W4A4_WEIGHT_MSE_FP8_SWEEP_CFG --no-baseline > gpurun_out/ptq_nvfp4_mse.json
run timeout -k 10 900 python benchmarks/ptq_llama.py --config INT8_DEFAULT_CFG --algorithm '{"method": "mse"}' --no-baseline > gpurun_out/ptq_int8_mse.json
run timeout -k 10 1200 python benchmarks/ptq_llama.py --config INT4_AWQ_CFG --samples 64 --algorithm '{"method": "awq_full", "alpha_step": 0.1}' --no-baseline > gpurun_out/ptq_int4_awq_full_64.json
cat gpurun_out/search.json; echo; cat gpurun_out/ptq_*.json
