#!/bin/bash
# r04 iteration: AWQ parity tests + search bench, histogram experiments, kernel-suite GPU tests,
# then C3 wall-clock.  Usage (on the GPU box): bash scripts/gpu_r04b.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04b}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_awq_gemm.py tests/test_gpu_awq_b128.py tests/test_gpu_kernels.py tests/test_gpu_hist_ref.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 10; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 500 python -u scripts/bench_awq_gemm.py 8192 5 > gpurun_out/${TAG}_awqbench.json 2> gpurun_out/${TAG}_awqbench.err || { tail -20 gpurun_out/${TAG}_awqbench.err; exit 11; }
cat gpurun_out/${TAG}_awqbench.err
timeout -k 10 300 python -u scripts/exp/bench_hist_exp.py > gpurun_out/${TAG}_hist.json 2> gpurun_out/${TAG}_hist.err || { tail -20 gpurun_out/${TAG}_hist.err; exit 12; }
cat gpurun_out/${TAG}_hist.json
timeout -k 10 300 python -u scripts/ptq_llama.py --config INT4_AWQ_CFG --no-baseline > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 13; }
cat gpurun_out/${TAG}_c3.json
