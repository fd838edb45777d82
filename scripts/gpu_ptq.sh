# GPU job: golden tests (quick) then PTQ e2e at 2 layers and full 32 layers.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_golden.py -q -m gpu -p no:cacheprovider > gpurun_out/t2.log 2>&1; echo "exit=$?" >> gpurun_out/t2.log
timeout -k 10 600 python benchmarks/ptq_llama.py --layers 2 --samples 64 > gpurun_out/ptq_small.json 2> gpurun_out/ptq_small.err || exit 21
timeout -k 10 900 python benchmarks/ptq_llama.py > gpurun_out/ptq_full.json 2> gpurun_out/ptq_full.err || exit 22
