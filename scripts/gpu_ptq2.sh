# GPU job: MoE golden test, Mixtral-8x7B FP8 PTQ (2 layers then full), Llama-3-8B INT4 AWQ (64 samples).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_mtq.py -q -m gpu -p no:cacheprovider > gpurun_out/t3.log 2>&1; echo "exit=$?" >> gpurun_out/t3.log
timeout -k 10 600 python scripts/ptq_llama.py --model mixtral-8x7b --layers 2 --samples 64 > gpurun_out/moe_small.json 2> gpurun_out/moe_small.err || exit 21
timeout -k 10 900 python scripts/ptq_llama.py --model mixtral-8x7b > gpurun_out/moe_full.json 2> gpurun_out/moe_full.err || exit 22
timeout -k 10 900 python scripts/ptq_llama.py --config INT4_AWQ_CFG --samples 64 > gpurun_out/awq_64.json 2> gpurun_out/awq_64.err || exit 23
