# GPU job: full -m gpu suite, amax variant sweep, AWQ + FP8 PTQ timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu --maxfail=20 -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/t1.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/sweep_amax.py > gpurun_out/sweep_amax.json 2> gpurun_out/sweep_amax.err || exit 21
timeout -k 10 900 python scripts/ptq_llama.py --config INT4_AWQ_CFG --samples 64 > gpurun_out/awq_64.json 2> gpurun_out/awq_64.err || exit 22
timeout -k 10 900 python scripts/ptq_llama.py > gpurun_out/ptq_fp8.json 2> gpurun_out/ptq_fp8.err || exit 23
