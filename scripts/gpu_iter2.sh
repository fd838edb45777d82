# GPU job: -m gpu suite, C4 sharded MXFP4 PTQ of Llama-3-70B dims on one GPU (stage = all layers).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu --maxfail=20 -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/t1.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/ptq_sharded.py --layers 4 --samples 64 > gpurun_out/c4_small.json 2> gpurun_out/c4_small.err || exit 21
timeout -k 10 1200 python scripts/ptq_sharded.py > gpurun_out/c4_full.json 2> gpurun_out/c4_full.err || exit 22
