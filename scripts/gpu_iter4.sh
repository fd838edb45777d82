set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu --maxfail=20 -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?; echo "exit=$rc" >> gpurun_out/t1.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --no-ptq --no-cpu > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err || exit 21
