# GPU job: full -m gpu suite + smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu --maxfail=40 -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
echo "exit=$rc" >> gpurun_out/t1.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
echo "smoke_exit=$?" >> gpurun_out/smoke.log
