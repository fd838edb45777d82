set -o pipefail
cd "$GRAFT_REPO_ROOT"
rocminfo | grep -m2 -E "gfx9|Marketing" > gpurun_out/rocminfo.txt || true
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu --maxfail=40 -p no:cacheprovider > gpurun_out/t1.log 2>&1
echo "exit=$?" >> gpurun_out/t1.log
