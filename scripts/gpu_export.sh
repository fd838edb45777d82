set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_export.py -q -m gpu -p no:cacheprovider > gpurun_out/t_export.log 2>&1; echo "exit=$?" >> gpurun_out/t_export.log
