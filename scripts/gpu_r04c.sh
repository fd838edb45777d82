#!/bin/bash
# r04 iteration c: kernel / golden / histogram / export GPU tests, export + histogram rocprof
# traces and PMC, the bench.py kernel table, then the C5 per-batch profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04c}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_hist_ref.py tests/test_gpu_export_exhaustive.py tests/test_gpu_export.py tests/test_gpu_compress.py tests/test_gpu_moe_nvfp4_once.py tests/test_gpu_dp_devices.py tests/test_gpu_qlinear.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 10; }
tail -1 gpurun_out/${TAG}_tests.log
bash scripts/gpu_prof_export.sh ${TAG}_pexp || exit 11
timeout -k 10 300 python -u bench.py --no-ptq --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 12; }
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['frac']);[print(k, v['frac']) for k, v in d['kernels'].items()]"
bash scripts/gpu_c5prof.sh ${TAG}_c5 || exit 13
