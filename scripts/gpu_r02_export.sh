#!/bin/bash
# r02 export packers: parity (exhaustive 16-bit sweeps + the existing export tests), A/B of the
# native fast paths vs the emulated conversions (bench.py kernel table), VALU / traffic counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/export
timeout -k 10 300 python -u -m pytest tests/test_gpu_export_exhaustive.py tests/test_gpu_kernels.py -k export -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/export/tests.log 2>&1 || { tail -40 gpurun_out/export/tests.log; exit 10; }
tail -2 gpurun_out/export/tests.log
MTQ_AMD_GROUP_VARIANT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_golden.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/export/tests_gv2.log 2>&1 || { tail -40 gpurun_out/export/tests_gv2.log; exit 9; }
tail -1 gpurun_out/export/tests_gv2.log
for rep in 1 2; do for gv in 0 2; do
  MTQ_AMD_GROUP_VARIANT=$gv timeout -k 10 120 python -u bench.py --steps 100 --warmup 20 --no-cpu --no-ptq --no-c3 --no-suite > gpurun_out/export/head_gv${gv}_$rep.json 2>/dev/null || exit 8
  python -c "import json;d=json.load(open('gpurun_out/export/head_gv${gv}_$rep.json'));print('gv',$gv,d['value'],d['roofline']['frac'],d['roofline']['mean_launch_ms'])"
done; done
for nat in 1 0; do
  MTQ_AMD_EXPORT_NATIVE=$nat timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-ptq --no-c3 > gpurun_out/export/bench_native$nat.json 2> gpurun_out/export/bench_native$nat.err || { tail -20 gpurun_out/export/bench_native$nat.err; exit 11; }
done
python - <<'PY'
import json
for nat in (1, 0):
    d = json.load(open(f"gpurun_out/export/bench_native{nat}.json"))
    print("native", nat, {k: v for k, v in d["kernels"].items() if k.startswith("export")})
PY
cd /tmp
for k in export_fp8 export_nvfp4 export_mxfp4; do
  for nat in 1 0; do
    MTQ_AMD_EXPORT_NATIVE=$nat timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d "$R/gpurun_out/export/pmc_valu_${k}_n$nat" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 10 --kernel $k > "$R/gpurun_out/export/pmc_valu_${k}_n$nat.log" 2>&1 || exit 12
  done
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/export/pmc_fetch_${k}" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 10 --kernel $k > "$R/gpurun_out/export/pmc_fetch_${k}.log" 2>&1 || exit 13
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/export/pmc_write_${k}" -o pmc --output-format csv -- python3 "$R/scripts/prof_kernel.py" --iters 10 --kernel $k > "$R/gpurun_out/export/pmc_write_${k}.log" 2>&1 || exit 14
done
find "$R/gpurun_out/export" -name "*kernel_trace.csv" -delete
echo ok
