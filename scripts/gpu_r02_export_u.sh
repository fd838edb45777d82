#!/bin/bash
# Export packers: vectors per lane (MTQ_AMD_EXPORT_U = 1, 2, 4) now that they are not VALU-bound.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/export_u
for rep in 1 2; do for u in 2 1 4; do
  MTQ_AMD_EXPORT_U=$u timeout -k 10 120 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-ptq --no-c3 > gpurun_out/export_u/u${u}_$rep.json 2>/dev/null || exit 8
  python -c "import json;d=json.load(open('gpurun_out/export_u/u${u}_$rep.json'));print('U=$u', {k: (v['frac'], v['ms']) for k, v in d['kernels'].items() if k.startswith('export')})"
done; done
