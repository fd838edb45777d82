#!/bin/bash
# FP8 block-128 bench primary: vectors per lane of the scalar-amax group kernel (MTQ_AMD_GROUP_U),
# interleaved, plus the r01 per-lane-load kernel (MTQ_AMD_GROUP_VARIANT=3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/groupu
for rep in 1 2; do for cfg in "U=2" "U=1" "U=4" "V=3"; do
  case $cfg in U=*) E="MTQ_AMD_GROUP_U=${cfg#U=}";; V=*) E="MTQ_AMD_GROUP_VARIANT=${cfg#V=}";; esac
  env $E timeout -k 10 120 python -u bench.py --steps 100 --warmup 20 --no-cpu --no-ptq --no-c3 --no-suite > gpurun_out/groupu/head_${cfg/=/}_$rep.json 2>/dev/null || exit 8
  python -c "import json;d=json.load(open('gpurun_out/groupu/head_${cfg/=/}_$rep.json'));print('$cfg',d['value'],d['roofline']['frac'],d['roofline']['mean_launch_ms'])"
done; done
