#!/bin/bash
# rocprofv3 kernel durations of the decode QuantLinear kernels per Llama shape, for the env
# settings given as arguments (NAME=ENVSTRING ...)
set -o pipefail
export PYTHONPATH=$PWD:$PWD/tensorrt-model-optimizer_amd
mkdir -p gpurun_out/qlprof
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/qlprof/$name -o ql -- python3 scripts/prof_qlinear.py > gpurun_out/qlprof/$name.log 2>&1 || { tail -20 gpurun_out/qlprof/$name.log; exit 1; }
  f=$(find gpurun_out/qlprof/$name -name "ql_results.db" | head -1)
  python3 scripts/rocpd_kernels.py $f qlinear > gpurun_out/qlprof/$name.json || exit 1
  echo "== $name ($envs)"; python3 -c "
import json; d=json.load(open('gpurun_out/qlprof/$name.json'))
for k,v in d.items(): print(k[-75:], v['n'], v['median_us'], v['min_us'])"
done
