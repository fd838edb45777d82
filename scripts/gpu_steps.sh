#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/$TAG/<name>.log.
# A step that fails normally (a test assertion) lets the next one run; a step that times out,
# aborts or faults (124, 137, 134, 139) ends the script there.  Usage, on the box:
#   bash scripts/gpu_steps.sh TAG 'name|seconds|command' ...
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -3 "$OUT/$name.log"
  case $rc in 124|137|134|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
done
