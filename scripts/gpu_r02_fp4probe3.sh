#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/probe_fp4_cvt16 > gpurun_out/fp4probe16.txt 2>&1 || { cat gpurun_out/fp4probe16.txt; exit 10; }
cat gpurun_out/fp4probe16.txt
