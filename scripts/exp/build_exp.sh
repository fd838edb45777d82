#!/bin/bash
# Build the measurement-only experiment libraries (scripts/exp/*.hip -> scripts/exp/lib*.so).
set -e
cd "$(dirname "$0")"
for f in *.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../../include -I../../tensorrt-model-optimizer_amd/csrc "$f" -o "lib${f%.hip}.so"
done
