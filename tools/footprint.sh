#!/bin/bash
# Build the RCCL-footprint probe (tools/footprint.hip) for bench.py --rccl-footprint.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/ab/footprint"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 "$R/tools/footprint.hip" \
  -o "$R/tools/ab/footprint/libfootprint.so"
