#!/bin/bash
# tnw32 epilogue through LDS (SC_TNW_EPI=1) against the scattered-piece stores (=0): the LN-fold
# GEMM standalone at the gate shape, the plain tnw32<4> (tile_m 3), then the C2 step with
# SC_LN_FOLD=2 on each against the default path.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${TAG:-r6e}
for v in epi0 epi1; do
  echo "== $v"
  SC_LIB_PATH=$PWD/tools/ab/$v/libstatecatcher_hip.so timeout -k 10 150 python3 -u tools/tn_bench.py --ln --shapes 0 2>&1 | grep -v amdgpu.ids || exit 1
  SC_LIB_PATH=$PWD/tools/ab/$v/libstatecatcher_hip.so timeout -k 10 150 python3 -u tools/tn_bench.py --tm 3 --shapes 0,2 --nolib 2>&1 | grep -v amdgpu.ids || exit 1
done
for rnd in 1 2; do
  for v in base epi0 epi1; do
    if [ $v = base ]; then env=""; else env="SC_LIB_PATH=$PWD/tools/ab/$v/libstatecatcher_hip.so SC_LN_FOLD=2"; fi
    env $env timeout -k 10 300 python3 -u bench.py --cpu-baseline off > gpurun_out/${TAG}_${v}_${rnd}.json 2> gpurun_out/${TAG}_${v}_${rnd}.err || exit 1
    python3 - gpurun_out/${TAG}_${v}_${rnd}.json $v $rnd <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], {k: v["avg_us"] for k, v in d["kernels"].items() if "gemm" in k})
PY
  done
done
