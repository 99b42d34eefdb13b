#!/bin/bash
# Grid-stride LayerNorm forward (default) vs one row per wave (tools/ab/lngs0): bitwise A/B,
# LayerNorm timing and the C2 bench, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5s}
V=$R/tools/ab/lngs0/libstatecatcher_hip.so
timeout -k 10 200 python3 -u tools/ln_ab.py save gpurun_out/${TAG}_a.pt > gpurun_out/${TAG}_ab.log 2>&1 || exit $?
SC_LIB_PATH=$V timeout -k 10 200 python3 -u tools/ln_ab.py save gpurun_out/${TAG}_b.pt >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
python3 tools/ln_ab.py compare gpurun_out/${TAG}_a.pt gpurun_out/${TAG}_b.pt; rc=$?
rm -f gpurun_out/${TAG}_a.pt gpurun_out/${TAG}_b.pt; [ $rc -eq 0 ] || exit $rc
for rnd in 1 2; do
  for v in cur lngs0; do
    if [ $v = cur ]; then L=""; else L=$V; fi
    echo "== $v ($rnd)"
    SC_LIB_PATH=$L timeout -k 10 120 python3 -u tools/scan_bench.py --only ln --iters 50 2>&1 | grep layernorm || exit $?
    SC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline off \
      > gpurun_out/${TAG}_$v.$rnd.json 2> gpurun_out/${TAG}_$v.$rnd.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$v.$rnd.json')); print('bench', d['ms_per_step'], d['loss_last'])"
  done
done
