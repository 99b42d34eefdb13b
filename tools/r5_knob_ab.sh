#!/bin/bash
# Same-box A/B of compile-time knobs on the C2 bench: base, then each tools/ab/<name> library,
# two rounds interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5l}
for rnd in 1 2; do
  for v in base fd2 csw slots5; do
    if [ $v = base ]; then L=""; else L="$R/tools/ab/$v/libstatecatcher_hip.so"; fi
    SC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline off \
      > gpurun_out/${TAG}_$v.$rnd.json 2> gpurun_out/${TAG}_$v.$rnd.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$v.$rnd.json')); k=d['kernels']; print('$v', d['ms_per_step'], k.get('lucy_scan_fwd',{}).get('avg_us'), k.get('lucy_scan_bwd',{}).get('avg_us'), k.get('gate_gemm_wgrad',{}).get('avg_us'))"
  done
done
