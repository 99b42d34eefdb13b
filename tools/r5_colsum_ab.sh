#!/bin/bash
# One sc_colsum_multi launch per gate projection (default) vs two sc_colsum launches
# (SC_COLSUM_MULTI=0): the C2 bench, interleaved, 3 rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5v}
for rnd in 1 2 3; do
  for v in 1 0; do
    SC_COLSUM_MULTI=$v timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --cpu-baseline off \
      > gpurun_out/${TAG}_$v.$rnd.json 2> gpurun_out/${TAG}_$v.$rnd.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$v.$rnd.json')); print('multi=$v', d['ms_per_step'], d['kernels']['gate_gemm_wgrad']['avg_us'], d['loss_last'])"
  done
done
