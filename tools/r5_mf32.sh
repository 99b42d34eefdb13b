#!/bin/bash
# wgrad on 32x32x16 MFMAs (tools/ab/mf32, SC_GEMM_MF32=1) against the shipped 16x16x32 kernel:
# the GEMM tests on the variant, then the weight-gradient timing and the C2 bench, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5o}
V=$R/tools/ab/mf32/libstatecatcher_hip.so
SC_LIB_PATH=$V timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_gemm.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rnd in 1 2; do
  for v in cur mf32; do
    if [ $v = cur ]; then L=""; else L=$V; fi
    echo "== $v ($rnd)"
    SC_LIB_PATH=$L timeout -k 10 200 python3 -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit $?
    SC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline off \
      > gpurun_out/${TAG}_$v.$rnd.json 2> gpurun_out/${TAG}_$v.$rnd.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$v.$rnd.json')); print('bench', d['ms_per_step'], d['kernels']['gate_gemm_wgrad'], d['loss_last'])"
  done
done
