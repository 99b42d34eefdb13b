#!/bin/bash
# Round-6 measurement call: the GEMM tests, the same-box A/B of layer 0's weight gradient
# (128-column MFMA tile vs the library), the measurement set (tools/gpu_profile.sh: bench line,
# kernel trace + stats, PMC FETCH / WRITE over the scans), then the C5 and C4 bench lines.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${TAG:-r6f}
timeout -k 10 600 python3 -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_gpu_gemm.py \
  > gpurun_out/${TAG}_gemm.log 2>&1; rc=$?; echo "gemm tests rc=$rc"; tail -2 gpurun_out/${TAG}_gemm.log
grep "layer-0 dW" gpurun_out/${TAG}_gemm.log
case $rc in 124|134|137|139) exit $rc;; esac
for rnd in 1 2; do
  for v in on off; do
    SC_WGRAD128=$([ $v = on ] && echo 1 || echo 0) timeout -k 10 300 python3 bench.py --cpu-baseline off \
      > gpurun_out/${TAG}_w128${v}_$rnd.json 2> gpurun_out/${TAG}_w128${v}_$rnd.err || { echo "bench failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], {k: v.get('avg_us') for k, v in d['kernels'].items() if 'gemm' in k})" gpurun_out/${TAG}_w128${v}_$rnd.json
  done
done
bash tools/gpu_profile.sh $TAG || exit $?
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for wl in rnnt xlstm; do
  timeout -k 10 400 python3 bench.py --workload $wl --cpu-baseline off > gpurun_out/bench_${TAG}_$wl.json \
    2> gpurun_out/bench_${TAG}_$wl.err || { echo "bench $wl failed"; tail -5 gpurun_out/bench_${TAG}_$wl.err; exit 1; }
  cut -c1-300 gpurun_out/bench_${TAG}_$wl.json
done
cut -c1-400 gpurun_out/bench_$TAG.json
