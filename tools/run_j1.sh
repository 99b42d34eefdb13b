set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mlstm.py -m gpu > gpurun_out/j4_test.log 2>&1
: > gpurun_out/m4_bench.log
for s in 1 0 1; do echo "== split $s" >> gpurun_out/m4_bench.log; SC_MLSTM_SPLIT=$s timeout -k 10 120 python3 -u tools/mlstm_bench.py --reps 10 >> gpurun_out/m4_bench.log 2>&1; done
timeout -k 10 400 python3 -u bench.py --workload xlstm --steps 8 --warmup 4 > gpurun_out/b4_xlstm.json 2> gpurun_out/b4_xlstm.err
echo done
