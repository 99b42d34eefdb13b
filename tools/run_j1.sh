set -e -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_xlstm_glue.py tests/test_gpu_c4.py -m gpu > gpurun_out/g12_test.log 2>&1
bash tools/run_ab.sh g12 "python3 -u bench.py --workload xlstm --steps 8 --warmup 3 --cpu-baseline off" old
echo done
