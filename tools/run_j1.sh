set -e -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -m gpu -k side_stream > gpurun_out/ws19_test.log 2>&1
echo done
