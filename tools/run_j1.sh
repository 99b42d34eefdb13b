set -e -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_torch_library.py -m gpu > gpurun_out/t15_test.log 2>&1
echo done
