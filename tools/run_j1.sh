set -e -o pipefail
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_parity_step.py -m gpu > gpurun_out/parity_measured.log 2>&1
echo done
