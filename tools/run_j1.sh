set -e -o pipefail
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_final.log 2>&1
echo done
