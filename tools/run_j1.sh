set -e -o pipefail
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1
tail -2 gpurun_out/fin_smoke.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/fin_gpu.log 2>&1
tail -2 gpurun_out/fin_gpu.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/fin_bench.log 2>&1
tail -1 gpurun_out/fin_bench.log
