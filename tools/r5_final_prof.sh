#!/bin/bash
# Round-5 measurement set: tools/gpu_profile.sh (bench line, rocprofv3 kernel-trace/stats, two PMC
# passes over the scans) for the default bf16 C2 bench, then the two PMC passes of the fp32 C2
# bench (roofline.traffic keyed "ctc/fp32"), the fp32 bench line, and the traffic table update.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r5}
O=$R/gpurun_out
bash "$R/tools/gpu_profile.sh" $TAG
cd /tmp && export TMPDIR=/tmp
echo "pmc fp32"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex "scan" -d "$O/pmc_fetch_${TAG}_fp32" -o run -- \
  python3 "$R/bench.py" --dtype fp32 --steps 2 --warmup 1 --cpu-baseline off > "$O/pmc_fetch_${TAG}_fp32.log" 2>&1
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex "scan" -d "$O/pmc_write_${TAG}_fp32" -o run -- \
  python3 "$R/bench.py" --dtype fp32 --steps 2 --warmup 1 --cpu-baseline off > "$O/pmc_write_${TAG}_fp32.log" 2>&1
find "$O/pmc_fetch_${TAG}_fp32" "$O/pmc_write_${TAG}_fp32" -type f ! -name "*counter_collection.csv" -delete
cp "$R/profiles/pmc_traffic.json" "$O/pmc_traffic_${TAG}.json"
python3 "$R/tools/pmc_traffic.py" $(ls "$O"/pmc_fetch_$TAG/*/*counter_collection.csv "$O"/pmc_fetch_$TAG/*counter_collection.csv 2>/dev/null | head -1) \
  $(ls "$O"/pmc_write_$TAG/*/*counter_collection.csv "$O"/pmc_write_$TAG/*counter_collection.csv 2>/dev/null | head -1) \
  "$O/pmc_traffic_${TAG}.json" ctc/bf16
python3 "$R/tools/pmc_traffic.py" $(ls "$O"/pmc_fetch_${TAG}_fp32/*/*counter_collection.csv "$O"/pmc_fetch_${TAG}_fp32/*counter_collection.csv 2>/dev/null | head -1) \
  $(ls "$O"/pmc_write_${TAG}_fp32/*/*counter_collection.csv "$O"/pmc_write_${TAG}_fp32/*counter_collection.csv 2>/dev/null | head -1) \
  "$O/pmc_traffic_${TAG}.json" ctc/fp32
echo "bench fp32"
timeout -k 10 500 python3 "$R/bench.py" --dtype fp32 > "$O/bench_${TAG}_fp32.json" 2> "$O/bench_${TAG}_fp32.err"
cat "$O/bench_$TAG.json" "$O/bench_${TAG}_fp32.json"
echo done
