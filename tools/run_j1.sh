set -e -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/round_run.sh r3d
O=$R/gpurun_out/mpmc_r3d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex mlstm_ -f csv -d $O/f -o run -- python3 $R/bench.py --workload xlstm --steps 2 --warmup 1 --cpu-baseline off > $O/f.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex mlstm_ -f csv -d $O/w -o run -- python3 $R/bench.py --workload xlstm --steps 2 --warmup 1 --cpu-baseline off > $O/w.log 2>&1
find $O -type f ! -name "*counter_collection.csv" -delete
cd $R && bash tools/prof_workloads.sh
echo alldone
