set -e -o pipefail
bash tools/run_ab.sh j10 "python3 -u tools/joint_probe.py 32 3" sb0 il ilsb0
echo done
