set -o pipefail
cd $GRAFT_REPO_ROOT
for gm in 1 2 4 8 16; do
  echo "== GM $gm"; SC_TN_GM=$gm timeout -k 10 120 python3 -u tools/tn_bench.py --tm 1 --shapes 0,4 --nolib 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== tn256"; timeout -k 10 120 python3 -u tools/tn_bench.py --tm 256 --shapes 0 --nolib 2>&1 | grep -v amdgpu.ids
