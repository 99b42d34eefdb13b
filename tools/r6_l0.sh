#!/bin/bash
# Layer 0's forward shape (48000 x 3584 x 128): tn256 (the default) against the one-wave tnw32
# with the LDS epilogue (its LN instance, the only one without spills; statistics ignored).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 150 python3 -u tools/tn_bench.py --tm 256 --shapes 1 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 150 python3 -u tools/tn_bench.py --ln --shapes 1 --nolib 2>&1 | grep -v amdgpu.ids || exit 1
