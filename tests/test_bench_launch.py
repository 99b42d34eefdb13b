"""bench.py's --gpus launcher: environment plumbing with a stub worker that never touches HIP,
and the loud failures (bad --gpus, WORLD_SIZE mismatch)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

STUB = ("import json, os, sys; keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', "
        "'MASTER_ADDR', 'MASTER_PORT', 'HSA_ENABLE_IPC_MODE_LEGACY']; "
        "open(os.path.join(sys.argv[1], os.environ['RANK'] + '.json'), 'w')"
        ".write(json.dumps({k: os.environ.get(k) for k in keys}))")


def test_spawn_ranks_environment(tmp_path):
    rc = bench.spawn_ranks(4, [sys.executable, "-c", STUB, str(tmp_path)], port=29611)
    assert rc == 0
    envs = [json.load(open(tmp_path / f"{r}.json")) for r in range(4)]
    for r, e in enumerate(envs):
        assert e == {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": "4",
                     "LOCAL_WORLD_SIZE": "4", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29611",
                     "HSA_ENABLE_IPC_MODE_LEGACY": "0"}


def test_spawn_ranks_propagates_failure(tmp_path):
    # rank 1 fails fast, rank 0 would sleep: the launcher returns rank 1's code and stops rank 0
    stub = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(30) if r == 0 else sys.exit(3)"
    rc = bench.spawn_ranks(2, [sys.executable, "-c", stub])
    assert rc == 3


@pytest.mark.parametrize("argv, env", [(["--gpus", "0"], {}),
                                       (["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0"}),
                                       (["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0"})])
def test_bad_gpus_exits_nonzero(argv, env):
    e = dict(os.environ)
    e.update(env)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, env=e,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "--gpus" in p.stderr
