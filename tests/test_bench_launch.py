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


def _fake_topology(root, simds):
    for i, s in enumerate(simds):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if s else 64}\nsimd_count {s}\n"
                                      f"gfx_target_version {90500 if s else 0}\n")


def test_count_gpus_from_kfd_topology(tmp_path, monkeypatch):
    """The parent counts GPUs from the KFD topology (CPU nodes have no SIMDs), capped by a
    visible-devices list, and never initialises HIP doing so."""
    import torch
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    _fake_topology(tmp_path, [0, 256, 256, 256, 256, 0, 256, 256, 256, 256])
    assert bench.count_gpus_without_hip(str(tmp_path)) == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3")
    assert bench.count_gpus_without_hip(str(tmp_path)) == 2
    assert not torch.cuda.is_initialized()


def test_gpus_without_a_countable_device_exits_nonzero(tmp_path):
    """No KFD topology and no working amdsmi (this container): --gpus 2 must fail loudly rather
    than fall back to a HIP device query in the parent."""
    if bench.count_gpus_without_hip() is not None:
        pytest.skip("this machine exposes GPUs")
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=e,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "cannot count GPUs" in p.stderr or "GPU(s) visible" in p.stderr
