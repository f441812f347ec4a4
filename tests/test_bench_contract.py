"""bench.py's output contract on CPU: rank 0 prints exactly one JSON line on stdout, so C-level prints made
while the RCCL communicator is created (its version banner) must land on stderr."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stdout_to_stderr_covers_c_level_writes():
    code = (
        "import os, sys\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "q = bench._StdoutToStderr()\n"
        "q.__enter__()\n"
        "os.write(1, b'RCCL version : banner\\n')\n"
        "print('python-level noise')\n"
        "q.__exit__()\n"
        "print('{\"metric\": \"m\"}')\n" % ROOT
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"metric": "m"}']
    assert "RCCL version" in r.stderr and "python-level noise" in r.stderr


def _bench(args, env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, env=env, cwd=ROOT)


def test_gpus_must_match_world_size():
    """--gpus N under torch.distributed.run with WORLD_SIZE != N exits non-zero before touching a device"""
    r = _bench(["--gpus", "4", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "does not match WORLD_SIZE" in r.stderr
    assert r.stdout.strip() == ""


def test_gpus_beyond_visible_devices_fails():
    """--gpus N in one process needs N visible devices (the multi-device context); never a silent 1-GPU run"""
    from sail_amd import capi
    if capi.device_count() >= 64:
        pytest.skip("that many devices are visible")
    r = _bench(["--gpus", "64", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "HIP devices are visible" in r.stderr
    assert r.stdout.strip() == ""
