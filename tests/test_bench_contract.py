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


class _FrameCtx:
    """stands in for a context whose reduced frame is `acc` (bench.validate_frame reads it with read_accum)"""

    def __init__(self, acc):
        self.acc = acc

    def read_accum(self):
        return self.acc.copy()


def test_validate_frame_refuses_a_broken_reduce(fixtures, capsys):
    """bench.py checks the reduced frame after its timed steps: every count == spp and oracle crops in tiles of
    several ranks; a reduce that drops or double-counts one rank's tiles ends the run (exit 3) with no number"""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    import oracle
    from sail_amd import capi
    sc = fixtures["scenes"]["C1"]
    W, H, B, spp, ngpu = 130, 70, 3, 2, 4
    masks = capi.plugin_masks(sc["plugins"])
    mvp = np.array(sc["mvp_rowmajor"])
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    good = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B)
    rep = bench.validate_frame(_FrameCtx(good), sc, masks, mvp, W, H, B, spp, inv, seeds, capi.PART_TILES, ngpu)
    assert rep["pixels_with_wrong_count"] == 0 and all(c["match"] for c in rep["oracle_crops"])
    assert {c["rank"] for c in rep["oracle_crops"]} >= {0, 3}
    for broken in ("dropped", "doubled", "wrong"):
        acc = good.copy()
        tile = acc[0:64, 64:128]  # tile 1 (rank 1 of 4)
        if broken == "dropped":
            tile[...] = 0.0
        elif broken == "doubled":
            tile[...] *= 2.0
        else:  # counts right, radiance of rank 3's tile perturbed
            acc[0:64, 0:64, 0] = np.nextafter(acc[0:64, 0:64, 0], np.float32(np.inf))
            acc[64:70, 128:130, 0] += 1e-3
        with pytest.raises(SystemExit) as e:
            bench.validate_frame(_FrameCtx(acc), sc, masks, mvp, W, H, B, spp, inv, seeds, capi.PART_TILES, ngpu)
        assert e.value.code == 3
    out = capsys.readouterr()
    assert out.out == "" and "failed validation" in out.err
