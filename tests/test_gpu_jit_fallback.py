"""The run-time kernels' failure path on the GPU: a process whose hipRTC cannot be opened (SAIL_HIPRTC names a missing
file) renders with the precompiled kernels, bit-exact against the oracle. Run in a child process: the library opens
hipRTC once per process (sail_jit.cpp). Needs a GPU."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from sail_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from sail_amd import capi
sc = json.load(open(sys.argv[2]))["scenes"]["C1"]
W, H, spp, B = 32, 24, 3, 6
inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
ctx = capi.Context(W, H)
ctx.set_scene_dict(sc)
ctx.render_schedule(inv, seeds, sc["eye"], B)
np.save(sys.argv[3], ctx.read_accum())
print(json.dumps({"kernel": ctx.kernel_name()}))
ctx.close()
"""


@pytest.mark.gpu
def test_missing_hiprtc_falls_back_to_precompiled_kernels(tmp_path, fixtures):
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    out = tmp_path / "acc.npy"
    env = dict(os.environ, SAIL_HIPRTC=str(tmp_path / "missing" / "libhiprtc.so.7"))
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, os.path.join(ROOT, "tests", "golden", "fixtures.json"), str(out)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["kernel"].startswith("sail_trace_kernel_cornell"), info  # not a run-time kernel
    sc = fixtures["scenes"]["C1"]
    W, H, spp, B = 32, 24, 3, 6
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    got = np.load(out)
    assert (got.view(np.uint32) == np.ascontiguousarray(want, np.float32).view(np.uint32)).all()
