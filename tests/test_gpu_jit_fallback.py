"""The run-time kernels' failure paths on the GPU: a process whose hipRTC cannot be opened (SAIL_HIPRTC names a missing
file), and one whose hipRTC is another ROCm's (PyTorch's: its code objects come from another compiler and are refused,
sail_jit.cpp sameCompiler), render with the precompiled kernels, bit-exact against the oracle. Run in a child process:
the library opens hipRTC once per process. The scene (ALL) has no code object in the cache shipped beside the library,
and the child's user cache is off, so the code object would have to be compiled. Needs a GPU."""
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
capi.set_jit_cache("")
sc = json.load(open(sys.argv[2]))["scenes"]["ALL"]
W, H, spp, B = 32, 24, 3, 6
inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
ctx = capi.Context(W, H)
ctx.set_scene_dict(sc)
ctx.render_schedule(inv, seeds, sc["eye"], B)
np.save(sys.argv[3], ctx.read_accum())
print(json.dumps({"kernel": ctx.kernel_name(), "info": ctx.kernel_info()}))
ctx.close()
"""


def _torch_hiprtc():
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "libhiprtc.so")
    return p if os.path.exists(p) else None


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["missing", "other_rocm"])
def test_unusable_hiprtc_falls_back_to_precompiled_kernels(tmp_path, fixtures, which):
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    if which == "missing":
        rtc = str(tmp_path / "missing" / "libhiprtc.so.7")
    else:
        rtc = _torch_hiprtc()
        if rtc is None:
            pytest.skip("no second hipRTC in this image")
    out = tmp_path / "acc.npy"
    env = dict(os.environ, SAIL_HIPRTC=rtc, AMD_COMGR_CACHE="0")
    r = subprocess.run([sys.executable, "-u", "-c", CHILD, ROOT, os.path.join(ROOT, "tests", "golden", "fixtures.json"),
                        str(out)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["kernel"] == "sail_trace_kernel_grouped" or info["kernel"] == "sail_trace_kernel", info  # all-plugin
    assert info["info"]["jit_state"] == capi.KERNEL_JIT_FAILED, info
    assert ("dlmopen" if which == "missing" else "produced by clang") in info["info"]["jit_error"], info
    sc = fixtures["scenes"]["ALL"]
    W, H, spp, B = 32, 24, 3, 6
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    got = np.load(out)
    assert (got.view(np.uint32) == np.ascontiguousarray(want, np.float32).view(np.uint32)).all()
