"""BASELINE.json configs[0] at its own size: the README Cornell box (frozen C1 scene), 256x256, 4 bounces, 64 spp, the
whole frame, against tests/golden/c1_full_256.json -- the hash of the frame the JS/Node software shader
(oracle/sail_soft.js, the north star's CPU fallback) renders, written by tests/golden/make_c1_full.py.

CPU: the C++ oracle's whole frame has that hash (three implementations agree at the configuration's full size).
GPU: the HIP path's whole frame has that hash, every float of every pixel, through the kernel a
default context launches for the scene (its run-time kernel), and through the precompiled Cornell kernel."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from sail_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_c1_full  # noqa: E402

with open(os.path.join(ROOT, "tests", "golden", "c1_full_256.json")) as _f:
    FIXTURE = json.load(_f)


def _sha(acc):
    return hashlib.sha256(np.ascontiguousarray(acc, dtype="<f4").tobytes()).hexdigest()


def test_fixture_is_configs0():
    assert (FIXTURE["width"], FIXTURE["height"], FIXTURE["bounces"], FIXTURE["spp"]) == (256, 256, 4, 64)
    assert FIXTURE["count_min_max"] == [64.0, 64.0]


def test_cpp_oracle_full_frame_matches_js_shader():
    import oracle
    sc, inv, seeds = make_c1_full.job()
    acc = oracle.render(sc, capi.plugin_masks(sc["plugins"]), 256, 256, inv, seeds, sc["eye"], 4)
    assert _sha(acc) == FIXTURE["sha256_accum_f32le"]


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [27, 0], ids=["runtime_kernel", "precompiled"])
def test_hip_full_frame_matches_js_shader(jit):
    sc, inv, seeds = make_c1_full.job()
    ctx = capi.Context(256, 256, device=0)
    try:
        ctx.set_debug(capi.DEBUG_JIT, jit)
        ctx.set_scene_dict(sc)
        ctx.kernel_ready(-1)
        ctx.render_schedule(inv, seeds, sc["eye"], 4)
        got = ctx.read_accum()
        name = ctx.kernel_name()
    finally:
        ctx.close()
    # a 256x256 frame is 16 tiles: the launch splits its samples into groups ("_grouped" + sail_accum_kernel)
    assert name.startswith("sail_trace_kernel_jit" if jit else "sail_trace_kernel_cornell"), name
    if _sha(got) != FIXTURE["sha256_accum_f32le"]:
        import oracle
        want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), 256, 256, inv, seeds, sc["eye"], 4)
        diff = int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))
        raise AssertionError(f"C1 256x256 frame differs from the JS shader's fixture; {diff} channels differ from the oracle")
