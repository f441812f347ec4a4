"""Seeded random scenes (tests/golden/fuzz_scenes.json, written by tests/golden/make_fuzz_scenes.js through this build's
Sail API): every shape, material, texture and light kind in random combinations, rooms open and closed, cameras inside
and outside. The fixed scenes of the other tests pin what the reference renders; these look for a combination that
one of the three implementations of the path handles differently from the others.

CPU: the fixture is what the generator writes; the JS/Node software shader (oracle/sail_soft.js) equals the C++ oracle
on every scene, bit for bit. GPU: the HIP path equals the oracle on every scene in each precompiled kernel form (the
one the plugin set selects, the all-plugin kernel, the pre-cull kernel) and, for a few scenes, in the run-time
kernel compiled for the scene; AOV maps, exact segment counts and picks too."""
import functools
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
from sail_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "fuzz_scenes.json")
GEN = os.path.join(ROOT, "tests", "golden", "make_fuzz_scenes.js")
SOFT = os.path.join(ROOT, "oracle", "sail_soft.js")
NODE = shutil.which("node") or shutil.which("nodejs")

with open(FIXTURE) as f:
    SCENES = json.load(f)
NAMES = sorted(SCENES)
W, H, SPP, B = 24, 16, 3, 6


def bit_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def schedule(sc, w, h, spp):
    return capi.schedule(np.array(sc["mvp_rowmajor"]), w, h, 0, spp)


@functools.lru_cache(maxsize=None)
def oracle_frame(name, w=W, h=H, spp=SPP, b=B):
    """the oracle's SUM frame, AOV maps and segment count of a fuzz scene"""
    sc = SCENES[name]
    inv, seeds = schedule(sc, w, h, spp)
    oracle.reset_counters()
    acc, an, ap = oracle.render(sc, capi.plugin_masks(sc["plugins"]), w, h, inv, seeds, sc["eye"], b, aov=True)
    segs, _ = oracle.counters()
    return acc, an, ap, segs


def test_fuzz_scene_kinds_covered():
    """the fixture exercises every plugin of every kind, scenes that the flat and the pre-cull paths take
    (SAIL_DEBUG_CULL_MIN_PRIMS default 8), and several lights of different kinds in one scene"""
    seen = {k: set() for k in ("shape", "material", "texture", "light")}
    for sc in SCENES.values():
        for k in seen:
            seen[k].update(sc["plugins"][k])
    assert seen["shape"] == {"cube", "sphere", "rectangle", "cone", "cylinder", "disk", "hyperboloid", "paraboloid",
                             "cornellbox"}
    assert seen["material"] == {"matte", "mirror", "metal", "glass"}
    assert seen["texture"] == {"checkerboard", "checkerboard2", "bilerp", "mixf", "scale", "uvf"}
    assert seen["light"] == {"area", "point", "spot"}
    ns = [sc["n"] for sc in SCENES.values()]
    assert min(ns) < 8 <= max(ns)
    assert any(sc["ln"] > 1 and len(sc["plugins"]["light"]) > 1 for sc in SCENES.values())  # mixed light kinds


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_fuzz_fixture_is_what_the_generator_writes(tmp_path):
    out = tmp_path / "fuzz.json"
    subprocess.run([NODE, GEN, str(out)], check=True, timeout=120)
    assert json.loads(out.read_text()) == SCENES


@pytest.mark.skipif(NODE is None, reason="node not installed")
@pytest.mark.parametrize("name", NAMES)
def test_fuzz_soft_js_equals_cpp_oracle(tmp_path, name):
    sc = SCENES[name]
    w, h, spp, b = 12, 10, 2, B
    inv, seeds = schedule(sc, w, h, spp)
    job = {"objects": sc["objects"], "n": sc["n"], "texparams": sc["texparams"], "tn": sc["tn"],
           "lights": sc["lights"], "ln": sc["ln"], "masks": list(capi.plugin_masks(sc["plugins"])), "W": w, "H": h,
           "inv": [float(v) for v in inv.reshape(-1)], "seeds": [float(v) for v in seeds], "eye": sc["eye"],
           "spp": spp, "maxBounces": b, "accumMode": 0, "aov": True}
    jp = tmp_path / "job.json"
    jp.write_text(json.dumps(job))
    out = subprocess.run([NODE, SOFT, str(jp), str(tmp_path / name)], capture_output=True, text=True, timeout=300,
                         check=True).stdout
    info = json.loads(out.strip().splitlines()[-1])
    got = np.fromfile(tmp_path / f"{name}.accum.f32", dtype=np.float32).reshape(h, w, 4)
    gn = np.fromfile(tmp_path / f"{name}.aovn.f32", dtype=np.float32).reshape(h, w, 4)
    gp = np.fromfile(tmp_path / f"{name}.aovp.f32", dtype=np.float32).reshape(h, w, 4)
    want, wn, wp, segs = oracle_frame(name, w, h, spp, b)
    same = bit_equal(got, want)
    assert same.all(), f"{name}: {int((~same).sum())} of {got.size} channels differ"
    assert bit_equal(gn, wn).all() and bit_equal(gp, wp).all()
    assert info["segments"] == segs


# ---- GPU ------------------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gpu():
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    return True


FORMS = {
    # the precompiled kernel the scene's plugin set selects (Cornell / room / all-plugin / pre-cull at >= 8 rows)
    "precompiled": {capi.DEBUG_JIT: 0},
    "generic": {capi.DEBUG_JIT: 0, capi.DEBUG_FORCE_GENERIC: 1, capi.DEBUG_CULL_MIN_PRIMS: 1000},
    "cull": {capi.DEBUG_JIT: 0, capi.DEBUG_CULL_MIN_PRIMS: 0},
}


def render_hip(sc, debug, launch=2):
    inv, seeds = schedule(sc, W, H, SPP)
    ctx = capi.Context(W, H, flags=capi.FLAG_AOV | capi.FLAG_SEGMENT_COUNT, debug=debug)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_launch_samples(launch)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        acc = ctx.read_accum()
        _, an, ap = ctx.readback(aov=True)
        return acc, an, ap, ctx.stats(), ctx.kernel_name()
    finally:
        ctx.close()


def check(name, got):
    acc, an, ap, st, kname = got
    want, wn, wp, segs = oracle_frame(name)
    same = bit_equal(acc, want)
    assert same.all(), f"{name} ({kname}): {int((~same).sum())} of {acc.size} channels differ"
    assert bit_equal(an, wn).all() and bit_equal(ap, wp).all(), kname
    assert st.segments == segs, kname


@pytest.mark.gpu
@pytest.mark.parametrize("form", sorted(FORMS))
@pytest.mark.parametrize("name", NAMES)
def test_fuzz_hip_equals_oracle(gpu, name, form):
    check(name, render_hip(SCENES[name], FORMS[form]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES[1::4])
def test_fuzz_ragged_frames_and_sample_groups(gpu, name):
    """a ragged frame (partial 16 x 16 blocks and strips), more bounces, launches of 3 samples split over 2 sample
    groups, in the kernel the scene selects"""
    w, h, spp, b = 37, 23, 5, 9
    sc = SCENES[name]
    inv, seeds = schedule(sc, w, h, spp)
    ctx = capi.Context(w, h, flags=capi.FLAG_SEGMENT_COUNT, debug={capi.DEBUG_SAMPLE_GROUPS: 2})
    try:
        ctx.set_scene_dict(sc)
        ctx.set_launch_samples(3)
        ctx.render_schedule(inv, seeds, sc["eye"], b)
        acc, st = ctx.read_accum(), ctx.stats()
    finally:
        ctx.close()
    want, _, _, segs = oracle_frame(name, w, h, spp, b)
    same = bit_equal(acc, want)
    assert same.all(), f"{name}: {int((~same).sum())} of {acc.size} channels differ"
    assert st.segments == segs


# run-time kernels (a hipRTC build each on the box): flat scenes of at most 8 rows compiled for their rows, the
# room-family and plain forms of larger flat scenes, the pre-cull form
JIT_CASES = [("F01", "rows"), ("F10", "rows"), ("F12", "rows"), ("F17", "flat"), ("F22", "flat"), ("F00", "cull"),
             ("F23", "cull")]


@pytest.mark.gpu
@pytest.mark.parametrize("name,mode", JIT_CASES)
def test_fuzz_jit_kernel_equals_oracle(gpu, name, mode):
    sc = SCENES[name]
    assert (sc["n"] <= 8) == (mode == "rows")
    debug = {capi.DEBUG_JIT: 27}
    if mode == "flat":
        debug[capi.DEBUG_CULL_MIN_PRIMS] = 1000
    elif mode == "cull":
        debug[capi.DEBUG_CULL_MIN_PRIMS] = 0
    got = render_hip(sc, debug)
    assert got[4].startswith("sail_trace_kernel_" + ("cull_jit" if mode == "cull" else "jit")), got[4]
    check(name, got)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES[::3])
def test_fuzz_pick_equals_oracle(gpu, name):
    sc = SCENES[name]
    rng = np.random.default_rng(int(name[1:]))
    mvp = np.array(sc["mvp_rowmajor"])
    inv = np.linalg.inv(mvp)
    eye = np.array(sc["eye"], dtype=np.float64)
    xs, ys = rng.uniform(-1, 1, 1024), rng.uniform(-1, 1, 1024)
    p = inv @ np.stack([xs, ys, np.zeros_like(xs), np.ones_like(xs)])
    d = (p[:3] / p[3]).T - eye
    rays = np.concatenate([np.concatenate([np.tile(eye, (len(d), 1)), d], axis=1),
                           np.concatenate([rng.uniform(0.5, 5.0, (1024, 3)), rng.normal(size=(1024, 3))], axis=1)])
    rays = rays.astype(np.float32)
    ctx = capi.Context(16, 16)
    try:
        ctx.set_scene_dict(sc)
        idx, t = ctx.pick(rays)
    finally:
        ctx.close()
    widx, wt = oracle.pick(sc, capi.plugin_masks(sc["plugins"])[0], rays)
    assert np.array_equal(idx, widx)
    assert np.array_equal(t.view(np.uint32), wt.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["tiles", "samples"])
@pytest.mark.parametrize("name", NAMES[2::6])
def test_fuzz_multi_device_partitions(gpu, name, mode):
    """the multi-device context over three "devices" on one GPU (sail_create_multi; the frame summed by a kernel) on a
    130 x 70 frame (three 64 x 64 tiles across, ragged), in 2 + 2 samples with a reduce in between: tiles bit for bit,
    a sample split to the rounding of its summation order; the AOV maps of the last sample bit for bit in both"""
    sc = SCENES[name]
    w, h, b, k = 130, 70, 6, 2
    inv, seeds = schedule(sc, w, h, 2 * k)
    part = capi.PART_TILES if mode == "tiles" else capi.PART_SAMPLES
    ctx = capi.Context(w, h, devices=[0, 0, 0], flags=capi.FLAG_AOV)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_partition(0, 1, part)
        ctx.render_schedule(inv[:k], seeds[:k], sc["eye"], b)
        ctx.read_accum()
        ctx.render_schedule(inv[k:], seeds[k:], sc["eye"], b)
        got = ctx.read_accum()
        _, gn, gp = ctx.readback(aov=True)
    finally:
        ctx.close()
    want, wn, wp, _ = oracle_frame(name, w, h, 2 * k, b)
    assert bit_equal(gn, wn).all() and bit_equal(gp, wp).all()
    assert (got[..., 3] == 2 * k).all()
    if mode == "tiles":
        same = bit_equal(got, want)
        assert same.all(), f"{name}: {int((~same).sum())} of {got.size} channels differ"
    else:
        fin = np.isfinite(want)
        assert (np.isfinite(got) == fin).all()
        assert np.allclose(got[fin], want[fin], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.skipif(NODE is None, reason="node not installed")
@pytest.mark.parametrize("name,mode,api,devices", [("F05", "sum", "frames", None), ("F19", "mix", "samples", None),
                                                   ("F23", "sum", "progressive", "0,0,0"), ("E05", "sum", "resume", None),
                                                   ("E13", "mix", "frames", "0,0")])
def test_fuzz_through_the_js_renderer(tmp_path, name, mode, api, devices):
    """the whole drop-in stack on random scenes: the scene built by the Sail JS API in Node (tests/js/render_check.js),
    Renderer.update / render through N-API into libsail_hip.so, against the oracle over the fixture's rows"""
    w, h, spp, b = 40, 30, 4, 6
    prefix = str(tmp_path / name)
    env = dict(os.environ, **({"SAIL_TEST_DEVICES": devices} if devices else {}))
    subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "render_check.js"), "fuzz:" + name, str(w), str(h), str(spp),
                    str(b), mode, api, prefix], cwd=ROOT, check=True, timeout=300, env=env)
    got = np.fromfile(prefix + ".accum.f32", dtype=np.float32).reshape(h, w, 4)
    sc = SCENES[name]
    inv, seeds = schedule(sc, w, h, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), w, h, inv, seeds, sc["eye"], b,
                         accum_mode=oracle.ACC_SUM if mode == "sum" else oracle.ACC_MIX)
    same = bit_equal(got, want)
    assert same.all(), f"{name}: {int((~same).sum())} of {got.size} channels differ"
