"""BASELINE.json's full frame sizes on the GPU, checked through properties that do not need a full CPU
render: oracle-rendered crops of the same frame (bit-exact), finiteness / sample counts, and the 8-rank
tile split emulated on one device summing to the 1-rank frame bit for bit."""
import json
import os
import zlib

import numpy as np
import pytest

import oracle
from sail_amd import capi

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def frozen():
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        return json.load(f)


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


# (config, scene, W, H, bounces, spp) — BASELINE.json configs[1..4] (C5: the converged Cornell render's 16 bounces)
FULL = [("C2", "C1", 1920, 1080, 8, 4), ("C3", "C3", 1920, 1080, 8, 2), ("C4", "C4", 3840, 2160, 12, 1),
        ("C5", "C1g", 1920, 1080, 16, 2)]


@pytest.mark.parametrize("cfg,name,W,H,B,spp", FULL)
def test_full_frame_crops_match_oracle(frozen, cfg, name, W, H, B, spp):
    sc = frozen[name]
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    ctx = capi.Context(W, H)
    ctx.set_scene_dict(sc)
    ctx.render_schedule(inv, seeds, sc["eye"], B)
    got = ctx.read_accum()
    ctx.close()
    assert np.isfinite(got).all()
    assert (got[..., 3] == spp).all()
    rng = np.random.default_rng(zlib.crc32(cfg.encode()))  # deterministic crops (str hash is salted)
    masks = capi.plugin_masks(sc["plugins"])
    c = 8
    crops = [(0, 0), (W - c, H - c), (W // 2 - c // 2, H // 2 - c // 2)] + \
            [(int(rng.integers(0, W - c)), int(rng.integers(0, H - c))) for _ in range(12)]
    for x0, y0 in crops:
        want = np.zeros((H, W, 4), np.float32)
        oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, crop=(x0, y0, c, c), accum=want)
        assert _bits_equal(got[y0:y0 + c, x0:x0 + c], want[y0:y0 + c, x0:x0 + c]), (cfg, x0, y0)


def test_c5_full_frame_sample_split_and_gaussian(frozen):
    """BASELINE configs[4] at its full frame size: 1920x1080, 16 bounces, the sample split over 3 "devices" of one
    GPU (the multi-device context's PART_SAMPLES path, summed in rank order) and the Gaussian r = 2, alpha = 2
    reconstruction pass (window.glsl:26-44) over the reduced frame. The split frame counts every sample once and
    equals the one-device frame to summation order; oracle crops of the uninterrupted frame match it to summation
    order; the display pass equals the oracle filter of the same mean image bit for bit over the whole frame."""
    sc = frozen["C1g"]
    W, H, B, spp = 1920, 1080, 16, 5
    flt = sc["filter"]
    w16 = np.array(flt["weights64"], np.float32)
    rx, ry = float(flt["radius"][0]), float(flt["radius"][1])
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    one = capi.Context(W, H)
    one.set_scene_dict(sc)
    one.render_schedule(inv, seeds, sc["eye"], B)
    ref = one.read_accum()
    one.close()
    ctx = capi.Context(W, H, devices=[0, 0, 0])
    try:
        ctx.set_scene_dict(sc)
        ctx.set_partition(0, 1, capi.PART_SAMPLES)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
        flt_out = ctx.filter(capi.FILTER_WINDOW, w16, rx, ry, 2.2)
    finally:
        ctx.close()
    assert (got[..., 3] == spp).all(), "every pixel counts each sample once"
    assert np.isfinite(got).all()
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-6)
    masks = capi.plugin_masks(sc["plugins"])
    c = 6
    for x0, y0 in [(0, 0), (W - c, H - c), (W // 2, H // 2), (W // 5, 2 * H // 3)]:
        want = np.zeros((H, W, 4), np.float32)
        oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, crop=(x0, y0, c, c), accum=want)
        assert _bits_equal(ref[y0:y0 + c, x0:x0 + c], want[y0:y0 + c, x0:x0 + c]), (x0, y0)
        assert np.allclose(got[y0:y0 + c, x0:x0 + c], want[y0:y0 + c, x0:x0 + c], rtol=1e-5, atol=1e-6)
    mean = got.copy()
    mean[..., :3] = got[..., :3] / got[..., 3:4]
    want_f = oracle.filter_image(mean, capi.FILTER_WINDOW, w16, rx, ry, 2.2)
    assert _bits_equal(flt_out, want_f)


def test_c2_eight_rank_split_equals_single_rank(frozen):
    sc = frozen["C1"]
    W, H, B, spp = 1920, 1080, 8, 2
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    total = np.zeros((H, W, 4), np.float32)
    ctx = capi.Context(W, H)
    ctx.set_scene_dict(sc)
    for rank in range(8):
        ctx.set_partition(rank, 8)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        total += ctx.read_accum()
    ctx.set_partition(0, 1)
    ctx.render_schedule(inv, seeds, sc["eye"], B)
    full = ctx.read_accum()
    ctx.close()
    assert _bits_equal(total, full)


@pytest.mark.parametrize("fused", ["1", "0"])
def test_c4_precull_conservative_full_frame(frozen, monkeypatch, fused):
    """the padded-box pre-cull only skips rows that cannot win: the full C4 frame with and without it is the same
    bit for bit (every pixel, 2 samples, 12 bounces; tools/cull_check.py), in the fused slab form the library
    picks for this scene and in the plain form (SAIL_CULL_FMA=0). C4's bounce rays include about 1.4 M
    axis-parallel ones per sample (a zero direction component, infinite reciprocal)."""
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_FMA, int(fused))
    sc = frozen["C4"]
    W, H, B, spp = 3840, 2160, 12, 2
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    out = {}
    for cull in ("0", "1000"):
        monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, int(cull))
        ctx = capi.Context(W, H)
        ctx.set_scene_dict(sc)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        out[cull] = ctx.read_accum()
        ctx.close()
    assert _bits_equal(out["0"], out["1000"])



def _far_eye(sc):
    ctr = np.array(sc["center"], np.float64)
    d = np.array(sc["eye"], np.float64) - ctr
    sc["eye"] = [float(v) for v in ctr + d * (6000.0 / np.linalg.norm(d))]
    o = np.array(sc["objects"], np.float32).reshape(-1, 18)
    assert o[0, 0] == 1  # row 0: the room cube [0,0,-1]..[10,10,10] would hide the scene from outside:
    o[0, 1:7] = [0.0, 0.0, 11.0, 10.0, 10.0, 12.0]  # keep only a back wall behind it
    sc["objects"] = [float(v) for v in o.ravel()]
    return 0.1  # field of view (degrees) that still frames the scene


def _big_room(sc):
    o = np.array(sc["objects"], np.float32).reshape(-1, 18)
    assert o[0, 0] == 1  # row 0: the room cube [0,0,-1]..[10,10,10]
    o[0, 1:4] -= 500.0
    o[0, 4:7] += 500.0
    sc["objects"] = [float(v) for v in o.ravel()]
    return 55.0


def _tiny_quadrics(sc):
    o = np.array(sc["objects"], np.float32).reshape(-1, 18)
    sph = o[:, 0] == 2  # Sphere rows: 2, c3, r (slot 4)
    qd = (o[:, 0] == 4) | (o[:, 0] == 5)  # Cone / Cylinder rows: id, p3, h, r (slot 5)
    assert sph.any() and qd.any()
    o[sph, 4] *= 0.01
    o[qd, 5] *= 0.01
    sc["objects"] = [float(v) for v in o.ravel()]
    return 55.0


@pytest.mark.parametrize("variant", ["far_eye", "big_room", "tiny_quadrics"])
def test_c4_precull_far_origins(frozen, monkeypatch, variant):
    """ray origins far from the primitives: the eye 6,000 units away (primary rays), the C4 room grown to
    1,010 units a side (bounce rays leaving its walls), or spheres, cones and cylinders shrunk 100x (origins
    many radii away). The reference's f32 quadric tests lose accuracy there
    (discriminant cancellation grows with the squared distance), so the padded pre-cull must still pass every
    row such a test can report as hit: with and without the pre-cull the frame is the same bit for bit, and
    it matches oracle crops"""
    sc = dict(frozen["C4"])
    fov = {"far_eye": _far_eye, "big_room": _big_room, "tiny_quadrics": _tiny_quadrics}[variant](sc)
    W, H, B, spp = 320, 180, 12, 2
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], fov, W / H, 1.0, 10000.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    out = {}
    for cull in ("0", "1000"):
        monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, int(cull))
        ctx = capi.Context(W, H)
        ctx.set_scene_dict(sc)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        out[cull] = ctx.read_accum()
        ctx.close()
    got = out["0"]
    assert got[..., :3].any()
    assert _bits_equal(out["0"], out["1000"]), int((out["0"] != out["1000"]).any(axis=2).sum())
    masks = capi.plugin_masks(sc["plugins"])
    c = 8
    for x0, y0 in [(W // 2 - c // 2, H // 2 - c // 2), (W // 3, H // 3), (0, 0)]:
        want = np.zeros((H, W, 4), np.float32)
        oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, crop=(x0, y0, c, c), accum=want)
        assert _bits_equal(got[y0:y0 + c, x0:x0 + c], want[y0:y0 + c, x0:x0 + c]), (x0, y0)
