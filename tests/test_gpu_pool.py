"""The path-pool kernels (traceTilePool: a pool of paths per workgroup in LDS, waves shaded one class at a time, every
sample staged and added in sample order by sail_accum_kernel) against the CPU oracle, bit for bit, through the C ABI
with SAIL_DEBUG_PATH_POOL. They serve the Cornell (C1/C2/C5) and room (C3, UI) plugin sets; every other scene keeps its
kernel. Needs an MI355X."""
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
def gpu():
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    return True


def bit_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def _render(sc, W, H, spp, B, pool=1, mode=capi.ACCUM_SUM, aov=False, launch=None, groups=0, part=None):
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    ctx = capi.Context(W, H, flags=(capi.FLAG_AOV if aov else 0) | capi.FLAG_SEGMENT_COUNT)
    try:
        ctx.set_debug(capi.DEBUG_PATH_POOL, pool)
        if groups:
            ctx.set_debug(capi.DEBUG_SAMPLE_GROUPS, groups)
        ctx.set_scene_dict(sc)
        if mode != capi.ACCUM_SUM:
            ctx.set_accum_mode(mode)
        if launch:
            ctx.set_launch_samples(launch)
        if part:
            ctx.set_partition(*part)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
        st = ctx.stats()
        name = ctx.kernel_name()
        gaov = ctx.readback(aov=True)[1:] if aov else None
    finally:
        ctx.close()
    return got, st, name, gaov, inv, seeds


def _oracle(sc, W, H, inv, seeds, B, mode=capi.ACCUM_SUM, aov=False):
    ao = {capi.ACCUM_SUM: oracle.ACC_SUM, capi.ACCUM_MIX: oracle.ACC_MIX, capi.ACCUM_COMPAT8: oracle.ACC_COMPAT8}[mode]
    oracle.reset_counters()
    res = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, accum_mode=ao, aov=aov)
    segs, _ = oracle.counters()
    return res, segs


@pytest.mark.parametrize("name,W,H,spp,B,launch,groups", [
    ("C1", 48, 32, 5, 8, 3, 0),     # Cornell set
    ("C1", 33, 17, 4, 8, None, 1),  # ragged tiles, one group: the whole launch in one pool
    ("C1", 70, 40, 7, 8, 7, 5),     # five groups of two samples (the last one short)
    ("C1g", 24, 24, 3, 16, None, 0),
    ("C3", 40, 40, 4, 8, 3, 0),     # room set: lights, textures, every material
    ("C3", 37, 21, 6, 8, None, 2),
    ("UI", 48, 48, 4, 5, None, 0),
])
def test_pool_bit_exact(gpu, fixtures, name, W, H, spp, B, launch, groups):
    sc = fixtures["scenes"][name]
    got, st, kname, _, inv, seeds = _render(sc, W, H, spp, B, launch=launch, groups=groups)
    want, segs = _oracle(sc, W, H, inv, seeds, B)
    assert kname.endswith("_pool"), kname
    assert bit_equal(got, want).all(), f"{name}: {(~bit_equal(got, want)).any(axis=2).sum()} pixels differ"
    assert st.segments == segs, "exact segment counter differs from the oracle's loop count"
    assert st.samples == spp


@pytest.mark.parametrize("mode", [capi.ACCUM_MIX, capi.ACCUM_COMPAT8])
def test_pool_running_mean_modes(gpu, fixtures, mode):
    sc = fixtures["scenes"]["UI"]
    got, _, _, _, inv, seeds = _render(sc, 40, 40, 6, 5, mode=mode, launch=4)
    want, _ = _oracle(sc, 40, 40, inv, seeds, 5, mode=mode)
    assert bit_equal(got, want).all()


@pytest.mark.parametrize("name", ["C1", "C3"])
def test_pool_aovs(gpu, fixtures, name):
    """the AOVs of the launch's last sample: written by whichever lane carries that sample's path at its first hit"""
    sc = fixtures["scenes"][name]
    got, _, _, gaov, inv, seeds = _render(sc, 32, 32, 3, 4, aov=True)
    (want, wn, wp), _ = _oracle(sc, 32, 32, inv, seeds, 4, aov=True)
    assert bit_equal(got, want).all()
    assert bit_equal(gaov[0], wn).all() and bit_equal(gaov[1], wp).all()


@pytest.mark.parametrize("B", [0, 1, 2])
def test_pool_short_paths(gpu, fixtures, B):
    """no bounce (every sample's radiance 0), one bounce (every path ends after its first shading, shadeLast), two"""
    sc = fixtures["scenes"]["C3"]
    got, st, _, _, inv, seeds = _render(sc, 24, 20, 3, B)
    want, segs = _oracle(sc, 24, 20, inv, seeds, B)
    assert bit_equal(got, want).all()
    assert st.segments == segs


def test_pool_tile_partition_and_generic_fallback(gpu, fixtures):
    """a 3-rank tile partition with the pool sums to the 1-rank frame; a scene outside both plugin sets keeps the
    generic kernel (and its bits) with the switch on"""
    sc = fixtures["scenes"]["C1"]
    W, H, spp, B = 150, 70, 3, 5
    parts = [_render(sc, W, H, spp, B, part=(r, 3))[0] for r in range(3)]
    full, _, _, _, inv, seeds = _render(sc, W, H, spp, B)
    want, _ = _oracle(sc, W, H, inv, seeds, B)
    assert bit_equal(sum(parts), full).all() and bit_equal(full, want).all()
    sa = fixtures["scenes"]["ALL"]
    got, _, kname, _, inv, seeds = _render(sa, 32, 24, 2, 5)
    assert "pool" not in kname
    assert bit_equal(got, _oracle(sa, 32, 24, inv, seeds, 5)[0]).all()


@pytest.mark.parametrize("cfg,name,W,H,B,spp", [("C2", "C1", 1920, 1080, 8, 3), ("C3", "C3", 1920, 1080, 8, 2)])
def test_pool_full_frame(gpu, cfg, name, W, H, B, spp):
    """BASELINE's full 1080p frames with the pool: every pixel counts each sample once, the frame equals the
    compacting kernel's bit for bit, and oracle crops match"""
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        sc = dict(json.load(f)[name])
    sc["mvp_rowmajor"] = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0).tolist()
    got, _, kname, _, inv, seeds = _render(sc, W, H, spp, B)
    base, _, kbase, _, _, _ = _render(sc, W, H, spp, B, pool=0)
    assert kname.endswith("_pool") and "pool" not in kbase
    assert (got[..., 3] == spp).all()
    assert bit_equal(got, base).all()
    rng = np.random.default_rng(zlib.crc32(cfg.encode()))
    masks = capi.plugin_masks(sc["plugins"])
    c = 8
    for x0, y0 in [(0, 0), (W - c, H - c)] + [(int(rng.integers(0, W - c)), int(rng.integers(0, H - c))) for _ in range(4)]:
        want = np.zeros((H, W, 4), np.float32)
        oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, crop=(x0, y0, c, c), accum=want)
        assert bit_equal(got[y0:y0 + c, x0:x0 + c], want[y0:y0 + c, x0:x0 + c]).all(), (cfg, x0, y0)
