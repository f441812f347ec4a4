"""HIP trace/filter kernels vs the CPU oracle (oracle/sail_oracle.cpp) through the C ABI. Needs an MI355X.

The bar is bit-exact agreement: both sides follow the reference's f32 expression order with contraction
off and the same bit-defined transcendental spec, so every pixel of the accumulated image must match.
The north-star tolerance (relative L2 < 1e-3 of the mean image) is asserted as well, as a backstop.
"""
import numpy as np
import pytest

import oracle
from sail_amd import capi

pytestmark = pytest.mark.gpu

L2_TOL = 1e-3  # north_star: per-pixel radiance match within 1e-3 relative L2


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (den if den > 0 else 1.0))


def bit_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return same


@pytest.fixture(scope="module")
def gpu():
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    return True


# ---- the bit-defined math spec ---------------------------------------------------------------------------
def _args(fn, rng, n):
    if fn in (0, 1, 2):   # sin/cos/tan: the hash RNG range (1e4..1e6) and sampling angles
        x = np.concatenate([rng.uniform(-1e6, 1e6, n // 2), rng.uniform(-7, 7, n // 2)])
        return x, None
    if fn == 3:
        return rng.normal(size=n) * 10 ** rng.uniform(-3, 3, n), rng.normal(size=n) * 10 ** rng.uniform(-3, 3, n)
    if fn == 4:
        return rng.uniform(-1, 1, n), None
    if fn == 5:
        return rng.uniform(0, 4, n), rng.uniform(0.1, 3, n)
    if fn == 6:
        return rng.normal(size=n) * 10 ** rng.uniform(-3, 3, n), None
    if fn == 7:  # ordinary magnitudes plus raw bit patterns (negative, zero, subnormal, inf, NaN, huge)
        bits = rng.integers(0, 2 ** 32, n // 2, dtype=np.uint64).astype(np.uint32).view(np.float32)
        return np.concatenate([(np.abs(rng.normal(size=n // 2)) * 10 ** rng.uniform(-10, 10, n // 2)).astype(np.float32), bits]), None
    if fn in (9, 10, 12):  # min / max / clamp: signed zeros, NaN, inf and ordinary values, every pairing
        special = np.array([0.0, -0.0, 1.0, -1.0, np.nan, np.inf, -np.inf, 0.5, 2.0, -1e-30], np.float32)
        xs, ys = np.meshgrid(special, special)
        x = np.concatenate([xs.ravel(), rng.normal(size=n).astype(np.float32)])
        y = np.concatenate([ys.ravel(), rng.normal(size=n).astype(np.float32)])
        return x, y
    if fn in (11, 14):  # GLSL divide a * RN(1/b) and its reciprocal over raw bit patterns (all classes)
        bits = rng.integers(0, 2 ** 32, (2, n), dtype=np.uint64).astype(np.uint32)
        return bits[0].view(np.float32), bits[1].view(np.float32)
    return rng.normal(size=n) * 100, rng.normal(size=n) * 10 ** rng.uniform(-5, 5, n)


@pytest.mark.parametrize("fn", list(range(13)) + [14])
def test_math_spec_bit_exact(gpu, fn):
    rng = np.random.default_rng(1000 + fn)
    x, y = _args(fn, rng, 1 << 18)
    x = np.asarray(x).astype(np.float32)
    y = (np.zeros_like(x) if y is None else np.asarray(y)).astype(np.float32)
    got = capi.math_probe(fn, x, y)
    want = oracle.math(fn, x, y)
    same = bit_equal(got, want)
    assert same.all(), f"fn {fn}: {int((~same).sum())} mismatches, e.g. x={x[~same][:3]} gpu={got[~same][:3]} cpu={want[~same][:3]}"


def test_sqrt01_equals_ieee_sqrt_on_its_domain(gpu):
    """sail_math.h sqrt01 (no scaling / class fix-ups) is used only where the argument is +-0, NaN or in [2^-96, 1]
    (the argument bounds are in its header); there it must be the IEEE square root: every 1024th f32 of that range,
    the 2^16 patterns nearest 2^-96 and 1, both zeros and NaN payloads (tools/sqrt01_probe.hip checks every one of
    them on the GPU)"""
    one, lo = int(np.float32(1.0).view(np.uint32)), int(np.float32(2.0 ** -96).view(np.uint32))
    bits = np.concatenate([np.arange(lo, one + 1, 1024, dtype=np.uint64),
                           np.arange(lo, lo + (1 << 16), dtype=np.uint64), np.array([0], np.uint64),
                           np.arange(one - (1 << 16), one + 1, dtype=np.uint64),
                           np.array([0x80000000, 0x7FC00000, 0xFFC00000, 0x7F800001, 0x7FFFFFFF], np.uint64)])
    x = bits.astype(np.uint32).view(np.float32)
    got = capi.math_probe(15, x, np.zeros_like(x))
    want = oracle.math(7, x, np.zeros_like(x))
    same = bit_equal(got, want)
    assert same.all(), f"{int((~same).sum())} mismatches, e.g. bits {bits[~same][:4]}"


# ---- trace parity ------------------------------------------------------------------------------------------
CASES = [
    # scene, W, H, spp, bounces
    ("C1", 64, 48, 8, 5),
    ("C1", 33, 17, 4, 8),     # ragged: partial tiles
    ("C3", 40, 40, 4, 8),
    ("UI", 48, 48, 4, 5),
    ("ALL", 40, 32, 4, 6),
    ("C4", 32, 32, 2, 12),
    ("C1g", 16, 16, 2, 16),
]


def _render_both(fixtures, name, W, H, spp, B, mode=capi.ACCUM_SUM, k0=0, aov=False, launch=None):
    sc = fixtures["scenes"][name]
    mvp = np.array(sc["mvp_rowmajor"])
    inv, seeds = capi.schedule(mvp, W, H, k0, spp)
    masks = capi.plugin_masks(sc["plugins"])
    ctx = capi.Context(W, H, flags=(capi.FLAG_AOV if aov else 0) | capi.FLAG_SEGMENT_COUNT)
    try:
        ctx.set_scene_dict(sc)
        if mode != capi.ACCUM_SUM:
            ctx.set_accum_mode(mode)
        if launch:
            ctx.set_launch_samples(launch)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
        st = ctx.stats()
        gaov = ctx.readback(aov=True)[1:] if aov else None
    finally:
        ctx.close()
    oracle.reset_counters()
    res = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, k0=0, accum_mode=mode, aov=aov)
    segs, _ = oracle.counters()
    want = res[0] if aov else res
    return got, want, st, segs, gaov, (res[1:] if aov else None)


@pytest.mark.parametrize("name,W,H,spp,B", CASES)
def test_trace_sum_bit_exact(gpu, fixtures, name, W, H, spp, B):
    got, want, st, segs, _, _ = _render_both(fixtures, name, W, H, spp, B, launch=3)
    same = bit_equal(got, want)
    frac = 1.0 - same.mean()
    gm = got[..., :3] / np.maximum(got[..., 3:4], 1)
    wm = want[..., :3] / np.maximum(want[..., 3:4], 1)
    assert rel_l2(gm, wm) < L2_TOL
    assert same.all(), f"{name}: {frac:.4%} of channels differ; rel L2 {rel_l2(gm, wm):.3e}"
    assert st.segments == segs, "exact segment counter differs from the oracle's loop count"
    assert st.samples == spp


@pytest.mark.parametrize("mode", [capi.ACCUM_MIX, capi.ACCUM_COMPAT8])
def test_trace_running_mean_modes(gpu, fixtures, mode):
    got, want, *_ = _render_both(fixtures, "UI", 40, 40, 6, 5, mode=mode, launch=4)
    assert bit_equal(got, want).all()


def test_aovs(gpu, fixtures):
    got, want, _, _, gaov, waov = _render_both(fixtures, "C3", 32, 32, 3, 4, aov=True)
    assert bit_equal(got, want).all()
    assert bit_equal(gaov[0], waov[0]).all()
    assert bit_equal(gaov[1], waov[1]).all()


def test_tile_partition_sums_to_full_frame(gpu, fixtures):
    """Emulate world=3 on one GPU: the rank accumulators are disjoint and sum to the 1-rank frame."""
    sc = fixtures["scenes"]["C1"]
    W, H, spp, B = 150, 70, 3, 5
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    full = None
    parts = []
    for world in (1, 3):
        for rank in range(world):
            ctx = capi.Context(W, H)
            ctx.set_scene_dict(sc)
            ctx.set_partition(rank, world)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            a = ctx.read_accum()
            ctx.close()
            if world == 1:
                full = a
            else:
                parts.append(a)
    covered = sum((p[..., 3] > 0).astype(int) for p in parts)
    assert (covered == 1).all(), "every pixel belongs to exactly one rank"
    assert bit_equal(sum(parts), full).all()


def test_sample_partition(gpu, fixtures):
    sc = fixtures["scenes"]["C1"]
    W, H, spp, B = 48, 32, 6, 5
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    tot = np.zeros((H, W, 4), np.float32)
    for rank in range(2):
        ctx = capi.Context(W, H)
        ctx.set_scene_dict(sc)
        ctx.set_partition(rank, 2, capi.PART_SAMPLES)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        tot += ctx.read_accum()
        ctx.close()
    ref = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    # same samples, summed in a different order: equal to rounding
    assert np.allclose(tot, ref, rtol=1e-5, atol=1e-5)
    assert rel_l2(tot[..., :3] / tot[..., 3:4], ref[..., :3] / ref[..., 3:4]) < 1e-6


# ---- display filter ------------------------------------------------------------------------------------------
def _weights(fixtures, name):
    return np.array([float(x) for x in fixtures["filters"][name]["weight_text"]], dtype=np.float32)


@pytest.mark.parametrize("kind,fname,r,gamma", [
    (capi.FILTER_COLOR, None, 0, 2.2), (capi.FILTER_GAMMA, None, 0, 2.2), (capi.FILTER_TONEMAPPING, None, 0, 2.2),
    (capi.FILTER_WINDOW, "gaussian", (1.5, 2.5), 2.2), (capi.FILTER_WINDOW, "sinc", (3.0, 3.0), 2.2),
    (capi.FILTER_WINDOW, "box", (1.5, 1.5), 2.2), (capi.FILTER_WINDOW, "mitchell", (2.0, 2.0), 2.2),
    (capi.FILTER_WINDOW, "triangle", (2.0, 2.0), 2.2), (capi.FILTER_GAMMA, None, 0, 1.8),
])
def test_filter_bit_exact(gpu, fixtures, kind, fname, r, gamma):
    sc = fixtures["scenes"]["C3"]
    W, H, spp, B = 45, 37, 3, 5
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    ctx = capi.Context(W, H)
    ctx.set_scene_dict(sc)
    ctx.render_schedule(inv, seeds, sc["eye"], B)
    w = _weights(fixtures, fname) if fname else None
    rx, ry = r if fname else (0.0, 0.0)
    got, got8 = ctx.filter(kind, w, rx, ry, gamma, want_u8=True)
    acc = ctx.read_accum()
    ctx.close()
    mean = acc.copy()
    mean[..., :3] = acc[..., :3] / acc[..., 3:4]
    want = oracle.filter_image(mean, kind, w, rx, ry, gamma)
    assert bit_equal(got, want).all()
    want8 = np.floor(np.clip(want[..., :3], 0, 1) * 255.0 + 0.5).astype(np.uint8)
    assert (got8[..., :3] == want8).all()


@pytest.mark.parametrize("cull", ["0", "1000"])
def test_update_objects_and_reset(gpu, fixtures, monkeypatch, cull):
    """Tracer.updateObjects path (tracer.js:25-40): new rows, accumulation restarts (with the pre-cull kernel
    forced on, the candidate sweep's per-chunk type masks are re-uploaded with the rows)."""
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, int(cull))
    sc = fixtures["scenes"]["C1"]
    W, H = 32, 32
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, 2)
    moved = np.array(sc["objects"], dtype=np.float32).reshape(sc["n"], 18)
    moved[2, 1] += 0.5  # sphere centre x
    ctx = capi.Context(W, H)
    ctx.set_scene_dict(sc)
    ctx.render_schedule(inv, seeds, sc["eye"], 4)
    ctx.lib.sail_update_objects(ctx.h, capi._ptr(moved.reshape(-1)), sc["n"])
    ctx.render_schedule(inv, seeds, sc["eye"], 4)
    got = ctx.read_accum()
    ctx.close()
    sc2 = dict(sc, objects=moved.reshape(-1).tolist())
    want = oracle.render(sc2, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], 4)
    assert bit_equal(got, want).all()


# ---- AOV display filters: wavelet.glsl (a-trous), normal.glsl, position.glsl ------------------------------------
@pytest.mark.parametrize("kind,r", [(capi.FILTER_WAVELET, (2.0, 2.0)), (capi.FILTER_WAVELET, (3.5, 1.25)),
                                    (capi.FILTER_NORMAL, (0.0, 0.0)), (capi.FILTER_POSITION, (0.0, 0.0))])
def test_aov_filters_bit_exact(gpu, fixtures, kind, r):
    sc = fixtures["scenes"]["C3"]
    W, H, spp, B = 41, 35, 3, 5
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    ctx = capi.Context(W, H, flags=capi.FLAG_AOV)
    ctx.set_scene_dict(sc)
    ctx.render_schedule(inv, seeds, sc["eye"], B)
    got, got8 = ctx.filter(kind, None, r[0], r[1], 2.2, want_u8=True)
    mean, nrm, pos = ctx.readback(aov=True)
    ctx.close()
    want = oracle.filter_aov(mean, nrm, pos, kind, r[0], r[1])
    assert bit_equal(got, want).all()
    want8 = np.floor(np.clip(want[..., :3], 0, 1) * 255.0 + 0.5).astype(np.uint8)
    assert (got8[..., :3] == want8).all()
    if kind == capi.FILTER_WAVELET:
        assert np.isfinite(got).all()


def test_aov_filter_needs_aov_flag(gpu, fixtures):
    ctx = capi.Context(8, 8)
    ctx.set_scene_dict(fixtures["scenes"]["C1"])
    with pytest.raises(RuntimeError):
        ctx.filter(capi.FILTER_WAVELET, None, 2.0, 2.0)
    ctx.close()


# ---- picking: sail_pick (GPU) vs the oracle's intersectObjects -------------------------------------------------
def _pick_rays(sc, W, H, count, rng):
    """camera rays through random pixels (Ray.generate, pickup.js:11-14: inverse(P*MV) * (x, y, 0, 1) / w - eye,
    not normalised) plus rays from random interior points in random directions"""
    mvp = np.array(sc["mvp_rowmajor"])
    inv = np.linalg.inv(mvp)
    eye = np.array(sc["eye"], dtype=np.float64)
    xs = rng.uniform(-1, 1, count // 2)
    ys = rng.uniform(-1, 1, count // 2)
    p = inv @ np.stack([xs, ys, np.zeros_like(xs), np.ones_like(xs)])
    d = (p[:3] / p[3]).T - eye
    cam = np.concatenate([np.tile(eye, (len(d), 1)), d], axis=1)
    o = rng.uniform(0.5, 5.0, (count - len(d), 3))
    dd = rng.normal(size=(count - len(d), 3))
    return np.concatenate([cam, np.concatenate([o, dd], axis=1)]).astype(np.float32)


@pytest.mark.parametrize("name", ["C1", "C3", "C4", "ALL", "UI"])
def test_pick_matches_oracle(gpu, fixtures, name):
    sc = fixtures["scenes"][name]
    rays = _pick_rays(sc, 64, 64, 4096, np.random.default_rng(5))
    ctx = capi.Context(16, 16)
    ctx.set_scene_dict(sc)
    idx, t = ctx.pick(rays)
    ctx.close()
    widx, wt = oracle.pick(sc, capi.plugin_masks(sc["plugins"])[0], rays)
    assert np.array_equal(idx, widx)
    assert np.array_equal(t.view(np.uint32), wt.view(np.uint32))
    assert (idx >= 0).mean() > 0.5


# ---- the padded-box pre-cull (scenes with >= 8 primitives) must not change a single bit -----------------------
@pytest.mark.parametrize("name,W,H,spp,B", [("C1", 48, 32, 4, 5), ("C3", 40, 40, 3, 8), ("ALL", 40, 32, 3, 6),
                                            ("UI", 32, 32, 3, 5), ("C4", 24, 24, 2, 12)])
@pytest.mark.parametrize("cull", ["0", "1000"])
def test_precull_forced_on_and_off(gpu, fixtures, monkeypatch, name, W, H, spp, B, cull):
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, int(cull))   # 0: cull every scene, 1000: never
    got, want, st, segs, _, _ = _render_both(fixtures, name, W, H, spp, B, launch=2)
    assert bit_equal(got, want).all()
    assert st.segments == segs


# ---- candidate sweep (pre-cull kernel): rows span three 64-row chunks, and every row has an identical twin,
# so equal distances from different rows are everywhere: the lower row must win, as in the in-order sweep ------
@pytest.mark.parametrize("cull", ["0", "1000"])
def test_candidate_sweep_chunks_and_ties(gpu, fixtures, monkeypatch, cull):
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, int(cull))
    sc = dict(fixtures["scenes"]["C4"])
    sc["objects"] = list(sc["objects"]) * 2
    sc["n"] = 2 * sc["n"]                       # 134 rows: chunks of 64, 64, 6
    fixtures = {"scenes": {"C4x2": sc}}
    got, want, st, segs, gaov, waov = _render_both(fixtures, "C4x2", 24, 16, 2, 8, aov=True, launch=2)
    assert bit_equal(got, want).all()
    assert bit_equal(gaov[0], waov[0]).all() and bit_equal(gaov[1], waov[1]).all()
    assert st.segments == segs


@pytest.mark.parametrize("extra_rows,extra_tp", [(0, 0), (6, 0), (0, 3), (6, 3)])
def test_precull_lds_table_limits(gpu, fixtures, extra_rows, extra_tp):
    """the pre-cull kernel's LDS copies hold scenes of up to 72 rows and texParams tables of up to 136 rows; past
    either limit that table is read from global memory: C4 (67 rows, 134 texParams rows) grown across each limit"""
    sc = dict(fixtures["scenes"]["C4"])
    assert sc["n"] + 6 > 72 and sc["tn"] + 3 > 136 and sc["n"] <= 72 and sc["tn"] <= 136
    objs, tp = list(sc["objects"]), list(sc["texparams"])
    sc["objects"] = objs + objs[18:18 * (1 + extra_rows)]       # duplicates of rows 1.. (ties: the lower row wins)
    sc["n"] = sc["n"] + extra_rows
    sc["texparams"] = tp + tp[:16 * extra_tp]
    sc["tn"] = sc["tn"] + extra_tp
    got, want, st, segs, gaov, waov = _render_both({"scenes": {"C4L": sc}}, "C4L", 40, 32, 2, 6, aov=True, launch=2)
    assert bit_equal(got, want).all()
    assert bit_equal(gaov[0], waov[0]).all() and bit_equal(gaov[1], waov[1]).all()
    assert st.segments == segs


# ---- plugin-set kernels: the Cornell-box kernel (C1 scenes by default) and the generic one agree bit for bit --
@pytest.mark.parametrize("force", ["0", "1"])
def test_plugin_set_kernels(gpu, fixtures, monkeypatch, force):
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_FORCE_GENERIC, int(force))
    got, want, st, segs, _, _ = _render_both(fixtures, "C1", 56, 40, 4, 6, launch=3)
    assert bit_equal(got, want).all()
    assert st.segments == segs


def test_kernel_selection(gpu, fixtures):
    """plugin-set dispatch: the smallest precompiled kernel covering the scene (sail_kernel_name)"""
    want = {"C1": "sail_trace_kernel_cornell", "C1g": "sail_trace_kernel_cornell", "C3": "sail_trace_kernel_room",
            "UI": "sail_trace_kernel_room", "C4": "sail_trace_kernel_cull"}
    for name, k in want.items():
        ctx = capi.Context(8, 8)
        ctx.set_scene_dict(fixtures["scenes"][name])
        assert ctx.kernel_name() == k, name
        ctx.close()


# ---- the wavefront split of the pre-cull path (study switch): bit-identical to the megakernel and the oracle ------
@pytest.mark.parametrize("name,W,H,spp,B,mode", [("C4", 70, 46, 3, 12, capi.ACCUM_SUM), ("ALL", 40, 32, 4, 6, capi.ACCUM_MIX),
                                                 ("AREA", 36, 30, 3, 5, capi.ACCUM_SUM), ("C3", 40, 40, 3, 8, capi.ACCUM_COMPAT8)])
def test_wavefront_split_bit_exact(gpu, fixtures, monkeypatch, name, W, H, spp, B, mode):
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_WAVEFRONT, 1)
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, 0)  # every scene on the pre-cull path
    got, want, st, segs, gaov, waov = _render_both(fixtures, name, W, H, spp, B, mode=mode, aov=True, launch=2)
    assert bit_equal(got, want).all()
    assert bit_equal(gaov[0], waov[0]).all() and bit_equal(gaov[1], waov[1]).all()
    assert st.segments == segs


# ---- sample groups (small per-rank frames): staged samples added in order are bit-identical ---------------------
@pytest.mark.parametrize("groups", [0, 3, 4])
@pytest.mark.parametrize("rank,world", [(0, 1), (1, 3)])
def test_precull_sample_groups_multi_tile(gpu, fixtures, groups, rank, world):
    """the pre-cull kernel's grouped form (1,024-thread workgroups, 16x64 strips) stages each sample in the 16x16
    slot order sail_accum_kernel reads: several tiles, ragged edges, a tile rank, the host's own group rule (0)"""
    sc = fixtures["scenes"]["C4"]
    W, H, B, spp = 150, 140, 4, 6
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    ctx = capi.Context(W, H, flags=capi.FLAG_AOV)
    try:
        if groups:
            ctx.set_debug(capi.DEBUG_SAMPLE_GROUPS, groups)
        ctx.set_scene_dict(sc)
        assert ctx.kernel_name() == "sail_trace_kernel_cull"
        ctx.set_partition(rank, world)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got, gn, gp = ctx.readback(aov=True)
        acc = ctx.read_accum()
    finally:
        ctx.close()
    want, wn, wp = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, aov=True)
    tx = (W + 63) // 64
    yy, xx = np.mgrid[0:H, 0:W]
    mine = (((yy // 64) * tx + xx // 64) % world) == rank
    assert bit_equal(acc[mine], want[mine]).all()
    assert (acc[~mine] == 0).all()
    assert bit_equal(gn[mine], wn[mine]).all() and bit_equal(gp[mine], wp[mine]).all()


@pytest.mark.parametrize("name", ["C1", "C3", "C4"])   # C4: the pre-cull kernel, 1024 threads when ungrouped
@pytest.mark.parametrize("groups", ["1", "2", "5"])
@pytest.mark.parametrize("mode", [capi.ACCUM_SUM, capi.ACCUM_MIX])
def test_sample_groups(gpu, fixtures, monkeypatch, name, groups, mode):
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_SAMPLE_GROUPS, int(groups))
    got, want, st, segs, gaov, waov = _render_both(fixtures, name, 40, 24, 7, 5, mode=mode, aov=True, launch=7)
    assert bit_equal(got, want).all()
    assert bit_equal(gaov[0], waov[0]).all() and bit_equal(gaov[1], waov[1]).all()
    assert st.segments == segs


# ---- category words outside the compiled sets (unknown, negative, NaN, huge): the zero material / texture paths,
# through the host-evaluated SailPrim.cats -------------------------------------------------------------------------
def test_odd_category_words(gpu, fixtures):
    sc = dict(fixtures["scenes"]["ALL"])
    tp = list(sc["texparams"])
    odd = [99.0, -5.0, float("nan"), 3e9, 31.0]
    for i, row in enumerate(range(0, sc["tn"], 2)):
        tp[row * 16] = odd[i % len(odd)]
    sc["texparams"] = tp
    got, want, st, segs, _, _ = _render_both({"scenes": {"ODD": sc}}, "ODD", 24, 20, 3, 6, launch=2)
    assert bit_equal(got, want).all()
    assert st.segments == segs


# ---- one sample per call (Renderer.render): the sample-record ring wraps after 4096 calls ---------------------------
@pytest.mark.parametrize("launch_spp", [1, 32])
def test_single_sample_frames_ring_wrap(gpu, fixtures, launch_spp):
    """4,100 one-sample frames across the wrap of the 4,096-record sample ring: one launch per frame (launch_spp 1)
    or queued 32 to a launch (sail_render's batching); the same frame either way"""
    sc = fixtures["scenes"]["C1"]
    W, H, B, spp = 8, 6, 4, 4100
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    ctx = capi.Context(W, H, flags=capi.FLAG_SEGMENT_COUNT)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_launch_samples(launch_spp)
        for k in range(spp):
            ctx.render(inv[k], sc["eye"], float(seeds[k]), B)
        got = ctx.read_accum()
        st = ctx.stats()
    finally:
        ctx.close()
    oracle.reset_counters()
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    segs, _ = oracle.counters()
    assert bit_equal(got, want).all()
    assert st.segments == segs and st.launches == (spp + launch_spp - 1) // launch_spp


# ---- degenerate rays through the division spec's fallback paths: exactly axis-aligned directions (zero and
# negative-zero components: reciprocals +-inf), origins on primitive planes, subnormal / huge components --------
def _degenerate_rays(sc, rng):
    objs = np.array(sc["objects"], np.float32).reshape(sc["n"], 18)
    pts = [objs[i, 1:4] for i in range(sc["n"])] + [objs[i, 4:7] for i in range(sc["n"])]  # row coordinates
    pts += [np.array(sc["eye"], np.float32)]
    dirs = []
    for ax in range(3):
        for s in (1.0, -1.0):
            d = np.zeros(3, np.float32); d[ax] = s; dirs.append(d)
            d2 = np.array([-0.0, -0.0, -0.0], np.float32); d2[ax] = s; dirs.append(d2)
    dirs += [np.array([1e-39, 1.0, 0.0], np.float32), np.array([3e38, 1e-3, -2.0], np.float32),
             np.array([0.0, 0.0, 0.0], np.float32), np.array([1.0, 1.0, 0.0], np.float32)]
    rays = []
    for p in pts:
        for d in dirs:
            rays.append(np.concatenate([p, d]))
            jit = p + rng.normal(size=3).astype(np.float32) * np.float32(0.25)
            rays.append(np.concatenate([jit, d]))
    return np.array(rays, np.float32)


@pytest.mark.parametrize("name", ["C1", "C3", "C4", "ALL"])
def test_pick_degenerate_rays(gpu, fixtures, name):
    sc = fixtures["scenes"][name]
    rays = _degenerate_rays(sc, np.random.default_rng(11))
    ctx = capi.Context(8, 8)
    ctx.set_scene_dict(sc)
    idx, t = ctx.pick(rays)
    ctx.close()
    widx, wt = oracle.pick(sc, capi.plugin_masks(sc["plugins"])[0], rays)
    assert np.array_equal(idx, widx)
    assert bit_equal(t, wt).all()


# ---- unusual viewpoints: inside the mirror sphere, on the light's plane, in a Cornell-box corner, looking straight
# along an axis (primary rays with exact zero components), outside the closed box --------------------------------
VIEWS = [("inside sphere", [2.0, 1.25, 2.7], [2.78, 2.73, 2.79]),
         ("light plane", [2.78, 5.487, 2.8], [2.78, 0.0, 3.3]),
         ("corner", [0.0, 0.0, -7.0], [5.56, 5.488, 5.592]),
         ("axis", [2.78, 2.73, -6.0], [2.78, 2.73, 5.0]),
         ("outside", [2.78, 2.73, -20.0], [2.78, 2.73, 2.79])]


@pytest.mark.parametrize("label,eye,center", VIEWS)
def test_unusual_viewpoints(gpu, fixtures, label, eye, center):
    sc = dict(fixtures["scenes"]["C1"])
    sc["eye"] = eye
    sc["mvp_rowmajor"] = capi.camera(eye, center, [0, 1, 0], 55.0, 1.0, 1.0, 100.0).tolist()
    got, want, st, segs, gaov, waov = _render_both({"scenes": {"V": sc}}, "V", 33, 21, 3, 6, aov=True, launch=2)
    assert bit_equal(got, want).all(), label
    assert bit_equal(gaov[0], waov[0]).all() and bit_equal(gaov[1], waov[1]).all(), label
    assert st.segments == segs, label


# ---- coverage scenes (tests/golden/make_fixtures.js, rows from the reference serializer) ---------------------------
# AREA: Disk / Sphere / Rectangle area lights (sampled with a pdf); AREA0: Cube / Cone / Cylinder / Hyperboloid /
# Paraboloid / Cornellbox area lights, whose samplers never write pdf (cube.glsl:50-52 ...; defined as 0, so their
# light samples are inf / NaN, which must match bit for bit too); N1 / N1S: one primitive (row coordinate 0/0);
# N0: no primitive (every primary ray misses); BILERP: the Bilerp texture on four UV maps
COVERAGE = [("AREA", 40, 32, 4, 6), ("AREA0", 40, 32, 1, 1), ("AREA0", 40, 32, 2, 3), ("AREA0", 32, 24, 4, 8),
            ("N1", 40, 32, 4, 6), ("N1S", 40, 32, 4, 5), ("N0", 24, 16, 2, 5), ("BILERP", 40, 32, 4, 6)]


@pytest.mark.parametrize("name,W,H,spp,B", COVERAGE)
@pytest.mark.parametrize("kernel", ["default", "generic", "cull"])
def test_coverage_scenes_bit_exact(gpu, fixtures, monkeypatch, name, W, H, spp, B, kernel):
    if kernel == "generic":
        monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_FORCE_GENERIC, 1)
        monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, 1000)
    elif kernel == "cull":
        monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, 0)
    got, want, st, segs, gaov, waov = _render_both(fixtures, name, W, H, spp, B, aov=True, launch=3)
    same = bit_equal(got, want)
    assert same.all(), f"{name}: {int((~same).sum())} channels differ"
    assert bit_equal(gaov[0], waov[0]).all() and bit_equal(gaov[1], waov[1]).all()
    assert st.segments == segs
    fin = np.isfinite(want[..., :3])
    if name == "AREA0":   # the pdf-less samplers: inf / NaN where a matte vertex sampled one, finite elsewhere
        assert (~fin).any() and fin.mean() > 0.5
    else:
        assert fin.all()
    if name == "N0":
        assert (want[..., :3] == 0).all() and segs == W * H * spp


@pytest.mark.parametrize("name", ["AREA0", "ALL", "BILERP", "N1"])
def test_cull_kernel_ungrouped_small_frames(gpu, fixtures, monkeypatch, name):
    """The ungrouped pre-cull kernel runs 1024-thread workgroups (16 x 64 pixel strips, sail_trace.hip SAIL_CULL_NT):
    forced on for small scenes and ragged frames (sample groups off), it must stay bit-exact"""
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_CULL_MIN_PRIMS, 0)
    monkeypatch.setitem(capi.DEBUG_DEFAULTS, capi.DEBUG_SAMPLE_GROUPS, 1)
    got, want, st, segs, gaov, waov = _render_both(fixtures, name, 70, 83, 3, 6, aov=True, launch=2)
    assert bit_equal(got, want).all()
    assert bit_equal(gaov[0], waov[0]).all() and bit_equal(gaov[1], waov[1]).all()
    assert st.segments == segs


def test_coverage_kernel_selection(gpu, fixtures):
    want = {"AREA": "sail_trace_kernel", "AREA0": "sail_trace_kernel_cull", "N1": "sail_trace_kernel_room",
            "N1S": "sail_trace_kernel_cornell", "N0": "sail_trace_kernel_room", "BILERP": "sail_trace_kernel"}
    for name, k in want.items():
        ctx = capi.Context(8, 8)
        ctx.set_scene_dict(fixtures["scenes"][name])
        assert ctx.kernel_name() == k, name
        ctx.close()


# ---- the last-bounce shortcut (sail_trace.hip shadeLast) on the materials it must decline or pass NaN through ----
# C1 uses the Cornell kernel (no light plugin), where shadeLast handles every path: Oren-Nayar matte (sigma > 0) must
# decline to the full bounce (f needs the sampled direction); an infinite kd makes the matte f inf / NaN, which the
# last bounce's direct term (0 + 0 * f) must carry into the radiance exactly as the full bounce does.
LAST_BOUNCE_MATS = {
    "oren_nayar": lambda tp: tp.__setitem__((slice(None), slice(2, 5)), np.where(tp[:, :1] == 1, [20.0, 0.6, 0.35], tp[:, 2:5])),
    "inf_kd": lambda tp: tp.__setitem__((0, 1), np.inf),
    "huge_kd": lambda tp: tp.__setitem__((2, 1), 3e38),
}


@pytest.mark.parametrize("variant", sorted(LAST_BOUNCE_MATS))
@pytest.mark.parametrize("B", [1, 3])
def test_last_bounce_shortcut_edge_materials(gpu, fixtures, variant, B):
    sc = dict(fixtures["scenes"]["C1"])
    tp = np.array(sc["texparams"], dtype=np.float32).reshape(sc["tn"], 16)
    LAST_BOUNCE_MATS[variant](tp)
    sc["texparams"] = tp.reshape(-1).tolist()
    W, H, spp = 24, 20, 3
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    ctx = capi.Context(W, H)
    try:
        ctx.set_scene_dict(sc)
        assert ctx.kernel_name() == "sail_trace_kernel_cornell"
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
    finally:
        ctx.close()
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    same = bit_equal(got, want)
    assert same.all(), f"{variant}, {B} bounces: {int((~same).sum())} channels differ"
    if variant == "inf_kd":
        assert np.isnan(got[..., :3]).any() or np.isinf(got[..., :3]).any()


# ---- the phase-timing build (the one instrumentation switch left in sail_trace.hip) ------------------------------
@pytest.mark.parametrize("name,W,H,spp,B", [("C1", 40, 24, 3, 6), ("C3", 40, 24, 3, 5), ("C4", 40, 24, 2, 6)])
def test_phase_timing_build_bit_exact(gpu, fixtures, monkeypatch, name, W, H, spp, B):
    """libsail_hip_phase.so (-DSAIL_PHASE_TIMING=1, tools/phase_profile.py) renders the oracle's bits in all three
    kernel families, through run-time kernels compiled instrumented as well, and its per-phase wave timers advance
    (summed over the library's kernels and the loaded run-time modules)"""
    import ctypes
    import os
    path = os.path.join(os.path.dirname(capi.LIB_PATH), "libsail_hip_phase.so")
    lib = capi.load(path)
    lib.sail_phase_read.restype = ctypes.c_int
    lib.sail_phase_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    monkeypatch.setattr(capi, "_lib", lib)
    buf = (ctypes.c_ulonglong * 12)()
    assert lib.sail_phase_read(buf, 1) == 0
    sc = fixtures["scenes"][name]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    ctx = capi.Context(W, H)
    try:
        assert ctx.lib is lib
        ctx.set_scene_dict(sc)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
        kname = ctx.kernel_name()
    finally:
        ctx.close()
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    assert bit_equal(got, want).all()
    assert "_jit" in kname, kname
    assert lib.sail_phase_read(buf, 0) == 0
    assert buf[0] > 0 and buf[1] > 0  # sweep and hit-record phases were timed


# ---- per-plugin-set kernels compiled at run time (sail_jit.cpp) ------------------------------------------------
@pytest.mark.parametrize("name,W,H,spp,B", [("ALL", 40, 32, 3, 6), ("AREA", 36, 28, 3, 5), ("BILERP", 33, 17, 2, 5)])
def test_jit_kernel_bit_exact(gpu, fixtures, name, W, H, spp, B):
    """a scene outside the precompiled Cornell / room sets runs a kernel hipRTC compiled for exactly its plugin set
    (at sail_set_scene, as the reference links its per-scene program in Tracer.update); its frame equals the
    oracle's and the all-plugin kernel's bit for bit, in one launch and in sample groups"""
    sc = fixtures["scenes"][name]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    out = {}
    one = {capi.DEBUG_SAMPLE_GROUPS: 1}  # a small frame would otherwise split its samples into groups
    plain = {capi.DEBUG_JIT: 1}  # the all-plugin kernel's form (SAIL_JIT_MODE_FLAT)
    room = {capi.DEBUG_JIT: 1 | 8}  # the room kernel's form (SAIL_JIT_MODE_ROOM, the default)
    for label, dbg in (("jit", {**plain, **one}), ("jit_groups", {**plain, capi.DEBUG_SAMPLE_GROUPS: 2}),
                       ("generic", {capi.DEBUG_JIT: 0, **one}),
                       ("jit_room", {**room, **one}), ("jit_room_groups", {**room, capi.DEBUG_SAMPLE_GROUPS: 3})):
        ctx = capi.Context(W, H, debug=dbg)
        try:
            ctx.set_scene_dict(sc)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            out[label] = (ctx.read_accum(), ctx.kernel_name())
        finally:
            ctx.close()
    assert out["jit"][1] == out["jit_room"][1] == "sail_trace_kernel_jit", out["jit"][1]
    assert out["jit_groups"][1] == out["jit_room_groups"][1] == "sail_trace_kernel_jit_grouped"
    assert out["generic"][1] == "sail_trace_kernel"
    for label, (acc, _) in out.items():
        assert bit_equal(acc, want).all(), label


def test_jit_kernel_multi_device_and_update(gpu, fixtures):
    """the run-time kernel on a multi-device context (one module per device, the code object compiled once)"""
    sc = fixtures["scenes"]["ALL"]
    W, H, spp, B = 48, 40, 2, 5
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    ctx = capi.Context(W, H, devices=[0, 0])
    try:
        ctx.set_scene_dict(sc)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        assert bit_equal(ctx.read_accum(), want).all()
        assert ctx.kernel_name().startswith("sail_trace_kernel_jit")
    finally:
        ctx.close()


@pytest.mark.parametrize("name,W,H,spp,B", [("C3", 40, 36, 3, 6), ("UI", 36, 28, 3, 5)])
def test_jit_room_set_kernel_bit_exact(gpu, fixtures, name, W, H, spp, B):
    """SAIL_DEBUG_JIT bit 4: a scene of the room kernel's set compiled for exactly its plugin set in the room kernel's
    form (first sample group accumulating at home, the others staged); bit-exact against the oracle and the
    precompiled room kernel, in one launch and in 2 and 3 sample groups"""
    sc = fixtures["scenes"][name]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    for dbg, kname in (({capi.DEBUG_JIT: 5, capi.DEBUG_SAMPLE_GROUPS: 1}, "sail_trace_kernel_jit"),
                       ({capi.DEBUG_JIT: 5, capi.DEBUG_SAMPLE_GROUPS: 2}, "sail_trace_kernel_jit_grouped"),
                       ({capi.DEBUG_JIT: 5, capi.DEBUG_SAMPLE_GROUPS: 3}, "sail_trace_kernel_jit_grouped"),
                       ({capi.DEBUG_JIT: 1, capi.DEBUG_SAMPLE_GROUPS: 2}, "sail_trace_kernel_room_grouped")):
        ctx = capi.Context(W, H, debug=dbg)
        try:
            ctx.set_scene_dict(sc)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            got = ctx.read_accum()
            assert ctx.kernel_name() == kname, (dbg, ctx.kernel_name())
        finally:
            ctx.close()
        assert bit_equal(got, want).all(), dbg


@pytest.mark.parametrize("name,W,H,spp,B", [("C1", 40, 24, 3, 6), ("C3", 40, 36, 3, 6), ("UI", 36, 28, 3, 5),
                                            ("ALL", 40, 32, 3, 6), ("BILERP", 33, 17, 2, 5), ("N1S", 24, 20, 2, 4)])
def test_jit_row_specialised_kernel_bit_exact(gpu, fixtures, name, W, H, spp, B):
    """SAIL_DEBUG_JIT bit 16: a flat scene compiled for its rows (count and shape types as constants: straight-line
    sweeps) in its family's form -- Cornell, room, or room form for the rest; bit-exact against the oracle, ungrouped
    and in 3 sample groups, and again after sail_update_objects moves the rows (same types: the same kernel)"""
    sc = fixtures["scenes"][name]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    for groups in (1, 3):
        ctx = capi.Context(W, H, debug={capi.DEBUG_JIT: 11 | 16, capi.DEBUG_SAMPLE_GROUPS: groups})
        try:
            ctx.set_scene_dict(sc)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            got = ctx.read_accum()
            assert ctx.kernel_name().startswith("sail_trace_kernel_jit"), ctx.kernel_name()
            assert bit_equal(got, want).all(), groups
            if groups == 3:
                rows = np.ascontiguousarray(np.asarray(sc["objects"], np.float32).reshape(-1))
                assert ctx.lib.sail_update_objects(ctx.h, capi._ptr(rows), sc["n"]) == 0  # Renderer.updateObjects
                ctx.render_schedule(inv, seeds, sc["eye"], B)
                assert bit_equal(ctx.read_accum(), want).all()
        finally:
            ctx.close()


def test_jit_row_kernel_recompiles_when_row_types_change(gpu, fixtures):
    """sail_update_objects that changes a row's shape type (C3's Cube and first Sphere rows swapped): the context
    compiles the kernel for the new rows at the next render, and the frame equals the oracle's for the new rows"""
    sc = dict(fixtures["scenes"]["C3"])
    W, H, spp, B = 36, 28, 2, 5
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    rows = np.asarray(sc["objects"], np.float32).reshape(sc["n"], 18)
    assert int(rows[1, 0]) == 1 and int(rows[2, 0]) == 2  # Cube, Sphere
    swapped = rows.copy()
    swapped[[1, 2]] = rows[[2, 1]]
    ctx = capi.Context(W, H, debug={capi.DEBUG_SAMPLE_GROUPS: 2})
    try:
        ctx.set_scene_dict(sc)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        first = ctx.read_accum()
        flat = np.ascontiguousarray(swapped.reshape(-1))
        assert ctx.lib.sail_update_objects(ctx.h, capi._ptr(flat), sc["n"]) == 0
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
        assert ctx.kernel_name().startswith("sail_trace_kernel_jit")
    finally:
        ctx.close()
    masks = capi.plugin_masks(sc["plugins"])
    assert bit_equal(first, oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B)).all()
    sc2 = dict(sc, objects=flat.tolist())
    assert bit_equal(got, oracle.render(sc2, masks, W, H, inv, seeds, sc["eye"], B)).all()


def test_jit_precull_kernel_bit_exact(gpu, fixtures):
    """SAIL_DEBUG_JIT bit 2: the pre-cull path (C4, 67 rows) compiled for exactly its plugin set, 1,024-thread
    workgroups like the precompiled pre-cull kernel; bit-exact against the oracle, with and without sample groups"""
    sc = fixtures["scenes"]["C4"]
    W, H, spp, B = 40, 24, 2, 6
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    for dbg, name in (({capi.DEBUG_JIT: 3, capi.DEBUG_SAMPLE_GROUPS: 1}, "sail_trace_kernel_cull_jit"),
                      ({capi.DEBUG_JIT: 3, capi.DEBUG_SAMPLE_GROUPS: 2}, "sail_trace_kernel_cull_jit_grouped"),
                      ({capi.DEBUG_JIT: 1, capi.DEBUG_SAMPLE_GROUPS: 1}, "sail_trace_kernel_cull")):
        ctx = capi.Context(W, H, debug=dbg)
        try:
            ctx.set_scene_dict(sc)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            got = ctx.read_accum()
            assert ctx.kernel_name() == name, (dbg, ctx.kernel_name())
        finally:
            ctx.close()
        assert bit_equal(got, want).all(), dbg


# ---- the scene's kernel built in the background ------------------------------------------------
def _reversed_c1(fixtures):
    """C1 with its object rows in reverse order: a row specialisation no other test and no shipped cache entry has"""
    sc = dict(fixtures["scenes"]["C1"])
    rows = np.asarray(sc["objects"], np.float32).reshape(sc["n"], 18)[::-1].copy()
    sc["objects"] = rows.reshape(-1).tolist()
    return sc


SWAP_CHILD = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
from sail_amd import capi
capi.set_jit_cache(sys.argv[2])
sc = json.loads(open(sys.argv[3]).read())
ctx = capi.Context(40, 24, debug={capi.DEBUG_JIT_WAIT: 0})
t0 = time.perf_counter()
ctx.set_scene_dict(sc)
dt = time.perf_counter() - t0
print(json.dumps({"set_scene_ms": dt * 1e3, "info": ctx.kernel_info()}))
ctx.close()
"""


def test_jit_swap_mid_frame_bit_exact(gpu, fixtures, tmp_path):
    """sail_set_scene returns at once (the reference's Renderer.update links in milliseconds, renderer.js:45-52) while the
    scene's kernel is built in the background; the first samples render on the precompiled Cornell kernel, the rest on
    the run-time kernel once it is loaded, and the frame across the swap equals the oracle's bit for bit. Then a new
    process with the now-warm disk cache loads the kernel inside sail_set_scene."""
    import json
    import os
    import subprocess
    import sys
    import time
    sc = _reversed_c1(fixtures)
    W, H, spp, B = 40, 24, 4, 6
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    cache = str(tmp_path / "jit")
    capi.set_jit_cache(cache)
    try:
        ctx = capi.Context(W, H, debug={capi.DEBUG_JIT_WAIT: 0})
        try:
            t0 = time.perf_counter()
            ctx.set_scene_dict(sc)
            cold_ms = (time.perf_counter() - t0) * 1e3
            assert ctx.kernel_info()["jit_state"] == capi.KERNEL_JIT_PENDING
            ctx.render_schedule(inv[:2], seeds[:2], sc["eye"], B)
            first = ctx.kernel_name()
            assert ctx.kernel_ready(-1)
            ctx.render_schedule(inv[2:], seeds[2:], sc["eye"], B)
            second = ctx.kernel_name()
            info = ctx.kernel_info()
            got = ctx.read_accum()
        finally:
            ctx.close()
    finally:
        capi.set_jit_cache(None)
    assert first.startswith("sail_trace_kernel_cornell"), first
    assert second.startswith("sail_trace_kernel_jit"), second
    assert info["jit_state"] == capi.KERNEL_JIT_READY and info["jit_from_cache"] == 0 and info["jit_compile_ms"] > 0
    assert bit_equal(got, want).all()
    assert cold_ms < 200.0, cold_ms
    assert len(os.listdir(cache)) == 1  # the code object went to the user cache
    scp = tmp_path / "scene.json"
    scp.write_text(json.dumps(sc))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", SWAP_CHILD, root, cache, str(scp)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    warm = json.loads(r.stdout.strip().splitlines()[-1])
    assert warm["info"]["jit_state"] == capi.KERNEL_JIT_READY and warm["info"]["jit_from_cache"] == 1, warm
    assert warm["info"]["jit_build_id"] == info["jit_build_id"], warm
    assert warm["set_scene_ms"] < 100.0, warm


def test_kernel_build_identity(gpu, fixtures):
    """sail_get_kernel_info: a run-time kernel's build id is its code object's hash (equal for equal specs, different
    for another spec), a precompiled kernel's is the library image's plus its name"""
    W, H, B = 32, 16, 4
    ids = {}
    for name, dbg in (("C1", {}), ("C3", {}), ("C1", {capi.DEBUG_JIT: 0})):
        sc = fixtures["scenes"][name]
        inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, 2)
        ctx = capi.Context(W, H, debug=dbg)
        try:
            ctx.set_scene_dict(sc)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            k = ctx.kernel_info()
            ids[(name, bool(dbg))] = (k["name"], k["build_id"], k["jit_build_id"])
        finally:
            ctx.close()
    (n1, b1, j1), (n3, b3, _), (n0, b0, j0) = ids[("C1", False)], ids[("C3", False)], ids[("C1", True)]
    assert n1.startswith("sail_trace_kernel_jit") and b1 == j1 and b1 != b3
    assert n0.startswith("sail_trace_kernel_cornell") and b0 != b1 and j0 == "0" * 16


def test_launch_samples_by_form(gpu, fixtures):
    """samples per launch default to the kernel form's (sail_set_launch_samples 0): the Cornell form with 16 samples in
    flight runs up to 1,024 per launch, a rank of 8 (1 in flight) and an explicit setting 64; the frame is the same bit
    for bit however the samples are split into launches"""
    sc = fixtures["scenes"]["C1"]
    W, H, B, spp = 1920, 1080, 3, 96
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    out = {}
    for label, launch, world in (("auto", None, 1), ("fixed", 64, 1), ("rank8", None, 8)):
        ctx = capi.Context(W, H)
        try:
            ctx.set_scene_dict(sc)
            if launch:
                ctx.set_launch_samples(launch)
            ctx.set_partition(0, world)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            out[label] = (ctx.read_accum(), ctx.stats().launches)
        finally:
            ctx.close()
    assert out["auto"][1] == 1 and out["fixed"][1] == 2 and out["rank8"][1] == 2, {k: v[1] for k, v in out.items()}
    assert bit_equal(out["auto"][0], out["fixed"][0]).all()
    mask = out["rank8"][0][..., 3] > 0  # rank 0's tiles
    assert mask.any() and bit_equal(out["rank8"][0][mask], out["auto"][0][mask]).all()


@pytest.mark.parametrize("mode", [capi.ACCUM_SUM, capi.ACCUM_MIX, capi.ACCUM_COMPAT8])
def test_whole_frame_launches_cross_a_launch_boundary(gpu, fixtures, mode):
    """the Cornell form with 16 samples in flight launches up to 1,024 samples at once: 1,100 samples run as 1,024 + 76,
    each pixel's running accumulator kept in LDS across the 64 + 5 sample steps, bit-exact against the oracle in every
    accumulation mode; and sail_set_launch_samples(0) returns a fixed launch size to the form's"""
    sc = fixtures["scenes"]["C1"]
    W, H, B, spp = 24, 16, 3, 1100
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, accum_mode=mode)
    ctx = capi.Context(W, H, debug={capi.DEBUG_JIT_NS: 16})
    try:
        ctx.set_accum_mode(mode)
        ctx.set_scene_dict(sc)
        ctx.set_launch_samples(64)
        ctx.set_launch_samples(0)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
        st = ctx.stats()
    finally:
        ctx.close()
    assert st.launches == 2
    assert bit_equal(got, want).all()


def test_cornell_form_follows_the_share_of_the_frame(gpu, fixtures):
    """the Cornell form holds 16 samples in flight for a large share of the frame and 1 for a rank of 8 (sail_capi.cpp
    jitNsFor): set_partition switches the run-time kernel, and back (both are in the cache shipped with the library)"""
    sc = fixtures["scenes"]["C1"]
    ctx = capi.Context(1920, 1080)
    try:
        ctx.set_scene_dict(sc)
        ids = []
        for world in (1, 8, 2, 1):
            ctx.set_partition(0, world)
            assert ctx.kernel_ready(-1)
            ids.append(ctx.kernel_info()["jit_build_id"])
        assert ids[0] == ids[2] == ids[3] != ids[1], ids
    finally:
        ctx.close()


@pytest.mark.parametrize("name,W,H,spp,B", [("C1", 37, 21, 7, 6), ("C3", 40, 36, 5, 6), ("C4", 36, 20, 5, 6),
                                            ("ALL", 33, 17, 3, 5)])
@pytest.mark.parametrize("ns,nt", [(4, 0), (16, 0), (16, 512), (4, 128), (1, 512)])
def test_samples_in_flight_bit_exact(gpu, fixtures, name, W, H, spp, B, ns, nt):
    """SAIL_DEBUG_JIT_NS: run-time kernels whose workgroups hold NS samples of 256 / NS pixels (1,024 / NS in the
    pre-cull form) -- each pixel's samples of a step added in sample order -- equal the oracle bit for bit: ragged frames,
    sample counts that are not a multiple of NS, 1 and 3 sample groups, the running-mean and 8-bit modes, and the AOVs
    of the launch's last sample"""
    sc = fixtures["scenes"][name]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    masks = capi.plugin_masks(sc["plugins"])
    for groups, mode in ((1, capi.ACCUM_SUM), (3, capi.ACCUM_SUM), (1, capi.ACCUM_MIX), (2, capi.ACCUM_COMPAT8)):
        dbg = {capi.DEBUG_JIT_NS: ns, capi.DEBUG_JIT_NT: nt, capi.DEBUG_SAMPLE_GROUPS: groups}
        ctx = capi.Context(W, H, flags=capi.FLAG_AOV, debug=dbg)
        try:
            ctx.set_accum_mode(mode)
            ctx.set_scene_dict(sc)
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            assert ctx.kernel_name().startswith(("sail_trace_kernel_jit", "sail_trace_kernel_cull_jit")), ctx.kernel_name()
            got = ctx.read_accum()
            _, gn, gp = ctx.readback(aov=True)
        finally:
            ctx.close()
        want, wn, wp = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, accum_mode=mode, aov=True)
        assert bit_equal(got, want).all(), (groups, mode)
        assert bit_equal(gn, wn).all() and bit_equal(gp, wp).all(), (groups, mode)
