"""Checkpoint / resume of a progressive render (sail_save_accum / sail_load_accum) and the queue of
one-sample frames behind sail_render (Renderer.render's launches batched). Needs a GPU.

The reference restarts its accumulation on every camera or object change and keeps it nowhere else
(src/core/renderer.js:57-60, src/scene/scene.js:65-68); a converged render (C5: 65,536 spp) is worth keeping.
The bar: render k -> save -> a NEW context -> load -> render k more equals the uninterrupted 2k-sample frame bit
for bit, whatever the partition, accumulation mode and device split."""
import numpy as np
import pytest

import oracle
from sail_amd import capi

pytestmark = pytest.mark.gpu


def bit_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


@pytest.fixture(scope="module")
def gpu():
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    return True


def _sched(sc, W, H, k0, spp):
    return capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, k0, spp)


def _make(W, H, devices, mode, accum, dbg=None):
    ctx = capi.Context(W, H, devices=devices, flags=capi.FLAG_AOV) if devices else capi.Context(W, H, flags=capi.FLAG_AOV)
    for opt, val in (dbg or {}).items():
        ctx.set_debug(opt, val)
    return ctx


def _setup(ctx, sc, mode, accum, rank_world=None):
    ctx.set_scene_dict(sc)
    ctx.set_accum_mode(accum)
    if rank_world:
        ctx.set_partition(rank_world[0], rank_world[1], mode)
    else:
        ctx.set_partition(0, 1, mode)


@pytest.mark.parametrize("devices,mode,accum,dbg", [
    (None, capi.PART_TILES, capi.ACCUM_SUM, None),
    (None, capi.PART_TILES, capi.ACCUM_MIX, None),
    (None, capi.PART_TILES, capi.ACCUM_COMPAT8, None),
    ([0, 0, 0], capi.PART_TILES, capi.ACCUM_SUM, None),
    ([0, 0, 0], capi.PART_TILES, capi.ACCUM_MIX, None),
    ([0, 0, 0], capi.PART_SAMPLES, capi.ACCUM_SUM, None),
    ([0], capi.PART_SAMPLES, capi.ACCUM_SUM, {capi.DEBUG_FORCE_RCCL: 1}),
])
@pytest.mark.parametrize("name,W,H,k,B", [("C3", 150, 70, 3, 5), ("C1", 64, 48, 4, 8)])
def test_resume_equals_uninterrupted(gpu, fixtures, devices, mode, accum, dbg, name, W, H, k, B):
    sc = fixtures["scenes"][name]
    inv, seeds = _sched(sc, W, H, 0, 2 * k)
    # uninterrupted: 2k samples on one context of the same shape
    ref = _make(W, H, devices, mode, accum, dbg)
    try:
        _setup(ref, sc, mode, accum)
        ref.render_schedule(inv, seeds, sc["eye"], B)
        want = ref.read_accum()
    finally:
        ref.close()
    a = _make(W, H, devices, mode, accum, dbg)
    try:
        _setup(a, sc, mode, accum)
        a.render_schedule(inv[:k], seeds[:k], sc["eye"], B)
        ck = a.save()
    finally:
        a.close()
    assert ck["k"] == k and len(ck["parts"]) == (len(devices) if devices else 1)
    b = _make(W, H, devices, mode, accum, dbg)
    try:
        _setup(b, sc, mode, accum)
        b.load(ck)
        assert b.save()["k"] == k
        b.render_schedule(inv[k:], seeds[k:], sc["eye"], B)
        got = b.read_accum()
        st = b.stats()
    finally:
        b.close()
    assert bit_equal(got, want).all()
    assert st.samples == 2 * k
    if mode == capi.PART_TILES and devices is None:  # and the CPU oracle's uninterrupted frame
        ao = {capi.ACCUM_SUM: oracle.ACC_SUM, capi.ACCUM_MIX: oracle.ACC_MIX, capi.ACCUM_COMPAT8: oracle.ACC_COMPAT8}[accum]
        want_o = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, accum_mode=ao)
        assert bit_equal(got, want_o).all()


def test_resume_from_whole_frame_tiles(gpu, fixtures):
    """part -1: a whole-frame accumulator (what a reduced readback gives) loaded into a 3-device tile context, each
    device keeping its own tiles, continues bit for bit; onto one device it is the same frame"""
    sc = fixtures["scenes"]["C3"]
    W, H, B, k = 150, 70, 5, 2
    inv, seeds = _sched(sc, W, H, 0, 2 * k)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    a = capi.Context(W, H, devices=[0, 0, 0])
    try:
        a.set_scene_dict(sc)
        a.render_schedule(inv[:k], seeds[:k], sc["eye"], B)
        frame = a.read_accum()
    finally:
        a.close()
    for devices in ([0, 0, 0], [0, 0], None):
        b = capi.Context(W, H, devices=devices) if devices else capi.Context(W, H)
        try:
            b.set_scene_dict(sc)
            b.load({"k": k, "frame": frame})
            b.render_schedule(inv[k:], seeds[k:], sc["eye"], B)
            got = b.read_accum()
        finally:
            b.close()
        assert bit_equal(got, want).all(), devices


def test_resume_per_process_rank(gpu, fixtures):
    """a per-process tile rank (sail_set_partition(1, 2)) saves and reloads its own accumulator"""
    sc = fixtures["scenes"]["C1"]
    W, H, B, k = 150, 70, 5, 2
    inv, seeds = _sched(sc, W, H, 0, 2 * k)
    a = capi.Context(W, H)
    try:
        a.set_scene_dict(sc)
        a.set_partition(1, 2)
        a.render_schedule(inv, seeds, sc["eye"], B)
        want = a.read_accum()
        a.reset()
        a.render_schedule(inv[:k], seeds[:k], sc["eye"], B)
        ck = a.save()
    finally:
        a.close()
    b = capi.Context(W, H)
    try:
        b.set_scene_dict(sc)
        b.set_partition(1, 2)
        b.load(ck)
        b.render_schedule(inv[k:], seeds[k:], sc["eye"], B)
        got = b.read_accum()
    finally:
        b.close()
    assert bit_equal(got, want).all()
    assert (got[..., 3] == 0).any() and (got[..., 3] == 2 * k).any()


def test_load_rejects_bad_parts(gpu, fixtures):
    sc = fixtures["scenes"]["C1"]
    ctx = capi.Context(16, 16, devices=[0, 0])
    z = np.zeros((16, 16, 4), np.float32)
    try:
        ctx.set_scene_dict(sc)
        with pytest.raises(capi.SailError):
            ctx.load({"k": 1, "parts": [z, z, z]})  # part 2 of 2
        k = capi.ctypes.c_uint64(0)
        assert ctx.lib.sail_save_accum(ctx.h, 5, capi._ptr(z), capi.ctypes.byref(k)) == -1
        assert ctx.lib.sail_load_accum(ctx.h, -2, capi._ptr(z), 0) == -1
    finally:
        ctx.close()


def test_load_rejects_mismatched_checkpoints(gpu, fixtures):
    """Context.load refuses a checkpoint that does not fit: wrong array shape, part count, size,
    accumulation mode or partition; and the C ABI refuses to use a multi-device frame whose parts are half loaded"""
    sc = fixtures["scenes"]["C1"]
    W, H, B = 24, 16, 3
    inv, seeds = _sched(sc, W, H, 0, 2)
    a = capi.Context(W, H, devices=[0, 0])
    try:
        a.set_scene_dict(sc)
        a.render_schedule(inv, seeds, sc["eye"], B)
        ck = a.save()
    finally:
        a.close()
    assert ck["width"] == W and ck["height"] == H and ck["partition"] == [0, 1, capi.PART_TILES]
    b = capi.Context(W, H, devices=[0, 0])
    try:
        b.set_scene_dict(sc)
        bad_shape = dict(ck, parts=[p[:, :-1] for p in ck["parts"]])
        with pytest.raises(capi.SailError, match="shape"):
            b.load(bad_shape)
        with pytest.raises(capi.SailError, match="parts"):
            b.load(dict(ck, parts=ck["parts"][:1]))
        with pytest.raises(capi.SailError, match="accum_mode"):
            b.load(dict(ck, accum_mode=capi.ACCUM_MIX))
        with pytest.raises(capi.SailError, match="partition"):
            b.load(dict(ck, partition=[0, 1, capi.PART_SAMPLES]))
        with pytest.raises(capi.SailError, match="width"):
            b.load(dict(ck, width=W + 1))
        # C ABI: part 0 alone leaves the frame half loaded -> every use is refused until part 1 arrives
        p0 = np.ascontiguousarray(ck["parts"][0])
        p1 = np.ascontiguousarray(ck["parts"][1])
        assert b.lib.sail_load_accum(b.h, 0, capi._ptr(p0), ck["k"]) == 0
        out = np.zeros((H, W, 4), np.float32)
        assert b.lib.sail_read_accum(b.h, capi._ptr(out)) == -4
        assert b.lib.sail_reduce(b.h, 0) == -4
        assert b.lib.sail_load_accum(b.h, 1, capi._ptr(p1), ck["k"] + 1) == -1  # a different checkpoint's part
        assert b.lib.sail_load_accum(b.h, 1, capi._ptr(p1), ck["k"]) == 0
        got = b.read_accum()
        b.load(ck)  # and through Context.load
        assert bit_equal(b.read_accum(), got).all()
        # sail_reset abandons a half-loaded checkpoint
        assert b.lib.sail_load_accum(b.h, 1, capi._ptr(p1), ck["k"]) == 0
        assert b.lib.sail_read_accum(b.h, capi._ptr(out)) == -4
        b.reset()
        assert b.lib.sail_read_accum(b.h, capi._ptr(out)) == 0
    finally:
        b.close()


@pytest.mark.parametrize("call", ["set_scene", "set_accum_mode", "set_partition"])
def test_half_loaded_checkpoint_abandoned_by_every_reset(gpu, fixtures, call):
    """every multi-device call that restarts the accumulation abandons a half-loaded checkpoint, like
    sail_reset: the frame is usable again, and a different checkpoint then loads part by part"""
    sc = fixtures["scenes"]["C1"]
    W, H, B = 24, 16, 3
    inv, seeds = _sched(sc, W, H, 0, 3)
    cks = []
    for n in (2, 3):
        a = capi.Context(W, H, devices=[0, 0])
        try:
            a.set_scene_dict(sc)
            a.render_schedule(inv[:n], seeds[:n], sc["eye"], B)
            cks.append(a.save())
        finally:
            a.close()
    assert cks[0]["k"] != cks[1]["k"]
    b = capi.Context(W, H, devices=[0, 0])
    try:
        b.set_scene_dict(sc)
        out = np.zeros((H, W, 4), np.float32)
        p0 = np.ascontiguousarray(cks[0]["parts"][0])
        assert b.lib.sail_load_accum(b.h, 0, capi._ptr(p0), cks[0]["k"]) == 0
        assert b.lib.sail_read_accum(b.h, capi._ptr(out)) == -4  # half loaded
        if call == "set_scene":
            b.set_scene_dict(sc)
        elif call == "set_accum_mode":
            b.set_accum_mode(capi.ACCUM_SUM)
        else:
            b.set_partition(0, 1, capi.PART_TILES)
        assert b.lib.sail_read_accum(b.h, capi._ptr(out)) == 0
        assert not out.any()  # restarted
        for i, part in enumerate(cks[1]["parts"]):  # the other checkpoint, part by part
            assert b.lib.sail_load_accum(b.h, i, capi._ptr(np.ascontiguousarray(part)), cks[1]["k"]) == 0
        want = capi.Context(W, H)
        try:
            want.set_scene_dict(sc)
            want.render_schedule(inv[:3], seeds[:3], sc["eye"], B)
            ref = want.read_accum()
        finally:
            want.close()
        assert bit_equal(b.read_accum(), ref).all()
    finally:
        b.close()


# ---- the sail_render queue (one-sample frames launched together) -------------------------------------------------
@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_render_queue_bit_exact_and_batched(gpu, fixtures, devices):
    """70 one-sample frames with launch_spp 32: 3 launches per device instead of 70, bit-identical to the oracle;
    a readback in the middle (the display) launches what is queued"""
    sc = fixtures["scenes"]["C3"]
    W, H, B, spp = 48, 40, 5, 70
    inv, seeds = _sched(sc, W, H, 0, spp)
    ctx = capi.Context(W, H, devices=devices) if devices else capi.Context(W, H)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_launch_samples(32)
        for s in range(spp):
            ctx.render(inv[s], sc["eye"], float(seeds[s]), B)
            if s == 9:
                mid = ctx.read_accum()
        got = ctx.read_accum()
        st = ctx.stats()
    finally:
        ctx.close()
    masks = capi.plugin_masks(sc["plugins"])
    assert bit_equal(mid, oracle.render(sc, masks, W, H, inv[:10], seeds[:10], sc["eye"], B)).all()
    assert bit_equal(got, oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B)).all()
    assert st.samples == spp
    assert st.launches == 1 + 1 + 1  # 10 before the readback; then 60 = 32 (a full queue) + 28 (the readback)


def test_render_queue_flushes_on_eye_and_bounce_change(gpu, fixtures):
    """a queued launch has one eye and one bounce count: a change launches the queue first (same frame as the
    oracle rendering each sample with its own eye and bounces)"""
    sc = fixtures["scenes"]["C1"]
    W, H = 40, 32
    inv, seeds = _sched(sc, W, H, 0, 6)
    eye2 = [sc["eye"][0] + 0.25, sc["eye"][1], sc["eye"][2]]
    plan = [(sc["eye"], 5), (sc["eye"], 5), (eye2, 5), (eye2, 3), (sc["eye"], 3), (sc["eye"], 3)]
    ctx = capi.Context(W, H)
    try:
        ctx.set_scene_dict(sc)
        for s, (eye, b) in enumerate(plan):
            ctx.render(inv[s], eye, float(seeds[s]), b)
        got = ctx.read_accum()
        st = ctx.stats()
    finally:
        ctx.close()
    want = np.zeros((H, W, 4), np.float32)
    masks = capi.plugin_masks(sc["plugins"])
    for s, (eye, b) in enumerate(plan):
        want = oracle.render(sc, masks, W, H, inv[s:s + 1], seeds[s:s + 1], eye, b, k0=s, accum=want)
    assert bit_equal(got, want).all()
    assert st.launches == 4


def test_render_queue_dropped_by_reset(gpu, fixtures):
    sc = fixtures["scenes"]["C1"]
    W, H, B = 24, 16, 4
    inv, seeds = _sched(sc, W, H, 0, 3)
    ctx = capi.Context(W, H)
    try:
        ctx.set_scene_dict(sc)
        ctx.render(inv[0], sc["eye"], float(seeds[0]), B)
        ctx.render(inv[1], sc["eye"], float(seeds[1]), B)
        ctx.reset()  # sampleCount = 0: the queued frames belong to the discarded accumulation
        ctx.render(inv[0], sc["eye"], float(seeds[0]), B)
        got = ctx.read_accum()
        st = ctx.stats()
    finally:
        ctx.close()
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv[:1], seeds[:1], sc["eye"], B)
    assert bit_equal(got, want).all()
    assert st.samples == 1 and st.launches == 1
