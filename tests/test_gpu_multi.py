"""Multi-GPU data path through the product C ABI, on one MI355X. Needs a GPU.

* The multi-device context (sail_create_multi, `new Sail.Renderer({devices})`): with devices [0] it must pass
  the parity cases bit for bit; with [0, 0, ...] the same partition and reduce logic runs with every "device"
  on GPU 0 (the frame is summed by a kernel instead of RCCL, which refuses two ranks on one GPU).
* Progressive rendering across reduces (render k -> reduce -> render k -> reduce) must equal the 2k-sample
  frame: tile partitions bit for bit (AOVs included), sample partitions to rounding of the summation order.
* The per-process sail_reduce (RCCL communicator, out-of-place into root's frame) at world 1.
* The display filter divides each texel by its own count (a tile rank's frame holds unrendered pixels).
"""
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


CASES = [("C1", 64, 48, 8, 5), ("C1", 33, 17, 4, 8), ("C3", 40, 40, 4, 8), ("UI", 48, 48, 4, 5),
         ("ALL", 40, 32, 4, 6), ("C4", 32, 32, 2, 12), ("C1g", 16, 16, 2, 16)]
# "rccl": the distinct-device branch (ncclCommInitAll + grouped ncclReduce into device 0) forced at one device by
# SAIL_DEBUG_FORCE_RCCL; "all": every visible GPU as distinct devices (skipped below 2: the driver's 8-GPU node)
RCCL1 = "rccl"
ALL_GPUS = "all"


def _devices(spec):
    """a device list, a forced-RCCL one-device context, or every visible GPU"""
    if spec == RCCL1:
        return [0], {capi.DEBUG_FORCE_RCCL: 1}
    if spec == ALL_GPUS:
        n = capi.device_count()
        if n < 2:
            pytest.skip("distinct-device reduce needs at least 2 GPUs")
        return list(range(n)), {}
    return spec, {}


def _ctx(W, H, spec, flags=0):
    devices, dbg = _devices(spec)
    ctx = capi.Context(W, H, devices=devices, flags=flags)
    for opt, val in dbg.items():
        ctx.set_debug(opt, val)
    return ctx


@pytest.mark.parametrize("name,W,H,spp,B", CASES)
@pytest.mark.parametrize("devices", [[0], [0, 0, 0], RCCL1, ALL_GPUS])
def test_multi_device_context_bit_exact(gpu, fixtures, name, W, H, spp, B, devices):
    sc = fixtures["scenes"][name]
    inv, seeds = _sched(sc, W, H, 0, spp)
    ctx = _ctx(W, H, devices, flags=capi.FLAG_SEGMENT_COUNT | capi.FLAG_AOV)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_launch_samples(3)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        got = ctx.read_accum()
        _, gn, gp = ctx.readback(aov=True)
        st = ctx.stats()
    finally:
        ctx.close()
    oracle.reset_counters()
    want, wn, wp = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, aov=True)
    segs, _ = oracle.counters()
    assert bit_equal(got, want).all()
    assert bit_equal(gn, wn).all() and bit_equal(gp, wp).all()
    assert st.segments == segs and st.samples == spp


@pytest.mark.parametrize("mode", [capi.PART_TILES, capi.PART_SAMPLES])
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0, 0], RCCL1, ALL_GPUS])
def test_progressive_reduces(gpu, fixtures, mode, devices):
    """render k -> readback (reduce) -> render k -> readback equals the 2k-sample single-device frame; the AOVs
    shown are the last sample's (k = 3 per half: with 2 or 5 devices the last sample is not device 0's)"""
    sc = fixtures["scenes"]["C3"]
    W, H, B, k = 150, 70, 5, 3
    inv, seeds = _sched(sc, W, H, 0, 2 * k)
    ctx = _ctx(W, H, devices, flags=capi.FLAG_AOV)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_partition(0, 1, mode)
        ctx.render_schedule(inv[:k], seeds[:k], sc["eye"], B)
        first = ctx.read_accum()
        ctx.render_schedule(inv[k:], seeds[k:], sc["eye"], B)
        got = ctx.read_accum()
        again = ctx.read_accum()          # no render in between: the same frame
        _, gn, gp = ctx.readback(aov=True)
        ndev = len(_devices(devices)[0])
    finally:
        ctx.close()
    masks = capi.plugin_masks(sc["plugins"])
    want_k = oracle.render(sc, masks, W, H, inv[:k], seeds[:k], sc["eye"], B)
    want, wn, wp = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, aov=True)
    assert bit_equal(got, again).all()
    assert (got[..., 3] == 2 * k).all(), "every pixel counts each sample once"
    assert bit_equal(gn, wn).all() and bit_equal(gp, wp).all()  # the last sample's AOVs, whoever rendered it
    if mode == capi.PART_TILES or ndev == 1:
        assert bit_equal(first, want_k).all()
        assert bit_equal(got, want).all()
    else:  # the same samples summed in rank order: equal to rounding
        assert np.allclose(first, want_k, rtol=1e-5, atol=1e-5)
        assert np.allclose(got, want, rtol=1e-5, atol=1e-5)


def test_multi_device_running_mean_tiles(gpu, fixtures):
    sc = fixtures["scenes"]["UI"]
    W, H, B, spp = 130, 66, 5, 4
    inv, seeds = _sched(sc, W, H, 0, spp)
    ctx = capi.Context(W, H, devices=[0, 0])
    try:
        ctx.set_scene_dict(sc)
        ctx.set_accum_mode(capi.ACCUM_MIX)
        for s in range(spp):
            ctx.render(inv[s], sc["eye"], float(seeds[s]), B)
            if s == 1:
                ctx.read_accum()
        got = ctx.read_accum()
    finally:
        ctx.close()
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, accum_mode=oracle.ACC_MIX)
    assert bit_equal(got, want).all()


def test_multi_device_rejects_running_mean_sample_split(gpu, fixtures):
    ctx = capi.Context(16, 16, devices=[0, 0])
    try:
        ctx.set_accum_mode(capi.ACCUM_MIX)
        with pytest.raises(capi.SailError):
            ctx.set_partition(0, 1, capi.PART_SAMPLES)
        with pytest.raises(capi.SailError):
            ctx.set_partition(1, 2, capi.PART_TILES)   # the devices split the frame among themselves
        with pytest.raises(capi.SailError):
            ctx.comm_init(b"\0" * 128, 1, 0)
    finally:
        ctx.close()


@pytest.mark.parametrize("kind,fname,r", [(capi.FILTER_WINDOW, "gaussian", (1.5, 2.5)),
                                          (capi.FILTER_WAVELET, None, (2.0, 2.0)),
                                          (capi.FILTER_TONEMAPPING, None, (0.0, 0.0))])
@pytest.mark.parametrize("mode,devices", [(capi.PART_TILES, [0, 0, 0]), (capi.PART_SAMPLES, [0, 0, 0]),
                                          (capi.PART_SAMPLES, RCCL1)])
def test_multi_device_display_filter(gpu, fixtures, kind, fname, r, mode, devices):
    """Renderer.image() on a multi-device context: the filter runs on device 0 over the reduced frame; with a
    sample split (spp 5 on 3 devices: the last sample is device 1's) the wavelet reads that sample's AOVs"""
    sc = fixtures["scenes"]["C3"]
    W, H, B, spp = 140, 72, 5, 5
    inv, seeds = _sched(sc, W, H, 0, spp)
    w = np.array([float(x) for x in fixtures["filters"][fname]["weight_text"]], np.float32) if fname else None
    ctx = _ctx(W, H, devices, flags=capi.FLAG_AOV)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_partition(0, 1, mode)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        acc = ctx.read_accum()
        got = ctx.filter(kind, w, r[0], r[1], 2.2)
    finally:
        ctx.close()
    want_acc, n, p = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, aov=True)
    if mode == capi.PART_TILES or devices == RCCL1:
        assert bit_equal(acc, want_acc).all()
    else:  # the filters read the frame the devices summed (rank order)
        assert np.allclose(acc, want_acc, rtol=1e-5, atol=1e-5)
    mean = acc.copy()
    mean[..., :3] = acc[..., :3] / acc[..., 3:4]
    mean[..., 3] = 1.0
    if kind == capi.FILTER_WAVELET:
        want = oracle.filter_aov(mean, n, p, kind, r[0], r[1])
    else:
        want = oracle.filter_image(mean, kind, w, r[0], r[1], 2.2)
    assert bit_equal(got, want).all()


def test_filter_divides_each_texel_by_its_own_count(gpu, fixtures):
    """a tile rank's own frame: unrendered pixels have count 0 and show 0, rendered ones their mean"""
    sc = fixtures["scenes"]["C3"]
    W, H, B, spp = 150, 70, 4, 3
    inv, seeds = _sched(sc, W, H, 0, spp)
    w = np.array([float(x) for x in fixtures["filters"]["gaussian"]["weight_text"]], np.float32)
    ctx = capi.Context(W, H)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_partition(1, 2)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        acc = ctx.read_accum()
        got = ctx.filter(capi.FILTER_WINDOW, w, 1.5, 2.5)
    finally:
        ctx.close()
    assert (acc[..., 3] == 0).any() and (acc[..., 3] == spp).any()
    cnt = np.where(acc[..., 3:4] > 0, acc[..., 3:4], 1.0).astype(np.float32)
    mean = acc.copy()
    mean[..., :3] = acc[..., :3] / cnt
    want = oracle.filter_image(mean, capi.FILTER_WINDOW, w, 1.5, 2.5, 2.2)
    assert bit_equal(got, want).all()


@pytest.mark.parametrize("mode", [capi.PART_TILES, capi.PART_SAMPLES])
def test_rccl_reduce_world1_progressive(gpu, fixtures, mode):
    """the per-process path (sail_comm_init + sail_reduce over RCCL) at one rank: the reduce lands in a separate
    frame, so reducing twice with a render in between neither double counts nor disturbs the accumulator"""
    sc = fixtures["scenes"]["C1"]
    W, H, B, k = 96, 64, 5, 2
    inv, seeds = _sched(sc, W, H, 0, 2 * k)
    ctx = capi.Context(W, H, flags=capi.FLAG_AOV)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_partition(0, 1, mode)
        ctx.comm_init(capi.comm_unique_id(), 1, 0)
        ctx.comm_init(capi.comm_unique_id(), 1, 0)   # a second init replaces the communicator
        ctx.render_schedule(inv[:k], seeds[:k], sc["eye"], B)
        ctx.reduce(0)
        ctx.reduce(0)
        first = ctx.read_accum()
        ctx.render_schedule(inv[k:], seeds[k:], sc["eye"], B)
        own = ctx.read_accum()                        # after a render: this rank's accumulator again
        ctx.reduce(0)
        got = ctx.read_accum()
        _, gn, gp = ctx.readback(aov=True)
        ctx.sync()
    finally:
        ctx.close()
    masks = capi.plugin_masks(sc["plugins"])
    want_k = oracle.render(sc, masks, W, H, inv[:k], seeds[:k], sc["eye"], B)
    want, wn, wp = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, aov=True)
    assert bit_equal(first, want_k).all()
    assert bit_equal(own, want).all() and bit_equal(got, want).all()
    assert bit_equal(gn, wn).all() and bit_equal(gp, wp).all()


def test_rccl_reduce_needs_comm(gpu, fixtures):
    ctx = capi.Context(8, 8)
    try:
        with pytest.raises(capi.SailError):
            ctx.reduce(0)
    finally:
        ctx.close()
