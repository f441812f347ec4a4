"""The per-process multi-GPU path with real ranks: two processes, one GPU each, a communicator from
sail_comm_unique_id / sail_comm_init and the product's sail_reduce (RCCL over xGMI) into rank 0's frame. The
reduced frame must equal the one-GPU render: bit for bit for tiles, to summation order for a sample split; a
second render + reduce must not double count. The contexts carry AOVs (SAIL_FLAG_AOV): with 2k samples the last one is
rank 1's under a sample split, so rank 0 is a non-owner root that receives rank 1's maps while sending a -0 map itself
(sail_reduce, aovOwner); the reduced AOVs must equal the oracle's bit for bit in both partitions. RCCL refuses two ranks on one GPU, so this skips below 2 GPUs (the
driver's 8-GPU node runs it); tests/test_partition_gloo.py covers the same partition + reduce on CPU ranks and
tests/test_gpu_multi.py the RCCL reduce at world 1 and the distinct-device grouped reduce."""
import os
import sys

import numpy as np
import pytest

import oracle
from sail_amd import capi

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, mode, sc, W, H, B, k, q_uid, q_out):
    sys.path.insert(0, ROOT)
    from sail_amd import capi as c
    if rank == 0:
        uid = c.comm_unique_id()
        for _ in range(world - 1):
            q_uid.put(uid)
    else:
        uid = q_uid.get(timeout=120)
    inv, seeds = c.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, 2 * k)
    ctx = c.Context(W, H, device=rank, flags=c.FLAG_AOV)
    try:
        ctx.set_scene_dict(sc)
        ctx.set_partition(rank, world, mode)
        ctx.comm_init(uid, world, rank)
        ctx.render_schedule(inv[:k], seeds[:k], sc["eye"], B)
        ctx.reduce(0)
        first = ctx.read_accum() if rank == 0 else None
        ctx.render_schedule(inv[k:], seeds[k:], sc["eye"], B)
        ctx.reduce(0)
        got = ctx.read_accum() if rank == 0 else None
        aov = ctx.readback(aov=True)[1:] if rank == 0 else None
        ctx.sync()
    finally:
        ctx.close()
    q_out.put((rank, first, got, aov))


@pytest.mark.parametrize("mode", [capi.PART_TILES, capi.PART_SAMPLES])
def test_two_ranks_rccl_reduce(fixtures, mode):
    if capi.device_count() < 2:
        pytest.skip("two RCCL ranks need two GPUs")
    import multiprocessing as mp
    sc = fixtures["scenes"]["C3"]
    W, H, B, k, world = 150, 70, 5, 3, 2
    ctx = mp.get_context("spawn")
    q_uid, q_out = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, mode, sc, W, H, B, k, q_uid, q_out)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, first, got, aov = q_out.get(timeout=240)
        res[r] = (first, got, aov)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    first, got, (gn, gp) = res[0]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, 2 * k)
    masks = capi.plugin_masks(sc["plugins"])
    want_k = oracle.render(sc, masks, W, H, inv[:k], seeds[:k], sc["eye"], B)
    want, wn, wp = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, aov=True)
    assert (got[..., 3] == 2 * k).all(), "every pixel counts each sample once"
    if mode == capi.PART_TILES:
        assert np.array_equal(first.view(np.uint32), want_k.view(np.uint32))
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    else:
        assert np.allclose(first, want_k, rtol=1e-5, atol=1e-5)
        assert np.allclose(got, want, rtol=1e-5, atol=1e-5)
    # the AOVs of the frame's last sample (rank 1's under a sample split; each rank's own tiles otherwise)
    same = lambda a, b: (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same(gn, wn).all() and same(gp, wp).all()
