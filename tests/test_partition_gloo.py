"""CPU, world_size 2 / 4 / 8 over gloo: the multi-GPU exchange as the library plans it, without a device.

Each rank renders its share with the CPU oracle: the 64x64 tiles `sail_partition_tiles` deals it (tile t -> rank
t % world), or the samples with index = rank (mod world). It then sends what the library's own reduce bookkeeping
says: `sail_plan_reduce` picks the root, the rank's sample count, and whether its AOV maps or -0 maps go into the AOV
reduce (`sail_reduce` and the multi-device reduce take these choices from the same function). The run is
progressive, with a resume in the middle: render -> reduce -> a whole-frame checkpoint, of which each rank keeps
what `sail_plan_keep` gives it (sail_load_accum part -1) -> render the rest -> reduce. Finally the ranks' own
accumulators are loaded part by part under `sail_plan_load_part`, which must refuse a part of another checkpoint and
report the load complete only after the last part.

Checked against the one-rank frame: accumulators bit for bit for tiles (every reduce adds exact zeros), to summation
order for a sample split; the AOV maps bit for bit in both partitions (a sample split shows the maps of the rank that
rendered the last sample). On MI355X the same partition runs through sail_set_partition + sail_reduce over RCCL
(tests/test_gpu_multi.py, tests/test_gpu_rccl_ranks.py)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


NEG0 = np.float32(-0.0)


def _render_share(oracle, capi, sc, masks, W, H, inv, seeds, B, mode, rank, world, ks, acc):
    """this rank's share of samples ks (global indices) into acc; returns its AOV maps of the share's last sample: -0
    outside what it rendered (the product initialises its maps so, sail_capi.cpp resetAccum)"""
    an = np.full((H, W, 4), NEG0, np.float32)
    ap = np.full((H, W, 4), NEG0, np.float32)
    if mode == "tiles":
        for x0, y0, w, h in capi.partition_tiles(W, H, rank, world):
            _, tn, tp = oracle.render(sc, masks, W, H, inv[ks], seeds[ks], sc["eye"], B, k0=int(ks[0]),
                                      crop=(int(x0), int(y0), int(w), int(h)), accum=acc, aov=True)
            an[y0:y0 + h, x0:x0 + w] = tn[y0:y0 + h, x0:x0 + w]
            ap[y0:y0 + h, x0:x0 + w] = tp[y0:y0 + h, x0:x0 + w]
    else:
        mine = ks[ks % world == rank]
        if mine.size:
            _, an, ap = oracle.render(sc, masks, W, H, inv[mine], seeds[mine], sc["eye"], B, accum=acc, aov=True)
    return an, ap


def _reduce(capi, W, H, rank, world, part, k, root, acc, an, ap):
    """the library's plan for this rank, then the exchange it prescribes (out of place: acc stays the rank's own)"""
    plan = capi.plan_reduce(W, H, rank, world, part, k, root)
    frame = torch.from_numpy(acc.copy())
    dist.reduce(frame, dst=root, op=dist.ReduceOp.SUM)
    maps = []
    for m in (an, ap):
        send = m if plan["send_own_aovs"] else np.full_like(m, NEG0)
        t = torch.from_numpy(send.copy())
        dist.reduce(t, dst=root, op=dist.ReduceOp.SUM)
        maps.append(t.numpy())
    return plan, frame.numpy(), maps


def _worker(rank, world, port, sc, W, H, spp, B, mode, root, q):
    import sys
    base = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, base)
    sys.path.insert(0, os.path.join(base, "tests"))
    import oracle
    from sail_amd import capi
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    part = capi.PART_TILES if mode == "tiles" else capi.PART_SAMPLES
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    masks = capi.plugin_masks(sc["plugins"])
    k1 = spp // 2
    report = {}
    # pass 1: samples 0 .. k1-1, reduced into root
    acc = np.zeros((H, W, 4), np.float32)
    an, ap = _render_share(oracle, capi, sc, masks, W, H, inv, seeds, B, mode, rank, world, np.arange(k1), acc)
    plan, f1, _ = _reduce(capi, W, H, rank, world, part, k1, root, acc, an, ap)
    rendered = k1 if mode == "tiles" else int(np.sum(np.arange(k1) % world == rank))
    report["plan1"] = (plan["receives"] == (rank == root), plan["samples"] == rendered,
                       plan["tiles"] == (len(capi.partition_tiles(W, H, rank, world)) if mode == "tiles"
                                         else ((W + 63) // 64) * ((H + 63) // 64)))
    # the whole-frame checkpoint goes from root to every rank; each keeps its part of it (sail_load_accum part -1)
    ck = torch.from_numpy(f1.copy())
    dist.broadcast(ck, src=root)
    acc = capi.plan_keep(W, H, rank, world, part, ck.numpy()).copy()
    # pass 2: samples k1 .. spp-1 on top (the AOV maps restart with the next sample)
    an, ap = _render_share(oracle, capi, sc, masks, W, H, inv, seeds, B, mode, rank, world, np.arange(k1, spp), acc)
    plan, f2, maps = _reduce(capi, W, H, rank, world, part, spp, root, acc, an, ap)
    report["owner"] = plan["aov_owner"]
    # part-wise load of every rank's own accumulator (as saved: part = rank, k = spp) on root, out of order, with a
    # part of another checkpoint in between
    parts = [torch.zeros((H, W, 4)) for _ in range(world)] if rank == root else None
    dist.gather(torch.from_numpy(acc.copy()), parts, dst=root)
    if rank == root:
        lp = capi.LoadParts(world)
        order = list(range(world))[::-1]
        checks = []
        lp.load(order[0], spp)
        try:
            lp.load(order[-1], spp + 1)  # another checkpoint's part: refused, state unchanged
            checks.append(False)
        except capi.SailError:
            checks.append(True)
        for p in order[1:]:
            checks.append(not lp.complete)
            lp.load(p, spp)
        checks.append(lp.complete and lp.k.value == spp)
        summed = np.sum(np.stack([t.numpy() for t in parts]), axis=0, dtype=np.float32) if mode == "tiles" else None
        report["parts"] = (all(checks), summed is None or np.array_equal(summed.view(np.uint32), f2.view(np.uint32)))
        q.put((f2, maps[0], maps[1], report))
    else:
        q.put((None, None, None, report))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode", ["tiles", "samples"])
def test_planned_reduce_equals_single_rank(fixtures, mode, world):
    import oracle
    from sail_amd import capi
    sc = fixtures["scenes"]["C3"]
    W, H, spp, B = 200, 140, 6, 4  # 12 tiles: at world 8 half the ranks own one tile, half two
    root = world - 1 if mode == "tiles" else 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sc, W, H, spp, B, mode, root, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    got, gn, gp, rep = next(r for r in results if r[0] is not None)
    for *_, r in results:
        assert all(r["plan1"]), r
    assert rep["parts"] == (True, True)
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want, wn, wp = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B, aov=True)
    if mode == "tiles":
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    else:
        assert rep["owner"] == (spp - 1) % world
        assert np.allclose(got, want, rtol=1e-6, atol=1e-6)
    assert np.array_equal(gn.view(np.uint32), wn.view(np.uint32))
    assert np.array_equal(gp.view(np.uint32), wp.view(np.uint32))


def test_plan_edges():
    """the plan's boundary cases: ranks owning no tile, an owner before any sample, bad arguments, part -1"""
    from sail_amd import capi
    p = capi.plan_reduce(64, 64, 3, 4, capi.PART_TILES, 5, 0)  # one tile, rank 3 owns none
    assert p["tiles"] == 0 and p["send_own_aovs"] == 1 and p["aov_owner"] == -1 and p["samples"] == 5
    p = capi.plan_reduce(130, 70, 1, 3, capi.PART_SAMPLES, 0, 1)
    assert p["aov_owner"] == 0 and p["send_own_aovs"] == 0 and p["samples"] == 0 and p["receives"] == 1
    assert capi.plan_reduce(130, 70, 2, 3, capi.PART_SAMPLES, 7, 0)["samples"] == 2  # samples 2 and 5
    for bad in [(0, 70, 0, 1, 0, 1, 0), (130, 70, 3, 3, 0, 1, 0), (130, 70, 0, 3, 2, 1, 0), (130, 70, 0, 3, 0, 1, 3)]:
        with pytest.raises(capi.SailError):
            capi.plan_reduce(*bad)
    sums = np.arange(130 * 70 * 4, dtype=np.float32).reshape(70, 130, 4)
    kept = [capi.plan_keep(130, 70, r, 3, capi.PART_TILES, sums) for r in range(3)]
    assert np.array_equal(np.sum(kept, axis=0), sums)  # disjoint tiles cover the frame
    assert np.array_equal(capi.plan_keep(130, 70, 0, 3, capi.PART_SAMPLES, sums), sums)
    assert not capi.plan_keep(130, 70, 2, 3, capi.PART_SAMPLES, sums).any()
    lp = capi.LoadParts(3)
    lp.load(1, 10)
    assert not lp.complete and lp.missing.value == 0b101
    lp.load(-1, 12)  # a whole frame replaces the half-loaded checkpoint
    assert lp.complete and lp.k.value == 12
    with pytest.raises(capi.SailError):
        lp.load(3, 12)
