"""CPU, world_size 2 over gloo: the multi-GPU data path (64x64 tiles dealt t % world, each rank's float4
accumulator zero outside its tiles, a sum-reduce into a separate frame on rank 0) reproduces the single-rank
frame bit for bit, also progressively (render -> reduce -> render -> reduce: every reduce sums the ranks'
cumulative accumulators afresh, as sail_reduce does). The ranks render with the CPU oracle here; on MI355X the
same partition runs through sail_set_partition + sail_reduce (RCCL) and tests/test_gpu_multi.py checks the
product's reduce (multi-device context, RCCL at one rank) on one device."""
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


def _worker(rank, world, port, sc, W, H, spp, B, mode, q, progressive=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    import oracle
    from sail_amd import capi
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    masks = capi.plugin_masks(sc["plugins"])
    acc = np.zeros((H, W, 4), np.float32)
    passes = [np.arange(spp) < spp // 2, np.arange(spp) >= spp // 2] if progressive else [np.ones(spp, bool)]
    frames = []
    for part in passes:
        if mode == "tiles":
            for x0, y0, w, h in capi.partition_tiles(W, H, rank, world):
                oracle.render(sc, masks, W, H, inv[part], seeds[part], sc["eye"], B,
                              crop=(int(x0), int(y0), int(w), int(h)), accum=acc)
        else:  # sample split: rank takes samples k = rank (mod world)
            sel = part & (np.arange(spp) % world == rank)
            oracle.render(sc, masks, W, H, inv[sel], seeds[sel], sc["eye"], B, accum=acc)
        # out of place: the accumulator stays this rank's own; the frame is rank 0's display copy
        frame = torch.zeros((H, W, 4), dtype=torch.float32)
        frame.copy_(torch.from_numpy(acc))
        dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)
        frames.append(frame.numpy().copy())
    if rank == 0:
        q.put(frames[-1])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("progressive", [False, True])
@pytest.mark.parametrize("mode", ["tiles", "samples"])
def test_two_rank_reduce_equals_single_rank(fixtures, mode, progressive):
    import oracle
    from sail_amd import capi
    sc = fixtures["scenes"]["C3"]
    W, H, spp, B = 130, 70, 4 if progressive else 2, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sc, W, H, spp, B, mode, q, progressive)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    want = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    if mode == "tiles":
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    else:
        assert np.allclose(got, want, rtol=1e-6, atol=1e-6)
