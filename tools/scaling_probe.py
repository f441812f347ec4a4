#!/usr/bin/env python3
"""Per-rank trace throughput for world sizes 1/2/4/8 emulated on one GPU (rank 0's tiles only, no collective):
predicts the strong-scaling efficiency of bench.py --gpus N before the reduce is added.
Usage: tools/scaling_probe.py [config] [spp]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sail_amd import capi  # noqa: E402


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    W, H, B = cfg["width"], cfg["height"], cfg["bounces"]
    sc = bench.load_scene(cfg["scene"])
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    base = None
    for world in (1, 2, 4, 8):
        for rank in ([0, world - 1] if world > 1 else [0]):
            ctx = capi.Context(W, H)
            ctx.set_scene_dict(sc)
            ctx.set_partition(rank, world, capi.PART_TILES)
            ctx.render_schedule(inv[:32], seeds[:32], sc["eye"], B)  # warm-up
            ctx.sync()
            ctx.reset()
            t0 = time.perf_counter()
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            ctx.sync()
            dt = time.perf_counter() - t0
            px = int(sum(int(w) * int(h) for _, _, w, h in capi.partition_tiles(W, H, rank, world)))
            rate = px * spp * B / dt / 1e9
            ctx.close()
            if base is None:
                base = rate
            print(json.dumps({"world": world, "rank": rank, "pixels": px, "s": round(dt, 4),
                              "Gseg_per_s_per_gpu": round(rate, 3), "vs_1gpu": round(rate / base, 3),
                              "frame_speedup_if_all_ranks_like_this": round(W * H / px * rate / base, 2)}), flush=True)


if __name__ == "__main__":
    main()
