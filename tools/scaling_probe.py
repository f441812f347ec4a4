#!/usr/bin/env python3
"""Per-rank trace throughput for world sizes 1/2/4/8 emulated on one GPU (rank 0's and rank N-1's share only, no
collective): predicts the strong-scaling efficiency of bench.py --gpus N before the reduce is added. A tile config
renders the rank's tiles; a sample-split config (C5) renders its samples k = rank mod N of the whole frame.
Usage: tools/scaling_probe.py [config] [spp] [--groups g] [--worlds 1,2,4,8] [--debug k=v,...]
--groups g fixes the sample-group count (SAIL_DEBUG_SAMPLE_GROUPS) instead of the host's occupancy rule; --rounds /
--cull-rounds change that rule's target (SAIL_DEBUG_GROUP_ROUNDS / SAIL_DEBUG_CULL_GROUP_ROUNDS)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sail_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C2")
    ap.add_argument("spp", nargs="?", type=int, default=256)
    ap.add_argument("--groups", type=int, default=0)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=0, help="SAIL_DEBUG_GROUP_ROUNDS (flat kernels)")
    ap.add_argument("--cull-rounds", type=int, default=0, help="SAIL_DEBUG_CULL_GROUP_ROUNDS")
    ap.add_argument("--lib", default=None, help="a variant build of libsail_hip.so (tools/build_variants.sh)")
    ap.add_argument("--debug", default="", help="extra sail_set_debug options, k=v[,k=v...] (e.g. 11=4: SAIL_DEBUG_JIT_NS)")
    a = ap.parse_args()
    if a.lib:
        capi._lib = capi.load(a.lib)
    cfg = bench.CONFIGS[a.config]
    spp = a.spp
    W, H, B = cfg["width"], cfg["height"], cfg["bounces"]
    part = capi.PART_SAMPLES if cfg.get("partition") == "samples" else capi.PART_TILES
    sc = bench.load_scene(cfg["scene"])
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    base = None
    for world in (int(w) for w in a.worlds.split(",")):
        for rank in ([0, world - 1] if world > 1 else [0]):
            ctx = capi.Context(W, H)
            if a.groups:
                ctx.set_debug(capi.DEBUG_SAMPLE_GROUPS, a.groups)
            if a.rounds:
                ctx.set_debug(capi.DEBUG_GROUP_ROUNDS, a.rounds)
            if a.cull_rounds:
                ctx.set_debug(capi.DEBUG_CULL_GROUP_ROUNDS, a.cull_rounds)
            for kv in filter(None, a.debug.split(",")):
                k, v = kv.split("=")
                ctx.set_debug(int(k), int(v))
            ctx.set_scene_dict(sc)
            ctx.set_partition(rank, world, part)
            ctx.render_schedule(inv[:32], seeds[:32], sc["eye"], B)  # warm-up
            ctx.sync()
            best = 1e30
            for _ in range(a.reps):
                ctx.reset()
                t0 = time.perf_counter()
                ctx.render_schedule(inv, seeds, sc["eye"], B)
                ctx.sync()
                best = min(best, time.perf_counter() - t0)
            st = ctx.stats()
            ctx.close()
            if part == capi.PART_TILES:
                px = int(sum(int(w) * int(h) for _, _, w, h in capi.partition_tiles(W, H, rank, world)))
                work = px * spp * B
                share = px / (W * H)
            else:
                mine = len(range(rank, spp, world))
                work = W * H * mine * B
                share = mine / spp
            rate = work / best / 1e9
            if base is None:
                base = rate
            print(json.dumps({"lib": os.path.basename(a.lib) if a.lib else "main", "config": a.config, "partition": "tiles" if part == capi.PART_TILES else "samples",
                              "spp": spp, "groups": a.groups or "auto", "rounds": a.rounds or a.cull_rounds or "default", "debug": a.debug, "world": world, "rank": rank,
                              "share": round(share, 5), "s": round(best, 4), "launches": int(st.launches),
                              "Gseg_per_s_per_gpu": round(rate, 3), "vs_1gpu": round(rate / base, 3),
                              "frame_speedup_if_all_ranks_like_this": round(rate / base / share, 2)}), flush=True)


if __name__ == "__main__":
    main()
