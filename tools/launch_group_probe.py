#!/usr/bin/env python3
"""Frame time over samples per launch x sample groups (auto rule, or 1 = every workgroup does all of a launch's
samples, no staging): short launches give short tails without the staging pass, at the price of more launches.
Usage: tools/launch_group_probe.py [C2 C3 C5]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sail_amd import capi  # noqa: E402

SPP = {"C2": 256, "C3": 128, "C5": 256, "C4": 32}


def main():
    for name in sys.argv[1:] or ["C2", "C3", "C5"]:
        cfg = bench.CONFIGS[name]
        sc = bench.load_scene(cfg["scene"])
        W, H, B, spp = cfg["width"], cfg["height"], cfg["bounces"], SPP[name]
        mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
        inv, seeds = capi.schedule(mvp, W, H, 0, spp)
        for launch in (4, 8, 16, 32, 64):
            for groups in (0, 1):
                ctx = capi.Context(W, H)
                if groups:
                    ctx.set_debug(capi.DEBUG_SAMPLE_GROUPS, groups)
                ctx.set_scene_dict(sc)
                ctx.set_launch_samples(launch)
                ctx.render_schedule(inv[:64], seeds[:64], sc["eye"], B)  # warm-up
                ctx.sync()
                best = 1e30
                for _ in range(3):
                    ctx.reset()
                    t0 = time.perf_counter()
                    ctx.render_schedule(inv, seeds, sc["eye"], B)
                    ctx.sync()
                    best = min(best, time.perf_counter() - t0)
                st = ctx.stats()
                kname = ctx.kernel_name()
                ctx.close()
                print(json.dumps({"config": name, "launch_spp": launch, "groups": groups or "auto", "kernel": kname,
                                  "launches": int(st.launches), "Gseg_per_s": round(W * H * spp * B / best / 1e9, 3)}),
                      flush=True)


if __name__ == "__main__":
    main()
