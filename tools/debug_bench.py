#!/usr/bin/env python3
"""Times one scene under several sail_set_debug settings (none may change a result: every accumulator is compared
bit for bit with the first setting's). Usage: tools/debug_bench.py SCENE [W H B SPP] -- "opt=val,opt=val" ...
Options by name: cull_min_prims, force_generic, cull_fma, sample_groups."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sail_amd import capi  # noqa: E402

NAMES = {"cull_min_prims": capi.DEBUG_CULL_MIN_PRIMS, "force_generic": capi.DEBUG_FORCE_GENERIC,
         "cull_fma": capi.DEBUG_CULL_FMA, "sample_groups": capi.DEBUG_SAMPLE_GROUPS}


def main():
    argv = sys.argv[1:]
    if argv and argv[0] == "--lib":  # an alternative build (tools/build_variants.sh)
        capi._lib = capi.load(argv[1])
        argv = argv[2:]
    sep = argv.index("--") if "--" in argv else len(argv)
    head, settings = argv[:sep], argv[sep + 1:] or [""]
    scene = head[0] if head else "C4"
    W, H, B, spp = (int(v) for v in head[1:5]) if len(head) >= 5 else ((3840, 2160, 12, 8) if scene == "C4" else (1920, 1080, 8, 64))
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        sc = json.load(f)[scene]
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    ref = None
    for st in settings:
        opts = dict(kv.split("=") for kv in st.split(",") if kv)
        ctx = capi.Context(W, H)
        for k, v in opts.items():
            ctx.set_debug(NAMES[k], int(v))
        ctx.set_scene_dict(sc)
        ctx.render_schedule(inv, seeds, sc["eye"], B)   # warm-up
        ctx.sync()
        best = 1e30
        for _ in range(3):
            ctx.reset()
            t0 = time.perf_counter()
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            ctx.sync()
            best = min(best, time.perf_counter() - t0)
        acc = ctx.read_accum()
        ctx.close()
        same = ref is None or np.array_equal(acc.view(np.uint32), ref.view(np.uint32))
        ref = acc if ref is None else ref
        print(json.dumps({"scene": scene, "setting": st or "default", "s": round(best, 4),
                          "Gseg_per_s": round(W * H * spp * B / best / 1e9, 3), "bit_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
