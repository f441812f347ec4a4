#!/usr/bin/env python3
"""Times every sail_amd/lib/variants/libsail_hip_*.so on a C2-shaped render and checks that each variant's
accumulator is bit-identical to the first (variants may change scheduling, never results)."""
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sail_amd import capi  # noqa: E402


def run(path, sc, W, H, B, spp, launch, reps, debug=None):
    lib = capi.load(path)
    saved = capi._lib
    capi._lib = lib
    try:
        mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
        inv, seeds = capi.schedule(mvp, W, H, 0, spp)
        ctx = capi.Context(W, H, debug=debug)
        ctx.set_scene_dict(sc)
        ctx.set_launch_samples(launch)
        ctx.render_schedule(inv, seeds, sc["eye"], B)  # warm-up
        ctx.sync()
        best = 1e30
        for _ in range(reps):
            ctx.reset()
            t0 = time.perf_counter()
            ctx.render_schedule(inv, seeds, sc["eye"], B)
            ctx.sync()
            best = min(best, time.perf_counter() - t0)
        st = ctx.stats()
        acc = ctx.read_accum()
        ctx.close()
        rng = np.random.default_rng(9)
        bits = rng.integers(0, 2 ** 32, (2, 1 << 22), dtype=np.uint64).astype(np.uint32)
        a, b = bits[0].view(np.float32), bits[1].view(np.float32)
        q, want = capi.math_probe(11, a, b), capi.math_probe(8, a, b)
        div_bad = int((~((q.view(np.uint32) == want.view(np.uint32)) | (np.isnan(q) & np.isnan(want)))).sum())
        return best, st.kernel_ms / max(st.launches, 1), acc, div_bad
    finally:
        capi._lib = saved


def main():
    """variant_bench.py SCENE [NAME=LIB[:OPT=VAL,...] ...]: each spec is a library (a path, or "main" for
    sail_amd/lib/libsail_hip.so) with sail_set_debug switches; without specs, every sail_amd/lib/variants/*.so."""
    scene = sys.argv[1] if len(sys.argv) > 1 else "C1"
    W, H, B, spp = (3840, 2160, 12, 8) if scene == "C4" else (1920, 1080, 8, 128)
    spp = int(os.environ.get("VARIANT_SPP", spp))
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        sc = json.load(f)[scene]
    specs = []
    for a in sys.argv[2:]:
        name, rest = a.split("=", 1)
        lib, _, opts = rest.partition(":")
        lib = capi.LIB_PATH if lib == "main" else os.path.join(ROOT, lib)
        dbg = {int(k): int(v) for k, v in (o.split("=") for o in opts.split(",") if o)}
        specs.append((name, lib, dbg))
    if not specs:
        specs = [(os.path.basename(p), p, None)
                 for p in sorted(glob.glob(os.path.join(ROOT, "sail_amd", "lib", "variants", "libsail_hip_*.so")))]
    rounds = int(os.environ.get("VARIANT_ROUNDS", "2"))  # ABCD ABCD: clock drift shows as a spread, not a bias
    launch = int(os.environ.get("VARIANT_LAUNCH", "64"))  # samples per launch (the product default since round 4)
    ref = None
    for name, p, dbg in specs * rounds:
        dt, ms, acc, div_bad = run(p, sc, W, H, B, spp, launch, 3, dbg)
        same = ref is None or np.array_equal(acc.view(np.uint32), ref.view(np.uint32))
        if ref is None:
            ref = acc
        segs = W * H * spp * B
        print(json.dumps({"variant": name, "scene": scene, "debug": dbg, "launch_spp": launch, "s": round(dt, 4), "ms_per_launch": round(ms, 3),
                          "Gseg_per_s": round(segs / dt / 1e9, 3), "bit_identical": bool(same), "divide_mismatches": div_bad}), flush=True)


if __name__ == "__main__":
    main()
