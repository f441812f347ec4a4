#!/usr/bin/env python3
"""Per-phase wave-time attribution of the trace kernel from a -DSAIL_PHASE_TIMING=1 build
(sail_amd/build.sh builds it as sail_amd/lib/libsail_hip_phase.so). Each wave accumulates s_memtime deltas between
convergence points of the bounce loop; the shares are of summed wave time (all waves, all launches). "sort + barriers"
is the path sort between the sweep and the hit record (LDS counts, scan, scatter, gather and the barriers' waits);
a sample's end (radiance read-back, accumulation or staging) falls into the next sample's "sweep". Round-4 files
before this note called the sort phase "accumulate".
Usage: tools/phase_profile.py sail_amd/lib/libsail_hip_phase.so [C1 C3 C4]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sail_amd import capi  # noqa: E402

PHASES = ["sweep", "hit record", "shading frame", "hash RNG", "BSDF sample", "light + shadow", "next ray",
          "sort: rank atomics", "sort: barrier 1 wait", "sort: scan + scatter", "sort: barrier 2 (+3) wait",
          "sample end: barriers + accumulation"]


def main():
    path = sys.argv[1]
    scenes = sys.argv[2:] or ["C1", "C3", "C4"]
    lib = capi.load(path)
    capi._lib = lib
    lib.sail_phase_read.restype = ctypes.c_int
    lib.sail_phase_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        frozen = json.load(f)
    buf = (ctypes.c_ulonglong * 12)()
    for name in scenes:
        sc = frozen[name]
        W, H, B, spp = (3840, 2160, 12, 8) if name == "C4" else (1920, 1080, 8, 64)
        mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
        inv, seeds = capi.schedule(mvp, W, H, 0, spp)
        dbg = {int(k): int(v) for k, v in (o.split("=") for o in os.environ.get("PHASE_DEBUG", "").split(",") if o)}
        ctx = capi.Context(W, H, debug=dbg)
        ctx.set_scene_dict(sc)
        lib.sail_phase_read(buf, 1)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        ctx.sync()
        lib.sail_phase_read(buf, 1)
        ctx.close()
        v = np.array(list(buf), dtype=np.float64)
        tot = v.sum()
        print(json.dumps({"scene": name, "shares": {p: round(x / tot, 4) for p, x in zip(PHASES, v)},
                          "wave_cycles_per_segment_wave": round(tot / (W * H * spp * B / 64), 1)}), flush=True)


if __name__ == "__main__":
    main()
