#!/usr/bin/env python3
"""Pre-cull outcome statistics from a -DSAIL_CULL_STATS=1 build: per (wave, primitive) test, how often some lane
passed (so the wave ran the exact test) and how many lanes did. Usage: tools/cull_stats.py lib.so [scene]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sail_amd import capi  # noqa: E402


def main():
    lib = capi.load(sys.argv[1])
    capi._lib = lib
    lib.sail_phase_read.restype = ctypes.c_int
    lib.sail_phase_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    name = sys.argv[2] if len(sys.argv) > 2 else "C4"
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        sc = json.load(f)[name]
    W, H, B, spp = 1920, 1080, 12, 2
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    ctx = capi.Context(W, H)
    ctx.set_scene_dict(sc)
    buf = (ctypes.c_ulonglong * 8)()
    lib.sail_phase_read(buf, 1)
    ctx.render_schedule(inv, seeds, sc["eye"], B)
    ctx.sync()
    lib.sail_phase_read(buf, 1)
    ctx.close()
    tests, executed, passing, active = list(buf)[:4]
    print(json.dumps({"scene": name, "kernel_tests": tests, "executed_frac": executed / tests,
                      "lanes_passing_per_executed": passing / max(executed, 1), "active_lanes_per_test": active / tests}))


if __name__ == "__main__":
    main()
