#!/usr/bin/env python3
"""Full-frame check that the pre-cull is conservative: the C4 frame (3840x2160, 12 bounces) rendered with the
pre-cull kernel and with the pre-cull disabled (DEBUG_CULL_MIN_PRIMS=1000: the in-order sweep over every row)
must be bit-identical. Usage: tools/cull_check.py [spp] [library .so, default the in-tree build]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sail_amd import capi  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    if len(sys.argv) > 2:
        capi._lib = capi.load(sys.argv[2])
    sc = json.load(open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")))["C4"]
    W, H, B = 3840, 2160, 12
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    out = {}
    for cull in ("0", "1000"):
        ctx = capi.Context(W, H, debug={capi.DEBUG_CULL_MIN_PRIMS: int(cull)})
        ctx.set_scene_dict(sc)
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        out[cull] = ctx.read_accum()
        kname = ctx.kernel_name()
        ctx.close()
        print(json.dumps({"cull_min_prims": cull, "kernel": kname}), flush=True)
    diff = (out["0"].view(np.uint32) != out["1000"].view(np.uint32)).any(axis=2)
    print(json.dumps({"pixels": W * H, "spp": spp, "pixels_differing": int(diff.sum())}))
    return 0 if not diff.any() else 1


if __name__ == "__main__":
    sys.exit(main())
