"""Writes tests/golden/c1_full_256.json: the hash of BASELINE.json configs[0] -- the README Cornell box (frozen C1 scene)
at 256x256, 4 bounces, 64 spp of the deterministic schedule, SUM accumulation -- as the JS/Node software shader
(oracle/sail_soft.js, the north star's CPU fallback) renders it in full. Data only: the frame's SHA-256 over its raw
little-endian f32 accumulator (row 0 = bottom, RGB sums + count) and a few sums. tests/test_c1_full.py checks the C++
oracle against it here and the HIP path against it on the GPU; bench.py's full C1 CPU render checks itself against it.
Run: python tests/golden/make_c1_full.py (about 30 s)."""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from sail_amd import capi  # noqa: E402

W = H = 256
B, SPP = 4, 64


def job():
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        sc = json.load(f)["C1"]
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, SPP)
    return sc, inv, seeds


def main():
    sc, inv, seeds = job()
    j = {"objects": sc["objects"], "n": sc["n"], "texparams": sc["texparams"], "tn": sc["tn"], "lights": sc["lights"],
         "ln": sc["ln"], "masks": list(capi.plugin_masks(sc["plugins"])), "W": W, "H": H,
         "inv": [float(v) for v in inv.reshape(-1)], "seeds": [float(v) for v in seeds], "eye": sc["eye"], "spp": SPP,
         "maxBounces": B, "accumMode": 0}
    with tempfile.TemporaryDirectory() as td:
        with open(os.path.join(td, "job.json"), "w") as f:
            json.dump(j, f)
        out = subprocess.run(["node", os.path.join(ROOT, "oracle", "sail_soft.js"), os.path.join(td, "job.json"),
                              os.path.join(td, "o")], capture_output=True, text=True, check=True).stdout
        acc = np.fromfile(os.path.join(td, "o.accum.f32"), dtype="<f4").reshape(H, W, 4)
    r = json.loads(out.strip().splitlines()[-1])
    rec = {"config": "BASELINE.json configs[0]: README Cornell box (frozen C1), 256x256, 4 bounces, 64 spp, SUM",
           "generator": "tests/golden/make_c1_full.py: oracle/sail_soft.js (Node %s), whole frame" % r["node"],
           "width": W, "height": H, "bounces": B, "spp": SPP, "segments": r["segments"],
           "sha256_accum_f32le": hashlib.sha256(acc.astype("<f4").tobytes()).hexdigest(),
           "rgb_sum_f64": [float(acc[..., c].astype(np.float64).sum()) for c in range(3)],
           "count_min_max": [float(acc[..., 3].min()), float(acc[..., 3].max())]}
    with open(os.path.join(ROOT, "tests", "golden", "c1_full_256.json"), "w") as f:
        json.dump(rec, f, indent=1)
        f.write("\n")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
