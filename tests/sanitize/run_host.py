"""Runs under the ASan/UBSan runtime (tests/test_sanitizers.py preloads it): drives the instrumented oracle and
the instrumented host side of libsail_hip (no device) over the fixture scenes and hostile inputs, and saves every
result under argv[1] for the parent test to compare with the plain builds. Any sanitizer report aborts."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402  (SAIL_ORACLE_LIB points it at the instrumented build)
from sail_amd import capi  # noqa: E402

out = sys.argv[1]
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "fixtures.json")))
lib = capi.load(os.environ["SAIL_LIB_ASAN"])
capi._lib = lib
res = {}

# ---- oracle: renders (every accumulation mode, AOVs), display filters, picks, spec math ----
for name, W, H, spp, B in [("C1", 12, 10, 2, 5), ("C3", 10, 8, 2, 8), ("C4", 8, 8, 1, 12), ("ALL", 10, 8, 2, 6),
                           ("AREA0", 8, 8, 2, 4), ("N0", 6, 4, 1, 3), ("N1", 8, 6, 2, 4), ("N1S", 8, 6, 2, 4),
                           ("BILERP", 8, 8, 2, 5), ("UI", 8, 8, 2, 5)]:
    sc = fx["scenes"][name]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    masks = capi.plugin_masks(sc["plugins"])
    for mode in (oracle.ACC_SUM, oracle.ACC_MIX, oracle.ACC_COMPAT8):
        acc, an, ap = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, accum_mode=mode, aov=True)
        res[f"{name}_{mode}"] = np.stack([acc, an, ap])
    mean = res[f"{name}_0"][0][..., :3] / np.maximum(res[f"{name}_0"][0][..., 3:4], 1)
    mean4 = np.concatenate([mean, np.ones_like(mean[..., :1])], axis=-1)
    res[f"{name}_filter_window"] = oracle.filter_image(mean4, 3, np.linspace(0.1, 1.0, 16), 2.0, 2.0)
    res[f"{name}_filter_gamma"] = oracle.filter_image(mean4, 1, None, 0, 0, 2.2)
    res[f"{name}_wavelet"] = oracle.filter_aov(mean4, res[f"{name}_0"][1], res[f"{name}_0"][2], 4, 1.0, 1.0)
    rng = np.random.default_rng(3)
    rays = np.concatenate([rng.uniform(-10, 10, (256, 3)), rng.normal(size=(256, 3))], axis=1)
    rays[:8, 3:] = 0.0                       # zero directions
    rays[8:16, 3] = np.inf                   # infinite components
    rays[16:24, 4] = np.nan
    idx, t = oracle.pick(sc, masks[0], rays)
    res[f"{name}_pick_idx"], res[f"{name}_pick_t"] = idx, t
rng = np.random.default_rng(4)
bits = rng.integers(0, 2 ** 32, 1 << 16, dtype=np.uint64).astype(np.uint32).view(np.float32)
specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3.4e38, -3.4e38, 1e15, 1e16], np.float32)
xs = np.concatenate([bits, specials])
for fn in (0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14):
    res[f"math_{fn}"] = oracle.math(fn, xs, xs[::-1].copy())

# ---- libsail_hip host side: host math, scene decode of hostile rows, partitions, error paths ----
for name in ("C1", "C3", "C4", "UI"):
    sc = fx["scenes"][name]
    mvp = capi.camera(sc["eye"], sc.get("center", [2.78, 2.73, 2.79]), [0, 1, 0], 55.0, 16 / 9, 1.0, 100.0)
    res[f"{name}_camera"] = mvp
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), 1920, 1080, 5, 64)
    res[f"{name}_schedule_inv"], res[f"{name}_schedule_seeds"] = inv, seeds
for name, sc in fx["scenes"].items():
    if sc["n"] > 0:
        res[f"{name}_bounds"] = capi.prim_bounds(sc["objects"], sc["n"], sc["tn"])
rows = rng.uniform(-5, 5, (64, 18)).astype(np.float32)
rows[:, 0] = rng.integers(-2, 12, 64)               # categories in and out of range
rows[::7, 4] = np.nan
rows[::5, 9] = np.inf
rows[::3, 10] = -1e30
rows[1::4, 8] = 1e9                                 # material / texture rows far out of range
res["fuzz_bounds"] = capi.prim_bounds(rows, 64, 3)
for W, H, world in [(1920, 1080, 8), (1, 1, 1), (65, 129, 3), (3840, 2160, 7)]:
    for r in range(world):
        res[f"tiles_{W}_{H}_{world}_{r}"] = capi.partition_tiles(W, H, r, world)
try:
    capi.Context(8, 8)
    raise SystemExit("sail_create succeeded without a device")
except capi.SailError as e:
    assert "device" in str(e).lower() or "hip" in str(e).lower(), str(e)
assert lib.sail_set_scene(None, None, 0, None, 0, None, 0, None) < 0
assert lib.sail_render(None, None, None, 0.0, 1) < 0
assert lib.sail_last_error(None) is not None
np.savez(out, **res)
print("sanitized host run ok:", len(res), "results")
