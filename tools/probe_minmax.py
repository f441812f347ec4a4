#!/usr/bin/env python3
"""GPU diagnostic: hardware fminf/fmaxf semantics on signed zeros and NaNs, and the shared-reciprocal
exact division (math probe fn 11) against IEEE f32 division over random bit patterns."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sail_amd import capi
nan = np.float32("nan")
vals = np.array([0.0, -0.0, 1.0, -1.0, nan, np.inf, -np.inf], np.float32)
X, Y = np.meshgrid(vals, vals)
x, y = X.ravel(), Y.ravel()
mn = capi.math_probe(9, x, y)
mx = capi.math_probe(10, x, y)
for a, b, c, d in zip(x, y, mn, mx):
    print(f"min({a!r:>6},{b!r:>6}) = {c!r:>6} sign={np.signbit(c)}   max = {d!r:>6} sign={np.signbit(d)}")
rng = np.random.default_rng(5)
bad = 0
tot = 0
for _ in range(20):
    a = rng.integers(0, 2**32, 1 << 22, dtype=np.uint64).astype(np.uint32).view(np.float32)
    b = rng.integers(0, 2**32, 1 << 22, dtype=np.uint64).astype(np.uint32).view(np.float32)
    got = capi.math_probe(11, a, b)
    want = capi.math_probe(8, a, b)
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    bad += int((~same).sum())
    tot += a.size
print(f"shared-reciprocal divide: {bad} mismatches of {tot}")
