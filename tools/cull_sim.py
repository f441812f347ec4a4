#!/usr/bin/env python3
"""would a closest-first / two-level cull beat the pre-cull kernel's flat mask build on C4?
Simulated on C4's own rays (CPU, numpy + the test oracle's exact picker): primary rays of 16x4 pixel strips (the
kernel's wave shape) at 3840x2160, then three bounces. Each bounce ray starts at the previous ray's exact closest hit
(tests/oracle.py pick = the shader's intersectObjects) and leaves in a random direction of the hemisphere that faces
back along the incoming ray (a stand-in for the BSDF sample: the test needs the rays' spread, not their weights). Bounce
waves are 64 rays drawn from a permutation of the bounce (the path sort groups paths by material and shape, not by
position or direction). Counted per 64-ray wave, in units of one padded-box test of one row (~18 VALU):
  flat:      every row (the shipped mask build: 67 rows);
  uniform:   G group boxes (k-means on the rows' box centres; rows of a group inside its box), then the rows of every
             group ANY lane of the wave enters (wave-uniform descent, scalar row reads like the flat build);
  per-lane:  G group boxes, then the rows of the groups that lane enters, as a per-lane loop: the wave runs the slowest
             lane's count (before the per-lane loop's own overhead and per-lane row reads);
and each with the bound of the ray's exact closest distance (a closest-first traversal's best case).
Also: the share of waves whose 64 rays share a direction octant after sorting a 1,024-path pool by octant (the
precondition of an octant-specialised slab test, which saves 6 of the 18 VALU per row).
Usage: python tools/cull_sim.py > profiles/r06_cull_sim.txt"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from sail_amd import capi  # noqa: E402
import oracle  # noqa: E402  (test infrastructure: the exact closest-hit picker)


def boxhit(o, d, lo, hi):
    with np.errstate(divide="ignore", invalid="ignore"):
        r = 1.0 / d
        t0 = (lo[None] - o[:, None]) * r[:, None]
        t1 = (hi[None] - o[:, None]) * r[:, None]
        return np.nanmax(np.minimum(t0, t1), -1), np.nanmin(np.maximum(t0, t1), -1)


def kmeans(x, k, rng, it=50):
    c = x[rng.choice(len(x), k, replace=False)]
    for _ in range(it):
        a = ((x[:, None] - c[None]) ** 2).sum(-1).argmin(1)
        for j in range(k):
            if (a == j).any():
                c[j] = x[a == j].mean(0)
    return a


def main():
    sc = json.load(open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")))["C4"]
    n = sc["n"]
    bb = capi.prim_bounds(sc["objects"], n, sc["tn"])
    lo, hi = bb[:, 0].astype(np.float64), bb[:, 1].astype(np.float64)
    masks = capi.plugin_masks(sc["plugins"])
    rng = np.random.default_rng(5)
    W, H = 3840, 2160
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, _ = capi.schedule(mvp, W, H, 0, 1)
    M = np.array(inv[0], np.float64).reshape(4, 4).T
    xs, ys = [], []
    for _ in range(400):
        x0, y0 = rng.integers(0, W // 16) * 16, rng.integers(0, H // 4) * 4
        yy, xx = np.mgrid[y0:y0 + 4, x0:x0 + 16]
        xs.append(xx.ravel()); ys.append(yy.ravel())
    xs, ys = np.concatenate(xs).astype(np.float64), np.concatenate(ys).astype(np.float64)
    ndc = np.stack([(xs + 0.5) / W * 2 - 1, (ys + 0.5) / H * 2 - 1, np.ones_like(xs), np.ones_like(xs)], -1)
    p = ndc @ M.T
    p = p[:, :3] / p[:, 3:4]
    eye = np.array(sc["eye"], np.float64)
    O, D = np.tile(eye, (len(xs), 1)), p - eye
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    cent = (lo + hi) / 2
    groups = {}
    for G in (4, 8, 12, 16):
        a = kmeans(cent[1:], G, rng)
        groups[G] = (np.array([lo[1:][a == j].min(0) for j in range(G)]), np.array([hi[1:][a == j].max(0) for j in range(G)]),
                     np.array([(a == j).sum() for j in range(G)]))
    print(f"C4: {n} rows (row 0 the enclosing room box, always entered); {len(xs)} paths in 64-ray waves")
    for depth in range(4):
        idx, t = oracle.pick(sc, masks[0], np.concatenate([O, D], 1).astype(np.float32))
        t = t.astype(np.float64)
        tmin, tmax = boxhit(O, D, lo, hi)
        ent = (tmin <= tmax) & (tmax >= 0)
        entt = ent & (tmin <= t[:, None] * 1.0001 + 1e-4)
        perm = np.arange(len(O)) if depth == 0 else rng.permutation(len(O))
        nw = len(O) // 64
        E, Et = ent[perm].reshape(nw, 64, n), entt[perm].reshape(nw, 64, n)
        kind = "primary (16x4 strips)" if depth == 0 else f"bounce {depth} (sorted pool: position-incoherent)"
        print(f"\n{kind}: rows entered per ray {ent.sum(1).mean():.2f} (bounded by the exact hit {entt.sum(1).mean():.2f});"
              f" rows any lane of a wave enters {E.any(1).sum(1).mean():.1f} ({Et.any(1).sum(1).mean():.1f})")
        print(f"   flat build: {n} row tests per wave")
        for G, (glo, ghi, sizes) in groups.items():
            gmin, gmax = boxhit(O, D, glo, ghi)
            gh = ((gmin <= gmax) & (gmax >= 0))[perm].reshape(nw, 64, G)
            ght = (((gmin <= gmax) & (gmax >= 0)) & (gmin <= t[:, None] * 1.0001 + 1e-4))[perm].reshape(nw, 64, G)
            uni, unit = (gh.any(1) * sizes).sum(1).mean(), (ght.any(1) * sizes).sum(1).mean()
            lane, lanet = (gh * sizes).sum(2).max(1).mean(), (ght * sizes).sum(2).max(1).mean()
            print(f"   G={G:2d}: uniform descent {1 + G + uni:5.1f} (closest-first bound {1 + G + unit:5.1f});"
                  f" per-lane descent, slowest lane {1 + G + lane:5.1f} ({1 + G + lanet:5.1f})")
        if depth > 0:
            octs = (D[:, 0] < 0).astype(int) + 2 * (D[:, 1] < 0) + 4 * (D[:, 2] < 0)
            pools = len(O) // 1024
            uniform = 0
            for q in range(pools):
                o = np.sort(octs[perm][q * 1024:(q + 1) * 1024])
                uniform += sum(len(set(o[w * 64:(w + 1) * 64])) == 1 for w in range(16))
            print(f"   octant-sorted 1,024-path pools: {uniform / (pools * 16):.0%} of waves direction-uniform")
        P = O + D * t[:, None]
        nd = rng.normal(size=O.shape)
        nd /= np.linalg.norm(nd, axis=1, keepdims=True)
        nd[(nd * D).sum(1) > 0] *= -1
        O, D = P - D * 1e-3, nd


if __name__ == "__main__":
    main()
