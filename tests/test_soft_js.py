"""CPU: the JS/Node software shader (oracle/sail_soft.js, BASELINE.json's CPU baseline) against the C++ oracle:
its exactly rounded f32 fma, the spec math, and whole renders of every frozen scene, bit for bit. Two
independent CPU restatements agreeing is what lets each of them check the HIP kernel."""
import ctypes
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
from sail_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node") or shutil.which("nodejs")
SOFT = os.path.join(ROOT, "oracle", "sail_soft.js")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def run_soft(job, tmp_path, name="job"):
    jp = tmp_path / f"{name}.json"
    jp.write_text(json.dumps(job))
    out = subprocess.run([NODE, SOFT, str(jp), str(tmp_path / name)], capture_output=True, text=True, timeout=600,
                         check=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def soft_math(fn, x, y, tmp_path):
    run_soft({"math": fn, "xHex": np.asarray(x, np.float32).tobytes().hex(),
              "yHex": np.asarray(y, np.float32).tobytes().hex()}, tmp_path, f"m{fn}")
    return np.fromfile(tmp_path / f"m{fn}.math.f32", dtype=np.float32)


def same_bits(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def test_fma32_is_correctly_rounded(tmp_path):
    """fma32 vs glibc fmaf (correctly rounded), on random triples and on constructed rounding midpoints"""
    libm = ctypes.CDLL("libm.so.6")
    libm.fmaf.restype = ctypes.c_float
    libm.fmaf.argtypes = [ctypes.c_float] * 3
    rng = np.random.default_rng(4)
    n = 3000
    a = (rng.normal(size=n) * 10.0 ** rng.uniform(-6, 6, n)).astype(np.float32)
    b = (rng.normal(size=n) * 10.0 ** rng.uniform(-6, 6, n)).astype(np.float32)
    p = a.astype(np.float64) * b.astype(np.float64)
    # c that puts p + c (nearly) on an f32 rounding midpoint: the TwoSum tie-break path
    r = p.astype(np.float32).astype(np.float64)
    up = np.nextafter(r.astype(np.float32), np.float32(np.inf)).astype(np.float64)
    c_mid = ((r + up) / 2 - p).astype(np.float32)
    c_rand = (rng.normal(size=n) * np.abs(p) * 10.0 ** rng.uniform(-9, 1, n)).astype(np.float32)
    xs = np.concatenate([a, a]); ys = np.concatenate([b, b]); cs = np.concatenate([c_mid, c_rand])
    res = []
    for x, y, c in zip(xs, ys, cs):
        res.append((float(x), float(y), float(c)))
    jp = tmp_path / "fma.js"
    jp.write_text("const s=require(%r);const t=%s;const o=new Float32Array(t.length);"
                  "t.forEach((v,i)=>{o[i]=s.fma32(Math.fround(v[0]),Math.fround(v[1]),Math.fround(v[2]));});"
                  "process.stdout.write(Buffer.from(o.buffer).toString('hex'));" % (SOFT, json.dumps(res)))
    got = np.frombuffer(bytes.fromhex(subprocess.run([NODE, str(jp)], capture_output=True, text=True, check=True).stdout),
                        dtype=np.float32)
    want = np.array([libm.fmaf(x, y, c) for x, y, c in res], dtype=np.float32)
    assert same_bits(got, want).all()


@pytest.mark.parametrize("fn", [0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 14])
def test_spec_math_matches_cpp_oracle(tmp_path, fn):
    rng = np.random.default_rng(50 + fn)
    n = 4000
    if fn in (0, 1, 2):
        x = np.concatenate([rng.uniform(-1e6, 1e6, n // 2), rng.uniform(-7, 7, n // 2)])
        y = np.zeros(n)
    elif fn == 4:
        x, y = rng.uniform(-1, 1, n), np.zeros(n)
    elif fn in (9, 10, 12):
        sp = np.array([0.0, -0.0, 1.0, -1.0, np.nan, np.inf, -np.inf, 0.5], np.float32)
        xx, yy = np.meshgrid(sp, sp)
        x = np.concatenate([xx.ravel(), rng.normal(size=n)])
        y = np.concatenate([yy.ravel(), rng.normal(size=n)])
    else:
        x = rng.normal(size=n) * 10 ** rng.uniform(-3, 3, n)
        y = rng.normal(size=n) * 10 ** rng.uniform(-3, 3, n)
    x, y = x.astype(np.float32), y.astype(np.float32)
    got = soft_math(fn, x, y, tmp_path)
    want = oracle.math(fn, x, y)
    assert same_bits(got, want).all(), f"fn {fn}: {int((~same_bits(got, want)).sum())} mismatches"


CASES = [("C1", 24, 18, 3, 5, 0), ("C1g", 16, 12, 2, 8, 1), ("C3", 20, 16, 2, 8, 0), ("C4", 12, 10, 2, 12, 0),
         ("UI", 16, 16, 2, 5, 2), ("ALL", 20, 16, 2, 6, 0)]


@pytest.mark.parametrize("name,W,H,spp,B,mode", CASES)
def test_soft_render_matches_cpp_oracle(tmp_path, fixtures, name, W, H, spp, B, mode):
    sc = fixtures["scenes"][name]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    masks = capi.plugin_masks(sc["plugins"])
    job = {"objects": sc["objects"], "n": sc["n"], "texparams": sc["texparams"], "tn": sc["tn"],
           "lights": sc["lights"], "ln": sc["ln"], "masks": list(masks), "W": W, "H": H,
           "inv": [float(v) for v in inv.reshape(-1)], "seeds": [float(v) for v in seeds], "eye": sc["eye"],
           "spp": spp, "maxBounces": B, "accumMode": mode, "aov": True}
    info = run_soft(job, tmp_path, name)
    got = np.fromfile(tmp_path / f"{name}.accum.f32", dtype=np.float32).reshape(H, W, 4)
    gn = np.fromfile(tmp_path / f"{name}.aovn.f32", dtype=np.float32).reshape(H, W, 4)
    gp = np.fromfile(tmp_path / f"{name}.aovp.f32", dtype=np.float32).reshape(H, W, 4)
    oracle.reset_counters()
    want, wn, wp = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, accum_mode=mode, aov=True)
    segs, _ = oracle.counters()
    assert same_bits(got, want).all(), f"{name}: {int((~same_bits(got, want)).sum())} of {got.size} differ"
    assert same_bits(gn, wn).all() and same_bits(gp, wp).all()
    assert info["segments"] == segs
