"""Test-side binding of the CPU parity oracle (oracle/sail_oracle.cpp). Test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# SAIL_ORACLE_LIB: an alternative build of the same source (tests/test_sanitizers.py: the ASan/UBSan one)
LIB = os.environ.get("SAIL_ORACLE_LIB") or os.path.join(ORACLE_DIR, "build", "libsail_oracle.so")
LIB_COUNT = os.path.join(ORACLE_DIR, "build", "libsail_oracle_count.so")

ACC_SUM, ACC_MIX, ACC_COMPAT8 = 0, 1, 2


def build():
    srcs = [os.path.join(ORACLE_DIR, f) for f in ("sail_oracle.cpp", "ref_math.h")]
    newest = max(os.path.getmtime(s) for s in srcs)
    if os.environ.get("SAIL_ORACLE_LIB"):
        return
    if not (os.path.exists(LIB) and os.path.exists(LIB_COUNT) and os.path.getmtime(LIB) >= newest):
        subprocess.check_call(["sh", os.path.join(ORACLE_DIR, "build.sh")])


_libs = {}


def lib(count: bool = False) -> ctypes.CDLL:
    key = bool(count)
    if key in _libs:
        return _libs[key]
    build()
    L = ctypes.CDLL(LIB_COUNT if count else LIB)
    f32p = ctypes.POINTER(ctypes.c_float)
    u32 = ctypes.c_uint32
    ci = ctypes.c_int
    L.oracle_render.restype = ci
    L.oracle_render.argtypes = [f32p, ci, f32p, ci, f32p, ci, u32, u32, u32, u32, ci, ci, ci, ci, ci, ci,
                                f32p, f32p, f32p, ci, ci, ci, ci, f32p, f32p, f32p]
    L.oracle_filter.restype = ci
    L.oracle_filter.argtypes = [f32p, ci, ci, ci, f32p, ctypes.c_float, ctypes.c_float, ctypes.c_float, f32p]
    L.oracle_filter_aov.restype = ci
    L.oracle_filter_aov.argtypes = [f32p, f32p, f32p, ci, ci, ci, ctypes.c_float, ctypes.c_float, f32p]
    L.oracle_pick.restype = ci
    L.oracle_pick.argtypes = [f32p, ci, f32p, ci, u32, f32p, ci, ctypes.POINTER(ctypes.c_int), f32p]
    L.oracle_math.restype = None
    L.oracle_math.argtypes = [ci, f32p, f32p, f32p, ci]
    L.oracle_intersect_t.restype = ctypes.c_float
    L.oracle_intersect_t.argtypes = [f32p, ci, f32p, ci, u32, f32p, f32p]
    L.oracle_segments.restype = ctypes.c_ulonglong
    L.oracle_ops.restype = ctypes.c_ulonglong
    L.oracle_ops_live.restype = ctypes.c_ulonglong
    L.oracle_reset_counters.restype = None
    _libs[key] = L
    return L


def _f(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _p(a):
    if a is None:
        return ctypes.cast(None, ctypes.POINTER(ctypes.c_float))
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def render(scene: dict, masks, W: int, H: int, inv: np.ndarray, seeds: np.ndarray, eye, max_bounces: int,
           k0: int = 0, accum_mode: int = ACC_SUM, crop=None, accum: np.ndarray | None = None,
           aov: bool = False, count: bool = False):
    """Render samples k0.. of the crop (x0, y0, w, h); returns accum (H, W, 4) [, aov_n, aov_p]."""
    L = lib(count)
    o, t, l = _f(scene["objects"]), _f(scene["texparams"]), _f(scene["lights"])
    if accum is None:
        accum = np.zeros((H, W, 4), dtype=np.float32)
    x0, y0, cw, ch = crop if crop is not None else (0, 0, W, H)
    inv, seeds, e = _f(inv), _f(seeds), _f(eye)
    an = np.zeros((H, W, 4), dtype=np.float32) if aov else None
    ap = np.zeros((H, W, 4), dtype=np.float32) if aov else None
    rc = L.oracle_render(_p(o), scene["n"], _p(t), scene["tn"], _p(l), scene["ln"], *[int(m) for m in masks],
                         W, H, x0, y0, cw, ch, _p(inv), _p(seeds), _p(e), int(seeds.size), k0, max_bounces,
                         accum_mode, _p(accum), _p(an), _p(ap))
    if rc:
        raise RuntimeError(f"oracle_render: {rc}")
    return (accum, an, ap) if aov else accum


def filter_image(mean: np.ndarray, kind: int, weights16=None, rx=0.0, ry=0.0, gamma_c=2.2) -> np.ndarray:
    L = lib()
    H, W = mean.shape[:2]
    m = _f(mean)
    out = np.zeros((H, W, 4), dtype=np.float32)
    w = _f(weights16 if weights16 is not None else np.zeros(16))
    rc = L.oracle_filter(_p(m), W, H, kind, _p(w), rx, ry, gamma_c, _p(out))
    if rc:
        raise RuntimeError(f"oracle_filter: {rc}")
    return out


def filter_aov(mean: np.ndarray, normal: np.ndarray, position: np.ndarray, kind: int, rx=0.0, ry=0.0) -> np.ndarray:
    """wavelet (4) / normal (5) / position (6) display filters over the mean image and the AOV maps"""
    L = lib()
    H, W = mean.shape[:2]
    m, n, p = _f(mean), _f(normal), _f(position)
    out = np.zeros((H, W, 4), dtype=np.float32)
    rc = L.oracle_filter_aov(_p(m), _p(n), _p(p), W, H, kind, rx, ry, _p(out))
    if rc:
        raise RuntimeError(f"oracle_filter_aov: {rc}")
    return out


def pick(sc: dict, shape_mask: int, rays) -> tuple:
    """the shader's intersectObjects for (count, 6) rays -> (object row or -1, distance)"""
    L = lib()
    r = _f(rays).reshape(-1, 6)
    idx = np.zeros(len(r), dtype=np.int32)
    t = np.zeros(len(r), dtype=np.float32)
    rc = L.oracle_pick(_p(_f(sc["objects"])), sc["n"], _p(_f(sc["texparams"])), sc["tn"], shape_mask, _p(r), len(r),
                       idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _p(t))
    if rc:
        raise RuntimeError(f"oracle_pick: {rc}")
    return idx, t


def math(fn: int, x, y=None) -> np.ndarray:
    L = lib()
    x = _f(x)
    y = _f(np.zeros_like(x) if y is None else y)
    out = np.zeros_like(x)
    L.oracle_math(fn, _p(x), _p(y), _p(out), int(x.size))
    return out


def intersect_t(objects, n, texparams, tn, shape_mask, o, d) -> float:
    L = lib()
    return float(L.oracle_intersect_t(_p(_f(objects)), n, _p(_f(texparams)), tn, shape_mask, _p(_f(o)), _p(_f(d))))


def counters(count: bool = False):
    L = lib(count)
    return int(L.oracle_segments()), int(L.oracle_ops())


def ops_live(count: bool = True) -> int:
    """ops of the live-op model (the last bounce's dead ops left out; the counting build only)"""
    return int(lib(count).oracle_ops_live())


def reset_counters(count: bool = False):
    lib(count).oracle_reset_counters()
