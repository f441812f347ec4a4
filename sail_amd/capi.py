"""ctypes binding of libsail_hip.so (include/sail_hip.h) for the Python side (tests, bench).

The product host API is the JavaScript one in sail_amd/js (Sail.Renderer / Scene / Camera over the
N-API addon); this module is the same C ABI seen from Python. It never falls back to anything: if
the HIP library is missing or a call fails, it raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SAIL_HIP_LIB: another build of the same library (a study variant, tools/study_build.sh), for the profiling tools
LIB_PATH = os.environ.get("SAIL_HIP_LIB") or os.path.join(_HERE, "lib", "libsail_hip.so")

SAIL_OK = 0
FLAG_AOV = 1
FLAG_SEGMENT_COUNT = 2
ACCUM_SUM, ACCUM_MIX, ACCUM_COMPAT8 = 0, 1, 2
PART_TILES, PART_SAMPLES = 0, 1
FILTER_COLOR, FILTER_GAMMA, FILTER_TONEMAPPING, FILTER_WINDOW = 0, 1, 2, 3
FILTER_WAVELET, FILTER_NORMAL, FILTER_POSITION = 4, 5, 6  # need FLAG_AOV
# sail_set_debug options (test / study switches; none changes a result)
DEBUG_CULL_MIN_PRIMS, DEBUG_FORCE_GENERIC, DEBUG_CULL_FMA, DEBUG_SAMPLE_GROUPS, DEBUG_FORCE_RCCL = 1, 2, 3, 4, 5
DEBUG_WAVEFRONT = 6
DEBUG_GROUP_ROUNDS = 7
DEBUG_CULL_GROUP_ROUNDS = 8
DEBUG_JIT = 9
DEBUG_JIT_WAIT = 10  # ms a launch waits for the scene's run-time kernel (-1: until built; the C ABI's default is 0)
DEBUG_JIT_NT = 12  # threads per workgroup of the run-time kernels (0: the form's own)
DEBUG_JIT_NS = 11  # samples of each pixel in flight per workgroup of the run-time kernels (0: the form's default)
KERNEL_JIT_NONE, KERNEL_JIT_PENDING, KERNEL_JIT_READY, KERNEL_JIT_FAILED = 0, 1, 2, 3
JIT_MODE_FLAT, JIT_MODE_CULL, JIT_MODE_ROOM = 0, 1, 2  # sail_jit_compile kernel forms (include/sail_hip.h)
# applied to every Context at creation (tests set entries with monkeypatch.setitem)
DEBUG_DEFAULTS: dict = {}

# exported symbols (kept in sync with include/sail_hip.h; tests/test_capi_symbols.py checks both ways)
EXPORTS = (
    "sail_create", "sail_create_multi", "sail_set_debug", "sail_destroy", "sail_last_error", "sail_device_count", "sail_device_info", "sail_set_scene",
    "sail_update_objects", "sail_set_accum_mode", "sail_set_partition", "sail_set_launch_samples",
    "sail_render", "sail_render_schedule", "sail_reset", "sail_sync", "sail_readback", "sail_read_accum",
    "sail_filter", "sail_get_stats", "sail_camera", "sail_jitter_inverse", "sail_schedule",
    "sail_comm_unique_id", "sail_comm_init", "sail_reduce", "sail_accum_device_ptr", "sail_partition_tiles",
    "sail_prim_bounds", "sail_math_probe", "sail_pick", "sail_kernel_name", "sail_filter_ms",
    "sail_abi_version", "sail_accum_parts", "sail_save_accum", "sail_load_accum", "sail_jit_compile",
    "sail_get_kernel_info", "sail_kernel_ready", "sail_set_jit_cache", "sail_jit_prebuild",
    "sail_plan_reduce", "sail_plan_keep", "sail_plan_load_part",
)


class SailError(RuntimeError):
    pass


class Plugins(ctypes.Structure):
    _fields_ = [("shape_mask", ctypes.c_uint32), ("material_mask", ctypes.c_uint32),
                ("texture_mask", ctypes.c_uint32), ("light_mask", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_uint64), ("segments", ctypes.c_uint64),
                ("nominal_segments", ctypes.c_uint64), ("kernel_ms", ctypes.c_double),
                ("last_launch_ms", ctypes.c_double), ("launches", ctypes.c_uint32)]


class KernelInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 64), ("build_id", ctypes.c_uint64), ("jit_state", ctypes.c_int),
                ("jit_from_cache", ctypes.c_int), ("jit_compile_ms", ctypes.c_double), ("jit_build_id", ctypes.c_uint64),
                ("jit_error", ctypes.c_char * 256)]


class ReducePlan(ctypes.Structure):
    _fields_ = [("receives", ctypes.c_int), ("tiles", ctypes.c_int), ("aov_owner", ctypes.c_int),
                ("send_own_aovs", ctypes.c_int), ("samples", ctypes.c_uint64)]


_SHAPES = {"cube": 1, "sphere": 2, "rectangle": 3, "cone": 4, "cylinder": 5, "disk": 6,
           "hyperboloid": 7, "paraboloid": 8, "cornellbox": 9}
_MATERIALS = {"matte": 1, "mirror": 2, "metal": 3, "glass": 4}
_TEXTURES = {"checkerboard": 5, "checkerboard2": 7, "bilerp": 8, "mixf": 9, "scale": 10, "uvf": 11}
_LIGHTS = {"area": 0, "point": 1, "spot": 2}


def plugin_masks(plugins: dict) -> tuple:
    """Scene.tracerConfig() plugin-name lists -> category bit masks (src/scene/scene.js:70-112)."""
    def mask(names, table):
        m = 0
        for nm in names:
            m |= 1 << table[nm]
        return m
    return (mask(plugins.get("shape", []), _SHAPES), mask(plugins.get("material", []), _MATERIALS),
            mask(plugins.get("texture", []), _TEXTURES), mask(plugins.get("light", []), _LIGHTS))


_lib = None


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libsail_hip.so (raises if it is absent: there is no CPU fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise SailError(f"HIP library not built: {p} (run python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(p)
    f32p = ctypes.POINTER(ctypes.c_float)
    f64p = ctypes.POINTER(ctypes.c_double)
    vp = ctypes.c_void_p
    sig = {
        "sail_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32]),
        "sail_create_multi": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                             ctypes.c_int, ctypes.c_uint32]),
        "sail_set_debug": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
        "sail_destroy": (None, [vp]),
        "sail_last_error": (ctypes.c_char_p, [vp]),
        "sail_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "sail_device_info": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
        "sail_set_scene": (ctypes.c_int, [vp, f32p, ctypes.c_int, f32p, ctypes.c_int, f32p, ctypes.c_int, ctypes.POINTER(Plugins)]),
        "sail_update_objects": (ctypes.c_int, [vp, f32p, ctypes.c_int]),
        "sail_set_accum_mode": (ctypes.c_int, [vp, ctypes.c_int]),
        "sail_set_partition": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
        "sail_set_launch_samples": (ctypes.c_int, [vp, ctypes.c_int]),
        "sail_render": (ctypes.c_int, [vp, f32p, f32p, ctypes.c_float, ctypes.c_int]),
        "sail_render_schedule": (ctypes.c_int, [vp, f32p, f32p, f32p, ctypes.c_int, ctypes.c_int]),
        "sail_reset": (ctypes.c_int, [vp]),
        "sail_sync": (ctypes.c_int, [vp]),
        "sail_readback": (ctypes.c_int, [vp, f32p, f32p, f32p]),
        "sail_read_accum": (ctypes.c_int, [vp, f32p]),
        "sail_filter": (ctypes.c_int, [vp, ctypes.c_int, f32p, ctypes.c_float, ctypes.c_float, ctypes.c_float, f32p, ctypes.POINTER(ctypes.c_uint8)]),
        "sail_get_stats": (ctypes.c_int, [vp, ctypes.POINTER(Stats)]),
        "sail_camera": (ctypes.c_int, [f64p, f64p, f64p, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, f64p]),
        "sail_jitter_inverse": (ctypes.c_int, [f64p, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int, f32p]),
        "sail_schedule": (ctypes.c_int, [f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p, f32p]),
        "sail_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
        "sail_comm_init": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]),
        "sail_reduce": (ctypes.c_int, [vp, ctypes.c_int]),
        "sail_accum_device_ptr": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]),
        "sail_partition_tiles": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
        "sail_prim_bounds": (ctypes.c_int, [f32p, ctypes.c_int, ctypes.c_int, f32p]),
        "sail_math_probe": (ctypes.c_int, [ctypes.c_int, f32p, f32p, f32p, ctypes.c_int]),
        "sail_abi_version": (ctypes.c_int, []),
        "sail_pick": (ctypes.c_int, [vp, f32p, ctypes.c_int, ctypes.POINTER(ctypes.c_int32), f32p]),
        "sail_kernel_name": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int]),
        "sail_filter_ms": (ctypes.c_int, [vp, f64p]),
        "sail_accum_parts": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int)]),
        "sail_save_accum": (ctypes.c_int, [vp, ctypes.c_int, f32p, ctypes.POINTER(ctypes.c_uint64)]),
        "sail_load_accum": (ctypes.c_int, [vp, ctypes.c_int, f32p, ctypes.c_uint64]),
        "sail_jit_compile": (ctypes.c_int, [ctypes.POINTER(Plugins), ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                            vp, ctypes.POINTER(ctypes.c_size_t)]),
        "sail_get_kernel_info": (ctypes.c_int, [vp, ctypes.POINTER(KernelInfo)]),
        "sail_kernel_ready": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
        "sail_set_jit_cache": (ctypes.c_int, [ctypes.c_char_p]),
        "sail_jit_prebuild": (ctypes.c_int, [f32p, ctypes.c_int, f32p, ctypes.c_int, f32p, ctypes.c_int, ctypes.POINTER(Plugins),
                                             ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
        "sail_plan_reduce": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ReducePlan)]),
        "sail_plan_keep": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p, f32p]),
        "sail_plan_load_part": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int,
                                               ctypes.c_int, ctypes.c_uint64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _ptr(a: Optional[np.ndarray], ct=ctypes.c_float):
    if a is None:
        return ctypes.cast(None, ctypes.POINTER(ct))
    return a.ctypes.data_as(ctypes.POINTER(ct))


# ---- host math (no device needed) ----------------------------------------------------------------------
def camera(eye, center, up=(0.0, 1.0, 0.0), fovy=55.0, aspect=1.0, znear=1.0, zfar=100.0) -> np.ndarray:
    lib = load()
    e, c, u = (np.ascontiguousarray(np.asarray(v, dtype=np.float64)) for v in (eye, center, up))
    out = np.zeros(16, dtype=np.float64)
    rc = lib.sail_camera(_ptr(e, ctypes.c_double), _ptr(c, ctypes.c_double), _ptr(u, ctypes.c_double),
                         fovy, aspect, znear, zfar, _ptr(out, ctypes.c_double))
    if rc:
        raise SailError(f"sail_camera: {rc}")
    return out.reshape(4, 4)


def jitter_inverse(mvp: np.ndarray, jx: float, jy: float, width: int, height: int) -> np.ndarray:
    lib = load()
    m = np.ascontiguousarray(np.asarray(mvp, dtype=np.float64).reshape(16))
    out = np.zeros(16, dtype=np.float32)
    rc = lib.sail_jitter_inverse(_ptr(m, ctypes.c_double), jx, jy, width, height, _ptr(out))
    if rc:
        raise SailError(f"sail_jitter_inverse: {rc}")
    return out


def schedule(mvp: np.ndarray, width: int, height: int, k0: int, spp: int):
    """The frozen sample schedule: (spp x 16 f32 inverse matrices, spp f32 seeds)."""
    lib = load()
    m = np.ascontiguousarray(np.asarray(mvp, dtype=np.float64).reshape(16))
    inv = np.zeros((spp, 16), dtype=np.float32)
    seeds = np.zeros(spp, dtype=np.float32)
    rc = lib.sail_schedule(_ptr(m, ctypes.c_double), width, height, k0, spp, _ptr(inv), _ptr(seeds))
    if rc:
        raise SailError(f"sail_schedule: {rc}")
    return inv, seeds


def partition_tiles(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """(x0, y0, w, h) of the 64x64 tiles a rank owns (tile t -> rank t % world)."""
    lib = load()
    n = lib.sail_partition_tiles(width, height, rank, world, ctypes.cast(None, ctypes.POINTER(ctypes.c_int)), 0)
    if n < 0:
        raise SailError(f"sail_partition_tiles: {n}")
    out = np.zeros((max(n, 1), 4), dtype=np.int32)
    lib.sail_partition_tiles(width, height, rank, world, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), n)
    return out[:n]


def plan_reduce(width: int, height: int, rank: int, world: int, mode: int, k: int, root: int = 0) -> dict:
    """The library's reduce bookkeeping for one rank (sail_plan_reduce, host-only): receives, tiles, aov_owner,
    send_own_aovs, samples."""
    lib = load()
    p = ReducePlan()
    rc = lib.sail_plan_reduce(width, height, rank, world, mode, k, root, ctypes.byref(p))
    if rc:
        raise SailError(f"sail_plan_reduce: {rc}: {lib.sail_last_error(None).decode()}")
    return {f: getattr(p, f) for f, _ in ReducePlan._fields_}


def plan_keep(width: int, height: int, rank: int, world: int, mode: int, sums: np.ndarray) -> np.ndarray:
    """What a rank keeps of a whole-frame accumulator when resuming from it (sail_plan_keep, host-only)."""
    lib = load()
    src = _f32(sums).reshape(-1)
    if src.size != width * height * 4:
        raise SailError("plan_keep: sums must hold W*H*4 floats")
    out = np.empty_like(src)
    rc = lib.sail_plan_keep(width, height, rank, world, mode, _ptr(src), _ptr(out))
    if rc:
        raise SailError(f"sail_plan_keep: {rc}")
    return out.reshape(height, width, 4)


class LoadParts:
    """A part-wise checkpoint load's bookkeeping (sail_plan_load_part, host-only): the parts still missing and the
    checkpoint's sample index."""

    def __init__(self, parts: int):
        self.parts = parts
        self.missing = ctypes.c_uint64(0)
        self.k = ctypes.c_uint64(0)

    def load(self, part: int, k: int) -> None:
        lib = load()
        rc = lib.sail_plan_load_part(ctypes.byref(self.missing), ctypes.byref(self.k), self.parts, part, k)
        if rc:
            raise SailError(lib.sail_last_error(None).decode())

    @property
    def complete(self) -> bool:
        return self.missing.value == 0


def prim_bounds(objects, n: int, tn: int) -> np.ndarray:
    """Object3D.boundbox() answered by the pre-cull's padded bounds: (n, 2, 3) min / max per object row
    (host-only, no device)."""
    lib = load()
    rows = _f32(objects).reshape(-1)
    if rows.size < 18 * n:
        raise SailError("prim_bounds: fewer than 18 floats per row")
    out = np.zeros((max(n, 1), 6), dtype=np.float32)
    rc = lib.sail_prim_bounds(_ptr(rows), n, tn, _ptr(out))
    if rc:
        raise SailError(f"sail_prim_bounds: {rc}")
    return out[:n].reshape(n, 2, 3)


def math_probe(fn: int, x: np.ndarray, y: Optional[np.ndarray] = None) -> np.ndarray:
    lib = load()
    x = _f32(x)
    y = _f32(np.zeros_like(x) if y is None else y)
    out = np.zeros_like(x)
    rc = lib.sail_math_probe(fn, _ptr(x), _ptr(y), _ptr(out), int(x.size))
    if rc:
        raise SailError(f"sail_math_probe: {lib.sail_last_error(None).decode()}")
    return out


def device_count() -> int:
    lib = load()
    n = ctypes.c_int(0)
    lib.sail_device_count(ctypes.byref(n))
    return n.value


def device_info(device: int = 0):
    """(compute units, peak engine clock in Hz) of a device."""
    lib = load()
    cus, khz = ctypes.c_int(0), ctypes.c_int(0)
    if lib.sail_device_info(device, ctypes.byref(cus), ctypes.byref(khz)) != 0:
        raise SailError(f"sail_device_info({device}) failed")
    return cus.value, khz.value * 1e3


def set_jit_cache(path: Optional[str]):
    """The process-wide user cache of run-time code objects (None: the default under ~/.cache, "": none)."""
    load().sail_set_jit_cache(None if path is None else path.encode())


def jit_prebuild(sc: dict, arch: str = "gfx950", cache_dir: Optional[str] = None) -> bool:
    """Host-only: build the run-time kernel a default context derives for scene `sc` into `cache_dir` (default: the
    cache shipped beside the library, sail_amd/lib/jit). Returns whether the scene gets one."""
    lib = load()
    o, t, l = _f32(sc["objects"]), _f32(sc["texparams"]), _f32(sc["lights"])
    pl = Plugins(*[int(m) for m in plugin_masks(sc["plugins"])])
    built = ctypes.c_int(0)
    d = cache_dir or os.path.join(_HERE, "lib", "jit")
    rc = lib.sail_jit_prebuild(_ptr(o), sc["n"], _ptr(t), sc["tn"], _ptr(l), sc["ln"], ctypes.byref(pl), arch.encode(),
                               d.encode(), ctypes.byref(built))
    if rc:
        raise SailError(f"sail_jit_prebuild: {rc}: {lib.sail_last_error(None).decode()}")
    return bool(built.value)


def comm_unique_id() -> bytes:
    lib = load()
    buf = ctypes.create_string_buffer(128)
    rc = lib.sail_comm_unique_id(buf)
    if rc:
        raise SailError(f"sail_comm_unique_id: {lib.sail_last_error(None).decode()}")
    return buf.raw


class Context:
    """A device context: the MI355X counterpart of Sail's Renderer/Tracer GPU state. With `devices` (a list of
    device ordinals) it is one multi-device context (sail_create_multi): the frame is split across them and
    reduced into device 0 on readback."""

    def __init__(self, width: int, height: int, device: int = -1, flags: int = 0, devices: Optional[Sequence[int]] = None,
                 debug: Optional[dict] = None):
        self.lib = load()
        self.W, self.H = int(width), int(height)
        h = ctypes.c_void_p()
        if devices is not None:
            dv = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            rc = self.lib.sail_create_multi(ctypes.byref(h), self.W, self.H, dv, len(devices), flags)
            what = "sail_create_multi"
        else:
            rc = self.lib.sail_create(ctypes.byref(h), self.W, self.H, device, flags)
            what = "sail_create"
        if rc:
            raise SailError(f"{what}: {rc}: {self.lib.sail_last_error(None).decode()}")
        self.h = h
        self._accum_mode = ACCUM_SUM          # the C ABI's default (sail_create)
        self._partition = (0, 1, PART_TILES)  # (rank, world, mode): checkpoints record and check these
        # the tests and bench.py want the scene's run-time kernel from the first launch (the C ABI's interactive default,
        # 0, launches the precompiled kernel until the background build is done; tests set 0 to render across the swap)
        for opt, val in {DEBUG_JIT_WAIT: -1, **DEBUG_DEFAULTS, **(debug or {})}.items():
            self.set_debug(opt, val)

    def set_debug(self, option: int, value: int):
        self._check(self.lib.sail_set_debug(self.h, int(option), int(value)), "sail_set_debug")

    def _check(self, rc: int, what: str):
        if rc:
            raise SailError(f"{what}: {rc}: {self.lib.sail_last_error(self.h).decode()}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.sail_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, objects, n: int, texparams, tn: int, lights, ln: int, masks: Sequence[int]):
        o, t, l = _f32(objects), _f32(texparams), _f32(lights)
        pl = Plugins(*[int(m) for m in masks])
        self._check(self.lib.sail_set_scene(self.h, _ptr(o), n, _ptr(t), tn, _ptr(l), ln, ctypes.byref(pl)),
                    "sail_set_scene")

    def set_scene_dict(self, sc: dict):
        self.set_scene(sc["objects"], sc["n"], sc["texparams"], sc["tn"], sc["lights"], sc["ln"],
                       plugin_masks(sc["plugins"]))

    def set_accum_mode(self, mode: int):
        self._check(self.lib.sail_set_accum_mode(self.h, mode), "sail_set_accum_mode")
        self._accum_mode = int(mode)

    def set_partition(self, rank: int, world: int, mode: int = PART_TILES):
        self._check(self.lib.sail_set_partition(self.h, rank, world, mode), "sail_set_partition")
        self._partition = (int(rank), int(world), int(mode))

    def set_launch_samples(self, spp: int):
        self._check(self.lib.sail_set_launch_samples(self.h, spp), "sail_set_launch_samples")

    def render_schedule(self, inv: np.ndarray, seeds: np.ndarray, eye, max_bounces: int):
        inv, seeds, e = _f32(inv), _f32(seeds), _f32(eye)
        self._check(self.lib.sail_render_schedule(self.h, _ptr(inv), _ptr(seeds), _ptr(e), int(seeds.size), max_bounces),
                    "sail_render_schedule")

    def render(self, inv: np.ndarray, eye, seed: float, max_bounces: int):
        inv, e = _f32(inv), _f32(eye)
        self._check(self.lib.sail_render(self.h, _ptr(inv), _ptr(e), float(seed), max_bounces), "sail_render")

    def reset(self):
        self._check(self.lib.sail_reset(self.h), "sail_reset")

    def sync(self):
        self._check(self.lib.sail_sync(self.h), "sail_sync")

    def readback(self, aov: bool = False):
        rgba = np.zeros((self.H, self.W, 4), dtype=np.float32)
        n = p = None
        if aov:
            n = np.zeros_like(rgba)
            p = np.zeros_like(rgba)
        self._check(self.lib.sail_readback(self.h, _ptr(rgba), _ptr(n), _ptr(p)), "sail_readback")
        return (rgba, n, p) if aov else rgba

    def read_accum(self) -> np.ndarray:
        rgba = np.zeros((self.H, self.W, 4), dtype=np.float32)
        self._check(self.lib.sail_read_accum(self.h, _ptr(rgba)), "sail_read_accum")
        return rgba

    def filter(self, kind: int, weights16=None, rx: float = 0.0, ry: float = 0.0, gamma_c: float = 2.2,
               want_u8: bool = False):
        out = np.zeros((self.H, self.W, 4), dtype=np.float32)
        out8 = np.zeros((self.H, self.W, 4), dtype=np.uint8) if want_u8 else None
        w = _f32(weights16) if weights16 is not None else None
        self._check(self.lib.sail_filter(self.h, kind, _ptr(w), rx, ry, gamma_c, _ptr(out),
                                         _ptr(out8, ctypes.c_uint8)), "sail_filter")
        return (out, out8) if want_u8 else out

    def pick(self, rays) -> tuple:
        """rays: (count, 6) origin+direction -> (object row index or -1, distance) per ray"""
        r = _f32(rays).reshape(-1, 6)
        idx = np.zeros(len(r), dtype=np.int32)
        t = np.zeros(len(r), dtype=np.float32)
        self._check(self.lib.sail_pick(self.h, _ptr(r), len(r), _ptr(idx, ctypes.c_int32), _ptr(t)), "sail_pick")
        return idx, t

    def filter_ms(self) -> float:
        v = ctypes.c_double()
        self._check(self.lib.sail_filter_ms(self.h, ctypes.byref(v)), "sail_filter_ms")
        return v.value

    def kernel_name(self) -> str:
        buf = ctypes.create_string_buffer(64)
        self._check(self.lib.sail_kernel_name(self.h, buf, 64), "sail_kernel_name")
        return buf.value.decode()

    def kernel_info(self) -> dict:
        k = KernelInfo()
        self._check(self.lib.sail_get_kernel_info(self.h, ctypes.byref(k)), "sail_get_kernel_info")
        return {"name": k.name.decode(), "build_id": f"{k.build_id:016x}", "jit_state": k.jit_state,
                "jit_from_cache": k.jit_from_cache, "jit_compile_ms": k.jit_compile_ms,
                "jit_build_id": f"{k.jit_build_id:016x}", "jit_error": k.jit_error.decode()}

    def kernel_id(self) -> str:
        """the last launch's kernel and its build identity, "name@hex16" (profiles are matched to kernels by it)"""
        k = self.kernel_info()
        return f"{k['name']}@{k['build_id']}"

    def kernel_ready(self, timeout_ms: int = -1) -> bool:
        r = ctypes.c_int(0)
        self._check(self.lib.sail_kernel_ready(self.h, int(timeout_ms), ctypes.byref(r)), "sail_kernel_ready")
        return bool(r.value)

    def stats(self) -> Stats:
        s = Stats()
        self._check(self.lib.sail_get_stats(self.h, ctypes.byref(s)), "sail_get_stats")
        return s

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        self._check(self.lib.sail_comm_init(self.h, uid, nranks, rank), "sail_comm_init")

    def reduce(self, root: int = 0):
        self._check(self.lib.sail_reduce(self.h, root), "sail_reduce")

    def _parts(self) -> int:
        n = ctypes.c_int(0)
        self._check(self.lib.sail_accum_parts(self.h, ctypes.byref(n)), "sail_accum_parts")
        return n.value

    def save(self) -> dict:
        """Checkpoint of the progressive render: {"k": next sample index, "parts": [H x W x 4 f32 accumulator per
        device], and the context it belongs to: width, height, accum_mode, partition (rank, world, mode)}
        (sail_save_accum)"""
        parts, k = [], ctypes.c_uint64(0)
        for i in range(self._parts()):
            a = np.zeros((self.H, self.W, 4), dtype=np.float32)
            self._check(self.lib.sail_save_accum(self.h, i, _ptr(a), ctypes.byref(k)), "sail_save_accum")
            parts.append(a)
        return {"k": int(k.value), "parts": parts, "width": self.W, "height": self.H,
                "accum_mode": self._accum_mode, "partition": list(self._partition)}

    def load(self, ckpt: dict):
        """Resume from save()'s checkpoint (every part, into a context of the same size, accumulation mode, partition
        and device count), or from a whole-frame accumulator {"k": k, "frame": H x W x 4} (sail_load_accum part -1).
        A checkpoint that does not fit this context raises SailError before anything is copied."""
        def arr(a, what):
            a = _f32(a)
            if a.shape != (self.H, self.W, 4):
                raise SailError(f"Context.load: {what} has shape {a.shape}, this context needs {(self.H, self.W, 4)}")
            return a
        for key, mine in (("width", self.W), ("height", self.H), ("accum_mode", self._accum_mode)):
            if key in ckpt and int(ckpt[key]) != mine:
                raise SailError(f"Context.load: checkpoint {key} {ckpt[key]} differs from this context's {mine}")
        if "partition" in ckpt and tuple(int(v) for v in ckpt["partition"]) != self._partition:
            raise SailError(f"Context.load: checkpoint partition {tuple(ckpt['partition'])} differs from {self._partition}")
        if "frame" in ckpt:
            f = arr(ckpt["frame"], "frame")
            self._check(self.lib.sail_load_accum(self.h, -1, _ptr(f), int(ckpt["k"])), "sail_load_accum")
            return
        parts = [arr(a, f"part {i}") for i, a in enumerate(ckpt["parts"])]
        if len(parts) != self._parts():
            raise SailError(f"Context.load: checkpoint has {len(parts)} parts, this context {self._parts()}")
        for i, a in enumerate(parts):
            self._check(self.lib.sail_load_accum(self.h, i, _ptr(a), int(ckpt["k"])), "sail_load_accum")

    def accum_device_ptr(self):
        p = ctypes.c_void_p()
        b = ctypes.c_size_t()
        self._check(self.lib.sail_accum_device_ptr(self.h, ctypes.byref(p), ctypes.byref(b)), "sail_accum_device_ptr")
        return p.value, b.value
