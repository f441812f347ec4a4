"""CPU: the run-time compiled plugin-set kernels (sail_jit.cpp) through the host-only sail_jit_compile. hipRTC compiles
the kernel sources embedded in the library with the product's floating-point flags: for the all-plugin set the flat
kernel pair is instruction-for-instruction the precompiled all-plugin kernel pair (so the run-time path cannot differ
in contraction, fast-math or packing), and specialised sets compile to the kernel names the contexts load."""
import ctypes
import os
import re
import shutil
import subprocess
import sys

import pytest

from sail_amd import capi

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _torch_runtime_loaded():
    """PyTorch-ROCm brings its own HIP runtime, hipRTC and comgr (an older ROCm, same sonames). Importing it first is
    the common case in a process that uses this library, and the run-time kernels must not depend on it."""
    import torch  # noqa: F401
    maps = open("/proc/self/maps").read()
    return "torch/lib/libhiprtc" in maps or "torch/lib/libamdhip64" in maps


def _compile(masks, mode, rows=()):
    lib = capi.load()
    pl = capi.Plugins(*masks)
    types = (ctypes.c_int32 * max(len(rows), 1))(*rows)
    n = ctypes.c_size_t(0)
    assert lib.sail_jit_compile(ctypes.byref(pl), mode, types, len(rows), None, ctypes.byref(n)) == 0, lib.sail_last_error(None)
    buf = ctypes.create_string_buffer(n.value)
    assert lib.sail_jit_compile(ctypes.byref(pl), mode, types, len(rows), buf, ctypes.byref(n)) == 0
    small = ctypes.c_size_t(16)
    assert lib.sail_jit_compile(ctypes.byref(pl), mode, types, len(rows), buf, ctypes.byref(small)) != 0  # too small
    return buf.raw


def _kernels(asm):
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = out.setdefault(m.group(1), [])
            continue
        t = re.sub(r"<[^>]*>|\s*//.*", "", re.sub(r"^\s*[0-9a-f]+:\s*", "", line.strip()))
        if cur is not None and t and not t.startswith(("s_nop", "s_code_end")):  # padding after the last function
            cur.append(t)
    return out


def _disasm(path):
    return subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", path], capture_output=True, text=True, check=True).stdout


@pytest.fixture(scope="module")
def product_kernels(tmp_path_factory):
    d = tmp_path_factory.mktemp("prod")
    lib = d / "libsail_hip.so"
    shutil.copy(capi.LIB_PATH, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], capture_output=True, text=True, cwd=d)
    co = [p for p in d.iterdir() if "amdgcn" in p.name]
    assert co, "no gfx950 code object in the library"
    return _kernels(_disasm(str(co[0])))


def test_all_plugin_jit_equals_precompiled_generic(tmp_path, product_kernels):
    assert _torch_runtime_loaded()  # the library's own toolchain compiles anyway (sail_jit.cpp: dlmopen)
    code = _compile([0xFFFFFFFF] * 4, 0)
    p = tmp_path / "jit.co"
    p.write_bytes(code)
    jit = _kernels(_disasm(str(p)))
    assert set(jit) == {"sail_trace_kernel_jit", "sail_trace_kernel_jit_grouped"}
    assert jit["sail_trace_kernel_jit"] == product_kernels["sail_trace_kernel"]
    assert jit["sail_trace_kernel_jit_grouped"] == product_kernels["sail_trace_kernel_grouped"]


@pytest.mark.parametrize("scene,mode,name", [("ALL", 0, "sail_trace_kernel_jit"), ("C4", 1, "sail_trace_kernel_cull_jit"),
                                             ("ALL", 2, "sail_trace_kernel_jit"), ("C3", 2, "sail_trace_kernel_jit")])
def test_plugin_set_kernel_compiles(tmp_path, fixtures, scene, mode, name):
    """every kernel form (sail_jit_mode: flat, pre-cull, flat in the room kernel's form) compiles for a scene's set"""
    code = _compile(capi.plugin_masks(fixtures["scenes"][scene]["plugins"]), mode)
    p = tmp_path / "jit.co"
    p.write_bytes(code)
    asm = _disasm(str(p))
    assert set(_kernels(asm)) == {name, name + "_grouped"}
    assert "v_pk_" not in asm  # no SLP packing, as the product build (-fno-slp-vectorize)


def test_room_form_of_the_room_set_equals_precompiled_room_kernel(tmp_path, product_kernels):
    """SAIL_JIT_MODE_ROOM compiled for the room kernel's own plugin set is the same kernel pair as the precompiled
    sail_trace_kernel_room (same source, launch bounds and flags)"""
    shapes = sum(1 << t for t in (1, 2, 3, 9))  # SAIL_KSET_ROOM_SHAPES: Cube, Sphere, Rectangle, Cornellbox
    code = _compile([shapes, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF], 2)
    p = tmp_path / "jit.co"
    p.write_bytes(code)
    jit = _kernels(_disasm(str(p)))
    assert jit["sail_trace_kernel_jit"] == product_kernels["sail_trace_kernel_room"]
    assert jit["sail_trace_kernel_jit_grouped"] == product_kernels["sail_trace_kernel_room_grouped"]


def test_cornell_set_flat_form_equals_precompiled_cornell_kernel(tmp_path, fixtures, product_kernels):
    """the flat form for the Cornell box's plugin set runs at the Cornell kernel's 8 waves: the same kernel pair"""
    code = _compile(capi.plugin_masks(fixtures["scenes"]["C1"]["plugins"]), 0)
    p = tmp_path / "jit.co"
    p.write_bytes(code)
    jit = _kernels(_disasm(str(p)))
    assert jit["sail_trace_kernel_jit"] == product_kernels["sail_trace_kernel_cornell"]
    assert jit["sail_trace_kernel_jit_grouped"] == product_kernels["sail_trace_kernel_cornell_grouped"]


@pytest.mark.parametrize("scene,mode", [("C1", 0), ("C3", 2), ("ALL", 2)])
def test_row_specialised_kernel_has_no_row_loop(tmp_path, fixtures, scene, mode):
    """compiled for the scene's rows (count and shape types), the kernel differs from the plugin-set-only one and
    still compiles to the same kernel names"""
    sc = fixtures["scenes"][scene]
    masks = capi.plugin_masks(sc["plugins"])
    types = [capi._SHAPES[b["shape"].lower()] for b in sc["boundbox"]]
    code = _compile(masks, mode, types)
    p = tmp_path / "jit.co"
    p.write_bytes(code)
    jit = _kernels(_disasm(str(p)))
    plain = _kernels(_disasm_bytes(tmp_path, _compile(masks, mode)))
    assert set(jit) == {"sail_trace_kernel_jit", "sail_trace_kernel_jit_grouped"}
    assert jit["sail_trace_kernel_jit"] != plain["sail_trace_kernel_jit"]


def _disasm_bytes(tmp_path, code):
    q = tmp_path / "plain.co"
    q.write_bytes(code)
    return _disasm(str(q))


def test_bad_specialisations_refused(fixtures):
    lib = capi.load()
    n = ctypes.c_size_t(0)
    pl = capi.Plugins(*capi.plugin_masks(fixtures["scenes"]["C1"]["plugins"]))
    none = (ctypes.c_int32 * 1)(0)
    assert lib.sail_jit_compile(ctypes.byref(pl), 3, none, 0, None, ctypes.byref(n)) != 0       # unknown form
    rect = (ctypes.c_int32 * 1)(3)                                                             # Rectangle: not compiled in
    assert lib.sail_jit_compile(ctypes.byref(pl), 0, rect, 1, None, ctypes.byref(n)) != 0
    assert lib.sail_jit_compile(ctypes.byref(pl), 1, (ctypes.c_int32 * 1)(1), 1, None, ctypes.byref(n)) != 0  # pre-cull
    assert lib.sail_jit_compile(ctypes.byref(pl), 0, (ctypes.c_int32 * 9)(*[1] * 9), 9, None, ctypes.byref(n)) != 0


def _child_compile(env, cache="", masks=(0x206, 6, 0, 0), mode=0):
    """sail_jit_compile in a child process (the library opens hipRTC once per process): (rc, message, code sha)"""
    child = (
        "import ctypes, hashlib, sys\n"
        f"sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})\n"
        "from sail_amd import capi\n"
        f"capi.set_jit_cache({cache!r})\n"
        f"lib = capi.load(); pl = capi.Plugins(*{tuple(masks)!r}); n = ctypes.c_size_t(0)\n"
        f"rc = lib.sail_jit_compile(ctypes.byref(pl), {mode}, None, 0, None, ctypes.byref(n))\n"
        "buf = ctypes.create_string_buffer(max(n.value, 1))\n"
        f"rc = rc or lib.sail_jit_compile(ctypes.byref(pl), {mode}, None, 0, buf, ctypes.byref(n))\n"
        "print(rc, hashlib.sha256(buf.raw).hexdigest() if rc == 0 else '-', lib.sail_last_error(None).decode())\n")
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rc, sha, msg = (r.stdout.strip().splitlines()[-1].split(" ", 2) + [""])[:3]
    return int(rc), msg, sha


def test_missing_hiprtc_is_an_error_not_a_crash(tmp_path):
    """SAIL_HIPRTC naming a missing library: sail_jit_compile fails with the dlmopen message (contexts then keep the
    precompiled kernels, tests/test_gpu_jit_fallback.py); no disk cache, so the code object must be compiled"""
    env = dict(os.environ, SAIL_HIPRTC=str(tmp_path / "missing" / "libhiprtc.so.7"))
    rc, msg, _ = _child_compile(env)
    assert rc != 0 and "dlmopen" in msg, msg


def _torch_hiprtc():
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "libhiprtc.so")
    return p if os.path.exists(p) else None


def test_other_hiprtc_is_refused(tmp_path):
    """A hipRTC of another ROCm (PyTorch's, ROCm 7.0, under the same soname) compiles, but its code object's producer
    is not the compiler that built this library's kernels: refused, so contexts keep the
    precompiled kernels rather than run a kernel whose arithmetic another code generator chose"""
    other = _torch_hiprtc()
    if other is None:
        pytest.skip("no second hipRTC in this image")
    env = dict(os.environ, SAIL_HIPRTC=other, AMD_COMGR_CACHE="0")
    rc, msg, _ = _child_compile(env)
    assert rc != 0 and "produced by clang" in msg, msg


def test_disk_cache_round_trip_and_corruption(tmp_path):
    """The code object lands in the user cache; a new process reads it back (same bytes); a corrupted file is
    rejected by its checksum and rebuilt, and the rebuilt file is whole again"""
    cache = str(tmp_path / "jit")
    env = dict(os.environ, AMD_COMGR_CACHE="0")
    masks = (0x206 | 8, 6, 0, 0)  # a set no other test compiles
    rc, _, sha1 = _child_compile(env, cache, masks)
    assert rc == 0
    files = sorted(os.listdir(cache))
    assert len(files) == 1 and files[0].endswith(".co")
    path = os.path.join(cache, files[0])
    raw = open(path, "rb").read()
    assert raw[:8] == b"SAILJIT1"
    rc, _, sha2 = _child_compile(dict(env, SAIL_HIPRTC=str(tmp_path / "none.so")), cache, masks)  # no compiler needed
    assert rc == 0 and sha2 == sha1
    bad = bytearray(raw)
    bad[len(bad) // 2] ^= 0xFF
    open(path, "wb").write(bytes(bad))
    rc, msg, _ = _child_compile(dict(env, SAIL_HIPRTC=str(tmp_path / "none.so")), cache, masks)
    assert rc != 0 and "dlmopen" in msg  # the corrupted object is not loaded: a compiler would be needed
    rc, _, sha3 = _child_compile(env, cache, masks)
    assert rc == 0 and sha3 == sha1 and open(path, "rb").read() == raw


def test_prebuild_fills_the_shipped_cache_layout(tmp_path, fixtures):
    """sail_jit_prebuild derives the spec a default context would (the frozen scenes: rows, pre-cull and room forms)
    and writes its code object into the given directory; the Cornell form in both of its shapes (16 samples in flight
    for a large share of the frame, 1 for a rank of 8: sail_capi.cpp jitNsFor)"""
    for name, count in (("C1", 2), ("C4", 1)):
        d = tmp_path / name
        assert capi.jit_prebuild(fixtures["scenes"][name], cache_dir=str(d))
        files = os.listdir(d)
        assert len(files) == count and all(open(d / f, "rb").read(8) == b"SAILJIT1" for f in files)


@pytest.mark.gpu
def test_box_compiler_matches_precompiled_kernels(tmp_path, fixtures, product_kernels):
    """on the GPU box itself, the hipRTC the library opens there compiles the all-plugin, room and
    Cornell sets to exactly the precompiled kernels' instructions (no disk cache: compiled in this process)"""
    capi.set_jit_cache("")
    try:
        test_all_plugin_jit_equals_precompiled_generic(tmp_path, product_kernels)
        test_room_form_of_the_room_set_equals_precompiled_room_kernel(tmp_path, product_kernels)
        test_cornell_set_flat_form_equals_precompiled_cornell_kernel(tmp_path, fixtures, product_kernels)
    finally:
        capi.set_jit_cache(None)


def test_two_precull_compiles_in_one_process(tmp_path):
    """Regression: with one thread per background build, the second pre-cull-form compile of a process faulted inside
    hipRTC (found on the GPU box, reproduced here); builds now share one long-lived worker thread. No caches."""
    env = dict(os.environ, AMD_COMGR_CACHE="0")
    child = (
        "import ctypes, sys\n"
        f"sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})\n"
        "from sail_amd import capi\n"
        "capi.set_jit_cache('')\n"
        "lib = capi.load(); n = ctypes.c_size_t(0)\n"
        "for masks in ((0xFFFFFFFF,) * 4, (0x206, 6, 0, 0)):\n"
        "    pl = capi.Plugins(*masks)\n"
        "    print(lib.sail_jit_compile(ctypes.byref(pl), 1, None, 0, None, ctypes.byref(n)), flush=True)\n")
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.split() == ["0", "0"]


def test_fork_child_builds_and_exits(tmp_path):
    """after fork() the child has no build worker. The child gets a fresh queue, so a compile there runs
    instead of queueing for a thread that does not exist, and the child's exit does not wait for the parent's jobs.
    The parent starts its worker with one compile first. No caches."""
    env = dict(os.environ, AMD_COMGR_CACHE="0")
    child = (
        "import ctypes, os, sys\n"
        f"sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})\n"
        "from sail_amd import capi\n"
        "capi.set_jit_cache('')\n"
        "lib = capi.load(); n = ctypes.c_size_t(0)\n"
        "pl = capi.Plugins(0x206, 6, 0, 0)\n"
        "assert lib.sail_jit_compile(ctypes.byref(pl), 0, None, 0, None, ctypes.byref(n)) == 0\n"
        "pid = os.fork()\n"
        "if pid == 0:\n"
        "    pl2 = capi.Plugins(0x206 | 16, 6, 0, 0)\n"
        "    rc = lib.sail_jit_compile(ctypes.byref(pl2), 0, None, 0, None, ctypes.byref(n))\n"
        "    print('child', rc, flush=True)\n"
        "    os._exit(0 if rc == 0 else 3)\n"
        "_, st = os.waitpid(pid, 0)\n"
        "print('parent', os.waitstatus_to_exitcode(st), flush=True)\n")
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.split() == ["child", "0", "parent", "0"]


@pytest.mark.gpu
def test_context_churn_skips_stale_builds_and_exits_promptly(tmp_path):
    """ADVICE r05 on the box: contexts that set a scene, render without waiting for its run-time kernel and close leave
    queued builds nobody holds. The worker drops them, so the next context's own kernel waits for at most the build
    that is running plus its own, not for every stale one; and a process exiting with a build queued waits for the
    running compile only. Its frame equals the precompiled kernel's bit for bit. No caches (AMD_COMGR_CACHE=0, no
    user cache): every build is a real hipRTC compile."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = (
        "import json, sys, time\n"
        "import numpy as np\n"
        f"sys.path.insert(0, {root!r})\n"
        "from sail_amd import capi\n"
        "capi.set_jit_cache('')\n"
        f"scenes = json.load(open({os.path.join(root, 'tests', 'golden', 'fuzz_scenes.json')!r}))\n"
        "W, H, B, spp = 24, 16, 4, 2\n"
        "FLAT = {capi.DEBUG_CULL_MIN_PRIMS: 1000}\n"
        "def frame(name, debug):\n"
        "    sc = scenes[name]\n"
        "    inv, seeds = capi.schedule(np.array(sc['mvp_rowmajor']), W, H, 0, spp)\n"
        "    ctx = capi.Context(W, H, debug={**FLAT, **debug})\n"
        "    try:\n"
        "        ctx.set_scene_dict(sc)\n"
        "        t0 = time.time()\n"
        "        ready = ctx.kernel_ready(-1) if debug.get(capi.DEBUG_JIT_WAIT) == -1 else None\n"
        "        waited = time.time() - t0\n"
        "        ctx.render_schedule(inv, seeds, sc['eye'], B)\n"
        "        return ctx.read_accum(), ctx.kernel_name(), waited, ready\n"
        "    finally:\n"
        "        ctx.close()\n"
        "_, k1, t1, r1 = frame('F02', {capi.DEBUG_JIT_WAIT: -1})\n"
        "for name in ('F03', 'F04', 'F05', 'F06', 'F07', 'F08'):\n"
        "    frame(name, {capi.DEBUG_JIT_WAIT: 0})\n"
        "got, k2, t2, r2 = frame('F09', {capi.DEBUG_JIT_WAIT: -1})\n"
        "want, k3, _, _ = frame('F09', {capi.DEBUG_JIT: 0})\n"
        "same = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))\n"
        "frame('F10', {capi.DEBUG_JIT_WAIT: 0})\n"
        "print(json.dumps({'k1': k1, 'k2': k2, 'k3': k3, 't1': t1, 't2': t2, 'ready': [r1, r2], 'same': same,\n"
        "                  'end': time.time()}), flush=True)\n")
    env = dict(os.environ, AMD_COMGR_CACHE="0")
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=600)
    done = __import__("time").time()
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    import json
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(dict(res, exit_s=done - res["end"])))
    assert res["ready"] == [True, True], res
    assert res["k1"].startswith("sail_trace_kernel_jit") and res["k2"].startswith("sail_trace_kernel_jit"), res
    assert not res["k3"].startswith("sail_trace_kernel_jit"), res
    assert res["same"], res
    t1 = max(res["t1"], 0.5)
    # six stale builds queued ahead: run one by one they would take about 7 t1; dropped, at most the running one + its own
    assert res["t2"] < 4 * t1, res
    assert done - res["end"] < 2 * t1 + 10, (done - res["end"], res)  # exit waits for the running compile only
