"""CPU: libsail_hip.so loads and exports exactly the entry points include/sail_hip.h declares; host-only
entry points work without a device and device entry points fail loudly (no silent CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from sail_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sail_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sail_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_python_binding_set():
    assert header_functions() == sorted(capi.EXPORTS)


def test_library_exports_every_declared_symbol():
    assert os.path.exists(capi.LIB_PATH), "build() must produce sail_amd/lib/libsail_hip.so"
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing
    lib = capi.load()
    for f in header_functions():
        assert hasattr(lib, f)


def test_abi_version():
    assert capi.load().sail_abi_version() == 4


def test_library_targets_gfx950(tmp_path):
    # llvm-objdump --offloading extracts the bundles next to its input: give it a copy in a scratch directory
    import shutil
    lib = str(tmp_path / "libsail_hip.so")
    shutil.copy(capi.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                         capture_output=True, text=True)
    text = out.stdout + out.stderr
    if "gfx950" not in text:
        # older objdump: look for the target id string in the embedded bundle
        blob = open(capi.LIB_PATH, "rb").read()
        assert b"gfx950" in blob
    else:
        assert "gfx950" in text


def test_device_entry_points_fail_loudly_without_gpu():
    if capi.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(capi.SailError):
        capi.Context(16, 16)
    with pytest.raises(capi.SailError):
        capi.Context(16, 16, devices=[0, 0])
    with pytest.raises(capi.SailError):
        capi.Context(16, 16, devices=[0, 1, 0])   # neither all distinct nor all the same device


def test_bad_arguments_are_rejected():
    lib = capi.load()
    with pytest.raises(capi.SailError):
        capi.schedule(np.eye(4) * 0.0, 16, 16, 0, 2)  # singular matrix
    null = capi._ptr(None, ctypes.c_int)
    assert lib.sail_partition_tiles(0, 10, 0, 1, null, 0) < 0
    assert lib.sail_partition_tiles(10, 10, 2, 2, null, 0) < 0


def test_null_context_is_rejected():
    lib = capi.load()
    for fn in ("sail_reset", "sail_sync"):
        assert getattr(lib, fn)(None) == -1
    assert lib.sail_set_debug(None, capi.DEBUG_CULL_MIN_PRIMS, 0) == -1
    assert lib.sail_reduce(None, 0) == -1
