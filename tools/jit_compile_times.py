#!/usr/bin/env python3
"""Run-time kernel build latency per form, on the GPU box: for each scene, a fresh process with a
copy of the library that has no shipped cache beside it, an empty user cache and the compiler's own cache off
(AMD_COMGR_CACHE=0) times sail_set_scene (the kernel's build starts in the background; it must return at once) and the
build itself (sail_get_kernel_info.jit_compile_ms); a second process with the now-warm user cache times sail_set_scene
again, which then loads the code object itself. JSON lines on stdout.
Usage: tools/jit_compile_times.py [SCENE ...]"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
from sail_amd import capi
capi.load(sys.argv[2]); capi._lib = capi.load(sys.argv[2])
capi.set_jit_cache(sys.argv[3])
sc = json.load(open(sys.argv[4]))[sys.argv[5]]
ctx = capi.Context(64, 64, debug={capi.DEBUG_JIT_WAIT: 0})
t0 = time.perf_counter(); ctx.set_scene_dict(sc); set_ms = (time.perf_counter() - t0) * 1e3
state_after_set = ctx.kernel_info()["jit_state"]
t0 = time.perf_counter(); ready = ctx.kernel_ready(-1); wait_ms = (time.perf_counter() - t0) * 1e3
k = ctx.kernel_info()
print(json.dumps({"set_scene_ms": round(set_ms, 2), "state_after_set_scene": ["none", "pending", "ready", "failed"][state_after_set],
                  "wait_ms": round(wait_ms, 1), "ready": ready, "compile_ms": round(k["jit_compile_ms"], 1),
                  "from_cache": ["hipRTC", "user cache", "shipped cache"][k["jit_from_cache"]], "error": k["jit_error"]}))
ctx.close()
"""


def main():
    scenes = sys.argv[1:] or ["C1", "C3", "C4", "UI", "ALL", "AREA"]
    frozen = os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")
    with tempfile.TemporaryDirectory() as td:
        lib = os.path.join(td, "lib", "libsail_hip.so")
        os.makedirs(os.path.dirname(lib))
        shutil.copy(os.path.join(ROOT, "sail_amd", "lib", "libsail_hip.so"), lib)  # no jit/ beside the copy
        env = dict(os.environ, AMD_COMGR_CACHE="0")
        for name in scenes:
            cache = os.path.join(td, "cache_" + name)
            rec = {"scene": name}
            for label in ("cold", "warm"):
                r = subprocess.run([sys.executable, "-c", CHILD, ROOT, lib, cache, frozen, name], env=env,
                                   capture_output=True, text=True, timeout=300)
                if r.returncode != 0:
                    raise SystemExit(r.stderr[-2000:])
                rec[label] = json.loads(r.stdout.strip().splitlines()[-1])
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
