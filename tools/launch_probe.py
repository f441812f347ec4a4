import json, os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
from sail_amd import capi
import bench
sc = bench.load_scene("C1"); W, H, B, spp = 1920, 1080, 8, 64
mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
inv, seeds = capi.schedule(mvp, W, H, 0, spp)
for L in (1, 2, 4, 8, 16, 32, 64):
    ctx = capi.Context(W, H); ctx.set_scene_dict(sc); ctx.set_launch_samples(L)
    ctx.render_schedule(inv, seeds, sc["eye"], B); ctx.sync()
    ctx.reset(); t0 = time.perf_counter(); ctx.render_schedule(inv, seeds, sc["eye"], B); ctx.sync(); dt = time.perf_counter() - t0
    st = ctx.stats(); ctx.close()
    print(json.dumps({"launch_spp": L, "wall_ms": round(dt * 1e3, 2), "kernel_ms_per_sample": round(st.kernel_ms / spp, 4), "launches": st.launches}))
# one sample per call, the way Renderer.render() issues frames: back to back, and with a host sync per frame
for sync in (False, True):
    ctx = capi.Context(W, H); ctx.set_scene_dict(sc)
    for k in range(4):
        ctx.render(inv[k], sc["eye"], float(seeds[k]), B)
    ctx.sync(); ctx.reset()
    t0 = time.perf_counter()
    for k in range(spp):
        ctx.render(inv[k], sc["eye"], float(seeds[k]), B)
        if sync:
            ctx.sync()
    ctx.sync(); dt = time.perf_counter() - t0
    st = ctx.stats(); ctx.close()
    print(json.dumps({"per_call": True, "sync_each": sync, "wall_ms": round(dt * 1e3, 2), "kernel_ms_per_sample": round(st.kernel_ms / spp, 4), "launches": st.launches}))
