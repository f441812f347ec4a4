#!/usr/bin/env python3
"""Headline benchmark: Msamples/s (path segments = paths x bounces per second) on BASELINE.json configs[1]:
the README Cornell box (frozen C1/C2 scene) at 1920x1080, 8 bounces, 1024 spp.

One step = one full progressive render of that frame: reset, 1024 samples through the trace megakernel,
and (N > 1) the RCCL sum-reduce of the per-rank float4 accumulators into rank 0. Frames are split into
64x64 tiles dealt round-robin to ranks (strong scaling: total work fixed). Inputs are resident on the
device before timing starts (scene rows uploaded by sail_set_scene; the per-sample camera schedule is
generated on the host and uploaded inside the step, ~64 KB, as the reference uploads uniforms per frame).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 either under torch.distributed.run (one
process per GPU, WORLD_SIZE = N, RCCL communicator per process) or as one process driving N GPUs through one
multi-device context (sail_create_multi: ncclCommInitAll + grouped reduce). Any other combination of --gpus and
WORLD_SIZE exits non-zero. Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sail_amd import capi  # noqa: E402

# BASELINE.json configs: [1] is the headline (default); the others are selectable with --config for study
CONFIGS = {
    "C2": {"workload": "cornell_box_readme_C2", "desc": "README Cornell box", "scene": "C1", "width": 1920, "height": 1080, "bounces": 8, "spp": 1024},
    "C3": {"workload": "materials_demo_C3", "desc": "materials demo", "scene": "C3", "width": 1920, "height": 1080, "bounces": 8, "spp": 1024},
    "C4": {"workload": "random64_C4", "desc": "random-64 primitives", "scene": "C4", "width": 3840, "height": 2160, "bounces": 12, "spp": 256},
    # converged render: sample split across ranks (full occupancy per GPU, RCCL sample-sum reduce), then the
    # Gaussian reconstruction filter on rank 0 inside the step (BASELINE configs[4])
    "C5": {"workload": "cornell_box_converged_C5", "desc": "README Cornell box (converged)", "scene": "C1g", "width": 1920,
           "height": 1080, "bounces": 16, "spp": 65536, "partition": "samples", "filter": "gaussian"},
}
CONFIG = CONFIGS["C2"]
FP32_PEAK_TFLOPS = 157.3   # MI355X FP32 vector (MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec
VALU_ISSUE_HW = 0.5      # one wave64 f32 VALU instruction per SIMD per 2 cycles (MI355X_MICROARCH.md)
VALU_ISSUE_PROBE = 0.42  # plain v_fma/mul/add_f32 wave-instructions per SIMD-cycle under load (tools/pk_probe.hip, profiles/r02_pk_probe.json)


def load_scene(name="C1"):
    """Frozen scene rows exported by this build's JS API (sail_amd/scenes/frozen.json; equal to the
    reference serializer's output, tests/test_js_host.py)."""
    with open(os.path.join(ROOT, "sail_amd", "scenes", "frozen.json")) as f:
        return json.load(f)[name]


def cpu_baseline_js(sc, masks, mvp, W, H, B, budget_s=12.0, threads=1, spp=8, full=False, frame_hash=False):
    """BASELINE.json's CPU baseline: the single-threaded JS/Node software shader (oracle/sail_soft.js, bit-exact
    with the C++ oracle and the HIP kernel) timed on the host on a bounded sample of the same frame: 32x32
    crops spiralling out from the centre, 8 spp each, until ~budget_s of render time (node start excluded).
    threads > 1: the same shader on that many worker_threads, crops dealt round-robin (SURVEY §8(d) optional)."""
    import shutil
    import subprocess
    import tempfile
    node = shutil.which("node") or shutil.which("nodejs")
    if node is None:
        return None
    c = 32
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    cx, cy = (W - c) // 2, (H - c) // 2
    if full:  # the whole frame (W and H multiples of 32), no time budget
        crops, budget_s = [[x, y, c, c] for y in range(0, H, c) for x in range(0, W, c)], 1e9
    else:
        offsets = sorted(((dx, dy) for dx in range(-30, 31) for dy in range(-17, 18)), key=lambda d: d[0] ** 2 + d[1] ** 2)
        crops = [[cx + dx * c, cy + dy * c, c, c] for dx, dy in offsets
                 if 0 <= cx + dx * c and 0 <= cy + dy * c and cx + dx * c + c <= W and cy + dy * c + c <= H]
    job = {"objects": sc["objects"], "n": sc["n"], "texparams": sc["texparams"], "tn": sc["tn"], "lights": sc["lights"],
           "ln": sc["ln"], "masks": list(masks), "W": W, "H": H, "inv": [float(v) for v in inv.reshape(-1)],
           "seeds": [float(v) for v in seeds], "eye": sc["eye"], "spp": spp, "maxBounces": B, "accumMode": 0,
           "crops": crops, "budgetSeconds": budget_s, "threads": threads, "writeAccum": bool(frame_hash)}
    with tempfile.TemporaryDirectory() as td:
        jp = os.path.join(td, "job.json")
        with open(jp, "w") as f:
            json.dump(job, f)
        out = subprocess.run([node, os.path.join(ROOT, "oracle", "sail_soft.js"), jp, os.path.join(td, "o")],
                             capture_output=True, text=True, timeout=(600 if full else budget_s * 10 + 60), check=True).stdout
        sha = None
        if frame_hash:
            import hashlib
            with open(os.path.join(td, "o.accum.f32"), "rb") as f:
                sha = hashlib.sha256(f.read()).hexdigest()
    r = json.loads(out.strip().splitlines()[-1])
    return {"value": r["segments"] / r["seconds"] / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "implementation": f"oracle/sail_soft.js on Node {r['node']}, "
                              + ("single thread" if threads == 1 else f"{threads} worker_threads"),
            "sample": (f"the whole {W}x{H} frame" if full else f"{r['crops']} centre-out {c}x{c} crops of the frame")
                      + f", {spp} spp x {B} bounces = {r['segments']} segments (exact count) in {r['seconds']:.2f} s",
            **({"frame_sha256": sha} if sha else {})}


def cpu_baseline_c1_full():
    """BASELINE.md's CPU plan: configs[0] (C1 = the README Cornell box at 256x256, 4 bounces, 64 spp,
    16,777,216 segments) rendered in full by the single-threaded JS/Node software shader (~30 s)."""
    sc = load_scene("C1")
    W = H = 256
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    r = cpu_baseline_js(sc, capi.plugin_masks(sc["plugins"]), mvp, W, H, 4, spp=64, full=True, frame_hash=True)
    if r:
        r["config"] = "C1: README Cornell box, 256x256, 4 bounces, 64 spp (BASELINE.json configs[0]), in full"
        # the frame it rendered against the committed hash of the same frame (tests/golden/c1_full_256.json), which
        # the GPU suite checks the HIP path against (tests/test_c1_full.py)
        with open(os.path.join(ROOT, "tests", "golden", "c1_full_256.json")) as f:
            r["frame_matches_fixture"] = r.get("frame_sha256") == json.load(f)["sha256_accum_f32le"]
    return r


def cpu_baseline(sc, masks, mvp, W, H, B, budget_s=10.0):
    """The CPU oracle (single-threaded C++ restatement of the shader) timed on a bounded sample of the same
    frame: 32x32 crops spiralling out from the centre, 4 spp each, until ~budget_s of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle  # test infrastructure: the CPU reference, used here only as the timed baseline
    spp, c = 8, 32
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)
    acc = np.zeros((H, W, 4), np.float32)
    cx, cy = (W - c) // 2, (H - c) // 2
    offsets = sorted(((dx, dy) for dx in range(-9, 10) for dy in range(-9, 10)), key=lambda d: d[0] ** 2 + d[1] ** 2)
    oracle.reset_counters()
    t0 = time.perf_counter()
    crops = 0
    for dx, dy in offsets:
        x0, y0 = cx + dx * c, cy + dy * c
        if x0 < 0 or y0 < 0 or x0 + c > W or y0 + c > H:
            continue
        oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, crop=(x0, y0, c, c), accum=acc)
        crops += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    segs, _ = oracle.counters()
    return {"value": segs / dt / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": f"oracle/sail_oracle.cpp single thread: {crops} centre-out {c}x{c} crops of the frame, {spp} spp x "
                      f"{B} bounces = {segs} segments (exact count) in {dt:.2f} s"}


def ops_per_segment(sc, masks, mvp, W, H, B):
    """Algorithmic f32 ops per segment from the op-counting oracle build (SURVEY §8(d) op model): (every op of the
    reference program, the live-op model without the last bounce's dead ops -- its throughput update, next ray,
    BSDF sample and material weight, which no output reads)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    inv, seeds = capi.schedule(mvp, W, H, 0, 2)
    oracle.reset_counters(count=True)
    acc = np.zeros((H, W, 4), np.float32)
    cw, ch = 64, 36
    oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, crop=((W - cw) // 2, (H - ch) // 2, cw, ch),
                  accum=acc, count=True)
    segs, ops = oracle.counters(count=True)
    return ops / max(segs, 1), oracle.ops_live() / max(segs, 1)


def profiled_traffic(workload, px, spp, bounces, kernel_id):
    """HBM bytes per trace launch from the committed rocprofv3 PMC summary (tools/pmc.sh + tools/pmc_summary.py ->
    profiles/r*_pmc_summary*.json) of the same workload, launch shape and kernel BUILD: the summary records the
    kernel_id ("name@build id": FNV-1a 64 of the run-time kernel's code object, or of the library image for a
    precompiled kernel) its profiled bench printed, and only an equal id matches. None when no summary profiled this
    very kernel (a rebuilt kernel is never matched to an older one's counters)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary*.json")), reverse=True):
        with open(path) as f:
            rec = json.load(f)
        L = rec.get("launch", {})
        if (rec.get("workload") == workload and L.get("pixels") == px and L.get("spp") == spp
                and L.get("bounces") == bounces and kernel_id and rec.get("kernel_id") == kernel_id):
            return rec["hbm"]["traffic_bytes"], os.path.relpath(path, ROOT), rec
    return None, None, None


def valu_issue(pmc, device):
    """Executed wave64 VALU instructions per SIMD-cycle of the profiled dispatch, from the committed PMC summary alone
    (the same one as `traffic`): SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x CUs x 4 SIMDs). GRBM_GUI_ACTIVE counts
    the busy cycles of each XCD over that dispatch, so numerator and denominator come from one run. Reported against
    the hardware ceiling (one wave64 f32 instruction per SIMD per 2 cycles, MI355X_MICROARCH.md) and, beside it, the
    plain-f32 rate tools/pk_probe.hip measured under load (0.42). f64 and transcendental instructions take 4-8 cycles,
    so this understates how busy the pipe is."""
    if not pmc or "SQ_INSTS_VALU" not in pmc.get("sq", {}) or "GRBM_GUI_ACTIVE" not in pmc.get("sq", {}):
        return None
    cus, _ = capi.device_info(device)
    sq = pmc["sq"]
    cycles = sq["GRBM_GUI_ACTIVE"] / 8.0
    per_cycle = sq["SQ_INSTS_VALU"] / (cycles * cus * 4)
    return {"per_simd_cycle": round(per_cycle, 4),
            "formula": "SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x CUs x 4)",
            "ceiling_hw_per_simd_cycle": VALU_ISSUE_HW, "frac_of_hw": round(per_cycle / VALU_ISSUE_HW, 4),
            "ceiling_probe_per_simd_cycle": VALU_ISSUE_PROBE, "frac_of_probe": round(per_cycle / VALU_ISSUE_PROBE, 4),
            "valu_per_segment_lane": round(pmc.get("derived", {}).get("valu_insts_per_segment_lane", 0.0), 1),
            "lane_utilisation": round(pmc.get("derived", {}).get("valu_lane_utilisation", 0.0), 3),
            "pmc_kernel": pmc.get("kernel")}


def validate_frame(ctx, sc, masks, mvp, W, H, B, spp, inv, seeds, part, ngpu):
    """After the timed steps: the reduced frame on rank 0 must be the whole frame. Every pixel counts each sample
    exactly once (a reduce that drops or double-counts a rank's tiles or samples fails this), and small crops in
    tiles of different ranks equal the CPU oracle's render of the same samples (the checker, run outside the timed
    region): bit for bit for a tile split, to summation order for a sample split. Returns a report; raises
    SystemExit if the frame is wrong, so no number is printed for it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle  # test infrastructure: the CPU checker of the frame the GPUs produced
    acc = ctx.read_accum()
    counts = acc[..., 3]
    bad_counts = int(np.count_nonzero(counts != np.float32(spp)))
    tx, ty = (W + 63) // 64, (H + 63) // 64
    ntiles = tx * ty
    # one crop in a tile of rank 0, of rank N-1 and in the last tile (a ragged one when W or H is not a multiple of 64)
    tiles = sorted({0, min(ngpu - 1, ntiles - 1), ntiles - 1})
    c = 4 if W * H * spp * B <= 2e10 else 2  # C4 / C5: smaller crops keep the oracle under a few seconds
    crops, worst = [], 0.0
    for t in tiles:
        x0 = (t % tx) * 64 + min(30, (W - (t % tx) * 64) // 2)
        y0 = (t // tx) * 64 + min(30, (H - (t // tx) * 64) // 2)
        x0, y0 = min(x0, W - c), min(y0, H - c)
        want = oracle.render(sc, masks, W, H, inv, seeds, sc["eye"], B, crop=(x0, y0, c, c))[y0:y0 + c, x0:x0 + c]
        got = acc[y0:y0 + c, x0:x0 + c]
        if part == capi.PART_TILES or ngpu == 1:
            ok = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        else:
            ok = bool(np.allclose(got, want, rtol=1e-4, atol=1e-6))
        worst = max(worst, float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1e-6))))
        crops.append({"tile": t, "rank": t % ngpu if part == capi.PART_TILES else "all", "x0": x0, "y0": y0,
                      "size": c, "match": ok})
    rep = {"pixels_with_wrong_count": bad_counts, "expected_count": spp, "oracle_crops": crops,
           "rule": "bit-exact" if (part == capi.PART_TILES or ngpu == 1) else "summation order (rtol 1e-4)",
           "max_rel_diff": worst}
    if bad_counts or not all(cr["match"] for cr in crops):
        print(json.dumps({"error": "reduced frame failed validation", "validation": rep}), file=sys.stderr, flush=True)
        raise SystemExit(3)
    return rep


class _StdoutToStderr:
    """Points file descriptor 1 at stderr (C-level prints included) between __enter__ and __exit__."""

    def __init__(self):
        self.saved = None

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        if self.saved is not None:
            sys.stdout.flush()
            os.dup2(self.saved, 1)
            os.close(self.saved)
            self.saved = None
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--launch-spp", type=int, default=0,
                    help="samples per kernel launch (default 0: the library's choice by kernel form, sail_set_launch_samples)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c1-full", action="store_true", help="skip the ~30 s full C1 render of the CPU baseline")
    ap.add_argument("--force-rccl", action="store_true",
                    help="one process: the multi-device context's RCCL reduce even at --gpus 1 (SAIL_DEBUG_FORCE_RCCL)")
    ap.add_argument("--wavefront", action="store_true",
                    help="study: the pre-cull path by the wavefront split instead of the megakernel (SAIL_DEBUG_WAVEFRONT)")
    ap.add_argument("--no-validate", action="store_true",
                    help="skip the check of the reduced frame after the timed steps (counts + oracle crops)")
    ap.add_argument("--force-comm", action="store_true",
                    help="exercise the torch.distributed + RCCL reduce path even with one rank")
    ap.add_argument("--debug", action="append", default=[], metavar="OPTION=VALUE",
                    help="study: a sail_set_debug switch (include/sail_hip.h), e.g. 9=1 for the path-pool kernels")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus < 1 or (world > 1 and args.gpus != world):
        sys.exit(f"bench.py: --gpus {args.gpus} does not match WORLD_SIZE {world} (one process per GPU under "
                 "torch.distributed.run, or --gpus N in one process)")
    # one process, N GPUs: the library's multi-device context splits the frame (no torch.distributed);
    # --force-rccl takes that path (ncclCommInitAll + the grouped reduce) at one GPU too
    multi = world == 1 and (args.gpus > 1 or args.force_rccl)
    if multi and capi.device_count() < args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but only {capi.device_count()} HIP devices are visible")
    # RCCL prints its version banner on stdout when a communicator is created; the contract is ONE JSON line
    # on stdout, so descriptor 1 points at stderr until the warm-up (communicator creation included) is done
    quiet = _StdoutToStderr()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    use_comm = world > 1 or args.force_comm
    if use_comm:
        import torch
        import torch.distributed as tdist
        quiet.__enter__()
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist

    cfg = CONFIGS[args.config]
    W, H, B = cfg["width"], cfg["height"], cfg["bounces"]
    spp = args.spp if args.spp else cfg["spp"]
    sc = load_scene(cfg["scene"])
    masks = capi.plugin_masks(sc["plugins"])
    # makePerspective(55, W/H, 1, 100) (camera.js:16) with the scene's frozen camera
    mvp = capi.camera(sc["eye"], sc["center"], [0, 1, 0], 55.0, W / H, 1.0, 100.0)
    inv, seeds = capi.schedule(mvp, W, H, 0, spp)

    ctx = capi.Context(W, H, devices=list(range(args.gpus))) if multi else capi.Context(W, H, device=local_rank)
    if multi and args.force_rccl:
        ctx.set_debug(capi.DEBUG_FORCE_RCCL, 1)
    if args.wavefront:
        ctx.set_debug(capi.DEBUG_WAVEFRONT, 1)
    debug = {int(k): int(v) for k, v in (d.split("=") for d in args.debug)}
    for opt, val in debug.items():
        ctx.set_debug(opt, val)
    ctx.set_scene_dict(sc)
    if args.launch_spp:
        ctx.set_launch_samples(args.launch_spp)
    # the scene's run-time kernel (built in the background at set_scene; from the cache shipped beside the library for
    # the frozen scenes) before the warm-up, so every timed launch runs it
    ctx.kernel_ready(-1)
    part = capi.PART_SAMPLES if cfg.get("partition") == "samples" else capi.PART_TILES
    flt = sc.get("filter") if cfg.get("filter") else None
    fweights = np.array(flt["weights64"], dtype=np.float32) if flt else None
    if multi:
        ctx.set_partition(0, 1, part)
    if use_comm:
        ctx.set_partition(rank, world, part)
        uid = [capi.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0], world, rank)

    def step():
        ctx.reset()
        ctx.render_schedule(inv, seeds, sc["eye"], B)
        if use_comm or multi:
            ctx.reduce(0)
        if flt and rank == 0:  # reconstruction filter of the reduced frame (window.glsl, gaussian r = 2)
            ctx.filter(capi.FILTER_WINDOW, fweights, flt["radius"][0], flt["radius"][1], 2.2)

    def barrier_sync():
        ctx.sync()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier_sync()
    quiet.__exit__()
    kernel_ms = 0.0
    launches = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        ctx.sync()
        st = ctx.stats()
        kernel_ms += st.kernel_ms
        launches += st.launches
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_segments = W * H * spp * B * args.steps  # nominal; closed scene: every path runs all bounces
    value = total_segments / elapsed / 1e6
    ngpu = args.gpus if multi else world
    validation = None
    if rank == 0 and not args.no_validate:  # after the timed region: the frame the steps produced is checked
        validation = validate_frame(ctx, sc, masks, mvp, W, H, B, spp, inv, seeds, part, ngpu)
    if rank == 0:
        avg_launch_s = (kernel_ms / max(launches, 1)) / 1e3
        # this rank's pixels per launch (rank 0 at N = 1: the full frame)
        tiles_px = W * H if (ngpu == 1 or part == capi.PART_SAMPLES) else None
        if tiles_px is None:
            tx, ty = (W + 63) // 64, (H + 63) // 64
            tiles_px = 0
            for t in range(0, tx * ty, ngpu):
                tiles_px += min(64, W - (t % tx) * 64) * min(64, H - (t // tx) * 64)
        # samples per launch: the library's choice by kernel form unless --launch-spp fixed it (each step renders spp
        # samples in launches of at most that many; stats count every device's launches)
        per_dev = launches / (args.gpus if multi else 1) / args.steps
        launch_spp = args.launch_spp or int(round(spp / per_dev))
        segs_per_launch = tiles_px * launch_spp * B
        ops_seg, ops_live = ops_per_segment(sc, masks, mvp, W, H, B)
        achieved_tflops = ops_seg * segs_per_launch / avg_launch_s / 1e12
        achieved_live = ops_live * segs_per_launch / avg_launch_s / 1e12
        hbm_gbs = (tiles_px * 32) / avg_launch_s / 1e9   # float4 accumulator read + write per pixel per launch
        kinfo = ctx.kernel_info()
        kernel_id = f"{kinfo['name']}@{kinfo['build_id']}"
        traffic, traffic_src, pmc = profiled_traffic(cfg["workload"], tiles_px, launch_spp, B, kernel_id)
        rec = {
            "metric": "Msamples/s (paths x bounces) at 1920x1080 Cornell box" if args.config == "C2"
                      else f"Msamples/s (paths x bounces), {cfg['workload']}",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": ngpu,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: frozen {cfg['desc']} scene rows (SURVEY §8(d), JS API == reference serializer), "
                    "deterministic sample schedule",
            "config": {"workload": cfg["workload"] + ("_wavefront_split" if args.wavefront else ""), "width": W, "height": H, "bounces": B, "spp": spp,
                       "launch_spp": launch_spp, "partition": f"tiles64x{ngpu}",
                       "processes": "one per GPU" if world > 1 else ("one (multi-device context)" if multi else "one"), "segments_per_step": W * H * spp * B,
                       **({"debug": debug} if debug else {})},
            "roofline": {
                # headline: the live-op model (ops some output reads: the last bounce's dead throughput update, next
                # ray, BSDF sample and material weight left out), so skipped dead work is never credited
                "bound": "valu", "achieved": round(achieved_live, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved_live / FP32_PEAK_TFLOPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "ops_per_segment_live": round(ops_live, 2),
                "formula": "ops_per_segment_live x pixels x launch_spp x bounces / avg_launch_s / 157.3e12",
                # the op model counts every add/mul/min/max/divide/transcendental as one op: its ceiling is one op
                # per lane per cycle (the FP32 peak above counts an FMA as two), so this is the pipe's fraction
                "frac_one_op_per_lane": round(achieved_live / (FP32_PEAK_TFLOPS / 2), 4),
                # the full op model: every op of the reference program, dead last-bounce ops included
                "ops_per_segment_full": round(ops_seg, 2), "achieved_full": round(achieved_tflops, 3),
                "frac_full": round(achieved_tflops / FP32_PEAK_TFLOPS, 4),
                "kernel": ctx.kernel_name(),
                "kernel_id": kernel_id,
                "jit": {"state": ["none", "pending", "ready", "failed"][kinfo["jit_state"]],
                        "code_object_from": ["hipRTC in this process", "user disk cache", "cache shipped with the library"][kinfo["jit_from_cache"]],
                        "compile_ms": round(kinfo["jit_compile_ms"], 1), **({"error": kinfo["jit_error"]} if kinfo["jit_error"] else {})},
                "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                # one launch = the HIP events around the trace kernel and, with sample groups (a "_grouped" kernel),
                # the sail_accum_kernel that adds the staged samples in order after it
                "launch_span": "trace kernel + sail_accum_kernel" if ctx.kernel_name().endswith("_grouped") else "trace kernel",
                "hbm": {"achieved": round(hbm_gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(hbm_gbs / HBM_PEAK_GBS, 6), "bytes_per_launch": tiles_px * 32},
                "valu_issue": valu_issue(pmc, local_rank),
            },
        }
        rec["validation"] = validation
        if flt:
            fms = ctx.filter_ms()
            fbytes = W * H * (16 + 16)  # mean-image read once from HBM (taps hit L2) + float4 write
            rec["filter"] = {"kind": flt["name"], "kernel": "sail_filter_kernel", "avg_ms": round(fms, 4),
                             "bound": "hbm", "bytes_per_pass": fbytes, "achieved": round(fbytes / (fms * 1e-3) / 1e9, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(fbytes / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
            rec["config"]["partition"] = f"{cfg.get('partition', 'tiles')}x{ngpu}"
        if not args.no_cpu_baseline and ngpu == 1:
            # the north star's JS/Node software shader; the C++ restatement is timed beside it for reference
            cpp = cpu_baseline(sc, masks, mvp, W, H, B, budget_s=5.0)
            js = cpu_baseline_js(sc, masks, mvp, W, H, B)
            nthr = max(1, min(16, os.cpu_count() or 1))  # the box's CPU share for one GPU is 16 cores
            jsmt = cpu_baseline_js(sc, masks, mvp, W, H, B, budget_s=6.0, threads=nthr) if (js and nthr > 1) else None
            rec["cpu_baseline"] = dict(js, cpp_port=cpp, worker_threads=jsmt) if js else cpp
            if js and not args.no_c1_full:
                rec["cpu_baseline"]["c1_full"] = cpu_baseline_c1_full()
        print(json.dumps(rec), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
