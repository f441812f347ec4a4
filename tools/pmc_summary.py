#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of tools/pmc.sh (gpurun_out/pmc/*) for the trace kernel into one JSON.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports
half of the bytes of a wide (16 B/lane) coalesced streaming read, which is this kernel's accumulator read,
so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.
Usage: tools/pmc_summary.py gpurun_out/pmc out.json [launch_pixels launch_spp bounces [workload]]
Counters are summed over the chip (all XCDs) per dispatch; each value here is the mean over dispatches.
"""
import collections
import csv
import json
import os
import sys


def load(pdir, name):
    """counter means over the trace-kernel dispatches of one pass, the kernels they were, and their mean duration
    (the counter CSV's own Start/End timestamps, ns): every summary states what it profiled and for how long"""
    path = os.path.join(pdir, name, "run_counter_collection.csv")
    agg = collections.defaultdict(list)
    disp = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if "sail_trace_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                disp[r["Dispatch_Id"]] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    kernels = sorted({k for k, _ in disp.values()})
    dur = sum(d for _, d in disp.values()) / max(len(disp), 1)
    return {k: sum(v) / len(v) for k, v in agg.items()}, {"kernels": kernels, "dispatches": len(disp), "mean_ns": dur}


def main():
    pdir, out = sys.argv[1], sys.argv[2]
    px = int(sys.argv[3]) if len(sys.argv) > 3 else 1920 * 1080
    spp = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    bounces = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    workload = sys.argv[6] if len(sys.argv) > 6 else "cornell_box_readme_C2"
    c = {}
    passes = {}
    for p in ("fetch", "write", "sq", "sq2"):
        if os.path.isdir(os.path.join(pdir, p)):
            vals, meta = load(pdir, p)
            c.update(vals)
            passes[p] = meta
    kernels = sorted({k for m in passes.values() for k in m["kernels"]})
    # the build identity of the profiled kernel, from the bench line each pass printed (roofline.kernel_id): bench.py
    # matches a summary to a kernel by it, so every pass must have profiled the same build
    ids = set()
    for p in passes:
        try:
            with open(os.path.join(pdir, p + ".log")) as f:
                for line in f:
                    if line.startswith("{") and '"roofline"' in line:
                        ids.add(json.loads(line)["roofline"].get("kernel_id"))
        except OSError:
            ids.add(None)
    kernel_id = ids.pop() if len(ids) == 1 else None
    fetch_b = c["FETCH_SIZE"] * 1024 * 2
    write_b = c["WRITE_SIZE"] * 1024
    alg = px * 32
    waves = c.get("SQ_WAVES", 0)
    segs = px * spp * bounces
    rec = {
        "kernel": kernels[0] if len(kernels) == 1 else kernels, "kernel_id": kernel_id, "workload": workload,
        "passes": passes, "launch": {"pixels": px, "spp": spp, "bounces": bounces, "nominal_segments": segs},
        "hbm": {"fetch_bytes_corrected": fetch_b, "write_bytes": write_b, "traffic_bytes": fetch_b + write_b,
                "algorithmic_bytes": alg, "traffic_over_algorithmic": (fetch_b + write_b) / alg,
                "raw_FETCH_SIZE_KiB": c["FETCH_SIZE"], "raw_WRITE_SIZE_KiB": c["WRITE_SIZE"]},
        "sq": {k: v for k, v in c.items() if k.startswith("SQ_") or k.startswith("GRBM")},
    }
    if waves and "SQ_INSTS_VALU" in c:
        rec["derived"] = {
            "valu_insts_per_wave": c["SQ_INSTS_VALU"] / waves,
            "valu_insts_per_segment_lane": c["SQ_INSTS_VALU"] * 64 / segs,
            "salu_insts_per_wave": c.get("SQ_INSTS_SALU", 0) / waves,
            # beyond the one float4 accumulator store per lane: scratch (register spill) stores
            "vmem_writes_per_wave": c.get("SQ_INSTS_VMEM_WR", 0) / waves,
            # per segment-lane as well: a grouped launch has more, shorter waves (fewer samples each)
            "vmem_writes_per_segment_lane": c.get("SQ_INSTS_VMEM_WR", 0) * 64 / segs,
            "vmem_reads_per_segment_lane": c.get("SQ_INSTS_VMEM_RD", 0) * 64 / segs,
        }
        sq = passes.get("sq")
        if sq and sq["mean_ns"] > 0 and "GRBM_GUI_ACTIVE" in c:
            # GRBM_GUI_ACTIVE counts GPU-busy cycles on each of the 8 XCDs: over the dispatch's own duration it is the
            # engine clock the kernel ran at; VALU wave-instructions per SIMD (1,024 of them) per such cycle
            clk = c["GRBM_GUI_ACTIVE"] / 8 / (sq["mean_ns"] * 1e-9)
            rec["derived"]["effective_clock_hz"] = clk
            rec["derived"]["valu_issue_per_simd_cycle"] = c["SQ_INSTS_VALU"] / (sq["mean_ns"] * 1e-9 * clk * 1024)
        if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
            # lanes doing work per VALU cycle; 1.0 = no divergence or masked lanes
            rec["derived"]["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
