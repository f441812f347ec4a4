#!/usr/bin/env python3
"""Summarise tools/pmc_mix.sh's two rocprofv3 passes (VALU instruction classes) for the trace kernel into one JSON:
the counters per dispatch (mean), the kernel they came from, and each class per segment-lane (64 x counter /
nominal segments of the launch) beside the algorithmic op count, so the executed/algorithmic inflation is attributed.
Usage: tools/pmc_mix_summary.py gpurun_out/pmc_mix out.json launch_pixels launch_spp bounces workload [ops_per_segment
       [pmc_summary.json]]
Refuses (exit 2, no output file) a mix whose passes profiled different builds or no identifiable build, and, when the
PMC summary the mix will be quoted beside is given (tools/pmc_summary.py's output for the same workload), a mix whose
kernel_id or launch shape differs from that summary's: a VALU mix is only ever quoted for the build it counted."""
import collections
import csv
import json
import os
import sys

CLASSES = ["SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32",
           "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
           "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT"]


def load(path):
    agg = collections.defaultdict(list)
    kernels, disp = set(), {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if "sail_trace_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                kernels.add(r["Kernel_Name"])
                disp[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return {k: sum(v) / len(v) for k, v in agg.items()}, kernels, sum(disp.values()) / max(len(disp), 1)


def main():
    pdir, out = sys.argv[1], sys.argv[2]
    px, spp, bounces, workload = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    ops = float(sys.argv[7]) if len(sys.argv) > 7 else None
    pair = sys.argv[8] if len(sys.argv) > 8 else None
    c, kernels, durs = {}, set(), {}
    for p in ("mix1", "mix2"):
        vals, ks, d = load(os.path.join(pdir, p, "run_counter_collection.csv"))
        c.update(vals)
        kernels |= ks
        durs[p] = d
    segs = px * spp * bounces
    per = {k.replace("SQ_INSTS_VALU_", "").lower(): c[k] * 64 / segs for k in CLASSES if k in c}
    total = c["SQ_INSTS_VALU"] * 64 / segs
    per["other (moves, selects, compares, min/max, bit ops, lane ops)"] = total - sum(per.values())
    ids = set()  # the profiled kernel's build identity, from each pass's bench line (roofline.kernel_id)
    for p in ("mix1", "mix2"):
        try:
            with open(os.path.join(pdir, p + ".log")) as f:
                ids |= {json.loads(x)["roofline"].get("kernel_id") for x in f if x.startswith("{") and '"roofline"' in x}
        except OSError:
            ids.add(None)
    kernel_id = ids.pop() if len(ids) == 1 else None
    if kernel_id is None:
        sys.exit("pmc_mix_summary: the passes did not profile one identifiable build (kernel_id missing or differing)")
    if pair:
        with open(pair) as f:
            summ = json.load(f)
        L = summ.get("launch", {})
        if summ.get("kernel_id") != kernel_id or summ.get("workload") != workload or \
                (L.get("pixels"), L.get("spp"), L.get("bounces")) != (px, spp, bounces):
            print(f"pmc_mix_summary: refused: the mix counted {kernel_id} ({workload}, {px} px x {spp} spp x {bounces}), "
                  f"{pair} is {summ.get('kernel_id')} ({summ.get('workload')}, {L.get('pixels')} px x {L.get('spp')} spp x "
                  f"{L.get('bounces')})", file=sys.stderr)
            sys.exit(2)
    rec = {"kernel": sorted(kernels)[0] if len(kernels) == 1 else sorted(kernels),
           "kernel_id": kernel_id, "workload": workload,
           "launch": {"pixels": px, "spp": spp, "bounces": bounces, "nominal_segments": segs},
           "source": "tools/pmc_mix.sh (rocprofv3 --pmc, two passes, kernel-trace only), mean per dispatch",
           "dispatch_mean_ns": durs, "counters": c,
           "valu_per_segment_lane": {"total": total, "by_class": per}}
    if pair:
        rec["paired_summary"] = os.path.basename(pair)
    if ops:
        rec["valu_per_segment_lane"]["algorithmic_ops_per_segment"] = ops
        rec["valu_per_segment_lane"]["inflation"] = total / ops
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec["valu_per_segment_lane"], indent=1))


if __name__ == "__main__":
    main()
