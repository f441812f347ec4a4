#!/usr/bin/env python3
"""Static ISA attribution report of the trace kernels (tools/isa.sh output /tmp/isa/trace_g.s): per kernel, the
instruction count by opcode class, by source function (the enclosing D / SM_D / __global__ definition of each
line-table entry in sail_trace.hip / sail_math.h) and the register-spill (scratch) instructions by function.
Static counts: code size per function and class, not execution frequency (no PC sampling on this pool).
Usage: python tools/isa_report.py > profiles/r02_isa_attribution.txt"""
import collections
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = {"sail_trace.hip": os.path.join(ROOT, "sail_amd", "csrc", "sail_trace.hip"),
       "sail_math.h": os.path.join(ROOT, "sail_amd", "csrc", "sail_math.h")}
KERNELS = ["sail_trace_kernel_cornell", "sail_trace_kernel_room", "sail_trace_kernel", "sail_trace_kernel_cull"]
CLASSES = [("scratch (spill)", r"^scratch_"), ("LDS", r"^ds_"), ("vector memory", r"^(global|buffer|flat)_"),
           ("scalar memory", r"^s_(load|buffer_load)"), ("f64", r"^v_\w+_f64"), ("transcendental", r"^v_(rcp|rsq|sqrt|sin|cos|exp|log)_"),
           ("f32 fma", r"^v_(fma|fmac|fmaak|fmamk|mad|mac)\w*_f32"), ("f32 mul", r"^v_mul_f32"), ("f32 add/sub", r"^v_(add|sub|subrev)_f32"),
           ("IEEE divide fallback", r"^v_div_"), ("min/max/med3", r"^v_(min|max|med3)\w*_f32"), ("compare", r"^v_cmp"),
           ("select", r"^v_cndmask"), ("move", r"^v_mov"), ("lane ops (readlane/writelane/bpermute)", r"^v_(readlane|writelane|readfirstlane)|^ds_bpermute"),
           ("int / bit", r"^v_(add|sub|and|or|xor|lshl|lshr|ashr|bfe|bfi|mbcnt|bcnt|ffb|cvt_u32|cvt_i32|mul_lo|mul_hi|alignbit|perm|not|min_u|max_u|min_i|max_i|lshl_add|lshl_or|add3)"),
           ("conversion", r"^v_cvt"), ("other VALU", r"^v_"), ("branch / exec", r"^s_(cbranch|branch|and_saveexec|andn2_saveexec|or_saveexec|xor_b64|or_b64 exec)"),
           ("other SALU", r"^s_")]


def functions(path):
    """line -> enclosing function name"""
    names, cur = {}, "?"
    for i, l in enumerate(open(path).read().split("\n"), 1):
        m = re.match(r"^(?:template <[^>]*>\s*)?(?:D|SM_D|__device__ __forceinline__|extern \"C\" __global__ void __launch_bounds__\([^)]*\))\s+[\w:<>*&, ]*?\b(operator\S+?|\w+)\s*\(", l)
        if m:
            cur = m.group(1)
            cur = "V3 arithmetic" if cur.startswith("operator") or cur in ("v3", "v3s", "v2") else cur
        elif re.match(r"^#define SAIL_TRACE_KERNELS", l):
            cur = "SAIL_TRACE_KERNELS"
        names[i] = cur
    return names


def main():
    fmap = {k: functions(v) for k, v in SRC.items()}
    lines = open("/tmp/isa/trace_g.s").read().split("\n")
    blocks, name = collections.defaultdict(list), None
    for l in lines:
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", l)
        if m:
            name = m.group(1)
            continue
        if name:
            blocks[name].append(l)
    print(__doc__.split("\n")[0])
    print("code object: gfx950, hipcc -O3 -ffp-contract=off -fno-slp-vectorize (sail_amd/build.sh flags) + -gline-tables-only\n")
    for k in KERNELS:
        cur, byfn, bycls, spill, total = "?", collections.Counter(), collections.Counter(), collections.Counter(), 0
        fncls = collections.defaultdict(collections.Counter)
        for l in blocks[k]:
            m = re.match(r"; (\S+):(\d+)", l)
            if m:
                f = m.group(1).split("/")[-1]
                cur = fmap[f].get(int(m.group(2)), "?") if f in fmap else f
                continue
            t = l.strip()
            if not t or t.startswith(";") or t.endswith(":"):
                continue
            op = t.split()[0]
            if op == "s_nop":
                continue
            total += 1
            cls = next(c for c, p in CLASSES if re.search(p, op)) if any(re.search(p, op) for c, p in CLASSES) else "other"
            bycls[cls] += 1
            byfn[cur] += 1
            fncls[cur][cls] += 1
            if cls == "scratch (spill)":
                spill[cur] += 1
        print(f"== {k}: {total} instructions (s_nop excluded)")
        print("   by class: " + ", ".join(f"{c} {n}" for c, n in bycls.most_common()))
        print("   by source function (top 25; class split of the largest 3 classes):")
        for fn, n in byfn.most_common(25):
            top = ", ".join(f"{c} {m}" for c, m in fncls[fn].most_common(3))
            print(f"     {n:6d}  {fn:28s} {top}")
        print("   spill instructions by function: " + (", ".join(f"{fn} {n}" for fn, n in spill.most_common(12)) or "none"))
        print()


if __name__ == "__main__":
    main()
