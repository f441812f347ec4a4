#!/usr/bin/env python3
"""Where the trace kernel's instructions come from: the run-time kernel a default context builds for a frozen scene,
compiled with line tables (tools/isa.sh flags + the spec's #define prefix, which sail_jit.cpp prints under SAIL_JIT_DEFS),
checked instruction for instruction against the code object shipped in sail_amd/lib/jit (the benched build), then each
instruction attributed through its inline stack (llvm-symbolizer --inlining) to the part of the bounce it belongs to and
classed: f32 arithmetic, transcendental, f64, int / bit, compare, move / select / lane, other VALU; SALU; LDS; memory.
Static counts (instructions in the code), per part of the bounce -- the dynamic weights are the phase timers' shares
(tools/phase_profile.py) and the PMC instruction mix (tools/pmc_mix.sh).
Usage: python tools/isa_regions.py C1 [--kernel sail_trace_kernel_jit] [--json out.json]"""
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", "-Wno-unused-function",
         "--offload-arch=gfx950", "--cuda-device-only", "-gline-tables-only"]

# part of the bounce <- the first inlined function under traceTileCompact (then refined by the one under it)
PARTS = [("sweepRay", "sweep"), ("closestT", "light + shadow"), ("hitRecord", "hit record"), ("quadLocalHit", "hit record"),
         ("rectLocalHit", "hit record"), ("shadeLast", "last bounce (shadeLast)"), ("accumulateSample", "sample end"),
         ("stageSample", "sample end"), ("keyRank", "sort"), ("waveScanIncl", "sort"), ("atomicAdd", "sort"),
         ("__shfl", "sort")]
SHADE = [("random2", "hash RNG"), ("material", "BSDF sample"), ("lightSample", "light + shadow"),
         ("lightPrep", "light + shadow"), ("mkRay", "next ray"), ("localToWorld", "next ray")]


def defines(scene):
    """the #define prefix of the run-time kernel a default context derives for the frozen scene (NS = the full-frame
    shape), from sail_jit_prebuild with SAIL_JIT_DEFS set (the cache key is printed with it)"""
    code = ("import json, sys; sys.path.insert(0, %r); from sail_amd import capi; capi.set_jit_cache(''); "
            "sc = json.load(open(%r))[%r]; capi.jit_prebuild(sc, cache_dir=%r)"
            % (ROOT, os.path.join(ROOT, "sail_amd", "scenes", "frozen.json"), scene, tempfile.mkdtemp()))
    err = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SAIL_JIT_DEFS="1"), capture_output=True,
                         text=True, check=True).stderr
    blocks = re.findall(r"sail_jit (\S+) ([0-9a-f]{16})\n((?:#define [^\n]*\n)+)", err)
    arch, key, defs = blocks[0]  # the first spec prebuilt is the full-frame one
    return key, [("-D%s=%s" % tuple(d[len("#define "):].split(" ", 1))) for d in defs.strip().split("\n")]


def instructions(co, kernel):
    out = subprocess.run([LLVM + "/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True, text=True,
                         check=True).stdout
    ins, on = [], False
    for l in out.split("\n"):
        m = re.match(r"^([0-9a-f]+) <(\S+)>:", l)
        if m:
            on = m.group(2) == kernel
            continue
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s+([0-9A-F]+):", l)
        if on and m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return ins


def cls(op):
    if op.startswith("s_"):
        return "SALU / branch"
    if op.startswith("ds_"):
        return "LDS"
    if re.match(r"(global|scratch|buffer|flat)_", op):
        return "memory"
    if not op.startswith("v_"):
        return "other"
    if re.search(r"_f64", op):
        return "VALU f64"
    if re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_", op):
        return "VALU transcendental"
    if re.match(r"v_(add|sub|subrev|mul|fma|fmac|fmaak|fmamk|mac|madak|madmk|ldexp|floor|rndne|fract|trunc|ceil|div_\w+)_f32", op):
        return "VALU f32 arith"
    if re.match(r"v_(min|max|min3|max3|med3)_f32", op):
        return "VALU min/max"
    if re.match(r"v_cmp", op):
        return "VALU compare"
    if re.match(r"v_(mov|cndmask|readlane|readfirstlane|writelane|mov_b64)", op):
        return "VALU move / select / lane"
    if re.match(r"v_cvt", op):
        return "VALU convert"
    return "VALU int / bit"


def part(names, line):
    """names: inline stack outermost first, below traceTileCompact"""
    if not names:
        return "kernel body (sort, gather, sample loop)" if 1929 <= line <= 2100 else "kernel body (setup, sample end)"
    top = names[0]
    if top.startswith(("mkRay", "operator+", "operator-", "operator*", "operator/")):
        return "primary ray (sample start)"
    if top.startswith("normalize"):
        return "AOVs (first hit)"
    if top.startswith("operator()"):
        return "sort (scatter, radiance slots)"
    if top.startswith(("constRow", "tileWork", "__syncthreads", "sail_trace_kernel", "??")):
        return "kernel body (setup, sample end)"
    if top.startswith("shadeBounce"):
        for n in names[1:]:
            for k, v in SHADE:
                if n.startswith(k):
                    return v
        return "shading frame / radiance"
    for k, v in PARTS:
        if top.startswith(k):
            return v
    return "other: " + top


def main():
    scene = sys.argv[1]
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else None
    key, defs = defines(scene)
    if kernel is None:
        kernel = "sail_trace_kernel_cull_jit" if "-DSAIL_JIT_CULL=1" in defs else "sail_trace_kernel_jit"
    td = tempfile.mkdtemp()
    src = os.path.join(ROOT, "sail_amd", "csrc", "sail_trace.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *defs, "-c", src, "-o", td + "/t.o"], check=True)
    subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + td + "/t.o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + td + "/t.co"], check=True)
    ins = instructions(td + "/t.co", kernel)
    shipped = os.path.join(ROOT, "sail_amd", "lib", "jit", key + ".co")
    same = None
    if os.path.exists(shipped):
        open(td + "/s.co", "wb").write(open(shipped, "rb").read()[32:])  # SAILJIT1 header: magic + 3 words
        same = [(o, a) for _, o, a in instructions(td + "/s.co", kernel)] == [(o, a) for _, o, a in ins]
    out = subprocess.run([LLVM + "/llvm-symbolizer", "--obj=" + td + "/t.co", "--inlining", "--functions=short"],
                         input="\n".join(hex(a) for a, _, _ in ins), capture_output=True, text=True).stdout
    blocks = out.strip("\n").split("\n\n")
    table = collections.defaultdict(collections.Counter)
    for (_, op, _), b in zip(ins, blocks):
        fr = b.split("\n")
        names = [fr[i] for i in range(0, len(fr), 2)]
        locs = [fr[i + 1] for i in range(0, len(fr) - 1, 2)]
        k = next((i for i, n in enumerate(names) if n.startswith("traceTileCompact")), len(names))
        line = int(locs[k].rsplit(":", 2)[1]) if k < len(locs) else 0
        table[part(names[:k][::-1], line)][cls(op)] += 1
    classes = ["VALU f32 arith", "VALU min/max", "VALU transcendental", "VALU f64", "VALU int / bit", "VALU compare",
               "VALU move / select / lane", "VALU convert", "SALU / branch", "LDS", "memory"]
    rec = {"scene": scene, "kernel": kernel, "cache_key": key, "instructions": len(ins),
           "identical_to_shipped_code_object": same, "defines": defs,
           "parts": {p: dict(c) for p, c in sorted(table.items(), key=lambda kv: -sum(v for k, v in kv[1].items() if k.startswith("VALU")))}}
    hdr = ["part of the bounce", "VALU"] + [c.replace("VALU ", "") for c in classes]
    print(f"{scene}: {kernel} (spec {key}), {len(ins)} instructions; identical to the shipped code object: {same}")
    print("| " + " | ".join(hdr) + " |")
    print("|" + "---|" * len(hdr))
    for p, c in rec["parts"].items():
        valu = sum(v for k, v in c.items() if k.startswith("VALU"))
        print("| " + " | ".join([p, str(valu)] + [str(c.get(k, 0)) for k in classes]) + " |")
    if "--json" in sys.argv:
        json.dump(rec, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
