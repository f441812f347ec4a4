"""Helpers for the generated-program literal pins (tests/test_reference_pins.py, tools/make_literal_map.py): the body
of a named function in a C++ / HIP source, and whether a literal of the reference's GLSL is used there -- as the same
f32 constant, or (texture column literals of the *_attr / parse* readers) as the same column of a decoded row."""
from __future__ import annotations

import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = ("C1", "C3", "C4", "ALL")
KERNEL_DEFAULT = "sail_amd/csrc/sail_trace.hip"
ORACLE_DEFAULT = "oracle/sail_oracle.cpp"
# where an unqualified name is looked up besides the default file (the math spec lives in headers)
EXTRA = {KERNEL_DEFAULT: ["sail_amd/csrc/sail_math.h"], ORACLE_DEFAULT: ["oracle/ref_math.h"]}

# functions of the generated program that no path of the trace runs (SURVEY §8(a) "Not on the hot path"):
# never called, or only reachable through Beckmann (never selected), transmission BxDFs nobody builds, noise
DEAD_FUNCTIONS = {
    "noise", "fbm", "turbulence", "Grad", "fade", "lerp", "noiseWeight", "beckmann_d", "beckmann_pdf",
    "beckmann_sample_wh", "lambertian_t_f", "lambertian_t_pdf", "lambertian_t_sample_f", "specular_t_f",
    "specular_t_pdf", "specular_t_sample_f", "cosDPhi", "tanTheta", "random", "cosineSampleHemisphere2",
    "uniformSampleDisk", "uniformSampleCone", "uniformSampleTriangle", "ortho", "modMatrix", "readVec2",
}
# literals the build replaces on purpose
GENERALISED = {
    # fstrace.glsl main: the previous frame is read at gl_FragCoord.xy / 512.0 (the fixed 512 x 512 canvas,
    # webgl.js:24); the build renders W x H and each pixel owns its accumulator, so the kernel has no such read
    ("main", "512.0"),
}

# literals the build reaches without writing them: the value is the same, by an exact rewrite
FOLDED = {
    ("intersectObjects", "1.0"): "faceObj's (reverseNormal ? -1.0 : 1.0) * normal . dir is written rev ? -nd : nd "
                                 "(hitRecord): negating the products is exact, so the sign is applied to the dot product",
    ("microfacet_d", "0.0"): "the distribution dispatch's fallback return 0.0 for a type other than Trowbridge-Reitz: "
                             "no material selects one (Beckmann is never built), so the build calls trD directly",
    ("microfacet_pdf", "0.0"): "same fallback of the pdf dispatch (trPdf is called directly)",
    ("microfacet_r_f", "0.001"): "return BLACK * 0.001: an exact zero vector, returned as v3s(0.0f)",
    ("microfacet_r_pdf", "0.001"): "its early return 0.001: microfacet_r_pdf is never called on the trace path "
                                   "(microfacet_r_sample_f computes its pdf inline, bsdf.glsl:193), so it has no counterpart",
    ("microfacet_r_sample_f", "0.001"): "return BLACK * 0.001: an exact zero vector, returned as v3s(0.0f)",
    ("microfacet_t_f", "0.001"): "return BLACK * 0.001: an exact zero vector, returned as v3s(0.0f)",
}

_cache: dict = {}


def source(path: str) -> str:
    if path not in _cache:
        with open(os.path.join(ROOT, path)) as f:
            _cache[path] = f.read()
    return _cache[path]


def _match_close(text: str, i: int, open_c: str, close_c: str) -> int:
    depth = 0
    for j in range(i, len(text)):
        if text[j] == open_c:
            depth += 1
        elif text[j] == close_c:
            depth -= 1
            if depth == 0:
                return j
    return -1


def function_bodies(path: str, name: str) -> list:
    """the bodies of every definition of `name` in the file (and its companion headers): an identifier followed by
    a parameter list and then `{` (optionally after `const`), brace-matched"""
    out = []
    for p in [path] + EXTRA.get(path, []):
        text = source(p)
        for m in re.finditer(r"(?<![\w.>])%s\s*\(" % re.escape(name), text):
            close = _match_close(text, m.end() - 1, "(", ")")
            if close < 0:
                continue
            rest = text[close + 1:close + 40]
            mm = re.match(r"\s*(const\s*)?\{", rest)
            if not mm:
                continue
            start = close + 1 + mm.end() - 1
            end = _match_close(text, start, "{", "}")
            if end > start:
                out.append(text[start:end + 1])
    return out


def float_bits(text: str) -> set:
    """f32 bit patterns of the floating literals of C++ text (1.0, .5, 1e-5, 12.9898f, 1.)"""
    vals = set()
    for m in re.finditer(r"(?<![\w.])(\d+\.\d*|\.\d+|\d+)([eE][-+]?\d+)?f?(?![\w.])", text):
        lit = m.group(1) + (m.group(2) or "")
        if "." in lit or "e" in lit.lower():
            vals.add(np.float32(float(lit)).view(np.uint32).item())
    return vals


def is_column(glsl_fn: str) -> bool:
    """the texture-row readers: their literals are column indices (material.js / texture.js / light.js rows)"""
    return glsl_fn.endswith("_attr") or glsl_fn.startswith("parse")


def literal_in_function(path: str, func: str, literal: str, kind: str) -> bool:
    bodies = function_bodies(path, func)
    if not bodies:
        return False
    body = "\n".join(bodies)
    if kind == "value":
        return np.float32(float(literal)).view(np.uint32).item() in float_bits(body)
    col = int(float(literal))
    pats = [r"\bTP3?\(\s*c\s*,\s*\w+\s*,\s*%d\s*\)" % col,            # kernel: decoded texParams row, column col
            r"\bL\[\s*%d\s*\]" % col,                                  # kernel: a lights row, column col
            r"\bread(?:Float|Vec3|Int|Bool)\((?:\s*[\w.]+\s*,)?\s*%d\.0f" % col]  # readFloat(col.0f, ...) (host / oracle)
    return any(re.search(p, body) for p in pats)
