"""Parity pins taken from the reference itself (tests/golden/make_fixtures.js imports /root/reference/bin/sail.js in
the build container and records data only):

* the reference picker (src/core/pickup.js:46-66) on a grid of mouse positions: its selections and distances,
  checked against this build's picker (the oracle's restated intersectObjects on CPU, sail_pick on the GPU);
* each object's reference boundbox() (src/scene/geometry.js), checked to lie inside the padded bounds the trace
  kernels' pre-cull tests (sail_prim_bounds, host-only);
* the generated trace program's #defines and the numeric literals of each of its functions
  (src/shader/const/define.glsl:1-64 and the plugins), checked against the constants of the HIP kernel and of the
  oracle restatement.
"""
import json
import os
import re

import numpy as np
import pytest

import literal_pins as lp
import oracle
from sail_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_SOURCES = ["sail_amd/csrc/sail_trace.hip", "sail_amd/csrc/sail_math.h", "sail_amd/csrc/sail_device.h",
                  "sail_amd/csrc/sail_capi.cpp"]
ORACLE_SOURCES = ["oracle/sail_oracle.cpp", "oracle/ref_math.h"]


def _src(paths):
    return "\n".join(open(os.path.join(ROOT, p)).read() for p in paths)


# ---- reference picker ------------------------------------------------------------------------------------------
def _picker_cases(fixtures, name):
    """(rays, reference rows, reference distances, stable mask) of the recorded mouse grid"""
    pk = fixtures["pick"][name]
    eye = np.array(pk["eye"], dtype=np.float32)
    picks = pk["picks"]
    rays = np.array([list(eye) + p["dir"] for p in picks], dtype=np.float32)
    rows = np.array([p["row"] for p in picks])
    ts = np.array([p["t"] if p["t"] is not None else 1e5 for p in picks])
    stable = np.array([p["stable"] for p in picks])
    return rays, rows, ts, stable


def _check_picks(fixtures, name, idx, t):
    """The reference picker and this build's agree on every stable grid position.

    Where they legitimately differ, the reference is the odd one out, for reasons in its own code:
    * Object3D / Cornellbox.boundbox() returns false (geometry.js:51-53), so the reference never selects the
      Cornell box: where it picks nothing, this build's picker may return the Cornell box's row;
    * its Rectangle intersect() tests the wrong plane: positions where either side selects a
      Rectangle are skipped.
    Distances agree to the f32 of the shader vs the f64 of the picker (relative 1e-4; the picker's MINVALUE 1e-4
    vs the shader's EPSILON 1e-5 never decides one of these rays)."""
    sc = fixtures["scenes"][name]
    shapes = [b["shape"] for b in sc["boundbox"]]
    rays, rows, ts, stable = _picker_cases(fixtures, name)
    unpickable = {i for i, b in enumerate(sc["boundbox"]) if b["min"] is None}
    rect = {i for i, s in enumerate(shapes) if s == "Rectangle"}
    checked = 0
    for k in np.nonzero(stable)[0]:
        ref, got = int(rows[k]), int(idx[k])
        if ref in rect or got in rect:
            continue
        if ref < 0:
            assert got < 0 or got in unpickable, (name, k, ref, got)
        else:
            assert got == ref, (name, k, ref, got, shapes[ref], shapes[got] if got >= 0 else None)
            assert abs(float(t[k]) - ts[k]) <= 1e-4 * abs(ts[k]) + 1e-6, (name, k, float(t[k]), ts[k])
        checked += 1
    assert checked >= 0.9 * len(rows)
    return checked


@pytest.mark.parametrize("name", ["C1", "C3", "UI", "C4"])
def test_oracle_picker_matches_reference_picker(fixtures, name):
    """the oracle's restated intersectObjects (bit-exact with sail_pick on the GPU) vs the reference's own picker"""
    rays, rows, _, _ = _picker_cases(fixtures, name)
    sc = fixtures["scenes"][name]
    idx, t = oracle.pick(sc, capi.plugin_masks(sc["plugins"])[0], rays)
    _check_picks(fixtures, name, idx, t)
    assert (rows >= 0).sum() >= 10  # the grids do select objects


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C1", "C3", "UI", "C4"])
def test_sail_pick_matches_reference_picker(fixtures, name):
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    rays, _, _, _ = _picker_cases(fixtures, name)
    ctx = capi.Context(8, 8)
    ctx.set_scene_dict(fixtures["scenes"][name])
    idx, t = ctx.pick(rays)
    ctx.close()
    _check_picks(fixtures, name, idx, t)


# ---- reference boundbox() inside the pre-cull's padded bounds -------------------------------------------------
# the reference's boundbox() adds a slack of 0.05 on flat axes (Disk: y, geometry.js:410-415; Rectangle: each axis
# where min == max, :202-215); the padded bound must contain the flat shape itself there, not the slack
SLACK = 0.05


@pytest.mark.parametrize("name", ["C1", "C3", "C4", "UI", "ALL", "AREA", "AREA0", "N1", "N1S", "BILERP"])
def test_reference_boundbox_inside_padded_bounds(fixtures, name):
    sc = fixtures["scenes"][name]
    ours = capi.prim_bounds(sc["objects"], sc["n"], sc["tn"]).astype(np.float64)
    checked = 0
    for i, b in enumerate(sc["boundbox"]):
        if b["min"] is None:     # Object3D / Cornellbox: no reference box (the pre-cull still bounds it)
            assert np.all(ours[i, 0] <= ours[i, 1]), (name, i)
            continue
        lo, hi = np.array(b["min"], dtype=np.float64), np.array(b["max"], dtype=np.float64)
        if b["shape"] == "Hyperboloid":
            # the reference box takes rMax = max(|p1.xy|, |p2.xy|) (geometry.js:459-463), but its own ah / ch
            # (:465-486, from p2 and the point p1 + 2 (p2 - p1)) describe a surface that need not pass through p1,
            # so that box is not the surface's extent: the radius the surface reaches on [zMin, zMax] is checked
            # (the reference's own intersect() hits are checked below)
            row = np.array(sc["objects"][18 * i:18 * i + 18], dtype=np.float64)
            ah, ch, z0, z1 = row[10], row[11], min(row[6], row[9]), max(row[6], row[9])
            zs = [z0, z1] + ([0.0] if z0 < 0.0 < z1 else [])
            r = max(np.sqrt(max((1.0 + ch * z * z) / ah, 0.0)) for z in zs)
            lo[[0, 2]] = row[[1, 3]] - r; hi[[0, 2]] = row[[1, 3]] + r
        if b["shape"] == "Disk":
            lo[1] += SLACK; hi[1] -= SLACK
        if b["shape"] == "Rectangle":
            rows = np.array(sc["objects"][18 * i:18 * i + 7], dtype=np.float64)
            flat = rows[1:4] == rows[4:7]
            lo[flat] += SLACK; hi[flat] -= SLACK
        assert np.all(ours[i, 0] <= lo) and np.all(hi <= ours[i, 1]), (name, i, b["shape"], lo, hi, ours[i])
        checked += 1
    assert checked >= 1 or sc["n"] == 0


@pytest.mark.parametrize("shape", ["cube", "sphere", "cone", "cylinder", "disk", "hyperboloid", "paraboloid"])
def test_reference_intersect_hits_inside_padded_bounds(fixtures, shape):
    """every hit point o + t d of the reference's own f64 intersect() (geometry.js:110-591, the picker's) lies in the
    padded bound of that primitive"""
    rec = fixtures["intersect"][shape]
    ours = capi.prim_bounds(rec["row"], 1, 2)[0].astype(np.float64)
    hits = 0
    for ray in rec["rays"]:
        if ray["t"] >= 1e5:
            continue
        p = np.array(ray["o"]) + ray["t"] * np.array(ray["d"])
        assert np.all(ours[0] <= p) and np.all(p <= ours[1]), (shape, p, ours)
        hits += 1
    assert hits >= 8


def test_prim_bounds_rejects_bad_arguments():
    lib = capi.load()
    assert lib.sail_prim_bounds(None, 3, 1, None) < 0
    assert lib.sail_prim_bounds(None, -1, 1, None) < 0
    assert lib.sail_prim_bounds(None, 0, 1, None) == 0


# ---- the generated trace program's constants ------------------------------------------------------------------
def _float_literals(text):
    """f32 values of the floating literals of C++ / GLSL text (1.0, .5, 1e-5, 12.9898f, 0x1p-126f excluded)"""
    vals = set()
    for m in re.finditer(r"(?<![\w.])(\d+\.\d*|\.\d+|\d+)([eE][-+]?\d+)?f?(?![\w.])", text):
        lit = m.group(1) + (m.group(2) or "")
        if "." in lit or "e" in lit.lower():
            vals.add(np.float32(float(lit)).view(np.uint32).item())
    return vals


DEAD_FUNCTIONS = lp.DEAD_FUNCTIONS


@pytest.mark.parametrize("name", ["C1", "C3", "C4", "ALL"])
def test_program_defines_match_kernel_and_oracle(fixtures, name):
    d = fixtures["program_constants"][name]["defines"]
    kern, orc = _src(KERNEL_SOURCES), _src(ORACLE_SOURCES)
    f32 = lambda v: np.float32(float(v)).view(np.uint32).item()  # noqa: E731
    # distances and epsilons: the same f32 in the kernel and in the oracle
    for define, names in {"MAX_DISTANCE": ["kMaxDistance", "kInf"], "INF": ["kInf"], "EPSILON": ["kEps"],
                          "ONEMINUSEPSILON": ["kOneMinusEps"], "PI": ["kPI"], "INVPI": ["kInvPI"],
                          "PIOVER2": ["kPiOver2"], "PIOVER4": ["kPiOver4"]}.items():
        for src, label in ((kern, "kernel"), (orc, "oracle")):
            for cname in names:
                m = re.search(r"\b%s\s*=\s*([0-9.eE+-]+)f?" % cname, src)
                assert m, (label, cname)
                assert f32(m.group(1)) == f32(d[define]), (label, define, d[define], m.group(1))
    # shape / light / material / texture ids: the kernel's enum values (sail_device.h) and the oracle's
    ids = {k: int(d[k]) for k in ("CUBE", "SPHERE", "RECTANGLE", "CONE", "CYLINDER", "DISK", "HYPERBOLOID",
                                   "PARABOLOID", "CORNELLBOX", "AREA", "POINT", "SPOT", "MATTE", "MIRROR", "METAL",
                                   "GLASS", "UNIFORM_COLOR", "CHECKERBOARD", "CHECKERBOARD2", "BILERP", "MIXF",
                                   "SCALE", "UVF")}
    dev = _src(["sail_amd/csrc/sail_device.h"])
    for k, v in ids.items():
        cname = {"UNIFORM_COLOR": "SAIL_TEX_UNIFORM"}.get(k, None)
        cands = [cname] if cname else ["SAIL_" + k, "SAIL_TEX_" + k]
        found = [int(m.group(1)) for c in cands for m in re.finditer(r"\b%s\s*=\s*(\d+)" % c, dev)]
        assert found and all(f == v for f in found), (k, v, found)
    # the texture row read divisors (OBJECTS/LIGHTS/TEX_PARAMS_LENGTH, define.glsl:1-3): 17 / 17 / 15
    assert (float(d["OBJECTS_LENGTH"]), float(d["LIGHTS_LENGTH"]), float(d["TEX_PARAMS_LENGTH"])) == (17.0, 17.0, 15.0)
    assert re.search(r"\bL\s*=\s*17\.0f", _src(["sail_amd/csrc/sail_capi.cpp"]))
    # the colours the shapes use (GREEN / BLUE / GREY for Cornellbox and checkerboard)
    lits_k, lits_o = _float_literals(kern), _float_literals(orc)
    for col in ("GREEN", "BLUE", "GREY"):
        for v in re.findall(r"[0-9.]+", d[col]):
            assert f32(v) in lits_k and f32(v) in lits_o, (col, v)
    # the object-space frame (OBJECT_SPACE_N/S/T = (0,1,0), (0,0,-1), (1,0,0))
    assert (d["OBJECT_SPACE_N"], d["OBJECT_SPACE_S"], d["OBJECT_SPACE_T"]) == ("vec3(0,1,0)", "vec3(0,0,-1)", "vec3(1,0,0)")
    # the kernel folds the frame's exact zero products into FMAs (W2L / L2W, sail_trace.hip), documented per row;
    # the oracle keeps the reference's full dot products over the literal frame
    assert "D V3 W2L(V3 v) {  // (dot(v, (0,0,-1)), dot(v, (1,0,0)), dot(v, (0,1,0)))" in kern
    assert "D V3 L2W(V3 v) {  // (0,0,-1) v.x + (1,0,0) v.y + (0,1,0) v.z" in kern
    for name, vec in (("OSN", "0.0f), F(1.0f), F(0.0f"), ("OSS", "0.0f), F(0.0f), F(-1.0f"), ("OST", "1.0f), F(0.0f), F(0.0f")):
        assert "static const V3 %s = {F(%s)};" % (name, vec) in orc, name


def _literal_map():
    with open(os.path.join(ROOT, "tests", "golden", "literal_map.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", list(lp.SCENES))
def test_program_literals_mapped_to_their_functions(fixtures, name):
    """every floating literal of every live function of the generated program has an entry in the committed table
    tests/golden/literal_map.json (data: GLSL function -> literal -> the kernel function and the oracle function
    that use it), and each entry holds in today's sources: the same f32 constant inside that function's body, or,
    for the texture-row readers, the same column of the decoded row. Folded literals state the exact rewrite."""
    lits = fixtures["program_constants"][name]["literals"]
    table = _literal_map()
    live = {fn: v for fn, v in lits.items() if fn not in lp.DEAD_FUNCTIONS}
    assert len(live) > 20
    problems = []
    for fn, vals in sorted(live.items()):
        for v in vals:
            if (fn, v) in lp.GENERALISED:
                continue
            e = table.get(fn, {}).get(v)
            if e is None:
                problems.append((fn, v, "not in literal_map.json"))
                continue
            if e["kind"] == "folded":
                if (fn, v) not in lp.FOLDED:
                    problems.append((fn, v, "folded without a recorded reason"))
                continue
            for side in ("kernel", "oracle"):
                path, func = e[side].rsplit(":", 1)
                if not lp.literal_in_function(path, func, v, e["kind"]):
                    problems.append((fn, v, side, e[side]))
    assert not problems, problems


def test_literal_map_is_not_vacuous():
    """the table names real functions, and its float entries are specific: a changed constant breaks the pin"""
    table = _literal_map()
    funcs = {e[s] for ent in table.values() for e in ent.values() if e["kind"] != "folded" for s in ("kernel", "oracle")}
    for f in funcs:
        path, name = f.rsplit(":", 1)
        assert lp.function_bodies(path, name), f
    # the hash constants sit in the hash functions of both implementations, not anywhere in the sources
    for v in ("12.9898", "78.233", "151.7182", "43758.5453", "63.7264", "10.873", "623.6736"):
        e = table["random2"][v]
        assert e["kernel"].endswith(":hash1") or e["kernel"].endswith(":random2"), e
        assert e["oracle"].endswith(":hash1") or e["oracle"].endswith(":random2"), e
    assert not lp.literal_in_function("sail_amd/csrc/sail_trace.hip", "hash1", "12.9897", "value")
    assert table["equalZero"]["1e-3"]["kernel"].endswith(":equalZero")
    assert table["point_sample"]["0.1"]["kernel"].endswith(":lightPrep")
