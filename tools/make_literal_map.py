#!/usr/bin/env python3
"""Builds tests/golden/literal_map.json: for every floating literal of every live function of the reference's
generated trace program (tests/golden/fixtures.json "program_constants", captured from the reference bundle), the
function of the HIP build and the function of the CPU oracle that use it.

The function-level correspondence (GLSL function -> candidate kernel / oracle functions) is written out below by
hand; this script resolves, for each literal, which candidate's body holds it and records that one. A literal that
is a texture column index (the *_attr / parse* readers) is matched as the column the build reads (an integer index
into a decoded row, or a readFloat column), not as a float constant. tests/test_reference_pins.py re-checks every
entry against the current sources.
Usage: python tools/make_literal_map.py  (rewrites tests/golden/literal_map.json)"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import literal_pins as lp  # noqa: E402

K, O = "kernel", "oracle"
# GLSL function -> ([kernel functions], [oracle functions]); "file:function" when the file is not the default
MAP = {
    "area_sample": (["lightPrep", "sampleGeometry"], ["light_sample", "sampleGeometry"]),
    "checkerboard": (["getSurfaceColor"], ["getSurfaceColor"]),
    "checkerboard2_attr": (["getSurfaceColor"], ["getSurfaceColor"]),
    "checkerboard_attr": (["getSurfaceColor"], ["getSurfaceColor"]),
    "computeDpDForCone": (["coneHit", "dpduRot"], ["intersectCone", "dpduRot", "finishLocal"]),
    "computeDpDForCornellbox": (["dpdBox"], ["computeDpDForBox"]),
    "computeDpDForCube": (["dpdBox"], ["computeDpDForBox"]),
    "computeDpDForCylinder": (["dpduRot"], ["dpduRot"]),
    "computeDpDForDisk": (["dpduRot", "diskHit"], ["dpduRot", "intersectDisk"]),
    "computeDpDForHyperboloid": (["dpduRot", "hypDpD"], ["dpduRot", "computeDpDForHyperboloid"]),
    "computeDpDForParaboloid": (["dpduRot", "paraDpD"], ["dpduRot", "computeDpDForParaboloid"]),
    "computeDpDForSphere": (["sphereHit", "dpduRot"], ["computeDpDForSphere", "dpduRot"]),
    "concentricSampleDisk": (["concentricSampleDisk"], ["concentricSampleDisk"]),
    "cosPhi": (["cosPhi"], ["cosPhi"]),
    "cosineSampleHemisphere": (["cosineSampleHemisphere"], ["cosineSampleHemisphere"]),
    "equalZero": (["equalZero"], ["equalZero"]),
    "falloff": (["lightPrep"], ["falloff"]),
    "frConductor": (["frConductor"], ["frConductor"]),
    "frDielectric": (["frDielectric"], ["frDielectric"]),
    "getCornellboxColor": (["cornellHit"], ["getCornellboxColor"]),
    "getCubeUV": (["cubeHit"], ["getCubeUV"]),
    "getSurfaceColor": (["getSurfaceColor"], ["getSurfaceColor"]),
    "glass": (["material"], ["glass"]),
    "glass_attr": (["material"], ["glass"]),
    "glass_f": (["material"], ["material", "glass"]),
    "intersectCone": (["coneT", "rootPick"], ["intersectCone"]),
    "intersectCornellbox": (["cornellT", "mkRay", "slab"], ["intersectCornellbox"]),
    "intersectCube": (["cubeT", "mkRay", "slab"], ["intersectCube"]),
    "intersectCylinder": (["cylinderT", "rootPick"], ["intersectCylinder"]),
    "intersectDisk": (["diskT", "diskHit"], ["intersectDisk"]),
    "intersectHyperboloid": (["hypT", "hypHit", "rootPick"], ["intersectHyperboloid"]),
    "intersectObjects": (["sweepRay", "hitRecord", "intersectObjects"], ["intersectObjects"]),
    "intersectParaboloid": (["paraT", "paraHit", "rootPick"], ["intersectParaboloid"]),
    "intersectRectangle": (["rectT", "rectHit"], ["intersectRectangle"]),
    "intersectSphere": (["sphereT", "sphereHit"], ["intersectSphere"]),
    "lambertian_r_pdf": (["material"], ["matte"]),
    "light_sample": (["lightPrep", "lightSample"], ["light_sample"]),
    "main": (["traceTileCompact", "accumulateSample", "storeAov", "sail_amd/csrc/sail_capi.cpp:cornerDirs"],
             ["oracle_render", "primaryDir", "cornerDirs"]),
    "matte_attr": (["material"], ["matte"]),
    "metal_attr": (["material"], ["metal"]),
    "microfacet_d": (["trD"], ["trD"]),
    "microfacet_pdf": (["trPdf", "trD"], ["trPdf", "trD"]),
    "microfacet_r_f": (["microR_f"], ["microfacet_r_f"]),
    "microfacet_r_pdf": (["microR_sample"], ["microfacet_r_sample_f"]),
    "microfacet_r_sample_f": (["microR_sample"], ["microfacet_r_sample_f"]),
    "microfacet_t_f": (["microT_f"], ["microfacet_t_f"]),
    "microfacet_t_pdf": (["microT_pdf"], ["microfacet_t_pdf"]),
    "microfacet_t_sample_f": (["microT_sample", "microT_pdf"], ["microfacet_t_sample_f", "microfacet_t_pdf"]),
    "mirror_attr": (["material"], ["mirror"]),
    "mix_attr": (["getSurfaceColor"], ["getSurfaceColor"]),
    "mixf": (["getSurfaceColor"], ["getSurfaceColor"]),
    "scale_attr": (["getSurfaceColor"], ["getSurfaceColor"]),
    "normalForCone": (["finishLocal", "sampleGeometry", "sgn"], ["normalForCone", "sgn"]),
    "normalForCornellbox": (["normalForCornellbox"], ["normalForCornellbox"]),
    "normalForCube": (["normalForCube"], ["normalForCube"]),
    "normalForCylinder": (["finishLocal", "sampleGeometry", "sgn"], ["normalForCylinder", "sgn"]),
    "normalForDisk": (["finishLocal", "sampleGeometry", "sgn"], ["normalForDisk", "sgn"]),
    "normalForHyperboloid": (["hypHit", "hypDpD", "sampleGeometry", "sgn"], ["normalForHyperboloid", "computeDpDForHyperboloid", "dpduRot", "sampleGeometry", "sgn"]),
    "normalForParaboloid": (["finishLocal", "sampleGeometry", "sgn"], ["normalForParaboloid", "sgn"]),
    "normalForRectangle": (["sail_amd/csrc/sail_capi.cpp:rectFrameHost", "rectFrame", "sgn"], ["normalForRectangle", "sgn"]),
    "normalForSphere": (["sphereHit", "sampleGeometry", "sgn"], ["normalForSphere", "sgn"]),
    "orenNayar_f": (["orenNayar_f"], ["orenNayar_f"]),
    "orenNayar_pdf": (["material"], ["matte"]),
    "parseArea": (["sail_amd/csrc/sail_capi.cpp:sail_set_scene", "lightPrep"], ["light_sample"]),
    "parseCone": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseConeCyl"]),
    "parseCornellbox": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseCornellbox"]),
    "parseCube": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseCube"]),
    "parseCylinder": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseConeCyl"]),
    "parseDisk": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseDisk"]),
    "parseHyperboloid": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseHyperboloid"]),
    "parseParaboloid": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseParaboloid"]),
    "parsePoint": (["lightPrep"], ["light_sample"]),
    "parseRectangle": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseRectangle"]),
    "parseSphere": (["sail_amd/csrc/sail_capi.cpp:decodePrims"], ["parseSphere"]),
    "parseSpot": (["lightPrep"], ["light_sample"]),
    "point_sample": (["lightPrep"], ["light_sample"]),
    "quadratic": (["quadratic"], ["quadratic"]),
    "random2": (["random2", "hash1"], ["random2", "hash1"]),
    "randomInt": (["random2", "hash1", "lightPrep"], ["randomInt", "hash1"]),
    "readVec3": (["sail_amd/csrc/sail_capi.cpp:readVec3", "TP3"], ["readVec3"]),
    "sampleDisk": (["sampleGeometry"], ["sampleDisk"]),
    "sampleGeometry": (["sampleGeometry"], ["sampleGeometry"]),
    "sampleRectangle": (["sampleGeometry"], ["sampleRectangle"]),
    "sin2Theta": (["sin2Theta"], ["sin2Theta"]),
    "sinPhi": (["sinPhi"], ["sinPhi"]),
    "specular_fr_pdf": (["material"], ["glass"]),
    "specular_fr_sample_f": (["material"], ["glass"]),
    "specular_r_pdf": (["material"], ["mirror", "material", "glass"]),
    "specular_r_sample_f": (["material"], ["mirror"]),
    "spot_sample": (["lightPrep"], ["light_sample"]),
    "testBoundbox": (["testBoundbox"], ["testBoundbox"]),
    "trace": (["shadeBounceT"], ["trace"]),
    "trowbridgeReitz_d": (["trD"], ["trD"]),
    "trowbridgeReitz_sample_wh": (["trSampleWh"], ["trSampleWh"]),
    "uniformSampleSphere": (["uniformSampleSphere"], ["uniformSampleSphere"]),
}


def main():
    with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
        pc = json.load(f)["program_constants"]
    lits = {}
    for name in lp.SCENES:
        for fn, vals in pc[name]["literals"].items():
            if fn not in lp.DEAD_FUNCTIONS:
                lits.setdefault(fn, set()).update(vals)
    out, unresolved = {}, []
    for fn in sorted(lits):
        vals = sorted(v for v in lits[fn] if (fn, v) not in lp.GENERALISED)
        if not vals:
            continue
        if fn not in MAP:
            unresolved.append((fn, "no mapping"))
            continue
        kc, oc = MAP[fn]
        entry = {}
        for v in vals:
            kind = "column" if lp.is_column(fn) else "value"
            if (fn, v) in lp.FOLDED:  # the build computes the same value without the literal (reason recorded)
                entry[v] = {"kind": "folded", "why": lp.FOLDED[(fn, v)]}
                continue
            hit = {}
            for side, cands, default in ((K, kc, lp.KERNEL_DEFAULT), (O, oc, lp.ORACLE_DEFAULT)):
                for cand in cands:
                    path, func = cand.split(":") if ":" in cand else (default, cand)
                    if lp.literal_in_function(path, func, v, kind):
                        hit[side] = f"{path}:{func}"
                        break
            if len(hit) != 2:
                unresolved.append((fn, v, hit))
            entry[v] = {"kind": kind, **hit}
        out[fn] = entry
    with open(os.path.join(ROOT, "tests", "golden", "literal_map.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    n = sum(len(e) for e in out.values())
    print(f"{n} literals in {len(out)} functions; unresolved: {unresolved}")


if __name__ == "__main__":
    main()
