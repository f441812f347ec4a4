#!/usr/bin/env python3
"""Study patches: exact string replacements applied to a COPY of sail_amd/csrc (tools/study_build.sh), so a variant is
built and measured (tools/variant_bench.py) without a build switch in the product sources. Every study is an entry of
tools/studies.json: {"round": r, "doc": what it measures, "patches": [{"file", "pairs": [[old, new], ...], "count": n}]};
each `old` must occur exactly `count` times (default 1) in the copy, else the study no longer applies and this fails.
The results of the round-4 studies are in profiles/NOTES_r04.md and profiles/r04_*.jsonl; many no longer apply to the
current sources and are kept as the record of what was measured.
Usage: tools/study.py NAME DIR | tools/study.py --list"""
import json
import os
import sys

CATALOGUE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "studies.json")


def apply(name, d):
    studies = json.load(open(CATALOGUE))
    if name not in studies:
        raise SystemExit(f"study {name!r} is not in {CATALOGUE}")
    for ptc in studies[name]["patches"]:
        p = os.path.join(d, ptc["file"])
        s = open(p).read()
        want = ptc.get("count", 1)
        for old, new in ptc["pairs"]:
            if s.count(old) != want:
                raise SystemExit(f"study {name}: {ptc['file']}: expected {want} match(es) of {old[:60]!r}, found {s.count(old)}")
            s = s.replace(old, new)
        open(p, "w").write(s)


def main():
    if sys.argv[1:] == ["--list"]:
        for k, v in json.load(open(CATALOGUE)).items():
            print(f"{k:20s} r{v['round']}  {v['doc'][:100]}")
        return
    apply(sys.argv[1], sys.argv[2])


if __name__ == "__main__":
    main()
