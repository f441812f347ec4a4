#!/usr/bin/env python3
"""Turns the working tree's uncommitted changes to sail_amd/csrc/* into a tools/studies.json entry (exact string
replacements with enough context to be unique), so that a measured-and-rejected variant is kept as a study instead of
a build switch in the product. Usage: tools/diff_to_study.py NAME ROUND "doc"  (then `git checkout sail_amd/csrc`)"""
import difflib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pairs_for(path):
    old = subprocess.run(["git", "show", "HEAD:" + path], cwd=ROOT, capture_output=True, text=True, check=True).stdout
    new = open(os.path.join(ROOT, path)).read()
    a, b = old.splitlines(keepends=True), new.splitlines(keepends=True)
    out = []
    cur = old  # the text as the pairs applied so far leave it (tools/study.py applies them in order)
    for tag, i1, i2, j1, j2 in difflib.SequenceMatcher(None, a, b, autojunk=False).get_opcodes():
        if tag == "equal":
            continue
        ctx = 0
        while True:  # grow the context until the old text occurs once, here and in what the earlier pairs left
            lo, hi = max(0, i1 - ctx), min(len(a), i2 + ctx)
            o = "".join(a[lo:hi])
            if o and old.count(o) == 1 and cur.count(o) == 1:
                n = "".join(a[lo:i1]) + "".join(b[j1:j2]) + "".join(a[i2:hi])
                out.append([o, n])
                cur = cur.replace(o, n)
                break
            ctx += 1
    assert cur == new, "the pairs do not reproduce " + path
    return out


def main():
    name, rnd, doc = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    files = subprocess.run(["git", "diff", "--name-only", "--", "sail_amd/csrc"], cwd=ROOT, capture_output=True, text=True,
                           check=True).stdout.split()
    patches = [{"file": os.path.basename(f), "pairs": pairs_for(f)} for f in files]
    cat = os.path.join(ROOT, "tools", "studies.json")
    d = json.load(open(cat))
    d[name] = {"round": rnd, "doc": doc, "patches": patches}
    json.dump(d, open(cat, "w"), indent=1)
    print(name, [(p["file"], len(p["pairs"])) for p in patches])


if __name__ == "__main__":
    main()
