"""Shared helper of the study patches: exact string replacements in a copied source tree (each must match once)."""
import os
import sys


def patch(fname, pairs):
    p = os.path.join(sys.argv[1], fname)
    s = open(p).read()
    for old, new in pairs:
        if s.count(old) != 1:
            raise SystemExit(f"{fname}: expected one match of {old[:60]!r}, found {s.count(old)}")
        s = s.replace(old, new)
    open(p, "w").write(s)
