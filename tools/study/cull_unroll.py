"""The pre-cull mask build's row loops unrolled by 4 by hand (the FUSED form): four rows' padded bounds are requested
by scalar loads together, so one wait covers four rows instead of one wait per row. Same operations per row, same
order of the mask bits: bit-identical."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("    for (int j = cnt - 1; j >= 32; j--) hi = shiftInMask(hi, padHitFMask(PRIM(c, base + j), q, B));\n"
     "    for (int j = (cnt < 32 ? cnt : 32) - 1; j >= 0; j--) lo = shiftInMask(lo, padHitFMask(PRIM(c, base + j), q, B));\n",
     """    int j = cnt - 1;
    for (; j >= 35; j -= 4) {
      const unsigned long long m0 = padHitFMask(PRIM(c, base + j), q, B), m1 = padHitFMask(PRIM(c, base + j - 1), q, B);
      const unsigned long long m2 = padHitFMask(PRIM(c, base + j - 2), q, B), m3 = padHitFMask(PRIM(c, base + j - 3), q, B);
      hi = shiftInMask(shiftInMask(shiftInMask(shiftInMask(hi, m0), m1), m2), m3);
    }
    for (; j >= 32; j--) hi = shiftInMask(hi, padHitFMask(PRIM(c, base + j), q, B));
    j = (cnt < 32 ? cnt : 32) - 1;
    for (; j >= 3; j -= 4) {
      const unsigned long long m0 = padHitFMask(PRIM(c, base + j), q, B), m1 = padHitFMask(PRIM(c, base + j - 1), q, B);
      const unsigned long long m2 = padHitFMask(PRIM(c, base + j - 2), q, B), m3 = padHitFMask(PRIM(c, base + j - 3), q, B);
      lo = shiftInMask(shiftInMask(shiftInMask(shiftInMask(lo, m0), m1), m2), m3);
    }
    for (; j >= 0; j--) lo = shiftInMask(lo, padHitFMask(PRIM(c, base + j), q, B));
"""),
])
