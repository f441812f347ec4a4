"""The pre-cull mask build at eight rows per step instead of four (scalar loads of eight rows' bounds together)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

STEP4 = """      const unsigned long long m0 = padHitFMask(PRIM(c, base + j), q, B), m1 = padHitFMask(PRIM(c, base + j - 1), q, B);
      const unsigned long long m2 = padHitFMask(PRIM(c, base + j - 2), q, B), m3 = padHitFMask(PRIM(c, base + j - 3), q, B);
"""
STEP8 = STEP4 + """      const unsigned long long m4 = padHitFMask(PRIM(c, base + j - 4), q, B), m5 = padHitFMask(PRIM(c, base + j - 5), q, B);
      const unsigned long long m6 = padHitFMask(PRIM(c, base + j - 6), q, B), m7 = padHitFMask(PRIM(c, base + j - 7), q, B);
"""
patch("sail_trace.hip", [
    ("    for (; j >= 35; j -= 4) {\n" + STEP4 + "      hi = shiftInMask(shiftInMask(shiftInMask(shiftInMask(hi, m0), m1), m2), m3);\n    }\n",
     "    for (; j >= 39; j -= 8) {\n" + STEP8 + "      hi = shiftInMask(shiftInMask(shiftInMask(shiftInMask(hi, m0), m1), m2), m3);\n"
     "      hi = shiftInMask(shiftInMask(shiftInMask(shiftInMask(hi, m4), m5), m6), m7);\n    }\n"
     "    for (; j >= 35; j -= 4) {\n" + STEP4 + "      hi = shiftInMask(shiftInMask(shiftInMask(shiftInMask(hi, m0), m1), m2), m3);\n    }\n"),
    ("    for (; j >= 3; j -= 4) {\n" + STEP4 + "      lo = shiftInMask(shiftInMask(shiftInMask(shiftInMask(lo, m0), m1), m2), m3);\n    }\n",
     "    for (; j >= 7; j -= 8) {\n" + STEP8 + "      lo = shiftInMask(shiftInMask(shiftInMask(shiftInMask(lo, m0), m1), m2), m3);\n"
     "      lo = shiftInMask(shiftInMask(shiftInMask(shiftInMask(lo, m4), m5), m6), m7);\n    }\n"
     "    for (; j >= 3; j -= 4) {\n" + STEP4 + "      lo = shiftInMask(shiftInMask(shiftInMask(shiftInMask(lo, m0), m1), m2), m3);\n    }\n"),
])
