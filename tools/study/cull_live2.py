"""segs_scalar's follow-up in every kernel: the pixel's frame coordinates (s, t and the triangle choice of the primary
ray) recomputed at each sample instead of held across the sample loop, and the accumulator's 64-bit pixel offset
recomputed where it is used: four fewer VGPRs live across the bounces. Same values (same operations)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("  const size_t pixG = (size_t)y * A.W + x;\n", ""),
    ("  float4 acc = (valid && home) ? A.accum[pixG] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);\n"
     "  const float s = ((float)x + 0.5f) / (float)A.W, t = ((float)y + 0.5f) / (float)A.H;\n"
     "  const bool tri0 = s + t <= 1.0f;\n",
     "  float4 acc = (valid && home) ? A.accum[(size_t)y * A.W + x] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);\n"),
    ("      ray = mkRay(eye, tri0 ?",
     "      const float s = ((float)x + 0.5f) / (float)A.W, t = ((float)y + 0.5f) / (float)A.H;\n"
     "      const bool tri0 = s + t <= 1.0f;\n"
     "      ray = mkRay(eye, tri0 ?"),
    ("  if (valid && home) A.accum[pixG] = acc;\n", "  if (valid && home) A.accum[(size_t)y * A.W + x] = acc;\n"),
])
