"""segs_scalar, plus the room form's running accumulator (the first sample group accumulating at home) kept in LDS
instead of four VGPRs across the sample loop: 4 KB more per 256-thread workgroup (21 KB; seven per CU at 7 waves).
Same additions in the same order."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch
from segs_scalar import PAIRS

patch("sail_trace.hip", PAIRS + [
    ("  float4 acc = (valid && home) ? A.accum[pixG] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);\n",
     "  __shared__ float4 sAcc[kHome ? NT : 1];\n"
     "  float4 acc = (valid && home) ? A.accum[pixG] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);\n"
     "  if constexpr (kHome) sAcc[li] = acc;\n"),
    ("      else accumulateSample(acc, er, S, A.accumMode);\n",
     "      else if constexpr (kHome) { float4 a = sAcc[li]; accumulateSample(a, er, S, A.accumMode); sAcc[li] = a; }\n"
     "      else accumulateSample(acc, er, S, A.accumMode);\n"),
    ("  if (valid && home) A.accum[pixG] = acc;\n",
     "  if constexpr (kHome) { if (valid && home) A.accum[pixG] = sAcc[li]; }\n  else if (valid && home) A.accum[pixG] = acc;\n"),
])
