"""The pre-cull kernel's sweep (its register peak) without the path's throughput and pixel index live in VGPRs: they
wait in the lane's own slot of the sort buffer (free between the shadow pass and the scatter; each lane reads back
its own slot before the counting barrier) and are read back after the sweep. Same values."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [("        sw = sweepRay(c, ray, depth == 1);\n        if (sw.best >= kMaxDistance) {  // the path leaves the scene: its radiance is final\n",
"""        if constexpr (CULL) {
          sSt2[3][li] = make_float2(fpdf.x, fpdf.y);
          sSt2[4][li] = make_float2(fpdf.z, __int_as_float(pixel));
        }
        sw = sweepRay(c, ray, depth == 1);
        if constexpr (CULL) {
          __asm__ volatile("" ::: "memory");
          const float2 qa = sSt2[3][li], qb = sSt2[4][li];
          fpdf = v3(qa.x, qa.y, qb.x);
          pixel = __float_as_int(qb.y);
        }
        if (sw.best >= kMaxDistance) {  // the path leaves the scene: its radiance is final
""")])
