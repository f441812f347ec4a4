"""No path sort at the first bounce: primary rays of a 16 x 4 (or 16 x 64) pixel strip are coherent, so their waves
mostly hold one primitive already and no path is dead yet; each lane keeps its own pixel's path (no scatter, no
gather, no barriers) for the first hit record and shading, and the sort resumes at bounce 2. Same paths, same
operations: bit-identical."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("      if constexpr (twoBar) {\n      // every wave scans the counts itself",
     "      if (depth > 1) {\n      if constexpr (twoBar) {\n      // every wave scans the counts itself"),
    ("      alive = li < nAlive;\n      ShadowPending sp;", "      alive = li < nAlive;\n      }\n      ShadowPending sp;"),
    ("      if (alive) {\n        if constexpr (kPack == 2) {\n          const float4 q0 = sSt4[0][li], q1 = sSt4[1][li], q2 = sSt4[2][li];",
     "      if (alive) {\n        if (depth == 1) {\n          keyG = key;\n        } else if constexpr (kPack == 2) {\n          const float4 q0 = sSt4[0][li], q1 = sSt4[1][li], q2 = sSt4[2][li];"),
])
