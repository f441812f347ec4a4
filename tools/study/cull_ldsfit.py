"""The pre-cull kernel with its LDS scene-table copies unconditional (valid for scenes of at most 72 rows and 136
texParams rows, as C4): the per-lane row and texParams pointers are then known to point into LDS, so the candidate
loops, hit record and material reads compile to ds_read instead of flat loads (which also wait on every outstanding
vector-memory load, the scratch reloads included)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("    if (A.n <= kLdsRows) {  // uniform\n      const float4* src = reinterpret_cast<const float4*>(A.prims);",
     "    {\n      const float4* src = reinterpret_cast<const float4*>(A.prims);"),
    ("    if (A.tn <= kLdsTp) {  // uniform\n      const float4* src = reinterpret_cast<const float4*>(A.texparams);",
     "    {\n      const float4* src = reinterpret_cast<const float4*>(A.texparams);"),
])
