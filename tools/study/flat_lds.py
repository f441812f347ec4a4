"""The flat kernels with LDS copies of the scene tables, typed as LDS (unconditional: valid for scenes of at most 8
rows and 16 texParams rows, as C1, C3 and UI): per-lane row and texParams reads (hit records of mixed waves,
materials, textures) become ds_read instead of global loads that share the vector-memory counter with the scratch
reloads. Round 3's copies were conditional (generic pointers: flat loads) and lost."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("  constexpr int kLdsRows = CULL ? kCullLdsRows : 0;\n  c.rowCopy = CULL;\n",
     "  constexpr int kLdsRows = CULL ? kCullLdsRows : 8;\n  c.rowCopy = true;\n"),
    ("    if (kLdsFitAll || A.n <= kLdsRows) {  // uniform", "    if (kLdsFitAll || !CULL || A.n <= kLdsRows) {  // uniform"),
    ("  constexpr int kLdsTp = CULL ? kCullLdsTp : 0;\n", "  constexpr int kLdsTp = CULL ? kCullLdsTp : 16;\n"),
    ("    if (kLdsFitAll || A.tn <= kLdsTp) {  // uniform", "    if (kLdsFitAll || !CULL || A.tn <= kLdsTp) {  // uniform"),
])
