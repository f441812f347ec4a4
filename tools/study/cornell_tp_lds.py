"""The Cornell form (C1 / C2 / C5) with only its texParams table in LDS (typed), the rows still read from global
memory (scalar loads in uniform waves): the room form's LDS tables cost the Cornell form 0.5 %."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("  constexpr int kLdsRows = CULL ? kCullLdsRows : (!CULL && kFlatTp > 0 && kRows > 0 ? kRows : 0);\n",
     "  constexpr int kLdsRows = CULL ? kCullLdsRows : (!CULL && FAM && kFlatTp > 0 && kRows > 0 ? kRows : 0);\n"),
])
patch("sail_capi.cpp", [
    ("    if (spec.rows && m == SAIL_JIT_MODE_ROOM && c->tn >= 1 && c->tn <= kSailJitMaxFlatTp) spec.tn = c->tn;\n",
     "    if (spec.rows && c->tn >= 1 && c->tn <= kSailJitMaxFlatTp) spec.tn = c->tn;\n"),
])
