"""Item 1 of VERDICT r03, the next structural attempt: the room kernel with the pre-cull kernel's compacted shadow
rays (lit matte paths park their shadow ray in the sort buffer; the workgroup's first threads trace them, so waves
without a lit matte path run no shadow sweep), at 7 waves per SIMD."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("  constexpr bool kShCompact = CULL && KL != 0u;",
     "  constexpr bool kShCompact = (CULL || KS == SAIL_KSET_ROOM_SHAPES) && KL != 0u;"),
    ("#define SAIL_ROOM_WAVES 7", "#define SAIL_ROOM_WAVES 7"),
])
