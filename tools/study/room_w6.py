"""Control for room_sh6: the room kernel at 6 waves per SIMD (80 VGPRs), nothing else changed."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [("#define SAIL_ROOM_WAVES 7", "#define SAIL_ROOM_WAVES 6")])
