"""Launch bounds of the run-time kernel forms (flat, pre-cull, room) set to {6, 6, 7} waves per SIMD instead of the
product's {6, 8, 7}: the occupancy of a kernel compiled for one scene's plugin set (fewer spills than the precompiled
all-plugin pair) may differ from the precompiled kernels' sweeps."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_jit.cpp", [("constexpr int kWaves[3] = {6, 8, 7}", "constexpr int kWaves[3] = {6, 6, 7}")])
