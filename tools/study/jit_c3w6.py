"""Room-set scenes' run-time kernel (room form, compiled for the scene's set and rows) at 6 waves per SIMD instead of 7."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_capi.cpp", [("""  if (mode == SAIL_JIT_MODE_ROOM) return kernelSet == SAIL_KSET_ROOM ? 7 : 8;""", """  if (mode == SAIL_JIT_MODE_ROOM) return kernelSet == SAIL_KSET_ROOM ? 6 : 8;""")])
