"""Cornell-set scenes' run-time kernel (flat form, compiled for the scene's set and rows) at 7 waves per SIMD instead of 8."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_capi.cpp", [("""  return kernelSet == SAIL_KSET_CORNELL ? 8 : 6;""", """  return kernelSet == SAIL_KSET_CORNELL ? 7 : 6;""")])
