"""Cornell-set scenes compiled in the room form (two-barrier sort, first sample group at home, one box record for Cube and Cornellbox) at 8 waves instead of the flat form."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_capi.cpp", [("""    if (!rows) return false;  // the Cornell kernel's set is the Cornell box's own
    m = SAIL_JIT_MODE_FLAT;""", """    if (!rows) return false;  // the Cornell kernel's set is the Cornell box's own
    m = SAIL_JIT_MODE_ROOM;""")])
