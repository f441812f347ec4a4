"""Item 7 of VERDICT r03: the room kernel's plugin set replaced by exactly the AREA scene's (Cube, Disk, Sphere,
Rectangle; Matte; checkerboard2; area lights), so AREA runs a kernel specialised to its plugin set instead of the
all-plugin sail_trace_kernel."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_device.h", [
    ("#define SAIL_KSET_ROOM_SHAPES ((1u << SAIL_CUBE) | (1u << SAIL_SPHERE) | (1u << SAIL_RECTANGLE) | (1u << SAIL_CORNELLBOX))",
     "#define SAIL_KSET_ROOM_SHAPES ((1u << SAIL_CUBE) | (1u << SAIL_DISK) | (1u << SAIL_SPHERE) | (1u << SAIL_RECTANGLE))"),
    ("#define SAIL_KSET_ROOM_MATS 0xffffffffu", "#define SAIL_KSET_ROOM_MATS (1u << SAIL_MATTE)"),
    ("#define SAIL_KSET_ROOM_TEX 0xffffffffu", "#define SAIL_KSET_ROOM_TEX (1u << SAIL_TEX_CHECKERBOARD2)"),
    ("#define SAIL_KSET_ROOM_LIGHTS 0xffffffffu", "#define SAIL_KSET_ROOM_LIGHTS (1u << SAIL_AREA)"),
])
