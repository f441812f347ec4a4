"""Item 7 of VERDICT r03: the room kernel's plugin set replaced by exactly the ALL scene's (Cornellbox, Sphere, Disk;
Matte, Metal, Glass; mixf, scale, uvf, checkerboard; point and spot lights), so ALL runs a kernel specialised to its
plugin set instead of the all-plugin sail_trace_kernel."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_device.h", [
    ("#define SAIL_KSET_ROOM_SHAPES ((1u << SAIL_CUBE) | (1u << SAIL_SPHERE) | (1u << SAIL_RECTANGLE) | (1u << SAIL_CORNELLBOX))",
     "#define SAIL_KSET_ROOM_SHAPES ((1u << SAIL_CORNELLBOX) | (1u << SAIL_SPHERE) | (1u << SAIL_DISK))"),
    ("#define SAIL_KSET_ROOM_MATS 0xffffffffu", "#define SAIL_KSET_ROOM_MATS ((1u << SAIL_MATTE) | (1u << SAIL_METAL) | (1u << SAIL_GLASS))"),
    ("#define SAIL_KSET_ROOM_TEX 0xffffffffu",
     "#define SAIL_KSET_ROOM_TEX ((1u << SAIL_TEX_MIXF) | (1u << SAIL_TEX_SCALE) | (1u << SAIL_TEX_UVF) | (1u << SAIL_TEX_CHECKERBOARD))"),
    ("#define SAIL_KSET_ROOM_LIGHTS 0xffffffffu", "#define SAIL_KSET_ROOM_LIGHTS ((1u << SAIL_POINT) | (1u << SAIL_SPOT))"),
])
