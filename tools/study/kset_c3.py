"""The room kernel compiled for exactly C3's plugin set (Rectangle, Cube, Sphere; Matte, Metal, Mirror, Glass;
checkerboard and checkerboard2; area lights) instead of the room family's (any material, texture and light): what a
run-time compiled room kernel would gain on C3."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_device.h", [
    ("#define SAIL_KSET_ROOM_SHAPES ((1u << SAIL_CUBE) | (1u << SAIL_SPHERE) | (1u << SAIL_RECTANGLE) | (1u << SAIL_CORNELLBOX))",
     "#define SAIL_KSET_ROOM_SHAPES ((1u << SAIL_CUBE) | (1u << SAIL_SPHERE) | (1u << SAIL_RECTANGLE))"),
    ("#define SAIL_KSET_ROOM_MATS 0xffffffffu",
     "#define SAIL_KSET_ROOM_MATS ((1u << SAIL_MATTE) | (1u << SAIL_METAL) | (1u << SAIL_MIRROR) | (1u << SAIL_GLASS))"),
    ("#define SAIL_KSET_ROOM_TEX 0xffffffffu",
     "#define SAIL_KSET_ROOM_TEX ((1u << SAIL_TEX_CHECKERBOARD) | (1u << SAIL_TEX_CHECKERBOARD2))"),
    ("#define SAIL_KSET_ROOM_LIGHTS 0xffffffffu", "#define SAIL_KSET_ROOM_LIGHTS (1u << SAIL_AREA)"),
])
