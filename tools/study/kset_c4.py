"""The pre-cull kernel compiled for exactly C4's plugin set (Cube, Sphere, Cone, Cylinder, Disk, Hyperboloid,
Paraboloid; every material; checkerboard and checkerboard2; area, point and spot lights) instead of every plugin:
what a run-time compiled pre-cull kernel would gain on C4."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_trace.hip", [
    ("SAIL_TRACE_KERNELS(sail_trace_kernel_cull, SAIL_CULL_WAVES, true, ~0u, ~0u, ~0u, ~0u, SAIL_CULL_NT, SAIL_CULL_GROUP_NT)",
     "SAIL_TRACE_KERNELS(sail_trace_kernel_cull, SAIL_CULL_WAVES, true, 0x1F6u, 0x1Eu, 0xA0u, 0x7u, SAIL_CULL_NT, SAIL_CULL_GROUP_NT)"),
])
