"""sail_amd — MI355X-native drop-in for ThinkLib/Sail's progressive path-trace hot path.

Layout:
  csrc/       HIP kernels (trace megakernel, display filter) + the C-ABI library (include/sail_hip.h)
  lib/        built libsail_hip.so (gfx950)
  js/         the Sail JavaScript API (Renderer / Scene / Camera / scene.add) over an N-API addon
  capi.py     the same C ABI from Python (tests, bench)
"""
from . import capi  # noqa: F401

__all__ = ["capi"]
