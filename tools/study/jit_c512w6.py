"""The run-time pre-cull kernel with 512-thread workgroups (16 x 32 strips) at 6 waves per SIMD (80 VGPRs, three
workgroups per CU within the LDS budget) instead of 1,024 threads at 8 waves: a kernel compiled for one scene's
plugin set spills less, so it may prefer registers to the larger sort pool."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

patch("sail_jit.cpp", [("constexpr int kWaves[3] = {6, 8, 7}, kThreads[3] = {256, 1024, 256};",
                        "constexpr int kWaves[3] = {6, 6, 7}, kThreads[3] = {256, 512, 256};")])
patch("sail_capi.cpp", [("const unsigned nt = jmode == SAIL_JIT_MODE_CULL ? 1024u : 256u;",
                         "const unsigned nt = jmode == SAIL_JIT_MODE_CULL ? 512u : 256u;")])
