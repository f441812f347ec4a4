"""The exact segment counter kept per wave in scalar registers (popcount of the live-lane ballot at each bounce)
instead of a per-lane VGPR counter and a 64-lane shuffle reduction at the end: one VGPR less across the whole
sample loop. The counts are the same."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

PAIRS = [("  unsigned segs = 0;\n", "  unsigned long long segsW = 0;  // wave-uniform\n"),
         ("      int key = 0;\n      if (alive) {\n        segs++;\n",
          "      int key = 0;\n      segsW += (unsigned long long)__popcll(__builtin_amdgcn_ballot_w64(alive));\n      if (alive) {\n"),
         ("""    unsigned long long v = segs;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) atomicAdd(&A.segCounter[(blockIdx.x * 4u + (unsigned)wave) % SAIL_SEG_SLOTS], v);""",
          """    if (lane == 0) atomicAdd(&A.segCounter[(blockIdx.x * 4u + (unsigned)wave) % SAIL_SEG_SLOTS], segsW);""")]
if __name__ == "__main__":
    patch("sail_trace.hip", PAIRS)
