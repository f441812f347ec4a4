"""Two bit-identical instruction cuts in the intersection code, measured together:
(1) every local-space intersect (sphere, cone, cylinder, hyperboloid, paraboloid, disk, the shared quadric loop) starts
    from W2L(ray.d), the same value for every row a sweep tests: compute it once per ray in mkRay (Ray.dl) instead of
    once per tested row (C3's four spheres, C4's quadrics);
(2) quadratic()'s two divisions q / A and C / q each guard their reciprocal's range; one guard for both (the fast
    Newton reciprocal when both divisors are in range, else the IEEE divides), as mkRay does for its three."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patch import patch

pairs = [
    ("struct Ray { V3 o, d; float rx, ry, rz; };", "struct Ray { V3 o, d; float rx, ry, rz; V3 dl; };"),
    ("  Ray r; r.o = o; r.d = d;\n", "  Ray r; r.o = o; r.d = d; r.dl = W2L(d);\n"),
    ("  t0 = fdiv(q, A);\n  t1 = fdiv(C, q);\n",
     "  const float aA = fabsf(A), aq = fabsf(q);\n"
     "  if (__builtin_expect(aA >= 0x1p-126f && aA <= 0x1p126f && aq >= 0x1p-126f && aq <= 0x1p126f, 1)) {\n"
     "    const float yA = __builtin_amdgcn_rcpf(A), yq = __builtin_amdgcn_rcpf(q);\n"
     "    t0 = q * fma_(fma_(-A, yA, 1.0f), yA, yA);\n"
     "    t1 = C * fma_(fma_(-q, yq, 1.0f), yq, yq);\n"
     "  } else {\n"
     "    float AA = A, qq = q;\n"
     "    __asm__ volatile(\"\" : \"+v\"(AA), \"+v\"(qq));\n"
     "    t0 = q * (1.0f / AA);\n"
     "    t1 = C * (1.0f / qq);\n"
     "  }\n"),
]
patch("sail_trace.hip", pairs)
# the seven intersects: "const V3 d = W2L(r0.d), o = W2L(r0.o - X);" -> "const V3 d = r0.dl, o = ..."
p = os.path.join(sys.argv[1], "sail_trace.hip")
s = open(p).read()
n = s.count("const V3 d = W2L(r0.d), o = W2L(r0.o - ")
assert n == 7, n
s = s.replace("const V3 d = W2L(r0.d), o = W2L(r0.o - ", "const V3 d = r0.dl, o = W2L(r0.o - ")
open(p, "w").write(s)
