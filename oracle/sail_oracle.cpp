// oracle/sail_oracle.cpp — TEST INFRASTRUCTURE: the CPU parity oracle for the Sail trace/filter path.
//
// Scalar, single-threaded, line-by-line restatement of the reference's generated trace fragment program
// (src/shader/**: fstrace + path + shape/material/light/texture plugins as assembled by
// src/core/shader.js:58-76 / src/shader/generator.js:107-123) and of the window/tonemap/gamma display
// filters (src/shader/filter/*.glsl). Every function cites the GLSL it restates. It deliberately keeps
// the reference's structure (texture-addressed scene reads, full hit record for every primitive hit,
// if-chains) so that it is an independent check of the optimised HIP kernel in sail_amd/csrc.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
//
// Defined semantics for what GLSL leaves open: uninitialised locals and unwritten `out`
// parameters are 0; min/max/clamp return the non-NaN operand; transcendentals follow ref_math.h; GLSL division
// a / b is a * RN(1/b) (ref_math.h div_s: the reciprocal-multiply form GPU compilers emit, correctly rounded);
// int() truncates (NaN -> 0); negative % follows C; a NaN texture row coordinate addresses row 0;
// a zero-height texture reads 0. Floating-point contraction is disabled at build time.
//
// Pinning (see DESIGN.md "Oracle"): the scene rows, camera matrices, filter tables and CPU intersect
// distances are checked against fixtures captured from the reference bundle itself
// (tests/golden/make_fixtures.js); shading arithmetic is pinned by the GLSL text plus analytic
// known-answer tests (tests/test_oracle_*.py). The GLSL itself cannot execute in this container.
//
// Build: oracle/build.sh -> oracle/build/libsail_oracle.so (+ libsail_oracle_count.so, SAIL_COUNT_OPS)
#include <cstring>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include "ref_math.h"

// The scalar type of all GLSL arithmetic. A class (not a typedef of float) so that GLSL division has its
// defined meaning a * RN(1/b) (ref_math.h div_s) everywhere; the SAIL_COUNT_OPS build also counts ops
// (every + - * / min max sqrt and transcendental = 1, SURVEY §8(d) op model).
#ifdef SAIL_COUNT_OPS
static unsigned long long g_ops = 0;
#define OPINC() (g_ops++)
#define OPC(k) (g_ops += (k))
#else
#define OPINC() ((void)0)
#define OPC(k) ((void)0)
#endif
struct F {
  float v;
  F() : v(0.0f) {}
  F(float x) : v(x) {}
  F(double x) : v((float)x) {}
  F(int x) : v((float)x) {}
  explicit operator float() const { return v; }
};
static inline F operator+(F a, F b) { OPINC(); return F(a.v + b.v); }
static inline F operator-(F a, F b) { OPINC(); return F(a.v - b.v); }
static inline F operator*(F a, F b) { OPINC(); return F(a.v * b.v); }
static inline F operator/(F a, F b) { OPINC(); return F(refm::div_s(a.v, b.v)); }
static inline F operator-(F a) { return F(-a.v); }
static inline bool operator<(F a, F b) { return a.v < b.v; }
static inline bool operator>(F a, F b) { return a.v > b.v; }
static inline bool operator<=(F a, F b) { return a.v <= b.v; }
static inline bool operator>=(F a, F b) { return a.v >= b.v; }
static inline bool operator==(F a, F b) { return a.v == b.v; }
static inline bool operator!=(F a, F b) { return a.v != b.v; }
static inline F& operator+=(F& a, F b) { a = a + b; return a; }
static inline F& operator*=(F& a, F b) { a = a * b; return a; }
static inline float raw(F a) { return a.v; }
static inline float fdiv_s(float a, float b) { return refm::div_s(a, b); }  // GLSL a / b on raw floats

// ---- scalar builtins (GLSL semantics, ref_math.h spec) ----------------------------------------------
static inline F fmin_(F a, F b) { OPC(1); return F(refm::fmin_s(raw(a), raw(b))); }
static inline F fmax_(F a, F b) { OPC(1); return F(refm::fmax_s(raw(a), raw(b))); }
static inline F clamp_(F x, F lo, F hi) { return fmin_(fmax_(x, lo), hi); }
static inline F sqrt_(F x) { OPC(1); return F(refm::sqrt_s(raw(x))); }
static inline F sin_(F x) { OPC(1); return F(refm::sin_s(raw(x))); }
static inline F cos_(F x) { OPC(1); return F(refm::cos_s(raw(x))); }
static inline F tan_(F x) { OPC(1); return F(refm::tan_s(raw(x))); }
static inline F atan_(F x) { OPC(1); return F(refm::atan_s(raw(x))); }
static inline F atan2_(F y, F x) { OPC(1); return F(refm::atan2_s(raw(y), raw(x))); }
static inline F acos_(F x) { OPC(1); return F(refm::acos_s(raw(x))); }
static inline F pow_(F x, F y) { OPC(1); return F(refm::pow_s(raw(x), raw(y))); }
static inline F floor_(F x) { OPC(1); return F(refm::floor_s(raw(x))); }
static inline F fract_(F x) { OPC(1); return F(refm::fract_s(raw(x))); }
static inline F abs_(F x) { return F(fabsf(raw(x))); }
static inline int toint(F x) { return refm::to_int(raw(x)); }
static inline bool isnan_(F x) { return raw(x) != raw(x); }

// ---- define.glsl constants (f32-rounded like a GLSL float literal) -------------------------------
static const float kMaxDistance = 1e5f, kEps = 1e-5f, kOneMinusEps = 0.9999f, kInf = 1e5f;
static const float kPI = 3.141592653589793f, kInvPI = 0.3183098861837907f;
static const float kPiOver2 = 1.570796326794896f, kPiOver4 = 0.785398163397448f;
static const float kObjLen = 17.0f, kLightLen = 17.0f, kTexLen = 15.0f;
enum { CUBE = 1, SPHERE = 2, RECTANGLE = 3, CONE = 4, CYLINDER = 5, DISK = 6, HYPERBOLOID = 7,
       PARABOLOID = 8, CORNELLBOX = 9 };
enum { AREA = 0, POINT = 1, SPOT = 2 };
enum { MATTE = 1, MIRROR = 2, METAL = 3, GLASS = 4 };
enum { UNIFORM_COLOR = 0, CHECKERBOARD = 5, CHECKERBOARD2 = 7, BILERP = 8, MIXF = 9, SCALE = 10, UVF = 11 };
enum { F_NOOP = 0, F_CONDUCTOR = 1, F_DIELECTRIC = 2 };

// ---- vec types ------------------------------------------------------------------------------------
struct V2 { F x, y; };
struct V3 { F x, y, z; };
static inline V2 v2(F x, F y) { V2 r; r.x = x; r.y = y; return r; }
static inline V3 v3(F x, F y, F z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline V3 v3s(F s) { return v3(s, s, s); }
static const V3 BLACKv = {F(0.0f), F(0.0f), F(0.0f)};
static const V3 WHITEv = {F(1.0f), F(1.0f), F(1.0f)};
static inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 operator/(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline V3 operator*(V3 a, F s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 operator*(F s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline V3 operator/(V3 a, F s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline V3 operator+(V3 a, F s) { return v3(a.x + s, a.y + s, a.z + s); }
static inline V3 operator-(V3 a, F s) { return v3(a.x - s, a.y - s, a.z - s); }
static inline V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V2 operator*(F s, V2 a) { return v2(s * a.x, s * a.y); }
static inline F dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline F length(V3 v) { return sqrt_(dot(v, v)); }
static inline V3 normalize(V3 v) { return v / length(v); }
static inline V3 vmin(V3 a, V3 b) { return v3(fmin_(a.x, b.x), fmin_(a.y, b.y), fmin_(a.z, b.z)); }
static inline V3 vmax(V3 a, V3 b) { return v3(fmax_(a.x, b.x), fmax_(a.y, b.y), fmax_(a.z, b.z)); }
static inline V3 vclamp(V3 x, V3 lo, V3 hi) { return vmin(vmax(x, lo), hi); }
static inline bool veq(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
static inline V3 reflect_(V3 I, V3 N) { return I - (F(2.0f) * dot(N, I)) * N; }  // GLSL spec formula
static inline V3 refract_(V3 I, V3 N, F eta) {                                  // GLSL spec formula
  const F dni = dot(N, I);
  const F k = F(1.0f) - eta * eta * (F(1.0f) - dni * dni);
  if (k < F(0.0f)) return BLACKv;
  return eta * I - (eta * dni + sqrt_(k)) * N;
}
static inline V3 mix3(V3 x, V3 y, F a) { return x * (F(1.0f) - a) + y * a; }

// utility.glsl:1-9
static inline V3 worldToLocal(V3 v, V3 ns, V3 ss, V3 ts) { return v3(dot(v, ss), dot(v, ts), dot(v, ns)); }
static inline V3 localToWorld(V3 v, V3 ns, V3 ss, V3 ts) {
  return v3(ss.x * v.x + ts.x * v.y + ns.x * v.z, ss.y * v.x + ts.y * v.y + ns.y * v.z,
            ss.z * v.x + ts.z * v.y + ns.z * v.z);
}
// define.glsl:62-64
static const V3 OSN = {F(0.0f), F(1.0f), F(0.0f)};
static const V3 OSS = {F(0.0f), F(0.0f), F(-1.0f)};
static const V3 OST = {F(1.0f), F(0.0f), F(0.0f)};
static inline V3 W2L(V3 v) { return worldToLocal(v, OSN, OSS, OST); }
static inline V3 L2W(V3 v) { return localToWorld(v, OSN, OSS, OST); }
static inline bool equalZero(F x) { return x < F(1e-3f) && x > F(-1e-3f); }  // utility.glsl:58-60

// utility.glsl:37-51
static bool quadratic(F A, F B, F C, F& t0, F& t1) {
  const F discrim = B * B - F(4.0f) * A * C;
  if (discrim < F(0.0f)) return false;
  const F rootDiscrim = sqrt_(discrim);
  F q;
  if (B < F(0.0f)) q = F(-0.5f) * (B - rootDiscrim);
  else q = F(-0.5f) * (B + rootDiscrim);
  t0 = q / A;
  t1 = C / q;
  if (t0 > t1) { F tmp = t0; t0 = t1; t1 = tmp; }
  return true;
}
// utility.glsl:53-56
static inline V3 sphericalDirection(F sinTheta, F cosTheta, F phi) {
  return v3(sinTheta * cos_(phi), sinTheta * sin_(phi), cosTheta);
}

// ---- scene textures (tracer.js:62-80 R32F, NEAREST, CLAMP_TO_EDGE; texhelper.glsl:1-36) -----------
struct Tex { const float* d; int w, h; };
struct Ctx {
  Tex objects, texParams, lights;
  int n, tn, ln;
  unsigned shapeMask, matMask, texMask, lightMask;
  F fcx, fcy, fcz;              // gl_FragCoord
  F timeSinceStart;
};
static Ctx C;

// NEAREST texel of a normalised coordinate; a NaN coordinate addresses texel 0
static inline int texel(float c, int size) {
  if (c != c) return 0;
  const float s = floorf(c * (float)size);
  if (!(s >= 0.0f)) return 0;
  if (s >= (float)(size - 1)) return size - 1;
  return (int)s;
}
static inline F fetch(const Tex& t, float cx, float cy) {
  if (t.h <= 0) return F(0.0f);  // zero-height texture (ln = 0) reads 0
  return F(t.d[texel(cy, t.h) * t.w + texel(cx, t.w)]);
}
// coordinate arithmetic is texture addressing, not shader arithmetic: kept in raw f32 (not counted)
static inline F readFloat(const Tex& t, float x, F y, float width) { return fetch(t, fdiv_s(x, width), raw(y)); }
static inline int readInt(const Tex& t, float x, F y, float width) { return toint(readFloat(t, x, y, width)); }
static inline bool readBool(const Tex& t, float x, F y, float width) { return readInt(t, x, y, width) == 1; }
static inline V3 readVec3(const Tex& t, float x, F y, float width) {
  float px = fdiv_s(x, width);
  V3 r;
  r.x = fetch(t, px, raw(y)); px += fdiv_s(1.0f, width);
  r.y = fetch(t, px, raw(y)); px += fdiv_s(1.0f, width);
  r.z = fetch(t, px, raw(y));
  return r;
}
static inline F rowCoord(int i, int n) { return F(fdiv_s((float)i, (float)(n - 1))); }  // float(i)/float(n-1)
static inline F matCoord(F v) { return F(fdiv_s(raw(v), (float)(C.tn - 1))); }         // readFloat(...)/float(tn-1)

// ---- struct.glsl:1-18 ------------------------------------------------------------------------------
struct Intersect {
  F d; V3 hit, normal, dpdu, dpdv; bool into; F matIndex; V3 sc, emission; F seed; int index; int matCategory;
};
static inline Intersect zeroIns() { Intersect r{}; return r; }
struct Ray { V3 origin, dir; };
static inline Ray ray_(V3 o, V3 d) { Ray r; r.origin = o; r.dir = d; return r; }

// ---- random.glsl:5-18 (gl_FragCoord-hashed) --------------------------------------------------------
static inline F hash1(F seed, F a, F b, F c) {
  const V3 p = v3(C.fcx + seed, C.fcy + seed, C.fcz + seed);
  return fract_(sin_(dot(p, v3(a, b, c))) * F(43758.5453f) + seed);
}
static inline V2 random2(F seed) {
  return v2(hash1(seed, F(12.9898f), F(78.233f), F(151.7182f)), hash1(seed, F(63.7264f), F(10.873f), F(623.6736f)));
}
static inline int randomInt(F seed, int mn, int mx) {
  return mn + toint(hash1(seed, F(12.9898f), F(78.233f), F(151.7182f)) * F((float)(mx - mn)));
}

// ---- sampler.glsl ----------------------------------------------------------------------------------
static inline V3 uniformSampleSphere(V2 u) {  // :1-5
  const F z = F(1.0f) - F(2.0f) * u.x;
  const F r = sqrt_(F(1.0f) - z * z);
  const F angle = F(2.0f) * F(kPI) * u.y;
  return v3(r * cos_(angle), r * sin_(angle), z);
}
static inline V3 cosineSampleHemisphere(V2 u) {  // :7-12
  const F r = sqrt_(u.x);
  const F angle = F(2.0f) * F(kPI) * u.y;
  return v3(r * cos_(angle), r * sin_(angle), sqrt_(F(1.0f) - u.x));
}
static inline V2 concentricSampleDisk(V2 u) {  // :26-41
  const F uOffset = F(2.0f) * u.x - F(1.0f);
  const F vOffset = F(2.0f) * u.y - F(1.0f);
  if (uOffset == F(0.0f) && vOffset == F(0.0f)) return v2(F(0.0f), F(0.0f));
  F theta, r;
  if (abs_(uOffset) > abs_(vOffset)) { r = uOffset; theta = (vOffset / uOffset) * F(kPiOver4); }
  else { r = vOffset; theta = F(kPiOver2) - (uOffset / vOffset) * F(kPiOver4); }
  return r * v2(cos_(theta), sin_(theta));
}

// ---- texture plugins (shader.texture.js:22-29 + texture/*.glsl) --------------------------------------
static V3 getSurfaceColor(V3 hit, V2 uv, F texIndex) {
  (void)hit;
  const Tex& tp = C.texParams;
  const int texCategory = readInt(tp, 0.0f, texIndex, kTexLen);
  if (texCategory == UNIFORM_COLOR) return readVec3(tp, 1.0f, texIndex, kTexLen);
  if (!((C.texMask >> texCategory) & 1u)) return BLACKv;
  switch (texCategory) {
    case CHECKERBOARD: {  // checkerboard.glsl:6-20
      const F size = readFloat(tp, 1.0f, texIndex, kTexLen);
      const F lineWidth = readFloat(tp, 2.0f, texIndex, kTexLen);
      const F width = F(0.5f) * lineWidth / size;
      const F fx = uv.x / size - floor_(uv.x / size), fy = uv.y / size - floor_(uv.y / size);
      const bool in_outline = (fx < width || fx > F(1.0f) - width) || (fy < width || fy > F(1.0f) - width);
      if (!in_outline) return WHITEv;
      return v3s(F(0.5f));
    }
    case CHECKERBOARD2: {  // checkerboard2.glsl:7-16
      const V3 c1 = readVec3(tp, 1.0f, texIndex, kTexLen), c2 = readVec3(tp, 4.0f, texIndex, kTexLen);
      const F size = readFloat(tp, 7.0f, texIndex, kTexLen);
      const V2 q = v2(floor_(uv.x / size), floor_(uv.y / size));
      if (toint(q.x + q.y) % 2 == 0) return c1;
      return c2;
    }
    case BILERP: {  // bilerp.glsl:8-13, intended math (the reference text does not compile: SURVEY a.7)
      const V3 c00 = readVec3(tp, 1.0f, texIndex, kTexLen), c01 = readVec3(tp, 4.0f, texIndex, kTexLen);
      const V3 c10 = readVec3(tp, 7.0f, texIndex, kTexLen), c11 = readVec3(tp, 10.0f, texIndex, kTexLen);
      return (F(1.0f) - uv.x) * (F(1.0f) - uv.y) * c00 + (F(1.0f) - uv.x) * (uv.y) * c01 +
             (uv.x) * (F(1.0f) - uv.y) * c10 + (uv.x) * (uv.y) * c11;
    }
    case MIXF: {  // mixf.glsl:7-12
      const V3 c1 = readVec3(tp, 1.0f, texIndex, kTexLen), c2 = readVec3(tp, 4.0f, texIndex, kTexLen);
      const F amount = readFloat(tp, 7.0f, texIndex, kTexLen);
      return (F(1.0f) - amount) * c1 + amount * c2;
    }
    case SCALE: {  // scale.glsl:6-10
      const V3 c1 = readVec3(tp, 1.0f, texIndex, kTexLen), c2 = readVec3(tp, 4.0f, texIndex, kTexLen);
      return c1 * c2;
    }
    case UVF:  // uvf.glsl:1-3
      return v3(uv.x - floor_(uv.x), uv.y - floor_(uv.y), F(0.0f));
    default: return BLACKv;
  }
}

// ---- boundbox.glsl:1-17 (struct Boundbox{vec3 max; vec3 min;}: constructor order is (max, min)) ----
struct Boundbox { V3 max, min; };
static bool testBoundbox(const Ray& ray, Boundbox box) {
  const V3 tMin = (box.min - ray.origin) / ray.dir;
  const V3 tMax = (box.max - ray.origin) / ray.dir;
  const V3 t1 = vmin(tMin, tMax), t2 = vmax(tMin, tMax);
  const F tNear = fmax_(fmax_(t1.x, t1.y), t1.z);
  const F tFar = fmin_(fmin_(t2.x, t2.y), t2.z);
  if (tNear < F(0.0f) && tFar < F(0.0f)) return false;
  return tNear < tFar;
}
static inline Boundbox BB(V3 a, V3 b) { Boundbox r; r.max = a; r.min = b; return r; }
static inline F sgn(bool rev) { return rev ? F(-1.0f) : F(1.0f); }

// ---- cube.glsl ----------------------------------------------------------------------------------------
struct Cube { V3 min, max; F matIndex, texIndex; V3 emission; bool reverseNormal; };
static Cube parseCube(F index) {  // :14-23
  const Tex& o = C.objects; Cube c;
  c.min = readVec3(o, 1.0f, index, kObjLen);
  c.max = readVec3(o, 4.0f, index, kObjLen);
  c.reverseNormal = readBool(o, 7.0f, index, kObjLen);
  c.matIndex = matCoord(readFloat(o, 8.0f, index, kObjLen));
  c.texIndex = matCoord(readFloat(o, 9.0f, index, kObjLen));
  c.emission = readVec3(o, 10.0f, index, kObjLen);
  return c;
}
static V3 normalForCube(V3 hit, const Cube& cube) {  // :25-38
  const F c = sgn(cube.reverseNormal);
  if (hit.x < cube.min.x + F(0.0001f)) return c * v3(F(-1.0f), F(0.0f), F(0.0f));
  else if (hit.x > cube.max.x - F(0.0001f)) return c * v3(F(1.0f), F(0.0f), F(0.0f));
  else if (hit.y < cube.min.y + F(0.0001f)) return c * v3(F(0.0f), F(-1.0f), F(0.0f));
  else if (hit.y > cube.max.y - F(0.0001f)) return c * v3(F(0.0f), F(1.0f), F(0.0f));
  else if (hit.z < cube.min.z + F(0.0001f)) return c * v3(F(0.0f), F(0.0f), F(-1.0f));
  return c * v3(F(0.0f), F(0.0f), F(1.0f));
}
static void computeDpDForBox(V3 normal, V3& dpdu, V3& dpdv) {  // cube.glsl:40-48, cornellbox.glsl:53-61
  if (abs_(normal.x) < F(0.5f)) dpdu = cross(normal, v3(F(1.0f), F(0.0f), F(0.0f)));
  else dpdu = cross(normal, v3(F(0.0f), F(1.0f), F(0.0f)));
  dpdv = cross(normal, dpdu);
}
static V2 getCubeUV(V3 hit, const Cube& cube) {  // :54-63 (face tests compare hit-min against min: bug kept)
  const V3 tr = cube.max - cube.min;
  hit = hit - cube.min;
  if (hit.x < cube.min.x + F(0.0001f) || hit.x > cube.max.x - F(0.0001f)) return v2(hit.y / tr.y, hit.z / tr.z);
  else if (hit.y < cube.min.y + F(0.0001f) || hit.y > cube.max.y - F(0.0001f)) return v2(hit.x / tr.x, hit.z / tr.z);
  return v2(hit.x / tr.x, hit.y / tr.y);
}
static Intersect intersectCube(const Ray& ray, const Cube& cube) {  // :65-87
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  const V3 tMin = (cube.min - ray.origin) / ray.dir;
  const V3 tMax = (cube.max - ray.origin) / ray.dir;
  const V3 t1 = vmin(tMin, tMax), t2 = vmax(tMin, tMax);
  const F tNear = fmax_(fmax_(t1.x, t1.y), t1.z);
  const F tFar = fmin_(fmin_(t2.x, t2.y), t2.z);
  F t = F(-1.0f);
  if (tNear > F(kEps) && tNear < tFar) t = tNear;
  else if (tNear < tFar) t = tFar;
  if (t > F(kEps)) {
    result.d = t;
    result.hit = ray.origin + t * ray.dir;
    result.normal = normalForCube(ray.origin + t * ray.dir, cube);
    computeDpDForBox(result.normal, result.dpdu, result.dpdv);
    result.matIndex = cube.matIndex;
    result.sc = getSurfaceColor(result.hit, getCubeUV(result.hit, cube), cube.texIndex);
    result.emission = cube.emission;
  }
  return result;
}

// ---- sphere.glsl ----------------------------------------------------------------------------------------
struct Sphere { V3 c; F r, matIndex, texIndex; V3 emission; bool reverseNormal; };
static bool testBoundboxForSphere(const Ray& ray, const Sphere& s) {  // :10-16
  return testBoundbox(ray, BB(s.c - v3s(s.r), s.c + v3s(s.r)));
}
static Sphere parseSphere(F index) {  // :18-27
  const Tex& o = C.objects; Sphere s;
  s.c = readVec3(o, 1.0f, index, kObjLen);
  s.r = readFloat(o, 4.0f, index, kObjLen);
  s.reverseNormal = readBool(o, 5.0f, index, kObjLen);
  s.matIndex = matCoord(readFloat(o, 6.0f, index, kObjLen));
  s.texIndex = matCoord(readFloat(o, 7.0f, index, kObjLen));
  s.emission = readVec3(o, 8.0f, index, kObjLen);
  return s;
}
static V3 normalForSphere(V3 hit, const Sphere& s) { return sgn(s.reverseNormal) * (hit - s.c) / s.r; }  // :29-31
static void computeDpDForSphere(V3 hit, F radius, V3& dpdu, V3& dpdv) {  // :33-43
  const F theta = acos_(clamp_(hit.z / radius, F(-1.0f), F(1.0f)));
  const F zRadius = sqrt_(hit.x * hit.x + hit.y * hit.y);
  const F invZRadius = F(1.0f) / zRadius;
  const F cosPhi = hit.x * invZRadius, sinPhi = hit.y * invZRadius;
  dpdu = v3(F(-2.0f) * F(kPI) * hit.y, F(2.0f) * F(kPI) * hit.x, F(0.0f));
  dpdv = F(kPI) * v3(hit.z * cosPhi, hit.z * sinPhi, -radius * sin_(theta));
}
static Intersect intersectSphere(Ray ray, const Sphere& s) {  // :45-86
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  ray.dir = W2L(ray.dir);
  ray.origin = W2L(ray.origin - s.c);
  const F a = dot(ray.dir, ray.dir);
  const F b = F(2.0f) * dot(ray.origin, ray.dir);
  const F c = dot(ray.origin, ray.origin) - s.r * s.r;
  F t1 = F(0.0f), t2 = F(0.0f), t;
  if (!quadratic(a, b, c, t1, t2)) return result;
  if (t2 < F(kEps)) return result;
  t = t1;
  if (t1 < F(kEps)) t = t2;
  if (t >= F(kMaxDistance)) return result;
  V3 hit = ray.origin + t * ray.dir;
  if (hit.x == F(0.0f) && hit.y == F(0.0f)) hit.x = F(1e-5f) * s.r;
  F phi = atan2_(hit.y, hit.x);
  if (phi < F(0.0f)) phi += F(2.0f) * F(kPI);
  const F u = phi / (F(2.0f) * F(kPI));
  const F theta = acos_(clamp_(hit.z / s.r, F(-1.0f), F(1.0f)));
  const F v = theta / F(kPI);
  result.d = t;
  result.hit = ray.origin + t * ray.dir;
  computeDpDForSphere(result.hit, s.r, result.dpdu, result.dpdv);
  result.normal = normalize(cross(result.dpdv, result.dpdu));
  result.matIndex = s.matIndex;
  result.sc = getSurfaceColor(result.hit, v2(u, v), s.texIndex);
  result.emission = s.emission;
  result.hit = L2W(result.hit) + s.c;
  result.normal = L2W(result.normal);
  result.dpdu = L2W(result.dpdu);
  result.dpdv = L2W(result.dpdv);
  return result;
}
static V3 sampleSphere(V2 u, const Sphere& s, F& pdf) {  // :88-92
  const V3 p = uniformSampleSphere(u);
  pdf = F(kInvPI) / (s.r * s.r);
  return p * s.r + s.c;
}

// ---- rectangle.glsl -------------------------------------------------------------------------------------
struct Rect { V3 min, max; F matIndex, texIndex; V3 emission; bool reverseNormal; };
static Rect parseRectangle(F index) {  // :14-23
  const Tex& o = C.objects; Rect r;
  r.min = readVec3(o, 1.0f, index, kObjLen);
  r.max = readVec3(o, 4.0f, index, kObjLen);
  r.reverseNormal = readBool(o, 7.0f, index, kObjLen);
  r.matIndex = matCoord(readFloat(o, 8.0f, index, kObjLen));
  r.texIndex = matCoord(readFloat(o, 9.0f, index, kObjLen));
  r.emission = readVec3(o, 10.0f, index, kObjLen);
  return r;
}
static V3 normalForRectangle(V3 hit, const Rect& r) {  // :25-30
  (void)hit;
  const V3 x = v3(r.max.x - r.min.x, F(0.0f), F(0.0f));
  const V3 y = v3(F(0.0f), r.max.y - r.min.y, r.max.z - r.min.z);
  const V3 normal = normalize(cross(x, y));
  return sgn(r.reverseNormal) * normal;
}
static Intersect intersectRectangle(Ray ray, const Rect& r) {  // :32-63
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  result.dpdu = v3(r.max.x - r.min.x, F(0.0f), F(0.0f));
  result.dpdv = v3(F(0.0f), r.max.y - r.min.y, r.max.z - r.min.z);
  result.normal = normalize(cross(result.dpdu, result.dpdv));
  const F maxX = length(result.dpdu), maxY = length(result.dpdv);
  const V3 ss = result.dpdu / maxX, ts = cross(result.normal, ss);
  ray.dir = worldToLocal(ray.dir, result.normal, ss, ts);
  ray.origin = worldToLocal(ray.origin - r.min, result.normal, ss, ts);
  if (ray.dir.z == F(0.0f)) return result;
  const F t = -ray.origin.z / ray.dir.z;
  if (t < F(kEps)) return result;
  const V3 hit = ray.origin + t * ray.dir;
  if (hit.x > maxX || hit.y > maxY || hit.x < F(-kEps) || hit.y < F(-kEps)) return result;
  result.d = t;
  result.matIndex = r.matIndex;
  result.sc = getSurfaceColor(hit, v2(hit.x / maxX, hit.y / maxY), r.texIndex);
  result.emission = r.emission;
  result.hit = localToWorld(hit, result.normal, ss, ts) + r.min;
  return result;
}
static V3 sampleRectangle(V2 u, const Rect& r, F& pdf) {  // :65-70
  const V3 x = v3(r.max.x - r.min.x, F(0.0f), F(0.0f));
  const V3 y = v3(F(0.0f), r.max.y - r.min.y, r.max.z - r.min.z);
  pdf = F(1.0f) / (length(x) * length(y));
  return r.min + x * u.x + y * u.y;
}

// ---- cone.glsl / cylinder.glsl (share the struct layout: p3, h, r) -------------------------------
struct ConeCyl { V3 p; F h, r, matIndex, texIndex; V3 emission; bool reverseNormal; };
static ConeCyl parseConeCyl(F index) {  // cone.glsl:19-29, cylinder.glsl:19-29
  const Tex& o = C.objects; ConeCyl c;
  c.p = readVec3(o, 1.0f, index, kObjLen);
  c.h = readFloat(o, 4.0f, index, kObjLen);
  c.r = readFloat(o, 5.0f, index, kObjLen);
  c.reverseNormal = readBool(o, 6.0f, index, kObjLen);
  c.matIndex = matCoord(readFloat(o, 7.0f, index, kObjLen));
  c.texIndex = matCoord(readFloat(o, 8.0f, index, kObjLen));
  c.emission = readVec3(o, 9.0f, index, kObjLen);
  return c;
}
static bool testBoundboxForConeCyl(const Ray& ray, const ConeCyl& c) {  // cone.glsl:11-17, cylinder.glsl:11-17
  return testBoundbox(ray, BB(c.p - v3(c.r, F(0.0f), c.r), c.p + v3(c.r, c.h, c.r)));
}
static V3 normalForCone(V3 hit, const ConeCyl& c) {  // cone.glsl:38-46
  hit = hit - c.p;
  const F tana = c.r / c.h;
  const F d = sqrt_(hit.x * hit.x + hit.y * hit.y);
  const F x1 = d / tana, x2 = d * tana;
  const V3 no = v3(F(0.0f), F(0.0f), c.h - x1 - x2);
  return sgn(c.reverseNormal) * normalize(hit - no);
}
static V3 normalForCylinder(V3 hit, const ConeCyl& c) {  // cylinder.glsl:36-38
  return sgn(c.reverseNormal) * normalize(v3(hit.x - c.p.x, hit.y - c.p.y, F(0.0f)));
}
static inline V3 dpduRot(V3 hit) { return v3(F(-2.0f) * F(kPI) * hit.y, F(2.0f) * F(kPI) * hit.x, F(0.0f)); }
static inline F phiOf(F y, F x) {
  F phi = atan2_(y, x);
  if (phi < F(0.0f)) phi += F(2.0f) * F(kPI);
  return phi;
}
static Intersect finishLocal(Intersect result, V3 hit, V2 uv, F matIndex, F texIndex, V3 emission, V3 p) {
  result.normal = normalize(cross(result.dpdu, result.dpdv));
  result.hit = hit;
  result.matIndex = matIndex;
  result.sc = getSurfaceColor(result.hit, uv, texIndex);
  result.emission = emission;
  result.hit = L2W(result.hit) + p;
  result.normal = L2W(result.normal);
  result.dpdu = L2W(result.dpdu);
  result.dpdv = L2W(result.dpdv);
  return result;
}
static Intersect intersectCone(Ray ray, const ConeCyl& c) {  // cone.glsl:48-99
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  ray.dir = W2L(ray.dir);
  ray.origin = W2L(ray.origin - c.p);
  F k = c.r / c.h;
  k = k * k;
  const V3 d = ray.dir, o = ray.origin;
  const F a = d.x * d.x + d.y * d.y - k * d.z * d.z;
  const F b = F(2.0f) * (d.x * o.x + d.y * o.y - k * d.z * (o.z - c.h));
  const F cc = o.x * o.x + o.y * o.y - k * (o.z - c.h) * (o.z - c.h);
  F t1 = F(0.0f), t2 = F(0.0f), t;
  if (!quadratic(a, b, cc, t1, t2)) return result;
  if (t2 < F(-kEps)) return result;
  t = t1;
  if (t1 < F(kEps)) t = t2;
  V3 hit = o + t * d;
  if (hit.z < F(-kEps) || hit.z > c.h) {
    if (t == t2) return result;
    t = t2;
    hit = o + t * d;
    if (hit.z < F(-kEps) || hit.z > c.h) return result;
  }
  if (t >= F(kMaxDistance)) return result;
  const F phi = phiOf(hit.y, hit.x);
  const F u = phi / (F(2.0f) * F(kPI));
  const F v = hit.z / c.h;
  result.d = t;
  {  // computeDpDForCone :31-36
    const F vv = hit.z / c.h;
    result.dpdu = dpduRot(hit);
    result.dpdv = v3(-hit.x / (F(1.0f) - vv), -hit.y / (F(1.0f) - vv), c.h);
  }
  return finishLocal(result, hit, v2(u, v), c.matIndex, c.texIndex, c.emission, c.p);
}
static Intersect intersectCylinder(Ray ray, const ConeCyl& c) {  // cylinder.glsl:40-90
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  ray.dir = W2L(ray.dir);
  ray.origin = W2L(ray.origin - c.p);
  const V3 d = ray.dir, o = ray.origin;
  const F a = d.x * d.x + d.y * d.y;
  const F b = F(2.0f) * (d.x * o.x + d.y * o.y);
  const F cc = o.x * o.x + o.y * o.y - c.r * c.r;
  F t1 = F(0.0f), t2 = F(0.0f), t;
  if (!quadratic(a, b, cc, t1, t2)) return result;
  if (t2 < F(-kEps)) return result;
  t = t1;
  if (t1 < F(kEps)) t = t2;
  V3 hit = o + t * d;
  if (hit.z < F(-kEps) || hit.z > c.h) {
    if (t == t2) return result;
    t = t2;
    hit = o + t * d;
    if (hit.z < F(-kEps) || hit.z > c.h) return result;
  }
  if (t >= F(kMaxDistance)) return result;
  const F phi = phiOf(hit.y, hit.x);
  const F u = phi / (F(2.0f) * F(kPI));
  const F v = hit.z / c.h;
  result.d = t;
  result.dpdu = dpduRot(hit);                      // computeDpDForCylinder :31-34
  result.dpdv = v3(F(0.0f), F(0.0f), c.h);
  return finishLocal(result, hit, v2(u, v), c.matIndex, c.texIndex, c.emission, c.p);
}

// ---- disk.glsl -----------------------------------------------------------------------------------------
struct Disk { V3 p; F r, innerR, matIndex, texIndex; V3 emission; bool reverseNormal; };
static Disk parseDisk(F index) {  // :15-25
  const Tex& o = C.objects; Disk k;
  k.p = readVec3(o, 1.0f, index, kObjLen);
  k.r = readFloat(o, 4.0f, index, kObjLen);
  k.innerR = readFloat(o, 5.0f, index, kObjLen);
  k.reverseNormal = readBool(o, 6.0f, index, kObjLen);
  k.matIndex = matCoord(readFloat(o, 7.0f, index, kObjLen));
  k.texIndex = matCoord(readFloat(o, 8.0f, index, kObjLen));
  k.emission = readVec3(o, 9.0f, index, kObjLen);
  return k;
}
static V3 normalForDisk(V3 hit, const Disk& k) { (void)hit; return sgn(k.reverseNormal) * v3(F(0.0f), F(1.0f), F(0.0f)); }
static Intersect intersectDisk(Ray ray, const Disk& k) {  // :36-75
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  ray.dir = W2L(ray.dir);
  ray.origin = W2L(ray.origin - k.p);
  if (ray.dir.z == F(0.0f)) return result;
  const F t = -ray.origin.z / ray.dir.z;
  if (t <= F(0.0f)) return result;
  const V3 hit = ray.origin + t * ray.dir;
  const F dist2 = hit.x * hit.x + hit.y * hit.y;
  if (dist2 > k.r * k.r || dist2 < k.innerR * k.innerR) return result;
  if (t >= F(kMaxDistance)) return result;
  const F phi = phiOf(hit.y, hit.x);
  const F u = phi / (F(2.0f) * F(kPI));
  const F rHit = sqrt_(dist2);
  const F oneMinusV = ((rHit - k.innerR) / (k.r - k.innerR));
  const F v = F(1.0f) - oneMinusV;
  result.d = t;
  result.dpdu = dpduRot(hit);                                                       // computeDpDForDisk :27-30
  result.dpdv = v3(hit.x, hit.y, F(0.0f)) * (k.innerR - k.r) / sqrt_(dist2);
  return finishLocal(result, hit, v2(u, v), k.matIndex, k.texIndex, k.emission, k.p);
}
static V3 sampleDisk(V2 u, const Disk& k, F& pdf) {  // :77-83
  const V2 pd = concentricSampleDisk(u);
  const V3 p = v3(pd.x * k.r + k.p.x, k.p.y, pd.y * k.r + k.p.z);
  const F area = F(2.0f) * F(kPI) * F(0.5f) * (k.r * k.r - k.innerR * k.innerR);
  pdf = F(1.0f) / area;
  return p;
}

// ---- hyperboloid.glsl ----------------------------------------------------------------------------------
struct Hyp { V3 p, p1, p2; F ah, ch, matIndex, texIndex; V3 emission; bool reverseNormal; };
static Hyp parseHyperboloid(F index) {  // :26-39
  const Tex& o = C.objects; Hyp h;
  h.p = readVec3(o, 1.0f, index, kObjLen);
  h.p1 = readVec3(o, 4.0f, index, kObjLen);
  h.p2 = readVec3(o, 7.0f, index, kObjLen);
  h.ah = readFloat(o, 10.0f, index, kObjLen);
  h.ch = readFloat(o, 11.0f, index, kObjLen);
  h.reverseNormal = readBool(o, 12.0f, index, kObjLen);
  h.matIndex = matCoord(readFloat(o, 13.0f, index, kObjLen));
  h.texIndex = matCoord(readFloat(o, 14.0f, index, kObjLen));
  h.emission = readVec3(o, 15.0f, index, kObjLen);
  return h;
}
static bool testBoundboxForHyperboloid(const Ray& ray, const Hyp& h) {  // :13-24
  const F r1 = sqrt_(h.p1.x * h.p1.x + h.p1.y * h.p1.y);
  const F r2 = sqrt_(h.p2.x * h.p2.x + h.p2.y * h.p2.y);
  const F rMax = fmax_(r1, r2);
  const F zMin = fmin_(h.p1.z, h.p2.z), zMax = fmax_(h.p1.z, h.p2.z);
  return testBoundbox(ray, BB(h.p - v3(rMax, -zMin, rMax), h.p + v3(rMax, zMax, rMax)));
}
static void computeDpDForHyperboloid(V3 hit, V3 p1, V3 p2, F phi, V3& dpdu, V3& dpdv) {  // :41-46
  const F sinPhi = sin_(phi), cosPhi = cos_(phi);
  dpdu = dpduRot(hit);
  dpdv = v3((p2.x - p1.x) * cosPhi - (p2.y - p1.y) * sinPhi, (p2.x - p1.x) * sinPhi + (p2.y - p1.y) * cosPhi,
            p2.z - p1.z);
}
static V3 normalForHyperboloid(V3 hit, const Hyp& h) {  // :48-58
  const F v = (hit.z - h.p1.z) / (h.p2.z - h.p1.z);
  const V3 pr = (F(1.0f) - v) * h.p1 + v * h.p2;
  const F phi = phiOf(pr.x * hit.y - hit.x * pr.y, hit.x * pr.x + hit.y * pr.y);
  V3 dpdu, dpdv;
  computeDpDForHyperboloid(hit, h.p1, h.p2, phi, dpdu, dpdv);
  const V3 normal = L2W(normalize(cross(dpdu, dpdv)));
  return sgn(h.reverseNormal) * normal;
}
static Intersect intersectHyperboloid(Ray ray, const Hyp& h) {  // :60-111
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  ray.dir = W2L(ray.dir);
  ray.origin = W2L(ray.origin - h.p);
  const V3 d = ray.dir, o = ray.origin;
  const F a = h.ah * d.x * d.x + h.ah * d.y * d.y - h.ch * d.z * d.z;
  const F b = F(2.0f) * (h.ah * d.x * o.x + h.ah * d.y * o.y - h.ch * d.z * o.z);
  const F c = h.ah * o.x * o.x + h.ah * o.y * o.y - h.ch * o.z * o.z - F(1.0f);
  F t1 = F(0.0f), t2 = F(0.0f), t;
  if (!quadratic(a, b, c, t1, t2)) return result;
  if (t2 < F(-kEps)) return result;
  t = t1;
  if (t1 < F(kEps)) t = t2;
  V3 hit = o + t * d;
  const F zMin = fmin_(h.p1.z, h.p2.z), zMax = fmax_(h.p1.z, h.p2.z);
  if (hit.z < zMin || hit.z > zMax) {
    if (t == t2) return result;
    t = t2;
    hit = o + t * d;
    if (hit.z < zMin || hit.z > zMax) return result;
  }
  if (t >= F(kMaxDistance)) return result;
  const F v = (hit.z - h.p1.z) / (h.p2.z - h.p1.z);
  const V3 pr = (F(1.0f) - v) * h.p1 + v * h.p2;
  const F phi = phiOf(pr.x * hit.y - hit.x * pr.y, hit.x * pr.x + hit.y * pr.y);
  const F u = phi / (F(2.0f) * F(kPI));
  result.d = t;
  computeDpDForHyperboloid(hit, h.p1, h.p2, phi, result.dpdu, result.dpdv);
  return finishLocal(result, hit, v2(u, v), h.matIndex, h.texIndex, h.emission, h.p);
}

// ---- paraboloid.glsl -----------------------------------------------------------------------------------
struct Para { V3 p; F z0, z1, r, matIndex, texIndex; V3 emission; bool reverseNormal; };
static Para parseParaboloid(F index) {  // :22-33
  const Tex& o = C.objects; Para q;
  q.p = readVec3(o, 1.0f, index, kObjLen);
  q.z0 = readFloat(o, 4.0f, index, kObjLen);
  q.z1 = readFloat(o, 5.0f, index, kObjLen);
  q.r = readFloat(o, 6.0f, index, kObjLen);
  q.reverseNormal = readBool(o, 7.0f, index, kObjLen);
  q.matIndex = matCoord(readFloat(o, 8.0f, index, kObjLen));
  q.texIndex = matCoord(readFloat(o, 9.0f, index, kObjLen));
  q.emission = readVec3(o, 10.0f, index, kObjLen);
  return q;
}
static bool testBoundboxForParaboloid(const Ray& ray, const Para& q) {  // :12-20
  const F zMin = fmin_(q.z0, q.z1), zMax = fmax_(q.z0, q.z1);
  return testBoundbox(ray, BB(q.p - v3(q.r, -zMin, q.r), q.p + v3(q.r, zMax, q.r)));
}
static void computeDpDForParaboloid(V3 hit, F zMax, F zMin, V3& dpdu, V3& dpdv) {  // :35-40
  dpdu = dpduRot(hit);
  dpdv = (zMax - zMin) * v3(hit.x / (F(2.0f) * hit.z), hit.y / (F(2.0f) * hit.z), F(1.0f));
}
static V3 normalForParaboloid(V3 hit, const Para& q) {  // :42-49
  const F zMin = fmin_(q.z0, q.z1), zMax = fmax_(q.z0, q.z1);
  V3 dpdu, dpdv;
  computeDpDForParaboloid(hit, zMax, zMin, dpdu, dpdv);
  const V3 normal = L2W(normalize(cross(dpdu, dpdv)));
  return sgn(q.reverseNormal) * normal;
}
static Intersect intersectParaboloid(Ray ray, const Para& q) {  // :51-103
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  ray.dir = W2L(ray.dir);
  ray.origin = W2L(ray.origin - q.p);
  const F zMin = fmin_(q.z0, q.z1), zMax = fmax_(q.z0, q.z1);
  const F k = zMax / (q.r * q.r);
  const V3 d = ray.dir, o = ray.origin;
  const F a = k * (d.x * d.x + d.y * d.y);
  const F b = F(2.0f) * k * (d.x * o.x + d.y * o.y) - d.z;
  const F c = k * (o.x * o.x + o.y * o.y) - o.z;
  F t1 = F(0.0f), t2 = F(0.0f), t;
  if (!quadratic(a, b, c, t1, t2)) return result;
  if (t2 < F(-kEps)) return result;
  t = t1;
  if (t1 < F(kEps)) t = t2;
  V3 hit = o + t * d;
  if (hit.z < zMin || hit.z > zMax) {
    if (t == t2) return result;
    t = t2;
    hit = o + t * d;
    if (hit.z < zMin || hit.z > zMax) return result;
  }
  if (t >= F(kMaxDistance)) return result;
  const F phi = phiOf(hit.y, hit.x);
  const F u = phi / (F(2.0f) * F(kPI));
  const F v = (hit.z - zMin) / (zMax - zMin);
  result.d = t;
  computeDpDForParaboloid(hit, zMax, zMin, result.dpdu, result.dpdv);
  return finishLocal(result, hit, v2(u, v), q.matIndex, q.texIndex, q.emission, q.p);
}

// ---- cornellbox.glsl ------------------------------------------------------------------------------------
struct Cornell { V3 min, max; F matIndex; bool reverseNormal; V3 emission; };
static Cornell parseCornellbox(F index) {  // :13-21 (matIndex read from slot 7 = reverseNormal: bug kept)
  const Tex& o = C.objects; Cornell b;
  b.min = readVec3(o, 1.0f, index, kObjLen);
  b.max = readVec3(o, 4.0f, index, kObjLen);
  b.matIndex = matCoord(readFloat(o, 7.0f, index, kObjLen));
  b.reverseNormal = false;
  b.emission = BLACKv;
  return b;
}
static V3 getCornellboxColor(V3 hit, V3 mn, V3 mx) {  // :23-37
  if (hit.x < mn.x + F(0.0001f)) return v3(F(0.25f), F(0.75f), F(0.25f));
  else if (hit.x > mx.x - F(0.0001f)) return v3(F(0.25f), F(0.25f), F(0.75f));
  else if (hit.y < mn.y + F(0.0001f)) return WHITEv;
  else if (hit.y > mx.y - F(0.0001f)) return WHITEv;
  else if (hit.z > mn.z + F(0.0001f)) return WHITEv;
  return BLACKv;
}
static V3 normalForCornellbox(V3 hit, const Cornell& b) {  // :39-51
  if (hit.x < b.min.x + F(0.0001f)) return v3(F(-1.0f), F(0.0f), F(0.0f));
  else if (hit.x > b.max.x - F(0.0001f)) return v3(F(1.0f), F(0.0f), F(0.0f));
  else if (hit.y < b.min.y + F(0.0001f)) return v3(F(0.0f), F(-1.0f), F(0.0f));
  else if (hit.y > b.max.y - F(0.0001f)) return v3(F(0.0f), F(1.0f), F(0.0f));
  else if (hit.z < b.min.z + F(0.0001f)) return v3(F(0.0f), F(0.0f), F(-1.0f));
  return v3(F(0.0f), F(0.0f), F(1.0f));
}
static Intersect intersectCornellbox(const Ray& ray, const Cornell& b) {  // :67-90
  Intersect result = zeroIns();
  result.d = F(kMaxDistance);
  const V3 tMin = (b.min - ray.origin) / ray.dir;
  const V3 tMax = (b.max - ray.origin) / ray.dir;
  const V3 t1 = vmin(tMin, tMax), t2 = vmax(tMin, tMax);
  const F tNear = fmax_(fmax_(t1.x, t1.y), t1.z);
  const F tFar = fmin_(fmin_(t2.x, t2.y), t2.z);
  F t = F(-1.0f);
  if (tNear < tFar) t = tFar;
  if (t > F(kEps)) {
    result.d = t;
    result.hit = ray.origin + t * ray.dir;
    result.normal = -normalForCornellbox(ray.origin + t * ray.dir, b);
    computeDpDForBox(result.normal, result.dpdu, result.dpdv);
    result.matIndex = b.matIndex;
    result.sc = getCornellboxColor(result.hit, b.min, b.max);
    result.emission = BLACKv;
  }
  return result;
}

// ---- intersectObjects (generated, shader.shape.js:28-51) ------------------------------------------------
static Intersect intersectObjects(const Ray& ray) {
  Intersect ins = zeroIns();
  ins.d = F(kMaxDistance);
  for (int i = 0; i < C.n; i++) {
    Intersect tmp = zeroIns();
    tmp.d = F(kMaxDistance);
    const F row = rowCoord(i, C.n);
    const int category = toint(fetch(C.objects, 0.0f, raw(row)));
    if (category >= 0 && category < 32 && ((C.shapeMask >> category) & 1u)) {
      bool rev = false;
      switch (category) {
        case CUBE: { const Cube x = parseCube(row); rev = x.reverseNormal; tmp = intersectCube(ray, x); break; }
        case SPHERE: {
          const Sphere x = parseSphere(row); rev = x.reverseNormal;
          if (!testBoundboxForSphere(ray, x)) continue;
          tmp = intersectSphere(ray, x); break;
        }
        case RECTANGLE: { const Rect x = parseRectangle(row); rev = x.reverseNormal; tmp = intersectRectangle(ray, x); break; }
        case CONE: {
          const ConeCyl x = parseConeCyl(row); rev = x.reverseNormal;
          if (!testBoundboxForConeCyl(ray, x)) continue;
          tmp = intersectCone(ray, x); break;
        }
        case CYLINDER: {
          const ConeCyl x = parseConeCyl(row); rev = x.reverseNormal;
          if (!testBoundboxForConeCyl(ray, x)) continue;
          tmp = intersectCylinder(ray, x); break;
        }
        case DISK: { const Disk x = parseDisk(row); rev = x.reverseNormal; tmp = intersectDisk(ray, x); break; }
        case HYPERBOLOID: {
          const Hyp x = parseHyperboloid(row); rev = x.reverseNormal;
          if (!testBoundboxForHyperboloid(ray, x)) continue;
          tmp = intersectHyperboloid(ray, x); break;
        }
        case PARABOLOID: {
          const Para x = parseParaboloid(row); rev = x.reverseNormal;
          if (!testBoundboxForParaboloid(ray, x)) continue;
          tmp = intersectParaboloid(ray, x); break;
        }
        case CORNELLBOX: { const Cornell x = parseCornellbox(row); rev = x.reverseNormal; tmp = intersectCornellbox(ray, x); break; }
        default: break;
      }
      const V3 nn = sgn(rev) * tmp.normal;
      const bool faceObj = dot(nn, ray.dir) < F(-kEps);
      tmp.emission = faceObj ? tmp.emission : BLACKv;
      tmp.index = i;
    }
    if (tmp.d < ins.d) ins = tmp;
  }
  ins.matCategory = readInt(C.texParams, 0.0f, ins.matIndex, kTexLen);
  ins.into = dot(ins.normal, ray.dir) < F(-kEps);
  if (!ins.into) ins.normal = -ins.normal;
  return ins;
}

// ---- sampleGeometry (generated, shader.shape.js:53-67) ---------------------------------------------------
static V3 sampleGeometry(V2 u, int i, V3& normal, F& pdf) {
  normal = BLACKv;
  pdf = F(0.0f);
  const F row = rowCoord(i, C.n);
  const int category = toint(fetch(C.objects, 0.0f, raw(row)));
  V3 result = BLACKv;
  if (!(category >= 0 && category < 32 && ((C.shapeMask >> category) & 1u))) return result;
  switch (category) {  // sampleX that never write pdf leave it 0 (unwritten out parameter)
    case CUBE: { const Cube x = parseCube(row); result = BLACKv; pdf = F(0.0f); normal = normalForCube(result, x); break; }
    case SPHERE: { const Sphere x = parseSphere(row); result = sampleSphere(u, x, pdf); normal = normalForSphere(result, x); break; }
    case RECTANGLE: { const Rect x = parseRectangle(row); result = sampleRectangle(u, x, pdf); normal = normalForRectangle(result, x); break; }
    case CONE: { const ConeCyl x = parseConeCyl(row); result = BLACKv; pdf = F(0.0f); normal = normalForCone(result, x); break; }
    case CYLINDER: { const ConeCyl x = parseConeCyl(row); result = BLACKv; pdf = F(0.0f); normal = normalForCylinder(result, x); break; }
    case DISK: { const Disk x = parseDisk(row); result = sampleDisk(u, x, pdf); normal = normalForDisk(result, x); break; }
    case HYPERBOLOID: { const Hyp x = parseHyperboloid(row); result = BLACKv; pdf = F(0.0f); normal = normalForHyperboloid(result, x); break; }
    case PARABOLOID: { const Para x = parseParaboloid(row); result = BLACKv; pdf = F(0.0f); normal = normalForParaboloid(result, x); break; }
    case CORNELLBOX: { const Cornell x = parseCornellbox(row); result = BLACKv; pdf = F(0.0f); normal = normalForCornellbox(result, x); break; }
    default: break;
  }
  return result;
}

// ---- ssutility.glsl ---------------------------------------------------------------------------------------
static inline F cosTheta(V3 w) { return w.z; }
static inline F cos2Theta(V3 w) { return w.z * w.z; }
static inline F absCosTheta(V3 w) { return abs_(w.z); }
static inline F sin2Theta(V3 w) { return fmax_(F(0.0f), F(1.0f) - cos2Theta(w)); }
static inline F sinTheta(V3 w) { return sqrt_(sin2Theta(w)); }
static inline F tan2Theta(V3 w) {
  const F cos2T = cos2Theta(w);
  if (cos2T < F(kEps)) return F(kInf);
  return sin2Theta(w) / cos2T;
}
static inline F cosPhi(V3 w) {
  const F st = sinTheta(w);
  return equalZero(st) ? F(1.0f) : clamp_(w.x / st, F(-1.0f), F(1.0f));
}
static inline F sinPhi(V3 w) {
  const F st = sinTheta(w);
  return equalZero(st) ? F(0.0f) : clamp_(w.y / st, F(-1.0f), F(1.0f));
}
static inline F cos2Phi(V3 w) { return cosPhi(w) * cosPhi(w); }
static inline F sin2Phi(V3 w) { return sinPhi(w) * sinPhi(w); }
static inline bool sameHemisphere(V3 w, V3 wp) { return w.z * wp.z > F(kEps); }

// ---- fresnel.glsl -----------------------------------------------------------------------------------------
struct Fresnel { int type; V3 etaI, etaT, k; };
static inline Fresnel fresnelD(F etaI, F etaT) { Fresnel f{}; f.etaI = v3s(etaI); f.etaT = v3s(etaT); f.type = F_DIELECTRIC; return f; }
static inline Fresnel fresnelC(V3 etaI, V3 etaT, V3 k) { Fresnel f; f.etaI = etaI; f.etaT = etaT; f.k = k; f.type = F_CONDUCTOR; return f; }
static inline Fresnel fresnelN() { Fresnel f{}; f.type = F_NOOP; return f; }
static F frDielectric(F cosThetaI, F etaI, F etaT) {  // :31-46
  cosThetaI = clamp_(cosThetaI, F(-1.0f), F(1.0f));
  const F sinThetaI = sqrt_(fmax_(F(0.0f), F(1.0f) - cosThetaI * cosThetaI));
  const F sinThetaT = etaI / etaT * sinThetaI;
  if (sinThetaT >= F(1.0f)) return F(1.0f);
  const F cosThetaT = sqrt_(fmax_(F(0.0f), F(1.0f) - sinThetaT * sinThetaT));
  const F TI = etaT * cosThetaI, IT = etaI * cosThetaT, II = etaI * cosThetaI, TT = etaT * cosThetaT;
  const F Rparl = (TI - IT) / (TI + IT);
  const F Rperp = (II - TT) / (II + TT);
  return (Rparl * Rparl + Rperp * Rperp) / F(2.0f);
}
static V3 frConductor(F cosThetaI, V3 etaI, V3 etaT, V3 k) {  // :48-70
  cosThetaI = clamp_(cosThetaI, F(-1.0f), F(1.0f));
  const V3 eta = etaT / etaI, etak = k / etaI;
  const F cosThetaI2 = cosThetaI * cosThetaI;
  const F sinThetaI2 = F(1.0f) - cosThetaI2;
  const V3 eta2 = eta * eta, etak2 = etak * etak;
  const V3 t0 = eta2 - etak2 - sinThetaI2;
  const V3 s = t0 * t0 + F(4.0f) * eta2 * etak2;
  const V3 a2plusb2 = v3(sqrt_(s.x), sqrt_(s.y), sqrt_(s.z));
  const V3 t1 = a2plusb2 + cosThetaI2;
  const V3 ah = F(0.5f) * (a2plusb2 + t0);
  const V3 a = v3(sqrt_(ah.x), sqrt_(ah.y), sqrt_(ah.z));
  const V3 t2 = F(2.0f) * cosThetaI * a;
  const V3 Rs = (t1 - t2) / (t1 + t2);
  const V3 t3 = cosThetaI2 * a2plusb2 + v3s(sinThetaI2 * sinThetaI2);
  const V3 t4 = t2 * sinThetaI2;
  const V3 Rp = Rs * (t3 - t4) / (t3 + t4);
  return F(0.5f) * (Rp + Rs);
}
static V3 frEvaluate(const Fresnel& f, F cosThetaI) {  // :72-77
  if (f.type == F_DIELECTRIC) return WHITEv * frDielectric(cosThetaI, f.etaI.x, f.etaT.x);
  else if (f.type == F_CONDUCTOR) return frConductor(cosThetaI, f.etaI, f.etaT, f.k);
  return WHITEv;
}

// ---- microfacet.glsl (TrowbridgeReitz only: Beckmann is never selected, SURVEY a.5) ---------------------
struct MD { F ax, ay; };
static V3 trSampleWh(V2 u, F ax, F ay, V3 wo) {  // :41-59
  F cosT = F(0.0f), phi = F(2.0f) * F(kPI) * u.x;
  if (ax == ay) {
    const F tanTheta2 = ax * ax * u.x / (F(1.0f) - u.x);
    cosT = F(1.0f) / sqrt_(F(1.0f) + tanTheta2);
  } else {
    phi = atan_(ay / ax * tan_(F(kPiOver2) + F(2.0f) * F(kPI) * u.x));
    if (u.x > F(0.5f)) phi += F(kPI);
    const F sP = sin_(phi), cP = cos_(phi);
    const F ax2 = ax * ax, ay2 = ay * ay;
    const F alpha2 = F(1.0f) / (cP * cP / ax2 + sP * sP / ay2);
    const F tanTheta2 = alpha2 * u.x / (F(1.0f) - u.x);
    cosT = F(1.0f) / sqrt_(F(1.0f) + tanTheta2);
  }
  const F sinT = sqrt_(fmax_(F(0.0f), F(1.0f) - cosT * cosT));
  V3 wh = sphericalDirection(sinT, cosT, phi);
  if (!sameHemisphere(wo, wh)) wh = -wh;
  return wh;
}
static F trD(F ax, F ay, V3 wh) {  // :61-67
  const F t2 = tan2Theta(wh);
  if (t2 >= F(kInf)) return F(0.001f);
  const F cos4Theta = cos2Theta(wh) * cos2Theta(wh);
  const F e = (cos2Phi(wh) / (ax * ax) + sin2Phi(wh) / (ay * ay)) * t2;
  return F(1.0f) / (F(kPI) * ax * ay * cos4Theta * (F(1.0f) + e) * (F(1.0f) + e));
}
static inline F trPdf(F ax, F ay, V3 wo, V3 wh) { (void)wo; return trD(ax, ay, wh) * absCosTheta(wh); }  // :69-71

// ---- bsdf.glsl ------------------------------------------------------------------------------------------
static V3 orenNayar_f(V3 R, F A, F B, V3 wo, V3 wi) {  // :45-66
  const F sinThetaI = sinTheta(wi), sinThetaO = sinTheta(wo);
  F maxCos = F(0.0f);
  if (sinThetaI > F(kEps) && sinThetaO > F(kEps)) {
    const F sinPhiI = sinPhi(wi), cosPhiI = cosPhi(wi);
    const F sinPhiO = sinPhi(wo), cosPhiO = cosPhi(wo);
    const F dCos = cosPhiI * cosPhiO + sinPhiI * sinPhiO;
    maxCos = fmax_(F(0.0f), dCos);
  }
  F sinAlpha, tanBeta;
  if (absCosTheta(wi) > absCosTheta(wo)) { sinAlpha = sinThetaO; tanBeta = sinThetaI / absCosTheta(wi); }
  else { sinAlpha = sinThetaI; tanBeta = sinThetaO / absCosTheta(wo); }
  return R * F(kInvPI) * (A + B * maxCos * sinAlpha * tanBeta);
}
struct MicroR { V3 R; Fresnel f; MD md; };
static V3 microfacet_r_f(const MicroR& mr, V3 wo, V3 wi) {  // :168-178
  const F cosThetaO = absCosTheta(wo), cosThetaI = absCosTheta(wi);
  V3 wh = wi + wo;
  if (cosThetaI < F(kEps) || cosThetaO < F(kEps)) return BLACKv * F(0.001f);
  if (equalZero(wh.x) && equalZero(wh.y) && equalZero(wh.z)) return BLACKv * F(0.001f);
  wh = normalize(wh);
  const V3 Fr = frEvaluate(mr.f, dot(wi, wh));
  return mr.R * trD(mr.md.ax, mr.md.ay, wh) * Fr / (F(4.0f) * cosThetaI * cosThetaO);
}
static V3 microfacet_r_sample_f(const MicroR& mr, V2 u, V3 wo, V3& wi, F& pdf) {  // :186-196
  if (wo.z < F(kEps)) return BLACKv * F(0.001f);
  const V3 wh = trSampleWh(u, mr.md.ax, mr.md.ay, wo);
  wi = reflect_(-wo, wh);
  if (!sameHemisphere(wo, wi)) return BLACKv * F(0.001f);
  pdf = trPdf(mr.md.ax, mr.md.ay, wo, wh) / (F(4.0f) * dot(wo, wh));
  return microfacet_r_f(mr, wo, wi);
}
struct MicroT { V3 T; F etaA, etaB; bool into; MD md; };
static V3 microfacet_t_f(const MicroT& mt, V3 wo, V3 wi) {  // :205-224
  if (sameHemisphere(wo, wi)) return BLACKv * F(0.001f);
  const F cosThetaO = cosTheta(wo), cosThetaI = cosTheta(wi);
  if (equalZero(cosThetaI) || equalZero(cosThetaO)) return BLACKv * F(0.001f);
  const F eta = mt.into ? (mt.etaB / mt.etaA) : (mt.etaA / mt.etaB);
  V3 wh = normalize(wo + wi * eta);
  if (wh.z < F(-kEps)) wh = -wh;
  const F Fd = frDielectric(dot(wo, wh), mt.etaA, mt.etaB);
  const F sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
  return (F(1.0f) - Fd) * mt.T *
         abs_(eta * eta * trD(mt.md.ax, mt.md.ay, wh) * abs_(dot(wi, wh)) * abs_(dot(wo, wh)) /
              (cosThetaI * cosThetaO * sqrtDenom * sqrtDenom));
}
static F microfacet_t_pdf(const MicroT& mt, V3 wo, V3 wi) {  // :226-235
  if (sameHemisphere(wo, wi)) return F(0.001f);
  const F eta = mt.into ? (mt.etaB / mt.etaA) : (mt.etaA / mt.etaB);
  const V3 wh = normalize(wo + wi * eta);
  const F sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
  const F dwh_dwi = abs_((eta * eta * dot(wi, wh)) / (sqrtDenom * sqrtDenom));
  return trPdf(mt.md.ax, mt.md.ay, wo, wh) * dwh_dwi;
}
static V3 microfacet_t_sample_f(const MicroT& mt, V2 u, V3 wo, V3& wi, F& pdf) {  // :237-244
  if (equalZero(wo.z)) return BLACKv * F(0.001f);
  const V3 wh = trSampleWh(u, mt.md.ax, mt.md.ay, wo);
  const F eta = mt.into ? (mt.etaA / mt.etaB) : (mt.etaB / mt.etaA);
  wi = refract_(-wo, wh, eta);
  pdf = microfacet_t_pdf(mt, wo, wi);
  return microfacet_t_f(mt, wo, wi);
}

// ---- material plugins (shader.material.js:21-29 + material/*.glsl) --------------------------------------
// Each plugin's `out vec3 wi` and local `float pdf` start at 0 (defined meaning of unwritten outs).
static V3 matte(V2 u, F matIndex, V3 sc, V3 wo, V3& wi, bool into, V3* f_out) {  // matte.glsl:8-37
  (void)into;
  const Tex& tp = C.texParams;
  const F kd = readFloat(tp, 1.0f, matIndex, kTexLen), sigma = readFloat(tp, 2.0f, matIndex, kTexLen);
  const F A = readFloat(tp, 3.0f, matIndex, kTexLen), B = readFloat(tp, 4.0f, matIndex, kTexLen);
  V3 f; F pdf = F(0.0f);
  wi = BLACKv;
  if (sigma < F(kEps)) {
    const V3 R = kd * sc;
    wi = cosineSampleHemisphere(u);                                   // lambertian_r_sample_f bsdf.glsl:15-19
    pdf = sameHemisphere(wo, wi) ? absCosTheta(wi) * F(kInvPI) : F(0.0f);
    f = R * F(kInvPI);
  } else {
    const V3 R = kd * sc;
    wi = cosineSampleHemisphere(u);                                   // orenNayar_sample_f bsdf.glsl:72-76
    pdf = sameHemisphere(wo, wi) ? absCosTheta(wi) * F(kInvPI) : F(0.0f);
    f = orenNayar_f(R, A, B, wo, wi);
  }
  const V3 fpdf = f * absCosTheta(wi) / pdf;
  // matte_f (:26-37)
  if (sigma < F(kEps)) *f_out = (kd * sc) * F(kInvPI);
  else *f_out = orenNayar_f(kd * sc, A, B, wo, wi);
  return fpdf;
}
static V3 mirror(V2 u, F matIndex, V3 sc, V3 wo, V3& wi, bool into) {  // mirror.glsl:5-17
  (void)u; (void)into;
  const F kr = readFloat(C.texParams, 1.0f, matIndex, kTexLen);
  const V3 R = kr * sc;
  wi = v3(-wo.x, -wo.y, wo.z);                                        // specular_r_sample_f bsdf.glsl:93-98
  const F pdf = F(1.0f);
  const V3 f = frEvaluate(fresnelN(), cosTheta(wi)) * R / absCosTheta(wi);
  return f * absCosTheta(wi) / pdf;
}
static V3 metal(V2 u, F matIndex, V3 sc, V3 wo, V3& wi, bool into) {  // metal.glsl:8-22
  (void)into;
  const Tex& tp = C.texParams;
  const F ur = readFloat(tp, 1.0f, matIndex, kTexLen), vr = readFloat(tp, 2.0f, matIndex, kTexLen);
  const V3 eta = readVec3(tp, 3.0f, matIndex, kTexLen), k = readVec3(tp, 6.0f, matIndex, kTexLen);
  MicroR mr; mr.R = sc; mr.f = fresnelC(WHITEv, eta, k); mr.md.ax = ur; mr.md.ay = vr;
  F pdf = F(0.0f);
  wi = BLACKv;
  const V3 f = microfacet_r_sample_f(mr, u, wo, wi, pdf);
  return f * absCosTheta(wi) / pdf;
}
static V3 glass(V2 u, F matIndex, V3 sc, V3 wo, V3& wi, bool into) {  // glass.glsl:10-36
  const Tex& tp = C.texParams;
  const F kr = readFloat(tp, 1.0f, matIndex, kTexLen), kt = readFloat(tp, 2.0f, matIndex, kTexLen);
  const F eta = readFloat(tp, 3.0f, matIndex, kTexLen);
  const F ur = readFloat(tp, 4.0f, matIndex, kTexLen), vr = readFloat(tp, 5.0f, matIndex, kTexLen);
  V3 f; F pdf = F(0.0f);
  wi = BLACKv;
  const bool isSpecular = ur < F(kEps) && vr < F(kEps);
  if (isSpecular) {  // specular_fr_sample_f bsdf.glsl:141-158 with SpecularFr(kr*sc, kt*sc, 1.0, eta, into)
    const V3 R = kr * sc, T = kt * sc;
    const F etaA = F(1.0f), etaB = eta;
    const F Fd = frDielectric(cosTheta(wo), etaA, etaB);
    if (u.x < Fd) {
      wi = v3(-wo.x, -wo.y, wo.z);
      pdf = F(1.0f);
      f = R / absCosTheta(wi);
    } else {
      const F etaI = into ? etaA : etaB, etaT = into ? etaB : etaA;
      wi = refract_(-wo, v3(F(0.0f), F(0.0f), F(1.0f)), etaI / etaT);
      const V3 ft = T * (F(1.0f) - Fd);
      pdf = F(1.0f);
      f = ft / absCosTheta(wi);
    }
  } else {
    MD md; md.ax = ur; md.ay = vr;
    const F p = u.x;
    u.x = fmin_(u.x * F(2.0f) - F(1.0f), F(kOneMinusEps));
    if (p < F(0.5f)) {
      MicroR mr; mr.R = kr * sc; mr.f = fresnelD(F(1.0f), eta); mr.md = md;
      f = microfacet_r_sample_f(mr, u, wo, wi, pdf);
    } else {
      MicroT mt; mt.T = kt * sc; mt.etaA = F(1.0f); mt.etaB = eta; mt.into = into; mt.md = md;
      f = microfacet_t_sample_f(mt, u, wo, wi, pdf);
    }
  }
  return f * absCosTheta(wi) / pdf;
}
static V3 material(const Intersect& ins, V3 wo, V3& wi, V3& f) {  // generated shader.material.js:21-29
  f = BLACKv;
  V3 fpdf = BLACKv;
  const int cat = ins.matCategory;
  if (!(cat >= 0 && cat < 32 && ((C.matMask >> cat) & 1u))) { wi = BLACKv; return fpdf; }
  const V2 u = random2(ins.seed);
  switch (cat) {
    case MATTE: fpdf = matte(u, ins.matIndex, ins.sc, wo, wi, ins.into, &f); break;
    case MIRROR: fpdf = mirror(u, ins.matIndex, ins.sc, wo, wi, ins.into); f = BLACKv; break;      // mirror_f = BLACK
    case METAL: fpdf = metal(u, ins.matIndex, ins.sc, wo, wi, ins.into); f = BLACKv; break;        // f unused off matte
    case GLASS: fpdf = glass(u, ins.matIndex, ins.sc, wo, wi, ins.into); f = BLACKv; break;        // f unused off matte
    default: break;
  }
  return fpdf;
}

// ---- lights (shader.light.js:12-31 + light/*.glsl) ---------------------------------------------------------
static bool testShadow(const Ray& ray) {  // shader.light.js:24-31
  const Intersect ins = intersectObjects(ray);
  return ins.d > F(kEps) && ins.d < F(kOneMinusEps);
}
static F falloff(F cosTotalWidth, F cosFalloffStart, V3 w) {  // spot.glsl:17-27
  const F cT = -w.y;
  if (cT < cosTotalWidth) return F(0.0f);
  if (cT >= cosFalloffStart) return F(1.0f);
  const F delta = (cT - cosTotalWidth) / (cosFalloffStart - cosTotalWidth);
  const F delta2 = delta * delta;
  return delta2 * delta2;
}
#ifdef SAIL_COUNT_OPS
// Live-op model (op-counting build only): a light sample whose contribution would be exactly +0 in every channel
// returns black whether or not its shadow ray is blocked, so that shadow test's ops are dead. The would-be
// contribution is evaluated here uncounted (the reference computes it only when unshadowed) and the test's ops
// are added to g_opsShadowDead.
static unsigned long long g_opsShadowDead = 0;
static uint32_t fbits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, sizeof u);
  return u;
}
static bool posZero3(V3 v) { return (fbits(raw(v.x)) | fbits(raw(v.y)) | fbits(raw(v.z))) == 0u; }
#define SHADOW_TEST(ray, would_expr)                                         \
  [&]() {                                                                    \
    const unsigned long long t0_ = g_ops;                                    \
    const bool sh_ = testShadow(ray);                                        \
    const unsigned long long testOps_ = g_ops - t0_, save_ = g_ops;          \
    const V3 would_ = (would_expr);                                          \
    g_ops = save_;                                                           \
    if (posZero3(would_)) g_opsShadowDead += testOps_;                       \
    return sh_;                                                              \
  }()
#else
#define SHADOW_TEST(ray, would_expr) testShadow(ray)
#endif
static V3 light_sample(const Intersect& ins) {
  V3 fpdf = BLACKv;
  const int index = randomInt(ins.seed, 0, C.ln);
  const int lightCategory = readInt(C.lights, 0.0f, F((float)index), kTexLen);  // integer row coordinate (bug kept)
  if (!(lightCategory >= 0 && lightCategory < 32 && ((C.lightMask >> lightCategory) & 1u))) return fpdf;
  const F row = rowCoord(index, C.ln);
  const Tex& L = C.lights;
  if (lightCategory == AREA) {  // area.glsl:6-23
    const int aindex = readInt(L, 1.0f, row, kLightLen);
    const V3 emission = readVec3(L, 2.0f, row, kLightLen);
    V3 normal; F pdf;
    const V3 p = sampleGeometry(random2(ins.seed), aindex, normal, pdf);
    const V3 toLight = p - ins.hit;
    const V3 normToLight = normalize(toLight);
    if (SHADOW_TEST(ray_(ins.hit, toLight),
                    emission * fmax_(F(0.0f), dot(normal, -normToLight)) * fmax_(F(0.0f), dot(normToLight, ins.normal)) / pdf))
      return BLACKv;
    fpdf = emission * fmax_(F(0.0f), dot(normal, -normToLight)) * fmax_(F(0.0f), dot(normToLight, ins.normal)) / pdf;
  } else if (lightCategory == POINT) {  // point.glsl:6-20
    const V3 from = readVec3(L, 1.0f, row, kLightLen), emission = readVec3(L, 4.0f, row, kLightLen);
    const V3 p = from + uniformSampleSphere(random2(ins.seed)) * F(0.1f);
    const V3 toLight = p - ins.hit;
    if (SHADOW_TEST(ray_(ins.hit, toLight), emission * fmax_(F(0.0f), dot(normalize(toLight), ins.normal)))) return BLACKv;
    fpdf = emission * fmax_(F(0.0f), dot(normalize(toLight), ins.normal));
  } else if (lightCategory == SPOT) {  // spot.glsl:8-39
    const F ctw = readFloat(L, 1.0f, row, kLightLen), cfs = readFloat(L, 2.0f, row, kLightLen);
    const V3 from = readVec3(L, 3.0f, row, kLightLen), emission = readVec3(L, 6.0f, row, kLightLen);
    const V3 toLight = from - ins.hit;
    if (SHADOW_TEST(ray_(ins.hit, toLight),
                    emission * falloff(ctw, cfs, -normalize(toLight)) * fmax_(F(0.0f), dot(normalize(toLight), ins.normal)) /
                        (length(toLight) * length(toLight))))
      return BLACKv;
    const V3 normToLight = normalize(toLight);
    const F d = length(toLight);
    fpdf = emission * falloff(ctw, cfs, -normToLight) * fmax_(F(0.0f), dot(normalize(toLight), ins.normal)) / (d * d);
  }
  return fpdf;
}

// ---- path.glsl ----------------------------------------------------------------------------------------------
static V3 shade(const Intersect& ins, V3 wo, V3& wi, V3& fpdf) {  // :1-14
  V3 f = BLACKv, direct = BLACKv;
  const V3 ss = normalize(ins.dpdu), ts = cross(ins.normal, ss);
  wo = worldToLocal(wo, ins.normal, ss, ts);
  wi = BLACKv;
  fpdf = vclamp(material(ins, wo, wi, f), BLACKv, WHITEv);
  wi = localToWorld(wi, ins.normal, ss, ts);
  if (veq(ins.emission, BLACKv) && ins.matCategory == MATTE) direct = direct + light_sample(ins) * f;
  return ins.emission + direct;
}
static unsigned long long g_segments = 0;
#ifdef SAIL_COUNT_OPS
// Live-op model (op-counting build only): after a path's last bounce only its radiance is read, so that bounce's
// throughput update, next ray, BSDF sample and material weight are dead. Its live ops are the radiance update
// e += (emission + direct) * fpdf and, on a lit matte surface, f (Lambert: (kd sc) / pi; Oren-Nayar: the shading
// frame, the hash and the cosine sample it needs) and the light sample with its shadow ray when the scene has
// lights. g_opsLastFull counts what the reference program does at the last bounce, g_opsLastLive the live part.
static unsigned long long g_opsLastFull = 0, g_opsLastLive = 0;
static void countLiveLast(const Intersect& ins, V3 woWorld, V3 fpdf) {
  V3 direct = BLACKv;
  if (veq(ins.emission, BLACKv) && ins.matCategory == MATTE && ((C.matMask >> MATTE) & 1u)) {
    const Tex& tp = C.texParams;
    const F kd = readFloat(tp, 1.0f, ins.matIndex, kTexLen), sigma = readFloat(tp, 2.0f, ins.matIndex, kTexLen);
    V3 f;
    if (sigma < F(kEps)) {
      f = (kd * ins.sc) * F(kInvPI);
    } else {
      const F A = readFloat(tp, 3.0f, ins.matIndex, kTexLen), B = readFloat(tp, 4.0f, ins.matIndex, kTexLen);
      const V3 ss = normalize(ins.dpdu), ts = cross(ins.normal, ss);
      const V3 wo = worldToLocal(woWorld, ins.normal, ss, ts);
      const V3 wi = cosineSampleHemisphere(random2(ins.seed));
      f = orenNayar_f(kd * ins.sc, A, B, wo, wi);
    }
    if (C.ln > 0 && C.lightMask != 0u) direct = direct + light_sample(ins) * f;
  }
  const V3 e = (ins.emission + direct) * fpdf;
  (void)e;
  OPC(3);  // the e + ... sum
}
#endif
static void trace(Ray ray, int maxDepth, V3& e, V3& n, V3& p) {  // :16-38
  V3 fpdf = WHITEv;
  e = BLACKv;
  int depth = 0;
  while (depth++ < maxDepth) {
    g_segments++;
    Intersect ins = intersectObjects(ray);
    ins.seed = C.timeSinceStart + F((float)depth);
    if (ins.d >= F(kMaxDistance)) break;
    if (depth == 1) { n = ins.normal; p = ins.hit; }
#ifdef SAIL_COUNT_OPS
    const bool last = depth == maxDepth;
    const unsigned long long before = g_ops;
    if (last) {  // count the live part on its own, then the reference's full bounce as usual
      countLiveLast(ins, -ray.dir, fpdf);
      g_opsLastLive += g_ops - before;
      g_ops = before;
    }
#endif
    V3 wi, _fpdf;
#ifdef SAIL_COUNT_OPS
    const unsigned long long shadowDead = g_opsShadowDead;  // the last bounce's full shading is not live-counted
#endif
    e = e + shade(ins, -ray.dir, wi, _fpdf) * fpdf;
#ifdef SAIL_COUNT_OPS
    if (last) g_opsShadowDead = shadowDead;
#endif
    fpdf = fpdf * _fpdf;
    const F outdot = dot(ins.normal, wi);
    ray.origin = ins.hit + ins.normal * (outdot > F(kEps) ? F(0.0001f) : F(-0.0001f));
    ray.dir = wi;
#ifdef SAIL_COUNT_OPS
    if (last) g_opsLastFull += g_ops - before;
#endif
  }
}

// ---- primary rays: vstrace.glsl:4-6 + the rasteriser's linear interpolation -----------------
// corner c: d_c = normalize((M*(c,0,1)).xyz/w - eye); v0=(-1,-1) v1=(-1,1) v2=(1,-1) v3=(1,1);
// fragment (x,y): s=(x+.5)/W, t=(y+.5)/H; tri0 (s+t<=1): d0+(d2-d0)s+(d1-d0)t; tri1: d3+(d1-d3)(1-s)+(d2-d3)(1-t)
static void cornerDirs(const float* M, const float* eye, V3 out[4]) {
  static const float cx[4] = {-1.0f, -1.0f, 1.0f, 1.0f}, cy[4] = {-1.0f, 1.0f, -1.0f, 1.0f};
  for (int c = 0; c < 4; c++) {
    float q[4];
    for (int r = 0; r < 4; r++) q[r] = M[0 * 4 + r] * cx[c] + M[1 * 4 + r] * cy[c] + M[2 * 4 + r] * 0.0f + M[3 * 4 + r] * 1.0f;
    const V3 w = v3(F(q[0]) / F(q[3]), F(q[1]) / F(q[3]), F(q[2]) / F(q[3]));  // ensure3byW, utility.glsl:11-13
    out[c] = normalize(w - v3(F(eye[0]), F(eye[1]), F(eye[2])));
  }
}
static V3 primaryDir(const V3 d[4], int x, int y, int W, int H) {
  const F s = F(((float)x + 0.5f) / (float)W), t = F(((float)y + 0.5f) / (float)H);
  if (raw(s) + raw(t) <= 1.0f) return d[0] + (d[2] - d[0]) * s + (d[1] - d[0]) * t;
  return d[3] + (d[1] - d[3]) * (F(1.0f) - s) + (d[2] - d[3]) * (F(1.0f) - t);
}

// ---- public oracle ABI (ctypes from tests/ and bench.py) -------------------------------------------------------
extern "C" {

enum { ACC_SUM = 0, ACC_MIX = 1, ACC_COMPAT8 = 2 };

static inline float q8(float v) {  // UNORM8 store + reload of a clamped value (GL round-to-nearest)
  v = refm::fmin_s(refm::fmax_s(v, 0.0f), 1.0f);
  return floorf(v * 255.0f + 0.5f) / 255.0f;
}

// Render samples k0..k0+spp-1 of the crop [x0,x0+cw)x[y0,y0+ch) of a W x H frame.
// accum: W*H*4 floats (row 0 = bottom). SUM: rgb += e, a += 1. MIX/COMPAT8: rgb = mix(e, rgb, k/(k+1)), a = 1.
// aov_n / aov_p (optional, W*H*4): n/2+0.5 and normalize(p) of the last sample (fstrace.glsl:15-16).
int oracle_render(const float* objects, int n, const float* texparams, int tn, const float* lights, int ln,
                  unsigned shape_mask, unsigned mat_mask, unsigned tex_mask, unsigned light_mask,
                  int W, int H, int x0, int y0, int cw, int ch,
                  const float* inv_mvp, const float* seeds, const float* eye, int spp, int k0,
                  int max_bounces, int accum_mode, float* accum, float* aov_n, float* aov_p) {
  if (W <= 0 || H <= 0 || n < 0 || tn < 0 || ln < 0 || spp < 0 || !accum) return -1;
  if (x0 < 0 || y0 < 0 || x0 + cw > W || y0 + ch > H) return -1;
  C.objects.d = objects; C.objects.w = 18; C.objects.h = n;
  C.texParams.d = texparams; C.texParams.w = 16; C.texParams.h = tn;
  C.lights.d = lights; C.lights.w = 18; C.lights.h = ln;
  C.n = n; C.tn = tn; C.ln = ln;
  C.shapeMask = shape_mask; C.matMask = mat_mask; C.texMask = tex_mask; C.lightMask = light_mask;
  for (int s = 0; s < spp; s++) {
    V3 d[4];
    cornerDirs(inv_mvp + 16 * s, eye, d);
    const V3 eyev = v3(F(eye[0]), F(eye[1]), F(eye[2]));
    C.timeSinceStart = F(seeds[s]);
    const int k = k0 + s;
    const float w = (float)((double)k / (double)(k + 1));  // tracer.js:97 (f64 divide, uploaded as f32)
    for (int y = y0; y < y0 + ch; y++) {
      for (int x = x0; x < x0 + cw; x++) {
        C.fcx = F((float)x + 0.5f); C.fcy = F((float)y + 0.5f); C.fcz = F(0.5f);
        V3 e, nn = BLACKv, pp = BLACKv;
        trace(ray_(eyev, primaryDir(d, x, y, W, H)), max_bounces, e, nn, pp);
        float* a = accum + 4 * ((size_t)y * W + x);
        if (accum_mode == ACC_SUM) {
          a[0] += raw(e.x); a[1] += raw(e.y); a[2] += raw(e.z); a[3] += 1.0f;
        } else {
          const V3 prev = v3(F(a[0]), F(a[1]), F(a[2]));
          const V3 m = mix3(e, prev, F(w));
          if (accum_mode == ACC_COMPAT8) { a[0] = q8(raw(m.x)); a[1] = q8(raw(m.y)); a[2] = q8(raw(m.z)); }
          else { a[0] = raw(m.x); a[1] = raw(m.y); a[2] = raw(m.z); }
          a[3] = 1.0f;
        }
        if (aov_n && s == spp - 1) {
          float* o = aov_n + 4 * ((size_t)y * W + x);
          const V3 q = nn / F(2.0f) + F(0.5f);
          o[0] = raw(q.x); o[1] = raw(q.y); o[2] = raw(q.z); o[3] = 1.0f;
        }
        if (aov_p && s == spp - 1) {
          float* o = aov_p + 4 * ((size_t)y * W + x);
          const V3 q = normalize(pp);
          o[0] = raw(q.x); o[1] = raw(q.y); o[2] = raw(q.z); o[3] = 1.0f;
        }
      }
    }
  }
  return 0;
}

unsigned long long oracle_segments(void) { return g_segments; }
void oracle_reset_counters(void) {
  g_segments = 0;
#ifdef SAIL_COUNT_OPS
  g_ops = 0;
  g_opsLastFull = 0;
  g_opsLastLive = 0;
  g_opsShadowDead = 0;
#endif
}
// ops of the live-op model: every op but the last bounce's dead ones (countLiveLast) and the shadow tests of
// light samples whose contribution would be +0 (SHADOW_TEST)
unsigned long long oracle_ops_live(void) {
#ifdef SAIL_COUNT_OPS
  return g_ops - g_opsLastFull + g_opsLastLive - g_opsShadowDead;
#else
  return 0;
#endif
}
unsigned long long oracle_ops(void) {
#ifdef SAIL_COUNT_OPS
  return g_ops;
#else
  return 0;
#endif
}

// ---- display filters (fsrender.glsl + filter/*.glsl), generalised from 512x512 to W x H ----------------------
// color map = mean image (W*H*4, alpha ignored). Sampling of the (non-NPOT, webgl.js:153-156) frame texture is
// LINEAR with the default REPEAT wrap. Output: W*H*4 float pixelFilter() value.
enum { FILTER_COLOR = 0, FILTER_GAMMA = 1, FILTER_TONEMAP = 2, FILTER_WINDOW = 3 };
static inline float wrapf(int i, int size) { int m = i % size; return (float)(m < 0 ? m + size : m); }
static void bilinear(const float* img, int W, int H, float u, float v, float out[3]) {
  const float fx = u * (float)W - 0.5f, fy = v * (float)H - 0.5f;
  const float x0f = floorf(fx), y0f = floorf(fy);
  const float a = fx - x0f, b = fy - y0f;
  const int xi = (int)x0f, yi = (int)y0f;
  const int xa = (int)wrapf(xi, W), xb = (int)wrapf(xi + 1, W), ya = (int)wrapf(yi, H), yb = (int)wrapf(yi + 1, H);
  for (int c = 0; c < 3; c++) {
    const float t00 = img[4 * ((size_t)ya * W + xa) + c], t10 = img[4 * ((size_t)ya * W + xb) + c];
    const float t01 = img[4 * ((size_t)yb * W + xa) + c], t11 = img[4 * ((size_t)yb * W + xb) + c];
    const float c0 = t00 * (1.0f - a) + t10 * a, c1 = t01 * (1.0f - a) + t11 * a;
    out[c] = c0 * (1.0f - b) + c1 * b;
  }
}
int oracle_filter(const float* mean, int W, int H, int kind, const float* weights16, float rx, float ry,
                  float gamma_c, float* out) {
  if (!mean || !out || W <= 0 || H <= 0) return -1;
  for (int y = 0; y < H; y++) {
    for (int x = 0; x < W; x++) {
      const float tcx = ((float)x + 0.5f) / (float)W, tcy = ((float)y + 0.5f) / (float)H;  // vsrender texCoord
      float col[3];
      const float* m = mean + 4 * ((size_t)y * W + x);
      float* o = out + 4 * ((size_t)y * W + x);
      if (kind == FILTER_COLOR) {  // color.glsl:1-4 (texel centre: bilinear == nearest)
        bilinear(mean, W, H, tcx, tcy, col);
        o[0] = col[0]; o[1] = col[1]; o[2] = col[2];
      } else if (kind == FILTER_GAMMA) {  // gamma.glsl:1-8
        bilinear(mean, W, H, tcx, tcy, col);
        const float g = fdiv_s(1.0f, gamma_c);
        o[0] = refm::pow_s(col[0], g); o[1] = refm::pow_s(col[1], g); o[2] = refm::pow_s(col[2], g);
      } else if (kind == FILTER_TONEMAP) {  // tonemapping.glsl:1-9
        bilinear(mean, W, H, tcx, tcy, col);
        for (int c = 0; c < 3; c++) {
          const float xx = refm::fmax_s(0.0f, col[c] - 0.004f);
          o[c] = fdiv_s(xx * (6.2f * xx + 0.5f), xx * (6.2f * xx + 1.7f) + 0.06f);
        }
      } else if (kind == FILTER_WINDOW) {  // window.glsl:1-44, FILTER_WINDOW_WIDTH 4
        float acc[3] = {0.0f, 0.0f, 0.0f};
        float weightSum = 0.0f;
        for (int i = 0; i < 4; i++) {
          for (int j = 0; j < 4; j++) {
            const float wi = fdiv_s(((float)j + 0.5f) * rx, 4.0f), wj = fdiv_s(((float)i + 0.5f) * ry, 4.0f);
            const float ox = fdiv_s(wi, (float)W), oy = fdiv_s(wj, (float)H);   // i/512.0, j/512.0 generalised
            float tmp[3] = {0.0f, 0.0f, 0.0f};
            int count = 0;
            const float cxs[4] = {tcx + ox, tcx + ox, tcx - ox, tcx - ox};
            const float cys[4] = {tcy + oy, tcy - oy, tcy + oy, tcy - oy};
            for (int q = 0; q < 4; q++) {  // windowSampler :1-8 (coord + x + y, + x - y, - x + y, - x - y)
              const float u = cxs[q], v = cys[q];
              if (u < 0.0f || u > 1.0f || v < 0.0f || v > 1.0f) continue;
              count++;
              float s3[3];
              bilinear(mean, W, H, u, v, s3);
              tmp[0] += s3[0]; tmp[1] += s3[1]; tmp[2] += s3[2];
            }
            const float weight = weights16[i * j + j];           // index bug kept (window.glsl:38)
            weightSum += weight * (float)count;
            acc[0] += tmp[0] * weight; acc[1] += tmp[1] * weight; acc[2] += tmp[2] * weight;
          }
        }
        o[0] = fdiv_s(acc[0], weightSum); o[1] = fdiv_s(acc[1], weightSum); o[2] = fdiv_s(acc[2], weightSum);
      } else {
        return -2;
      }
      (void)m;
      o[3] = 1.0f;
    }
  }
  return 0;
}

// ---- AOV filters: wavelet.glsl:5-54 (a-trous), normal.glsl, position.glsl -------------------------------------------
// mean, nrm, pos: W*H*4 maps (alpha ignored: RGB textures read alpha 1). kind 4 wavelet (FILTER_WAVELET_R = (rx, ry);
// the 512 / 1280 texture-space constants generalise to W / 2.5 W), 5 normal, 6 position.
int oracle_filter_aov(const float* mean, const float* nrm, const float* pos, int W, int H, int kind, float rx,
                      float ry, float* out) {
  if (!mean || !nrm || !pos || !out || W <= 0 || H <= 0 || kind < 4 || kind > 6) return -1;
  const float hk[5] = {0.375f, 0.25f, 0.0625f, 0.0625f, 0.25f};          // wavelet.glsl:29
  const float dW = (float)W, dH = (float)H, dW2 = dW * 2.5f, dH2 = dH * 2.5f;
  for (int y = 0; y < H; y++) {
    for (int x = 0; x < W; x++) {
      const float tcx = ((float)x + 0.5f) / (float)W, tcy = ((float)y + 0.5f) / (float)H;
      float* o = out + 4 * ((size_t)y * W + x);
      if (kind == 5 || kind == 6) {
        float m[3];
        bilinear(kind == 5 ? nrm : pos, W, H, tcx, tcy, m);
        o[0] = m[0]; o[1] = m[1]; o[2] = m[2]; o[3] = 1.0f;
        continue;
      }
      float cval[4], pval[4];
      bilinear(mean, W, H, tcx, tcy, cval); cval[3] = 1.0f;               // texture(colorMap, texCoord)
      bilinear(pos, W, H, tcx, tcy, pval); pval[3] = 1.0f;
      float color[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      float weightSum = 0.0f;
      for (int n = 0; n < 3; n++) {
        const float stepwidth = refm::pow_s(2.0f, (float)n) - 1.0f;
        int count = 0;
        for (int i = 0; i < 5; i++) {
          for (int j = 0; j < 5; j++, count++) {
            const int delt = abs(count - 12);
            float h = 0.0f;
            if (delt % (refm::to_int(stepwidth) + 1) == 0) h = hk[(delt / (refm::to_int(stepwidth) + 1)) % 5];
            if (h == 0.0f) continue;
            const float u = (tcx - fdiv_s(rx, dW)) + fdiv_s(((float)j + 0.5f) * rx, dW2);
            const float v = (tcy - fdiv_s(ry, dH)) + fdiv_s(((float)i + 0.5f) * ry, dH2);
            // W() :5-22
            float ctmp[4], ptmp[4], t[4];
            bilinear(mean, W, H, u, v, ctmp); ctmp[3] = 1.0f;
            for (int k = 0; k < 4; k++) t[k] = cval[k] - ctmp[k];
            float dist2 = t[0] * t[0] + t[1] * t[1] + t[2] * t[2] + t[3] * t[3];
            const float c_w = refm::fmin_s(refm::exp_s(fdiv_s(-(dist2), 4.0f)), 1.0f);
            dist2 = refm::fmax_s(fdiv_s(t[0] * t[0] + t[1] * t[1] + t[2] * t[2] + t[3] * t[3], stepwidth * stepwidth), 0.0f);
            const float n_w = refm::fmin_s(refm::exp_s(fdiv_s(-(dist2), 128.0f)), 1.0f);
            bilinear(pos, W, H, u, v, ptmp); ptmp[3] = 1.0f;
            for (int k = 0; k < 4; k++) t[k] = pval[k] - ptmp[k];
            dist2 = t[0] * t[0] + t[1] * t[1] + t[2] * t[2] + t[3] * t[3];
            const float p_w = refm::fmin_s(refm::exp_s(fdiv_s(-(dist2), 1.0f)), 1.0f);
            const float weight = c_w * n_w * p_w * h;
            for (int k = 0; k < 4; k++) ctmp[k] *= weight;
            weightSum += weight;
            for (int k = 0; k < 4; k++) color[k] += ctmp[k];
          }
        }
      }
      for (int k = 0; k < 4; k++) o[k] = fdiv_s(color[k], weightSum);
    }
  }
  return 0;
}

// ---- exported spec math for the GPU bit-parity test ----------------------------------------------------------
void oracle_math(int fn, const float* x, const float* y, float* out, int count) {
  for (int i = 0; i < count; i++) {
    switch (fn) {
      case 0: out[i] = refm::sin_s(x[i]); break;
      case 1: out[i] = refm::cos_s(x[i]); break;
      case 2: out[i] = refm::tan_s(x[i]); break;
      case 3: out[i] = refm::atan2_s(y[i], x[i]); break;
      case 4: out[i] = refm::acos_s(x[i]); break;
      case 5: out[i] = refm::pow_s(x[i], y[i]); break;
      case 6: out[i] = refm::atan_s(x[i]); break;
      case 7: out[i] = refm::sqrt_s(x[i]); break;
      case 8: out[i] = x[i] / y[i]; break;  // IEEE divide
      case 9: out[i] = refm::fmin_s(x[i], y[i]); break;
      case 10: out[i] = refm::fmax_s(x[i], y[i]); break;
      case 11: out[i] = refm::div_s(x[i], y[i]); break;  // GLSL divide spec
      case 14: out[i] = refm::rcp_s(x[i]); break;        // its reciprocal
      case 12: out[i] = refm::fmin_s(refm::fmax_s(x[i], 0.0f), 1.0f); break;
      default: out[i] = 0.0f; break;
    }
  }
}

// ---- single-primitive intersection distance (for the reference intersect() fixtures) -----------------------------
float oracle_intersect_t(const float* objects, int n, const float* texparams, int tn, unsigned shape_mask,
                         const float* o, const float* d) {
  C.objects.d = objects; C.objects.w = 18; C.objects.h = n;
  C.texParams.d = texparams; C.texParams.w = 16; C.texParams.h = tn;
  C.n = n; C.tn = tn; C.shapeMask = shape_mask; C.texMask = 0xffffffffu;
  const Intersect ins = intersectObjects(ray_(v3(F(o[0]), F(o[1]), F(o[2])), v3(F(d[0]), F(d[1]), F(d[2]))));
  return raw(ins.d);
}

// picking with the shader's intersectObjects (shader.shape.js:28-51): first row with the smallest d, -1 on a miss
int oracle_pick(const float* objects, int n, const float* texparams, int tn, unsigned shape_mask, const float* rays,
                int count, int* index, float* t) {
  C.objects.d = objects; C.objects.w = 18; C.objects.h = n;
  C.texParams.d = texparams; C.texParams.w = 16; C.texParams.h = tn;
  C.n = n; C.tn = tn; C.shapeMask = shape_mask; C.texMask = 0xffffffffu;
  for (int i = 0; i < count; i++) {
    const float* q = rays + 6 * i;
    const Intersect ins = intersectObjects(ray_(v3(F(q[0]), F(q[1]), F(q[2])), v3(F(q[3]), F(q[4]), F(q[5]))));
    t[i] = raw(ins.d);
    index[i] = ins.d < F(kMaxDistance) ? ins.index : -1;
  }
  return 0;
}

}  // extern "C"

// ---- unit probes of individual restated functions (known-answer tests) ----------------------------------------
extern "C" int oracle_probe(int fn, const float* in, float* out) {
  switch (fn) {
    case 0: out[0] = raw(frDielectric(F(in[0]), F(in[1]), F(in[2]))); return 0;
    case 1: {
      const V3 r = frConductor(F(in[0]), WHITEv, v3(F(in[1]), F(in[2]), F(in[3])), v3(F(in[4]), F(in[5]), F(in[6])));
      out[0] = raw(r.x); out[1] = raw(r.y); out[2] = raw(r.z); return 0;
    }
    case 2: {
      F t0 = F(0.0f), t1 = F(0.0f);
      const bool ok = quadratic(F(in[0]), F(in[1]), F(in[2]), t0, t1);
      out[0] = ok ? 1.0f : 0.0f; out[1] = raw(t0); out[2] = raw(t1); return 0;
    }
    case 3: { const V3 r = cosineSampleHemisphere(v2(F(in[0]), F(in[1]))); out[0] = raw(r.x); out[1] = raw(r.y); out[2] = raw(r.z); return 0; }
    case 4: out[0] = raw(trD(F(in[0]), F(in[1]), v3(F(in[2]), F(in[3]), F(in[4])))); return 0;
    case 5: {
      C.fcx = F(in[1]); C.fcy = F(in[2]); C.fcz = F(0.5f);
      const V2 r = random2(F(in[0])); out[0] = raw(r.x); out[1] = raw(r.y); return 0;
    }
    case 6: { const V2 r = concentricSampleDisk(v2(F(in[0]), F(in[1]))); out[0] = raw(r.x); out[1] = raw(r.y); return 0; }
    case 7: { const V3 r = uniformSampleSphere(v2(F(in[0]), F(in[1]))); out[0] = raw(r.x); out[1] = raw(r.y); out[2] = raw(r.z); return 0; }
    case 8: {  // Lambert matte throughput f*|cos|/pdf for R = in[0..2], wo = (0,0,1), u = in[3..4]
      const V3 R = v3(F(in[0]), F(in[1]), F(in[2]));
      const V3 wi = cosineSampleHemisphere(v2(F(in[3]), F(in[4])));
      const F pdf = sameHemisphere(v3(F(0.0f), F(0.0f), F(1.0f)), wi) ? absCosTheta(wi) * F(kInvPI) : F(0.0f);
      const V3 r = (R * F(kInvPI)) * absCosTheta(wi) / pdf;
      out[0] = raw(r.x); out[1] = raw(r.y); out[2] = raw(r.z); return 0;
    }
    default: return -1;
  }
}
