// sail_trace.hip — the MI355X (gfx950) trace megakernel and display-filter kernel.
//
// Re-implements the per-pixel loop of Sail's generated trace fragment program
// (src/shader/main/fstrace.glsl:6-17 -> trace/path.glsl:16-38 -> generated intersectObjects /
// material / light_sample / getSurfaceColor, shader.*.js) and the display pass
// (main/fsrender.glsl + filter/window.glsl:26-44, tonemapping.glsl, gamma.glsl, color.glsl).
//
// MI355X design:
//  * one lane = one pixel; a 256-thread workgroup covers a 16x16 pixel block, each wave a coherent 16x4 strip;
//    the grid walks only this rank's 64x64 partition tiles (interleaved t % world);
//  * all `spp` samples of a launch loop inside the lane with the radiance sum / running mean in
//    registers: HBM sees one float4 read + one float4 write per pixel per launch;
//  * the scene is decoded once on the host into 128-B primitive records; the primitive loop index is
//    wave-uniform, so every record field arrives through the scalar cache into SGPRs (no LDS copy, no
//    VGPRs), and material/texture/light rows are read with per-lane indices from L1/L2;
//  * intersectObjects is split into a t-only pass over all primitives and ONE full hit record
//    (normal, dpdu/dpdv, UV, texture) for the closest primitive; the reference builds the full record
//    for every primitive hit (shader.shape.js:44-50). The strict-`<`, first-index tie rule and every
//    f32 operation up to t are kept, so results are bit-identical to the oracle's restatement;
//  * per-sample camera corners and seeds arrive precomputed (SailSample, scalar loads);
//  * all f32 math follows the reference expression order with contraction off; transcendentals use
//    the bit-defined spec in sail_math.h.
#if !defined(__HIPCC_RTC__)  // hipRTC (the per-plugin-set kernels, sail_jit.cpp) provides the HIP runtime and stdint
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif
#include "sail_device.h"
#include "sail_math.h"
#include "sail_scan.h"

using namespace sm;

// Round 4 pruned every measured-and-rejected variant out of this file (their numbers stay in DESIGN.md §6 and
// profiles/r0*_variants_*.jsonl). What remains is what the four plugin-set kernels run; choices that differ between
// kernels are compile-time constants of the kernel template (CULL, KS, ...), not build switches. The one build switch
// left, SAIL_PHASE_TIMING, is instrumentation: tests/test_gpu_parity.py renders through its build too.

#define D __device__ __forceinline__

#if defined(SAIL_PHASE_TIMING) && SAIL_PHASE_TIMING
// the phase-timing build's per-phase wave-cycle sums: C linkage, so that a run-time compiled module's own copy can be
// found by name (sail_jit_phase_read)
extern "C" __device__ unsigned long long g_sailPhase[12];
__device__ unsigned long long g_sailPhase[12];
#endif

namespace {

constexpr float kMaxDistance = 1e5f, kEps = 1e-5f, kOneMinusEps = 0.9999f, kInf = 1e5f;
constexpr float kPI = 3.141592653589793f, kInvPI = 0.3183098861837907f;
constexpr float kPiOver2 = 1.570796326794896f, kPiOver4 = 0.785398163397448f;

struct V3 { float x, y, z; };
struct V2 { float x, y; };
D V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
D V3 v3s(float s) { return v3(s, s, s); }
D V2 v2(float x, float y) { V2 r; r.x = x; r.y = y; return r; }
D V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
D V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
D V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
// GLSL division (sail_math.h fdiv: a * RN(1/b)); a vector over a scalar shares one reciprocal
D V3 operator/(V3 a, V3 b) { return v3(fdiv(a.x, b.x), fdiv(a.y, b.y), fdiv(a.z, b.z)); }
D V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
D V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
D V3 operator/(V3 a, float s) { const float r = rcp_rn(s); return v3(a.x * r, a.y * r, a.z * r); }
D V3 operator+(V3 a, float s) { return v3(a.x + s, a.y + s, a.z + s); }
D V3 operator-(V3 a, float s) { return v3(a.x - s, a.y - s, a.z - s); }
D V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
D V2 operator*(float s, V2 a) { return v2(s * a.x, s * a.y); }
D float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
D float length(V3 v) { return sqrtf_(dot(v, v)); }
D V3 normalize(V3 v) { return v / length(v); }
D V3 vmin(V3 a, V3 b) { return v3(fmin_(a.x, b.x), fmin_(a.y, b.y), fmin_(a.z, b.z)); }
D V3 vmax(V3 a, V3 b) { return v3(fmax_(a.x, b.x), fmax_(a.y, b.y), fmax_(a.z, b.z)); }
D V3 vclamp01(V3 x) { return v3(clamp_(x.x, 0.0f, 1.0f), clamp_(x.y, 0.0f, 1.0f), clamp_(x.z, 0.0f, 1.0f)); }
D bool isBlack(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
D V3 reflect_(V3 I, V3 N) { return I - (2.0f * dot(N, I)) * N; }
D V3 refract_(V3 I, V3 N, float eta) {
  const float dni = dot(N, I);
  const float k = 1.0f - eta * eta * (1.0f - dni * dni);
  if (k < 0.0f) return v3s(0.0f);
  return eta * I - (eta * dni + sqrtf_(k)) * N;
}
D V3 worldToLocal(V3 v, V3 ns, V3 ss, V3 ts) { return v3(dot(v, ss), dot(v, ts), dot(v, ns)); }
D V3 localToWorld(V3 v, V3 ns, V3 ss, V3 ts) {
  return v3(ss.x * v.x + ts.x * v.y + ns.x * v.z, ss.y * v.x + ts.y * v.y + ns.y * v.z,
            ss.z * v.x + ts.z * v.y + ns.z * v.z);
}
// Box faces (Cube, Cornellbox): normal, dpdu, dpdv, ss and ts all have components in {0, +-1}, so every product of
// their dot products, cross products and frame changes is exact, and each a*b + c rounds once: written fma(a, b, c),
// bit for bit the unfused sum (the zero-sum sign rule of fma is the addition's; 0 * inf / NaN is NaN either way).
// Measured bit-identical with ~20 fewer VALU per box-face bounce: C2 -1.2 %, C3 -0.8 % (the second shading-frame
// branch costs more than it saves there), C4 +0.9 %: the pre-cull kernel only (Hit.axis).
D float dotX(V3 a, V3 b) { return fma_(a.z, b.z, fma_(a.y, b.y, a.x * b.x)); }
D V3 crossX(V3 a, V3 b) {
  return v3(fma_(a.y, b.z, -(a.z * b.y)), fma_(a.z, b.x, -(a.x * b.z)), fma_(a.x, b.y, -(a.y * b.x)));
}
D V3 localToWorldX(V3 v, V3 ns, V3 ss, V3 ts) {
  return v3(fma_(ns.x, v.z, fma_(ts.x, v.y, ss.x * v.x)), fma_(ns.y, v.z, fma_(ts.y, v.y, ss.y * v.x)),
            fma_(ns.z, v.z, fma_(ts.z, v.y, ss.z * v.x)));
}
// OBJECT_SPACE_N/S/T (define.glsl:62-64): the full dot products of the reference, so -0 / NaN propagate the same.
// A product with an exact 0 is exact (a signed zero, or NaN), so "a*0 + b" rounds once either way and is written
// fma(a, 0, b): bit for bit the same sum (the zero-sum sign rule of fma is the addition's) in fewer instructions.
D V3 W2L(V3 v) {  // (dot(v, (0,0,-1)), dot(v, (1,0,0)), dot(v, (0,1,0)))
  return v3(fma_(v.y, 0.0f, v.x * 0.0f) - v.z, fma_(v.z, 0.0f, fma_(v.y, 0.0f, v.x)), fma_(v.z, 0.0f, fma_(v.x, 0.0f, v.y)));
}
D V3 L2W(V3 v) {  // (0,0,-1) v.x + (1,0,0) v.y + (0,1,0) v.z, row by row as localToWorld sums them
  return v3(fma_(v.z, 0.0f, fma_(v.x, 0.0f, v.y)), fma_(v.y, 0.0f, v.x * 0.0f) + v.z, fma_(v.z, 0.0f, fma_(v.y, 0.0f, -v.x)));
}
D bool equalZero(float x) { return x < 1e-3f && x > -1e-3f; }
D float sgn(int rev) { return rev ? -1.0f : 1.0f; }

D bool quadratic(float A, float B, float C, float& t0, float& t1) {  // utility.glsl:37-51
  const float discrim = B * B - 4.0f * A * C;
  if (discrim < 0.0f) return false;
  const float rootDiscrim = sqrtf_(discrim);
  float q;
  if (B < 0.0f) q = -0.5f * (B - rootDiscrim);
  else q = -0.5f * (B + rootDiscrim);
  t0 = fdiv(q, A);
  t1 = fdiv(C, q);
  if (t0 > t1) { const float tmp = t0; t0 = t1; t1 = tmp; }
  return true;
}

// A ray carries the reciprocals of its direction: every slab test divides by the same three components, and
// under the GLSL division spec a / d.x is a * RN(1/d.x), so a slab is six subtractions and six multiplies.
struct Ray { V3 o, d; float rx, ry, rz; };
D Ray mkRay(V3 o, V3 d) {
  Ray r; r.o = o; r.d = d;
  // one range guard for the three components (rcp_rn guards each)
  const float mx = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z)), mn = fminf(fminf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
  // wave-uniform: the IEEE reciprocals (equal to the Newton step in range) for every lane when some lane is out of range
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(mn >= 0x1p-126f && mx <= 0x1p126f)) == 0ull, 1)) {
    const float y0 = __builtin_amdgcn_rcpf(d.x), y1 = __builtin_amdgcn_rcpf(d.y), y2 = __builtin_amdgcn_rcpf(d.z);
    r.rx = fma_(fma_(-d.x, y0, 1.0f), y0, y0);
    r.ry = fma_(fma_(-d.y, y1, 1.0f), y1, y1);
    r.rz = fma_(fma_(-d.z, y2, 1.0f), y2, y2);
  } else {
    r.rx = 1.0f / d.x; r.ry = 1.0f / d.y; r.rz = 1.0f / d.z;
  }
  return r;
}
// ---- optional phase timing (-DSAIL_PHASE_TIMING=1: libsail_hip_phase.so, tools/phase_profile.py): per-wave
// s_memtime deltas per phase of the bounce, summed over the launch; the results are those of the plain build
#ifndef SAIL_PHASE_TIMING
#define SAIL_PHASE_TIMING 0
#endif
#if SAIL_PHASE_TIMING
struct PhaseClock { unsigned long long t, acc[12]; };
#define PHASE_MARK(pc, k) do { const unsigned long long now_ = __builtin_amdgcn_s_memtime(); (pc).acc[k] += now_ - (pc).t; (pc).t = now_; } while (0)
#else
struct PhaseClock {};
#define PHASE_MARK(pc, k) do { (void)(pc); } while (0)
#endif
struct Hit {
  float d; V3 hit, normal, dpdu, dpdv; bool into; int matRow; V3 sc, emission; int matCategory;
  float nd;  // dot(geometric normal before the into flip, ray direction)
  bool axis; // box face in the pre-cull kernel: normal / dpdu / dpdv components in {0, +-1} (dotX, crossX)
};
struct Ctx {
  const float* tp; const float* lt; const int32_t* lightObjRow; const SailPrim* prims;
  const SailPrim* cprims;  // rows for the candidate loops' per-lane reads: an LDS copy when it fits (kCullLdsRows)
  const float* tpl;        // texParams rows, an LDS copy when they fit (kCullLdsTp)
  bool rowCopy, tpCopy;    // per-lane hit-record / light-sampler row reads and texParams reads go through cprims / tpl
  const unsigned long long* typeMasks;
  int n, tn, ln;
  uint32_t matMask, texMask, lightMask;
  float fcx, fcy;
  int shadowAnyHit;
  int cullPrims;
  int cullFma;     // the candidate sweep's pre-cull in the fused form (padHitF)
  int cullPrimary; // primary rays may use the pre-cull (the eye is near the scene)
  // plugin sets compiled into this kernel instantiation (compile-time constants after inlining): the
  // reference generates one GLSL program per scene plugin set (shader.js combinefs); this build precompiles
  // kernels for plugin subsets and dispatches the smallest one that covers the scene
  uint32_t kShapes, kMats, kTex, kLights;
};
#define HAS(set, id) (((set) >> (id)) & 1u)

// Scene rows are read through the constant address space: the kernels also store to global memory (AOVs,
// stage, accumulator) through pointers the compiler cannot prove disjoint from the scene, and without this
// a wave-uniform primitive read becomes a per-lane vector load (VGPRs + TA cycles) instead of a scalar load.
template <typename T> using ConstAS = const __attribute__((address_space(4))) T;
template <typename T> D const T& constRow(const T* base, int i) { return *(const T*)((ConstAS<T>*)base + i); }
#define PRIM(c, i) constRow<SailPrim>((c).prims, (i))

D V3 P3(const SailPrim& p, int k) { return v3(p.a[k], p.a[k + 1], p.a[k + 2]); }
D float TP(const Ctx& c, int row, int col) {
  if (c.tpCopy) return c.tpl[row * 16 + col];  // kernels with table copies in LDS (compile-time)
  return constRow<float>(c.tp, row * 16 + col);
}
D V3 TP3(const Ctx& c, int row, int col) { return v3(TP(c, row, col), TP(c, row, col + 1), TP(c, row, col + 2)); }

// the square root of the warps and BSDF terms whose argument is in [0, 1] by construction (sail_math.h sqrt01)
#define SQRT01(x) sqrt01(x)
// ---- random.glsl:5-18 ---------------------------------------------------------------------------------
D float hash1(const Ctx& c, float seed, float a, float b, float cc) {
  const V3 p = v3(c.fcx + seed, c.fcy + seed, 0.5f + seed);
  return fract_(sinf_(dot(p, v3(a, b, cc))) * 43758.5453f + seed);
}
D V2 random2(const Ctx& c, float seed) {
  return v2(hash1(c, seed, 12.9898f, 78.233f, 151.7182f), hash1(c, seed, 63.7264f, 10.873f, 623.6736f));
}

// ---- sampler.glsl ---------------------------------------------------------------------------------------
D V3 uniformSampleSphere(V2 u) {
  const float z = 1.0f - 2.0f * u.x;
  const float r = SQRT01(1.0f - z * z);
  const float angle = 2.0f * kPI * u.y;
  float s, co; sincosf_(angle, s, co);
  return v3(r * co, r * s, z);
}
D V3 cosineSampleHemisphere(V2 u) {
  const float r = SQRT01(u.x);
  const float angle = 2.0f * kPI * u.y;
  float s, co; sincosf_(angle, s, co);
  return v3(r * co, r * s, SQRT01(1.0f - u.x));
}
D V2 concentricSampleDisk(V2 u) {
  const float uOffset = 2.0f * u.x - 1.0f, vOffset = 2.0f * u.y - 1.0f;
  if (uOffset == 0.0f && vOffset == 0.0f) return v2(0.0f, 0.0f);
  float theta, r;
  if (fabsf(uOffset) > fabsf(vOffset)) { r = uOffset; theta = fdiv(vOffset, uOffset) * kPiOver4; }
  else { r = vOffset; theta = kPiOver2 - fdiv(uOffset, vOffset) * kPiOver4; }
  float s, co; sincosf_(theta, s, co);
  return r * v2(co, s);
}

// ---- textures (shader.texture.js:22-29) ----------------------------------------------------------------
// The pre-cull kernel's two checkerboards share uv / size and its floor, so a wave holding both runs them once (same
// operations). Measured (bit-identical, profiles/r03_variants_tex_shared.jsonl, three rounds): C3 -1.4 %, C4 +0.7 %
// (its 64 rows mix both textures in most waves), so the flat kernels keep one branch per texture.
// UNIFORM_COLOR ignores uv, so hit records skip the UV arithmetic (atan2/acos/divides) for it
D int matCat(const SailPrim& p) { return (int)(short)(p.cats & 0xffff); }
D int texCat(const SailPrim& p) { return p.cats >> 16; }
D bool needsUV(const SailPrim& p) { return texCat(p) != SAIL_TEX_UNIFORM; }
D V3 getSurfaceColor(const Ctx& c, V2 uv, const SailPrim& p) {
  const int texRow = p.texRow, cat = texCat(p);
  if (cat == SAIL_TEX_UNIFORM) return TP3(c, texRow, 1);
  if (cat < 0 || cat >= 32 || !((c.texMask >> cat) & 1u)) return v3s(0.0f);
  // c.cullPrims is a compile-time constant in every kernel (the pre-cull ones set 1)
  if (c.cullPrims &&
      ((cat == SAIL_TEX_CHECKERBOARD && HAS(c.kTex, SAIL_TEX_CHECKERBOARD)) ||
       (cat == SAIL_TEX_CHECKERBOARD2 && HAS(c.kTex, SAIL_TEX_CHECKERBOARD2)))) {
    const bool cb1 = cat == SAIL_TEX_CHECKERBOARD;
    const float size = cb1 ? TP(c, texRow, 1) : TP(c, texRow, 7);
    const float sx = fdiv(uv.x, size), sy = fdiv(uv.y, size);
    const float qx = floorf(sx), qy = floorf(sy);
    if (cb1) {
      const float width = fdiv(0.5f * TP(c, texRow, 2), size);
      const float fx = sx - qx, fy = sy - qy;
      const bool in_outline = (fx < width || fx > 1.0f - width) || (fy < width || fy > 1.0f - width);
      return in_outline ? v3s(0.5f) : v3s(1.0f);
    }
    return (to_int(qx + qy) % 2 == 0) ? TP3(c, texRow, 1) : TP3(c, texRow, 4);
  }
  switch (cat) {
    case SAIL_TEX_CHECKERBOARD: if (!HAS(c.kTex, SAIL_TEX_CHECKERBOARD)) break; {
      const float size = TP(c, texRow, 1), lineWidth = TP(c, texRow, 2);
      const float width = fdiv(0.5f * lineWidth, size);
      const float fx = fdiv(uv.x, size) - floorf(fdiv(uv.x, size)), fy = fdiv(uv.y, size) - floorf(fdiv(uv.y, size));
      const bool in_outline = (fx < width || fx > 1.0f - width) || (fy < width || fy > 1.0f - width);
      return in_outline ? v3s(0.5f) : v3s(1.0f);
    }
    case SAIL_TEX_CHECKERBOARD2: if (!HAS(c.kTex, SAIL_TEX_CHECKERBOARD2)) break; {
      const float size = TP(c, texRow, 7);
      const float qx = floorf(fdiv(uv.x, size)), qy = floorf(fdiv(uv.y, size));
      return (to_int(qx + qy) % 2 == 0) ? TP3(c, texRow, 1) : TP3(c, texRow, 4);
    }
    case SAIL_TEX_BILERP: if (!HAS(c.kTex, SAIL_TEX_BILERP)) break; {
      const V3 c00 = TP3(c, texRow, 1), c01 = TP3(c, texRow, 4), c10 = TP3(c, texRow, 7), c11 = TP3(c, texRow, 10);
      return (1.0f - uv.x) * (1.0f - uv.y) * c00 + (1.0f - uv.x) * (uv.y) * c01 + (uv.x) * (1.0f - uv.y) * c10 +
             (uv.x) * (uv.y) * c11;
    }
    case SAIL_TEX_MIXF: if (!HAS(c.kTex, SAIL_TEX_MIXF)) break; {
      const float amount = TP(c, texRow, 7);
      return (1.0f - amount) * TP3(c, texRow, 1) + amount * TP3(c, texRow, 4);
    }
    case SAIL_TEX_SCALE: if (!HAS(c.kTex, SAIL_TEX_SCALE)) break; return TP3(c, texRow, 1) * TP3(c, texRow, 4);
    case SAIL_TEX_UVF: if (!HAS(c.kTex, SAIL_TEX_UVF)) break; return v3(uv.x - floorf(uv.x), uv.y - floorf(uv.y), 0.0f);
    default: break;
  }
  return v3s(0.0f);
}

// ---- slab boxes: cube.glsl:65-87, cornellbox.glsl:67-90, boundbox.glsl:6-17 ------------------------------
struct Slab { float tNear, tFar; };
D Slab slab(V3 bmin, V3 bmax, const Ray& r) {
  const V3 a0 = bmin - r.o, a1 = bmax - r.o;
  const V3 tMin = v3(a0.x * r.rx, a0.y * r.ry, a0.z * r.rz);  // (bmin - o) / d
  const V3 tMax = v3(a1.x * r.rx, a1.y * r.ry, a1.z * r.rz);
  const V3 t1 = vmin(tMin, tMax), t2 = vmax(tMin, tMax);
  Slab s;
  s.tNear = fmax_(fmax_(t1.x, t1.y), t1.z);
  s.tFar = fmin_(fmin_(t2.x, t2.y), t2.z);
  return s;
}
// Boundbox(max, min) constructor order (boundbox.glsl:1-4): the `min` member is the 2nd argument
D bool testBoundbox(const Ray& r, V3 bmax, V3 bmin) {
  const Slab s = slab(bmin, bmax, r);
  if (s.tNear < 0.0f && s.tFar < 0.0f) return false;
  return s.tNear < s.tFar;
}
D float cubeT(const SailPrim& p, const Ray& r) {
  const Slab s = slab(P3(p, 0), P3(p, 3), r);
  float t = -1.0f;
  if (s.tNear > kEps && s.tNear < s.tFar) t = s.tNear;
  else if (s.tNear < s.tFar) t = s.tFar;
  return (t > kEps) ? t : kMaxDistance;
}
D float cornellT(const SailPrim& p, const Ray& r) {
  const Slab s = slab(P3(p, 0), P3(p, 3), r);
  float t = -1.0f;
  if (s.tNear < s.tFar) t = s.tFar;
  return (t > kEps) ? t : kMaxDistance;
}
D V3 normalForCube(V3 hit, const SailPrim& p) {  // cube.glsl:25-38
  const float c = sgn(p.rev);
  const V3 mn = P3(p, 0), mx = P3(p, 3);
  if (hit.x < mn.x + 0.0001f) return c * v3(-1.0f, 0.0f, 0.0f);
  else if (hit.x > mx.x - 0.0001f) return c * v3(1.0f, 0.0f, 0.0f);
  else if (hit.y < mn.y + 0.0001f) return c * v3(0.0f, -1.0f, 0.0f);
  else if (hit.y > mx.y - 0.0001f) return c * v3(0.0f, 1.0f, 0.0f);
  else if (hit.z < mn.z + 0.0001f) return c * v3(0.0f, 0.0f, -1.0f);
  return c * v3(0.0f, 0.0f, 1.0f);
}
D V3 normalForCornellbox(V3 hit, const SailPrim& p) {  // cornellbox.glsl:39-51
  const V3 mn = P3(p, 0), mx = P3(p, 3);
  if (hit.x < mn.x + 0.0001f) return v3(-1.0f, 0.0f, 0.0f);
  else if (hit.x > mx.x - 0.0001f) return v3(1.0f, 0.0f, 0.0f);
  else if (hit.y < mn.y + 0.0001f) return v3(0.0f, -1.0f, 0.0f);
  else if (hit.y > mx.y - 0.0001f) return v3(0.0f, 1.0f, 0.0f);
  else if (hit.z < mn.z + 0.0001f) return v3(0.0f, 0.0f, -1.0f);
  return v3(0.0f, 0.0f, 1.0f);
}
D void dpdBox(V3 normal, V3& dpdu, V3& dpdv) {
  const V3 n = normal;  // cross(n, (1,0,0)) / cross(n, (0,1,0)) with the exact zero products folded (see W2L)
  if (fabsf(n.x) < 0.5f) dpdu = v3(fma_(n.y, 0.0f, n.z * -0.0f), fma_(n.x, -0.0f, n.z), fma_(n.x, 0.0f, -n.y));
  else dpdu = v3(fma_(n.y, 0.0f, -n.z), fma_(n.z, 0.0f, n.x * -0.0f), fma_(n.y, -0.0f, n.x));
  dpdv = cross(normal, dpdu);
}
D void cubeHit(const Ctx& c, const SailPrim& p, const Ray& r, float t, Hit& h) {
  h.hit = r.o + t * r.d;
  h.normal = normalForCube(r.o + t * r.d, p);
  dpdBox(h.normal, h.dpdu, h.dpdv);
  V2 uv = v2(0.0f, 0.0f);
  if (needsUV(p)) {
    const V3 mn = P3(p, 0), mx = P3(p, 3);
    const V3 tr = mx - mn, hh = h.hit - mn;  // getCubeUV cube.glsl:54-63
    if (hh.x < mn.x + 0.0001f || hh.x > mx.x - 0.0001f) uv = v2(fdiv(hh.y, tr.y), fdiv(hh.z, tr.z));
    else if (hh.y < mn.y + 0.0001f || hh.y > mx.y - 0.0001f) uv = v2(fdiv(hh.x, tr.x), fdiv(hh.z, tr.z));
    else uv = v2(fdiv(hh.x, tr.x), fdiv(hh.y, tr.y));
  }
  h.sc = getSurfaceColor(c, uv, p);
}
// The wall colour chain (cornellbox.glsl:53-65) tests the same face conditions in the same order as the normal
// chain (:39-51), except its last test, z > mn.z + 0.0001 where the normal's is z < mn.z + 0.0001: one chain sets
// both (z < t excludes z > t; after it the colour test is made as written). Same values, each face test once:
// 1 = one branch chain, 2 = branch-free selects. Bit-identical but slower (C2 -4.7 % / -3.8 %: more constant moves per
// branch and more spills), so the default keeps the reference's two chains.
D void cornellHit(const SailPrim& p, const Ray& r, float t, Hit& h) {
  h.hit = r.o + t * r.d;
  h.normal = -normalForCornellbox(r.o + t * r.d, p);
  dpdBox(h.normal, h.dpdu, h.dpdv);
  const V3 mn = P3(p, 0), mx = P3(p, 3), x = h.hit;
  if (x.x < mn.x + 0.0001f) h.sc = v3(0.25f, 0.75f, 0.25f);
  else if (x.x > mx.x - 0.0001f) h.sc = v3(0.25f, 0.25f, 0.75f);
  else if (x.y < mn.y + 0.0001f) h.sc = v3s(1.0f);
  else if (x.y > mx.y - 0.0001f) h.sc = v3s(1.0f);
  else if (x.z > mn.z + 0.0001f) h.sc = v3s(1.0f);
  else h.sc = v3s(0.0f);
}

// The room kernel's one hit record for both axis-aligned box shapes (a wave holding Cube and Cornellbox lanes runs one
// face chain instead of two). The face chains test the same conditions; the Cube's normal is sgn(rev) * n and the
// Cornellbox's is -n == -1 * n bit for bit (zeros included); only the surface colour differs (texture vs wall chain).
// Measured (bit-identical, profiles/r03_variants_box_unified*.jsonl): room kernel C3 +0.7 %; every kernel C2 -0.8 %,
// C4 +0.1 %; only in mixed waves C2 +-0.2 %, C3 -0.7 %, so the room kernel alone takes it.
D void boxHit(const Ctx& c, const SailPrim& p, const Ray& r, float t, Hit& h, bool cornell) {
  h.hit = r.o + t * r.d;
  const float s = cornell ? -1.0f : sgn(p.rev);
  h.normal = s * normalForCornellbox(r.o + t * r.d, p);
  dpdBox(h.normal, h.dpdu, h.dpdv);
  const V3 mn = P3(p, 0), mx = P3(p, 3), x = h.hit;
  if (cornell) {
    if (x.x < mn.x + 0.0001f) h.sc = v3(0.25f, 0.75f, 0.25f);
    else if (x.x > mx.x - 0.0001f) h.sc = v3(0.25f, 0.25f, 0.75f);
    else if (x.y < mn.y + 0.0001f) h.sc = v3s(1.0f);
    else if (x.y > mx.y - 0.0001f) h.sc = v3s(1.0f);
    else if (x.z > mn.z + 0.0001f) h.sc = v3s(1.0f);
    else h.sc = v3s(0.0f);
  } else {
    V2 uv = v2(0.0f, 0.0f);
    if (needsUV(p)) {
      const V3 tr = mx - mn, hh = h.hit - mn;  // getCubeUV cube.glsl:54-63
      if (hh.x < mn.x + 0.0001f || hh.x > mx.x - 0.0001f) uv = v2(fdiv(hh.y, tr.y), fdiv(hh.z, tr.z));
      else if (hh.y < mn.y + 0.0001f || hh.y > mx.y - 0.0001f) uv = v2(fdiv(hh.x, tr.x), fdiv(hh.z, tr.z));
      else uv = v2(fdiv(hh.x, tr.x), fdiv(hh.y, tr.y));
    }
    h.sc = getSurfaceColor(c, uv, p);
  }
}

// The quadrics' bounding-box test (testBoundboxFor*) and their root search are both pure predicates on the
// ray, so their order is free: the discriminant rejects most rays more cheaply than the six-divide slab test,
// and only candidate hits pay the exact slab test (same results; C3 +4 %, C4 +5 %, measured).
// ---- sphere.glsl:45-86 ---------------------------------------------------------------------------------------
D float sphereT(const SailPrim& p, const Ray& r0, V3* hitOut) {
  const V3 c = P3(p, 0);
  const float rad = p.a[3];
  const V3 d = W2L(r0.d), o = W2L(r0.o - c);
  const float a = dot(d, d), b = 2.0f * dot(o, d), cc = dot(o, o) - rad * rad;
  float t1 = 0.0f, t2 = 0.0f;
  if (!quadratic(a, b, cc, t1, t2)) return kMaxDistance;
  if (t2 < kEps) return kMaxDistance;
  float t = t1;
  if (t1 < kEps) t = t2;
  if (t >= kMaxDistance) return kMaxDistance;
  if (!testBoundbox(r0, c - v3s(rad), c + v3s(rad))) return kMaxDistance;
  if (hitOut) *hitOut = o + t * d;
  return t;
}
D float phiOf(float y, float x) {
  float phi = atan2f_(y, x);
  if (phi < 0.0f) phi += 2.0f * kPI;
  return phi;
}
D V3 dpduRot(V3 hit) { return v3(-2.0f * kPI * hit.y, 2.0f * kPI * hit.x, 0.0f); }
// cross(a, b) with a.z == 0 (crossZa) or b.z == 0 (crossZb), the exact zero products folded as in W2L
D V3 crossZa(V3 a, V3 b) {
  return v3(fma_(b.y, -0.0f, a.y * b.z), fma_(b.x, 0.0f, -(a.x * b.z)), a.x * b.y - a.y * b.x);
}
D V3 crossZb(V3 a, V3 b) {
  return v3(fma_(a.y, 0.0f, -(a.z * b.y)), fma_(a.x, -0.0f, a.z * b.x), a.x * b.y - a.y * b.x);
}
D void sphereHit(const Ctx& c, const SailPrim& p, V3 hl, Hit& h) {
  const float rad = p.a[3];
  // theta of the UV and of computeDpDForSphere (:33-43) are the same value: the pole guard touches x only
  const float theta = acosf_(clamp_(fdiv(hl.z, rad), -1.0f, 1.0f));
  V2 uv = v2(0.0f, 0.0f);
  if (needsUV(p)) {
    V3 hit = hl;
    if (hit.x == 0.0f && hit.y == 0.0f) hit.x = 1e-5f * rad;
    uv = v2(fdiv(phiOf(hit.y, hit.x), 2.0f * kPI), fdiv(theta, kPI));
  }
  const float th2 = theta;
  const float zRadius = sqrtf_(hl.x * hl.x + hl.y * hl.y);
  const float invZRadius = rcp_rn(zRadius);
  const float cosPhi = hl.x * invZRadius, sinPhi = hl.y * invZRadius;
  const V3 dpdu = dpduRot(hl);
  const V3 dpdv = kPI * v3(hl.z * cosPhi, hl.z * sinPhi, -rad * sinf_(th2));
  const V3 nl = normalize(crossZb(dpdv, dpdu));  // dpdu.z == 0
  h.sc = getSurfaceColor(c, uv, p);
  h.hit = L2W(hl) + P3(p, 0);
  h.normal = L2W(nl);
  h.dpdu = L2W(dpdu);
  h.dpdv = L2W(dpdv);
}

// ---- rectangle.glsl:32-63 ---------------------------------------------------------------------------------
struct RectFrame { V3 dpdu, dpdv, normal, ss, ts; float maxX, maxY; };
D RectFrame rectFrame(const SailPrim& p) {  // rectangle.glsl:32-44; the divides/roots are per scene (host)
  RectFrame f;
  const V3 mn = P3(p, 0), mx = P3(p, 3);
  f.dpdu = v3(mx.x - mn.x, 0.0f, 0.0f);
  f.dpdv = v3(0.0f, mx.y - mn.y, mx.z - mn.z);
  f.normal = P3(p, 6); f.ss = P3(p, 9); f.ts = P3(p, 12);
  f.maxX = p.a[15]; f.maxY = p.a[16];
  return f;
}
D float rectT(const SailPrim& p, const Ray& r, V3* hitOut) {
  const RectFrame f = rectFrame(p);
  const V3 d = worldToLocal(r.d, f.normal, f.ss, f.ts);
  const V3 o = worldToLocal(r.o - P3(p, 0), f.normal, f.ss, f.ts);
  if (d.z == 0.0f) return kMaxDistance;
  const float t = fdiv(-o.z, d.z);
  if (t < kEps) return kMaxDistance;
  const V3 hit = o + t * d;
  if (hit.x > f.maxX || hit.y > f.maxY || hit.x < -kEps || hit.y < -kEps) return kMaxDistance;
  if (hitOut) *hitOut = hit;
  return t;
}
D void rectHit(const Ctx& c, const SailPrim& p, V3 hl, Hit& h) {
  const RectFrame f = rectFrame(p);
  h.dpdu = f.dpdu; h.dpdv = f.dpdv; h.normal = f.normal;
  h.sc = getSurfaceColor(c, needsUV(p) ? v2(fdiv(hl.x, f.maxX), fdiv(hl.y, f.maxY)) : v2(0.0f, 0.0f), p);
  h.hit = localToWorld(hl, f.normal, f.ss, f.ts) + P3(p, 0);
}

// ---- cone.glsl:48-99 / cylinder.glsl:40-90 / hyperboloid.glsl:60-111 / paraboloid.glsl:51-103 ---------------
// shared tail: two-root retry against the z range, then the MAX_DISTANCE test
D bool rootPick(float t1, float t2, V3 o, V3 d, float zlo, float zhi, bool epsLo, float& t, V3& hit) {
  t = t1;
  if (t1 < kEps) t = t2;
  hit = o + t * d;
  const bool out = epsLo ? (hit.z < -kEps || hit.z > zhi) : (hit.z < zlo || hit.z > zhi);
  if (out) {
    if (t == t2) return false;
    t = t2;
    hit = o + t * d;
    const bool out2 = epsLo ? (hit.z < -kEps || hit.z > zhi) : (hit.z < zlo || hit.z > zhi);
    if (out2) return false;
  }
  return t < kMaxDistance;
}
D float coneT(const SailPrim& p, const Ray& r0, V3* hitOut) {
  const V3 pp = P3(p, 0);
  const float h = p.a[3], rad = p.a[4];
  const V3 d = W2L(r0.d), o = W2L(r0.o - pp);
  const float k = p.a[5];  // (rad / h)^2, per scene
  const float a = d.x * d.x + d.y * d.y - k * d.z * d.z;
  const float b = 2.0f * (d.x * o.x + d.y * o.y - k * d.z * (o.z - h));
  const float cc = o.x * o.x + o.y * o.y - k * (o.z - h) * (o.z - h);
  float t1 = 0.0f, t2 = 0.0f, t; V3 hit;
  if (!quadratic(a, b, cc, t1, t2)) return kMaxDistance;
  if (t2 < -kEps) return kMaxDistance;
  if (!rootPick(t1, t2, o, d, 0.0f, h, true, t, hit)) return kMaxDistance;
  if (!testBoundbox(r0, pp - v3(rad, 0.0f, rad), pp + v3(rad, h, rad))) return kMaxDistance;
  if (hitOut) *hitOut = hit;
  return t;
}
D float cylinderT(const SailPrim& p, const Ray& r0, V3* hitOut) {
  const V3 pp = P3(p, 0);
  const float h = p.a[3], rad = p.a[4];
  const V3 d = W2L(r0.d), o = W2L(r0.o - pp);
  const float a = d.x * d.x + d.y * d.y;
  const float b = 2.0f * (d.x * o.x + d.y * o.y);
  const float cc = o.x * o.x + o.y * o.y - rad * rad;
  float t1 = 0.0f, t2 = 0.0f, t; V3 hit;
  if (!quadratic(a, b, cc, t1, t2)) return kMaxDistance;
  if (t2 < -kEps) return kMaxDistance;
  if (!rootPick(t1, t2, o, d, 0.0f, h, true, t, hit)) return kMaxDistance;
  if (!testBoundbox(r0, pp - v3(rad, 0.0f, rad), pp + v3(rad, h, rad))) return kMaxDistance;
  if (hitOut) *hitOut = hit;
  return t;
}
D float hypT(const SailPrim& p, const Ray& r0, V3* hitOut) {
  const V3 pp = P3(p, 0);
  const float ah = p.a[9], ch = p.a[10];
  const V3 d = W2L(r0.d), o = W2L(r0.o - pp);
  const float a = ah * d.x * d.x + ah * d.y * d.y - ch * d.z * d.z;
  const float b = 2.0f * (ah * d.x * o.x + ah * d.y * o.y - ch * d.z * o.z);
  const float cc = ah * o.x * o.x + ah * o.y * o.y - ch * o.z * o.z - 1.0f;
  float t1 = 0.0f, t2 = 0.0f, t; V3 hit;
  if (!quadratic(a, b, cc, t1, t2)) return kMaxDistance;
  if (t2 < -kEps) return kMaxDistance;
  const float zMin = p.a[12], zMax = p.a[13];
  if (!rootPick(t1, t2, o, d, zMin, zMax, false, t, hit)) return kMaxDistance;
  {  // testBoundboxForHyperboloid :13-24 (rMax, zMin, zMax per scene)
    const float rMax = p.a[11], zMin = p.a[12], zMax = p.a[13];
    if (!testBoundbox(r0, pp - v3(rMax, -zMin, rMax), pp + v3(rMax, zMax, rMax))) return kMaxDistance;
  }
  if (hitOut) *hitOut = hit;
  return t;
}
D float paraT(const SailPrim& p, const Ray& r0, V3* hitOut) {
  const V3 pp = P3(p, 0);
  const float z0 = p.a[3], z1 = p.a[4], rad = p.a[5];
  const float zMin = fmin_(z0, z1), zMax = fmax_(z0, z1);
  const V3 d = W2L(r0.d), o = W2L(r0.o - pp);
  const float k = p.a[6];  // zMax / (rad * rad), per scene
  const float a = k * (d.x * d.x + d.y * d.y);
  const float b = 2.0f * k * (d.x * o.x + d.y * o.y) - d.z;
  const float cc = k * (o.x * o.x + o.y * o.y) - o.z;
  float t1 = 0.0f, t2 = 0.0f, t; V3 hit;
  if (!quadratic(a, b, cc, t1, t2)) return kMaxDistance;
  if (t2 < -kEps) return kMaxDistance;
  if (!rootPick(t1, t2, o, d, zMin, zMax, false, t, hit)) return kMaxDistance;
  if (!testBoundbox(r0, pp - v3(rad, -zMin, rad), pp + v3(rad, zMax, rad))) return kMaxDistance;
  if (hitOut) *hitOut = hit;
  return t;
}
D float diskT(const SailPrim& p, const Ray& r0, V3* hitOut) {  // disk.glsl:36-75
  const V3 pp = P3(p, 0);
  const float rad = p.a[3], ri = p.a[4];
  const V3 d = W2L(r0.d), o = W2L(r0.o - pp);
  if (d.z == 0.0f) return kMaxDistance;
  const float t = fdiv(-o.z, d.z);
  if (t <= 0.0f) return kMaxDistance;
  const V3 hit = o + t * d;
  const float dist2 = hit.x * hit.x + hit.y * hit.y;
  if (dist2 > rad * rad || dist2 < ri * ri) return kMaxDistance;
  if (t >= kMaxDistance) return kMaxDistance;
  if (hitOut) *hitOut = hit;
  return t;
}
// The pre-cull kernel's candidate sweep tests cones, cylinders, hyperboloids and paraboloids in one
// loop (quadT) instead of one loop per type. A wave then runs max-over-lanes(quadric candidates) iterations instead
// of the sum over the four types of max-over-lanes(candidates of the type). Per type only the coefficients and the
// z-range / box parameters differ; the ray transform, the root solve, rootPick and the box test are shared. Same
// operations on the same values as coneT / cylinderT / hypT / paraT (box test last). Candidates are visited out of
// row order either way (the take rule keeps the in-order winner).
// Measured (bit-identical, profiles/r03_variants_quad_shared.jsonl, three rounds): C4 +0.9 %; with the sphere in the
// same loop (its own root rule) -5.4 %, with the planar disk -0.6 %.
D float quadT(const SailPrim& p, const Ray& r0, V3* hitOut) {
  const int ty = p.type;
  const V3 pp = P3(p, 0);
  const V3 d = W2L(r0.d), o = W2L(r0.o - pp);
  float a, b, cc, zlo, zhi, bA, bB, bC;
  bool epsLo;
  if (ty == SAIL_CONE) {
    const float h = p.a[3], rad = p.a[4], k = p.a[5];
    a = d.x * d.x + d.y * d.y - k * d.z * d.z;
    b = 2.0f * (d.x * o.x + d.y * o.y - k * d.z * (o.z - h));
    cc = o.x * o.x + o.y * o.y - k * (o.z - h) * (o.z - h);
    zlo = 0.0f; zhi = h; epsLo = true; bA = rad; bB = 0.0f; bC = h;
  } else if (ty == SAIL_CYLINDER) {
    const float h = p.a[3], rad = p.a[4];
    a = d.x * d.x + d.y * d.y;
    b = 2.0f * (d.x * o.x + d.y * o.y);
    cc = o.x * o.x + o.y * o.y - rad * rad;
    zlo = 0.0f; zhi = h; epsLo = true; bA = rad; bB = 0.0f; bC = h;
  } else if (ty == SAIL_HYPERBOLOID) {
    const float ah = p.a[9], ch = p.a[10];
    a = ah * d.x * d.x + ah * d.y * d.y - ch * d.z * d.z;
    b = 2.0f * (ah * d.x * o.x + ah * d.y * o.y - ch * d.z * o.z);
    cc = ah * o.x * o.x + ah * o.y * o.y - ch * o.z * o.z - 1.0f;
    zlo = p.a[12]; zhi = p.a[13]; epsLo = false; bA = p.a[11]; bB = -p.a[12]; bC = p.a[13];
  } else {  // SAIL_PARABOLOID
    const float z0 = p.a[3], z1 = p.a[4], rad = p.a[5];
    const float zMin = fmin_(z0, z1), zMax = fmax_(z0, z1);
    const float k = p.a[6];
    a = k * (d.x * d.x + d.y * d.y);
    b = 2.0f * k * (d.x * o.x + d.y * o.y) - d.z;
    cc = k * (o.x * o.x + o.y * o.y) - o.z;
    zlo = zMin; zhi = zMax; epsLo = false; bA = rad; bB = -zMin; bC = zMax;
  }
  float t1 = 0.0f, t2 = 0.0f, t; V3 hit;
  if (!quadratic(a, b, cc, t1, t2)) return kMaxDistance;
  if (t2 < -kEps) return kMaxDistance;
  if (!rootPick(t1, t2, o, d, zlo, zhi, epsLo, t, hit)) return kMaxDistance;
  if (!testBoundbox(r0, pp - v3(bA, bB, bA), pp + v3(bA, bC, bA))) return kMaxDistance;
  if (hitOut) *hitOut = hit;
  return t;
}
// local-space tail shared by the quadrics and the disk: normal from dpdu x dpdv, texture, back to world
// dpdu is dpduRot(hit) for every caller (z == 0)
D void finishLocal(const Ctx& c, const SailPrim& p, V3 hl, V2 uv, V3 dpdu, V3 dpdv, Hit& h) {
  const V3 nl = normalize(crossZa(dpdu, dpdv));
  h.sc = getSurfaceColor(c, uv, p);
  h.hit = L2W(hl) + P3(p, 0);
  h.normal = L2W(nl);
  h.dpdu = L2W(dpdu);
  h.dpdv = L2W(dpdv);
}
D void coneHit(const Ctx& c, const SailPrim& p, V3 hit, Hit& h) {
  const float hh = p.a[3];
  const V2 uv = needsUV(p) ? v2(fdiv(phiOf(hit.y, hit.x), 2.0f * kPI), fdiv(hit.z, hh)) : v2(0.0f, 0.0f);
  const float vv = fdiv(hit.z, hh);
  const V3 dpdv = v3(fdiv(-hit.x, 1.0f - vv), fdiv(-hit.y, 1.0f - vv), hh);
  finishLocal(c, p, hit, uv, dpduRot(hit), dpdv, h);
}
D void cylinderHit(const Ctx& c, const SailPrim& p, V3 hit, Hit& h) {
  const float hh = p.a[3];
  const V2 uv = needsUV(p) ? v2(fdiv(phiOf(hit.y, hit.x), 2.0f * kPI), fdiv(hit.z, hh)) : v2(0.0f, 0.0f);
  finishLocal(c, p, hit, uv, dpduRot(hit), v3(0.0f, 0.0f, hh), h);
}
D void hypDpD(V3 hit, V3 p1, V3 p2, float phi, V3& dpdu, V3& dpdv) {  // hyperboloid.glsl:41-46
  float sinPhi, cosPhi; sincosf_(phi, sinPhi, cosPhi);
  dpdu = dpduRot(hit);
  dpdv = v3((p2.x - p1.x) * cosPhi - (p2.y - p1.y) * sinPhi, (p2.x - p1.x) * sinPhi + (p2.y - p1.y) * cosPhi, p2.z - p1.z);
}
D void hypHit(const Ctx& c, const SailPrim& p, V3 hit, Hit& h) {
  const V3 p1 = P3(p, 3), p2 = P3(p, 6);
  const float v = fdiv(hit.z - p1.z, p2.z - p1.z);
  const V3 pr = (1.0f - v) * p1 + v * p2;
  const float phi = phiOf(pr.x * hit.y - hit.x * pr.y, hit.x * pr.x + hit.y * pr.y);
  const float u = fdiv(phi, 2.0f * kPI);
  V3 dpdu, dpdv;
  hypDpD(hit, p1, p2, phi, dpdu, dpdv);
  finishLocal(c, p, hit, v2(u, v), dpdu, dpdv, h);
}
D void paraDpD(V3 hit, float zMax, float zMin, V3& dpdu, V3& dpdv) {  // paraboloid.glsl:35-40
  dpdu = dpduRot(hit);
  dpdv = (zMax - zMin) * v3(fdiv(hit.x, 2.0f * hit.z), fdiv(hit.y, 2.0f * hit.z), 1.0f);
}
D void paraHit(const Ctx& c, const SailPrim& p, V3 hit, Hit& h) {
  const float zMin = fmin_(p.a[3], p.a[4]), zMax = fmax_(p.a[3], p.a[4]);
  const V2 uv = needsUV(p) ? v2(fdiv(phiOf(hit.y, hit.x), 2.0f * kPI), fdiv(hit.z - zMin, zMax - zMin)) : v2(0.0f, 0.0f);
  V3 dpdu, dpdv;
  paraDpD(hit, zMax, zMin, dpdu, dpdv);
  finishLocal(c, p, hit, uv, dpdu, dpdv, h);
}
D void diskHit(const Ctx& c, const SailPrim& p, V3 hit, Hit& h) {
  const float rad = p.a[3], ri = p.a[4];
  const float dist2 = hit.x * hit.x + hit.y * hit.y;
  V2 uv = v2(0.0f, 0.0f);
  if (needsUV(p)) {
    const float rHit = sqrtf_(dist2);
    const float oneMinusV = fdiv(rHit - ri, rad - ri);
    uv = v2(fdiv(phiOf(hit.y, hit.x), 2.0f * kPI), 1.0f - oneMinusV);
  }
  const V3 dpdv = v3(hit.x, hit.y, 0.0f) * (ri - rad) / sqrtf_(dist2);
  finishLocal(c, p, hit, uv, dpduRot(hit), dpdv, h);
}
// localHit, the pre-cull kernel's one hit record for the six local-space shapes (sphere, cone, cylinder, hyperboloid, paraboloid,
// disk). Each computes the same tail -- the azimuth phiOf (atan2) of its UV, dpdu = dpduRot(hit), a normalised cross,
// the texture and four local-to-world transforms -- so a wave whose lanes hit different shape types (the pre-cull
// kernel sorts by material, then shape) runs that tail once instead of once per type. Per type only the phi
// arguments, the v coordinate, dpdv and the cross order differ. Same operations on the same values as sphereHit and
// the finishLocal callers above. Measured (bit-identical, profiles/r03_variants_local_shared.jsonl, three rounds):
// pre-cull kernel C4 +3.3 %, C2/C3 unchanged; only its mixed waves +3.2 %; every kernel C4 +3.1 %, C3 -0.8 %.
D void localHit(const Ctx& c, const SailPrim& p, V3 hl, Hit& h) {
  const int ty = p.type;
  const bool nUV = needsUV(p);
  // the azimuth's arguments: (y, x) of the hit, the sphere's pole guard, the hyperboloid's rotated frame
  float py = hl.y, px = hl.x, theta = 0.0f, hv = 0.0f;
  V3 p1 = v3s(0.0f), p2 = v3s(0.0f);
  bool needPhi = nUV;
  if (ty == SAIL_SPHERE) {
    theta = acosf_(clamp_(fdiv(hl.z, p.a[3]), -1.0f, 1.0f));
    if (hl.x == 0.0f && hl.y == 0.0f) px = 1e-5f * p.a[3];
  } else if (ty == SAIL_HYPERBOLOID) {
    p1 = P3(p, 3); p2 = P3(p, 6);
    hv = fdiv(hl.z - p1.z, p2.z - p1.z);
    const V3 pr = (1.0f - hv) * p1 + hv * p2;
    py = pr.x * hl.y - hl.x * pr.y; px = hl.x * pr.x + hl.y * pr.y;
    needPhi = true;
  }
  float phi = 0.0f, u = 0.0f;
  if (needPhi) { phi = phiOf(py, px); u = fdiv(phi, 2.0f * kPI); }
  V2 uv = v2(0.0f, 0.0f);
  const V3 dpdu = dpduRot(hl);
  V3 dpdv, nc;
  switch (ty) {
    case SAIL_SPHERE: {
      const float rad = p.a[3];
      if (nUV) uv = v2(u, fdiv(theta, kPI));
      const float zRadius = sqrtf_(hl.x * hl.x + hl.y * hl.y);
      const float invZRadius = rcp_rn(zRadius);
      const float cosPhi = hl.x * invZRadius, sinPhi = hl.y * invZRadius;
      dpdv = kPI * v3(hl.z * cosPhi, hl.z * sinPhi, -rad * sinf_(theta));
      nc = crossZb(dpdv, dpdu);
      break;
    }
    case SAIL_CONE: {
      const float hh = p.a[3];
      if (nUV) uv = v2(u, fdiv(hl.z, hh));
      const float vv = fdiv(hl.z, hh);
      dpdv = v3(fdiv(-hl.x, 1.0f - vv), fdiv(-hl.y, 1.0f - vv), hh);
      nc = crossZa(dpdu, dpdv);
      break;
    }
    case SAIL_CYLINDER: {
      const float hh = p.a[3];
      if (nUV) uv = v2(u, fdiv(hl.z, hh));
      dpdv = v3(0.0f, 0.0f, hh);
      nc = crossZa(dpdu, dpdv);
      break;
    }
    case SAIL_HYPERBOLOID: {
      uv = v2(u, hv);
      float sinPhi, cosPhi; sincosf_(phi, sinPhi, cosPhi);
      dpdv = v3((p2.x - p1.x) * cosPhi - (p2.y - p1.y) * sinPhi, (p2.x - p1.x) * sinPhi + (p2.y - p1.y) * cosPhi, p2.z - p1.z);
      nc = crossZa(dpdu, dpdv);
      break;
    }
    case SAIL_PARABOLOID: {
      const float zMin = fmin_(p.a[3], p.a[4]), zMax = fmax_(p.a[3], p.a[4]);
      if (nUV) uv = v2(u, fdiv(hl.z - zMin, zMax - zMin));
      dpdv = (zMax - zMin) * v3(fdiv(hl.x, 2.0f * hl.z), fdiv(hl.y, 2.0f * hl.z), 1.0f);
      nc = crossZa(dpdu, dpdv);
      break;
    }
    default: {  // SAIL_DISK
      const float rad = p.a[3], ri = p.a[4];
      const float dist2 = hl.x * hl.x + hl.y * hl.y;
      if (nUV) {
        const float rHit = sqrtf_(dist2);
        const float oneMinusV = fdiv(rHit - ri, rad - ri);
        uv = v2(u, 1.0f - oneMinusV);
      }
      dpdv = v3(hl.x, hl.y, 0.0f) * (ri - rad) / sqrtf_(dist2);
      nc = crossZa(dpdu, dpdv);
      break;
    }
  }
  const V3 nl = normalize(nc);
  h.sc = getSurfaceColor(c, uv, p);
  h.hit = L2W(hl) + P3(p, 0);
  h.normal = L2W(nl);
  h.dpdu = L2W(dpdu);
  h.dpdv = L2W(dpdv);
}

// hl (may be null): the local-space hit point of the shapes whose hit record starts from it
// type: the row's shape id (p.type, or a compile-time constant in a kernel compiled for the scene's rows)
D float primTy(const Ctx& c, int type, const SailPrim& p, const Ray& r, V3* hl) {
  switch (type) {
    case SAIL_CUBE: if (HAS(c.kShapes, SAIL_CUBE)) return cubeT(p, r); break;
    case SAIL_SPHERE: if (HAS(c.kShapes, SAIL_SPHERE)) return sphereT(p, r, hl); break;
    case SAIL_RECTANGLE: if (HAS(c.kShapes, SAIL_RECTANGLE)) return rectT(p, r, hl); break;
    case SAIL_CONE: if (HAS(c.kShapes, SAIL_CONE)) return coneT(p, r, hl); break;
    case SAIL_CYLINDER: if (HAS(c.kShapes, SAIL_CYLINDER)) return cylinderT(p, r, hl); break;
    case SAIL_DISK: if (HAS(c.kShapes, SAIL_DISK)) return diskT(p, r, hl); break;
    case SAIL_HYPERBOLOID: if (HAS(c.kShapes, SAIL_HYPERBOLOID)) return hypT(p, r, hl); break;
    case SAIL_PARABOLOID: if (HAS(c.kShapes, SAIL_PARABOLOID)) return paraT(p, r, hl); break;
    case SAIL_CORNELLBOX: if (HAS(c.kShapes, SAIL_CORNELLBOX)) return cornellT(p, r); break;
    default: break;
  }
  return kMaxDistance;
}
D float primT(const Ctx& c, const SailPrim& p, const Ray& r, V3* hl) { return primTy(c, p.type, p, r, hl); }

// A kernel compiled at run time for the scene's primitive rows (sail_jit.cpp, SAIL_JIT_N > 0) knows their count and
// shape types: the flat sweeps become straight-line code over the rows, each row's intersection test chosen at compile
// time (no per-row type dispatch, no loop). Same operations in the same order as the loops below (measured on the
// Cornell box, tools/study/c1_struct.py: C1 +1.9 %).
#if defined(SAIL_JIT) && SAIL_JIT_N > 0
constexpr int kRows = SAIL_JIT_N;
constexpr int kRowType[SAIL_JIT_N] = {SAIL_JIT_TYPES};
#else
constexpr int kRows = 0;
constexpr int kRowType[1] = {0};
#endif
// the row of the scene's Cornellbox in a kernel compiled for its rows (-1: none)
constexpr int cornellRowOf() {
  for (int i = 0; i < kRows; i++)
    if (kRowType[i] == SAIL_CORNELLBOX) return i;
  return -1;
}
constexpr int kCornellRow = cornellRowOf();
template <int I>
D void sweepRows(const Ctx& c, const Ray& r, float& best, int& bi, V3& bhl) {
  if constexpr (I < kRows) {
    V3 hl = v3s(0.0f);
    const float t = primTy(c, kRowType[I], PRIM(c, I), r, &hl);
    if (t < best) { best = t; bi = I; bhl = hl; }
    sweepRows<I + 1>(c, r, best, bi, bhl);
  }
}
template <int I>
D void closestRows(const Ctx& c, const Ray& r, float& best) {
  if constexpr (I < kRows) {
    const float t = primTy(c, kRowType[I], PRIM(c, I), r, nullptr);
    if (t < best) {
      best = t;
      if (c.shadowAnyHit && best > kEps && best < kOneMinusEps) return;  // as closestT's loop
    }
    closestRows<I + 1>(c, r, best);
  }
}

// Cheap conservative pre-cull: the ray against the primitive's padded bounds in f32 (sail_capi.cpp
// padPrimBounds). It rejects only rays that miss the padded box or enter it beyond the closest distance so
// far (with margin); such a primitive's exact test could only return a miss or a larger distance.
D bool padHit(const SailPrim& p, const Ray& r, float best) {
  const float ix = r.rx, iy = r.ry, iz = r.rz;
  const float x0 = (p.a[18] - r.o.x) * ix, x1 = (p.a[21] - r.o.x) * ix;
  const float y0 = (p.a[19] - r.o.y) * iy, y1 = (p.a[22] - r.o.y) * iy;
  const float z0 = (p.a[20] - r.o.z) * iz, z1 = (p.a[23] - r.o.z) * iz;
  const float tmin = fmax_(fmax_(fmin_(x0, x1), fmin_(y0, y1)), fmin_(z0, z1));
  const float tmax = fmin_(fmin_(fmax_(x0, x1), fmax_(y0, y1)), fmax_(z0, z1));
  return !(tmin > tmax) && !(tmax < 0.0f) && !(tmin > best * 1.0001f + 1e-4f);
}


// ---- candidate sweep (pre-cull kernel) ----------------------------------------------------------------------
// In the uniform sweep a wave runs a primitive's exact test whenever any lane passes its pre-cull; on C4
// (67 primitives, incoherent bounce rays) that is 35 % of the (wave, primitive) pairs with 4.7 of 53 lanes
// passing. Here every lane first collects its candidates of a 64-row chunk into a bit mask (uniform pre-cull
// loop, scalar row reads), then, one shape type at a time, each lane tests its own next candidate of that
// type: the wave runs max-over-lanes iterations instead of one per primitive any lane needs. Candidates are
// visited out of row order, so a hit replaces the best one when it is nearer, or equally near with a lower
// row -- the winner of the in-order "t < best" sweep. Pre-culled rows cannot win (padHit), nor tie.
// Candidate loops without exec-mask nesting (idle lanes test a real row of the type, `take` keeps them out) were
// bit-identical and C4 -0.8 % (the idle lanes' own branches cost more than the saved masking).
// candidate masks built from descending rows shifted into two 32-bit halves (one select + one v_lshl_or per
// row instead of a 64-bit shift, two moves, two selects and two ors): C4 +2.7 %. Packing the x/y slab
// arithmetic of padHit into v_pk_add_f32 / v_pk_mul_f32 was measured at -3.4 %.
// Fused pre-cull form (A.cullPrims == 2): each slab plane as fma(a, R, -RN(o R)), 2 FMAs per axis instead of
// 2 subtractions + 2 multiplies, o R hoisted per ray. Against the plain form each plane moves by at most
// |o| 2^-24 (the host enables it only while that is far inside the padding: sail_capi.cpp cullFmaOk). The
// reciprocals are clamped to +-1e30 first: for an axis-parallel ray (R = +-inf) the plain form gives the
// slab (+-inf, +-inf) while a R - o R would be inf - inf = NaN, which min/max then drop from one side only
// (measured: 1.4 M rays of one C4 frame culled wrongly without the clamp). NaN reciprocals stay NaN.
struct CullRay { float rx, ry, rz, ox, oy, oz; };
D float clampRcp(float v) { return fabsf(v) > 1e30f ? __builtin_copysignf(1e30f, v) : v; }
D CullRay cullRay(const Ray& r) {
  CullRay q;
  q.rx = clampRcp(r.rx); q.ry = clampRcp(r.ry); q.rz = clampRcp(r.rz);
  q.ox = -(r.o.x * q.rx); q.oy = -(r.o.y * q.ry); q.oz = -(r.o.z * q.rz);
  return q;
}
// Mask build in the fused form, B = best * 1.0001 + 1e-4 (> 0) computed once per chunk by the caller. The row's
// outcome is the compare's own lane mask: the bit is
// shifted in by one v_addc (v + v + carry, the carry-in being that lane mask) instead of a select and a v_lshl_or,
// and min(tmax, B) is one v_min_f32 -- the compiler's own fold of the three tests, which re-canonicalised the
// loop-invariant B on every row (tmax and B are arithmetic results, never signalling NaNs, so the plain hardware
// min is the same value). Two fewer VALU per row of the ~20 of each pre-cull test.
D unsigned long long padHitFMask(const SailPrim& p, const CullRay& q, float B) {
  const float x0 = fma_(p.a[18], q.rx, q.ox), x1 = fma_(p.a[21], q.rx, q.ox);
  const float y0 = fma_(p.a[19], q.ry, q.oy), y1 = fma_(p.a[22], q.ry, q.oy);
  const float z0 = fma_(p.a[20], q.rz, q.oz), z1 = fma_(p.a[23], q.rz, q.oz);
  const float tmin = fmax_(fmax_(fmin_(x0, x1), fmin_(y0, y1)), fmin_(z0, z1));
  const float tmax = fmin_(fmin_(fmax_(x0, x1), fmax_(y0, y1)), fmax_(z0, z1));
  float mB;
  __asm__("v_min_f32 %0, %1, %2" : "=v"(mB) : "v"(tmax), "v"(B));
  // !(tmin > tmax) && !(tmin > B) == !(tmin > min(tmax, B)): a NaN tmax leaves B on either side
  return __builtin_amdgcn_ballot_w64(!(tmin > mB)) & __builtin_amdgcn_ballot_w64(!(tmax < 0.0f));
}
D unsigned shiftInMask(unsigned v, unsigned long long laneMask) {
  unsigned r;
  unsigned long long carryOut;
  __asm__("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(carryOut) : "v"(v), "s"(laneMask));
  return r;
}
// one 64-row chunk's candidate mask: descending rows shifted into two 32-bit halves (one v_addc per row in the fused
// form; one select and one v_lshl_or per row in the plain one)
template <bool FUSED>
D unsigned long long chunkMask(const Ctx& c, const Ray& r, const CullRay& q, int base, int cnt, float bound) {
  unsigned lo = 0u, hi = 0u;
  const float B = bound * 1.0001f + 1e-4f;
  if (FUSED) {
    // four rows per step (their bounds requested by scalar loads together, fewer waits; C4 +1.7 %,
    // profiles/r04_cull_unroll.jsonl), the bits shifted in the same descending order as one row per step
    int j = cnt - 1;
    for (; j >= 35; j -= 4) {
      const unsigned long long m0 = padHitFMask(PRIM(c, base + j), q, B), m1 = padHitFMask(PRIM(c, base + j - 1), q, B);
      const unsigned long long m2 = padHitFMask(PRIM(c, base + j - 2), q, B), m3 = padHitFMask(PRIM(c, base + j - 3), q, B);
      hi = shiftInMask(shiftInMask(shiftInMask(shiftInMask(hi, m0), m1), m2), m3);
    }
    for (; j >= 32; j--) hi = shiftInMask(hi, padHitFMask(PRIM(c, base + j), q, B));
    j = (cnt < 32 ? cnt : 32) - 1;
    for (; j >= 3; j -= 4) {
      const unsigned long long m0 = padHitFMask(PRIM(c, base + j), q, B), m1 = padHitFMask(PRIM(c, base + j - 1), q, B);
      const unsigned long long m2 = padHitFMask(PRIM(c, base + j - 2), q, B), m3 = padHitFMask(PRIM(c, base + j - 3), q, B);
      lo = shiftInMask(shiftInMask(shiftInMask(shiftInMask(lo, m0), m1), m2), m3);
    }
    for (; j >= 0; j--) lo = shiftInMask(lo, padHitFMask(PRIM(c, base + j), q, B));
    return ((unsigned long long)hi << 32) | lo;
  }
  for (int j = cnt - 1; j >= 32; j--) hi = (hi << 1) | (padHit(PRIM(c, base + j), r, bound) ? 1u : 0u);
  for (int j = (cnt < 32 ? cnt : 32) - 1; j >= 0; j--) lo = (lo << 1) | (padHit(PRIM(c, base + j), r, bound) ? 1u : 0u);
  return ((unsigned long long)hi << 32) | lo;
}
template <int T> D float typedT(const SailPrim& p, const Ray& r, V3* hl) {
  if constexpr (T == SAIL_CUBE) return cubeT(p, r);
  else if constexpr (T == SAIL_SPHERE) return sphereT(p, r, hl);
  else if constexpr (T == SAIL_RECTANGLE) return rectT(p, r, hl);
  else if constexpr (T == SAIL_CONE) return coneT(p, r, hl);
  else if constexpr (T == SAIL_CYLINDER) return cylinderT(p, r, hl);
  else if constexpr (T == SAIL_DISK) return diskT(p, r, hl);
  else if constexpr (T == SAIL_HYPERBOLOID) return hypT(p, r, hl);
  else if constexpr (T == SAIL_PARABOLOID) return paraT(p, r, hl);
  else if constexpr (T == SAIL_CORNELLBOX) return cornellT(p, r);
  else return kMaxDistance;
}
// HIT = false (shadow rays): only the closest distance is read, so neither the winner's row nor its local hit point
// is kept, and an equally near candidate changes nothing (a tie leaves the distance's value as it is; +-0 compare
// equal and both fail the caller's d > EPSILON). Four fewer live registers in the shadow sweep, where the
// shading state is live.
template <int T, bool HIT>
D void candType(const Ctx& c, const Ray& r, int base, unsigned long long cand, float& best, int& bi, V3& bhl) {
  if (!HAS(c.kShapes, T)) return;
  const unsigned long long tm = constRow<unsigned long long>(c.typeMasks, (base >> 6) * 16 + T);
  unsigned long long m = cand & tm;
  while (__ballot(m != 0ull)) {
    if (m != 0ull) {
      const int i = base + __builtin_ctzll(m);
      m &= m - 1ull;
      const SailPrim& p = c.cprims[i];
      if (HIT) {
        V3 hl = v3s(0.0f);
        const float t = typedT<T>(p, r, &hl);
        if (t < best || (t == best && i < bi)) { best = t; bi = i; bhl = hl; }
      } else {
        const float t = typedT<T>(p, r, nullptr);
        if (t < best) best = t;
      }
    }
  }
}
// the four quadric types' candidates in one loop (quadT)
template <bool HIT>
D void candQuad(const Ctx& c, const Ray& r, int base, unsigned long long cand, float& best, int& bi, V3& bhl) {
  const uint32_t kq = c.kShapes & ((1u << SAIL_CONE) | (1u << SAIL_CYLINDER) | (1u << SAIL_HYPERBOLOID) |
                                   (1u << SAIL_PARABOLOID));
  if (kq == 0u) return;
  const unsigned long long* tms = c.typeMasks + (base >> 6) * 16;
  unsigned long long tm = 0ull;
  if (HAS(kq, SAIL_CONE)) tm |= constRow<unsigned long long>(tms, SAIL_CONE);
  if (HAS(kq, SAIL_CYLINDER)) tm |= constRow<unsigned long long>(tms, SAIL_CYLINDER);
  if (HAS(kq, SAIL_HYPERBOLOID)) tm |= constRow<unsigned long long>(tms, SAIL_HYPERBOLOID);
  if (HAS(kq, SAIL_PARABOLOID)) tm |= constRow<unsigned long long>(tms, SAIL_PARABOLOID);
  unsigned long long m = cand & tm;
  while (__ballot(m != 0ull)) {
    if (m != 0ull) {
      const int i = base + __builtin_ctzll(m);
      m &= m - 1ull;
      const SailPrim& p = c.cprims[i];
      if (HIT) {
        V3 hl = v3s(0.0f);
        const float t = quadT(p, r, &hl);
        if (t < best || (t == best && i < bi)) { best = t; bi = i; bhl = hl; }
      } else {
        const float t = quadT(p, r, nullptr);
        if (t < best) best = t;
      }
    }
  }
}
// limit: the pre-cull distance bound before any hit (kMaxDistance, or 1 for shadow rays: see closestT)
template <bool HIT>
D void candSweep(const Ctx& c, const Ray& r, float limit, float& best, int& bi, V3& bhl) {
  const CullRay q = cullRay(r);
  for (int base = 0; base < c.n; base += 64) {
    const int cnt = c.n - base < 64 ? c.n - base : 64;
    const float bound = fmin_(best, limit);
    const unsigned long long cand =
        c.cullFma ? chunkMask<true>(c, r, q, base, cnt, bound) : chunkMask<false>(c, r, q, base, cnt, bound);
    candType<SAIL_CUBE, HIT>(c, r, base, cand, best, bi, bhl);
    candType<SAIL_CORNELLBOX, HIT>(c, r, base, cand, best, bi, bhl);
    candType<SAIL_RECTANGLE, HIT>(c, r, base, cand, best, bi, bhl);
    candType<SAIL_DISK, HIT>(c, r, base, cand, best, bi, bhl);
    candType<SAIL_SPHERE, HIT>(c, r, base, cand, best, bi, bhl);
    candQuad<HIT>(c, r, base, cand, best, bi, bhl);
  }
}

// closest distance only (shadow rays, testShadow shader.light.js:24-31). The caller only asks whether the
// closest distance lies in (EPSILON, 1 - EPSILON): a primitive whose padded box starts beyond 1 cannot change
// that answer (if it were the closest, every distance would be >= 1 - EPSILON), so the pre-cull bound
// starts at 1 instead of MAX_DISTANCE. Returned distances beyond that bound are not exact.
D float closestT(const Ctx& c, const Ray& r) {
  float best = kMaxDistance;
  if (c.cullPrims && !c.shadowAnyHit) {
    int bi = -1; V3 bhl = v3s(0.0f);
    candSweep<false>(c, r, 1.0f, best, bi, bhl);
    return best;
  }
  if constexpr (kRows > 0) {
    if (!c.cullPrims) {  // compile-time: the flat kernels
      closestRows<0>(c, r, best);
      return best;
    }
  }
  for (int i = 0; i < c.n; i++) {
    if (c.cullPrims && !padHit(PRIM(c, i), r, fmin_(best, 1.0f))) continue;
    const float t = primT(c, PRIM(c, i), r, nullptr);
    if (t < best) {
      best = t;
      if (c.shadowAnyHit && best > kEps && best < kOneMinusEps) break;  // exact: no prim returns t <= EPSILON
    }
  }
  return best;
}

// generated intersectObjects (shader.shape.js:28-51), split in two: one sweep keeps the winner's distance and
// local hit point, then one full record is built for the winner alone
struct Sweep { float best; int bi; V3 bhl; };
// primary: a camera ray, pre-culled only when the eye is near the scene (SailTraceArgs.cullPrimary)
D Sweep sweepRay(const Ctx& c, const Ray& r, bool primary) {
  float best = kMaxDistance;
  int bi = -1;
  V3 bhl = v3s(0.0f);
  const bool cull = c.cullPrims && (!primary || c.cullPrimary);
  if (cull) {
    candSweep<true>(c, r, kMaxDistance, best, bi, bhl);
    Sweep sw; sw.best = best; sw.bi = bi; sw.bhl = bhl;
    return sw;
  }
  if constexpr (kRows > 0) {
    if (!c.cullPrims) {  // compile-time: the flat kernels
      sweepRows<0>(c, r, best, bi, bhl);
      Sweep sw; sw.best = best; sw.bi = bi; sw.bhl = bhl;
      return sw;
    }
  }
  for (int i = 0; i < c.n; i++) {
    V3 hl = v3s(0.0f);
    const float t = primT(c, PRIM(c, i), r, &hl);
    if (t < best) { best = t; bi = i; bhl = hl; }
  }
  Sweep sw; sw.best = best; sw.bi = bi; sw.bhl = bhl;
  return sw;
}
// The winner's local hit point from the ray and its distance: every local-space intersect above ends with
// hit = o + t * d on the same local o and d (W2L of the ray for the quadrics and the disk, the rectangle's frame), so
// this is the sweep's own value bit for bit -- the compacting kernels recompute it instead of moving it through LDS
// (packed path state, traceTileCompact).
D V3 quadLocalHit(const SailPrim& p, const Ray& r, float t) {
  const V3 d = W2L(r.d), o = W2L(r.o - P3(p, 0));
  return o + t * d;
}
D V3 rectLocalHit(const SailPrim& p, const Ray& r, float t) {
  const RectFrame f = rectFrame(p);
  const V3 d = worldToLocal(r.d, f.normal, f.ss, f.ts);
  const V3 o = worldToLocal(r.o - P3(p, 0), f.normal, f.ss, f.ts);
  return o + t * d;
}
// BOXU: the room family's one box record for Cube and Cornellbox (boxHit)
template <bool RECOMP_HL = false, bool BOXU = false>
D Hit hitRecord(const Ctx& c, const Ray& r, const Sweep& sw) {
  const float best = sw.best;
  const int bi = sw.bi;
  Hit h;
  h.d = best;
  // precondition: bi >= 0 is a sweep winner, so its shape is compiled into this kernel (primT returns
  // MAX_DISTANCE for any other row, which never wins): no zero record is needed on any path -- a divergent
  // zero default would be materialised for every lane before the dispatch
  const SailPrim& p = c.rowCopy ? c.cprims[bi] : PRIM(c, bi);
#define BHL (RECOMP_HL ? quadLocalHit(p, r, best) : sw.bhl)
  // compile-time constants: the room kernel's shared box record (boxHit), the pre-cull kernel's shared local-space
  // record (localHit)
  constexpr bool boxU = BOXU;
  const bool localU = c.cullPrims != 0;
  const uint32_t kLocal = c.kShapes & ((1u << SAIL_SPHERE) | (1u << SAIL_CONE) | (1u << SAIL_CYLINDER) |
                                       (1u << SAIL_HYPERBOLOID) | (1u << SAIL_PARABOLOID) | (1u << SAIL_DISK));
  if (boxU && ((HAS(c.kShapes, SAIL_CUBE) && p.type == SAIL_CUBE) ||
               (HAS(c.kShapes, SAIL_CORNELLBOX) && p.type == SAIL_CORNELLBOX))) {
    boxHit(c, p, r, best, h, HAS(c.kShapes, SAIL_CORNELLBOX) && p.type == SAIL_CORNELLBOX);
  } else if (localU && ((kLocal >> p.type) & 1u)) {
    localHit(c, p, BHL, h);
  } else
  switch (p.type) {
    case SAIL_CUBE: if (!boxU && HAS(c.kShapes, SAIL_CUBE)) { cubeHit(c, p, r, best, h); break; } __builtin_unreachable();
    case SAIL_SPHERE: if (!localU && HAS(c.kShapes, SAIL_SPHERE)) { sphereHit(c, p, BHL, h); break; } __builtin_unreachable();
    case SAIL_RECTANGLE: if (HAS(c.kShapes, SAIL_RECTANGLE)) { rectHit(c, p, RECOMP_HL ? rectLocalHit(p, r, best) : sw.bhl, h); break; } __builtin_unreachable();
    case SAIL_CONE: if (!localU && HAS(c.kShapes, SAIL_CONE)) { coneHit(c, p, BHL, h); break; } __builtin_unreachable();
    case SAIL_CYLINDER: if (!localU && HAS(c.kShapes, SAIL_CYLINDER)) { cylinderHit(c, p, BHL, h); break; } __builtin_unreachable();
    case SAIL_DISK: if (!localU && HAS(c.kShapes, SAIL_DISK)) { diskHit(c, p, BHL, h); break; } __builtin_unreachable();
    case SAIL_HYPERBOLOID: if (!localU && HAS(c.kShapes, SAIL_HYPERBOLOID)) { hypHit(c, p, BHL, h); break; } __builtin_unreachable();
    case SAIL_PARABOLOID: if (!localU && HAS(c.kShapes, SAIL_PARABOLOID)) { paraHit(c, p, BHL, h); break; } __builtin_unreachable();
    case SAIL_CORNELLBOX: if (!boxU && HAS(c.kShapes, SAIL_CORNELLBOX)) { cornellHit(p, r, best, h); break; } __builtin_unreachable();
    default: __builtin_unreachable();
  }
#undef BHL
  h.matRow = p.matRow;
  h.emission = v3(p.em[0], p.em[1], p.em[2]);
  // faceObj test (shader.shape.js:47-49) on sgn(rev) * normal: (-n).d is exactly -(n.d) (negated products,
  // round-to-nearest is symmetric), so one dot product serves it and the into test below
  h.axis = c.cullPrims && (p.type == SAIL_CUBE || p.type == SAIL_CORNELLBOX);
  const float nd = h.axis ? dotX(h.normal, r.d) : dot(h.normal, r.d);
  if (!((p.rev ? -nd : nd) < -kEps)) h.emission = v3s(0.0f);
  h.matCategory = matCat(p);
  h.into = nd < -kEps;
  h.nd = nd;
  if (!h.into) h.normal = -h.normal;
  return h;
}
// wave-uniform winner: the same record with the row index in an SGPR (scalar row loads)
template <bool RECOMP_HL = false, bool BOXU = false>
D Hit hitRecordU(const Ctx& c, const Ray& r, const Sweep& sw) {
  const int b0 = __builtin_amdgcn_readfirstlane(sw.bi);
  if (__all(sw.bi == b0)) {
    Sweep su = sw;
    su.bi = b0;
    return hitRecord<RECOMP_HL, BOXU>(c, r, su);
  }
  return hitRecord<RECOMP_HL, BOXU>(c, r, sw);
}

// ---- sampleGeometry for area lights (shader.shape.js:53-67) -----------------------------------------------------
D V3 sampleGeometry(const Ctx& c, V2 u, int row, V3& normal, float& pdf) {
  normal = v3s(0.0f);
  pdf = 0.0f;
  const SailPrim& p = c.rowCopy ? c.cprims[row] : PRIM(c, row);
  const float s = sgn(p.rev);
  switch (p.type) {
    case SAIL_SPHERE: if (!HAS(c.kShapes, SAIL_SPHERE)) break; {
      const V3 q = uniformSampleSphere(u);
      const float rad = p.a[3];
      pdf = fdiv(kInvPI, rad * rad);
      const V3 res = q * rad + P3(p, 0);
      normal = s * (res - P3(p, 0)) / rad;
      return res;
    }
    case SAIL_RECTANGLE: if (!HAS(c.kShapes, SAIL_RECTANGLE)) break; {
      const V3 mn = P3(p, 0), mx = P3(p, 3);
      const V3 x = v3(mx.x - mn.x, 0.0f, 0.0f), y = v3(0.0f, mx.y - mn.y, mx.z - mn.z);
      pdf = p.a[17];                                   // 1 / (length(x) * length(y)), per scene
      const V3 res = mn + x * u.x + y * u.y;
      normal = s * P3(p, 6);                           // normalize(cross(x, y)) == the frame normal
      return res;
    }
    case SAIL_DISK: if (!HAS(c.kShapes, SAIL_DISK)) break; {
      const V2 pd = concentricSampleDisk(u);
      const V3 pp = P3(p, 0);
      const float rad = p.a[3], ri = p.a[4];
      const V3 res = v3(pd.x * rad + pp.x, pp.y, pd.y * rad + pp.z);
      const float area = 2.0f * kPI * 0.5f * (rad * rad - ri * ri);
      pdf = rcp_rn(area);
      normal = s * v3(0.0f, 1.0f, 0.0f);
      return res;
    }
    case SAIL_CUBE: if (HAS(c.kShapes, SAIL_CUBE)) normal = normalForCube(v3s(0.0f), p); return v3s(0.0f);
    case SAIL_CORNELLBOX: if (HAS(c.kShapes, SAIL_CORNELLBOX)) normal = normalForCornellbox(v3s(0.0f), p); return v3s(0.0f);
    case SAIL_CONE: {  // cone.glsl:38-46 at BLACK
      const V3 hit = v3s(0.0f) - P3(p, 0);
      const float h = p.a[3], rad = p.a[4];
      const float tana = fdiv(rad, h);
      const float dd = sqrtf_(hit.x * hit.x + hit.y * hit.y);
      const float x1 = fdiv(dd, tana), x2 = dd * tana;
      normal = s * normalize(hit - v3(0.0f, 0.0f, h - x1 - x2));
      return v3s(0.0f);
    }
    case SAIL_CYLINDER: if (!HAS(c.kShapes, SAIL_CYLINDER)) break; {
      const V3 pp = P3(p, 0);
      normal = s * normalize(v3(0.0f - pp.x, 0.0f - pp.y, 0.0f));
      return v3s(0.0f);
    }
    case SAIL_HYPERBOLOID: if (!HAS(c.kShapes, SAIL_HYPERBOLOID)) break; {
      const V3 hit = v3s(0.0f), p1 = P3(p, 3), p2 = P3(p, 6);
      const float v = fdiv(hit.z - p1.z, p2.z - p1.z);
      const V3 pr = (1.0f - v) * p1 + v * p2;
      const float phi = phiOf(pr.x * hit.y - hit.x * pr.y, hit.x * pr.x + hit.y * pr.y);
      V3 dpdu, dpdv;
      hypDpD(hit, p1, p2, phi, dpdu, dpdv);
      normal = s * L2W(normalize(cross(dpdu, dpdv)));
      return v3s(0.0f);
    }
    case SAIL_PARABOLOID: if (!HAS(c.kShapes, SAIL_PARABOLOID)) break; {
      const float zMin = fmin_(p.a[3], p.a[4]), zMax = fmax_(p.a[3], p.a[4]);
      V3 dpdu, dpdv;
      paraDpD(v3s(0.0f), zMax, zMin, dpdu, dpdv);
      normal = s * L2W(normalize(cross(dpdu, dpdv)));
      return v3s(0.0f);
    }
    default: break;
  }
  return v3s(0.0f);
}

// ---- ssutility.glsl / fresnel.glsl / microfacet.glsl / bsdf.glsl --------------------------------------------------
D float absCosTheta(V3 w) { return fabsf(w.z); }
D float sin2Theta(V3 w) { return fmax_(0.0f, 1.0f - w.z * w.z); }
D float sinTheta(V3 w) { return SQRT01(sin2Theta(w)); }
D float tan2Theta(V3 w) {
  const float cos2T = w.z * w.z;
  if (cos2T < kEps) return kInf;
  return fdiv(sin2Theta(w), cos2T);
}
D float cosPhi(V3 w) { const float st = sinTheta(w); return equalZero(st) ? 1.0f : clamp_(fdiv(w.x, st), -1.0f, 1.0f); }
D float sinPhi(V3 w) { const float st = sinTheta(w); return equalZero(st) ? 0.0f : clamp_(fdiv(w.y, st), -1.0f, 1.0f); }
D bool sameHemisphere(V3 w, V3 wp) { return w.z * wp.z > kEps; }

D float frDielectric(float cosThetaI, float etaI, float etaT) {
  cosThetaI = clamp_(cosThetaI, -1.0f, 1.0f);
  const float sinThetaI = SQRT01(fmax_(0.0f, 1.0f - cosThetaI * cosThetaI));
  const float sinThetaT = fdiv(etaI, etaT) * sinThetaI;
  if (sinThetaT >= 1.0f) return 1.0f;
  const float cosThetaT = SQRT01(fmax_(0.0f, 1.0f - sinThetaT * sinThetaT));
  const float TI = etaT * cosThetaI, IT = etaI * cosThetaT, II = etaI * cosThetaI, TT = etaT * cosThetaT;
  const float Rparl = fdiv(TI - IT, TI + IT), Rperp = fdiv(II - TT, II + TT);
  return fdiv(Rparl * Rparl + Rperp * Rperp, 2.0f);
}
D V3 frConductor(float cosThetaI, V3 etaI, V3 etaT, V3 k) {
  cosThetaI = clamp_(cosThetaI, -1.0f, 1.0f);
  const V3 eta = etaT / etaI, etak = k / etaI;
  const float cosThetaI2 = cosThetaI * cosThetaI, sinThetaI2 = 1.0f - cosThetaI2;
  const V3 eta2 = eta * eta, etak2 = etak * etak;
  const V3 t0 = eta2 - etak2 - sinThetaI2;
  const V3 s = t0 * t0 + 4.0f * eta2 * etak2;
  const V3 a2plusb2 = v3(sqrtf_(s.x), sqrtf_(s.y), sqrtf_(s.z));
  const V3 t1 = a2plusb2 + cosThetaI2;
  const V3 ah = 0.5f * (a2plusb2 + t0);
  const V3 a = v3(sqrtf_(ah.x), sqrtf_(ah.y), sqrtf_(ah.z));
  const V3 t2 = 2.0f * cosThetaI * a;
  const V3 Rs = (t1 - t2) / (t1 + t2);
  const V3 t3 = cosThetaI2 * a2plusb2 + v3s(sinThetaI2 * sinThetaI2);
  const V3 t4 = t2 * sinThetaI2;
  const V3 Rp = Rs * (t3 - t4) / (t3 + t4);
  return 0.5f * (Rp + Rs);
}
// Fresnel: type 0 noop (WHITE), 1 conductor(etaI=WHITE, eta, k), 2 dielectric(1, eta)
struct Fr { int type; V3 eta, k; float etaT; };
D V3 frEvaluate(const Fr& f, float cosThetaI) {
  if (f.type == 2) return v3s(1.0f) * frDielectric(cosThetaI, 1.0f, f.etaT);
  else if (f.type == 1) return frConductor(cosThetaI, v3s(1.0f), f.eta, f.k);
  return v3s(1.0f);
}
D V3 trSampleWh(V2 u, float ax, float ay, V3 wo) {  // microfacet.glsl:41-59
  float cosT = 0.0f, phi = 2.0f * kPI * u.x;
  float sp, cp;  // sin/cos of the final phi: the anisotropic branch has them already
  if (ax == ay) {
    const float tanTheta2 = fdiv(ax * ax * u.x, 1.0f - u.x);
    cosT = rcp_rn(sqrtf_(1.0f + tanTheta2));
    sincosf_(phi, sp, cp);
  } else {
    phi = atanf_(fdiv(ay, ax) * tanf_(kPiOver2 + 2.0f * kPI * u.x));
    if (u.x > 0.5f) phi += kPI;
    float sP, cP; sincosf_(phi, sP, cP);
    const float ax2 = ax * ax, ay2 = ay * ay;
    const float alpha2 = rcp_rn(fdiv(cP * cP, ax2) + fdiv(sP * sP, ay2));
    const float tanTheta2 = fdiv(alpha2 * u.x, 1.0f - u.x);
    cosT = rcp_rn(sqrtf_(1.0f + tanTheta2));
    sp = sP; cp = cP;
  }
  const float sinT = SQRT01(fmax_(0.0f, 1.0f - cosT * cosT));
  V3 wh = v3(sinT * cp, sinT * sp, cosT);
  if (!sameHemisphere(wo, wh)) wh = -wh;
  return wh;
}
D float trD(float ax, float ay, V3 wh) {  // microfacet.glsl:61-67
  const float t2 = tan2Theta(wh);
  if (t2 >= kInf) return 0.001f;
  const float c2 = wh.z * wh.z;
  const float cos4Theta = c2 * c2;
  const float cp = cosPhi(wh), sp = sinPhi(wh);
  const float e = (fdiv(cp * cp, ax * ax) + fdiv(sp * sp, ay * ay)) * t2;
  return rcp_rn(kPI * ax * ay * cos4Theta * (1.0f + e) * (1.0f + e));
}
D float trPdf(float ax, float ay, V3 wh) { return trD(ax, ay, wh) * absCosTheta(wh); }
D V3 microR_f(V3 R, const Fr& fr, float ax, float ay, V3 wo, V3 wi) {  // bsdf.glsl:168-178
  const float cosThetaO = absCosTheta(wo), cosThetaI = absCosTheta(wi);
  V3 wh = wi + wo;
  if (cosThetaI < kEps || cosThetaO < kEps) return v3s(0.0f);
  if (equalZero(wh.x) && equalZero(wh.y) && equalZero(wh.z)) return v3s(0.0f);
  wh = normalize(wh);
  const V3 F = frEvaluate(fr, dot(wi, wh));
  return R * trD(ax, ay, wh) * F / (4.0f * cosThetaI * cosThetaO);
}
D V3 microR_sample(V3 R, const Fr& fr, float ax, float ay, V2 u, V3 wo, V3& wi, float& pdf) {  // :186-196
  if (wo.z < kEps) return v3s(0.0f);
  const V3 wh = trSampleWh(u, ax, ay, wo);
  wi = reflect_(-wo, wh);
  if (!sameHemisphere(wo, wi)) return v3s(0.0f);
  pdf = fdiv(trPdf(ax, ay, wh), 4.0f * dot(wo, wh));
  return microR_f(R, fr, ax, ay, wo, wi);
}
D V3 microT_f(V3 T, float etaB, bool into, float ax, float ay, V3 wo, V3 wi) {  // :205-224 (etaA = 1)
  if (sameHemisphere(wo, wi)) return v3s(0.0f);
  const float cosThetaO = wo.z, cosThetaI = wi.z;
  if (equalZero(cosThetaI) || equalZero(cosThetaO)) return v3s(0.0f);
  const float eta = into ? fdiv(etaB, 1.0f) : rcp_rn(etaB);
  V3 wh = normalize(wo + wi * eta);
  if (wh.z < -kEps) wh = -wh;
  const float Fd = frDielectric(dot(wo, wh), 1.0f, etaB);
  const float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
  return (1.0f - Fd) * T *
         fabsf(fdiv(eta * eta * trD(ax, ay, wh) * fabsf(dot(wi, wh)) * fabsf(dot(wo, wh)),
                    cosThetaI * cosThetaO * sqrtDenom * sqrtDenom));
}
D float microT_pdf(float etaB, bool into, float ax, float ay, V3 wo, V3 wi) {  // :226-235
  if (sameHemisphere(wo, wi)) return 0.001f;
  const float eta = into ? fdiv(etaB, 1.0f) : rcp_rn(etaB);
  const V3 wh = normalize(wo + wi * eta);
  const float sqrtDenom = dot(wo, wh) + eta * dot(wi, wh);
  const float dwh_dwi = fabsf(fdiv(eta * eta * dot(wi, wh), sqrtDenom * sqrtDenom));
  return trPdf(ax, ay, wh) * dwh_dwi;
}
D V3 microT_sample(V3 T, float etaB, bool into, float ax, float ay, V2 u, V3 wo, V3& wi, float& pdf) {
  if (equalZero(wo.z)) return v3s(0.0f);
  const V3 wh = trSampleWh(u, ax, ay, wo);
  const float eta = into ? rcp_rn(etaB) : fdiv(etaB, 1.0f);
  wi = refract_(-wo, wh, eta);
  pdf = microT_pdf(etaB, into, ax, ay, wo, wi);
  return microT_f(T, etaB, into, ax, ay, wo, wi);
}
D V3 orenNayar_f(V3 R, float A, float B, V3 wo, V3 wi) {  // bsdf.glsl:45-66
  const float sinThetaI = sinTheta(wi), sinThetaO = sinTheta(wo);
  float maxCos = 0.0f;
  if (sinThetaI > kEps && sinThetaO > kEps) {
    const float sinPhiI = sinPhi(wi), cosPhiI = cosPhi(wi), sinPhiO = sinPhi(wo), cosPhiO = cosPhi(wo);
    const float dCos = cosPhiI * cosPhiO + sinPhiI * sinPhiO;
    maxCos = fmax_(0.0f, dCos);
  }
  float sinAlpha, tanBeta;
  if (absCosTheta(wi) > absCosTheta(wo)) { sinAlpha = sinThetaO; tanBeta = fdiv(sinThetaI, absCosTheta(wi)); }
  else { sinAlpha = sinThetaI; tanBeta = fdiv(sinThetaO, absCosTheta(wo)); }
  return R * kInvPI * (A + B * maxCos * sinAlpha * tanBeta);
}

// material() (shader.material.js:21-29): returns fpdf; f only for MATTE (the only consumer, path.glsl:10-11)
D V3 material(const Ctx& c, const Hit& ins, V2 u, V3 wo, V3& wi, V3& f) {
  f = v3s(0.0f);
  wi = v3s(0.0f);
  const int cat = ins.matCategory;
  if (cat < 0 || cat >= 32 || !((c.matMask >> cat) & 1u)) return v3s(0.0f);
  const int m = ins.matRow;
  const V3 sc = ins.sc;
  float pdf = 0.0f;
  V3 fs = v3s(0.0f);
  switch (cat) {
    case SAIL_MATTE: if (!HAS(c.kMats, SAIL_MATTE)) break; {  // matte.glsl:8-37
      const float kd = TP(c, m, 1), sigma = TP(c, m, 2), A = TP(c, m, 3), B = TP(c, m, 4);
      const V3 R = kd * sc;
      wi = cosineSampleHemisphere(u);
      pdf = sameHemisphere(wo, wi) ? absCosTheta(wi) * kInvPI : 0.0f;
      if (sigma < kEps) { fs = R * kInvPI; f = (kd * sc) * kInvPI; }
      else { fs = orenNayar_f(R, A, B, wo, wi); f = orenNayar_f(kd * sc, A, B, wo, wi); }
      break;
    }
    case SAIL_MIRROR: if (!HAS(c.kMats, SAIL_MIRROR)) break; {  // mirror.glsl:5-17, specular_r_sample_f bsdf.glsl:93-98
      const float kr = TP(c, m, 1);
      const V3 R = kr * sc;
      wi = v3(-wo.x, -wo.y, wo.z);
      pdf = 1.0f;
      fs = v3s(1.0f) * R / absCosTheta(wi);
      break;
    }
    case SAIL_METAL: if (!HAS(c.kMats, SAIL_METAL)) break; {  // metal.glsl:8-22
      Fr fr; fr.type = 1; fr.eta = TP3(c, m, 3); fr.k = TP3(c, m, 6); fr.etaT = 0.0f;
      fs = microR_sample(sc, fr, TP(c, m, 1), TP(c, m, 2), u, wo, wi, pdf);
      break;
    }
    case SAIL_GLASS: if (!HAS(c.kMats, SAIL_GLASS)) break; {  // glass.glsl:10-36
      const float kr = TP(c, m, 1), kt = TP(c, m, 2), eta = TP(c, m, 3), ur = TP(c, m, 4), vr = TP(c, m, 5);
      if (ur < kEps && vr < kEps) {  // specular_fr_sample_f bsdf.glsl:141-158
        const float Fd = frDielectric(wo.z, 1.0f, eta);
        if (u.x < Fd) {
          wi = v3(-wo.x, -wo.y, wo.z);
          pdf = 1.0f;
          fs = (kr * sc) / absCosTheta(wi);
        } else {
          const float etaI = ins.into ? 1.0f : eta, etaT = ins.into ? eta : 1.0f;
          wi = refract_(-wo, v3(0.0f, 0.0f, 1.0f), fdiv(etaI, etaT));
          const V3 ft = (kt * sc) * (1.0f - Fd);
          pdf = 1.0f;
          fs = ft / absCosTheta(wi);
        }
      } else {
        const float p = u.x;
        V2 uu = u;
        uu.x = fmin_(u.x * 2.0f - 1.0f, kOneMinusEps);
        if (p < 0.5f) {
          Fr fr; fr.type = 2; fr.etaT = eta; fr.eta = v3s(0.0f); fr.k = v3s(0.0f);
          fs = microR_sample(kr * sc, fr, ur, vr, uu, wo, wi, pdf);
        } else {
          fs = microT_sample(kt * sc, eta, ins.into, ur, vr, uu, wo, wi, pdf);
        }
      }
      break;
    }
    default: break;
  }
  return fs * absCosTheta(wi) / pdf;
}

// ---- lights (shader.light.js:12-22, light/*.glsl) ---------------------------------------------------------------
// (one uniformSampleSphere shared by point lights and sphere area lights was bit-identical and C4 -0.35 %,
// profiles/r03_variants_light_shared.jsonl: the extra light-row read cost more than the second evaluation)
D bool testShadow(const Ctx& c, const Ray& r) {
  const float d = closestT(c, r);
  return d > kEps && d < kOneMinusEps;
}
// The light categories only differ in how they build the shadow ray and the unoccluded contribution; the
// shadow sweep itself (the expensive part) is shared, so a wave whose lanes picked different light kinds
// runs one sweep instead of one per kind. Contribution and visibility are independent pure functions of the
// same inputs, so evaluating the contribution first changes no bit.
// lightPrep: everything of light_sample but its shadow test -- whether the sample is lit, its unoccluded
// contribution and the shadow ray (from the hit point along the unnormalised toLight)
struct LightPrep { bool lit; V3 contrib, toLight; };
D LightPrep lightPrep(const Ctx& c, const Hit& ins, V2 u2) {
  LightPrep lp;
  lp.lit = false; lp.contrib = v3s(0.0f); lp.toLight = v3s(0.0f);
  // randomInt(seed,0,ln) = int(random2(seed).x * ln): the same hash as the BSDF sample's first component
  if (c.kLights == 0) return lp;                              // no light plugin compiled in
  const int index = to_int(u2.x * (float)c.ln);
  if (c.ln <= 0) return lp;
  const int catRow = (index <= 0) ? 0 : c.ln - 1;           // readInt(lights, vec2(0, index)) : integer row coord
  const int cat = to_int(c.lt[catRow * 18]);
  if (cat < 0 || cat >= 32 || !((c.lightMask >> cat) & 1u)) return lp;
  const int row = (c.ln == 1) ? 0 : (index < 0 ? 0 : (index > c.ln - 1 ? c.ln - 1 : index));
  const float* L = c.lt + row * 18;
  V3 contrib = v3s(0.0f), toLight = v3s(0.0f);
  bool lit = false;
  if (cat == SAIL_AREA && HAS(c.kLights, SAIL_AREA)) {  // light/area.glsl
    const V3 em = v3(L[2], L[3], L[4]);
    V3 normal; float pdf;
    const V3 p = sampleGeometry(c, u2, c.lightObjRow[row], normal, pdf);
    toLight = p - ins.hit;
    const V3 nt = normalize(toLight);
    contrib = em * fmax_(0.0f, dot(normal, -nt)) * fmax_(0.0f, dot(nt, ins.normal)) / pdf;
    lit = true;
  } else if (cat == SAIL_POINT && HAS(c.kLights, SAIL_POINT)) {  // light/point.glsl:13-20
    const V3 from = v3(L[1], L[2], L[3]), em = v3(L[4], L[5], L[6]);
    const V3 p = from + uniformSampleSphere(u2) * 0.1f;
    toLight = p - ins.hit;
    contrib = em * fmax_(0.0f, dot(normalize(toLight), ins.normal));
    lit = true;
  } else if (cat == SAIL_SPOT && HAS(c.kLights, SAIL_SPOT)) {  // light/spot.glsl
    const float ctw = L[1], cfs = L[2];
    const V3 from = v3(L[3], L[4], L[5]), em = v3(L[6], L[7], L[8]);
    toLight = from - ins.hit;
    const V3 nt = normalize(toLight);
    const float d = length(toLight);
    float fall;
    {  // falloff spot.glsl:17-27 with w = -normToLight
      const float cT = -(-nt).y;
      if (cT < ctw) fall = 0.0f;
      else if (cT >= cfs) fall = 1.0f;
      else { const float delta = fdiv(cT - ctw, cfs - ctw); const float d2 = delta * delta; fall = d2 * d2; }
    }
    contrib = em * fall * fmax_(0.0f, dot(normalize(toLight), ins.normal)) / (d * d);
    lit = true;
  }
  lp.lit = lit; lp.contrib = contrib; lp.toLight = toLight;
  return lp;
}
// Dead shadow tests: a light sample whose unoccluded contribution is exactly +0 in every channel (the sample behind
// the surface or the light facing away, a spot light's falloff 0) returns that +0 vector whether or not its shadow
// ray is blocked, so the shadow sweep is skipped; any other value (-0, NaN, a nonzero channel) takes the sweep
D bool posZero3(const V3& v) {
  return (__float_as_uint(v.x) | __float_as_uint(v.y) | __float_as_uint(v.z)) == 0u;
}
D V3 lightSample(const Ctx& c, const Hit& ins, V2 u2) {
  const LightPrep lp = lightPrep(c, ins, u2);
  if (!lp.lit) return v3s(0.0f);
  if (posZero3(lp.contrib)) return v3s(0.0f);
  // testShadow(Ray(hit, toLight)) (shader.light.js:24-31): unnormalised direction, no origin offset
  if (testShadow(c, mkRay(ins.hit, lp.toLight))) return v3s(0.0f);
  return lp.contrib;
}

// The path's final bounce: only its radiance is read afterwards (the throughput and the next ray are dead), so the
// BSDF sample is needed there only for f -- the light term's weight, which a matte surface alone sets -- and a
// Lambertian matte f (kd * sc / pi, matte.glsl) does not depend on the sample. shadeLast adds that bounce's
// radiance without the shading frame, BSDF sample or next ray, by the same expression on the same values as
// shadeBounce; it declines (false) for an Oren-Nayar matte, whose f needs the sampled direction, and for any matte
// path when a light plugin is compiled in (its light sample and shadow sweep stay in shadeBounce alone: a second
// inlined shadow sweep multiplied the pre-cull kernel's spills).
// Measured bit-identical: C2 +4.2 %, C3 +2.6 %, C4 -0.6 % (its 12-bounce paths are mostly matte with lights, which
// decline), so every kernel but the pre-cull one takes it.
D bool shadeLast(const Ctx& c, const Hit& ins, float seed, const V3& fpdf, V3& e) {
  const bool matteLit = isBlack(ins.emission) && ins.matCategory == SAIL_MATTE;  // path.glsl:10-11
  if (matteLit && c.kLights != 0) return false;
  V3 f = v3s(0.0f);
  // material()'s matte branch (the plugin in the scene and compiled in)
  if (matteLit && ((c.matMask >> SAIL_MATTE) & 1u) && HAS(c.kMats, SAIL_MATTE)) {
    const float kd = TP(c, ins.matRow, 1), sigma = TP(c, ins.matRow, 2);
    if (!(sigma < kEps)) return false;
    f = (kd * ins.sc) * kInvPI;
  }
  (void)seed;
  V3 direct = v3s(0.0f);
  if (matteLit)  // no light plugin: lightSample is 0, and 0 + 0 * f == fma(f, 0, 0) bit for bit
    direct = v3(fma_(f.x, 0.0f, 0.0f), fma_(f.y, 0.0f, 0.0f), fma_(f.z, 0.0f, 0.0f));
  const V3 sh = ins.emission + direct;
  e = e + sh * fpdf;
  return true;
}

// ---- path.glsl:1-38 ------------------------------------------------------------------------------------------------
// shade() (path.glsl:1-14) + the bounce bookkeeping of trace() (path.glsl:27-36): radiance, throughput, next ray
// A lit matte path's light sample whose shadow test is left to a later pass (the wavefront split, SAIL_DEBUG_WAVEFRONT):
// everything the radiance update e += (emission + light * f) * fpdf needs once the shadow ray's answer is known
// e holds the dark outcome of the radiance update (the light blocked); eLit the unblocked one, to be taken when the
// shadow ray from `hit` along `toLight` is not blocked. Both are shadeBounce's e += (emission + (0 + light * f)) * fpdf.
struct ShadowPending { bool pending; V3 toLight, hit, eLit; };
// DEFER: a lit matte path's shadow ray is handed to onShadow(hit, toLight, eLit) where it is made (so that nothing of it
// stays live through the rest of the bounce) and e takes the blocked outcome
template <bool DEFER, class OnShadow>
D void shadeBounceT(const Ctx& c, const Hit& ins, Ray& ray, float seed, V3& fpdf, V3& e, PhaseClock& pc, OnShadow&& onShadow);
D void shadeBounce(const Ctx& c, const Hit& ins, Ray& ray, float seed, V3& fpdf, V3& e, PhaseClock& pc) {
  shadeBounceT<false>(c, ins, ray, seed, fpdf, e, pc, [](const V3&, const V3&, const V3&) {});
}
// the deferred shadow ray into a ShadowPending (the pre-cull kernel's compacted shadow rays, the wavefront split)
D void shadeBounceP(const Ctx& c, const Hit& ins, Ray& ray, float seed, V3& fpdf, V3& e, PhaseClock& pc, ShadowPending& sp) {
  sp.pending = false;
  shadeBounceT<true>(c, ins, ray, seed, fpdf, e, pc, [&](const V3& hit, const V3& toLight, const V3& eLit) {
    sp.pending = true; sp.hit = hit; sp.toLight = toLight; sp.eLit = eLit;
  });
}
template <bool DEFER, class OnShadow>
D void shadeBounceT(const Ctx& c, const Hit& ins, Ray& ray, float seed, V3& fpdf, V3& e, PhaseClock& pc, OnShadow&& onShadow) {
  {
    // shade()
    // box faces have axis-aligned unit dpdu: dot == 1 exactly, sqrt(1) == 1 and v / 1 == v bit for bit
    // worldToLocal(-ray.d, normal, ss, ts): its z is dot(-d, +-n) = -+(n.d) exactly (negated products, symmetric
    // rounding), already known from the hit record's into test
    const V3 nd3 = -ray.d;
    V3 ss, ts, wo;
    if (ins.axis) {  // box face: unit dpdu (ss = dpdu, as below), exact products
      ss = ins.dpdu;
      ts = crossX(ins.normal, ss);
      wo = v3(dotX(nd3, ss), dotX(nd3, ts), ins.into ? -ins.nd : ins.nd);
    } else {
      const float dd = dot(ins.dpdu, ins.dpdu);
      ss = (dd == 1.0f) ? ins.dpdu : ins.dpdu / sqrtf_(dd);
      ts = cross(ins.normal, ss);
      wo = v3(dot(nd3, ss), dot(nd3, ts), ins.into ? -ins.nd : ins.nd);
    }
    // the hash is evaluated only for materials that consume it (matte/metal/glass; mirror is deterministic)
    PHASE_MARK(pc, 2);  // shading frame
    const V2 u2 = (ins.matCategory != SAIL_MIRROR) ? random2(c, seed) : v2(0.0f, 0.0f);
    PHASE_MARK(pc, 3);  // hash RNG
    V3 wiL, f;
    const V3 mat = material(c, ins, u2, wo, wiL, f);
    const V3 _fpdf = vclamp01(mat);
    const V3 wi = ins.axis ? localToWorldX(wiL, ins.normal, ss, ts) : localToWorld(wiL, ins.normal, ss, ts);
    PHASE_MARK(pc, 4);  // BSDF sample
    V3 direct = v3s(0.0f);
    if (isBlack(ins.emission) && ins.matCategory == SAIL_MATTE) {
      if (c.kLights == 0) {  // no light plugin: lightSample is 0, and 0 + 0 * f == fma(f, 0, 0) bit for bit
        direct = v3(fma_(f.x, 0.0f, 0.0f), fma_(f.y, 0.0f, 0.0f), fma_(f.z, 0.0f, 0.0f));
      } else if (DEFER) {  // lightSample's light prep now; its shadow test later picks one of the two outcomes
        const LightPrep lp = lightPrep(c, ins, u2);
        if (lp.lit && !posZero3(lp.contrib)) {
          V3 dLit = v3s(0.0f);
          dLit = dLit + lp.contrib * f;
          onShadow(ins.hit, lp.toLight, e + (ins.emission + dLit) * fpdf);
        }
        direct = direct + v3s(0.0f) * f;  // the dark outcome (light 0), or no shadow ray at all
      } else {
        direct = direct + lightSample(c, ins, u2) * f;
      }
    }
    PHASE_MARK(pc, 5);  // light sample + shadow ray
    {
      const V3 sh = ins.emission + direct;
      e = e + sh * fpdf;
    }
    fpdf = fpdf * _fpdf;
    const float outdot = ins.axis ? dotX(ins.normal, wi) : dot(ins.normal, wi);
    ray = mkRay(ins.hit + ins.normal * (outdot > kEps ? 0.0001f : -0.0001f), wi);
    PHASE_MARK(pc, 6);  // next ray
  }
}

D float q8(float v) {
  v = clamp_(v, 0.0f, 1.0f);
  return floorf(v * 255.0f + 0.5f) / 255.0f;
}
// fstrace.glsl:13 accumulation of one sample (SUM: running sums + count; MIX / COMPAT8: the reference's
// mix(e, cache, k/(k+1)), COMPAT8 through the UNORM8 frame store)
D void accumulateSample(float4& acc, V3 e, const SailSample& S, int mode) {
  if (mode == 0) {
    acc.x += e.x; acc.y += e.y; acc.z += e.z; acc.w += 1.0f;
  } else {
    const float w = S.mixw;
    float mx = e.x * (1.0f - w) + acc.x * w, my = e.y * (1.0f - w) + acc.y * w, mz = e.z * (1.0f - w) + acc.z * w;
    if (mode == 2) { mx = q8(mx); my = q8(my); mz = q8(mz); }
    acc.x = mx; acc.y = my; acc.z = mz; acc.w = 1.0f;
  }
}
// the workgroup's 16x16 block and sample range: blockIdx.x = group * (ownedTiles * 16) + block. Ungrouped
// launches (one workgroup per block, every sample) are a separate compile-time instance, so they carry none of
// the group bookkeeping in registers (sample groups add VGPR/SGPR spills to the flat kernels otherwise).
struct TileWork { int ownedTile, sub, kBeg, kEnd, bid; };
// A workgroup's pixel block: PX pixels (NT threads / NS samples in flight per pixel), BW x BH, 4096 / PX per 64x64 tile:
// 16 x NT/16 strips with one sample in flight (NT = 256: 16 x 16; the pre-cull kernels' 1,024: 16 x 64), square blocks
// otherwise (8 x 8 or 4 x 4 pixels x 4 or 16 samples)
template <int PX> struct BlockGeo {
  static constexpr int kBW = PX >= 128 ? 16 : (PX >= 32 ? 8 : 4);
  static constexpr int kBH = PX / kBW;
  static constexpr int kPerRow = 64 / kBW;  // blocks per tile row
  static constexpr int kPer = 4096 / PX;     // blocks per tile
  static_assert(kBW * kBH == PX && PX >= 16 && 4096 % PX == 0 && kBW * kPerRow == 64, "pixel block shape");
};
template <bool GROUPED, int PX = 256>
D TileWork tileWork(const SailTraceArgs& A) {
  constexpr int kPer = BlockGeo<PX>::kPer;
  TileWork w;
  if (GROUPED) {
    const int nb = A.ownedTiles * kPer;
    const int bid = (int)blockIdx.x % nb, group = (int)blockIdx.x / nb;
    w.bid = bid;
    w.kBeg = group * A.groupSpp;
    w.kEnd = w.kBeg + A.groupSpp < A.spp ? w.kBeg + A.groupSpp : A.spp;
  } else {
    w.bid = (int)blockIdx.x;
    w.kBeg = 0;
    w.kEnd = A.spp;
  }
  w.ownedTile = w.bid / kPer; w.sub = w.bid % kPer;
  return w;
}
// The staged radiance of sample k at pixel p of block bid (groups after the first; the first group, which holds
// the launch's first samples, adds its own to the accumulator directly): stage planes 3k..3k+2, in the slot order
// sail_accum_kernel reads -- slot (ownedTile * 16 + block16) * 256 + (y mod 16) * 16 + (x mod 16) -- whatever the block
template <int PX = 256>
D void stageSample(const SailTraceArgs& A, int k, int bid, int p, V3 e) {
  using G = BlockGeo<PX>;
  size_t slot;
  if (PX == 256 && G::kBW == 16) {
    slot = (size_t)bid * 256 + p;
  } else {
    const int ownedTile = bid / G::kPer, sub = bid % G::kPer;
    const int ly = (sub / G::kPerRow) * G::kBH + p / G::kBW, lx = (sub % G::kPerRow) * G::kBW + p % G::kBW;
    slot = ((size_t)ownedTile * 16 + (size_t)((ly >> 4) * 4 + (lx >> 4))) * 256 + (size_t)((ly & 15) * 16 + (lx & 15));
  }
  // three planes per sample (12 B per pixel instead of a float4's 16)
  float* const st = A.stage + (size_t)k * 3u * (size_t)A.stageStride + slot;
  st[0] = e.x;
  st[A.stageStride] = e.y;
  st[2 * A.stageStride] = e.z;
}

}  // namespace

// Path compaction: after every primitive sweep the workgroup's 256 live paths are sorted through LDS by
// (shape type, material) so that the hit record and the shading, the divergent half of a bounce, run on
// waves of like paths; dead paths drop out, so whole waves idle past the end of the live range. A path's
// state (ray, throughput, radiance, pixel, sweep result: 18 words) migrates between lanes; every path's
// arithmetic is unchanged, so the result is bit-identical to the unsorted kernel. The radiance of a sample
// goes back to the pixel's own lane through LDS before it is accumulated, in sample order.
// The sort key is the winning primitive row for scenes of fewer than 64 rows, else (material, shape) material-major:
// matte paths, which alone run the light sample and its shadow sweep, share waves (C4 +5.2 %; ordering the by-row key
// the same way through a host rank table: C3 -2.8 %).
// After the sort, a wave whose live paths have different sort keys runs at issue priority kPrioMixed (C3 +7.3 %).
// Path state moves through LDS packed: three float4 per path in the flat kernels (ds_*_b128), six float2 in the
// pre-cull kernel (ds_*_b64), the local hit point recomputed; the flat kernels keep each pixel's radiance as one float4
// (measured with priority 2, Gseg/s C1 / C3 / C4: six float2 89.6 / 29.0 / 9.40, three float4 90.0 / 29.0 / 9.10,
// + float4 radiance 90.1 / 29.15 / 9.10 and 90.3 / 29.15 / 9.10; unpacked, no priority 86.0 / 26.3 / 9.04).
// The sort's prefix sum over the key counts is six DPP adds (sail_scan.h).
// Barriers per bounce: two in the pre-cull and room kernels (every wave scans double-buffered counts itself), three in
// the Cornell kernel (one wave scans). Bit-identical; with the DPP scan and the live count by readlane C2 -1.0 % with
// two, C3 +1.1 % (twice), C4 +1.3-1.7 %. Deferring each sample's read-back past the next sample's first barrier (no
// end-of-sample barriers) was bit-identical and slower: C2 -2.3 %, C3 -6.6 %, C4 -2.2 %.
// The pre-cull kernel copies scenes of at most kCullLdsRows rows into LDS per workgroup, and its candidate loops, hit
// record and light sampler read their per-lane rows from there (C4 +4.3 %), with texParams tables of at most
// kCullLdsTp rows as well (+8.8 % together). 72 + 136 rows keep the block at 79.9 KB: two 1,024-thread workgroups per
// CU. The same copies in the flat kernels lost (C2 -6 %, C3 +-0).
// Compacted shadow rays (pre-cull kernel): lit matte paths leave their shadow rays in the sort buffer (compacted, after
// a barrier that ends the bounce's gathers) and the workgroup's first threads trace them, so waves whose lanes have no
// shadow ray (non-matte, unlit, contribution +0) do no shadow sweep; the radiance slot holds the shadowed outcome until
// the tracing thread writes the lit one. Measured (gpurun_out/r03m, bit-identical): C4 +3.1 % (spills 74 -> 105
// VGPRs); in the room kernel C3 -25 % (its spills 41 -> 85).
// NT threads per workgroup: a 16 x NT/16 pixel block, 4096/NT blocks per 64x64 tile. A larger workgroup sorts a
// larger pool of paths (fewer mixed waves) at the price of a wider barrier.
constexpr int kCullLdsRows = SAIL_CULL_LDS_ROWS, kCullLdsTp = SAIL_CULL_LDS_TP;
// A pre-cull kernel compiled at run time for a scene whose tables fit (SAIL_JIT_LDSFIT) copies them unconditionally:
// the per-lane row and texParams pointers are then known to point into LDS, so those reads are ds_read instead of flat
// loads, which also wait on every outstanding vector-memory load, scratch reloads included (C4 +3.1 %,
// profiles/r04_cull_ldsfit.jsonl).
#if defined(SAIL_JIT) && SAIL_JIT_LDSFIT
constexpr bool kLdsFitAll = true;
#else
constexpr bool kLdsFitAll = false;
#endif
// A flat kernel compiled for the scene's rows (kRows > 0) and its texParams row count (SAIL_JIT_TN > 0, at most 32 so
// that the Cornell form keeps 8 workgroups per CU) copies both tables into LDS the same way: the per-lane row reads of
// mixed waves' hit records and the material / texture reads become ds_read, off the counter the scratch reloads wait
// on (C3 +2.8 %, UI +2.2 %, profiles/r04_flat_lds.jsonl; the host asks for it in the room form only: the Cornell form
// measured -0.5 %). Round 3's flat-kernel copies were conditional (flat loads) and lost.
#if defined(SAIL_JIT) && defined(SAIL_JIT_TN) && SAIL_JIT_TN > 0
constexpr int kFlatTp = SAIL_JIT_TN;
#else
constexpr int kFlatTp = 0;
#endif
constexpr int kPrioMixed = 2;
// NS samples of each pixel in flight per workgroup (1, 4 or 16): the workgroup's NT lanes hold NT / NS pixels x NS samples
// (lane li: sample slot li / PX of pixel li % PX), so one workgroup finishes a launch's samples of its block NS times
// sooner. The short units end a launch with a short tail without splitting the samples over workgroups (sample groups:
// every sample's radiance staged in HBM and added in order by sail_accum_kernel); each pixel's NS radiances of a step
// wait in LDS and its lane adds them in sample order, so the sums are those of one sample at a time, bit for bit.
template <bool CULL, bool GROUPED, uint32_t KS, uint32_t KM, uint32_t KT, uint32_t KL, int NT, bool FAM, int NS = 1>
__device__ __forceinline__ void traceTileCompact(const SailTraceArgs& A) {
  static_assert(NT == 128 || NT == 256 || NT == 512 || NT == 1024, "workgroups of 2, 4, 8 or 16 waves");
  static_assert(NS == 1 || NS == 4 || NS == 16, "samples in flight");
  constexpr int kPX = NT / NS;  // pixels per workgroup
  using G = BlockGeo<kPX>;
  constexpr int kKeys = 64;                // key = 1 + type * 5 + material category (types 0..9) < 64
  constexpr int kPack = CULL ? 1 : 2;
  constexpr bool kE4 = !CULL;
  // packed path state, 2: three float4 per path -- ray o + d.x, d.yz + throughput.xy, throughput.z + distance +
  // pixel | row << 10 + key (ds_write_b128 / ds_read_b128: 3 + 3 LDS instructions instead of 15 + 15); 1: six
  // float2 (ds_*_b64); the local hit point is recomputed (hitRecord<true>). The unused form is one element.
  __shared__ float4 sSt4[kPack == 2 ? 3 : 1][kPack == 2 ? NT : 1];
  __shared__ float2 sSt2[kPack == 1 ? 6 : 1][kPack == 1 ? NT : 1];
  // each pixel's radiance: one float4 (one ds_read_b128 / ds_write_b128) or three floats
  __shared__ float4 sE4[kE4 ? NT : 1];
  __shared__ float sE[kE4 ? 1 : 3][kE4 ? 1 : NT];
  auto E_LOAD = [&](int i) -> V3 {
    if constexpr (kE4) return v3(sE4[i].x, sE4[i].y, sE4[i].z);
    else return v3(sE[0][i], sE[1][i], sE[2][i]);
  };
  auto E_STORE = [&](int i, const V3& v) {
    if constexpr (kE4) sE4[i] = make_float4(v.x, v.y, v.z, 0.0f);
    else { sE[0][i] = v.x; sE[1][i] = v.y; sE[2][i] = v.z; }
  };
  constexpr bool kShCompact = CULL && KL != 0u;
  __shared__ int sShCnt[2];
  int shph = 0;
  constexpr bool twoBar = CULL || FAM;
  constexpr bool kSort1 = CULL || FAM;  // sort the paths at the first bounce too
  __shared__ int sCnt2[twoBar ? 2 : 1][kKeys];  // [0] alone in the three-barrier sort
  __shared__ int sStart[twoBar ? 1 : kKeys + 1];
  const TileWork tw = tileWork<GROUPED, kPX>(A);
  const int ownedTile = tw.ownedTile;
  if (ownedTile >= A.ownedTiles) return;  // uniform over the workgroup
  const int sub = tw.sub;
  const int tile = A.rank + ownedTile * A.world;
  const int tx = tile % A.tilesX, ty = tile / A.tilesX;
  const int li = threadIdx.x, lane = li & 63, wave = li >> 6;
  const int x0 = tx * 64 + (sub % G::kPerRow) * G::kBW, y0 = ty * 64 + (sub / G::kPerRow) * G::kBH;
  // a path's home slot (the lane it started on) names its pixel and its sample slot
  auto homeX = [&](int h) { return x0 + (h % kPX) % G::kBW; };
  auto homeY = [&](int h) { return y0 + (h % kPX) / G::kBW; };
  const int mySlot = li / kPX;
  const int x = homeX(li), y = homeY(li);
  const bool valid = x < A.W && y < A.H;   // ragged tiles: invalid lanes still serve migrated paths

  Ctx c;
  c.tp = A.texparams; c.lt = A.lights; c.lightObjRow = A.lightObjRow; c.typeMasks = A.typeMasks;
  c.prims = A.prims;
  c.cprims = A.prims;
  c.tpl = A.texparams;
  c.rowCopy = false;
  c.tpCopy = false;
  c.n = A.n; c.tn = A.tn; c.ln = A.ln;
  c.matMask = A.matMask; c.texMask = A.texMask; c.lightMask = A.lightMask;
  c.fcx = 0.0f; c.fcy = 0.0f;
  c.shadowAnyHit = A.shadowAnyHit;
  c.cullPrims = CULL ? 1 : 0;
  c.cullFma = CULL && A.cullPrims == 2;
  c.cullPrimary = A.cullPrimary;
  c.kShapes = KS; c.kMats = KM; c.kTex = KT; c.kLights = KL;

  if (li < (twoBar ? 2 : 1) * kKeys) sCnt2[li / kKeys][li % kKeys] = 0;
  if (li < 2) sShCnt[li] = 0;
  // the pre-cull kernel's candidate loops, hit record and light sampler read rows per lane: from an LDS copy of the
  // scene when it fits
  constexpr int kLdsRows = CULL ? kCullLdsRows : (!CULL && kFlatTp > 0 && kRows > 0 ? kRows : 0);
  c.rowCopy = kLdsRows > 0;
  __shared__ float4 sPrimL[kLdsRows > 0 ? kLdsRows * (int)(sizeof(SailPrim) / 16) : 1];
  constexpr bool kFlatLds = !CULL && kFlatTp > 0 && kRows > 0;
  if constexpr (kLdsFitAll) {
    if (A.n > kLdsRows || A.tn > kCullLdsTp) return;  // never launched so (sail_capi.cpp jitKernels); uniform
  }
  if constexpr (kFlatLds) {
    if (A.n != kRows || A.tn != kFlatTp) return;  // never launched so (sail_capi.cpp jitKernels); uniform
  }
  if constexpr (kLdsRows > 0) {
    if (kLdsFitAll || kFlatLds || A.n <= kLdsRows) {  // uniform
      const float4* src = reinterpret_cast<const float4*>(A.prims);
      const int nv = A.n * (int)(sizeof(SailPrim) / 16);
      for (int i = li; i < nv; i += NT) sPrimL[i] = src[i];
      c.cprims = reinterpret_cast<const SailPrim*>(sPrimL);
    }
  }
  constexpr int kLdsTp = CULL ? kCullLdsTp : (!CULL && kFlatTp > 0 && kRows > 0 ? kFlatTp : 0);
  c.tpCopy = kLdsTp > 0;
  __shared__ float4 sTpL[kLdsTp > 0 ? kLdsTp * 4 : 1];
  if constexpr (kLdsTp > 0) {
    if (kLdsFitAll || kFlatLds || A.tn <= kLdsTp) {  // uniform
      const float4* src = reinterpret_cast<const float4*>(A.texparams);
      for (int i = li; i < A.tn * 4; i += NT) sTpL[i] = src[i];
      c.tpl = reinterpret_cast<const float*>(sTpL);
    }
  }
  int ph = 0;
  // the seeds of the step's NS samples (NS > 1: a gathered path reads its own)
  __shared__ float sSeed[NS];
  if (NS > 1 && li < NS) sSeed[li] = constRow<SailSample>(A.samples, min(tw.kBeg + li, tw.kEnd - 1)).seed;
  __syncthreads();
  // sort key: the winning primitive row when there are few enough rows (no row reads for the key, and a wave's
  // paths share their primitive and material rows; C2 +3.7 %, C3 +1.2 %), else (shape type, material category).
  // A waterfall over the wave's rows with the row index in an SGPR (scalar row loads) was measured: the
  // duplicated shading body doubled the spills, C2 -40 %.
  const bool byPrim = A.n < kKeys;
  const size_t pixG = (size_t)y * A.W + x;
  constexpr bool grouped = GROUPED;
  // a room-family kernel's first group accumulates its samples itself (SailTraceArgs.groupHome)
  constexpr bool kHome = FAM && !CULL;
  const bool home = !grouped || (kHome && tw.kBeg == 0);
  const bool pixLane = li < kPX;  // the lane that adds its pixel's samples (every lane when NS == 1)
  // the pixel's running accumulator: in registers, or, with samples in flight (flat forms), in an LDS slot of its lane
  // (the Cornell form: 32 float4, 512 B; the room form measured more spills with it), so that no VGPR stays live across the sample loop for it
  constexpr bool kAccLds = NS >= 16 && !CULL;
  __shared__ float4 sAcc[kAccLds ? kPX : 1];
  float4 acc = (valid && home && pixLane) ? A.accum[pixG] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if constexpr (kAccLds) {
    if (pixLane) sAcc[li] = acc;  // read back only by this lane
  }
  const float s = ((float)x + 0.5f) / (float)A.W, t = ((float)y + 0.5f) / (float)A.H;
  const bool tri0 = s + t <= 1.0f;
  const V3 eye = v3(A.eye[0], A.eye[1], A.eye[2]);
  // the exact segment counter: per wave in scalar registers in the pre-cull kernels (popcount of the live-lane ballot
  // at each bounce; C4 +1.8 %, profiles/r04_live_state.jsonl), per lane in the flat ones (there the scalar form measured
  // C1 -0.2 %, C3 -0.6 %)
  unsigned segs = 0;
  unsigned long long segsW = 0;
  PhaseClock pc;
#if SAIL_PHASE_TIMING
  for (int q = 0; q < 12; q++) pc.acc[q] = 0;
  pc.t = __builtin_amdgcn_s_memtime();
#endif
  for (int k = tw.kBeg; k < tw.kEnd; k += NS) {
    const int ks = k + mySlot;  // this lane's sample (NS == 1: k, uniform)
    const bool inRange = NS == 1 || ks < tw.kEnd;
    const SailSample& S = constRow<SailSample>(A.samples, NS == 1 ? k : (inRange ? ks : k));
    const bool aovs = A.aovN || A.aovP;  // AOVs of the launch's last sample
    bool alive = valid && inRange;
    int pixel = li;  // the path's home slot
    auto pathSeed = [&](int h) { if constexpr (NS == 1) return S.seed; else return sSeed[h / kPX]; };
    Ray ray;
    {
      const V3 d0 = v3(S.d[0][0], S.d[0][1], S.d[0][2]), d1 = v3(S.d[1][0], S.d[1][1], S.d[1][2]);
      const V3 d2 = v3(S.d[2][0], S.d[2][1], S.d[2][2]), d3 = v3(S.d[3][0], S.d[3][1], S.d[3][2]);
      ray = mkRay(eye, tri0 ? (d0 + (d2 - d0) * s + (d1 - d0) * t) : (d3 + (d1 - d3) * (1.0f - s) + (d2 - d3) * (1.0f - t)));
    }
    V3 fpdf = v3s(1.0f);
    // the path's radiance lives in LDS at its pixel: one path per pixel, updated in bounce order
    E_STORE(li, v3s(0.0f));
    for (int depth = 1; depth <= A.maxBounces; depth++) {
      Sweep sw;
      sw.best = kMaxDistance; sw.bi = -1; sw.bhl = v3s(0.0f);
      int key = 0;
      if constexpr (CULL) segsW += (unsigned long long)__popcll(__builtin_amdgcn_ballot_w64(alive));
      if (alive) {
        if constexpr (!CULL) segs++;
        sw = sweepRay(c, ray, depth == 1);
        if (sw.best >= kMaxDistance) {  // the path leaves the scene: its radiance is final
          if (depth == 1 && aovs && k + pixel / kPX == A.spp - 1) {  // fstrace.glsl:15-16 with n = p = 0 (GLSL: undefined)
            const size_t g = (size_t)homeY(pixel) * A.W + homeX(pixel);
            const V3 qn = v3s(0.0f) / 2.0f + 0.5f, qp = normalize(v3s(0.0f));
            if (A.aovN) A.aovN[g] = make_float4(qn.x, qn.y, qn.z, 1.0f);
            if (A.aovP) A.aovP[g] = make_float4(qp.x, qp.y, qp.z, 1.0f);
          }
          alive = false;
        } else if (byPrim) {
          key = 1 + sw.bi;
          // the room form compiled for rows with a Cornellbox sorts its hits by face, the normal / wall-colour chains'
          // first true test on the same hit point the record computes, so that a wave's box records take one face
          // branch (UI +3.4 %; the Cornell form measured -5.5 %: its 512-path pool splits into too many partial waves,
          // profiles/r05_facekey_*.jsonl)
          if constexpr (FAM && !CULL && kCornellRow >= 0) {
            if (sw.bi == kCornellRow) {
              const SailPrim& cp = PRIM(c, kCornellRow);
              const V3 h = ray.o + sw.best * ray.d, mn = P3(cp, 0), mx = P3(cp, 3);
              const int face = h.x < mn.x + 0.0001f ? 0 : h.x > mx.x - 0.0001f ? 1 : h.y < mn.y + 0.0001f ? 2
                             : h.y > mx.y - 0.0001f ? 3 : h.z < mn.z + 0.0001f ? 4 : 5;
              key = 1 + kRows + face;
            }
          }
        } else {
          const SailPrim& p = PRIM(c, sw.bi);
          int mc = matCat(p);
          mc = (mc >= 0 && mc < 5) ? mc : 0;
          key = 1 + mc * 10 + p.type;
        }
      }
      PHASE_MARK(pc, 0);
      // ---- counting sort of the live paths by key (LDS atomics for the per-key rank, one wave scans)
      int rank = 0;
      int nAlive;
      // a path's state into sorted slot d
      // after the scatter a lane's old path state is dead (a live lane gathers a new one, a dead lane reads none): say
      // so, or the compiler keeps it live across the sort for the lanes that gather nothing
      auto dropState = [&]() {
        ray.o = v3s(0.0f); ray.d = v3s(0.0f); ray.rx = ray.ry = ray.rz = 0.0f;
        fpdf = v3s(0.0f); sw.best = 0.0f; sw.bi = 0; pixel = 0;
      };
      auto scatterTo = [&](int d) {
        if constexpr (kPack == 2) {
          sSt4[0][d] = make_float4(ray.o.x, ray.o.y, ray.o.z, ray.d.x);
          sSt4[1][d] = make_float4(ray.d.y, ray.d.z, fpdf.x, fpdf.y);
          sSt4[2][d] = make_float4(fpdf.z, sw.best, __int_as_float(pixel | (sw.bi << 10)), __int_as_float(key));
        } else {
          sSt2[0][d] = make_float2(ray.o.x, ray.o.y); sSt2[1][d] = make_float2(ray.o.z, ray.d.x);
          sSt2[2][d] = make_float2(ray.d.y, ray.d.z); sSt2[3][d] = make_float2(fpdf.x, fpdf.y);
          sSt2[4][d] = make_float2(fpdf.z, sw.best);
          sSt2[5][d] = make_float2(__int_as_float(pixel | (sw.bi << 10)), __int_as_float(key));
        }
      };
      // the flat-form kernels (Cornell box, all-plugin) leave the first bounce unsorted: primary rays of a 16 x 4 strip
      // mostly hit one row already and none is dead yet, so each lane keeps its own pixel's path (C1 +1.1 %; the room
      // and pre-cull kernels keep the sort, where skipping it measured C3 -1.6 %, C4 -9.2 %:
      // profiles/r04_skip_sort1.jsonl)
      const bool sortNow = kSort1 || depth > 1;
      if (sortNow) {
      if constexpr (twoBar) {
      // every wave scans the counts itself (the start of a lane's key by a cross-lane read), so no barrier
      // between the scan and the scatter; the counts alternate between two buffers, the one just read being
      // cleared by wave 0 after the scatter barrier, two bounces before it is counted into again
      if (alive) rank = atomicAdd(&sCnt2[ph][key], 1);
      PHASE_MARK(pc, 7);  // rank atomics
      __syncthreads();
      PHASE_MARK(pc, 8);  // barrier 1 wait
      {
        const int v = sCnt2[ph][lane];
        const int incl = waveScanIncl(v);
        nAlive = __builtin_amdgcn_readlane(incl, 63);
        const int start = __shfl(incl - v, key, 64);
        if (alive) scatterTo(start + rank);
        dropState();
      }
      PHASE_MARK(pc, 9);  // scan + scatter
      __syncthreads();
      PHASE_MARK(pc, 10);  // barrier 2 wait
      if (wave == 0) sCnt2[ph][lane] = 0;
      ph ^= 1;
      } else {
      int* const sCnt = sCnt2[0];
      if (alive) rank = atomicAdd(&sCnt[key], 1);
      PHASE_MARK(pc, 7);  // rank atomics
      __syncthreads();
      PHASE_MARK(pc, 8);  // barrier 1 wait
      if (wave == 0) {
        const int v = sCnt[lane];
        const int incl = waveScanIncl(v);
        sStart[lane] = incl - v;
        if (lane == 63) sStart[kKeys] = incl;
        sCnt[lane] = 0;
      }
      PHASE_MARK(pc, 9);  // scan
      __syncthreads();
      PHASE_MARK(pc, 10);  // barrier 2 wait
      nAlive = sStart[kKeys];
      if (alive) scatterTo(sStart[key] + rank);
      dropState();
      PHASE_MARK(pc, 9);  // scatter
      __syncthreads();
      PHASE_MARK(pc, 10);  // barrier 3 wait
      }
      alive = li < nAlive;
      }
      ShadowPending sp;
      sp.pending = false;
      V3 eLit = v3s(0.0f);
      int keyG = 0;  // the gathered path's sort key
      PHASE_MARK(pc, 9);
      if (alive) {
        if (!sortNow) {
          keyG = key;
        } else if constexpr (kPack == 2) {
          const float4 q0 = sSt4[0][li], q1 = sSt4[1][li], q2 = sSt4[2][li];
          const int pk = __float_as_int(q2.z);
          keyG = __float_as_int(q2.w);
          ray.o = v3(q0.x, q0.y, q0.z);
          ray.d = v3(q0.w, q1.x, q1.y);
          fpdf = v3(q1.z, q1.w, q2.x);
          sw.best = q2.y;
          pixel = pk & 1023;
          sw.bi = pk >> 10;
          sw.bhl = v3s(0.0f);  // recomputed by hitRecord<true>
        } else {
          const float2 q0 = sSt2[0][li], q1 = sSt2[1][li], q2 = sSt2[2][li], q3 = sSt2[3][li], q4 = sSt2[4][li];
          const int pk = __float_as_int(sSt2[5][li].x);
          keyG = __float_as_int(sSt2[5][li].y);
          ray.o = v3(q0.x, q0.y, q1.x);
          ray.d = v3(q1.y, q2.x, q2.y);
          fpdf = v3(q3.x, q3.y, q4.x);
          sw.best = q4.y;
          pixel = pk & 1023;
          sw.bi = pk >> 10;
          sw.bhl = v3s(0.0f);  // recomputed by hitRecord<true>
        }
        ray.rx = ray.ry = ray.rz = 0.0f;  // not used past the sweep: the next ray is rebuilt by mkRay
        {  // a wave whose live paths have different sort keys runs several hit-record / material branches: raise its
           // issue priority so that its workgroup's next barrier is not held up by it (the other waves wait there)
          const int k0 = __builtin_amdgcn_readfirstlane(keyG);
          const bool mixedW = __builtin_amdgcn_ballot_w64(keyG != k0) != 0ull;
          if (mixedW) __builtin_amdgcn_s_setprio(kPrioMixed);
          else __builtin_amdgcn_s_setprio(0);
        }
        c.fcx = (float)homeX(pixel) + 0.5f;
        c.fcy = (float)homeY(pixel) + 0.5f;
        const float seed = pathSeed(pixel) + (float)depth;
        const Hit ins = hitRecordU<true, FAM && !CULL>(c, ray, sw);
        PHASE_MARK(pc, 1);
        if (depth == 1 && aovs && k + pixel / kPX == A.spp - 1) {
          const size_t g = (size_t)homeY(pixel) * A.W + homeX(pixel);
          const V3 qn = ins.normal / 2.0f + 0.5f, qp = normalize(ins.hit);
          if (A.aovN) A.aovN[g] = make_float4(qn.x, qn.y, qn.z, 1.0f);
          if (A.aovP) A.aovP[g] = make_float4(qp.x, qp.y, qp.z, 1.0f);
        }
        V3 e = E_LOAD(pixel);
        if (!(!CULL && depth == A.maxBounces && shadeLast(c, ins, seed, fpdf, e))) {
          if constexpr (kShCompact) {
            shadeBounceP(c, ins, ray, seed, fpdf, e, pc, sp);  // e: the dark outcome
            eLit = sp.eLit;
          } else {
            shadeBounce(c, ins, ray, seed, fpdf, e, pc);
          }
        }
        E_STORE(pixel, e);
      }
      if constexpr (kShCompact) {
        if (c.ln > 0) {  // uniform
          const bool pend = alive && sp.pending;
          __syncthreads();  // every gather of this bounce is done: the sort buffer takes the shadow rays
          const unsigned long long bm = __builtin_amdgcn_ballot_w64(pend);
          if (bm != 0ull) {  // uniform over the wave
            int base = 0;
            if (lane == 0) base = atomicAdd(&sShCnt[shph], __popcll(bm));
            base = __shfl(base, 0, 64);
            if (pend) {
              const int d = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
              const V3 o = sp.hit, dl = sp.toLight;
              if constexpr (kPack == 2) {
                sSt4[0][d] = make_float4(o.x, o.y, o.z, dl.x);
                sSt4[1][d] = make_float4(dl.y, dl.z, eLit.x, eLit.y);
                sSt4[2][d] = make_float4(eLit.z, __int_as_float(pixel), 0.0f, 0.0f);
              } else {
                sSt2[0][d] = make_float2(o.x, o.y); sSt2[1][d] = make_float2(o.z, dl.x);
                sSt2[2][d] = make_float2(dl.y, dl.z); sSt2[3][d] = make_float2(eLit.x, eLit.y);
                sSt2[4][d] = make_float2(eLit.z, __int_as_float(pixel));
              }
            }
          }
          __syncthreads();
          const int nSh = sShCnt[shph];
          if (li == 0) sShCnt[shph ^ 1] = 0;  // the previous bounce's count: every read of it is done
          shph ^= 1;
          if (li < nSh) {  // testShadow(Ray(hit, toLight)) of the light sample (shader.light.js:24-31)
            V3 o, dl, el;
            int pix;
            if constexpr (kPack == 2) {
              const float4 q0 = sSt4[0][li], q1 = sSt4[1][li], q2 = sSt4[2][li];
              o = v3(q0.x, q0.y, q0.z); dl = v3(q0.w, q1.x, q1.y); el = v3(q1.z, q1.w, q2.x);
              pix = __float_as_int(q2.y);
            } else {
              const float2 q0 = sSt2[0][li], q1 = sSt2[1][li], q2 = sSt2[2][li], q3 = sSt2[3][li], q4 = sSt2[4][li];
              o = v3(q0.x, q0.y, q1.x); dl = v3(q1.y, q2.x, q2.y); el = v3(q3.x, q3.y, q4.x);
              pix = __float_as_int(q4.y);
            }
            if (!testShadow(c, mkRay(o, dl))) E_STORE(pix, el);
          }
        }
      }
    }
    __syncthreads();
    if constexpr (NS == 1) {
      if (valid) {
        const V3 er = E_LOAD(li);
        if (!home) stageSample<kPX>(A, k, tw.bid, li, er);
        else accumulateSample(acc, er, S, A.accumMode);
      }
    } else {
      if (valid && pixLane) {  // the pixel's samples of this step, in sample order
        if constexpr (kAccLds) acc = sAcc[li];
        for (int j = 0; j < NS && k + j < tw.kEnd; j++) {
          const V3 er = E_LOAD(j * kPX + li);
          if (!home) stageSample<kPX>(A, k + j, tw.bid, li, er);
          else accumulateSample(acc, er, constRow<SailSample>(A.samples, k + j), A.accumMode);
        }
        if constexpr (kAccLds) sAcc[li] = acc;
      }
      if (li < NS && k + NS + li < tw.kEnd) sSeed[li] = constRow<SailSample>(A.samples, k + NS + li).seed;
    }
    __syncthreads();
    PHASE_MARK(pc, 11);  // sample end: barriers, accumulation / staging
  }
  if constexpr (kAccLds) {
    if (pixLane) acc = sAcc[li];
  }
  if (valid && home && pixLane) A.accum[pixG] = acc;
#if SAIL_PHASE_TIMING
  if (lane == 0)
    for (int q = 0; q < 12; q++) atomicAdd(&g_sailPhase[q], pc.acc[q]);
#endif
  if (A.segCounter) {
    unsigned long long v = segsW;
    if constexpr (!CULL) {
      v = segs;
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    }
    if (lane == 0) atomicAdd(&A.segCounter[(blockIdx.x * 4u + (unsigned)wave) % SAIL_SEG_SLOTS], v);
  }
}
// Path compaction (traceTileCompact) in every plugin-set kernel: C2 +6 %, C3 +12 %, C4 +10 % (measured;
// earlier builds with more live state lost to spills in the flat kernels).
// Each plugin set has an ungrouped kernel (one workgroup per 16 x NT/16 block, every sample) and a _grouped one
// (sample groups: G workgroups per block, staged radiance added by sail_accum_kernel). Launch bounds: waves per SIMD
// and threads per workgroup, chosen by the occupancy sweeps of DESIGN.md §5 (sail_launch_trace sizes the grids).
// fam: the room family's choices for a flat kernel -- the two-barrier sort, the first sample group accumulating its
// samples itself (SailTraceArgs.groupHome) and one box record for Cube and Cornellbox.
#define SAIL_TRACE_KERNELS_NS(name, waves, cull, ks, km, kt, kl, nt, gnt, fam, ns)                                 \
  extern "C" __global__ void __launch_bounds__(nt, waves) name(SailTraceArgs A) {                                \
    traceTileCompact<cull, false, ks, km, kt, kl, nt, fam, ns>(A);                                               \
  }                                                                                                              \
  extern "C" __global__ void __launch_bounds__(gnt, waves) name##_grouped(SailTraceArgs A) {                     \
    traceTileCompact<cull, true, ks, km, kt, kl, gnt, fam, ns>(A);                                               \
  }
#define SAIL_TRACE_KERNELS(name, waves, cull, ks, km, kt, kl, nt, gnt, fam) \
  SAIL_TRACE_KERNELS_NS(name, waves, cull, ks, km, kt, kl, nt, gnt, fam, 1)
#if defined(SAIL_JIT)
// A per-plugin-set kernel compiled at run time by hipRTC (sail_jit.cpp), like the reference's per-scene program
// (tracerConfig -> Generator.generate, src/scene/scene.js:70-112, src/shader/generator.js:107-123): the plugin masks,
// the pre-cull choice, the family and the launch bounds arrive as macros, and only this kernel pair is compiled.
#ifndef SAIL_JIT_NS
#define SAIL_JIT_NS 1
#endif
#if SAIL_JIT_CULL
SAIL_TRACE_KERNELS_NS(sail_trace_kernel_cull_jit, SAIL_JIT_WAVES, true, SAIL_JIT_KS, SAIL_JIT_KM, SAIL_JIT_KT, SAIL_JIT_KL,
                      SAIL_JIT_NT, SAIL_JIT_NT, false, SAIL_JIT_NS)
#else
SAIL_TRACE_KERNELS_NS(sail_trace_kernel_jit, SAIL_JIT_WAVES, false, SAIL_JIT_KS, SAIL_JIT_KM, SAIL_JIT_KT, SAIL_JIT_KL,
                      SAIL_JIT_NT, SAIL_JIT_NT, SAIL_JIT_FAM != 0, SAIL_JIT_NS)
#endif
#else
// every plugin (any scene of fewer than 8 primitives outside the two sets below)
#define SAIL_GENERIC_WAVES 6
SAIL_TRACE_KERNELS(sail_trace_kernel, SAIL_GENERIC_WAVES, false, ~0u, ~0u, ~0u, ~0u, 256, 256, false)
// the README Cornell box plugin set (C1/C2/C5): Cube + Sphere + Cornellbox, Matte + Mirror, uniform colours
#define SAIL_CORNELL_WAVES 8
#define SAIL_CORNELL_NT 256
#define SAIL_CORNELL_GROUP_NT 256
SAIL_TRACE_KERNELS(sail_trace_kernel_cornell, SAIL_CORNELL_WAVES, false, SAIL_KSET_CORNELL_SHAPES, SAIL_KSET_CORNELL_MATS,
                   SAIL_KSET_CORNELL_TEX, SAIL_KSET_CORNELL_LIGHTS, SAIL_CORNELL_NT, SAIL_CORNELL_GROUP_NT, false)
// rooms of boxes, spheres and rectangle lights (C3 materials demo, UI demo); occupancy measured 5/6/7/8 waves
#define SAIL_ROOM_WAVES 7
#define SAIL_ROOM_NT 256
#define SAIL_ROOM_GROUP_NT 256
SAIL_TRACE_KERNELS(sail_trace_kernel_room, SAIL_ROOM_WAVES, false, SAIL_KSET_ROOM_SHAPES, SAIL_KSET_ROOM_MATS,
                   SAIL_KSET_ROOM_TEX, SAIL_KSET_ROOM_LIGHTS, SAIL_ROOM_NT, SAIL_ROOM_GROUP_NT, true)
// the pre-cull kernel serves scenes with many primitives (C4); 1,024-thread workgroups (16 x 64 strips)
#define SAIL_CULL_WAVES 8
#define SAIL_CULL_NT 1024
#define SAIL_CULL_GROUP_NT 1024
SAIL_TRACE_KERNELS(sail_trace_kernel_cull, SAIL_CULL_WAVES, true, ~0u, ~0u, ~0u, ~0u, SAIL_CULL_NT, SAIL_CULL_GROUP_NT, false)

// ---- wavefront split of the pre-cull path (study switch SAIL_DEBUG_WAVEFRONT; DESIGN.md §9 of round 2) -------------------
// The megakernel keeps each path in registers and LDS across its bounces and sorts the workgroup's paths between the
// sweep and the shading. Here one sample of every owned pixel is traced bounce by bounce with the state in HBM and
// four kernels per bounce pass: the sweep, the hit record + shading (a lit matte path's shadow test deferred), the
// shadow sweep of the deferred tests with the radiance update they hold back, then (per sample) the accumulation.
// Each kernel runs with only its own live state. Same functions, same operations in the same order: bit-identical.
namespace {
struct WfPix { int x, y; bool valid; };
D WfPix wfPixel(const SailTraceArgs& A, long long slot) {
  const int ownedTile = (int)(slot >> 12), local = (int)(slot & 4095);
  const int tile = A.rank + ownedTile * A.world;
  WfPix q;
  q.x = (tile % A.tilesX) * 64 + (local & 63);
  q.y = (tile / A.tilesX) * 64 + (local >> 6);
  q.valid = ownedTile < A.ownedTiles && q.x < A.W && q.y < A.H;
  return q;
}
D Ctx wfCtx(const SailTraceArgs& A) {
  Ctx c;
  c.tp = A.texparams; c.lt = A.lights; c.lightObjRow = A.lightObjRow; c.typeMasks = A.typeMasks;
  c.prims = A.prims;
  c.cprims = A.prims;
  c.tpl = A.texparams;
  c.rowCopy = false;
  c.tpCopy = false;
  c.n = A.n; c.tn = A.tn; c.ln = A.ln;
  c.matMask = A.matMask; c.texMask = A.texMask; c.lightMask = A.lightMask;
  c.fcx = 0.0f; c.fcy = 0.0f;
  c.shadowAnyHit = A.shadowAnyHit;
  c.cullPrims = 1;
  c.cullFma = A.cullPrims == 2;
  c.cullPrimary = A.cullPrimary;
  c.kShapes = ~0u; c.kMats = ~0u; c.kTex = ~0u; c.kLights = ~0u;
  return c;
}
}  // namespace
// primary rays of sample k
extern "C" __global__ void __launch_bounds__(256) sail_wf_primary(SailTraceArgs A, SailWfState S, int k) {
  const long long slot = (long long)blockIdx.x * 256 + threadIdx.x;
  const WfPix q = wfPixel(A, slot);
  const SailSample& sm = constRow<SailSample>(A.samples, k);
  const float s = ((float)q.x + 0.5f) / (float)A.W, t = ((float)q.y + 0.5f) / (float)A.H;
  const V3 d0 = v3(sm.d[0][0], sm.d[0][1], sm.d[0][2]), d1 = v3(sm.d[1][0], sm.d[1][1], sm.d[1][2]);
  const V3 d2 = v3(sm.d[2][0], sm.d[2][1], sm.d[2][2]), d3 = v3(sm.d[3][0], sm.d[3][1], sm.d[3][2]);
  const V3 dir = (s + t <= 1.0f) ? (d0 + (d2 - d0) * s + (d1 - d0) * t) : (d3 + (d1 - d3) * (1.0f - s) + (d2 - d3) * (1.0f - t));
  S.o[slot] = make_float4(A.eye[0], A.eye[1], A.eye[2], q.valid ? 1.0f : 0.0f);
  S.d[slot] = make_float4(dir.x, dir.y, dir.z, 0.0f);
  S.f[slot] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
  S.e[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}
// the closest-hit sweep of every live path
extern "C" __global__ void __launch_bounds__(256) sail_wf_sweep(SailTraceArgs A, SailWfState S, int k, int depth) {
  const long long slot = (long long)blockIdx.x * 256 + threadIdx.x;
  const float4 o = S.o[slot];
  unsigned seg = 0;
  if (o.w != 0.0f) {
    const Ctx c = wfCtx(A);
    const float4 d = S.d[slot];
    const Ray ray = mkRay(v3(o.x, o.y, o.z), v3(d.x, d.y, d.z));
    const Sweep sw = sweepRay(c, ray, depth == 1);
    seg = 1;
    if (sw.best >= kMaxDistance) {  // the path leaves the scene
      S.o[slot] = make_float4(o.x, o.y, o.z, 0.0f);
      if (depth == 1 && (A.aovN || A.aovP) && k == A.spp - 1) {
        const WfPix q = wfPixel(A, slot);
        const size_t g = (size_t)q.y * A.W + q.x;
        const V3 qn = v3s(0.0f) / 2.0f + 0.5f, qp = normalize(v3s(0.0f));
        if (A.aovN) A.aovN[g] = make_float4(qn.x, qn.y, qn.z, 1.0f);
        if (A.aovP) A.aovP[g] = make_float4(qp.x, qp.y, qp.z, 1.0f);
      }
    } else {
      S.s[slot] = make_float4(sw.best, __int_as_float(sw.bi), 0.0f, 0.0f);
    }
  }
  if (A.segCounter) {
    unsigned long long v = seg;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&A.segCounter[(blockIdx.x * 4u + (threadIdx.x >> 6)) % SAIL_SEG_SLOTS], v);
  }
}
// hit record and shading of every live path; a lit matte path's shadow test and radiance update are deferred
extern "C" __global__ void __launch_bounds__(256) sail_wf_shade(SailTraceArgs A, SailWfState S, int k, int depth) {
  const long long slot = (long long)blockIdx.x * 256 + threadIdx.x;
  const float4 o = S.o[slot];
  if (o.w == 0.0f) { S.sp[0][slot].w = 0.0f; return; }
  Ctx c = wfCtx(A);
  const WfPix q = wfPixel(A, slot);
  c.fcx = (float)q.x + 0.5f; c.fcy = (float)q.y + 0.5f;
  const float4 d = S.d[slot], fp = S.f[slot], ee = S.e[slot], sv = S.s[slot];
  Ray ray;
  ray.o = v3(o.x, o.y, o.z); ray.d = v3(d.x, d.y, d.z); ray.rx = ray.ry = ray.rz = 0.0f;
  Sweep sw;
  sw.best = sv.x; sw.bi = __float_as_int(sv.y); sw.bhl = v3s(0.0f);
  const Hit ins = hitRecord<true>(c, ray, sw);
  if (depth == 1 && (A.aovN || A.aovP) && k == A.spp - 1) {
    const size_t g = (size_t)q.y * A.W + q.x;
    const V3 qn = ins.normal / 2.0f + 0.5f, qp = normalize(ins.hit);
    if (A.aovN) A.aovN[g] = make_float4(qn.x, qn.y, qn.z, 1.0f);
    if (A.aovP) A.aovP[g] = make_float4(qp.x, qp.y, qp.z, 1.0f);
  }
  V3 fpdf = v3(fp.x, fp.y, fp.z), e = v3(ee.x, ee.y, ee.z);
  const float seed = constRow<SailSample>(A.samples, k).seed + (float)depth;
  PhaseClock pc;
  ShadowPending sp;
  shadeBounceP(c, ins, ray, seed, fpdf, e, pc, sp);
  S.e[slot] = make_float4(e.x, e.y, e.z, 0.0f);
  S.f[slot] = make_float4(fpdf.x, fpdf.y, fpdf.z, 0.0f);
  S.o[slot] = make_float4(ray.o.x, ray.o.y, ray.o.z, 1.0f);
  S.d[slot] = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.0f);
  S.sp[0][slot] = make_float4(sp.hit.x, sp.hit.y, sp.hit.z, sp.pending ? 1.0f : 0.0f);
  if (sp.pending) {
    S.sp[1][slot] = make_float4(sp.toLight.x, sp.toLight.y, sp.toLight.z, 0.0f);
    S.sp[2][slot] = make_float4(sp.eLit.x, sp.eLit.y, sp.eLit.z, 0.0f);
  }
}
// the deferred shadow tests (testShadow, shader.light.js:24-31): the radiance holds the blocked outcome of the update,
// replaced by the unblocked one (ShadowPending.eLit) when the ray is not blocked
extern "C" __global__ void __launch_bounds__(256) sail_wf_shadow(SailTraceArgs A, SailWfState S) {
  const long long slot = (long long)blockIdx.x * 256 + threadIdx.x;
  const float4 h = S.sp[0][slot];
  if (h.w == 0.0f) return;
  const Ctx c = wfCtx(A);
  const float4 tl = S.sp[1][slot], el = S.sp[2][slot];
  if (!testShadow(c, mkRay(v3(h.x, h.y, h.z), v3(tl.x, tl.y, tl.z)))) S.e[slot] = make_float4(el.x, el.y, el.z, 0.0f);
}
// sample k's radiance into the accumulator (sample order: one launch per sample)
extern "C" __global__ void __launch_bounds__(256) sail_wf_accum(SailTraceArgs A, SailWfState S, int k) {
  const long long slot = (long long)blockIdx.x * 256 + threadIdx.x;
  const WfPix q = wfPixel(A, slot);
  if (!q.valid) return;
  const size_t pix = (size_t)q.y * A.W + q.x;
  float4 acc = A.accum[pix];
  const float4 ee = S.e[slot];
  accumulateSample(acc, v3(ee.x, ee.y, ee.z), constRow<SailSample>(A.samples, k), A.accumMode);
  A.accum[pix] = acc;
}
hipError_t sail_launch_wavefront(const SailTraceArgs& A, const SailWfState& S, hipStream_t s) {
  const unsigned blocks = (unsigned)A.ownedTiles * 16u;  // 4096 slots per owned tile, 256 per workgroup
  for (int k = 0; k < A.spp; k++) {
    hipLaunchKernelGGL(sail_wf_primary, dim3(blocks), dim3(256), 0, s, A, S, k);
    for (int depth = 1; depth <= A.maxBounces; depth++) {
      hipLaunchKernelGGL(sail_wf_sweep, dim3(blocks), dim3(256), 0, s, A, S, k, depth);
      hipLaunchKernelGGL(sail_wf_shade, dim3(blocks), dim3(256), 0, s, A, S, k, depth);
      hipLaunchKernelGGL(sail_wf_shadow, dim3(blocks), dim3(256), 0, s, A, S);
    }
    hipLaunchKernelGGL(sail_wf_accum, dim3(blocks), dim3(256), 0, s, A, S, k);
  }
  return hipGetLastError();
}

// ---- sample groups: add the staged per-sample radiance to the accumulator in sample order ---------------------
extern "C" __global__ void __launch_bounds__(256) sail_accum_kernel(SailTraceArgs A) {
  const int bid = (int)blockIdx.x;
  const int ownedTile = bid >> 4, sub = bid & 15;
  const int tile = A.rank + ownedTile * A.world;
  const int tx = tile % A.tilesX, ty = tile / A.tilesX;
  const int li = threadIdx.x;
  const int x = tx * 64 + (sub & 3) * 16 + (li & 15), y = ty * 64 + (sub >> 2) * 16 + (li >> 4);
  if (x >= A.W || y >= A.H) return;
  const size_t pix = (size_t)y * A.W + x;
  float4 acc = A.accum[pix];  // holds the first group's samples already (SAIL_GROUP_HOME)
  const float* st = A.stage + (long long)bid * 256 + li;
  const size_t ss = (size_t)A.stageStride;
  int k = A.groupHome ? A.groupSpp : 0;
  // eight samples' planes loaded ahead of their in-order additions (the pass is HBM-bound: keep loads in flight;
  // 0.189 -> 0.180 ms per C2 launch)
  for (; k + 8 <= A.spp; k += 8) {
    float v[8][3];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const float* q = st + (size_t)(k + j) * 3u * ss;
      v[j][0] = q[0]; v[j][1] = q[ss]; v[j][2] = q[2 * ss];
    }
#pragma unroll
    for (int j = 0; j < 8; j++)
      accumulateSample(acc, v3(v[j][0], v[j][1], v[j][2]), constRow<SailSample>(A.samples, k + j), A.accumMode);
  }
  for (; k < A.spp; k++) {
    const float* q = st + (size_t)k * 3u * ss;
    accumulateSample(acc, v3(q[0], q[ss], q[2 * ss]), constRow<SailSample>(A.samples, k), A.accumMode);
  }
  A.accum[pix] = acc;
}

// ---- multi-device frame reduction without RCCL (a multi-device context whose devices are all one GPU) ----------
// dst = ((src0 + src1) + src2) + ...: the sum of the ranks' frames in rank order
extern "C" __global__ void __launch_bounds__(256) sail_sum_kernel(SailSumArgs A) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= A.n) return;
  float4 v = A.src[0][i];
  for (int k = 1; k < A.nsrc; k++) {
    const float4 w = A.src[k][i];
    v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
  }
  A.dst[i] = v;
}
// AOV maps of a tile-partitioned rank hold -0 outside its tiles: x + (-0) == x for every x (+0, -0 and NaN
// included), so the sum over ranks reproduces the owning rank's AOV bits exactly (a +0 fill would turn -0 into +0)
extern "C" __global__ void __launch_bounds__(256) sail_negzero_unowned_kernel(float4* a, float4* b, int W, int H,
                                                                             int rank, int world) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= W || y >= H) return;
  const int tilesX = (W + 63) / 64;
  const int tile = (y >> 6) * tilesX + (x >> 6);
  if (tile % world == rank) return;
  const float4 nz = make_float4(-0.0f, -0.0f, -0.0f, -0.0f);
  const size_t pix = (size_t)y * W + x;
  if (a) a[pix] = nz;
  if (b) b[pix] = nz;
}

// ---- display filter (fsrender.glsl + filter/*.glsl), W x H generalisation of the 512 x 512 pass ---------------------
// Every map is sampled as the reference's frame textures are: LINEAR, default REPEAT wrap (webgl.js:153-156),
// RGB (texture() returns alpha 1). The colour map is the mean image (SUM accumulators divided per texel).
namespace {
D int wrapi(int i, int size) { int m = i % size; return m < 0 ? m + size : m; }
struct Tap { int xa, xb, ya, yb; float a, b; };
D Tap tapAt(int W, int H, float u, float v) {
  const float fx = u * (float)W - 0.5f, fy = v * (float)H - 0.5f;
  const float x0f = floorf(fx), y0f = floorf(fy);
  Tap t;
  t.a = fx - x0f; t.b = fy - y0f;
  const int xi = (int)x0f, yi = (int)y0f;
  t.xa = wrapi(xi, W); t.xb = wrapi(xi + 1, W); t.ya = wrapi(yi, H); t.yb = wrapi(yi + 1, H);
  return t;
}
D V3 texel(const SailFilterArgs& A, const float4* img, bool mean, int x, int y) {
  const float4 v = img[(size_t)y * A.W + x];
  if (mean && A.accumMode == 0) {  // each texel's own count (a reduced tile frame may mix counts; 0: unrendered)
    const float cnt = v.w > 0.0f ? v.w : 1.0f;
    return v3(v.x / cnt, v.y / cnt, v.z / cnt);
  }
  return v3(v.x, v.y, v.z);
}
D V3 bilerp(V3 t00, V3 t10, V3 t01, V3 t11, float a, float b) {
  const V3 c0 = t00 * (1.0f - a) + t10 * a, c1 = t01 * (1.0f - a) + t11 * a;
  return c0 * (1.0f - b) + c1 * b;
}
D V3 sample(const SailFilterArgs& A, const float4* img, bool mean, float u, float v) {
  const Tap t = tapAt(A.W, A.H, u, v);
  return bilerp(texel(A, img, mean, t.xa, t.ya), texel(A, img, mean, t.xb, t.ya), texel(A, img, mean, t.xa, t.yb),
                texel(A, img, mean, t.xb, t.yb), t.a, t.b);
}
D float dot4(V3 t, float w) { return t.x * t.x + t.y * t.y + t.z * t.z + w * w; }
// window filters: the workgroup's 16x16 pixels plus a halo of mean texels staged in LDS once (one divide per
// texel instead of one per tap read); taps that would leave the tile read global memory as before
constexpr int kFiltMaxT = 32;
struct FiltTile { const float* r; const float* g; const float* b; int x0, y0, T; };
D V3 sampleTile(const SailFilterArgs& A, const FiltTile& tl, float u, float v) {
  const float fx = u * (float)A.W - 0.5f, fy = v * (float)A.H - 0.5f;
  const float x0f = floorf(fx), y0f = floorf(fy);
  const float a = fx - x0f, b = fy - y0f;
  const int lx = (int)x0f - tl.x0, ly = (int)y0f - tl.y0;
  if (lx < 0 || ly < 0 || lx + 1 >= tl.T || ly + 1 >= tl.T) return sample(A, A.accum, true, u, v);
  const int i00 = ly * tl.T + lx, i01 = i00 + tl.T;
  return bilerp(v3(tl.r[i00], tl.g[i00], tl.b[i00]), v3(tl.r[i00 + 1], tl.g[i00 + 1], tl.b[i00 + 1]),
                v3(tl.r[i01], tl.g[i01], tl.b[i01]), v3(tl.r[i01 + 1], tl.g[i01 + 1], tl.b[i01 + 1]), a, b);
}
}  // namespace

extern "C" __global__ void __launch_bounds__(256) sail_filter_kernel(SailFilterArgs A) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  __shared__ float sTR[kFiltMaxT * kFiltMaxT], sTG[kFiltMaxT * kFiltMaxT], sTB[kFiltMaxT * kFiltMaxT];
  FiltTile tl;
  tl.r = sTR; tl.g = sTG; tl.b = sTB;
  tl.T = 16 + 2 * A.halo;
  tl.x0 = (int)blockIdx.x * 16 - A.halo; tl.y0 = (int)blockIdx.y * 16 - A.halo;
  if (A.kind == 3 && A.halo > 0) {  // uniform over the grid
    for (int i = threadIdx.x; i < tl.T * tl.T; i += 256) {
      const int ly = i / tl.T, lx = i - ly * tl.T;
      const V3 m = texel(A, A.accum, true, wrapi(tl.x0 + lx, A.W), wrapi(tl.y0 + ly, A.H));  // REPEAT wrap
      sTR[i] = m.x; sTG[i] = m.y; sTB[i] = m.z;
    }
    __syncthreads();
  }
  if (x >= A.W || y >= A.H) return;
  const float tcx = ((float)x + 0.5f) / (float)A.W, tcy = ((float)y + 0.5f) / (float)A.H;
  float o[4] = {0.0f, 0.0f, 0.0f, 1.0f};
  if (A.kind <= 2) {  // color.glsl / gamma.glsl / tonemapping.glsl
    const V3 cv = sample(A, A.accum, true, tcx, tcy);
    const float col[3] = {cv.x, cv.y, cv.z};
    for (int c = 0; c < 3; c++) {
      if (A.kind == 0) o[c] = col[c];
      else if (A.kind == 1) o[c] = powf_(col[c], rcp_rn(A.gammaC));
      else {
        const float xx = fmax_(0.0f, col[c] - 0.004f);
        o[c] = fdiv(xx * (6.2f * xx + 0.5f), xx * (6.2f * xx + 1.7f) + 0.06f);
      }
    }
  } else if (A.kind == 3) {  // window.glsl:1-44, FILTER_WINDOW_WIDTH 4
    V3 acc = v3s(0.0f);
    float weightSum = 0.0f;
    for (int i = 0; i < 4; i++) {
      for (int j = 0; j < 4; j++) {
        const float wi = fdiv(((float)j + 0.5f) * A.rx, 4.0f), wj = fdiv(((float)i + 0.5f) * A.ry, 4.0f);
        const float ox = fdiv(wi, (float)A.W), oy = fdiv(wj, (float)A.H);
        V3 tmp = v3s(0.0f);
        int count = 0;
        for (int q = 0; q < 4; q++) {
          const float u = (q < 2) ? tcx + ox : tcx - ox;
          const float v = (q & 1) ? tcy - oy : tcy + oy;
          if (u < 0.0f || u > 1.0f || v < 0.0f || v > 1.0f) continue;
          count++;
          tmp = tmp + (A.halo > 0 ? sampleTile(A, tl, u, v) : sample(A, A.accum, true, u, v));
        }
        const float weight = A.weights[i * j + j];
        weightSum += weight * (float)count;
        acc = acc + tmp * weight;
      }
    }
    o[0] = fdiv(acc.x, weightSum); o[1] = fdiv(acc.y, weightSum); o[2] = fdiv(acc.z, weightSum);
  } else if (A.kind == 4) {  // wavelet.glsl:5-54 (edge-avoiding a-trous over the colour and position maps)
    const V3 cval = sample(A, A.accum, true, tcx, tcy);
    const V3 pval = sample(A, A.aovP, false, tcx, tcy);
    // the reference reads normalMap (nval, ntmp) but never uses it: its "normal" weight reuses the colour
    // difference (wavelet.glsl:11-12)
    const float hk[5] = {0.375f, 0.25f, 0.0625f, 0.0625f, 0.25f};
    const float dW = (float)A.W, dH = (float)A.H, dW2 = dW * 2.5f, dH2 = dH * 2.5f;  // 512, 1280 at 512^2
    float col[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    float weightSum = 0.0f;
    for (int n = 0; n < 3; n++) {
      const float stepwidth = powf_(2.0f, (float)n) - 1.0f;
      const int div = to_int(stepwidth) + 1;
      int count = 0;
      for (int i = 0; i < 5; i++) {
        for (int j = 0; j < 5; j++, count++) {
          const int delt = abs(count - 12);
          float h = 0.0f;
          if (delt % div == 0) h = hk[(delt / div) % 5];
          if (h == 0.0f) continue;
          const float u = (tcx - fdiv(A.rx, dW)) + fdiv(((float)j + 0.5f) * A.rx, dW2);
          const float v = (tcy - fdiv(A.ry, dH)) + fdiv(((float)i + 0.5f) * A.ry, dH2);
          const V3 ctmp = sample(A, A.accum, true, u, v);
          const V3 t = cval - ctmp;
          const float tw = 1.0f - 1.0f;
          const float c_w = fmin_(expf_(fdiv(-(dot4(t, tw)), 4.0f)), 1.0f);
          const float d2 = fmax_(fdiv(dot4(t, tw), stepwidth * stepwidth), 0.0f);
          const float n_w = fmin_(expf_(fdiv(-(d2), 128.0f)), 1.0f);
          const V3 tp = pval - sample(A, A.aovP, false, u, v);
          const float p_w = fmin_(expf_(fdiv(-(dot4(tp, tw)), 1.0f)), 1.0f);
          const float weight = c_w * n_w * p_w * h;
          weightSum += weight;
          col[0] += ctmp.x * weight; col[1] += ctmp.y * weight; col[2] += ctmp.z * weight; col[3] += 1.0f * weight;
        }
      }
    }
    for (int c = 0; c < 4; c++) o[c] = fdiv(col[c], weightSum);
  } else {  // normal.glsl / position.glsl: the AOV map at the texel
    const V3 m = sample(A, A.kind == 5 ? A.aovN : A.aovP, false, tcx, tcy);
    o[0] = m.x; o[1] = m.y; o[2] = m.z;
  }
  const size_t pix = (size_t)y * A.W + x;
  if (A.out) A.out[pix] = make_float4(o[0], o[1], o[2], o[3]);
  if (A.out8) {
    for (int c = 0; c < 3; c++) A.out8[4 * pix + c] = (uint8_t)(int)(clamp_(o[c], 0.0f, 1.0f) * 255.0f + 0.5f);
    A.out8[4 * pix + 3] = 255;
  }
}

// ---- picking (replaces the CPU picker, src/core/pickup.js:46-66): the trace kernel's own primitive sweep
// for caller-supplied rays; index = the first object row with the smallest distance, -1 on a miss ---------------
extern "C" __global__ void __launch_bounds__(64) sail_pick_kernel(const SailPrim* prims, int n, const float* rays,
                                                                   int count, int32_t* index, float* tOut) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const float* q = rays + 6 * (size_t)i;
  const Ray r = mkRay(v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]));
  Ctx c;
  c.kShapes = ~0u;
  float best = kMaxDistance;
  int bi = -1;
  for (int k = 0; k < n; k++) {
    const float t = primT(c, constRow<SailPrim>(prims, k), r, nullptr);
    if (t < best) { best = t; bi = k; }
  }
  index[i] = bi;
  tOut[i] = best;
}

// ---- spec-math probe for the CPU/GPU bit-parity test ----------------------------------------------------------------
extern "C" __global__ void sail_math_kernel(int fn, const float* x, const float* y, float* out, int count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  float r = 0.0f;
  switch (fn) {
    case 0: r = sinf_(x[i]); break;
    case 1: r = cosf_(x[i]); break;
    case 2: r = tanf_(x[i]); break;
    case 3: r = atan2f_(y[i], x[i]); break;
    case 4: r = acosf_(x[i]); break;
    case 5: r = powf_(x[i], y[i]); break;
    case 6: r = atanf_(x[i]); break;
    case 7: r = sqrtf_(x[i]); break;
    case 8: r = x[i] / y[i]; break;
    case 9: r = fmin_(x[i], y[i]); break;
    case 10: r = fmax_(x[i], y[i]); break;
    case 11: r = fdiv(x[i], y[i]); break;  // GLSL divide spec
    case 14: r = rcp_rn(x[i]); break;
    case 15: r = sqrt01(x[i]); break;  // callers guarantee [0, 1] or NaN
    case 12: r = clamp_(x[i], 0.0f, 1.0f); break;
    default: break;
  }
  out[i] = r;
}

// 1 in the phase-timing build: its run-time kernels are compiled instrumented too (sail_jit.cpp defsFor)
extern const int sail_trace_phase_timing = SAIL_PHASE_TIMING;
#if SAIL_PHASE_TIMING
int sail_jit_phase_read(unsigned long long out[12], int reset);  // sail_jit.cpp: the loaded run-time modules' sums
// phase-timing readout (tools/phase_profile.py): the precompiled kernels' sums plus every loaded run-time module's
extern "C" int sail_phase_read(unsigned long long out[12], int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sailPhase), 12 * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_sailPhase), z, sizeof z) != hipSuccess) return -1;
  }
  return sail_jit_phase_read(out, reset);
}
#endif

// ---- host launch wrappers (called by sail_capi.cpp) ----------------------------------------------------------------
hipError_t sail_launch_trace(const SailTraceArgs& A, int blocks, hipStream_t s) {
  const bool g = A.sampleGroups > 1;
#define SAIL_LAUNCH(k) hipLaunchKernelGGL(g ? k##_grouped : k, dim3(blocks), dim3(256), 0, s, A)
  // ungrouped launches of an NT-thread kernel: blocks = ownedTiles * 16 of 256 threads -> ownedTiles * 4096 / NT
#define SAIL_LAUNCH_NT(k, nt, gnt)                                                              \
  do {                                                                                          \
    if (g) hipLaunchKernelGGL(k##_grouped, dim3(blocks * 256 / (gnt)), dim3(gnt), 0, s, A);     \
    else hipLaunchKernelGGL(k, dim3(blocks * 256 / (nt)), dim3(nt), 0, s, A);                     \
  } while (0)
  if (A.kernelSet == SAIL_KSET_CORNELL) SAIL_LAUNCH_NT(sail_trace_kernel_cornell, SAIL_CORNELL_NT, SAIL_CORNELL_GROUP_NT);
  else if (A.kernelSet == SAIL_KSET_ROOM) SAIL_LAUNCH_NT(sail_trace_kernel_room, SAIL_ROOM_NT, SAIL_ROOM_GROUP_NT);
  else if (A.cullPrims) SAIL_LAUNCH_NT(sail_trace_kernel_cull, SAIL_CULL_NT, SAIL_CULL_GROUP_NT);
  else SAIL_LAUNCH(sail_trace_kernel);
#undef SAIL_LAUNCH
#undef SAIL_LAUNCH_NT
  return hipGetLastError();
}
hipError_t sail_launch_accum(const SailTraceArgs& A, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(sail_accum_kernel, dim3(blocks), dim3(256), 0, s, A);
  return hipGetLastError();
}
hipError_t sail_launch_sum(const SailSumArgs& A, hipStream_t s) {
  hipLaunchKernelGGL(sail_sum_kernel, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, s, A);
  return hipGetLastError();
}
hipError_t sail_launch_negzero_unowned(float4* a, float4* b, int W, int H, int rank, int world, hipStream_t s) {
  hipLaunchKernelGGL(sail_negzero_unowned_kernel, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, a, b, W, H,
                     rank, world);
  return hipGetLastError();
}
hipError_t sail_launch_filter(const SailFilterArgs& A, hipStream_t s) {
  hipLaunchKernelGGL(sail_filter_kernel, dim3((A.W + 15) / 16, (A.H + 15) / 16), dim3(256), 0, s, A);
  return hipGetLastError();
}
hipError_t sail_launch_pick(const SailPrim* prims, int n, const float* rays, int count, int32_t* index, float* t,
                            hipStream_t s) {
  hipLaunchKernelGGL(sail_pick_kernel, dim3((count + 63) / 64), dim3(64), 0, s, prims, n, rays, count, index, t);
  return hipGetLastError();
}
hipError_t sail_launch_math(int fn, const float* x, const float* y, float* out, int count) {
  hipLaunchKernelGGL(sail_math_kernel, dim3((count + 255) / 256), dim3(256), 0, 0, fn, x, y, out, count);
  return hipGetLastError();
}
#endif  // !SAIL_JIT
