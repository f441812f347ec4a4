// sail_math.h — device implementation of the build's bit-defined f32 math spec v3 ("compat" RNG mode).
//
// GLSL leaves sin/cos/atan/acos/pow accuracy to the vendor, and Sail's hash RNG
// (src/shader/util/random.glsl:1-18) evaluates sin() at 1e4..1e6 where one ulp decides the sample, so
// the build defines each transcendental as a fixed IEEE operation sequence: a Cody-Waite reduction for
// sin/cos/tan (three f32 FMAs below 2^20, exact f64 beyond: reduce_spec), then f32 polynomials with explicit FMAs
// (bounds in DESIGN.md §4). The library is compiled with -ffp-contract=off, so no other FMA is formed. The CPU oracle
// carries an independent copy of the spec (oracle/ref_math.h); the GPU tests check them bit-for-bit.
#pragma once
#if !defined(__HIPCC_RTC__)
#include <hip/hip_runtime.h>
#endif

namespace sm {

#define SM_D __device__ __forceinline__

// Cody-Waite split of pi/2 (33 significant bits per part: k*P_i exact for |k| < 2^20)
constexpr double kTwoOverPi = 0.6366197723675814;
constexpr double kP1 = 1.5707963267341256;
constexpr double kP2 = 6.077100506303966e-11;
constexpr double kP3 = 2.0222662487959506e-21;

SM_D double reduce_pio2(double x, int& q) {
  if (!(fabs(x) < 1e15)) { q = 0; return __builtin_nan(""); }
  const double k = floor(x * kTwoOverPi + 0.5);
  double r = x - k * kP1;
  r = r - k * kP2;
  r = r - k * kP3;
  // q = k mod 4 (two's complement, = (long long)k & 3): k is integral with |k| < 2^50, so k + 1.5*2^52 is exact
  // and its low word holds k mod 2^32 (one f64 add instead of the compiler's 64-bit conversion sequence)
  q = (int)(__double2loint(k + 6755399441055744.0) & 3);
  return r;
}
constexpr double kLn2Hi = 0.6931471803691238;
constexpr double kLn2Lo = 1.9082149292705877e-10;
constexpr double kInvLn2 = 1.4426950408889634;
SM_D double ldexp_i(double m, int e) {
  while (e > 0) { const int s = e > 60 ? 60 : e; m = m * (double)(1ull << s); e -= s; }
  while (e < 0) { const int s = -e > 60 ? 60 : -e; m = m / (double)(1ull << s); e += s; }
  return m;
}
SM_D double exp_d(double x) {
  if (x != x) return x;
  if (x > 709.0) return __builtin_inf();
  if (x < -745.0) return 0.0;
  const double k = floor(x * kInvLn2 + 0.5);
  const double r = (x - k * kLn2Hi) - k * kLn2Lo;
  double p = 1.0 / 6227020800.0;
  p = p * r + 1.0 / 479001600.0;
  p = p * r + 1.0 / 39916800.0;
  p = p * r + 1.0 / 3628800.0;
  p = p * r + 1.0 / 362880.0;
  p = p * r + 1.0 / 40320.0;
  p = p * r + 1.0 / 5040.0;
  p = p * r + 1.0 / 720.0;
  p = p * r + 1.0 / 120.0;
  p = p * r + 1.0 / 24.0;
  p = p * r + 1.0 / 6.0;
  p = p * r + 0.5;
  p = p * r + 1.0;
  p = p * r + 1.0;
  return ldexp_i(p, (int)k);
}
SM_D double log_d(double x) {
  if (x != x || x < 0.0) return __builtin_nan("");
  if (x == 0.0) return -__builtin_inf();
  if (x == __builtin_inf()) return x;
  int e = 0;
  double m = x;
  while (m >= 1.4142135623730951) { m = m * 0.5; e++; }
  while (m < 0.7071067811865476) { m = m * 2.0; e--; }
  const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
  double p = 1.0 / 23.0;
  p = p * s2 + 1.0 / 21.0;
  p = p * s2 + 1.0 / 19.0;
  p = p * s2 + 1.0 / 17.0;
  p = p * s2 + 1.0 / 15.0;
  p = p * s2 + 1.0 / 13.0;
  p = p * s2 + 1.0 / 11.0;
  p = p * s2 + 1.0 / 9.0;
  p = p * s2 + 1.0 / 7.0;
  p = p * s2 + 1.0 / 5.0;
  p = p * s2 + 1.0 / 3.0;
  p = p * s2 + 1.0;
  return ((double)e * kLn2Hi + (2.0 * s) * p) + (double)e * kLn2Lo;
}

// ---- f32 spec functions (spec v3): f32 / f64 reduction for sin/cos/tan (reduce_spec), then f32 polynomials with explicit
//      fused multiply-adds (v_fma_f32 is correctly rounded: identical to the oracle's fmaf) ----
constexpr float kS0 = -0.166666641831398f, kS1 = 0.008332744240760803f, kS2 = -0.0001958730281330645f;
constexpr float kC0 = 0.0416666641831398f, kC1 = -0.0013888344401493669f, kC2 = 2.455315006955061e-05f;
constexpr float kA0 = -0.3333333134651184f, kA1 = 0.19999729096889496f, kA2 = -0.142783522605896f,
                kA3 = 0.11032091081142426f, kA4 = -0.08650501817464828f, kA5 = 0.062368933111429214f,
                kA6 = -0.03571782633662224f, kA7 = 0.01341481227427721f, kA8 = -0.002364102052524686f;
constexpr float kB0 = 0.16666673123836517f, kB1 = 0.07498858869075775f, kB2 = 0.045000601559877396f,
                kB3 = 0.026559552177786827f, kB4 = 0.03807495906949043f;
constexpr float kPiF = 3.14159274f, kPiO2F = 1.57079637f;

SM_D float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
SM_D float sinpoly_f(float r) {
  const float z = r * r;
  return fma_(r * z, fma_(fma_(kS2, z, kS1), z, kS0), r);
}
SM_D float cospoly_f(float r) {
  const float z = r * r;
  return fma_(z * z, fma_(fma_(kC2, z, kC1), z, kC0), fma_(-0.5f, z, 1.0f));
}
// spec v3 reduction: for |x| < 2^20 (every hash argument of a frame up to ~60,000 samples, and every angle) the
// f32 Cody-Waite reduction GPU libraries use: j = rint(RN(x * 2/pi)), r = x - j*(A + B + C) by three FMAs (A + B + C =
// pi/2 to 2^-76; the first FMA is exact, each later one rounds once). Within 2.5 ulp of sin/cos for |x| < 1e4 and
// within 2^-22 absolutely below 2^20 (tests/test_oracle_fixtures.py); beyond 2^20, the exact f64 reduction of v2.
constexpr float kInvPiO2F = 0x1.45f306p-1f, kPiO2A = 0x1.921fb6p+0f, kPiO2B = -0x1.777a5cp-25f,
                kPiO2C = -0x1.ee59dap-50f;
SM_D float reduce_spec(float x, int& q) {
  if (__builtin_expect(__builtin_fabsf(x) < 0x1p20f, 1)) {
    const float j = __builtin_rintf(x * kInvPiO2F);
    float r = fma_(-j, kPiO2A, x);
    r = fma_(-j, kPiO2B, r);
    r = fma_(-j, kPiO2C, r);
    q = (int)j & 3;
    return r;
  }
  return (float)reduce_pio2((double)x, q);
}
SM_D void sincosf_(float x, float& so, float& co) {
  int q; const float rf = reduce_spec(x, q);
  const float s = sinpoly_f(rf), c = cospoly_f(rf);
  // the quadrant by bits, branch-free: odd q swaps sin and cos; the sign flips of -s / -c are sign-bit xors (exact)
  const bool odd = (q & 1) != 0;
  const unsigned fs = (unsigned)(q & 2) << 30, fc = (unsigned)((q + 1) & 2) << 30;
  so = __uint_as_float(__float_as_uint(odd ? c : s) ^ fs);
  co = __uint_as_float(__float_as_uint(odd ? s : c) ^ fc);
}
SM_D float sinf_(float x) { float s, c; sincosf_(x, s, c); return s; }
SM_D float cosf_(float x) { float s, c; sincosf_(x, s, c); return c; }
SM_D float tanf_(float x) {
  int q; const float rf = reduce_spec(x, q);
  const float s = sinpoly_f(rf), c = cospoly_f(rf);
  return (q & 1) ? (-c / s) : (s / c);
}
SM_D float atan01_f(float t) {
  const float z = t * t;
  float p = kA8;
  p = fma_(p, z, kA7); p = fma_(p, z, kA6); p = fma_(p, z, kA5); p = fma_(p, z, kA4);
  p = fma_(p, z, kA3); p = fma_(p, z, kA2); p = fma_(p, z, kA1); p = fma_(p, z, kA0);
  return fma_(t * z, p, t);
}
SM_D float atan2f_(float y, float x) {
  if (y != y || x != x) return y + x;
  if (y == 0.0f && x == 0.0f) return 0.0f;
  const float ay = fabsf(y), ax = fabsf(x);
  float r = (ay <= ax) ? atan01_f(ay / ax) : kPiO2F - atan01_f(ax / ay);
  if (x < 0.0f) r = kPiF - r;
  return (y < 0.0f) ? -r : r;
}
SM_D float atanf_(float x) { return atan2f_(x, 1.0f); }
SM_D float asinpoly_f(float x) {
  const float z = x * x;
  float p = kB4;
  p = fma_(p, z, kB3); p = fma_(p, z, kB2); p = fma_(p, z, kB1); p = fma_(p, z, kB0);
  return fma_(x * z, p, x);
}
SM_D float acosf_(float x) {
  if (!(x >= -1.0f && x <= 1.0f)) return __builtin_nanf("");
  const float ax = fabsf(x);
  if (ax <= 0.5f) return kPiO2F - asinpoly_f(x);
  const float a2 = 2.0f * asinpoly_f(__builtin_sqrtf((1.0f - ax) * 0.5f));
  return (x > 0.0f) ? a2 : kPiF - a2;
}
SM_D float powf_(float x, float y) {
  if (x != x || y != y) return __builtin_nanf("");
  if (y == 0.0f) return 1.0f;
  if (x < 0.0f) return __builtin_nanf("");
  if (x == 0.0f) return (y > 0.0f) ? 0.0f : __builtin_inff();
  return (float)exp_d((double)y * log_d((double)x));
}
SM_D float expf_(float x) { return (float)exp_d((double)x); }  // wavelet weights only
// GLSL min/max/clamp: the hardware v_min_f32/v_max_f32 (a NaN operand yields the other; -0 < +0)
SM_D float fmin_(float a, float b) { return __builtin_fminf(a, b); }
SM_D float fmax_(float a, float b) { return __builtin_fmaxf(a, b); }
// clamp = max then min. With the bounds (0, 1) or (-1, 1) that is exactly one v_med3_f32 (which the compiler
// may also fold into the producing instruction's output clamp modifier): equal for every f32 x, NaN and signed
// zeros included (tools/med3_probe.hip, all 2^32 inputs on an MI355X, profiles/r02_med3_probe.json)
SM_D float clamp_(float x, float lo, float hi) {
  if (__builtin_constant_p(lo) && __builtin_constant_p(hi) && (lo == 0.0f || lo == -1.0f) && hi == 1.0f)
    return __builtin_amdgcn_fmed3f(x, lo, hi);
  return fmin_(fmax_(x, lo), hi);
}
SM_D float fract_(float x) { return x - floorf(x); }
// sqrtf_ for arguments that are +-0, NaN or in [2^-96, 1] by construction, where v_sqrt_f32 plus the
// two-neighbour residual correction equals the IEEE square root bit for bit (tools/sqrt01_probe.hip: every such f32
// on an MI355X; below 2^-96 the hardware root needs the general lowering's scaling). The callers' arguments:
//  * max(0, 1 - t), 1 - t with t in [0, 1]: 0, or at least 2^-24 (1 - t is exact for t > 1/2, >= 1/2 otherwise);
//  * fract(y) of the hash (random.glsl), y = RN(A + s), A = RN(sin(.) 43758.5453), s = RN(seed + depth): a nonzero
//    y below 1 is a multiple of the smaller ulp of A and s; |s| is 0 or >= 2^-24 (seed near -depth has ulp >=
//    2^-24), |A| is 0 or far above 2^-60 (the sine of an f32 argument of magnitude >= 75 stays above ~2^-30), so
//    fract(y) is 0 or above 2^-84; y >= 1 leaves multiples of 2^-23.
// The general lowering's scaling and class fix-ups (7 instructions) are not needed there.
SM_D float sqrt01(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
  float r = s;
  if (__builtin_fmaf(-sdn, s, x) <= 0.0f) r = sdn;
  if (__builtin_fmaf(-sup, s, x) > 0.0f) r = sup;
  return r;
}
// The general square root is the IEEE one. (The same residual-corrected core with the IEEE root behind a branch for
// tiny, subnormal and negative arguments was exact on all 2^32 inputs, profiles/r03_sqrt_probe.json, but measured
// C2 +0.1 %, C3 -0.5 %, C4 -0.6 %.)
SM_D float sqrtg(float x) { return __builtin_sqrtf(x); }
SM_D float sqrtf_(float x) { return sqrtg(x); }
// GLSL division a / b := a * RN(1/b) (the reciprocal-multiply form shader compilers emit, with the reciprocal
// correctly rounded; oracle/ref_math.h div_s). RN(1/b) = one Newton step from the hardware reciprocal, equal to
// the IEEE 1.0f / b for every f32 b with 2^-126 <= |b| <= 2^126 (all 2^32 inputs checked on an MI355X:
// tools/rcp_probe.hip); zero, inf, NaN, subnormal and huge divisors take the IEEE divide. Literal divisors fold.
SM_D float rcp_rn(float b) {
  if (__builtin_constant_p(b)) return 1.0f / b;
  const float ab = __builtin_fabsf(b);
  // the IEEE fallback sits behind a real branch: an empty volatile asm on its input keeps the compiler from
  // if-converting it (the select form ran the ~12-instruction IEEE divide at every call; C2 +0.8 %). The branch is
  // wave-uniform (round 6): taken when some active lane's divisor is out of range, and then for every active lane -- the
  // IEEE 1.0f / b equals the Newton step's result wherever that is in range -- so the common case runs no exec-mask
  // bookkeeping (C1 +1.2 %, C3 -0.3 %, C4 +1.5 %, bit-identical; profiles/r06_uniform_guards.jsonl).
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(ab >= 0x1p-126f && ab <= 0x1p126f)) != 0ull, 0)) {
    float bb = b;
    __asm__ volatile("" : "+v"(bb));
    return 1.0f / bb;
  }
  const float y0 = __builtin_amdgcn_rcpf(b);
  return fma_(fma_(-b, y0, 1.0f), y0, y0);
}
SM_D float fdiv(float a, float b) { return a * rcp_rn(b); }
SM_D int to_int(float x) {
  if (x != x) return 0;
  if (x >= 2147483647.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

}  // namespace sm
