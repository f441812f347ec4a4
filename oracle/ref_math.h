// oracle/ref_math.h — TEST INFRASTRUCTURE (CPU oracle only; never linked into the product).
//
// Bit-defined fp32 transcendentals ("compat" math spec v3, SURVEY §7 hard parts: RNG parity).
// GLSL leaves sin/cos/atan/acos/pow precision to the vendor (random.glsl:1-18 evaluates sin at
// arguments of 1e4..1e6, where a 1-ulp difference yields an unrelated sample), so the build DEFINES
// each one as a fixed sequence of IEEE-754 operations: range reduction for sin/cos/tan (three f32 FMAs below 2^20,
// exact f64 beyond), then f32
// polynomials with explicit fused multiply-adds (fmaf); no contraction anywhere else, no libm.
// The HIP kernel implements the same spec independently in sail_amd/csrc/sail_math.h; the GPU parity
// tests check the two bit-for-bit over millions of arguments.
//
// Also defined here (GLSL semantics the reference leaves open, SURVEY §7 "undefined behaviour"):
//   min/max  -> IEEE-754-2019 minimumNumber/maximumNumber (NaN -> other operand, -0 < +0), which is what
//               GLSL min/max compile to on AMD GPUs (v_min_f32 / v_max_f32)
//   sqrt     -> IEEE correctly-rounded f32 sqrt
//   a / b    -> a * RN(1/b): the reciprocal-multiply form GPU shader compilers emit for GLSL division (GLSL ES
//               3.00 §4.5.1 allows 2.5 ulp), with the reciprocal correctly rounded so that every implementation
//               reproduces it (the MI355X sequence is checked against 1.0f/b for all 2^32 inputs,
//               tools/rcp_probe.hip). Applies to every GLSL float division; the spec functions above keep
//               their internal IEEE divides.
//   int(x)   -> truncation, NaN -> 0, saturating
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

namespace refm {

static inline double dfloor(double x) { return floor(x); }  // exact on every platform

// ---- sin / cos / tan range reduction: Cody-Waite 3-part pi/2 in f64 (each part 33 significant bits, so
//      k*P_i is exact for |k| < 2^20, i.e. |x| < ~1.6e6).
static const double kTwoOverPi = 0.6366197723675814;
static const double kP1 = 1.5707963267341256;
static const double kP2 = 6.077100506303966e-11;
static const double kP3 = 2.0222662487959506e-21;

// returns quadrant q (0..3) and reduced r
static inline double reduce_pio2(double x, int* q) {
  if (!(fabs(x) < 1e15)) { *q = 0; return NAN; }          // inf / NaN / absurd range
  const double k = dfloor(x * kTwoOverPi + 0.5);
  double r = x - k * kP1;
  r = r - k * kP2;
  r = r - k * kP3;
  long long ki = (long long)k;
  *q = (int)(ki & 3);
  return r;
}
// ---- exp2 / log2 in f64 (gamma filter pow only)
static inline double ldexp_i(double m, int e) {  // m * 2^e by repeated exact scaling
  while (e > 0) { const int s = e > 60 ? 60 : e; m = m * (double)(1ull << s); e -= s; }
  while (e < 0) { const int s = -e > 60 ? 60 : -e; m = m / (double)(1ull << s); e += s; }
  return m;
}
static const double kLn2Hi = 0.6931471803691238;
static const double kLn2Lo = 1.9082149292705877e-10;
static const double kInvLn2 = 1.4426950408889634;
static inline double exp_d(double x) {
  if (x != x) return x;
  if (x > 709.0) return INFINITY;
  if (x < -745.0) return 0.0;
  const double k = dfloor(x * kInvLn2 + 0.5);
  const double r = (x - k * kLn2Hi) - k * kLn2Lo;        // |r| <= ~0.347
  double p = 1.0 / 6227020800.0;                          // 1/13!
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
static inline double log_d(double x) {
  if (x != x || x < 0.0) return NAN;
  if (x == 0.0) return -INFINITY;
  if (x == INFINITY) return x;
  int e = 0;
  double m = x;                                            // bring m into [sqrt(1/2), sqrt(2))
  while (m >= 1.4142135623730951) { m = m * 0.5; e++; }
  while (m < 0.7071067811865476) { m = m * 2.0; e--; }
  const double s = (m - 1.0) / (m + 1.0), s2 = s * s;     // |s| <= 0.1716
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

// ---- the f32 spec functions (spec v3) ------------------------------------------------------------------
// sin/cos/tan: the f64 Cody-Waite reduction above (exact k*P_i for |x| < ~1.6e6, which covers the hash
// RNG's 1e4..1e6 arguments), then ONE rounding of r to f32 and f32 polynomials evaluated with fused
// multiply-adds (fmaf: correctly rounded on every platform). atan/atan2/acos are f32 throughout.
// Coefficients: least-squares fits made for this build (tools/fit_spec_math.py); accuracy <= 2 ulp.
static const float kS0 = -0.166666641831398f, kS1 = 0.008332744240760803f, kS2 = -0.0001958730281330645f;
static const float kC0 = 0.0416666641831398f, kC1 = -0.0013888344401493669f, kC2 = 2.455315006955061e-05f;
static const float kA[9] = {-0.3333333134651184f, 0.19999729096889496f, -0.142783522605896f, 0.11032091081142426f,
                            -0.08650501817464828f, 0.062368933111429214f, -0.03571782633662224f,
                            0.01341481227427721f, -0.002364102052524686f};
static const float kB[5] = {0.16666673123836517f, 0.07498858869075775f, 0.045000601559877396f,
                            0.026559552177786827f, 0.03807495906949043f};
static const float kPiF = 3.14159274f, kPiO2F = 1.57079637f;

static inline float sinpoly_f(float r) {  // r + r^3 P(r^2), |r| <= pi/4
  const float z = r * r;
  const float p = fmaf(fmaf(kS2, z, kS1), z, kS0);
  return fmaf(r * z, p, r);
}
static inline float cospoly_f(float r) {  // 1 - r^2/2 + r^4 Q(r^2)
  const float z = r * r;
  const float q = fmaf(fmaf(kC2, z, kC1), z, kC0);
  return fmaf(z * z, q, fmaf(-0.5f, z, 1.0f));
}
// spec v3 reduction (sail_math.h reduce_spec): |x| < 2^20 -> j = rint(RN(x * 2/pi)) (round half to even), then
// r = x - j*(A + B + C) by three FMAs; beyond, the f64 reduction above rounded to f32
static const float kInvPiO2F = 0x1.45f306p-1f, kPiO2A = 0x1.921fb6p+0f, kPiO2B = -0x1.777a5cp-25f,
                   kPiO2C = -0x1.ee59dap-50f;
static inline float reduce_spec(float x, int* q) {
  if (fabsf(x) < 0x1p20f) {
    const float j = rintf(x * kInvPiO2F);   // default rounding mode: to nearest, ties to even
    float r = fmaf(-j, kPiO2A, x);
    r = fmaf(-j, kPiO2B, r);
    r = fmaf(-j, kPiO2C, r);
    *q = (int)j & 3;
    return r;
  }
  return (float)reduce_pio2((double)x, q);
}
static inline void sincos_s(float x, float* so, float* co) {
  int q; const float rf = reduce_spec(x, &q);
  const float s = sinpoly_f(rf), c = cospoly_f(rf);
  switch (q) {
    case 0: *so = s; *co = c; break;
    case 1: *so = c; *co = -s; break;
    case 2: *so = -s; *co = -c; break;
    default: *so = -c; *co = s; break;
  }
}
static inline float sin_s(float x) { float s, c; sincos_s(x, &s, &c); return s; }
static inline float cos_s(float x) { float s, c; sincos_s(x, &s, &c); return c; }
static inline float tan_s(float x) {
  int q; const float rf = reduce_spec(x, &q);
  const float s = sinpoly_f(rf), c = cospoly_f(rf);
  return (q & 1) ? (-c / s) : (s / c);
}
static inline float atan01_f(float t) {  // atan on [0, 1]: t + t^3 P(t^2)
  const float z = t * t;
  float p = kA[8];
  for (int i = 7; i >= 0; i--) p = fmaf(p, z, kA[i]);
  return fmaf(t * z, p, t);
}
static inline float atan2_s(float y, float x) {
  if (y != y || x != x) return y + x;
  if (y == 0.0f && x == 0.0f) return 0.0f;  // GLSL: undefined; defined 0
  const float ay = fabsf(y), ax = fabsf(x);
  float r = (ay <= ax) ? atan01_f(ay / ax) : kPiO2F - atan01_f(ax / ay);
  if (x < 0.0f) r = kPiF - r;
  return (y < 0.0f) ? -r : r;
}
static inline float atan_s(float x) { return atan2_s(x, 1.0f); }
static inline float asinpoly_f(float x) {  // asin on [-0.5, 0.5]: x + x^3 P(x^2)
  const float z = x * x;
  float p = kB[4];
  for (int i = 3; i >= 0; i--) p = fmaf(p, z, kB[i]);
  return fmaf(x * z, p, x);
}
static inline float acos_s(float x) {
  if (!(x >= -1.0f && x <= 1.0f)) return NAN;
  const float ax = fabsf(x);
  if (ax <= 0.5f) return kPiO2F - asinpoly_f(x);
  const float a2 = 2.0f * asinpoly_f(sqrtf((1.0f - ax) * 0.5f));
  return (x > 0.0f) ? a2 : kPiF - a2;
}
static inline float pow_s(float x, float y) {  // display gamma only: f64 exp/log
  if (x != x || y != y) return NAN;
  if (y == 0.0f) return 1.0f;
  if (x < 0.0f) return NAN;                                // GLSL: undefined for x < 0
  if (x == 0.0f) return (y > 0.0f) ? 0.0f : INFINITY;
  return (float)exp_d((double)y * log_d((double)x));
}
static inline float exp_s(float x) { return (float)exp_d((double)x); }
static inline float log_s(float x) { return (float)log_d((double)x); }

// GLSL builtins with defined NaN behaviour
// min/max as the MI355X v_min_f32/v_max_f32 compute them (measured: tools/probe_minmax.py): a NaN operand
// yields the other operand; -0 orders below +0 whatever the operand order.
static inline float fmin_s(float a, float b) {
  if (a != a) return b;
  if (b != b) return a;
  if (a < b) return a;
  if (b < a) return b;
  return signbit(a) ? a : b;
}
static inline float fmax_s(float a, float b) {
  if (a != a) return b;
  if (b != b) return a;
  if (a > b) return a;
  if (b > a) return b;
  return signbit(a) ? b : a;
}
static inline float floor_s(float x) { return floorf(x); }
static inline float fract_s(float x) { return x - floorf(x); }
static inline float sqrt_s(float x) { return sqrtf(x); }
static inline float rcp_s(float b) { return 1.0f / b; }              // RN(1/b), IEEE
static inline float div_s(float a, float b) { return a * rcp_s(b); }  // GLSL a / b
static inline int to_int(float x) {
  if (x != x) return 0;
  if (x >= 2147483647.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

}  // namespace refm
