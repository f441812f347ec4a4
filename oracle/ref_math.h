// oracle/ref_math.h — TEST INFRASTRUCTURE (CPU oracle only; never linked into the product).
//
// Bit-defined fp32 transcendentals ("compat" math spec, SURVEY §7 hard parts: RNG parity).
// GLSL leaves sin/cos/atan/acos/pow precision to the vendor (random.glsl:1-18 evaluates sin at
// arguments of 1e4..1e6, where a 1-ulp difference yields an unrelated sample), so the build DEFINES
// each one as: promote the f32 argument to f64, evaluate a fixed sequence of IEEE-754 f64 basic
// operations (+ - * / only; no FMA contraction, no libm), round the result to f32 once.
// The HIP kernel implements the same spec independently in sail_amd/csrc/sail_math.h; the GPU parity
// tests check the two bit-for-bit over millions of arguments.
//
// Also defined here (GLSL semantics the reference leaves open, SURVEY §7 "undefined behaviour"):
//   min/max  -> select form that returns the non-NaN operand (GPU v_min/v_max behaviour); ties keep a
//   sqrt     -> IEEE correctly-rounded f32 sqrt
//   int(x)   -> truncation, NaN -> 0, saturating
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

namespace refm {

static inline double dfloor(double x) { return floor(x); }  // exact on every platform

// ---- sin / cos: Cody-Waite 3-part pi/2 reduction (each part 33 significant bits, so k*Pi is exact
//      for |k| < 2^20, i.e. |x| < ~1.6e6) followed by Taylor polynomials on [-pi/4, pi/4].
static const double kTwoOverPi = 0.6366197723675814;
static const double kP1 = 1.5707963267341256;
static const double kP2 = 6.077100506303966e-11;
static const double kP3 = 2.0222662487959506e-21;

static inline double sin_poly(double r) {  // r - r^3/3! + ... - r^19/19!
  const double r2 = r * r;
  double p = -8.22063524662433e-18;
  p = p * r2 + 2.8114572543455206e-15;
  p = p * r2 + -7.647163731819816e-13;
  p = p * r2 + 1.6059043836821613e-10;
  p = p * r2 + -2.505210838544172e-08;
  p = p * r2 + 2.7557319223985893e-06;
  p = p * r2 + -0.0001984126984126984;
  p = p * r2 + 0.008333333333333333;
  p = p * r2 + -0.16666666666666666;
  return r + (r * r2) * p;
}
static inline double cos_poly(double r) {  // 1 - r^2/2! + ... - r^18/18!
  const double r2 = r * r;
  double p = -1.5619206968586225e-16;
  p = p * r2 + 4.779477332387385e-14;
  p = p * r2 + -1.1470745597729725e-11;
  p = p * r2 + 2.08767569878681e-09;
  p = p * r2 + -2.755731922398589e-07;
  p = p * r2 + 2.48015873015873e-05;
  p = p * r2 + -0.001388888888888889;
  p = p * r2 + 0.041666666666666664;
  p = p * r2 + -0.5;
  return 1.0 + r2 * p;
}
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
static inline double sin_d(double x) {
  int q; const double r = reduce_pio2(x, &q);
  switch (q) {
    case 0: return sin_poly(r);
    case 1: return cos_poly(r);
    case 2: return -sin_poly(r);
    default: return -cos_poly(r);
  }
}
static inline double cos_d(double x) {
  int q; const double r = reduce_pio2(x, &q);
  switch (q) {
    case 0: return cos_poly(r);
    case 1: return -sin_poly(r);
    case 2: return -cos_poly(r);
    default: return sin_poly(r);
  }
}

// ---- atan / atan2: |a| in [0,1] reduced twice (pi/4 then pi/8 shifts) to |z| <= tan(pi/16),
//      then the odd Taylor series to z^23.
static const double kPi = 3.141592653589793;
static const double kPiO2 = 1.5707963267948966;
static const double kPiO4 = 0.7853981633974483;
static const double kPiO8 = 0.39269908169872414;
static const double kTanPiO8 = 0.41421356237309503;
static const double kTanPiO16 = 0.198912367379658;

static inline double atan_series(double z) {
  const double z2 = z * z;
  double p = 1.0 / 23.0;
  p = -p * z2 + 1.0 / 21.0;
  p = -p * z2 + 1.0 / 19.0;
  p = -p * z2 + 1.0 / 17.0;
  p = -p * z2 + 1.0 / 15.0;
  p = -p * z2 + 1.0 / 13.0;
  p = -p * z2 + 1.0 / 11.0;
  p = -p * z2 + 1.0 / 9.0;
  p = -p * z2 + 1.0 / 7.0;
  p = -p * z2 + 1.0 / 5.0;
  p = -p * z2 + 1.0 / 3.0;
  p = -p * z2 + 1.0;
  return z * p;
}
// atan for a in [0, 1]
static inline double atan01(double a) {
  double off = 0.0;
  if (a > kTanPiO8) { a = (a - 1.0) / (a + 1.0); off = kPiO4; }     // a in (-0.4143, 0]
  if (a > kTanPiO16) { a = (a - kTanPiO8) / (1.0 + a * kTanPiO8); off = off + kPiO8; }
  else if (a < -kTanPiO16) { a = (a + kTanPiO8) / (1.0 - a * kTanPiO8); off = off - kPiO8; }
  return off + atan_series(a);
}
static inline double atan2_d(double y, double x) {
  if (y != y || x != x) return y + x;                       // NaN
  if (y == 0.0 && x == 0.0) return 0.0;                    // GLSL: undefined; defined 0
  const double ay = fabs(y), ax = fabs(x);
  double r;
  if (ay <= ax) r = atan01(ay / ax);                        // |angle| <= pi/4
  else r = kPiO2 - atan01(ax / ay);
  if (x < 0.0) r = kPi - r;
  return (y < 0.0) ? -r : r;
}

// ---- f64 sqrt from a correctly rounded f32 seed plus one Newton step (basic ops only)
static inline double sqrt_d(double v) {
  if (!(v > 0.0)) return (v == 0.0) ? 0.0 : NAN;
  const double s0 = (double)sqrtf((float)v);
  if (s0 == 0.0) return 0.0;
  return s0 + (v - s0 * s0) / (2.0 * s0);
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

// ---- the f32 spec functions
static inline float sin_s(float x) { return (float)sin_d((double)x); }
static inline float cos_s(float x) { return (float)cos_d((double)x); }
static inline float tan_s(float x) {
  int q; const double r = reduce_pio2((double)x, &q);
  const double s = sin_poly(r), c = cos_poly(r);
  return (float)((q & 1) ? (-c / s) : (s / c));
}
static inline float atan2_s(float y, float x) { return (float)atan2_d((double)y, (double)x); }
static inline float atan_s(float x) { return (float)atan2_d((double)x, 1.0); }
static inline float acos_s(float x) {
  const double d = (double)x;
  if (!(d >= -1.0 && d <= 1.0)) return NAN;
  return (float)atan2_d(sqrt_d((1.0 - d) * (1.0 + d)), d);
}
static inline float pow_s(float x, float y) {
  if (x != x || y != y) return NAN;
  if (y == 0.0f) return 1.0f;
  if (x < 0.0f) return NAN;                                // GLSL: undefined for x < 0
  if (x == 0.0f) return (y > 0.0f) ? 0.0f : INFINITY;
  return (float)exp_d((double)y * log_d((double)x));
}
static inline float exp_s(float x) { return (float)exp_d((double)x); }
static inline float log_s(float x) { return (float)log_d((double)x); }

// GLSL builtins with defined NaN behaviour
static inline float fmin_s(float a, float b) { return (b < a) ? b : ((a != a) ? b : a); }
static inline float fmax_s(float a, float b) { return (a < b) ? b : ((a != a) ? b : a); }
static inline float floor_s(float x) { return floorf(x); }
static inline float fract_s(float x) { return x - floorf(x); }
static inline float sqrt_s(float x) { return sqrtf(x); }
static inline int to_int(float x) {
  if (x != x) return 0;
  if (x >= 2147483647.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

}  // namespace refm
