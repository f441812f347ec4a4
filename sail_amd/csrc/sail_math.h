// sail_math.h — device implementation of the build's bit-defined f32 math spec ("compat" RNG mode).
//
// GLSL leaves sin/cos/atan/acos/pow accuracy to the vendor, and Sail's hash RNG
// (src/shader/util/random.glsl:1-18) evaluates sin() at 1e4..1e6 where one ulp decides the sample, so
// the build defines each transcendental as: f32 argument -> f64, a fixed sequence of IEEE f64 basic
// operations (no FMA: the library is compiled with -ffp-contract=off), one rounding back to f32.
// The CPU oracle carries an independent copy of the same spec (oracle/ref_math.h); the GPU tests check
// the two bit-for-bit. MI355X runs f64 VALU at half the f32 rate, so a spec sin costs ~25 f64 ops.
#pragma once
#include <hip/hip_runtime.h>

namespace sm {

#define SM_D __device__ __forceinline__

// Cody-Waite split of pi/2 (33 significant bits per part: k*P_i exact for |k| < 2^20)
constexpr double kTwoOverPi = 0.6366197723675814;
constexpr double kP1 = 1.5707963267341256;
constexpr double kP2 = 6.077100506303966e-11;
constexpr double kP3 = 2.0222662487959506e-21;

SM_D double sin_poly(double r) {
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
SM_D double cos_poly(double r) {
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
SM_D double reduce_pio2(double x, int& q) {
  if (!(fabs(x) < 1e15)) { q = 0; return __builtin_nan(""); }
  const double k = floor(x * kTwoOverPi + 0.5);
  double r = x - k * kP1;
  r = r - k * kP2;
  r = r - k * kP3;
  q = (int)((long long)k & 3);
  return r;
}
SM_D double sin_d(double x) {
  int q; const double r = reduce_pio2(x, q);
  const double s = sin_poly(r), c = cos_poly(r);
  return q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
}
SM_D double cos_d(double x) {
  int q; const double r = reduce_pio2(x, q);
  const double s = sin_poly(r), c = cos_poly(r);
  return q == 0 ? c : (q == 1 ? -s : (q == 2 ? -c : s));
}
// sin and cos of one argument with one reduction (both results are the spec values)
SM_D void sincos_d(double x, double& so, double& co) {
  int q; const double r = reduce_pio2(x, q);
  const double s = sin_poly(r), c = cos_poly(r);
  so = q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
  co = q == 0 ? c : (q == 1 ? -s : (q == 2 ? -c : s));
}

constexpr double kPi = 3.141592653589793;
constexpr double kPiO2 = 1.5707963267948966;
constexpr double kPiO4 = 0.7853981633974483;
constexpr double kPiO8 = 0.39269908169872414;
constexpr double kTanPiO8 = 0.41421356237309503;
constexpr double kTanPiO16 = 0.198912367379658;

SM_D double atan_series(double z) {
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
SM_D double atan01(double a) {
  double off = 0.0;
  if (a > kTanPiO8) { a = (a - 1.0) / (a + 1.0); off = kPiO4; }
  if (a > kTanPiO16) { a = (a - kTanPiO8) / (1.0 + a * kTanPiO8); off = off + kPiO8; }
  else if (a < -kTanPiO16) { a = (a + kTanPiO8) / (1.0 - a * kTanPiO8); off = off - kPiO8; }
  return off + atan_series(a);
}
SM_D double atan2_d(double y, double x) {
  if (y != y || x != x) return y + x;
  if (y == 0.0 && x == 0.0) return 0.0;
  const double ay = fabs(y), ax = fabs(x);
  double r;
  if (ay <= ax) r = atan01(ay / ax);
  else r = kPiO2 - atan01(ax / ay);
  if (x < 0.0) r = kPi - r;
  return (y < 0.0) ? -r : r;
}
SM_D double sqrt_d(double v) {
  if (!(v > 0.0)) return (v == 0.0) ? 0.0 : __builtin_nan("");
  const double s0 = (double)__builtin_sqrtf((float)v);
  if (s0 == 0.0) return 0.0;
  return s0 + (v - s0 * s0) / (2.0 * s0);
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

// ---- f32 spec functions ----
SM_D float sinf_(float x) { return (float)sin_d((double)x); }
SM_D float cosf_(float x) { return (float)cos_d((double)x); }
SM_D void sincosf_(float x, float& s, float& c) {
  double sd, cd; sincos_d((double)x, sd, cd); s = (float)sd; c = (float)cd;
}
SM_D float tanf_(float x) {
  int q; const double r = reduce_pio2((double)x, q);
  const double s = sin_poly(r), c = cos_poly(r);
  return (float)((q & 1) ? (-c / s) : (s / c));
}
SM_D float atan2f_(float y, float x) { return (float)atan2_d((double)y, (double)x); }
SM_D float atanf_(float x) { return (float)atan2_d((double)x, 1.0); }
SM_D float acosf_(float x) {
  const double d = (double)x;
  if (!(d >= -1.0 && d <= 1.0)) return __builtin_nanf("");
  return (float)atan2_d(sqrt_d((1.0 - d) * (1.0 + d)), d);
}
SM_D float powf_(float x, float y) {
  if (x != x || y != y) return __builtin_nanf("");
  if (y == 0.0f) return 1.0f;
  if (x < 0.0f) return __builtin_nanf("");
  if (x == 0.0f) return (y > 0.0f) ? 0.0f : __builtin_inff();
  return (float)exp_d((double)y * log_d((double)x));
}
// GLSL min/max/clamp with defined NaN behaviour (return the non-NaN operand; ties keep the first)
SM_D float fmin_(float a, float b) { return (b < a) ? b : ((a != a) ? b : a); }
SM_D float fmax_(float a, float b) { return (a < b) ? b : ((a != a) ? b : a); }
SM_D float clamp_(float x, float lo, float hi) { return fmin_(fmax_(x, lo), hi); }
SM_D float fract_(float x) { return x - floorf(x); }
SM_D float sqrtf_(float x) { return __builtin_sqrtf(x); }
SM_D int to_int(float x) {
  if (x != x) return 0;
  if (x >= 2147483647.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}

}  // namespace sm
