// sail_hostmath.cpp — the reference's host-side double-precision math, restated so that every host
// language (JS via N-API, Python via ctypes) gets bit-identical per-sample uniforms from one place.
//   Camera.makePerspective / makeLookAt       src/scene/camera.js:16-57
//   Scene.mat = projection x modelview         src/scene/scene.js:40-42
//   Matrix.multiply / toRightTriangular / inverse / flatten / Translation, Vector.dot/cross/toUnitVector
//                                              src/utils/matrix.js:97-115, 324-350, 391-419, 501-527, 612-622, 683-698
//   jittered inverse per frame                 src/core/tracer.js:94-96
// Operation order follows the Sylvester-style library exactly (e.g. Vector.dot sums from the last
// component down), so the f32 uniforms equal what the reference uploads (checked against
// tests/golden/fixtures.json). Compiled with -ffp-contract=off.
#include <math.h>
#include <stdint.h>
#include <string.h>
#include "../../include/sail_hip.h"

namespace {

struct M4 { double e[4][4]; };

double vdot3(const double* a, const double* b) {  // matrix.js:97-103: product += a[n-1]*b[n-1], n = 3..1
  double p = 0.0;
  for (int n = 3; n >= 1; n--) p += a[n - 1] * b[n - 1];
  return p;
}
void vcross3(const double* A, const double* B, double* r) {  // matrix.js:105-115
  r[0] = (A[1] * B[2]) - (A[2] * B[1]);
  r[1] = (A[2] * B[0]) - (A[0] * B[2]);
  r[2] = (A[0] * B[1]) - (A[1] * B[0]);
}
void vunit3(double* v) {  // toUnitVector: x / modulus, modulus = sqrt(dot(v, v))
  const double r = sqrt(vdot3(v, v));
  if (r == 0.0) return;
  for (int i = 0; i < 3; i++) v[i] = v[i] / r;
}
M4 mmul(const M4& a, const M4& b) {  // matrix.js:324-350: sum = 0; sum += a[i][c]*b[c][j], c = 0..3
  M4 r;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      double sum = 0.0;
      for (int c = 0; c < 4; c++) sum += a.e[i][c] * b.e[c][j];
      r.e[i][j] = sum;
    }
  return r;
}
// toRightTriangular on an n x kp row set (matrix.js:391-419)
void rightTriangular(double* M, int n, int kp) {
  for (int i = 0; i < n; i++) {
    if (M[i * kp + i] == 0.0) {
      for (int j = i + 1; j < n; j++) {
        if (M[j * kp + i] != 0.0) {
          for (int p = 0; p < kp; p++) M[i * kp + p] = M[i * kp + p] + M[j * kp + p];
          break;
        }
      }
    }
    if (M[i * kp + i] != 0.0) {
      for (int j = i + 1; j < n; j++) {
        const double multiplier = M[j * kp + i] / M[i * kp + i];
        double els[8];
        for (int p = 0; p < kp; p++) els[p] = (p <= i) ? 0.0 : M[j * kp + p] - M[i * kp + p] * multiplier;
        for (int p = 0; p < kp; p++) M[j * kp + p] = els[p];
      }
    }
  }
}
bool minverse(const M4& m, M4& out) {  // matrix.js:501-527 (+ isSingular via determinant, :423-437)
  double T[16];
  memcpy(T, m.e, sizeof(T));
  rightTriangular(T, 4, 4);
  double det = T[0];
  for (int i = 1; i < 4; i++) det = det * T[i * 4 + i];
  if (det == 0.0) return false;
  double A[4 * 8];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) A[i * 8 + j] = (j < 4) ? m.e[i][j] : (j - 4 == i ? 1.0 : 0.0);
  rightTriangular(A, 4, 8);
  for (int i = 3; i >= 0; i--) {
    const double divisor = A[i * 8 + i];
    double els[8];
    for (int p = 0; p < 8; p++) els[p] = A[i * 8 + p] / divisor;
    for (int p = 0; p < 8; p++) A[i * 8 + p] = els[p];
    for (int p = 4; p < 8; p++) out.e[i][p - 4] = els[p];
    for (int j = 0; j < i; j++) {
      double nj[8];
      for (int p = 0; p < 8; p++) nj[p] = A[j * 8 + p] - A[i * 8 + p] * A[j * 8 + i];
      for (int p = 0; p < 8; p++) A[j * 8 + p] = nj[p];
    }
  }
  return true;
}
uint32_t xorshift32(uint32_t& s) {
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  return s;
}

}  // namespace

extern "C" int sail_camera(const double eye[3], const double center[3], const double up[3], double fovy,
                           double aspect, double znear, double zfar, double out[16]) {
  if (!eye || !center || !up || !out) return SAIL_E_INVALID;
  // makePerspective (camera.js:16-35)
  const double top = znear * tan(fovy * M_PI / 360.0);
  const double bottom = -top, left = bottom * aspect, right = top * aspect;
  const double X = 2 * znear / (right - left), Y = 2 * znear / (top - bottom);
  const double A = (right + left) / (right - left), B = (top + bottom) / (top - bottom);
  const double Cc = -(zfar + znear) / (zfar - znear), Dd = -2 * zfar * znear / (zfar - znear);
  M4 P = {{{X, 0, A, 0}, {0, Y, B, 0}, {0, 0, Cc, Dd}, {0, 0, -1, 0}}};
  // makeLookAt (camera.js:37-57)
  double z[3] = {eye[0] - center[0], eye[1] - center[1], eye[2] - center[2]};
  vunit3(z);
  double x[3], y[3];
  vcross3(up, z, x);
  vunit3(x);
  vcross3(z, x, y);
  vunit3(y);
  for (int i = 0; i < 3; i++) x[i] = x[i] * -1;
  M4 m = {{{x[0], x[1], x[2], 0}, {y[0], y[1], y[2], 0}, {z[0], z[1], z[2], 0}, {0, 0, 0, 1}}};
  M4 t = {{{1, 0, 0, -eye[0]}, {0, 1, 0, -eye[1]}, {0, 0, 1, -eye[2]}, {0, 0, 0, 1}}};
  const M4 mv = mmul(m, t);
  const M4 mat = mmul(P, mv);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) out[i * 4 + j] = mat.e[i][j];
  return SAIL_OK;
}

extern "C" int sail_jitter_inverse(const double mvp[16], double jx, double jy, int width, int height, float inv[16]) {
  if (!mvp || !inv || width <= 0 || height <= 0) return SAIL_E_INVALID;
  // Matrix.Translation(new Vector([jx, jy, 0]).multiply(1/512)) generalised to 1/W, 1/H (tracer.js:94-96)
  M4 T = {{{1, 0, 0, jx * (1.0 / width)}, {0, 1, 0, jy * (1.0 / height)}, {0, 0, 1, 0 * (1.0 / width)}, {0, 0, 0, 1}}};
  M4 m;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) m.e[i][j] = mvp[i * 4 + j];
  M4 r;
  if (!minverse(mmul(T, m), r)) return SAIL_E_INVALID;
  for (int j = 0; j < 4; j++)  // flatten(): column-major (matrix.js:612-622)
    for (int i = 0; i < 4; i++) inv[j * 4 + i] = (float)r.e[i][j];
  return SAIL_OK;
}

extern "C" int sail_schedule(const double mvp[16], int width, int height, int k0, int spp, float* inv, float* seeds) {
  if (!mvp || spp < 0 || k0 < 0 || (spp > 0 && (!inv || !seeds))) return SAIL_E_INVALID;
  for (int s = 0; s < spp; s++) {
    const int k = k0 + s;
    uint32_t st = 0x5A11u + (uint32_t)k;
    const double r1 = (double)xorshift32(st) / 4294967296.0;
    const double r2 = (double)xorshift32(st) / 4294967296.0;
    const int rc = sail_jitter_inverse(mvp, r1 * 2 - 1, r2 * 2 - 1, width, height, inv + 16 * s);
    if (rc) return rc;
    // timeSinceStart = ms * 0.001 with ms = round(1000 (k+1) / 60)  (JS Math.round: half up)
    const double ms = floor(1000.0 * (k + 1) / 60.0 + 0.5);
    seeds[s] = (float)(ms * 0.001);
  }
  return SAIL_OK;
}
