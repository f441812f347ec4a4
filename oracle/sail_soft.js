'use strict';
// oracle/sail_soft.js — TEST INFRASTRUCTURE: the JS/Node software restatement of the Sail trace shader.
//
// BASELINE.json's north star names "a single-thread JS/Node software fallback of the same shader" as the CPU
// baseline; this is it. It restates the generated GLSL trace program (src/shader/**, as assembled by
// src/core/shader.js:58-76) in plain JavaScript with f32 semantics — Math.fround after every operation, the
// build's compat math spec (oracle/ref_math.h) with an exactly rounded f32 fused multiply-add — and follows
// oracle/sail_oracle.cpp function for function, so the two CPU restatements and the HIP kernel can be checked
// against each other bit for bit (tests/test_soft_js.py). It is never part of the product: only tests/ and
// bench.py's cpu_baseline leg run it.
//
// Usage (Node): const soft = require('./oracle/sail_soft'); soft.render(scene, opts) -> {accum, segments}
//   or: node oracle/sail_soft.js job.json out.f32   (job: scene rows, masks, W, H, crop, inv, seeds, eye, ...)

const f = Math.fround;
// GLSL division a / b := a * RN(1/b) (oracle/ref_math.h div_s): f(1 / b) is RN32(1/b) (the f64 quotient of two
// f32 values never lies within 2^-49 of an f32 rounding midpoint it does not equal) and a * r is exact in f64
const fdiv = (a, b) => f(a * f(1 / b));

// ---- f32 bit helpers and an exactly rounded f32 fma -------------------------------------------------------
const _f32 = new Float32Array(1), _u32 = new Uint32Array(_f32.buffer);
function nextUp32(x) {   // x: a finite f32 value
  if (x === 0) return 1.401298464324817e-45;
  _f32[0] = x;
  if (x > 0) _u32[0] += 1; else _u32[0] -= 1;
  return _f32[0];
}
function nextDown32(x) { return -nextUp32(-x); }
// RN32(a*b + c) for f32 a, b, c: the f64 product is exact; TwoSum gives the exact sum s + err; RN32(s) is
// the answer unless s is an f32 rounding midpoint, where err decides the direction.
function fma32(a, b, c) {
  const p = a * b;
  const s = p + c;
  if (!isFinite(s)) return f(s);
  const bb = s - p;
  const err = (p - (s - bb)) + (c - bb);
  const r = f(s);
  if (err === 0 || r === s) return r;
  const other = r < s ? nextUp32(r) : nextDown32(r);
  if ((r + other) / 2 !== s) return r;
  const lo = Math.min(r, other), hi = Math.max(r, other);
  return err > 0 ? hi : lo;
}

// ---- compat math spec v3 (oracle/ref_math.h) --------------------------------------------------------------
const kTwoOverPi = 0.6366197723675814, kP1 = 1.5707963267341256, kP2 = 6.077100506303966e-11,
  kP3 = 2.0222662487959506e-21;
function reducePio2(x) {  // -> [r (f64), q]
  if (!(Math.abs(x) < 1e15)) return [NaN, 0];
  const k = Math.floor(x * kTwoOverPi + 0.5);
  let r = x - k * kP1;
  r = r - k * kP2;
  r = r - k * kP3;
  return [r, ((k % 4) + 4) % 4];
}
const kS0 = f(-0.166666641831398), kS1 = f(0.008332744240760803), kS2 = f(-0.0001958730281330645);
const kC0 = f(0.0416666641831398), kC1 = f(-0.0013888344401493669), kC2 = f(2.455315006955061e-05);
const kA = [-0.3333333134651184, 0.19999729096889496, -0.142783522605896, 0.11032091081142426,
  -0.08650501817464828, 0.062368933111429214, -0.03571782633662224, 0.01341481227427721,
  -0.002364102052524686].map(f);
const kB = [0.16666673123836517, 0.07498858869075775, 0.045000601559877396, 0.026559552177786827,
  0.03807495906949043].map(f);
const kPiF = f(3.14159274), kPiO2F = f(1.57079637);
function sinpoly(r) { const z = f(r * r); return fma32(f(r * z), fma32(fma32(kS2, z, kS1), z, kS0), r); }
function cospoly(r) { const z = f(r * r); return fma32(f(z * z), fma32(fma32(kC2, z, kC1), z, kC0), fma32(f(-0.5), z, 1)); }
// spec v3 reduction (oracle/ref_math.h reduce_spec): |x| < 2^20 -> j = rint(RN(x * 2/pi)), ties to even, then three
// exactly rounded f32 FMAs; beyond, the f64 reduction rounded to f32. -> [rf (f32), q]
const kInvPiO2F = f(0.6366197466850281), kPiO2A = f(1.5707963705062866), kPiO2B = f(-4.371138828673793e-08),
  kPiO2C = f(-1.7151245100058819e-15);
function rintEven(v) {  // v: an f32 value; exact (v - floor(v) is exact below 2^52)
  const n = Math.floor(v), d = v - n;
  if (d > 0.5) return n + 1;
  if (d < 0.5) return n;
  return (n % 2 === 0) ? n : n + 1;
}
function reduceSpec(x) {
  if (Math.abs(x) < 1048576) {
    const j = rintEven(f(x * kInvPiO2F)), mj = -j;
    let r = fma32(mj, kPiO2A, x);
    r = fma32(mj, kPiO2B, r);
    r = fma32(mj, kPiO2C, r);
    return [r, ((j % 4) + 4) % 4];
  }
  const [r, q] = reducePio2(x);
  return [f(r), q];
}
function sincos(x) {
  const [rf, q] = reduceSpec(x);
  const s = sinpoly(rf), c = cospoly(rf);
  switch (q) {
    case 0: return [s, c];
    case 1: return [c, -s];
    case 2: return [-s, -c];
    default: return [-c, s];
  }
}
function sin_(x) { return sincos(x)[0]; }
function cos_(x) { return sincos(x)[1]; }
function tan_(x) {
  const [rf, q] = reduceSpec(x);
  const s = sinpoly(rf), c = cospoly(rf);
  return (q & 1) ? f(-c / s) : f(s / c);
}
function atan01(t) {
  const z = f(t * t);
  let p = kA[8];
  for (let i = 7; i >= 0; i--) p = fma32(p, z, kA[i]);
  return fma32(f(t * z), p, t);
}
function atan2_(y, x) {
  if (y !== y || x !== x) return f(y + x);
  if (y === 0 && x === 0) return 0;
  const ay = Math.abs(y), ax = Math.abs(x);
  let r = (ay <= ax) ? atan01(f(ay / ax)) : f(kPiO2F - atan01(f(ax / ay)));
  if (x < 0) r = f(kPiF - r);
  return (y < 0) ? -r : r;
}
function atan_(x) { return atan2_(x, 1); }
function asinpoly(x) {
  const z = f(x * x);
  let p = kB[4];
  for (let i = 3; i >= 0; i--) p = fma32(p, z, kB[i]);
  return fma32(f(x * z), p, x);
}
function acos_(x) {
  if (!(x >= -1 && x <= 1)) return NaN;
  const ax = Math.abs(x);
  if (ax <= 0.5) return f(kPiO2F - asinpoly(x));
  const a2 = f(2 * asinpoly(f(Math.sqrt(f(f(1 - ax) * 0.5)))));
  return (x > 0) ? a2 : f(kPiF - a2);
}
const signbit = (a) => a < 0 || Object.is(a, -0);
function fmin_(a, b) {  // v_min_f32: a NaN operand yields the other; -0 < +0
  if (a !== a) return b;
  if (b !== b) return a;
  if (a < b) return a;
  if (b < a) return b;
  return signbit(a) ? a : b;
}
function fmax_(a, b) {
  if (a !== a) return b;
  if (b !== b) return a;
  if (a > b) return a;
  if (b > a) return b;
  return signbit(a) ? b : a;
}
const clamp_ = (x, lo, hi) => fmin_(fmax_(x, lo), hi);
const sqrt_ = (x) => f(Math.sqrt(x));
const floor_ = (x) => Math.floor(x);
const fract_ = (x) => f(x - Math.floor(x));
function toint(x) {
  if (x !== x) return 0;
  if (x >= 2147483647) return 2147483647;
  if (x <= -2147483648) return -2147483648;
  return Math.trunc(x);
}

// ---- define.glsl constants ----------------------------------------------------------------------------------
const kMaxDistance = f(1e5), kEps = f(1e-5), kOneMinusEps = f(0.9999), kInf = f(1e5);
const kPI = f(3.141592653589793), kInvPI = f(0.3183098861837907);
const kPiOver2 = f(1.570796326794896), kPiOver4 = f(0.785398163397448);
const kObjLen = 17, kLightLen = 17, kTexLen = 15;
const CUBE = 1, SPHERE = 2, RECTANGLE = 3, CONE = 4, CYLINDER = 5, DISK = 6, HYPERBOLOID = 7, PARABOLOID = 8,
  CORNELLBOX = 9;
const AREA = 0, POINT = 1, SPOT = 2;
const MATTE = 1, MIRROR = 2, METAL = 3, GLASS = 4;
const UNIFORM_COLOR = 0, CHECKERBOARD = 5, CHECKERBOARD2 = 7, BILERP = 8, MIXF = 9, SCALE = 10, UVF = 11;
const F_NOOP = 0, F_CONDUCTOR = 1, F_DIELECTRIC = 2;
const E4 = f(0.0001), E3 = f(1e-3);

// ---- vec3 as [x, y, z] ----------------------------------------------------------------------------------
const v3 = (x, y, z) => [x, y, z];
const v3s = (s) => [s, s, s];
const BLACK = [0, 0, 0], WHITE = [1, 1, 1];
const vadd = (a, b) => [f(a[0] + b[0]), f(a[1] + b[1]), f(a[2] + b[2])];
const vsub = (a, b) => [f(a[0] - b[0]), f(a[1] - b[1]), f(a[2] - b[2])];
const vmul = (a, b) => [f(a[0] * b[0]), f(a[1] * b[1]), f(a[2] * b[2])];
const vdiv = (a, b) => [fdiv(a[0], b[0]), fdiv(a[1], b[1]), fdiv(a[2], b[2])];
const vmuls = (a, s) => [f(a[0] * s), f(a[1] * s), f(a[2] * s)];     // a * s
const smulv = (s, a) => [f(s * a[0]), f(s * a[1]), f(s * a[2])];     // s * a
const vdivs = (a, s) => [fdiv(a[0], s), fdiv(a[1], s), fdiv(a[2], s)];
const vadds = (a, s) => [f(a[0] + s), f(a[1] + s), f(a[2] + s)];
const vneg = (a) => [-a[0], -a[1], -a[2]];
const dot = (a, b) => f(f(f(a[0] * b[0]) + f(a[1] * b[1])) + f(a[2] * b[2]));
const cross = (a, b) => [f(f(a[1] * b[2]) - f(a[2] * b[1])), f(f(a[2] * b[0]) - f(a[0] * b[2])),
  f(f(a[0] * b[1]) - f(a[1] * b[0]))];
const length = (v) => sqrt_(dot(v, v));
const normalize = (v) => vdivs(v, length(v));
const vmin = (a, b) => [fmin_(a[0], b[0]), fmin_(a[1], b[1]), fmin_(a[2], b[2])];
const vmax = (a, b) => [fmax_(a[0], b[0]), fmax_(a[1], b[1]), fmax_(a[2], b[2])];
const vclamp01 = (x) => vmin(vmax(x, BLACK), WHITE);
const veq = (a, b) => a[0] === b[0] && a[1] === b[1] && a[2] === b[2];
const reflect_ = (I, N) => vsub(I, smulv(f(2 * dot(N, I)), N));
function refract_(I, N, eta) {
  const dni = dot(N, I);
  const k = f(1 - f(f(eta * eta) * f(1 - f(dni * dni))));
  if (k < 0) return BLACK;
  return vsub(smulv(eta, I), smulv(f(f(eta * dni) + sqrt_(k)), N));
}
const worldToLocal = (v, ns, ss, ts) => [dot(v, ss), dot(v, ts), dot(v, ns)];
const localToWorld = (v, ns, ss, ts) => [
  f(f(f(ss[0] * v[0]) + f(ts[0] * v[1])) + f(ns[0] * v[2])),
  f(f(f(ss[1] * v[0]) + f(ts[1] * v[1])) + f(ns[1] * v[2])),
  f(f(f(ss[2] * v[0]) + f(ts[2] * v[1])) + f(ns[2] * v[2]))];
const OSN = [0, 1, 0], OSS = [0, 0, -1], OST = [1, 0, 0];
const W2L = (v) => worldToLocal(v, OSN, OSS, OST);
const L2W = (v) => localToWorld(v, OSN, OSS, OST);
const equalZero = (x) => x < E3 && x > -E3;
function quadratic(A, B, Cc) {  // utility.glsl:37-51 -> null | [t0, t1]
  const discrim = f(f(B * B) - f(f(4 * A) * Cc));
  if (discrim < 0) return null;
  const root = sqrt_(discrim);
  const q = (B < 0) ? f(f(-0.5) * f(B - root)) : f(f(-0.5) * f(B + root));
  let t0 = fdiv(q, A), t1 = fdiv(Cc, q);
  if (t0 > t1) { const tmp = t0; t0 = t1; t1 = tmp; }
  return [t0, t1];
}

// ---- scene textures: R32F, NEAREST, CLAMP_TO_EDGE (texhelper.glsl) ---------------------------------------
class Ctx {
  constructor(job) {
    this.objects = { d: job.objects, w: 18, h: job.n };
    this.texParams = { d: job.texparams, w: 16, h: job.tn };
    this.lights = { d: job.lights, w: 18, h: job.ln };
    this.n = job.n; this.tn = job.tn; this.ln = job.ln;
    [this.shapeMask, this.matMask, this.texMask, this.lightMask] = job.masks;
    this.fcx = 0; this.fcy = 0; this.fcz = 0.5;
    this.timeSinceStart = 0;
    this.segments = 0;
  }
}
let C = null;
function texel(c, size) {
  if (c !== c) return 0;
  const s = Math.floor(f(c * size));
  if (!(s >= 0)) return 0;
  if (s >= size - 1) return size - 1;
  return s;
}
function fetch(t, cx, cy) {
  if (t.h <= 0) return 0;
  return t.d[texel(cy, t.h) * t.w + texel(cx, t.w)];
}
const readFloat = (t, x, y, width) => fetch(t, fdiv(x, width), y);
const readInt = (t, x, y, width) => toint(readFloat(t, x, y, width));
const readBool = (t, x, y, width) => readInt(t, x, y, width) === 1;
function readVec3(t, x, y, width) {
  let px = fdiv(x, width);
  const step = fdiv(1, width);
  const a = fetch(t, px, y); px = f(px + step);
  const b = fetch(t, px, y); px = f(px + step);
  return [a, b, fetch(t, px, y)];
}
const rowCoord = (i, n) => fdiv(i, (n - 1));
const matCoord = (v) => fdiv(v, (C.tn - 1));

function zeroIns() {
  return { d: 0, hit: BLACK, normal: BLACK, dpdu: BLACK, dpdv: BLACK, into: false, matIndex: 0, sc: BLACK,
    emission: BLACK, seed: 0, index: 0, matCategory: 0 };
}

// ---- random.glsl:5-18 -----------------------------------------------------------------------------------
function hash1(seed, a, b, c) {
  const p = [f(C.fcx + seed), f(C.fcy + seed), f(C.fcz + seed)];
  return fract_(f(f(sin_(dot(p, [a, b, c])) * f(43758.5453)) + seed));
}
const H = [f(12.9898), f(78.233), f(151.7182), f(63.7264), f(10.873), f(623.6736)];
const random2 = (seed) => [hash1(seed, H[0], H[1], H[2]), hash1(seed, H[3], H[4], H[5])];
const randomInt = (seed, mn, mx) => mn + toint(f(hash1(seed, H[0], H[1], H[2]) * f(mx - mn)));

// ---- sampler.glsl --------------------------------------------------------------------------------------
const TWO_PI = f(2 * kPI);
function uniformSampleSphere(u) {
  const z = f(1 - f(2 * u[0]));
  const r = sqrt_(f(1 - f(z * z)));
  const angle = f(TWO_PI * u[1]);
  return [f(r * cos_(angle)), f(r * sin_(angle)), z];
}
function cosineSampleHemisphere(u) {
  const r = sqrt_(u[0]);
  const angle = f(TWO_PI * u[1]);
  return [f(r * cos_(angle)), f(r * sin_(angle)), sqrt_(f(1 - u[0]))];
}
function concentricSampleDisk(u) {
  const uO = f(f(2 * u[0]) - 1), vO = f(f(2 * u[1]) - 1);
  if (uO === 0 && vO === 0) return [0, 0];
  let theta, r;
  if (Math.abs(uO) > Math.abs(vO)) { r = uO; theta = f(fdiv(vO, uO) * kPiOver4); }
  else { r = vO; theta = f(kPiOver2 - f(fdiv(uO, vO) * kPiOver4)); }
  return [f(r * cos_(theta)), f(r * sin_(theta))];
}

// ---- textures (shader.texture.js:22-29) -------------------------------------------------------------------
function getSurfaceColor(uv, texIndex) {
  const tp = C.texParams;
  const cat = readInt(tp, 0, texIndex, kTexLen);
  if (cat === UNIFORM_COLOR) return readVec3(tp, 1, texIndex, kTexLen);
  if (!((C.texMask >>> cat) & 1)) return BLACK;
  switch (cat) {
    case CHECKERBOARD: {
      const size = readFloat(tp, 1, texIndex, kTexLen), lineWidth = readFloat(tp, 2, texIndex, kTexLen);
      const width = fdiv(f(0.5 * lineWidth), size);
      const fx = f(fdiv(uv[0], size) - floor_(fdiv(uv[0], size))), fy = f(fdiv(uv[1], size) - floor_(fdiv(uv[1], size)));
      const out = (fx < width || fx > f(1 - width)) || (fy < width || fy > f(1 - width));
      return out ? v3s(0.5) : WHITE;
    }
    case CHECKERBOARD2: {
      const c1 = readVec3(tp, 1, texIndex, kTexLen), c2 = readVec3(tp, 4, texIndex, kTexLen);
      const size = readFloat(tp, 7, texIndex, kTexLen);
      const qx = floor_(fdiv(uv[0], size)), qy = floor_(fdiv(uv[1], size));
      return (toint(f(qx + qy)) % 2 === 0) ? c1 : c2;
    }
    case BILERP: {
      const c00 = readVec3(tp, 1, texIndex, kTexLen), c01 = readVec3(tp, 4, texIndex, kTexLen);
      const c10 = readVec3(tp, 7, texIndex, kTexLen), c11 = readVec3(tp, 10, texIndex, kTexLen);
      const ou = f(1 - uv[0]), ov = f(1 - uv[1]);
      return vadd(vadd(vadd(smulv(f(ou * ov), c00), smulv(f(ou * uv[1]), c01)), smulv(f(uv[0] * ov), c10)),
        smulv(f(uv[0] * uv[1]), c11));
    }
    case MIXF: {
      const c1 = readVec3(tp, 1, texIndex, kTexLen), c2 = readVec3(tp, 4, texIndex, kTexLen);
      const amount = readFloat(tp, 7, texIndex, kTexLen);
      return vadd(smulv(f(1 - amount), c1), smulv(amount, c2));
    }
    case SCALE: return vmul(readVec3(tp, 1, texIndex, kTexLen), readVec3(tp, 4, texIndex, kTexLen));
    case UVF: return [f(uv[0] - floor_(uv[0])), f(uv[1] - floor_(uv[1])), 0];
    default: return BLACK;
  }
}

// ---- boundbox.glsl (constructor order (max, min)) ---------------------------------------------------------
function slabT(mn, mx, ray) {
  const tMin = vdiv(vsub(mn, ray.o), ray.d), tMax = vdiv(vsub(mx, ray.o), ray.d);
  const t1 = vmin(tMin, tMax), t2 = vmax(tMin, tMax);
  return [fmax_(fmax_(t1[0], t1[1]), t1[2]), fmin_(fmin_(t2[0], t2[1]), t2[2])];
}
function testBoundbox(ray, bmax, bmin) {
  const [tNear, tFar] = slabT(bmin, bmax, ray);
  if (tNear < 0 && tFar < 0) return false;
  return tNear < tFar;
}
const sgn = (rev) => (rev ? -1 : 1);

// ---- cube.glsl / cornellbox.glsl ---------------------------------------------------------------------------
function parseCube(index) {
  const o = C.objects;
  return { min: readVec3(o, 1, index, kObjLen), max: readVec3(o, 4, index, kObjLen),
    rev: readBool(o, 7, index, kObjLen), matIndex: matCoord(readFloat(o, 8, index, kObjLen)),
    texIndex: matCoord(readFloat(o, 9, index, kObjLen)), emission: readVec3(o, 10, index, kObjLen) };
}
function normalForCube(hit, c) {
  const s = sgn(c.rev);
  if (hit[0] < f(c.min[0] + E4)) return smulv(s, [-1, 0, 0]);
  if (hit[0] > f(c.max[0] - E4)) return smulv(s, [1, 0, 0]);
  if (hit[1] < f(c.min[1] + E4)) return smulv(s, [0, -1, 0]);
  if (hit[1] > f(c.max[1] - E4)) return smulv(s, [0, 1, 0]);
  if (hit[2] < f(c.min[2] + E4)) return smulv(s, [0, 0, -1]);
  return smulv(s, [0, 0, 1]);
}
function dpdBox(normal) {
  const dpdu = Math.abs(normal[0]) < 0.5 ? cross(normal, [1, 0, 0]) : cross(normal, [0, 1, 0]);
  return [dpdu, cross(normal, dpdu)];
}
function getCubeUV(hit, c) {  // cube.glsl:54-63 (face tests compare hit-min against min: kept)
  const tr = vsub(c.max, c.min);
  hit = vsub(hit, c.min);
  if (hit[0] < f(c.min[0] + E4) || hit[0] > f(c.max[0] - E4)) return [fdiv(hit[1], tr[1]), fdiv(hit[2], tr[2])];
  if (hit[1] < f(c.min[1] + E4) || hit[1] > f(c.max[1] - E4)) return [fdiv(hit[0], tr[0]), fdiv(hit[2], tr[2])];
  return [fdiv(hit[0], tr[0]), fdiv(hit[1], tr[1])];
}
function intersectCube(ray, c) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const [tNear, tFar] = slabT(c.min, c.max, ray);
  let t = -1;
  if (tNear > kEps && tNear < tFar) t = tNear;
  else if (tNear < tFar) t = tFar;
  if (t > kEps) {
    r.d = t;
    r.hit = vadd(ray.o, smulv(t, ray.d));
    r.normal = normalForCube(vadd(ray.o, smulv(t, ray.d)), c);
    [r.dpdu, r.dpdv] = dpdBox(r.normal);
    r.matIndex = c.matIndex;
    r.sc = getSurfaceColor(getCubeUV(r.hit, c), c.texIndex);
    r.emission = c.emission;
  }
  return r;
}
function parseCornellbox(index) {
  const o = C.objects;
  return { min: readVec3(o, 1, index, kObjLen), max: readVec3(o, 4, index, kObjLen),
    matIndex: matCoord(readFloat(o, 7, index, kObjLen)), rev: false, emission: BLACK };
}
function cornellColor(hit, mn, mx) {
  if (hit[0] < f(mn[0] + E4)) return [0.25, 0.75, 0.25];
  if (hit[0] > f(mx[0] - E4)) return [0.25, 0.25, 0.75];
  if (hit[1] < f(mn[1] + E4)) return WHITE;
  if (hit[1] > f(mx[1] - E4)) return WHITE;
  if (hit[2] > f(mn[2] + E4)) return WHITE;
  return BLACK;
}
function normalForCornellbox(hit, b) {
  if (hit[0] < f(b.min[0] + E4)) return [-1, 0, 0];
  if (hit[0] > f(b.max[0] - E4)) return [1, 0, 0];
  if (hit[1] < f(b.min[1] + E4)) return [0, -1, 0];
  if (hit[1] > f(b.max[1] - E4)) return [0, 1, 0];
  if (hit[2] < f(b.min[2] + E4)) return [0, 0, -1];
  return [0, 0, 1];
}
function intersectCornellbox(ray, b) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const [tNear, tFar] = slabT(b.min, b.max, ray);
  let t = -1;
  if (tNear < tFar) t = tFar;
  if (t > kEps) {
    r.d = t;
    r.hit = vadd(ray.o, smulv(t, ray.d));
    r.normal = vneg(normalForCornellbox(vadd(ray.o, smulv(t, ray.d)), b));
    [r.dpdu, r.dpdv] = dpdBox(r.normal);
    r.matIndex = b.matIndex;
    r.sc = cornellColor(r.hit, b.min, b.max);
    r.emission = BLACK;
  }
  return r;
}

// ---- sphere.glsl ------------------------------------------------------------------------------------------
function parseSphere(index) {
  const o = C.objects;
  return { c: readVec3(o, 1, index, kObjLen), r: readFloat(o, 4, index, kObjLen), rev: readBool(o, 5, index, kObjLen),
    matIndex: matCoord(readFloat(o, 6, index, kObjLen)), texIndex: matCoord(readFloat(o, 7, index, kObjLen)),
    emission: readVec3(o, 8, index, kObjLen) };
}
// Boundbox(max, min) argument order as the GLSL writes it (sphere.glsl:10-16 etc.): the first corner is `max`
const testBoundboxForSphere = (ray, s) => testBoundbox(ray, vsub(s.c, v3s(s.r)), vadd(s.c, v3s(s.r)));
const normalForSphere = (hit, s) => vdivs(smulv(sgn(s.rev), vsub(hit, s.c)), s.r);
const dpduRot = (h) => [f(f(f(-2) * kPI) * h[1]), f(f(2 * kPI) * h[0]), 0];
function phiOf(y, x) {
  let phi = atan2_(y, x);
  if (phi < 0) phi = f(phi + TWO_PI);
  return phi;
}
function intersectSphere(ray0, s) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const d = W2L(ray0.d), o = W2L(vsub(ray0.o, s.c));
  const a = dot(d, d), b = f(2 * dot(o, d)), c = f(dot(o, o) - f(s.r * s.r));
  const q = quadratic(a, b, c);
  if (!q) return r;
  const [t1, t2] = q;
  if (t2 < kEps) return r;
  let t = t1;
  if (t1 < kEps) t = t2;
  if (t >= kMaxDistance) return r;
  const hit = vadd(o, smulv(t, d));
  if (hit[0] === 0 && hit[1] === 0) hit[0] = f(f(1e-5) * s.r);
  const u = fdiv(phiOf(hit[1], hit[0]), TWO_PI);
  const theta = acos_(clamp_(fdiv(hit[2], s.r), -1, 1));
  const v = fdiv(theta, kPI);
  r.d = t;
  r.hit = vadd(o, smulv(t, d));
  {  // computeDpDForSphere :33-43
    const h = r.hit;
    const th = acos_(clamp_(fdiv(h[2], s.r), -1, 1));
    const zRadius = sqrt_(f(f(h[0] * h[0]) + f(h[1] * h[1])));
    const inv = fdiv(1, zRadius);
    const cosPhi = f(h[0] * inv), sinPhi = f(h[1] * inv);
    r.dpdu = dpduRot(h);
    r.dpdv = smulv(kPI, [f(h[2] * cosPhi), f(h[2] * sinPhi), f(-s.r * sin_(th))]);
  }
  r.normal = normalize(cross(r.dpdv, r.dpdu));
  r.matIndex = s.matIndex;
  r.sc = getSurfaceColor([u, v], s.texIndex);
  r.emission = s.emission;
  r.hit = vadd(L2W(r.hit), s.c);
  r.normal = L2W(r.normal);
  r.dpdu = L2W(r.dpdu);
  r.dpdv = L2W(r.dpdv);
  return r;
}
function sampleSphere(u, s) {
  const p = uniformSampleSphere(u);
  return [vadd(vmuls(p, s.r), s.c), fdiv(kInvPI, f(s.r * s.r))];
}

// ---- rectangle.glsl ---------------------------------------------------------------------------------------
function parseRectangle(index) {
  const o = C.objects;
  return { min: readVec3(o, 1, index, kObjLen), max: readVec3(o, 4, index, kObjLen), rev: readBool(o, 7, index, kObjLen),
    matIndex: matCoord(readFloat(o, 8, index, kObjLen)), texIndex: matCoord(readFloat(o, 9, index, kObjLen)),
    emission: readVec3(o, 10, index, kObjLen) };
}
const rectX = (q) => [f(q.max[0] - q.min[0]), 0, 0];
const rectY = (q) => [0, f(q.max[1] - q.min[1]), f(q.max[2] - q.min[2])];
const normalForRectangle = (hit, q) => smulv(sgn(q.rev), normalize(cross(rectX(q), rectY(q))));
function intersectRectangle(ray, q) {
  const r = zeroIns();
  r.d = kMaxDistance;
  r.dpdu = rectX(q);
  r.dpdv = rectY(q);
  r.normal = normalize(cross(r.dpdu, r.dpdv));
  const maxX = length(r.dpdu), maxY = length(r.dpdv);
  const ss = vdivs(r.dpdu, maxX), ts = cross(r.normal, ss);
  const d = worldToLocal(ray.d, r.normal, ss, ts), o = worldToLocal(vsub(ray.o, q.min), r.normal, ss, ts);
  if (d[2] === 0) return r;
  const t = fdiv(-o[2], d[2]);
  if (t < kEps) return r;
  const hit = vadd(o, smulv(t, d));
  if (hit[0] > maxX || hit[1] > maxY || hit[0] < -kEps || hit[1] < -kEps) return r;
  r.d = t;
  r.matIndex = q.matIndex;
  r.sc = getSurfaceColor([fdiv(hit[0], maxX), fdiv(hit[1], maxY)], q.texIndex);
  r.emission = q.emission;
  r.hit = vadd(localToWorld(hit, r.normal, ss, ts), q.min);
  return r;
}
function sampleRectangle(u, q) {
  const x = rectX(q), y = rectY(q);
  return [vadd(vadd(q.min, vmuls(x, u[0])), vmuls(y, u[1])), fdiv(1, f(length(x) * length(y)))];
}

// ---- cone.glsl / cylinder.glsl / disk.glsl / hyperboloid.glsl / paraboloid.glsl ----------------------------
function parseConeCyl(index) {
  const o = C.objects;
  return { p: readVec3(o, 1, index, kObjLen), h: readFloat(o, 4, index, kObjLen), r: readFloat(o, 5, index, kObjLen),
    rev: readBool(o, 6, index, kObjLen), matIndex: matCoord(readFloat(o, 7, index, kObjLen)),
    texIndex: matCoord(readFloat(o, 8, index, kObjLen)), emission: readVec3(o, 9, index, kObjLen) };
}
const testBoundboxForConeCyl = (ray, c) => testBoundbox(ray, vsub(c.p, [c.r, 0, c.r]), vadd(c.p, [c.r, c.h, c.r]));
function normalForCone(hit, c) {
  hit = vsub(hit, c.p);
  const tana = fdiv(c.r, c.h);
  const d = sqrt_(f(f(hit[0] * hit[0]) + f(hit[1] * hit[1])));
  const x1 = fdiv(d, tana), x2 = f(d * tana);
  return smulv(sgn(c.rev), normalize(vsub(hit, [0, 0, f(f(c.h - x1) - x2)])));
}
const normalForCylinder = (hit, c) => smulv(sgn(c.rev), normalize([f(hit[0] - c.p[0]), f(hit[1] - c.p[1]), 0]));
function finishLocal(r, hit, uv, matIndex, texIndex, emission, p) {
  r.normal = normalize(cross(r.dpdu, r.dpdv));
  r.hit = hit;
  r.matIndex = matIndex;
  r.sc = getSurfaceColor(uv, texIndex);
  r.emission = emission;
  r.hit = vadd(L2W(r.hit), p);
  r.normal = L2W(r.normal);
  r.dpdu = L2W(r.dpdu);
  r.dpdv = L2W(r.dpdv);
  return r;
}
// two-root retry against the z range (cone/cylinder: [-EPS, h]; hyperboloid/paraboloid: [zMin, zMax])
function rootPick(t1, t2, o, d, zlo, zhi) {
  let t = t1;
  if (t1 < kEps) t = t2;
  let hit = vadd(o, smulv(t, d));
  if (hit[2] < zlo || hit[2] > zhi) {
    if (t === t2) return null;
    t = t2;
    hit = vadd(o, smulv(t, d));
    if (hit[2] < zlo || hit[2] > zhi) return null;
  }
  if (t >= kMaxDistance) return null;
  return [t, hit];
}
function intersectCone(ray0, c) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const d = W2L(ray0.d), o = W2L(vsub(ray0.o, c.p));
  let k = fdiv(c.r, c.h);
  k = f(k * k);
  const ozh = f(o[2] - c.h);
  const a = f(f(f(d[0] * d[0]) + f(d[1] * d[1])) - f(f(k * d[2]) * d[2]));
  const b = f(2 * f(f(f(d[0] * o[0]) + f(d[1] * o[1])) - f(f(k * d[2]) * ozh)));
  const cc = f(f(f(o[0] * o[0]) + f(o[1] * o[1])) - f(f(k * ozh) * ozh));
  const q = quadratic(a, b, cc);
  if (!q || q[1] < -kEps) return r;
  const pk = rootPick(q[0], q[1], o, d, -kEps, c.h);
  if (!pk) return r;
  const [t, hit] = pk;
  const u = fdiv(phiOf(hit[1], hit[0]), TWO_PI), v = fdiv(hit[2], c.h);
  r.d = t;
  const vv = fdiv(hit[2], c.h);
  r.dpdu = dpduRot(hit);
  r.dpdv = [fdiv(-hit[0], f(1 - vv)), fdiv(-hit[1], f(1 - vv)), c.h];
  return finishLocal(r, hit, [u, v], c.matIndex, c.texIndex, c.emission, c.p);
}
function intersectCylinder(ray0, c) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const d = W2L(ray0.d), o = W2L(vsub(ray0.o, c.p));
  const a = f(f(d[0] * d[0]) + f(d[1] * d[1]));
  const b = f(2 * f(f(d[0] * o[0]) + f(d[1] * o[1])));
  const cc = f(f(f(o[0] * o[0]) + f(o[1] * o[1])) - f(c.r * c.r));
  const q = quadratic(a, b, cc);
  if (!q || q[1] < -kEps) return r;
  const pk = rootPick(q[0], q[1], o, d, -kEps, c.h);
  if (!pk) return r;
  const [t, hit] = pk;
  const u = fdiv(phiOf(hit[1], hit[0]), TWO_PI), v = fdiv(hit[2], c.h);
  r.d = t;
  r.dpdu = dpduRot(hit);
  r.dpdv = [0, 0, c.h];
  return finishLocal(r, hit, [u, v], c.matIndex, c.texIndex, c.emission, c.p);
}
function parseDisk(index) {
  const o = C.objects;
  return { p: readVec3(o, 1, index, kObjLen), r: readFloat(o, 4, index, kObjLen), innerR: readFloat(o, 5, index, kObjLen),
    rev: readBool(o, 6, index, kObjLen), matIndex: matCoord(readFloat(o, 7, index, kObjLen)),
    texIndex: matCoord(readFloat(o, 8, index, kObjLen)), emission: readVec3(o, 9, index, kObjLen) };
}
function intersectDisk(ray0, k) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const d = W2L(ray0.d), o = W2L(vsub(ray0.o, k.p));
  if (d[2] === 0) return r;
  const t = fdiv(-o[2], d[2]);
  if (t <= 0) return r;
  const hit = vadd(o, smulv(t, d));
  const dist2 = f(f(hit[0] * hit[0]) + f(hit[1] * hit[1]));
  if (dist2 > f(k.r * k.r) || dist2 < f(k.innerR * k.innerR)) return r;
  if (t >= kMaxDistance) return r;
  const u = fdiv(phiOf(hit[1], hit[0]), TWO_PI);
  const oneMinusV = fdiv(f(sqrt_(dist2) - k.innerR), f(k.r - k.innerR));
  const v = f(1 - oneMinusV);
  r.d = t;
  r.dpdu = dpduRot(hit);
  r.dpdv = vdivs(vmuls([hit[0], hit[1], 0], f(k.innerR - k.r)), sqrt_(dist2));
  return finishLocal(r, hit, [u, v], k.matIndex, k.texIndex, k.emission, k.p);
}
function sampleDisk(u, k) {
  const pd = concentricSampleDisk(u);
  const p = [f(f(pd[0] * k.r) + k.p[0]), k.p[1], f(f(pd[1] * k.r) + k.p[2])];
  const area = f(f(f(2 * kPI) * 0.5) * f(f(k.r * k.r) - f(k.innerR * k.innerR)));
  return [p, fdiv(1, area)];
}
function parseHyperboloid(index) {
  const o = C.objects;
  return { p: readVec3(o, 1, index, kObjLen), p1: readVec3(o, 4, index, kObjLen), p2: readVec3(o, 7, index, kObjLen),
    ah: readFloat(o, 10, index, kObjLen), ch: readFloat(o, 11, index, kObjLen), rev: readBool(o, 12, index, kObjLen),
    matIndex: matCoord(readFloat(o, 13, index, kObjLen)), texIndex: matCoord(readFloat(o, 14, index, kObjLen)),
    emission: readVec3(o, 15, index, kObjLen) };
}
function testBoundboxForHyperboloid(ray, h) {
  const r1 = sqrt_(f(f(h.p1[0] * h.p1[0]) + f(h.p1[1] * h.p1[1])));
  const r2 = sqrt_(f(f(h.p2[0] * h.p2[0]) + f(h.p2[1] * h.p2[1])));
  const rMax = fmax_(r1, r2), zMin = fmin_(h.p1[2], h.p2[2]), zMax = fmax_(h.p1[2], h.p2[2]);
  return testBoundbox(ray, vsub(h.p, [rMax, -zMin, rMax]), vadd(h.p, [rMax, zMax, rMax]));
}
function hypDpD(hit, p1, p2, phi) {
  const [sinPhi, cosPhi] = sincos(phi);
  const dx = f(p2[0] - p1[0]), dy = f(p2[1] - p1[1]);
  return [dpduRot(hit), [f(f(dx * cosPhi) - f(dy * sinPhi)), f(f(dx * sinPhi) + f(dy * cosPhi)), f(p2[2] - p1[2])]];
}
function hypPhi(hit, h) {
  const v = fdiv(f(hit[2] - h.p1[2]), f(h.p2[2] - h.p1[2]));
  const pr = vadd(smulv(f(1 - v), h.p1), smulv(v, h.p2));
  return [v, phiOf(f(f(pr[0] * hit[1]) - f(hit[0] * pr[1])), f(f(hit[0] * pr[0]) + f(hit[1] * pr[1])))];
}
function normalForHyperboloid(hit, h) {
  const [, phi] = hypPhi(hit, h);
  const [dpdu, dpdv] = hypDpD(hit, h.p1, h.p2, phi);
  return smulv(sgn(h.rev), L2W(normalize(cross(dpdu, dpdv))));
}
function intersectHyperboloid(ray0, h) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const d = W2L(ray0.d), o = W2L(vsub(ray0.o, h.p));
  const a = f(f(f(f(h.ah * d[0]) * d[0]) + f(f(h.ah * d[1]) * d[1])) - f(f(h.ch * d[2]) * d[2]));
  const b = f(2 * f(f(f(f(h.ah * d[0]) * o[0]) + f(f(h.ah * d[1]) * o[1])) - f(f(h.ch * d[2]) * o[2])));
  const c = f(f(f(f(f(h.ah * o[0]) * o[0]) + f(f(h.ah * o[1]) * o[1])) - f(f(h.ch * o[2]) * o[2])) - 1);
  const q = quadratic(a, b, c);
  if (!q || q[1] < -kEps) return r;
  const zMin = fmin_(h.p1[2], h.p2[2]), zMax = fmax_(h.p1[2], h.p2[2]);
  const pk = rootPick(q[0], q[1], o, d, zMin, zMax);
  if (!pk) return r;
  const [t, hit] = pk;
  const [v, phi] = hypPhi(hit, h);
  const u = fdiv(phi, TWO_PI);
  r.d = t;
  [r.dpdu, r.dpdv] = hypDpD(hit, h.p1, h.p2, phi);
  return finishLocal(r, hit, [u, v], h.matIndex, h.texIndex, h.emission, h.p);
}
function parseParaboloid(index) {
  const o = C.objects;
  return { p: readVec3(o, 1, index, kObjLen), z0: readFloat(o, 4, index, kObjLen), z1: readFloat(o, 5, index, kObjLen),
    r: readFloat(o, 6, index, kObjLen), rev: readBool(o, 7, index, kObjLen),
    matIndex: matCoord(readFloat(o, 8, index, kObjLen)), texIndex: matCoord(readFloat(o, 9, index, kObjLen)),
    emission: readVec3(o, 10, index, kObjLen) };
}
function testBoundboxForParaboloid(ray, q) {
  const zMin = fmin_(q.z0, q.z1), zMax = fmax_(q.z0, q.z1);
  return testBoundbox(ray, vsub(q.p, [q.r, -zMin, q.r]), vadd(q.p, [q.r, zMax, q.r]));
}
function paraDpD(hit, zMax, zMin) {
  const h2 = f(2 * hit[2]);
  return [dpduRot(hit), smulv(f(zMax - zMin), [fdiv(hit[0], h2), fdiv(hit[1], h2), 1])];
}
function normalForParaboloid(hit, q) {
  const zMin = fmin_(q.z0, q.z1), zMax = fmax_(q.z0, q.z1);
  const [dpdu, dpdv] = paraDpD(hit, zMax, zMin);
  return smulv(sgn(q.rev), L2W(normalize(cross(dpdu, dpdv))));
}
function intersectParaboloid(ray0, q) {
  const r = zeroIns();
  r.d = kMaxDistance;
  const d = W2L(ray0.d), o = W2L(vsub(ray0.o, q.p));
  const zMin = fmin_(q.z0, q.z1), zMax = fmax_(q.z0, q.z1);
  const k = fdiv(zMax, f(q.r * q.r));
  const a = f(k * f(f(d[0] * d[0]) + f(d[1] * d[1])));
  const b = f(f(f(2 * k) * f(f(d[0] * o[0]) + f(d[1] * o[1]))) - d[2]);
  const c = f(f(k * f(f(o[0] * o[0]) + f(o[1] * o[1]))) - o[2]);
  const qq = quadratic(a, b, c);
  if (!qq || qq[1] < -kEps) return r;
  const pk = rootPick(qq[0], qq[1], o, d, zMin, zMax);
  if (!pk) return r;
  const [t, hit] = pk;
  const u = fdiv(phiOf(hit[1], hit[0]), TWO_PI), v = fdiv(f(hit[2] - zMin), f(zMax - zMin));
  r.d = t;
  [r.dpdu, r.dpdv] = paraDpD(hit, zMax, zMin);
  return finishLocal(r, hit, [u, v], q.matIndex, q.texIndex, q.emission, q.p);
}

// ---- intersectObjects (generated, shader.shape.js:28-51) -----------------------------------------------------
function intersectObjects(ray) {
  let ins = zeroIns();
  ins.d = kMaxDistance;
  for (let i = 0; i < C.n; i++) {
    let tmp = zeroIns();
    tmp.d = kMaxDistance;
    const row = rowCoord(i, C.n);
    const cat = toint(fetch(C.objects, 0, row));
    if (cat >= 0 && cat < 32 && ((C.shapeMask >>> cat) & 1)) {
      let rev = false, x;
      switch (cat) {
        case CUBE: x = parseCube(row); rev = x.rev; tmp = intersectCube(ray, x); break;
        case SPHERE: x = parseSphere(row); rev = x.rev; if (!testBoundboxForSphere(ray, x)) continue; tmp = intersectSphere(ray, x); break;
        case RECTANGLE: x = parseRectangle(row); rev = x.rev; tmp = intersectRectangle(ray, x); break;
        case CONE: x = parseConeCyl(row); rev = x.rev; if (!testBoundboxForConeCyl(ray, x)) continue; tmp = intersectCone(ray, x); break;
        case CYLINDER: x = parseConeCyl(row); rev = x.rev; if (!testBoundboxForConeCyl(ray, x)) continue; tmp = intersectCylinder(ray, x); break;
        case DISK: x = parseDisk(row); rev = x.rev; tmp = intersectDisk(ray, x); break;
        case HYPERBOLOID: x = parseHyperboloid(row); rev = x.rev; if (!testBoundboxForHyperboloid(ray, x)) continue; tmp = intersectHyperboloid(ray, x); break;
        case PARABOLOID: x = parseParaboloid(row); rev = x.rev; if (!testBoundboxForParaboloid(ray, x)) continue; tmp = intersectParaboloid(ray, x); break;
        case CORNELLBOX: x = parseCornellbox(row); rev = x.rev; tmp = intersectCornellbox(ray, x); break;
        default: break;
      }
      const nn = smulv(sgn(rev), tmp.normal);
      if (!(dot(nn, ray.d) < -kEps)) tmp.emission = BLACK;
      tmp.index = i;
    }
    if (tmp.d < ins.d) ins = tmp;
  }
  ins.matCategory = readInt(C.texParams, 0, ins.matIndex, kTexLen);
  ins.into = dot(ins.normal, ray.d) < -kEps;
  if (!ins.into) ins.normal = vneg(ins.normal);
  return ins;
}

// ---- sampleGeometry (generated, shader.shape.js:53-67) -> [point, normal, pdf] -----------------------------------
function sampleGeometry(u, i) {
  const row = rowCoord(i, C.n);
  const cat = toint(fetch(C.objects, 0, row));
  if (!(cat >= 0 && cat < 32 && ((C.shapeMask >>> cat) & 1))) return [BLACK, BLACK, 0];
  switch (cat) {
    case CUBE: return [BLACK, normalForCube(BLACK, parseCube(row)), 0];
    case SPHERE: { const x = parseSphere(row); const [p, pdf] = sampleSphere(u, x); return [p, normalForSphere(p, x), pdf]; }
    case RECTANGLE: { const x = parseRectangle(row); const [p, pdf] = sampleRectangle(u, x); return [p, normalForRectangle(p, x), pdf]; }
    case CONE: return [BLACK, normalForCone(BLACK, parseConeCyl(row)), 0];
    case CYLINDER: return [BLACK, normalForCylinder(BLACK, parseConeCyl(row)), 0];
    case DISK: { const x = parseDisk(row); const [p, pdf] = sampleDisk(u, x); return [p, smulv(sgn(x.rev), [0, 1, 0]), pdf]; }
    case HYPERBOLOID: return [BLACK, normalForHyperboloid(BLACK, parseHyperboloid(row)), 0];
    case PARABOLOID: return [BLACK, normalForParaboloid(BLACK, parseParaboloid(row)), 0];
    case CORNELLBOX: return [BLACK, normalForCornellbox(BLACK, parseCornellbox(row)), 0];
    default: return [BLACK, BLACK, 0];
  }
}

// ---- ssutility / fresnel / microfacet / bsdf ------------------------------------------------------------------
const absCosTheta = (w) => Math.abs(w[2]);
const cos2Theta = (w) => f(w[2] * w[2]);
const sin2Theta = (w) => fmax_(0, f(1 - cos2Theta(w)));
const sinTheta = (w) => sqrt_(sin2Theta(w));
function tan2Theta(w) { const c2 = cos2Theta(w); return c2 < kEps ? kInf : fdiv(sin2Theta(w), c2); }
function cosPhi(w) { const st = sinTheta(w); return equalZero(st) ? 1 : clamp_(fdiv(w[0], st), -1, 1); }
function sinPhi(w) { const st = sinTheta(w); return equalZero(st) ? 0 : clamp_(fdiv(w[1], st), -1, 1); }
const cos2Phi = (w) => f(cosPhi(w) * cosPhi(w));
const sin2Phi = (w) => f(sinPhi(w) * sinPhi(w));
const sameHemisphere = (w, wp) => f(w[2] * wp[2]) > kEps;
function frDielectric(cosThetaI, etaI, etaT) {
  cosThetaI = clamp_(cosThetaI, -1, 1);
  const sinThetaI = sqrt_(fmax_(0, f(1 - f(cosThetaI * cosThetaI))));
  const sinThetaT = f(fdiv(etaI, etaT) * sinThetaI);
  if (sinThetaT >= 1) return 1;
  const cosThetaT = sqrt_(fmax_(0, f(1 - f(sinThetaT * sinThetaT))));
  const TI = f(etaT * cosThetaI), IT = f(etaI * cosThetaT), II = f(etaI * cosThetaI), TT = f(etaT * cosThetaT);
  const Rparl = fdiv(f(TI - IT), f(TI + IT)), Rperp = fdiv(f(II - TT), f(II + TT));
  return fdiv(f(f(Rparl * Rparl) + f(Rperp * Rperp)), 2);
}
function frConductor(cosThetaI, etaI, etaT, k) {
  cosThetaI = clamp_(cosThetaI, -1, 1);
  const eta = vdiv(etaT, etaI), etak = vdiv(k, etaI);
  const c2 = f(cosThetaI * cosThetaI), s2 = f(1 - c2);
  const eta2 = vmul(eta, eta), etak2 = vmul(etak, etak);
  const t0 = [f(f(eta2[0] - etak2[0]) - s2), f(f(eta2[1] - etak2[1]) - s2), f(f(eta2[2] - etak2[2]) - s2)];
  const s = vadd(vmul(t0, t0), vmul(smulv(4, eta2), etak2));
  const a2pb2 = [sqrt_(s[0]), sqrt_(s[1]), sqrt_(s[2])];
  const t1 = vadds(a2pb2, c2);
  const ah = smulv(0.5, vadd(a2pb2, t0));
  const a = [sqrt_(ah[0]), sqrt_(ah[1]), sqrt_(ah[2])];
  const t2 = smulv(f(2 * cosThetaI), a);
  const Rs = vdiv(vsub(t1, t2), vadd(t1, t2));
  const t3 = vadd(smulv(c2, a2pb2), v3s(f(s2 * s2)));
  const t4 = vmuls(t2, s2);
  const Rp = vdiv(vmul(Rs, vsub(t3, t4)), vadd(t3, t4));
  return smulv(0.5, vadd(Rp, Rs));
}
function frEvaluate(fr, cosThetaI) {
  if (fr.type === F_DIELECTRIC) return vmuls(WHITE, frDielectric(cosThetaI, fr.etaI, fr.etaT));
  if (fr.type === F_CONDUCTOR) return frConductor(cosThetaI, fr.etaIv, fr.etaTv, fr.k);
  return WHITE;
}
function trSampleWh(u, ax, ay, wo) {
  let cosT = 0, phi = f(TWO_PI * u[0]);
  if (ax === ay) {
    const tanTheta2 = fdiv(f(f(ax * ax) * u[0]), f(1 - u[0]));
    cosT = fdiv(1, sqrt_(f(1 + tanTheta2)));
  } else {
    phi = atan_(f(fdiv(ay, ax) * tan_(f(kPiOver2 + f(TWO_PI * u[0])))));
    if (u[0] > 0.5) phi = f(phi + kPI);
    const [sP, cP] = sincos(phi);
    const ax2 = f(ax * ax), ay2 = f(ay * ay);
    const alpha2 = fdiv(1, f(fdiv(f(cP * cP), ax2) + fdiv(f(sP * sP), ay2)));
    const tanTheta2 = fdiv(f(alpha2 * u[0]), f(1 - u[0]));
    cosT = fdiv(1, sqrt_(f(1 + tanTheta2)));
  }
  const sinT = sqrt_(fmax_(0, f(1 - f(cosT * cosT))));
  const [sp, cp] = sincos(phi);
  let wh = [f(sinT * cp), f(sinT * sp), cosT];
  if (!sameHemisphere(wo, wh)) wh = vneg(wh);
  return wh;
}
function trD(ax, ay, wh) {
  const t2 = tan2Theta(wh);
  if (t2 >= kInf) return f(0.001);
  const cos4 = f(cos2Theta(wh) * cos2Theta(wh));
  const e = f(f(fdiv(cos2Phi(wh), f(ax * ax)) + fdiv(sin2Phi(wh), f(ay * ay))) * t2);
  const ope = f(1 + e);
  return fdiv(1, f(f(f(f(f(kPI * ax) * ay) * cos4) * ope) * ope));
}
const trPdf = (ax, ay, wh) => f(trD(ax, ay, wh) * absCosTheta(wh));
function orenNayarF(R, A, B, wo, wi) {
  const sinThetaI = sinTheta(wi), sinThetaO = sinTheta(wo);
  let maxCos = 0;
  if (sinThetaI > kEps && sinThetaO > kEps) {
    const sinPhiI = sinPhi(wi), cosPhiI = cosPhi(wi), sinPhiO = sinPhi(wo), cosPhiO = cosPhi(wo);
    maxCos = fmax_(0, f(f(cosPhiI * cosPhiO) + f(sinPhiI * sinPhiO)));
  }
  let sinAlpha, tanBeta;
  if (absCosTheta(wi) > absCosTheta(wo)) { sinAlpha = sinThetaO; tanBeta = fdiv(sinThetaI, absCosTheta(wi)); }
  else { sinAlpha = sinThetaI; tanBeta = fdiv(sinThetaO, absCosTheta(wo)); }
  return vmuls(vmuls(R, kInvPI), f(A + f(f(f(B * maxCos) * sinAlpha) * tanBeta)));
}
const TINY = vmuls(BLACK, f(0.001));
function microRF(mr, wo, wi) {
  const cosThetaO = absCosTheta(wo), cosThetaI = absCosTheta(wi);
  let wh = vadd(wi, wo);
  if (cosThetaI < kEps || cosThetaO < kEps) return TINY;
  if (equalZero(wh[0]) && equalZero(wh[1]) && equalZero(wh[2])) return TINY;
  wh = normalize(wh);
  const Fr = frEvaluate(mr.f, dot(wi, wh));
  return vdivs(vmul(vmuls(mr.R, trD(mr.ax, mr.ay, wh)), Fr), f(f(4 * cosThetaI) * cosThetaO));
}
function microRSample(mr, u, wo, out) {
  if (wo[2] < kEps) return TINY;
  const wh = trSampleWh(u, mr.ax, mr.ay, wo);
  out.wi = reflect_(vneg(wo), wh);
  if (!sameHemisphere(wo, out.wi)) return TINY;
  out.pdf = fdiv(trPdf(mr.ax, mr.ay, wh), f(4 * dot(wo, wh)));
  return microRF(mr, wo, out.wi);
}
function microTF(mt, wo, wi) {
  if (sameHemisphere(wo, wi)) return TINY;
  const cosThetaO = wo[2], cosThetaI = wi[2];
  if (equalZero(cosThetaI) || equalZero(cosThetaO)) return TINY;
  const eta = mt.into ? fdiv(mt.etaB, mt.etaA) : fdiv(mt.etaA, mt.etaB);
  let wh = normalize(vadd(wo, vmuls(wi, eta)));
  if (wh[2] < -kEps) wh = vneg(wh);
  const Fd = frDielectric(dot(wo, wh), mt.etaA, mt.etaB);
  const sqrtDenom = f(dot(wo, wh) + f(eta * dot(wi, wh)));
  const num = f(f(f(f(f(eta * eta) * trD(mt.ax, mt.ay, wh)) * Math.abs(dot(wi, wh))) * Math.abs(dot(wo, wh))));
  const den = f(f(f(cosThetaI * cosThetaO) * sqrtDenom) * sqrtDenom);
  return vmuls(smulv(f(1 - Fd), mt.T), Math.abs(fdiv(num, den)));
}
function microTPdf(mt, wo, wi) {
  if (sameHemisphere(wo, wi)) return f(0.001);
  const eta = mt.into ? fdiv(mt.etaB, mt.etaA) : fdiv(mt.etaA, mt.etaB);
  const wh = normalize(vadd(wo, vmuls(wi, eta)));
  const sqrtDenom = f(dot(wo, wh) + f(eta * dot(wi, wh)));
  const dwh = Math.abs(fdiv(f(f(eta * eta) * dot(wi, wh)), f(sqrtDenom * sqrtDenom)));
  return f(trPdf(mt.ax, mt.ay, wh) * dwh);
}
function microTSample(mt, u, wo, out) {
  if (equalZero(wo[2])) return TINY;
  const wh = trSampleWh(u, mt.ax, mt.ay, wo);
  const eta = mt.into ? fdiv(mt.etaA, mt.etaB) : fdiv(mt.etaB, mt.etaA);
  out.wi = refract_(vneg(wo), wh, eta);
  out.pdf = microTPdf(mt, wo, out.wi);
  return microTF(mt, wo, out.wi);
}

// ---- material plugins (shader.material.js:21-29 + material/*.glsl); out = {wi, pdf, f} -------------------------
function matte(u, mi, sc, wo, out) {
  const tp = C.texParams;
  const kd = readFloat(tp, 1, mi, kTexLen), sigma = readFloat(tp, 2, mi, kTexLen);
  const A = readFloat(tp, 3, mi, kTexLen), B = readFloat(tp, 4, mi, kTexLen);
  const R = smulv(kd, sc);
  out.wi = cosineSampleHemisphere(u);
  const pdf = sameHemisphere(wo, out.wi) ? f(absCosTheta(out.wi) * kInvPI) : 0;
  const fs = sigma < kEps ? vmuls(R, kInvPI) : orenNayarF(R, A, B, wo, out.wi);
  const fpdf = vdivs(vmuls(fs, absCosTheta(out.wi)), pdf);
  out.f = sigma < kEps ? vmuls(smulv(kd, sc), kInvPI) : orenNayarF(smulv(kd, sc), A, B, wo, out.wi);
  return fpdf;
}
function mirror(mi, sc, wo, out) {
  const kr = readFloat(C.texParams, 1, mi, kTexLen);
  const R = smulv(kr, sc);
  out.wi = [-wo[0], -wo[1], wo[2]];
  const fs = vdivs(vmul(WHITE, R), absCosTheta(out.wi));
  return vdivs(vmuls(fs, absCosTheta(out.wi)), 1);
}
function metal(u, mi, sc, wo, out) {
  const tp = C.texParams;
  const ur = readFloat(tp, 1, mi, kTexLen), vr = readFloat(tp, 2, mi, kTexLen);
  const eta = readVec3(tp, 3, mi, kTexLen), k = readVec3(tp, 6, mi, kTexLen);
  const mr = { R: sc, f: { type: F_CONDUCTOR, etaIv: WHITE, etaTv: eta, k }, ax: ur, ay: vr };
  out.pdf = 0;
  out.wi = BLACK;
  const fs = microRSample(mr, u, wo, out);
  return vdivs(vmuls(fs, absCosTheta(out.wi)), out.pdf);
}
function glass(u, mi, sc, wo, into, out) {
  const tp = C.texParams;
  const kr = readFloat(tp, 1, mi, kTexLen), kt = readFloat(tp, 2, mi, kTexLen), eta = readFloat(tp, 3, mi, kTexLen);
  const ur = readFloat(tp, 4, mi, kTexLen), vr = readFloat(tp, 5, mi, kTexLen);
  let fs;
  out.pdf = 0;
  out.wi = BLACK;
  if (ur < kEps && vr < kEps) {
    const R = smulv(kr, sc), T = smulv(kt, sc);
    const Fd = frDielectric(wo[2], 1, eta);
    if (u[0] < Fd) {
      out.wi = [-wo[0], -wo[1], wo[2]];
      out.pdf = 1;
      fs = vdivs(R, absCosTheta(out.wi));
    } else {
      const etaI = into ? 1 : eta, etaT = into ? eta : 1;
      out.wi = refract_(vneg(wo), [0, 0, 1], fdiv(etaI, etaT));
      out.pdf = 1;
      fs = vdivs(vmuls(T, f(1 - Fd)), absCosTheta(out.wi));
    }
  } else {
    const p = u[0];
    const uu = [fmin_(f(f(u[0] * 2) - 1), kOneMinusEps), u[1]];
    if (p < 0.5) fs = microRSample({ R: smulv(kr, sc), f: { type: F_DIELECTRIC, etaI: 1, etaT: eta }, ax: ur, ay: vr }, uu, wo, out);
    else fs = microTSample({ T: smulv(kt, sc), etaA: 1, etaB: eta, into, ax: ur, ay: vr }, uu, wo, out);
  }
  return vdivs(vmuls(fs, absCosTheta(out.wi)), out.pdf);
}
function material(ins, wo, out) {
  out.f = BLACK;
  out.wi = BLACK;
  const cat = ins.matCategory;
  if (!(cat >= 0 && cat < 32 && ((C.matMask >>> cat) & 1))) return BLACK;
  const u = random2(ins.seed);
  switch (cat) {
    case MATTE: return matte(u, ins.matIndex, ins.sc, wo, out);
    case MIRROR: { const r = mirror(ins.matIndex, ins.sc, wo, out); out.f = BLACK; return r; }
    case METAL: { const r = metal(u, ins.matIndex, ins.sc, wo, out); out.f = BLACK; return r; }
    case GLASS: { const r = glass(u, ins.matIndex, ins.sc, wo, ins.into, out); out.f = BLACK; return r; }
    default: return BLACK;
  }
}

// ---- lights (shader.light.js:12-31 + light/*.glsl) -----------------------------------------------------------
function testShadow(ray) {
  const ins = intersectObjects(ray);
  return ins.d > kEps && ins.d < kOneMinusEps;
}
function lightSample(ins) {
  const index = randomInt(ins.seed, 0, C.ln);
  const cat = readInt(C.lights, 0, index, kTexLen);   // integer row coordinate (reference bug kept)
  if (!(cat >= 0 && cat < 32 && ((C.lightMask >>> cat) & 1))) return BLACK;
  const row = rowCoord(index, C.ln);
  const L = C.lights;
  if (cat === AREA) {
    const aindex = readInt(L, 1, row, kLightLen);
    const em = readVec3(L, 2, row, kLightLen);
    const [p, normal, pdf] = sampleGeometry(random2(ins.seed), aindex);
    const toLight = vsub(p, ins.hit);
    const nt = normalize(toLight);
    if (testShadow({ o: ins.hit, d: toLight })) return BLACK;
    return vdivs(vmuls(vmuls(em, fmax_(0, dot(normal, vneg(nt)))), fmax_(0, dot(nt, ins.normal))), pdf);
  } else if (cat === POINT) {
    const from = readVec3(L, 1, row, kLightLen), em = readVec3(L, 4, row, kLightLen);
    const p = vadd(from, vmuls(uniformSampleSphere(random2(ins.seed)), f(0.1)));
    const toLight = vsub(p, ins.hit);
    if (testShadow({ o: ins.hit, d: toLight })) return BLACK;
    return vmuls(em, fmax_(0, dot(normalize(toLight), ins.normal)));
  } else if (cat === SPOT) {
    const ctw = readFloat(L, 1, row, kLightLen), cfs = readFloat(L, 2, row, kLightLen);
    const from = readVec3(L, 3, row, kLightLen), em = readVec3(L, 6, row, kLightLen);
    const toLight = vsub(from, ins.hit);
    if (testShadow({ o: ins.hit, d: toLight })) return BLACK;
    const nt = normalize(toLight);
    const d = length(toLight);
    const cT = -(-nt[1]);
    let fall;
    if (cT < ctw) fall = 0;
    else if (cT >= cfs) fall = 1;
    else { const delta = fdiv(f(cT - ctw), f(cfs - ctw)); const d2 = f(delta * delta); fall = f(d2 * d2); }
    return vdivs(vmuls(vmuls(em, fall), fmax_(0, dot(normalize(toLight), ins.normal))), f(d * d));
  }
  return BLACK;
}

// ---- path.glsl ----------------------------------------------------------------------------------------------
function shade(ins, wo, out) {
  let direct = BLACK;
  const ss = normalize(ins.dpdu), ts = cross(ins.normal, ss);
  const woL = worldToLocal(wo, ins.normal, ss, ts);
  const m = { wi: BLACK, f: BLACK, pdf: 0 };
  out.fpdf = vclamp01(material(ins, woL, m));
  out.wi = localToWorld(m.wi, ins.normal, ss, ts);
  if (veq(ins.emission, BLACK) && ins.matCategory === MATTE) direct = vadd(direct, vmul(lightSample(ins), m.f));
  return vadd(ins.emission, direct);
}
function trace(ray, maxDepth, aov) {
  let fpdf = WHITE, e = BLACK;
  let depth = 0;
  while (depth++ < maxDepth) {
    C.segments++;
    const ins = intersectObjects(ray);
    ins.seed = f(C.timeSinceStart + depth);
    if (ins.d >= kMaxDistance) break;
    if (depth === 1 && aov) { aov.n = ins.normal; aov.p = ins.hit; }
    const out = {};
    e = vadd(e, vmul(shade(ins, vneg(ray.d), out), fpdf));
    fpdf = vmul(fpdf, out.fpdf);
    const outdot = dot(ins.normal, out.wi);
    ray = { o: vadd(ins.hit, vmuls(ins.normal, outdot > kEps ? E4 : f(-0.0001))), d: out.wi };
  }
  return e;
}

// ---- primary rays (vstrace.glsl:4-6 + rasteriser interpolation) -------------------------------------------------
function cornerDirs(M, eye) {  // M: 16 f32, column-major
  const cx = [-1, -1, 1, 1], cy = [-1, 1, -1, 1];
  const out = [];
  for (let c = 0; c < 4; c++) {
    const q = [];
    for (let r = 0; r < 4; r++) q.push(f(f(f(f(M[r] * cx[c]) + f(M[4 + r] * cy[c])) + f(M[8 + r] * 0)) + f(M[12 + r] * 1)));
    const w = [fdiv(q[0], q[3]), fdiv(q[1], q[3]), fdiv(q[2], q[3])];
    out.push(normalize(vsub(w, eye)));
  }
  return out;
}
function primaryDir(d, x, y, W, H) {
  const s = f(f(x + 0.5) / W), t = f(f(y + 0.5) / H);
  if (f(s + t) <= 1) return vadd(vadd(d[0], vmuls(vsub(d[2], d[0]), s)), vmuls(vsub(d[1], d[0]), t));
  return vadd(vadd(d[3], vmuls(vsub(d[1], d[3]), f(1 - s))), vmuls(vsub(d[2], d[3]), f(1 - t)));
}
const q8 = (v) => f(f(Math.floor(f(f(fmin_(fmax_(v, 0), 1) * 255) + 0.5))) / 255);

// render(job): job = {objects, n, texparams, tn, lights, ln, masks: [shape, mat, tex, light], W, H,
//   crop: [x0, y0, cw, ch], inv: Float32Array(spp*16), seeds: Float32Array(spp), eye: [3], spp, k0,
//   maxBounces, accumMode (0 sum, 1 mix, 2 compat8), accum (optional Float32Array W*H*4), aov (bool)}
function render(job) {
  C = new Ctx({ objects: Float32Array.from(job.objects), n: job.n, texparams: Float32Array.from(job.texparams), tn: job.tn,
    lights: Float32Array.from(job.lights || []), ln: job.ln, masks: job.masks });
  const { W, H } = job;
  const [x0, y0, cw, ch] = job.crop || [0, 0, W, H];
  const accum = job.accum || new Float32Array(W * H * 4);
  const aovN = job.aov ? new Float32Array(W * H * 4) : null, aovP = job.aov ? new Float32Array(W * H * 4) : null;
  const eye = Array.from(job.eye, f);
  const k0 = job.k0 || 0, mode = job.accumMode || 0;
  for (let s = 0; s < job.spp; s++) {
    const d = cornerDirs(Array.from(job.inv.slice(16 * s, 16 * s + 16), f), eye);
    C.timeSinceStart = f(job.seeds[s]);
    const k = k0 + s;
    const w = f(k / (k + 1));
    for (let y = y0; y < y0 + ch; y++) {
      for (let x = x0; x < x0 + cw; x++) {
        C.fcx = f(x + 0.5); C.fcy = f(y + 0.5); C.fcz = 0.5;
        const aov = { n: BLACK, p: BLACK };
        const e = trace({ o: eye, d: primaryDir(d, x, y, W, H) }, job.maxBounces, aov);
        const i = 4 * (y * W + x);
        if (mode === 0) {
          accum[i] = f(accum[i] + e[0]); accum[i + 1] = f(accum[i + 1] + e[1]); accum[i + 2] = f(accum[i + 2] + e[2]);
          accum[i + 3] = f(accum[i + 3] + 1);
        } else {
          const prev = [accum[i], accum[i + 1], accum[i + 2]];
          const m = vadd(vmuls(e, f(1 - w)), vmuls(prev, w));
          if (mode === 2) { accum[i] = q8(m[0]); accum[i + 1] = q8(m[1]); accum[i + 2] = q8(m[2]); }
          else { accum[i] = m[0]; accum[i + 1] = m[1]; accum[i + 2] = m[2]; }
          accum[i + 3] = 1;
        }
        if (job.aov && s === job.spp - 1) {
          const qn = vadds(vdivs(aov.n, 2), 0.5), qp = normalize(aov.p);
          aovN.set([qn[0], qn[1], qn[2], 1], i);
          aovP.set([qp[0], qp[1], qp[2], 1], i);
        }
      }
    }
  }
  return { accum, aovN, aovP, segments: C.segments };
}

// the spec math by the oracle's fn ids (tests: bit-exact vs oracle_math)
function mathFn(fn, x, y) {
  switch (fn) {
    case 0: return sin_(x);
    case 1: return cos_(x);
    case 2: return tan_(x);
    case 3: return atan2_(y, x);
    case 4: return acos_(x);
    case 6: return atan_(x);
    case 7: return sqrt_(x);
    case 8: return f(x / y);
    case 9: return fmin_(x, y);
    case 10: return fmax_(x, y);
    case 11: return fdiv(x, y);  // GLSL divide spec
    case 12: return clamp_(x, 0, 1);
    case 13: return fma32(x, y, f(0.25));  // the exact f32 fma itself
    case 14: return f(1 / x);
    default: return NaN;
  }
}

module.exports = { render, mathFn, fma32 };

// CLI: node oracle/sail_soft.js job.json out_prefix -> out_prefix.accum.f32 (+ .aovn/.aovp) and a JSON line
// timed baseline: render crops in order until the time budget is spent (one thread, or worker `w` of `nw`
// taking crops w, w + nw, ...)
function timedCrops(job, w = 0, nw = 1) {
  const accum = new Float32Array(job.W * job.H * 4);
  let segments = 0, done = 0, sec = 0;
  const t0 = process.hrtime.bigint();
  for (let i = w; i < job.crops.length; i += nw) {
    segments += render(Object.assign({}, job, { crop: job.crops[i], accum })).segments;
    done++;
    sec = Number(process.hrtime.bigint() - t0) / 1e9;
    if (sec >= job.budgetSeconds) break;
  }
  return { segments, seconds: sec, crops: done, accum };
}

let wt = null;
try { wt = require('worker_threads'); } catch (e) { wt = null; }
if (wt && !wt.isMainThread && wt.workerData && wt.workerData.sailCrops) {
  const d = wt.workerData;
  const { segments, seconds, crops } = timedCrops(d.job, d.w, d.nw);  // the counts only, not the frame
  wt.parentPort.postMessage({ segments, seconds, crops });
} else if (require.main === module) {
  const fs = require('fs');
  const [jobPath, outPrefix] = process.argv.slice(2);
  const job = JSON.parse(fs.readFileSync(jobPath, 'utf8'));
  if (job.crops && job.threads > 1 && wt) {  // the same shader on job.threads worker threads
    const nw = job.threads;
    const t0 = process.hrtime.bigint();
    let left = nw, segments = 0, crops = 0;
    for (let w = 0; w < nw; w++) {
      const worker = new wt.Worker(__filename, { workerData: { sailCrops: true, job, w, nw } });
      worker.on('message', (r) => {
        segments += r.segments; crops += r.crops;
        if (--left === 0) {
          const sec = Number(process.hrtime.bigint() - t0) / 1e9;
          process.stdout.write(JSON.stringify({ segments, seconds: sec, crops, threads: nw, node: process.version }) + '\n');
        }
      });
      worker.on('error', (e) => { process.stderr.write(String(e) + '\n'); process.exitCode = 1; });
    }
  } else if (job.math !== undefined) {  // {math: fn, xHex, yHex: little-endian f32 arrays as hex} -> f32 results
    const hex = (h) => { const b = Buffer.from(h, 'hex'); return new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.length)); };
    const x = hex(job.xHex), y = hex(job.yHex);
    const out = new Float32Array(x.length);
    for (let i = 0; i < out.length; i++) out[i] = mathFn(job.math, x[i], y[i]);
    fs.writeFileSync(outPrefix + '.math.f32', Buffer.from(out.buffer));
    process.stdout.write(JSON.stringify({ n: out.length }) + '\n');
  } else if (job.crops) {
    const r = timedCrops(job);
    // writeAccum: the frame the timed crops rendered (bench.py's full C1 render checks it against tests/golden)
    if (job.writeAccum) fs.writeFileSync(outPrefix + '.accum.f32', Buffer.from(r.accum.buffer));
    process.stdout.write(JSON.stringify({ segments: r.segments, seconds: r.seconds, crops: r.crops, node: process.version }) + '\n');
  } else {
    if (job.accumB64) job.accum = new Float32Array(Buffer.from(job.accumB64, 'base64').buffer.slice(0));
    const t0 = process.hrtime.bigint();
    const r = render(job);
    const s = Number(process.hrtime.bigint() - t0) / 1e9;
    fs.writeFileSync(outPrefix + '.accum.f32', Buffer.from(r.accum.buffer));
    if (r.aovN) { fs.writeFileSync(outPrefix + '.aovn.f32', Buffer.from(r.aovN.buffer)); fs.writeFileSync(outPrefix + '.aovp.f32', Buffer.from(r.aovP.buffer)); }
    process.stdout.write(JSON.stringify({ segments: r.segments, seconds: s, node: process.version }) + '\n');
  }
}
