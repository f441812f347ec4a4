'use strict';
// Writes tests/golden/fuzz_scenes.json: seeded random scenes built with this build's Sail API (sail_amd/js, whose
// serializer tests/test_js_host.py pins to the reference's rows) and exported exactly as the frozen scenes are
// (sail_amd/js/tools/export_scenes.js). Data only: rows, plugin lists, camera.
//
// Each scene draws an enclosure (a matte Cube room, a Cornellbox, or none -- mostly over a ground rectangle -- so
// that rays escape), 2-14 objects of
// the eight analytic shapes at random places and sizes, each with a random material (Matte with and without the
// Oren-Nayar sigma, Mirror, isotropic and anisotropic Metal, smooth and rough Glass), texture (uniform colour,
// Checkerboard, Checkerboard2, Bilerp, Mix, Scale, UV), sometimes an emission or a reversed normal, 1-3 lights
// (Area lights on the samplers with a pdf -- Sphere, Disk, Rectangle -- point and spot lights), and a camera
// inside the room, or inside or outside an open scene. With lights of different kinds the reference reads a light's
// category from the wrong row (light_sample, kept: oracle/sail_oracle.cpp), so some scenes sample an area light on a
// pdf-less shape and turn NaN, as the reference does. tests/test_fuzz_scenes.py renders them with the C++ oracle,
// the JS software shader and every HIP kernel form, bit for bit.
// Run: node tests/golden/make_fuzz_scenes.js [out.json]  (default: tests/golden/fuzz_scenes.json)
const fs = require('fs');
const path = require('path');
const Sail = require('../../sail_amd/js');
const { exportScene } = require('../../sail_amd/js/tools/export_scenes');

const COUNT = 48;

function xorshift32(seed) {
  let s = seed >>> 0;
  return () => {
    s ^= (s << 13) >>> 0; s >>>= 0;
    s ^= s >>> 17;
    s ^= (s << 5) >>> 0; s >>>= 0;
    return s / 4294967296;
  };
}

function makeScene(seed) {
  const u = xorshift32(0x9E3779B9 ^ (seed * 2654435761));
  for (let i = 0; i < 8; i++) u();  // decorrelate nearby seeds
  const pick = (a) => a[Math.floor(u() * a.length) % a.length];
  const range = (lo, hi) => lo + (hi - lo) * u();
  const colour = () => [range(0.05, 1), range(0.05, 1), range(0.05, 1)];
  const point = () => [range(0.6, 4.9), range(0.3, 4.8), range(0.2, 5.0)];

  const material = () => {
    switch (Math.floor(u() * 6)) {
      case 0: return new Sail.Matte(range(0.2, 1));
      case 1: return new Sail.Matte(range(0.2, 1), range(5, 40));  // Oren-Nayar
      case 2: return new Sail.Mirror(range(0.3, 1));
      case 3: return new Sail.Metal(range(0.005, 0.3));
      case 4: return new Sail.Metal(0.01, range(0.01, 0.3), range(0.01, 0.3),
        [range(0.2, 3), range(0.2, 3), range(0.2, 3)], [range(1, 6), range(1, 6), range(1, 6)]);
      default: return u() < 0.5 ? new Sail.Glass(range(0.5, 1), range(0.5, 1), range(1.2, 1.9))
        : new Sail.Glass(1, 1, range(1.2, 1.9), range(0.01, 0.3), range(0.01, 0.3));
    }
  };
  const texture = () => {
    switch (Math.floor(u() * 7)) {
      case 0: return Sail.Color.createTexture(colour());
      case 1: return new Sail.Checkerboard(range(0.05, 0.5), range(0.005, 0.05));
      case 2: return new Sail.Checkerboard2(colour(), colour(), range(0.05, 0.5));
      case 3: return new Sail.Bilerp(colour(), colour(), colour(), colour());
      case 4: return new Sail.Mix(colour(), colour(), range(0, 1));
      case 5: return new Sail.Scale(colour(), colour());
      default: return new Sail.UV();
    }
  };
  const emission = () => (u() < 0.12 ? [range(0.5, 4), range(0.5, 4), range(0.5, 4)] : [0, 0, 0]);
  const shape = (kind, mat, tex, em, rev) => {
    const p = point(), z = range(0.15, 0.9);
    switch (kind) {
      case 0: return new Sail.Sphere(p, z, mat, tex, em, rev);
      case 1: return new Sail.Cube(p, [p[0] + range(0.1, 1), p[1] + range(0.1, 1), p[2] + range(0.1, 1)], mat, tex, em, rev);
      case 2: {  // axis-aligned rectangle: one coordinate shared by min and max
        const q = [p[0] + range(0.2, 1.2), p[1] + range(0.2, 1.2), p[2] + range(0.2, 1.2)];
        q[Math.floor(u() * 3) % 3] = p[Math.floor(u() * 3) % 3];
        for (let a = 0; a < 3; a++) if (q[a] < p[a]) q[a] = p[a];
        let flat = 0;
        for (let a = 0; a < 3; a++) if (q[a] === p[a]) flat++;
        if (flat !== 1) q[1] = p[1];
        return new Sail.Rectangle(p, q, mat, tex, em, rev);
      }
      case 3: return new Sail.Cone(p, range(0.3, 1.5), z, mat, tex, em, rev);
      case 4: return new Sail.Cylinder(p, range(0.3, 1.5), z, mat, tex, em, rev);
      case 5: return new Sail.Disk(p, z, u() < 0.5 ? 0 : range(0, 0.8) * z, mat, tex, em, rev);
      case 6: return new Sail.Hyperboloid(p, [z, 0, 0], [range(0.3, 0.8) * z, range(0.3, 0.8) * z, range(1, 2.5) * z],
        mat, tex, em, rev);
      default: return new Sail.Paraboloid(p, 0, range(0.5, 2) * z, z, mat, tex, em, rev);
    }
  };

  const scene = new Sail.Scene();
  const room = Math.floor(u() * 3);  // 0: Cube room, 1: Cornellbox, 2: open
  if (room === 0) scene.add(new Sail.Cube([0, 0, -7], [5.56, 5.488, 5.592], new Sail.Matte(range(0.4, 0.9)), texture()));
  else if (room === 1) scene.add(new Sail.Cornellbox([0, 0, -7], [5.56, 5.488, 5.592]));
  else if (u() < 0.7) scene.add(new Sail.Rectangle([-4, 0, -4], [10, 0, 10], material(), texture()));  // open: a ground
  const nObj = 2 + Math.floor(u() * 13);
  for (let i = 0; i < nObj; i++) scene.add(shape(Math.floor(u() * 8), material(), texture(), emission(), u() < 0.1));
  const nLights = 1 + Math.floor(u() * 3);
  for (let i = 0; i < nLights; i++) {
    const kind = Math.floor(u() * 4);
    const em = [range(1, 6), range(1, 6), range(1, 6)];
    const matte = new Sail.Matte(0.7);
    if (kind === 0) scene.add(new Sail.AreaLight(new Sail.Sphere([range(1, 4.5), range(4, 5.2), range(0.5, 4.5)], range(0.1, 0.4), matte, Sail.Color.WHITE), em));
    else if (kind === 1) {
      const y = range(4.5, 5.47), x = range(0.5, 4), z = range(0.5, 4);
      scene.add(new Sail.AreaLight(new Sail.Rectangle([x, y, z], [x + range(0.3, 1.2), y, z + range(0.3, 1.2)], matte, Sail.Color.BLACK), em));
    } else if (kind === 2) {
      scene.add(new Sail.AreaLight(new Sail.Disk([range(1, 4.5), range(4.5, 5.4), range(0.5, 4.5)], range(0.2, 0.7), range(0, 0.1), matte, Sail.Color.BLACK), em));
    } else if (kind === 3) {
      if (u() < 0.5) scene.add(new Sail.PointLight([range(0.5, 5), range(3, 5.3), range(-1, 5)], em));
      else scene.add(new Sail.SpotLight([range(0.5, 5), range(4, 5.3), range(0, 5)], range(15, 60), range(1, 10), em));
    }
  }
  const inside = room !== 2 || u() < 0.5;  // a closed room is seen from inside
  const eye = inside ? [range(1.5, 4), range(1.5, 4), range(-5, -1)] : [range(-1, 6.5), range(0, 6), range(-8, -3)];
  scene.add(new Sail.Camera(eye, [range(2, 3.5), range(1.5, 3.5), range(2, 3.5)]));
  return scene;
}

// Edge scenes: a random scene as above, then the whole scene scaled by 10^-3 .. 10^3 (rows, lights and camera), with
// degenerate and extreme members added -- zero / negative radii and heights, inverted boxes, zero-area rectangles,
// disks with the hole wider than the disk, Metal of roughness 0, Glass of eta 1 and below 1, Matte of kd > 1 and
// sigma 90, checkerboards finer than a pixel, Mix amounts outside [0, 1], negative and huge emission, spot cones of 0
// and 180 degrees, an area light on a zero-radius sphere -- and the camera far away or inside an object.
function makeEdgeScene(seed) {
  const u = xorshift32(0x85EBCA6B ^ (seed * 2246822519));
  for (let i = 0; i < 8; i++) u();
  const range = (lo, hi) => lo + (hi - lo) * u();
  const k = [1e-3, 1e-2, 1, 1e2, 1e3][Math.floor(u() * 5)];
  const S = (v) => v.map((x) => x * k);
  const p = () => S([range(0.6, 4.9), range(0.3, 4.8), range(0.2, 5.0)]);
  const mats = [() => new Sail.Matte(range(1, 3)), () => new Sail.Matte(0.7, 90), () => new Sail.Metal(0),
    () => new Sail.Glass(1, 1, 1.0), () => new Sail.Glass(1, 1, range(0.5, 0.95)), () => new Sail.Mirror(1),
    () => new Sail.Metal(0.01, 0.5, 0.001)];
  const texs = [() => new Sail.Checkerboard(1e-4 * k, 0.5 * k), () => new Sail.Mix([1, 0, 0], [0, 1, 0], range(-2, 3)),
    () => new Sail.Scale([-1, 0.5, 2], [1, -1, 0.5]), () => Sail.Color.createTexture([range(0, 2), 0, range(0, 2)]),
    () => new Sail.UV(), () => new Sail.Checkerboard2([1, 1, 1], [0, 0, 0], 1e-4 * k)];
  const mat = () => mats[Math.floor(u() * mats.length)]();
  const tex = () => texs[Math.floor(u() * texs.length)]();
  const scene = new Sail.Scene();
  const room = Math.floor(u() * 3);
  if (room === 0) scene.add(new Sail.Cube(S([0, 0, -7]), S([5.56, 5.488, 5.592]), new Sail.Matte(0.7), tex()));
  else if (room === 1) { const cb = new Sail.Cornellbox([0, 0, -7], [5.56, 5.488, 5.592]); cb.scale(k); scene.add(cb); }
  const makers = [
    () => new Sail.Sphere(p(), 0, mat(), tex()),
    () => new Sail.Sphere(p(), -0.5 * k, mat(), tex()),
    () => { const a = p(); return new Sail.Cube(a, [a[0] - 0.5 * k, a[1] + 0.5 * k, a[2] - 0.5 * k], mat(), tex()); },
    () => { const a = p(); return new Sail.Rectangle(a, [a[0], a[1] + 0.5 * k, a[2]], mat(), tex()); },
    () => new Sail.Disk(p(), 0.5 * k, 0.8 * k, mat(), tex()),
    () => new Sail.Cone(p(), 0, 0.5 * k, mat(), tex()),
    () => new Sail.Cone(p(), -0.8 * k, 0.5 * k, mat(), tex()),
    () => new Sail.Cylinder(p(), 0.8 * k, 0, mat(), tex()),
    () => new Sail.Paraboloid(p(), 0.8 * k, 0.1 * k, 0.5 * k, mat(), tex()),
    () => new Sail.Sphere(p(), range(0.3, 0.9) * k, mat(), tex(), [range(-3, -0.5), 2, 2]),
    () => new Sail.Sphere(p(), range(0.3, 0.9) * k, mat(), tex(), [1e30, 1e30, 1e30]),
    () => new Sail.Cylinder(p(), range(0.3, 1.5) * k, range(0.2, 0.8) * k, mat(), tex()),
    () => new Sail.Hyperboloid(p(), [0.5 * k, 0, 0], [0.25 * k, 0.25 * k, k], mat(), tex()),
  ];
  const nObj = 3 + Math.floor(u() * 10);
  for (let i = 0; i < nObj; i++) scene.add(makers[Math.floor(u() * makers.length)]());
  const lights = [
    () => new Sail.SpotLight(S([2.78, 5, 2.5]), 0, 0, [5, 5, 5]),
    () => new Sail.SpotLight(S([2.78, 5, 2.5]), 180, 200, [5, 5, 5]),
    () => new Sail.PointLight(S([range(0.5, 5), range(0.5, 5), range(0.5, 5)]), [3 * k * k, 3 * k * k, 3 * k * k]),
    () => new Sail.AreaLight(new Sail.Sphere(S([2.5, 5, 2.5]), 0, new Sail.Matte(0.7), Sail.Color.WHITE), [4, 4, 4]),
    () => new Sail.AreaLight(new Sail.Disk(S([2.5, 5.3, 2.5]), 0.6 * k, 0.2 * k, new Sail.Matte(0.7), Sail.Color.BLACK), [4, 4, 4]),
  ];
  const nLights = Math.floor(u() * 3);
  for (let i = 0; i < nLights; i++) scene.add(lights[Math.floor(u() * lights.length)]());
  const view = Math.floor(u() * 3);  // 0: inside the scene, 1: far away, 2: inside the first object's bounds
  const eye = view === 0 ? S([range(1.5, 4), range(1.5, 4), range(-5, -1)])
    : view === 1 ? S([range(-3, 9) * 1e3, range(-1, 8) * 1e3, -1e4]) : scene.objects[room === 2 ? 0 : 1].boundbox().min.elements.slice();
  scene.add(new Sail.Camera(eye, S([range(2, 3.5), range(1.5, 3.5), range(2, 3.5)])));
  return scene;
}
const EDGE_COUNT = 16;

if (require.main === module) {
  const out = {};
  for (let k = 0; k < COUNT; k++) out[`F${String(k).padStart(2, '0')}`] = exportScene(makeScene(k + 1));
  for (let k = 0; k < EDGE_COUNT; k++) out[`E${String(k).padStart(2, '0')}`] = exportScene(makeEdgeScene(k + 1));
  const file = process.argv[2] || path.join(__dirname, 'fuzz_scenes.json');
  fs.writeFileSync(file, JSON.stringify(out));
}
module.exports = { makeScene, makeEdgeScene, COUNT, EDGE_COUNT };
