'use strict';
// The frozen benchmark scenes of SURVEY §8(d), written with the Sail API, plus the UI demo script
// (ui/ui.js:10-44) and a scene exercising every texture/material kind (test coverage).
const Sail = require('./index');

// C1 / C2 / C5: README Cornell box, minimally fixed (README.md:34-66 throws as written: SURVEY §0.5)
function readmeCornell(gaussian) {
  const scene = new Sail.Scene();
  scene.add(new Sail.Cube([2.13, 5.487, 2.27], [3.43, 5.488, 3.32], new Sail.Matte(0.7),
    Sail.Color.createTexture([0, 0, 0]), [8, 8, 8]));
  scene.add(new Sail.Cornellbox([0, 0, -7], [5.560, 5.488, 5.592]));
  scene.add(new Sail.Sphere([2, 1.25, 2.70], 1.2, new Sail.Mirror(1.0), Sail.Color.WHITE));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  if (gaussian) {
    scene.filter = 'gaussian';
    scene.filter.addParam('r', 'vec2(2.0,2.0)');
    scene.filter.addParam('alpha', '2.0');
  }
  return scene;
}

// C3: materials demo
function materialsDemo() {
  const scene = new Sail.Scene();
  const matte = new Sail.Matte(0.7);
  scene.add(new Sail.AreaLight(new Sail.Rectangle([2.13, 5.48, 2.27], [3.43, 5.48, 3.32], matte, Sail.Color.BLACK), [4, 4, 4]));
  scene.add(new Sail.Cube([0, 0, -7], [5.56, 5.488, 5.592], matte, new Sail.Checkerboard(0.1, 0.01)));
  scene.add(new Sail.Sphere([1.0, 0.8, 1.5], 0.8, new Sail.Metal(0, 0.01, 0.1), Sail.Color.WHITE));
  scene.add(new Sail.Sphere([2.2, 0.8, 2.8], 0.8, new Sail.Mirror(1.0), Sail.Color.WHITE));
  scene.add(new Sail.Sphere([3.4, 0.8, 1.5], 0.8, new Sail.Glass(1, 1, 1.5), Sail.Color.WHITE));
  scene.add(new Sail.Sphere([4.6, 0.8, 2.8], 0.8, matte, new Sail.Checkerboard2([1, 1, 1], [0.2, 0.2, 0.2], 0.1)));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  scene.filter = 'gaussian';
  scene.filter.addParam('r', 'vec2(2.0,2.0)');
  scene.filter.addParam('alpha', '2.0');
  return scene;
}

function xorshift32(seed) {
  let s = seed >>> 0;
  return () => {
    s ^= (s << 13) >>> 0; s >>>= 0;
    s ^= s >>> 17;
    s ^= (s << 5) >>> 0; s >>>= 0;
    return s / 4294967296;
  };
}

// C4: 64 random analytic primitives + 4 lights
function random64() {
  const scene = new Sail.Scene();
  scene.add(new Sail.Cube([0, 0, -1], [10, 10, 10], new Sail.Matte(0.7), Sail.Color.WHITE));
  const u = xorshift32(0xC4);
  for (let i = 0; i < 64; i++) {
    const p = [0.5 + 9 * u(), 0.5 + 9 * u(), 1.5 + 8 * u()];
    const z = 0.2 + 0.6 * u();
    const mat = [new Sail.Matte(0.7), new Sail.Mirror(1), new Sail.Metal(0, 0.01, 0.1), new Sail.Glass(1, 1, 1.5)][i % 4];
    const tex = [Sail.Color.WHITE, new Sail.Checkerboard(0.1, 0.01), new Sail.Checkerboard2([1, 1, 1], [0.2, 0.2, 0.2], 0.1)][i % 3];
    let ob;
    switch (i % 8) {
      case 0: case 7: ob = new Sail.Sphere(p, z, mat, tex); break;
      case 1: ob = new Sail.Cube(p, [p[0] + z, p[1] + z, p[2] + z], mat, tex); break;
      case 2: ob = new Sail.Cone(p, 2 * z, z, mat, tex); break;
      case 3: ob = new Sail.Cylinder(p, 2 * z, z, mat, tex); break;
      case 4: ob = new Sail.Hyperboloid(p, [z, 0, 0], [0.5 * z, 0.5 * z, 2 * z], mat, tex); break;
      case 5: ob = new Sail.Paraboloid(p, 0, 2 * z, z, mat, tex); break;
      default: ob = new Sail.Disk(p, z, 0.2 * z, mat, tex); break;
    }
    scene.add(ob);
  }
  scene.add(new Sail.AreaLight(new Sail.Sphere([3, 8, 5], 0.3, new Sail.Matte(0.7), Sail.Color.WHITE), [4, 4, 4]));
  scene.add(new Sail.AreaLight(new Sail.Sphere([7, 8, 5], 0.3, new Sail.Matte(0.7), Sail.Color.WHITE), [4, 4, 4]));
  scene.add(new Sail.PointLight([5, 9, 3], [2, 2, 2]));
  scene.add(new Sail.SpotLight([5, 9.5, 6], 30, 5, [6, 6, 6]));
  scene.add(new Sail.Camera([5, 5, 0], [5, 5, 10]));
  return scene;
}

// ui/ui.js:10-44
function uiDemo() {
  const scene = new Sail.Scene();
  const camera = new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]);
  const matte = new Sail.Matte(0.7);
  const mirror = new Sail.Mirror(1.0);
  const glass = new Sail.Glass(1, 1, 1.5);
  scene.add(new Sail.AreaLight(new Sail.Rectangle([2.13, 5.48, 2.27], [3.43, 5.48, 3.32], matte, Sail.Color.BLACK), [1, 1, 1]));
  scene.add(new Sail.Cornellbox());
  scene.add(new Sail.Sphere([1.5, 1.25, 2.70], 1.2, mirror, Sail.Color.WHITE));
  scene.add(new Sail.Sphere([3.9, 1.25, 1.70], 1.2, glass, Sail.Color.WHITE));
  scene.add(camera);
  scene.filter = 'tonemapping';
  scene.trace = 'path';
  return scene;
}

function allKinds() {
  const scene = new Sail.Scene();
  scene.add(new Sail.Cornellbox([0, 0, -7], [5.56, 5.488, 5.592]));
  scene.add(new Sail.Sphere([1, 1, 1], 0.5, new Sail.Matte(0.8, 20), new Sail.Mix([1, 0, 0], [0, 0, 1], 0.25)));
  scene.add(new Sail.Sphere([2.5, 1, 1], 0.5, new Sail.Metal(0.1, 0.05, 0.2), new Sail.Scale([1, 0.5, 0.5], [0.5, 1, 1])));
  scene.add(new Sail.Sphere([4, 1, 1], 0.5, new Sail.Glass(1, 1, 1.5, 0.1, 0.1), new Sail.UV()));
  scene.add(new Sail.Disk([2.78, 0.01, 3], 1.0, 0.3, new Sail.Matte(0.5), new Sail.Checkerboard(0.2, 0.02)));
  scene.add(new Sail.PointLight([2.78, 5, 2], [3, 3, 3]));
  scene.add(new Sail.SpotLight([2.78, 5.3, 3], 40, 10, [5, 5, 5]));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  scene.filter = 'sinc';
  scene.filter.addParam('r', 'vec2(2.0,2.0)');
  scene.filter.addParam('tau', '3.0');
  return scene;
}

// ---- coverage scenes (round 2): every geometry as an AreaLight, zero / one primitive, Bilerp --------------
// AreaLight accepts any geometry (src/scene/light.js:40-55). Disk, Sphere and Rectangle sample a point with a
// pdf (disk.glsl:77-83, sphere.glsl:88-92, rectangle.glsl:65-70); Cube, Cone, Cylinder, Hyperboloid,
// Paraboloid and Cornellbox return BLACK without writing pdf (cube.glsl:50-52 etc.): defined as pdf = 0.
function areaGood() {
  const scene = new Sail.Scene();
  const matte = new Sail.Matte(0.7);
  scene.add(new Sail.Cube([0, 0, -7], [5.56, 5.488, 5.592], matte, Sail.Color.WHITE));
  scene.add(new Sail.AreaLight(new Sail.Disk([1.5, 5.3, 2.5], 0.5, 0.1, matte, Sail.Color.BLACK), [3, 3, 3]));
  scene.add(new Sail.AreaLight(new Sail.Sphere([4.0, 4.6, 3.0], 0.3, matte, Sail.Color.WHITE), [4, 4, 4]));
  scene.add(new Sail.AreaLight(new Sail.Rectangle([2.5, 5.47, 1.0], [3.2, 5.47, 1.8], matte, Sail.Color.BLACK), [2, 2, 2]));
  scene.add(new Sail.Sphere([2.0, 1.0, 2.5], 1.0, new Sail.Matte(0.7), new Sail.Checkerboard2([1, 1, 1], [0.2, 0.2, 0.2], 0.1)));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
function areaBlack() {
  const scene = new Sail.Scene();
  const matte = new Sail.Matte(0.7);
  // a mirror room: paths reach the lights' surfaces (finite radiance) besides the matte sphere and floor
  // disk, whose light samples divide by the unwritten pdf (inf / NaN radiance)
  scene.add(new Sail.Cube([0, 0, -7], [5.56, 5.488, 5.592], new Sail.Mirror(0.9), Sail.Color.WHITE));
  scene.add(new Sail.Disk([2.0, 0.01, 1.0], 1.2, 0.0, matte, Sail.Color.WHITE));
  scene.add(new Sail.AreaLight(new Sail.Cube([0.5, 4.5, 3.0], [1.0, 5.0, 3.5], matte, Sail.Color.WHITE), [2, 2, 2]));
  scene.add(new Sail.AreaLight(new Sail.Cone([1.5, 4.0, 3.0], 0.8, 0.4, matte, Sail.Color.WHITE), [2, 2, 2]));
  scene.add(new Sail.AreaLight(new Sail.Cylinder([2.5, 4.0, 3.0], 0.8, 0.3, matte, Sail.Color.WHITE), [2, 2, 2]));
  scene.add(new Sail.AreaLight(new Sail.Hyperboloid([3.5, 4.0, 3.0], [0.3, 0, 0], [0.15, 0.15, 0.8], matte, Sail.Color.WHITE), [2, 2, 2]));
  scene.add(new Sail.AreaLight(new Sail.Paraboloid([4.5, 4.0, 3.0], 0, 0.8, 0.4, matte, Sail.Color.WHITE), [2, 2, 2]));
  scene.add(new Sail.AreaLight(new Sail.Cornellbox([0.2, 0.2, 4.0], [1.0, 1.0, 4.8]), [2, 2, 2]));
  scene.add(new Sail.Sphere([2.5, 1.0, 2.0], 0.8, matte, Sail.Color.WHITE));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
// n = 1: the row coordinate float(i)/float(n-1) is 0/0 (shader.shape.js:34): row 0. A closed room (every ray
// hits) with a point light (ln = 1), and a lone emissive sphere (rays around it miss)
function oneRoom() {
  const scene = new Sail.Scene();
  scene.add(new Sail.Cube([0, 0, -7], [5.56, 5.488, 5.592], new Sail.Matte(0.7), new Sail.Checkerboard(0.1, 0.01)));
  scene.add(new Sail.PointLight([2.78, 5, 2], [3, 3, 3]));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
function oneSphere() {
  const scene = new Sail.Scene();
  scene.add(new Sail.Sphere([2.78, 2.73, 2.79], 1.5, new Sail.Matte(0.7), Sail.Color.WHITE, [0.5, 0.8, 1.0]));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
// n = 0: every primary ray misses (the AOV miss branch), with a light row that is never sampled
function emptyScene() {
  const scene = new Sail.Scene();
  scene.add(new Sail.PointLight([2.78, 5, 2], [3, 3, 3]));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
// Bilerp (bilerp.glsl:1-13; the reference's GLSL does not compile, the intended bilinear math is built) on
// shapes with different UV maps
function bilerpScene() {
  const scene = new Sail.Scene();
  const matte = new Sail.Matte(0.7);
  const bl = () => new Sail.Bilerp([1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0]);
  scene.add(new Sail.AreaLight(new Sail.Rectangle([2.13, 5.48, 2.27], [3.43, 5.48, 3.32], matte, Sail.Color.BLACK), [4, 4, 4]));
  scene.add(new Sail.Cornellbox([0, 0, -7], [5.56, 5.488, 5.592]));
  scene.add(new Sail.Sphere([1.2, 1.0, 2.5], 0.9, matte, bl()));
  scene.add(new Sail.Cube([2.4, 0.0, 1.5], [3.3, 1.2, 2.4], matte, bl()));
  scene.add(new Sail.Cylinder([4.2, 0.0, 2.5], 1.5, 0.6, matte, bl()));
  scene.add(new Sail.Disk([2.78, 0.01, 3.8], 1.0, 0.2, matte, bl()));
  scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}

const SCENES = {
  C1: () => readmeCornell(false), C1g: () => readmeCornell(true), C3: materialsDemo, C4: random64, UI: uiDemo, ALL: allKinds,
  AREA: areaGood, AREA0: areaBlack, N1: oneRoom, N1S: oneSphere, N0: emptyScene, BILERP: bilerpScene,
};
module.exports = { SCENES, readmeCornell, materialsDemo, random64, uiDemo, allKinds };
