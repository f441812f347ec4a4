// Golden-fixture generator (test infrastructure; runs ONLY in the build container).
//
// Loads the reference bundle /root/reference/bin/sail.js (in sync with src/, SURVEY §0.3) inside a
// Node `vm` context with a stub `window` and a recording WebGL2 `gl` Proxy (SURVEY Appendix C), builds
// the frozen benchmark scenes of SURVEY §8(d) through the reference's own public API, and writes ONLY
// DATA to tests/golden/fixtures.json:
//   * the serialized objects / texParams / lights rows exactly as uploaded by Tracer.update
//     (src/core/tracer.js:42-90 -> texImage2D R32F), n / tn / ln, plugin lists (scene.js:70-112)
//   * scene.mat (P*MV, src/scene/scene.js:40-42) and eye
//   * inverse(T(jitter) * P*MV) for fixed jitters (tracer.js:94-96, matrix.js:501-527), flattened
//     column-major as uploaded (webgl.js:102-103)
//   * the window-filter weight tables as emitted into the render program (filter/*.js)
//   * CPU double-precision intersect() distances for 7 shape types (src/scene/geometry.js:110-591)
//   * host-derived constants: Matte A/B, SpotLight cosines, Hyperboloid ah/ch
//   * sha256 of every generated GLSL program (identity of the codegen the oracle restates)
// No reference source text is written. The output is committed; the GPU box never reads /root/reference.
//
// Usage: node tests/golden/make_fixtures.js [/root/reference/bin/sail.js] > tests/golden/fixtures.json
'use strict';
const fs = require('fs');
const vm = require('vm');
const crypto = require('crypto');

const bundlePath = process.argv[2] || '/root/reference/bin/sail.js';
const src = fs.readFileSync(bundlePath, 'utf8');

// ---- recording gl stub ---------------------------------------------------------------------------
const calls = [];
let objCounter = 0;
const glTarget = {};
const gl = new Proxy(glTarget, {
  get(t, prop) {
    if (typeof prop !== 'string') return undefined;
    if (/^[A-Z0-9_]+$/.test(prop)) return prop;            // enums are their own names
    if (prop === 'getExtension') return () => null;        // WebGL2: OES_texture_float not exposed
    if (/^get.*Parameter$/.test(prop)) return () => true;
    if (/^create/.test(prop)) return () => ({ id: ++objCounter });
    if (prop === 'getUniformLocation') return (p, name) => ({ name });
    if (prop === 'getAttribLocation') return () => 0;
    return (...args) => { calls.push([prop, args]); };
  },
});
const canvas = { getContext: () => gl, width: 512, height: 512, addEventListener() {} };
const sandbox = {
  console, Math, Date, Float32Array, Uint16Array, Uint8Array, Array, Object, JSON, isFinite, isNaN,
  parseFloat, parseInt, alert: (m) => { throw new Error('alert: ' + m); },
  document: { getElementById: () => canvas, body: {}, documentElement: {} },
  requestAnimationFrame: () => 0,
};
sandbox.window = sandbox;
sandbox.gl = null;
vm.createContext(sandbox);
vm.runInContext(src, sandbox, { filename: 'sail.js' });
const S = sandbox.Sail;

function f32list(arr) { return Array.from(new Float32Array(arr)); }

function lastUploads(sinceIdx) {
  // texImage2D(target, level, internal, w, h, border, format, type, data)
  const ups = [];
  for (let i = sinceIdx; i < calls.length; i++) {
    const [name, a] = calls[i];
    if (name === 'texImage2D' && a[2] === 'R32F') ups.push({ w: a[3], h: a[4], data: Array.from(a[8]) });
  }
  return ups;
}
function shaderSources(sinceIdx) {
  const out = [];
  for (let i = sinceIdx; i < calls.length; i++) if (calls[i][0] === 'shaderSource') out.push(calls[i][1][1]);
  return out;
}
const sha = (s) => crypto.createHash('sha256').update(s).digest('hex');

// ---- frozen scenes (SURVEY §8(d)) ------------------------------------------------------------------
function sceneC1(filter) {
  const scene = new S.Scene();
  scene.add(new S.Cube([2.13, 5.487, 2.27], [3.43, 5.488, 3.32], new S.Matte(0.7),
    S.Color.createTexture([0, 0, 0]), [8, 8, 8]));
  scene.add(new S.Cornellbox([0, 0, -7], [5.560, 5.488, 5.592]));
  scene.add(new S.Sphere([2, 1.25, 2.70], 1.2, new S.Mirror(1.0), S.Color.WHITE));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  if (filter) { scene.filter = 'gaussian'; scene.filter.addParam('r', 'vec2(2.0,2.0)'); scene.filter.addParam('alpha', '2.0'); }
  return scene;
}
function sceneC3() {
  const scene = new S.Scene();
  const matte = new S.Matte(0.7);
  scene.add(new S.AreaLight(new S.Rectangle([2.13, 5.48, 2.27], [3.43, 5.48, 3.32], matte, S.Color.BLACK), [4, 4, 4]));
  scene.add(new S.Cube([0, 0, -7], [5.56, 5.488, 5.592], matte, new S.Checkerboard(0.1, 0.01)));
  scene.add(new S.Sphere([1.0, 0.8, 1.5], 0.8, new S.Metal(0, 0.01, 0.1), S.Color.WHITE));
  scene.add(new S.Sphere([2.2, 0.8, 2.8], 0.8, new S.Mirror(1.0), S.Color.WHITE));
  scene.add(new S.Sphere([3.4, 0.8, 1.5], 0.8, new S.Glass(1, 1, 1.5), S.Color.WHITE));
  scene.add(new S.Sphere([4.6, 0.8, 2.8], 0.8, matte, new S.Checkerboard2([1, 1, 1], [0.2, 0.2, 0.2], 0.1)));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  scene.filter = 'gaussian'; scene.filter.addParam('r', 'vec2(2.0,2.0)'); scene.filter.addParam('alpha', '2.0');
  return scene;
}
function xorshift32(seed) {
  let s = seed >>> 0;
  return () => { s ^= (s << 13) >>> 0; s >>>= 0; s ^= s >>> 17; s ^= (s << 5) >>> 0; s >>>= 0; return s / 4294967296; };
}
function sceneC4() {
  const scene = new S.Scene();
  scene.add(new S.Cube([0, 0, -1], [10, 10, 10], new S.Matte(0.7), S.Color.WHITE));
  const u = xorshift32(0xC4);
  for (let i = 0; i < 64; i++) {
    const p = [0.5 + 9 * u(), 0.5 + 9 * u(), 1.5 + 8 * u()];
    const z = 0.2 + 0.6 * u();
    const mat = [new S.Matte(0.7), new S.Mirror(1), new S.Metal(0, 0.01, 0.1), new S.Glass(1, 1, 1.5)][i % 4];
    const tex = [S.Color.WHITE, new S.Checkerboard(0.1, 0.01), new S.Checkerboard2([1, 1, 1], [0.2, 0.2, 0.2], 0.1)][i % 3];
    let ob;
    switch (i % 8) {
      case 0: case 7: ob = new S.Sphere(p, z, mat, tex); break;
      case 1: ob = new S.Cube(p, [p[0] + z, p[1] + z, p[2] + z], mat, tex); break;
      case 2: ob = new S.Cone(p, 2 * z, z, mat, tex); break;
      case 3: ob = new S.Cylinder(p, 2 * z, z, mat, tex); break;
      case 4: ob = new S.Hyperboloid(p, [z, 0, 0], [0.5 * z, 0.5 * z, 2 * z], mat, tex); break;
      case 5: ob = new S.Paraboloid(p, 0, 2 * z, z, mat, tex); break;
      case 6: ob = new S.Disk(p, z, 0.2 * z, mat, tex); break;
    }
    scene.add(ob);
  }
  scene.add(new S.AreaLight(new S.Sphere([3, 8, 5], 0.3, new S.Matte(0.7), S.Color.WHITE), [4, 4, 4]));
  scene.add(new S.AreaLight(new S.Sphere([7, 8, 5], 0.3, new S.Matte(0.7), S.Color.WHITE), [4, 4, 4]));
  scene.add(new S.PointLight([5, 9, 3], [2, 2, 2]));
  scene.add(new S.SpotLight([5, 9.5, 6], 30, 5, [6, 6, 6]));
  scene.add(new S.Camera([5, 5, 0], [5, 5, 10]));
  return scene;
}
function sceneUI() {  // ui/ui.js:10-44 demo script
  const scene = new S.Scene();
  const camera = new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]);
  const matte = new S.Matte(0.7);
  const mirror = new S.Mirror(1.0);
  const glass = new S.Glass(1, 1, 1.5);
  scene.add(new S.AreaLight(new S.Rectangle([2.13, 5.48, 2.27], [3.43, 5.48, 3.32], matte, S.Color.BLACK), [1, 1, 1]));
  scene.add(new S.Cornellbox());
  scene.add(new S.Sphere([1.5, 1.25, 2.70], 1.2, mirror, S.Color.WHITE));
  scene.add(new S.Sphere([3.9, 1.25, 1.70], 1.2, glass, S.Color.WHITE));
  scene.add(camera);
  scene.filter = 'tonemapping';
  scene.trace = 'path';
  return scene;
}
function sceneAllTextures() {  // every texture / material kind once (Bilerp excluded: its GLSL does not compile, SURVEY a.7)
  const scene = new S.Scene();
  scene.add(new S.Cornellbox([0, 0, -7], [5.56, 5.488, 5.592]));
  scene.add(new S.Sphere([1, 1, 1], 0.5, new S.Matte(0.8, 20), new S.Mix([1, 0, 0], [0, 0, 1], 0.25)));
  scene.add(new S.Sphere([2.5, 1, 1], 0.5, new S.Metal(0.1, 0.05, 0.2), new S.Scale([1, 0.5, 0.5], [0.5, 1, 1])));
  scene.add(new S.Sphere([4, 1, 1], 0.5, new S.Glass(1, 1, 1.5, 0.1, 0.1), new S.UV()));
  scene.add(new S.Disk([2.78, 0.01, 3], 1.0, 0.3, new S.Matte(0.5), new S.Checkerboard(0.2, 0.02)));
  scene.add(new S.PointLight([2.78, 5, 2], [3, 3, 3]));
  scene.add(new S.SpotLight([2.78, 5.3, 3], 40, 10, [5, 5, 5]));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  scene.filter = 'sinc'; scene.filter.addParam('r', 'vec2(2.0,2.0)'); scene.filter.addParam('tau', '3.0');
  return scene;
}

// ---- coverage scenes (round 2): every geometry as an AreaLight, zero / one primitive, Bilerp --------------
// AreaLight accepts any geometry (src/scene/light.js:40-55). Disk, Sphere and Rectangle sample a point with a
// pdf (disk.glsl:77-83, sphere.glsl:88-92, rectangle.glsl:65-70); Cube, Cone, Cylinder, Hyperboloid,
// Paraboloid and Cornellbox return BLACK without writing pdf (cube.glsl:50-52 etc.): defined as pdf = 0.
function sceneAreaGood() {
  const scene = new S.Scene();
  const matte = new S.Matte(0.7);
  scene.add(new S.Cube([0, 0, -7], [5.56, 5.488, 5.592], matte, S.Color.WHITE));
  scene.add(new S.AreaLight(new S.Disk([1.5, 5.3, 2.5], 0.5, 0.1, matte, S.Color.BLACK), [3, 3, 3]));
  scene.add(new S.AreaLight(new S.Sphere([4.0, 4.6, 3.0], 0.3, matte, S.Color.WHITE), [4, 4, 4]));
  scene.add(new S.AreaLight(new S.Rectangle([2.5, 5.47, 1.0], [3.2, 5.47, 1.8], matte, S.Color.BLACK), [2, 2, 2]));
  scene.add(new S.Sphere([2.0, 1.0, 2.5], 1.0, new S.Matte(0.7), new S.Checkerboard2([1, 1, 1], [0.2, 0.2, 0.2], 0.1)));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
function sceneAreaBlack() {
  const scene = new S.Scene();
  const matte = new S.Matte(0.7);
  // a mirror room: paths reach the lights' surfaces (finite radiance) besides the matte sphere and floor
  // disk, whose light samples divide by the unwritten pdf (inf / NaN radiance)
  scene.add(new S.Cube([0, 0, -7], [5.56, 5.488, 5.592], new S.Mirror(0.9), S.Color.WHITE));
  scene.add(new S.Disk([2.0, 0.01, 1.0], 1.2, 0.0, matte, S.Color.WHITE));
  scene.add(new S.AreaLight(new S.Cube([0.5, 4.5, 3.0], [1.0, 5.0, 3.5], matte, S.Color.WHITE), [2, 2, 2]));
  scene.add(new S.AreaLight(new S.Cone([1.5, 4.0, 3.0], 0.8, 0.4, matte, S.Color.WHITE), [2, 2, 2]));
  scene.add(new S.AreaLight(new S.Cylinder([2.5, 4.0, 3.0], 0.8, 0.3, matte, S.Color.WHITE), [2, 2, 2]));
  scene.add(new S.AreaLight(new S.Hyperboloid([3.5, 4.0, 3.0], [0.3, 0, 0], [0.15, 0.15, 0.8], matte, S.Color.WHITE), [2, 2, 2]));
  scene.add(new S.AreaLight(new S.Paraboloid([4.5, 4.0, 3.0], 0, 0.8, 0.4, matte, S.Color.WHITE), [2, 2, 2]));
  scene.add(new S.AreaLight(new S.Cornellbox([0.2, 0.2, 4.0], [1.0, 1.0, 4.8]), [2, 2, 2]));
  scene.add(new S.Sphere([2.5, 1.0, 2.0], 0.8, matte, S.Color.WHITE));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
// n = 1: the row coordinate float(i)/float(n-1) is 0/0 (shader.shape.js:34): row 0. A closed room (every ray
// hits) with a point light (ln = 1), and a lone emissive sphere (rays around it miss)
function sceneOneRoom() {
  const scene = new S.Scene();
  scene.add(new S.Cube([0, 0, -7], [5.56, 5.488, 5.592], new S.Matte(0.7), new S.Checkerboard(0.1, 0.01)));
  scene.add(new S.PointLight([2.78, 5, 2], [3, 3, 3]));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
function sceneOneSphere() {
  const scene = new S.Scene();
  scene.add(new S.Sphere([2.78, 2.73, 2.79], 1.5, new S.Matte(0.7), S.Color.WHITE, [0.5, 0.8, 1.0]));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
// n = 0: every primary ray misses (the AOV miss branch), with a light row that is never sampled
function sceneEmpty() {
  const scene = new S.Scene();
  scene.add(new S.PointLight([2.78, 5, 2], [3, 3, 3]));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}
// Bilerp (bilerp.glsl:1-13; the reference's GLSL does not compile, the intended bilinear math is built) on
// shapes with different UV maps
function sceneBilerp() {
  const scene = new S.Scene();
  const matte = new S.Matte(0.7);
  const bl = () => new S.Bilerp([1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0]);
  scene.add(new S.AreaLight(new S.Rectangle([2.13, 5.48, 2.27], [3.43, 5.48, 3.32], matte, S.Color.BLACK), [4, 4, 4]));
  scene.add(new S.Cornellbox([0, 0, -7], [5.56, 5.488, 5.592]));
  scene.add(new S.Sphere([1.2, 1.0, 2.5], 0.9, matte, bl()));
  scene.add(new S.Cube([2.4, 0.0, 1.5], [3.3, 1.2, 2.4], matte, bl()));
  scene.add(new S.Cylinder([4.2, 0.0, 2.5], 1.5, 0.6, matte, bl()));
  scene.add(new S.Disk([2.78, 0.01, 3.8], 1.0, 0.2, matte, bl()));
  scene.add(new S.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
  return scene;
}

// ---- the reference picker (src/core/pickup.js:46-66) on a grid of 512x512-canvas mouse positions: its selection
// (the object's row: scene.objects order = serialized row order), the distance object.intersect() returns for it,
// the picker's own ray (Ray.generate, pickup.js:9-12), and whether the four positions 0.75 px away pick the same
// object (away from silhouettes)
function pickGrid(scene, step) {
  S.Control.update(scene);                        // Control.pick = new Pickup(scene)
  const picker = S.Control.pick;
  const inv = scene.mat.inverse();
  const rows = [];
  const sel = () => scene.objects.indexOf(scene.select);
  for (let y = step / 2; y < 512; y += step) {
    for (let x = step / 2; x < 512; x += step) {
      picker.pick(x, y);
      const row = sel();
      let stable = true;
      for (const [dx, dy] of [[0.75, 0], [-0.75, 0], [0, 0.75], [0, -0.75]]) {
        picker.pick(x + dx, y + dy);
        if (sel() !== row) stable = false;
      }
      const dir = inv.multiply(new S.Vector([(x / 512) * 2 - 1, 1 - (y / 512) * 2, 0, 1])).divideByW().ensure3()
        .subtract(scene.eye);
      const t = row >= 0 ? scene.objects[row].intersect({ origin: scene.eye, dir }) : null;
      // the ray as the f32 values sail_pick receives (Math.fround), t to 9 significant digits: data size
      rows.push({ x, y, row, t: t === null ? null : +t.toPrecision(9), stable, dir: Array.from(dir.elements, Math.fround) });
    }
  }
  return { eye: Array.from(scene.eye.elements), picks: rows };
}
// each object's boundbox() (src/scene/geometry.js: false for Object3D/Cornellbox, slack of 0.05 on flat axes)
function boundboxes(scene) {
  return scene.objects.map((o) => {
    const b = o.boundbox();
    return b ? { min: Array.from(b.min.elements), max: Array.from(b.max.elements), shape: o.constructor.name }
      : { min: null, max: null, shape: o.constructor.name };
  });
}
// the generated trace program's #defines (name -> value text) and the numeric literals of each of its functions,
// as data: which constants the restatement must carry (tests/test_reference_constants.py)
function programConstants(srcs) {
  const prog = srcs.find((s) => /void trace\(/.test(s) && /intersectObjects/.test(s));
  if (!prog) return null;
  const defines = {};
  const re = /^#define\s+(\w+)\s+(.*)$/gm;
  let m;
  while ((m = re.exec(prog))) defines[m[1]] = m[2].trim();
  // function bodies by brace depth; a header is the text before a depth-0 '{'
  const literals = {};
  let depth = 0, fn = null, start = 0;
  for (let i = 0; i < prog.length; i++) {
    const ch = prog[i];
    if (ch === '{') {
      if (depth === 0) {
        const head = prog.slice(start, i);
        const h = /(\w+)\s*\([^()]*\)\s*$/.exec(head.replace(/\s+/g, ' '));
        fn = h ? h[1] : null;
        start = i + 1;
      }
      depth++;
    } else if (ch === '}') {
      depth--;
      if (depth === 0) {
        if (fn) {
          const body = prog.slice(start, i).replace(/\/\/.*$/gm, '');
          const lits = body.match(/(?<![\w.])(\d+\.\d*|\.\d+|\d+)([eE][-+]?\d+)?(?![\w.])/g) || [];
          literals[fn] = Array.from(new Set((literals[fn] || []).concat(lits.filter((x) => /[.eE]/.test(x)))));
        }
        fn = null;
        start = i + 1;
      }
    } else if (depth === 0 && ch === ';') {
      start = i + 1;
    }
  }
  return { defines, literals };
}

function capture(name, scene) {
  const renderer = new S.Renderer(canvas);
  const c0 = calls.length;
  renderer.update(scene);
  const ups = lastUploads(c0);
  const srcs = shaderSources(c0);
  const cfg = scene.tracerConfig();
  const objs = ups[0], tps = ups[1], lts = ups[2];
  const mat = scene.mat.elements.map((r) => r.slice());
  const result = {
    n: objs.h, tn: tps.h, ln: lts.h,
    objects: f32list(objs.data), texparams: f32list(tps.data), lights: f32list(lts.data),
    plugins: {
      shape: cfg.shape.map((p) => p.name), material: cfg.material.map((p) => p.name),
      texture: cfg.texture.map((p) => p.name), light: cfg.light.map((p) => p.name),
    },
    filter: { name: scene.filter.name, params: Object.assign({}, scene.filter.params) },
    mvp_rowmajor: mat, eye: Array.from(scene.eye.elements),
    glsl_sha256: srcs.map(sha), glsl_lines: srcs.map((s) => s.split('\n').length),
    boundbox: boundboxes(scene),
  };
  // weight table as emitted into the render program (window filters only)
  for (const s of srcs) {
    const m = /windowWeightTable\[FILTER_WINDOW_LENGTH\] = float\[FILTER_WINDOW_LENGTH\]\(([^)]*)\);/.exec(s);
    if (m) result.filter.weight_text = m[1].split(',').map((x) => x.trim());
    const rr = /#define FILTER_WINDOW_RADIUS (.*)/.exec(s);
    if (rr) result.filter.radius_text = rr[1].trim();
  }
  // per-sample uniforms for fixed jitters: inverse(T(j/512) * P*MV), flattened column-major (webgl.js:103)
  result.inverse = [];
  const jit = [[0, 0], [0.25, -0.75], [-1, 1], [0.999, -0.5]];
  for (const [jx, jy] of jit) {
    const inv = S.Matrix.Translation(new S.Vector([jx, jy, 0]).multiply(1 / 512)).multiply(scene.mat).inverse();
    result.inverse.push({ jx, jy, scale: 1 / 512, colmajor: inv.flatten() });
  }
  return result;
}

const out = { generator: 'tests/golden/make_fixtures.js', bundle_sha256: sha(src), scenes: {} };
out.scenes.C1 = capture('C1', sceneC1(false));
out.scenes.C1g = capture('C1g', sceneC1(true));
out.scenes.C3 = capture('C3', sceneC3());
out.scenes.C4 = capture('C4', sceneC4());
out.scenes.UI = capture('UI', sceneUI());
out.scenes.ALL = capture('ALL', sceneAllTextures());
out.scenes.AREA = capture('AREA', sceneAreaGood());
out.scenes.AREA0 = capture('AREA0', sceneAreaBlack());
out.scenes.N1 = capture('N1', sceneOneRoom());
out.scenes.N1S = capture('N1S', sceneOneSphere());
out.scenes.N0 = capture('N0', sceneEmpty());
out.scenes.BILERP = capture('BILERP', sceneBilerp());

// ---- reference picker selections (pickup.js) and the trace program's constants ------------------------------
out.pick = {};
for (const [name, mk, step] of [['C1', () => sceneC1(false), 32], ['C3', sceneC3, 32], ['UI', sceneUI, 32], ['C4', sceneC4, 16]])
  out.pick[name] = pickGrid(mk(), step);
out.program_constants = {};
for (const [name, mk] of [['C1', () => sceneC1(false)], ['C3', sceneC3], ['C4', sceneC4], ['ALL', sceneAllTextures]]) {
  const c0 = calls.length;
  new S.Renderer(canvas).update(mk());
  out.program_constants[name] = programConstants(shaderSources(c0));
}

// ---- box / triangle / mitchell tables through the same codegen ----------------------------------
out.filters = {};
for (const [fname, params] of [
  ['box', { r: 'vec2(1.5,1.5)' }],
  ['triangle', { r: 'vec2(2.0,2.0)' }],
  ['mitchell', { r: 'vec2(2.0,2.0)', b: '0.33', c: '0.33' }],
  ['sinc', { r: 'vec2(3.0,3.0)', tau: '3.0' }],
  ['gaussian', { r: 'vec2(1.5,2.5)', alpha: '0.25' }],
]) {
  const scene = sceneC1(false);
  scene.filter = fname;
  for (const k of Object.keys(params)) scene.filter.addParam(k, params[k]);
  const c = capture('f_' + fname, scene);
  out.filters[fname] = Object.assign({ params }, c.filter);
}

// ---- CPU intersect() distances (double precision, MINVALUE=1e-4, geometry.js:110-591) -----------
const u = xorshift32(0x1234);
const V = (a) => new S.Vector(a);
const M = new S.Matte(0.7), T = S.Color.WHITE;
const shapes = {
  cube: new S.Cube([1, 1, 1], [2, 2.5, 3], M, T),
  sphere: new S.Sphere([1.5, 1.5, 1.5], 0.75, M, T),
  cone: new S.Cone([1.5, 1, 1.5], 1.5, 0.6, M, T),
  cylinder: new S.Cylinder([1.5, 1, 1.5], 1.2, 0.5, M, T),
  disk: new S.Disk([1.5, 1.2, 1.5], 0.8, 0.2, M, T),
  hyperboloid: new S.Hyperboloid([1.5, 1, 1.5], [0.5, 0, 0], [0.25, 0.25, 1.0], M, T),
  paraboloid: new S.Paraboloid([1.5, 1, 1.5], 0, 1.2, 0.6, M, T),
};
out.intersect = {};
for (const [name, sh] of Object.entries(shapes)) {
  const rows = [];
  sh.gen(0);
  for (let k = 0; k < 64; k++) {
    // origins around the object, directions aimed near its centre so ~half the rays hit
    const o = [1.5 + (u() * 2 - 1) * 3, 1.5 + (u() * 2 - 1) * 3, 1.5 + (u() * 2 - 1) * 3];
    const tgt = [1.5 + (u() * 2 - 1) * 0.8, 1.6 + (u() * 2 - 1) * 0.8, 1.5 + (u() * 2 - 1) * 0.8];
    const d = [tgt[0] - o[0], tgt[1] - o[1], tgt[2] - o[2]];
    const t = sh.intersect({ origin: V(o), dir: V(d) });
    rows.push({ o, d, t });
  }
  out.intersect[name] = { row: f32list(sh.gen(0)), rays: rows };
}
out.host_constants = {
  matte_20: (() => { const m = new S.Matte(0.8, 20); return { A: m.A, B: m.B, row: f32list(m.gen()) }; })(),
  spot_40_10: (() => { const s = new S.SpotLight([0, 0, 0], 40, 10, [1, 1, 1]); return { cosTotalWidth: s.cosTotalWidth, cosFalloffStart: s.cosFalloffStart }; })(),
  hyperboloid: (() => { const h = shapes.hyperboloid; return { ah: h.ah, ch: h.ch }; })(),
  metal_default: f32list(new S.Metal(0, 0.01, 0.1).gen()),
};

process.stdout.write(JSON.stringify(out));
