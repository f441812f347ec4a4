'use strict';
// Renderer.update on a scene whose run-time kernel no cache holds (the README Cornell box with its objects added in
// reverse order: a row specialisation of its own): update() must return at once while the kernel builds in the
// background (the reference links its program inside Renderer.update in milliseconds, src/core/renderer.js:45-52);
// frames render on the precompiled kernel until the run-time one is loaded, then on it. Writes the accumulator, the
// scene rows (for the oracle) and the timings. Run with XDG_CACHE_HOME pointing at an empty directory for a cold
// user cache; a second run with the same directory measures the warm one. Needs an MI355X.
// argv: out_prefix W H spp bounces
const fs = require('fs');
const { performance } = require('perf_hooks');
const Sail = require('../../sail_amd/js');
const [out, W, H, spp, B] = process.argv.slice(2);
const scene = new Sail.Scene();
scene.add(new Sail.Sphere([2, 1.25, 2.70], 1.2, new Sail.Mirror(1.0), Sail.Color.WHITE));
scene.add(new Sail.Cornellbox([0, 0, -7], [5.560, 5.488, 5.592]));
scene.add(new Sail.Cube([2.13, 5.487, 2.27], [3.43, 5.488, 3.32], new Sail.Matte(0.7), Sail.Color.createTexture([0, 0, 0]), [8, 8, 8]));
scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
const r = new Sail.Renderer({ width: +W, height: +H, deterministic: true, accumulation: 'sum', maxBounces: +B,
  display: false, aov: false });
const t0 = performance.now();
r.update(scene);
const updateMs = performance.now() - t0;
const afterUpdate = r.kernelInfo();
const half = Math.floor(+spp / 2);
for (let i = 0; i < half; i++) r.render(scene);
r.stats();  // launches the queued frames now
const first = r.kernelInfo().name;
const t1 = performance.now();
const ready = r.kernelReady(-1);
const waitMs = performance.now() - t1;
for (let i = half; i < +spp; i++) r.render(scene);
const acc = r.readAccum();
const info = r.kernelInfo();
fs.writeFileSync(out + '.accum.f32', Buffer.from(acc.buffer));
const s = scene.serialize();
const cfg = scene.tracerConfig();
fs.writeFileSync(out + '.json', JSON.stringify({
  scene: { n: s.n, tn: s.tn, ln: s.ln, objects: Array.from(s.objects), texparams: Array.from(s.texparams),
    lights: Array.from(s.lights), eye: scene.eye.elements.slice(), mvp_rowmajor: scene.mat.elements.map((x) => x.slice()),
    plugins: { shape: cfg.shape.map((p) => p.name), material: cfg.material.map((p) => p.name),
      texture: cfg.texture.map((p) => p.name), light: cfg.light.map((p) => p.name) } },
  update_ms: updateMs, state_after_update: afterUpdate.jitState, first_kernel: first, wait_ms: waitMs, ready,
  last_kernel: info.name, from_cache: info.jitFromCache, compile_ms: info.jitCompileMs }));
r.destroy();
