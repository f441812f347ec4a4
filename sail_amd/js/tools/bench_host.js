'use strict';
// JS-host throughput through the N-API addon: the README Cornell box built with the Sail API (the C2 scene),
// rendered (a) the reference's way, one progressive sample per renderer.render(scene) call (tracer.js:92-101,
// one launch per call), and (b) with renderSamples(scene, spp) (one schedule, 32-sample launches).
// Wall time is taken in JS around the calls and a readPixels() that waits for the device; the kernel time
// comes from the library's HIP events (renderer.stats()).
//   node sail_amd/js/tools/bench_host.js [--width 1920] [--height 1080] [--bounces 8] [--frames 1024] [--spp 1024]
const path = require('path');
const Sail = require(path.join(__dirname, '..'));

function args() {
  const o = { width: 1920, height: 1080, bounces: 8, frames: 1024, spp: 1024 };
  const a = process.argv.slice(2);
  for (let i = 0; i < a.length; i += 2) o[a[i].replace(/^--/, '')] = parseInt(a[i + 1], 10);
  return o;
}

function cornell(o) {
  const scene = new Sail.Scene();
  scene.add(new Sail.Cube([2.13, 5.487, 2.27], [3.43, 5.488, 3.32], new Sail.Matte(0.7),
    Sail.Color.createTexture([0, 0, 0]), [8, 8, 8]));
  scene.add(new Sail.Cornellbox([0, 0, -7], [5.560, 5.488, 5.592]));
  scene.add(new Sail.Sphere([2, 1.25, 2.70], 1.2, new Sail.Mirror(1.0), Sail.Color.WHITE));
  const cam = new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]);
  cam.makePerspective(55, o.width / o.height, 1, 100);  // the C2 view (SURVEY §8(d)); the reference passes aspect 1
  scene.add(cam);
  return scene;
}

function run(o, perFrame) {
  const scene = cornell(o);
  const r = new Sail.Renderer({ width: o.width, height: o.height, maxBounces: o.bounces, deterministic: true,
    accumulation: 'sum', aov: false, display: false });
  r.update(scene);
  r.kernelReady(-1);  // the scene's run-time kernel, built in the background, serves every timed frame
  // warm-up (module load, first launches), then a fresh frame
  if (perFrame) for (let i = 0; i < 4; i++) r.render(scene); else r.renderSamples(scene, 32);
  r.readPixels();
  scene.sampleCount = 0;
  const n = perFrame ? o.frames : o.spp;
  const t0 = process.hrtime.bigint();
  if (perFrame) for (let i = 0; i < n; i++) r.render(scene); else r.renderSamples(scene, n);
  r.readPixels();
  const ms = Number(process.hrtime.bigint() - t0) / 1e6;
  const st = r.stats();
  r.destroy();
  const segs = o.width * o.height * n * o.bounces;
  return { mode: perFrame ? 'render() per frame' : 'renderSamples()', samples: n, wall_ms: +ms.toFixed(2),
    kernel_ms: +st.kernelMs.toFixed(2), launches: st.launches,
    msamples_per_s_wall: +(segs / (ms * 1e-3) / 1e6).toFixed(1) };
}

const o = args();
const res = [run(o, true), run(o, false)];
process.stdout.write(JSON.stringify({ workload: 'cornell_box_readme_C2 via the JS API', width: o.width,
  height: o.height, bounces: o.bounces, node: process.version, results: res }) + '\n');
