'use strict';
// Renders a frozen (or random) scene through Sail.Renderer -> N-API -> libsail_hip.so and writes the raw accumulator
// (and the canvas pixels) for tests/test_js_host.py to compare with the CPU oracle. Needs an MI355X.
// argv: scene W H spp bounces mode(sum|mix) api(samples|frames|progressive|resume) out_prefix [filter [filter-r]]
// env SAIL_TEST_DEVICES=0,0,0: a multi-device Renderer ({devices: [...]}); progressive = half the samples as
// frames, a display pass (reduces the devices' frames), the other half, then the readback
const fs = require('fs');
const Sail = require('../../sail_amd/js');
const { SCENES } = require('../../sail_amd/js/scenes');
const [name, W, H, spp, B, mode, api, out, filter, filterR] = process.argv.slice(2);
// fuzz:F07 / fuzz:E03: a seeded random / edge scene of tests/golden/make_fuzz_scenes.js, built here by the Sail API
const fuzz = name.startsWith('fuzz:') ? require('../golden/make_fuzz_scenes') : null;
const scene = fuzz ? (name[5] === 'E' ? fuzz.makeEdgeScene : fuzz.makeScene)(+name.slice(6) + 1) : SCENES[name]();
if (filter) {  // the reference's scene.filter = name; scene.filter.addParam('r', ...) flow
  scene.filter = filter;
  if (filterR) scene.filter.addParam('r', filterR);
}
const devices = process.env.SAIL_TEST_DEVICES ? process.env.SAIL_TEST_DEVICES.split(',').map(Number) : undefined;
const opts = { width: +W, height: +H, deterministic: true, accumulation: mode, maxBounces: +B, display: false, devices };
let r = new Sail.Renderer(opts);
r.update(scene);
if (api === 'samples') r.renderSamples(scene, +spp);
else if (api === 'resume') {  // half the samples as frames, save(), a NEW renderer, load(), the other half
  const half = Math.floor(+spp / 2);
  for (let i = 0; i < half; i++) r.render(scene);
  const ck = r.save();
  r.destroy();
  r = new Sail.Renderer(opts);
  r.update(scene);
  r.load(ck, scene);
  for (let i = half; i < +spp; i++) r.render(scene);
}
else if (api === 'progressive') {
  const half = Math.floor(+spp / 2);
  for (let i = 0; i < half; i++) r.render(scene);
  r.image();
  for (let i = half; i < +spp; i++) r.render(scene);
} else for (let i = 0; i < +spp; i++) r.render(scene);
fs.writeFileSync(out + '.accum.f32', Buffer.from(r.readAccum().buffer));
fs.writeFileSync(out + '.rgba8', Buffer.from(r.image().buffer));
if (filter) {
  const rb = r.lib.readback(r.ctx, true);
  fs.writeFileSync(out + '.mean.f32', Buffer.from(rb.rgba.buffer));
  fs.writeFileSync(out + '.normal.f32', Buffer.from(rb.normal.buffer));
  fs.writeFileSync(out + '.position.f32', Buffer.from(rb.position.buffer));
}
const st = r.stats();
fs.writeFileSync(out + '.stats.json', JSON.stringify(st));
r.destroy();
