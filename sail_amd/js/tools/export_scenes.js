'use strict';
// Serialises the frozen scenes through this build's Sail API (no device needed) to JSON:
// rows exactly as Renderer.update hands them to libsail_hip.so, the plugin lists, P*MV, eye and the
// display-filter configuration. Used by bench.py (sail_amd/scenes/frozen.json) and tests/test_js_host.py;
// exportScene is shared with tests/golden/make_fuzz_scenes.js.
// Usage: node sail_amd/js/tools/export_scenes.js [out.json]
const fs = require('fs');
const { SCENES } = require('../scenes');
const { filterConfig } = require('../src/filter');

function exportScene(scene) {
  const s = scene.serialize();
  const cfg = scene.tracerConfig();
  const f = scene.filter;
  const out = {
    n: s.n, tn: s.tn, ln: s.ln,
    objects: Array.from(s.objects), texparams: Array.from(s.texparams), lights: Array.from(s.lights),
    plugins: { shape: cfg.shape.map((p) => p.name), material: cfg.material.map((p) => p.name),
      texture: cfg.texture.map((p) => p.name), light: cfg.light.map((p) => p.name) },
    mvp_rowmajor: scene.mat.elements.map((r) => r.slice()),
    eye: scene.eye.elements.slice(),
    center: scene.camera.center.elements.slice(),
    filter: { name: f.name, params: Object.assign({}, f.params) },
  };
  const fc = filterConfig(f);
  if (fc.weights64) { out.filter.weights64 = fc.weights64; out.filter.radius = [fc.rx, fc.ry]; }
  return out;
}

if (require.main === module) {
  const result = {};
  for (const [name, make] of Object.entries(SCENES)) result[name] = exportScene(make());
  const text = JSON.stringify(result);
  if (process.argv[2]) fs.writeFileSync(process.argv[2], text);
  else process.stdout.write(text);
}
module.exports = { exportScene };
