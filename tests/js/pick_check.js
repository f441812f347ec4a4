'use strict';
// Drives Sail.Control / Pickup against a live Renderer (GPU): picks a grid of pixels, then drags the mirror
// sphere of the README Cornell box. Writes the rays it cast (as f32, what crossed the C ABI), the picked object
// rows and the drag result for tests/test_js_host.py to check against the oracle. argv: out.json
const fs = require('fs');
const Sail = require('../../sail_amd/js');
const { Pickup } = require('../../sail_amd/js/src/control');
const { SCENES } = require('../../sail_amd/js/scenes');
const out = process.argv[2];
const W = 64, H = 48;
const scene = SCENES.C1();
const r = new Sail.Renderer({ width: W, height: H, deterministic: true, maxBounces: 4, display: false });
Sail.Control.update(scene);
r.update(scene);
const pk = new Pickup(scene);
const rays = [], picked = [];
for (let y = 0; y < H; y += 3) {
  for (let x = 0; x < W; x += 3) {
    const ray = pk._ray(x, y);
    rays.push(...Float32Array.from([...ray.origin.elements, ...ray.dir.elements]));
    const hit = pk.pick(x, y);
    picked.push(hit ? scene.objects.indexOf(scene.select) : -1);
  }
}
// click the sphere (object row 2) and drag it 6 pixels to the right
let sx = -1, sy = -1;
for (let y = 0; y < H && sx < 0; y++) for (let x = 0; x < W; x++) {
  const ray = pk._ray(x, y);
  if (r.pick(ray.origin.elements, ray.dir.elements).index === 2) { sx = x; sy = y; break; }
}
scene.select = null;
Sail.Control.mousedown(sx, sy);            // no selection yet: picks the sphere
const selected = scene.objects.indexOf(scene.select);
const before = scene.select.c.elements.slice();
Sail.Control.mouseup(sx, sy);
Sail.Control.mousedown(sx, sy);            // selection present: starts a drag on its bounding box
const began = scene.moving;
Sail.Control.mousemove(sx + 6, sy);
r.render(scene);                           // scene.moving: sampleCount = 0 and the object rows are re-uploaded
Sail.Control.mouseup(sx + 6, sy);
r.render(scene);
const after = scene.select.c.elements.slice();
fs.writeFileSync(out, JSON.stringify({ rays, picked, selected, began, before, after, sampleCount: scene.sampleCount }));
r.destroy();
