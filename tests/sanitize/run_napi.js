'use strict';
// Runs under the ASan/UBSan runtime with SAIL_NAPI = the instrumented addon (tests/test_sanitizers.py): the
// addon's host entry points with good and hostile arguments, the scene API serialising every frozen scene, and the
// fail-loudly paths that need a device. Prints one JSON line of results for the parent test to compare.
const Sail = require('../../sail_amd/js/index');
const native = require('../../sail_amd/js/src/native').load();
const scenes = require('../../sail_amd/js/scenes');

const out = {};
const mvp = native.camera([2.78, 2.73, -6], [2.78, 2.73, 2.79], [0, 1, 0], 55, 16 / 9, 1, 100);
out.camera = Array.from(mvp);
out.jitter = Array.from(native.jitterInverse(mvp, 0.25, -0.75, 1920, 1080));
const sch = native.schedule(mvp, 1920, 1080, 3, 17);
out.scheduleInv = Array.from(sch.inv);
out.scheduleSeeds = Array.from(sch.seeds);
out.tiles = Array.from(native.partitionTiles(1920, 1080, 3, 8));
// hostile arguments: every one must throw a JS error, none may touch memory it does not own
const bad = [
  () => native.camera([1, 2], [0, 0, 0], [0, 1, 0], 55, 1, 1, 100),
  () => native.jitterInverse(new Float64Array(3), 0, 0, 8, 8),
  () => native.schedule(new Float64Array(16), 8, 8, 0, -1),
  () => native.partitionTiles(0, 10, 0, 1),
  () => native.partitionTiles(10, 10, 5, 2),
  () => native.camera('x', [0, 0, 0], [0, 1, 0], 55, 1, 1, 100),
  () => native.schedule([1, 2, 3], 8, 8, 0, 1),
  () => native.setScene(null, new Float32Array(18), 1),
  () => native.create(-5, 8, 0, 0),
  () => native.create(8, 8, 0, 0),                   // no device here
  () => native.createMulti(8, 8, Int32Array.from([0, 0]), 0),
  () => new Sail.Renderer({ width: 8, height: 8 }),
];
out.badThrown = bad.map((f) => { try { f(); return false; } catch (e) { return e instanceof Error; } });
// the scene API over every frozen scene (pure JS, serialisation as the reference uploads it)
out.rows = {};
for (const [name, make] of Object.entries(scenes.SCENES)) {
  const sc = make();
  const s = sc.serialize ? sc.serialize() : null;
  if (s) out.rows[name] = { n: s.n, tn: s.tn, ln: s.ln, sum: Array.from(s.objects).reduce((a, b) => a + b, 0) };
}
process.stdout.write(JSON.stringify(out) + '\n');
