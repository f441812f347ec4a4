'use strict';
// Loads the N-API addon (sail_amd/js/native/build/sail_napi.node -> libsail_hip.so). There is no software
// fallback: without the addon or a HIP device the Renderer throws, like the reference's alert() path.
const path = require('path');

let cached = null;
function load() {
  if (cached) return cached;
  const p = process.env.SAIL_NAPI || path.join(__dirname, '..', 'native', 'build', 'sail_napi.node');
  try {
    cached = require(p);
  } catch (e) {
    throw new Error(`Sail: the MI355X addon is not built (${p}): ${e.message}. Run sail_amd/js/native/build.sh`);
  }
  return cached;
}
module.exports = { load };
