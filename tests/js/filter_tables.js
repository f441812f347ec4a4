'use strict';
// prints the window-weight tables this build's JS host computes for the given filter params (JSON on argv)
const { PluginParams } = require('../../sail_amd/js/src/scene');
const { filterConfig } = require('../../sail_amd/js/src/filter');
const spec = JSON.parse(process.argv[2]);
const out = {};
for (const [name, params] of Object.entries(spec)) {
  const pp = new PluginParams(name);
  for (const [k, v] of Object.entries(params)) pp.addParam(k, v);
  const fc = filterConfig(pp);
  out[name] = { weights64: fc.weights64, radius: [fc.rx, fc.ry] };
}
process.stdout.write(JSON.stringify(out));
