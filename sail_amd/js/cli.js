#!/usr/bin/env node
'use strict';
// Headless Sail: run a scene script the way the reference's editor does (ui/ui.js:47-52: eval the code, which
// assigns `scene`, then Renderer.update(scene)), render N samples on the GPU and write the frame to disk.
//
//   node sail_amd/js/cli.js scene.js [--width 512] [--height 512] [--spp 64] [--bounces 5] [--device -1]
//        [--filter <name>] [--filter-r 'vec2(2.0,2.0)'] [--gamma 2.2] [--deterministic]
//        [--png out.png] [--pfm out.pfm] [--exr out.exr] [--stats]
//
// The script sees `Sail` (the full API) and must assign `scene` (a Sail.Scene with a camera), exactly as the
// editor text does. --filter overrides scene.filter for the PNG; the PFM and EXR are always the unfiltered mean image.
const fs = require('fs');
const path = require('path');
const vm = require('vm');
const Sail = require('./index');
const { writePFM, writePNG, writeEXR } = require('./src/image');

function parse(argv) {
  const opt = { width: 512, height: 512, spp: 64, bounces: 5, device: -1, deterministic: false, stats: false };
  const rest = [];
  for (let i = 0; i < argv.length; i++) {
    const a = argv[i];
    const val = () => { if (i + 1 >= argv.length) throw new Error(`${a} needs a value`); return argv[++i]; };
    switch (a) {
      case '--width': opt.width = parseInt(val(), 10); break;
      case '--height': opt.height = parseInt(val(), 10); break;
      case '--spp': opt.spp = parseInt(val(), 10); break;
      case '--bounces': opt.bounces = parseInt(val(), 10); break;
      case '--device': opt.device = parseInt(val(), 10); break;
      case '--filter': opt.filter = val(); break;
      case '--filter-r': opt.filterR = val(); break;
      case '--gamma': opt.gamma = val(); break;
      case '--png': opt.png = val(); break;
      case '--pfm': opt.pfm = val(); break;
      case '--exr': opt.exr = val(); break;
      case '--deterministic': opt.deterministic = true; break;
      case '--stats': opt.stats = true; break;
      case '-h': case '--help': opt.help = true; break;
      default:
        if (a.startsWith('--')) throw new Error(`unknown option ${a}`);
        rest.push(a);
    }
  }
  opt.script = rest[0];
  return opt;
}

function loadScene(file) {
  const code = fs.readFileSync(file, 'utf8');
  const context = { Sail, console, Math, scene: undefined };
  vm.createContext(context);
  vm.runInContext(code, context, { filename: path.basename(file) });
  if (!context.scene || !(context.scene instanceof Sail.Scene)) throw new Error(`${file} did not assign a Sail.Scene to \`scene\``);
  return context.scene;
}

function main() {
  const opt = parse(process.argv.slice(2));
  if (opt.help || !opt.script) {
    process.stdout.write(fs.readFileSync(__filename, 'utf8').split('\n').slice(2, 11).map((l) => l.replace(/^\/\/ ?/, '')).join('\n') + '\n');
    return opt.help ? 0 : 2;
  }
  const scene = loadScene(opt.script);
  if (opt.filter) scene.filter = opt.filter;
  if (opt.filterR) scene.filter.addParam('r', opt.filterR);
  if (opt.gamma) scene.filter.addParam('c', opt.gamma);
  const needAov = ['wavelet', 'normal', 'position'].includes(scene.filter.name);
  const r = new Sail.Renderer({ width: opt.width, height: opt.height, device: opt.device, maxBounces: opt.bounces,
    deterministic: opt.deterministic, accumulation: 'sum', aov: needAov, display: false });
  r.update(scene);
  const t0 = process.hrtime.bigint();
  r.renderSamples(scene, opt.spp);
  const mean = r.readPixels();
  const ms = Number(process.hrtime.bigint() - t0) / 1e6;
  if (opt.pfm) writePFM(opt.pfm, opt.width, opt.height, mean);
  if (opt.exr) writeEXR(opt.exr, opt.width, opt.height, mean);
  if (opt.png) writePNG(opt.png, opt.width, opt.height, r.image());
  if (opt.stats) {
    const st = r.stats();
    process.stdout.write(JSON.stringify({ width: opt.width, height: opt.height, spp: opt.spp, bounces: opt.bounces,
      ms, segments: st.segments, kernelMs: st.kernelMs, filter: scene.filter.name }) + '\n');
  }
  r.destroy();
  return 0;
}

try {
  process.exitCode = main();
} catch (e) {
  process.stderr.write(`sail: ${e.message}\n`);
  process.exitCode = 1;
}
