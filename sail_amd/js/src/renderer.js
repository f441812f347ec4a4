'use strict';
// Sail.Renderer over libsail_hip.so (through the N-API addon) in place of the WebGL2 programs.
//   new Renderer(canvas | {width, height, device, devices, ...})   src/core/renderer.js:9-39
//     devices: N (GPUs 0..N-1) or an array of ordinals -> one multi-device context (sail_create_multi): the
//     frame's tiles are dealt across the GPUs and summed into GPU 0 (RCCL) before each display / readback
//   renderer.update(scene)        -> Tracer.update (tracer.js:42-90): rows + plugin set -> sail_set_scene
//   renderer.updateObjects(scene) -> Tracer.updateObjects (tracer.js:25-40) -> sail_update_objects
//   renderer.render(scene)        -> Tracer.render (tracer.js:92-101): one progressive sample with a
//                                    jittered inverse camera matrix and a time seed -> sail_render, then the
//                                    display filter (renderer.js:63) -> sail_filter, painted to the canvas
// Extensions (same API object): renderSamples(scene, spp) runs a whole deterministic sample schedule in
// one call; readPixels() / readAOV() / image() read the float frame back (the reference never reads back).
const native = require('./native');
const { filterConfig } = require('./filter');

const MAXBOUNCES = 5;  // define.glsl:6
const ACCUM = { sum: 0, mix: 1, compat8: 2 };
const SHAPE_ID = { cube: 1, sphere: 2, rectangle: 3, cone: 4, cylinder: 5, disk: 6, hyperboloid: 7, paraboloid: 8, cornellbox: 9 };
const MAT_ID = { matte: 1, mirror: 2, metal: 3, glass: 4 };
const TEX_ID = { checkerboard: 5, checkerboard2: 7, bilerp: 8, mixf: 9, scale: 10, uvf: 11 };
const LIGHT_ID = { area: 0, point: 1, spot: 2 };

function masksOf(cfg) {
  const m = (list, table) => list.reduce((acc, p) => acc | (1 << table[p.name]), 0) >>> 0;
  return [m(cfg.shape, SHAPE_ID), m(cfg.material, MAT_ID), m(cfg.texture, TEX_ID), m(cfg.light, LIGHT_ID)];
}
function rowMajor(mat) {
  const out = new Float64Array(16);
  for (let i = 0; i < 4; i++) for (let j = 0; j < 4; j++) out[i * 4 + j] = mat.elements[i][j];
  return out;
}

class Renderer {
  constructor(target = {}, options = {}) {
    const isCanvas = target && typeof target.getContext === 'function';
    const opts = isCanvas ? options : Object.assign({}, target, options);
    this.canvas = isCanvas ? target : null;
    this.width = opts.width || (this.canvas && this.canvas.width) || 512;    // webgl.js:24 (512 x 512)
    this.height = opts.height || (this.canvas && this.canvas.height) || 512;
    this.device = opts.device === undefined ? -1 : opts.device;
    this.devices = opts.devices === undefined ? null
      : (Array.isArray(opts.devices) ? opts.devices.slice() : Array.from({ length: opts.devices }, (_, i) => i));
    if (this.devices && this.devices.length < 1) throw new Error('Renderer: devices must name at least one GPU');
    this.maxBounces = opts.maxBounces || MAXBOUNCES;
    this.deterministic = !!opts.deterministic;  // frozen schedule (SURVEY §8(d)) instead of Math.random + clock
    // a sample split sums every device's own samples, so it accumulates sums (a running mean cannot be split)
    this.accumulation = opts.accumulation || (opts.partition === 'samples' ? 'sum' : 'mix');
    if (!(this.accumulation in ACCUM)) throw new Error(`Renderer: unknown accumulation '${this.accumulation}'`);
    if (opts.partition !== undefined && opts.partition !== 'tiles' && opts.partition !== 'samples')
      throw new Error(`Renderer: unknown partition '${opts.partition}' (tiles | samples)`);
    if (opts.partition === 'samples' && this.accumulation !== 'sum' && this.devices && this.devices.length > 1)
      throw new Error("Renderer: partition 'samples' needs accumulation 'sum' (a running mean cannot be split by samples)");
    this.aov = opts.aov !== false;
    this.display = opts.display === undefined ? !!this.canvas : !!opts.display;
    this.lib = native.load();
    const flags = (this.aov ? 1 : 0) | 2;
    this.ctx = this.devices ? this.lib.createMulti(this.width, this.height, Int32Array.from(this.devices), flags)
      : this.lib.create(this.width, this.height, this.device, flags);
    if (opts.partition === 'samples') this.lib.setPartition(this.ctx, 0, 1, 1);
    this.lib.setAccumMode(this.ctx, ACCUM[this.accumulation]);
    // update() links the scene's program in the background (a hipRTC build takes seconds, the reference's GL link
    // milliseconds: renderer.js:45-52); until it is loaded render() uses the precompiled kernel of the scene's plugin
    // set, with identical frames. waitKernel (ms, -1 = until built) makes each launch wait for it instead [0].
    if (opts.waitKernel !== undefined) this.lib.setDebug(this.ctx, 10, opts.waitKernel);
    this.timeStart = Date.now();
    this.filter = filterConfig({ name: 'color', params: {} });
    this.pixels = null;
    this.n = 0;
  }

  update(scene) {
    // the picker (Control / Pickup) finds the renderer that holds this scene on the device
    Object.defineProperty(scene, 'renderer', { value: this, writable: true, configurable: true, enumerable: false });
    this.filter = filterConfig(scene.rendererConfig().filter);
    const s = scene.serialize();
    this.lib.setScene(this.ctx, s.objects, s.n, s.texparams, s.tn, s.lights, s.ln, masksOf(scene.tracerConfig()));
    this.n = s.n;
    scene.sampleCount = 0;
  }

  updateObjects(scene) {
    this.lib.updateObjects(this.ctx, scene.serializeObjects(), this.n);
  }

  _mvp(scene) { return rowMajor(scene.mat); }

  render(scene) {
    if (scene.moving) {
      scene.sampleCount = 0;
      this.updateObjects(scene);
    }
    if (scene.sampleCount === 0) this.lib.reset(this.ctx);  // textureWeight 0: the frame restarts
    const k = scene.sampleCount++;
    const mvp = this._mvp(scene);
    const eye = Float32Array.from(scene.eye.elements);
    let inv, seed;
    if (this.deterministic) {
      const sch = this.lib.schedule(mvp, this.width, this.height, k, 1);
      inv = sch.inv; seed = sch.seeds[0];
    } else {
      inv = this.lib.jitterInverse(mvp, Math.random() * 2 - 1, Math.random() * 2 - 1, this.width, this.height);
      seed = (Date.now() - this.timeStart) * 0.001;
    }
    this.lib.render(this.ctx, inv, eye, seed, this.maxBounces);
    if (this.display) this.present();
  }

  // many samples in one launch sequence, deterministic schedule k0 .. k0+spp-1
  renderSamples(scene, spp) {
    if (scene.moving) { scene.sampleCount = 0; this.updateObjects(scene); }
    if (scene.sampleCount === 0) this.lib.reset(this.ctx);
    const sch = this.lib.schedule(this._mvp(scene), this.width, this.height, scene.sampleCount, spp);
    this.lib.renderSchedule(this.ctx, sch.inv, sch.seeds, Float32Array.from(scene.eye.elements), this.maxBounces);
    scene.sampleCount += spp;
    if (this.display) this.present();
  }

  // the display pass: pixelFilter over the accumulated frame -> RGBA8 (row 0 = bottom, GL order)
  image() {
    const f = this.filter;
    if (f.aov && !this.aov) throw new Error('this display filter reads the AOVs: create the Renderer with aov: true');
    return this.lib.filter(this.ctx, f.kind, f.weights, f.rx, f.ry, f.gamma).rgba8;
  }

  present() {
    this.pixels = this.image();
    if (this.canvas) {
      const g = this.canvas.getContext('2d');
      if (g && typeof g.createImageData === 'function') {
        const img = g.createImageData(this.width, this.height);
        const rowBytes = this.width * 4;
        for (let y = 0; y < this.height; y++) {  // GL rows are bottom-up, canvas rows top-down
          img.data.set(this.pixels.subarray((this.height - 1 - y) * rowBytes, (this.height - y) * rowBytes), y * rowBytes);
        }
        g.putImageData(img, 0, 0);
      }
    }
    return this.pixels;
  }

  // Pickup.pick on the GPU: the trace kernel's primitive sweep for one ray -> {index (object row, -1 = miss), t}
  pick(origin, dir) {
    const rays = Float32Array.from([...origin, ...dir]);
    const r = this.lib.pick(this.ctx, rays);
    return { index: r.index[0], t: r.t[0] };
  }
  // many rays at once: Float32Array of 6 floats per ray -> {index: Int32Array, t: Float32Array}
  pickRays(rays) { return this.lib.pick(this.ctx, rays); }

  // checkpoint of a progressive render: {k: samples so far, parts: [Float32Array accumulator per device],
  // width, height}; load() into a renderer of the same size, scene, devices and accumulation continues it bit for bit
  save() {
    const ck = this.lib.saveAccum(this.ctx);
    return { k: ck.k, parts: ck.parts, width: this.width, height: this.height, accumulation: this.accumulation };
  }
  // Order: update(scene) first (it resets the accumulation), then load(ckpt, scene): the scene is required, because
  // its sampleCount must become k, or the next render() would restart the accumulation and drop the loaded samples.
  load(ckpt, scene) {
    if (!scene) throw new Error('Renderer.load(ckpt, scene): the scene is required (its sampleCount continues at ckpt.k)');
    if (ckpt.width !== this.width || ckpt.height !== this.height) throw new Error('Renderer.load: checkpoint size differs');
    if (ckpt.accumulation && ckpt.accumulation !== this.accumulation) throw new Error('Renderer.load: accumulation mode differs');
    if (ckpt.frame) this.lib.loadAccum(this.ctx, -1, ckpt.frame, ckpt.k);
    else ckpt.parts.forEach((p, i) => this.lib.loadAccum(this.ctx, i, p, ckpt.k));
    scene.sampleCount = ckpt.k;  // the next render() draws sample k (its jitter and seed)
  }

  readPixels() { return this.lib.readback(this.ctx, false).rgba; }
  readAccum() { return this.lib.readAccum(this.ctx); }
  readAOV() { const r = this.lib.readback(this.ctx, true); return { normal: r.normal, position: r.position }; }
  stats() { return this.lib.stats(this.ctx); }
  // whether the scene's run-time compiled kernel serves the next render (waiting up to timeoutMs for its build)
  kernelReady(timeoutMs = -1) { return this.lib.kernelReady(this.ctx, timeoutMs); }
  kernelInfo() { return this.lib.kernelInfo(this.ctx); }
  destroy() { if (this.ctx) { this.lib.destroy(this.ctx); this.ctx = null; } }
}

module.exports = { Renderer, masksOf, MAXBOUNCES };
