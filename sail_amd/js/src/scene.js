'use strict';
// The Sail scene API (index.js:15-46): geometry, materials, textures, lights, camera, Color, Scene.
// Constructors, defaults and gen() row layouts follow src/scene/*.js so that the rows handed to
// libsail_hip.so equal what the reference uploads as R32F textures (tracer.js:42-90; SURVEY Appendix A).
const { Vector, Matrix } = require('./la');

const OBJECTS_LENGTH = 18, TEXPARAMS_LENGTH = 16, LIGHTS_LENGTH = 18;  // webgl.js:137-139

function pad(row, len) { while (row.length < len) row.push(0); return row; }
function vec(v) { return v instanceof Vector ? v : new Vector(v); }
function el(v, i) { return v instanceof Vector ? v.e(i) : v[i - 1]; }

// ---- generator.js:4-25 PluginParams (the one-decimal getParam regex is part of the behaviour) -----------
class PluginParams {
  constructor(name) { this.name = name; this.params = {}; }
  addParam(name, value) { this.params[name] = value; }
  getParam(name) {
    const m = String(this.params[name]).match(/-?\d+\.\d+?/g);
    return m ? m.map(parseFloat) : m;
  }
  getParamName(name, generatorName) { return `${generatorName}_${this.name}_${name}`.toUpperCase(); }
}

// ---- materials (src/scene/material.js) ------------------------------------------------------------------
class Material {
  get pluginName() { return this._pluginName; }
  set pluginName(n) {}
  gen(data) { return pad(data, TEXPARAMS_LENGTH); }
}
class Matte extends Material {
  constructor(kd = 1, sigma = 0) {
    super();
    if (kd <= 0) kd = 1;
    this.kd = kd; this.sigma = sigma; this.A = 0; this.B = 0;
    this._pluginName = 'matte';
    if (this.sigma !== 0) {  // Oren-Nayar A/B (material.js:28-34)
      const s = sigma * Math.PI / 180, s2 = s * s;
      this.A = 1.0 - (s2 / (2.0 * (s2 + 0.33)));
      this.B = 0.45 * s2 / (s2 + 0.09);
    }
  }
  gen() { return super.gen([1, this.kd, this.sigma, this.A, this.B]); }
}
class Mirror extends Material {
  constructor(kr = 1.0) { super(); if (kr <= 0) kr = 0.5; this.kr = kr; this._pluginName = 'mirror'; }
  gen() { return super.gen([2, this.kr]); }
}
class Metal extends Material {
  constructor(roughness = 0.01, uroughness = 0, vroughness = 0, eta, k) {
    super();
    this.uroughness = uroughness === 0 ? roughness : uroughness;
    this.vroughness = vroughness === 0 ? roughness : vroughness;
    this.eta = eta ? vec(eta) : new Vector([9.530817595377695, 6.635831967341377, 4.47513354108444]);
    this.k = k ? vec(k) : new Vector([13.028170336874789, 8.112634272577575, 5.502811570992323]);
    this._pluginName = 'metal';
  }
  gen() {
    return super.gen([3, this.uroughness, this.vroughness, this.eta.e(1), this.eta.e(2), this.eta.e(3),
      this.k.e(1), this.k.e(2), this.k.e(3)]);
  }
}
class Glass extends Material {
  constructor(kr = 1, kt = 1, eta, uroughness = 0, vroughness = 0) {
    super();
    this.kr = kr; this.kt = kt; this.eta = eta; this.uroughness = uroughness; this.vroughness = vroughness;
    this._pluginName = 'glass';
  }
  gen() { return super.gen([4, this.kr, this.kt, this.eta, this.uroughness, this.vroughness]); }
}

// ---- textures (src/scene/texture.js) ------------------------------------------------------------------------
class Texture {
  get pluginName() { return this._pluginName; }
  set pluginName(n) {}
  gen(data) { return pad(data, TEXPARAMS_LENGTH); }
}
class UniformColor extends Texture {
  constructor(color) { super(); this.color = vec(color); this._pluginName = undefined; }  // inlined by the tracer
  gen() { return super.gen([0, this.color.e(1), this.color.e(2), this.color.e(3)]); }
}
class Checkerboard extends Texture {
  constructor(size = 0.1, lineWidth = 0.01) {
    super();
    if (size <= 0) size = 0.3;
    if (lineWidth < 0) lineWidth = 0.03;
    this.size = size; this.lineWidth = lineWidth; this._pluginName = 'checkerboard';
  }
  gen() { return super.gen([5, this.size, this.lineWidth]); }
}
class Checkerboard2 extends Texture {
  constructor(color1 = [1, 1, 1], color2 = [0, 0, 0], size = 0.1) {
    super(); this.color1 = vec(color1); this.color2 = vec(color2); this.size = size; this._pluginName = 'checkerboard2';
  }
  gen() { return super.gen([7, ...this.color1.elements, ...this.color2.elements, this.size]); }
}
class Bilerp extends Texture {
  constructor(c00, c01, c10, c11) {
    super();
    this.color00 = vec(c00); this.color01 = vec(c01); this.color10 = vec(c10); this.color11 = vec(c11);
    this._pluginName = 'bilerp';
  }
  gen() {
    return super.gen([8, ...this.color00.elements, ...this.color01.elements, ...this.color10.elements, ...this.color11.elements]);
  }
}
class Mix extends Texture {
  constructor(color1, color2, amount) { super(); this.color1 = vec(color1); this.color2 = vec(color2); this.amount = amount; this._pluginName = 'mixf'; }
  gen() { return super.gen([9, ...this.color1.elements, ...this.color2.elements, this.amount]); }
}
class Scale extends Texture {
  constructor(color1, color2) { super(); this.color1 = vec(color1); this.color2 = vec(color2); this._pluginName = 'scale'; }
  gen() { return super.gen([10, ...this.color1.elements, ...this.color2.elements]); }
}
class UV extends Texture {
  constructor() { super(); this._pluginName = 'uvf'; }
  gen() { return super.gen([11]); }
}

class Color {  // src/core/color.js
  static createTexture(color) { return new UniformColor(Array.isArray(color) ? color : color.flatten()); }
  static get BLACK() { return new UniformColor([0, 0, 0]); }
  static get WHITE() { return new UniformColor([1, 1, 1]); }
  static get GREEN() { return new UniformColor([0, 1, 0]); }
  static get BLUE() { return new UniformColor([0, 0, 1]); }
  static get RED() { return new UniformColor([1, 0, 0]); }
}

// ---- geometry (src/scene/geometry.js gen(); row = [id, params..., reverseNormal, mat, tex, emission]) ----
class Object3D {
  constructor(material, texture, emission = [0, 0, 0], reverseNormal = false) {
    this.material = material;
    this.texture = texture;
    this.emission = vec(emission);
    this.reverseNormal = reverseNormal ? 1 : 0;
    this.texparamsID = 0;
    this.temporaryTranslation = Vector.Zero(3);
    this.light = !this.emission.eql([0, 0, 0]);
    this._pluginName = '';
  }
  get pluginName() { return this._pluginName; }
  set pluginName(n) {}
  boundbox() { return false; }
  temporaryTranslate(v) { this.temporaryTranslation = vec(v); }
  translate() { this.temporaryTranslation = Vector.Zero(3); }
  genTexparams() { return [...this.material.gen(), ...this.texture.gen()]; }
  _row(params, texparamID) {
    this.texparamID = texparamID;
    const row = params.concat([this.reverseNormal, texparamID, texparamID + 1, ...this.emission.elements]);
    return pad(row, OBJECTS_LENGTH);
  }
}
class Cube extends Object3D {
  constructor(min, max, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.min = vec(min); this.max = vec(max); this._pluginName = 'cube';
  }
  boundbox() { return { min: this.min, max: this.max }; }
  translate() { this.min = this.min.add(this.temporaryTranslation); this.max = this.max.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) { this.translate(); return this._row([1, ...this.min.elements, ...this.max.elements], id); }
}
class Sphere extends Object3D {
  constructor(c, r, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.c = vec(c); this.r = r; this._pluginName = 'sphere';
  }
  boundbox() { const r = new Vector([this.r, this.r, this.r]); return { min: this.c.subtract(r), max: this.c.add(r) }; }
  translate() { this.c = this.c.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) { this.translate(); return this._row([2, ...this.c.elements, this.r], id); }
}
class Rectangle extends Object3D {
  constructor(min, max, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.min = vec(min); this.max = vec(max); this._pluginName = 'rectangle';
  }
  boundbox() {
    const min = this.min.dup(), max = this.max.dup();
    for (let a = 0; a < 3; a++) if (max.elements[a] === min.elements[a]) { max.elements[a] += 0.05; min.elements[a] -= 0.05; }
    return { min, max };
  }
  translate() { this.min = this.min.add(this.temporaryTranslation); this.max = this.max.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) { this.translate(); return this._row([3, ...this.min.elements, ...this.max.elements], id); }
}
class Cone extends Object3D {
  constructor(position, height, radius, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.position = vec(position); this.height = height; this.radius = radius; this._pluginName = 'cone';
  }
  boundbox() {
    return { min: this.position.subtract([this.radius, 0, this.radius]), max: this.position.add([this.radius, this.height, this.radius]) };
  }
  translate() { this.position = this.position.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) { this.translate(); return this._row([4, ...this.position.elements, this.height, this.radius], id); }
}
class Cylinder extends Object3D {
  constructor(position, height, radius, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.position = vec(position); this.height = height; this.radius = radius; this._pluginName = 'cylinder';
  }
  boundbox() {
    return { min: this.position.subtract([this.radius, 0, this.radius]), max: this.position.add([this.radius, this.height, this.radius]) };
  }
  translate() { this.position = this.position.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) { this.translate(); return this._row([5, ...this.position.elements, this.height, this.radius], id); }
}
class Disk extends Object3D {
  constructor(position, radius, innerRadius, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.position = vec(position); this.radius = radius; this.innerRadius = innerRadius; this._pluginName = 'disk';
  }
  boundbox() {
    return { min: this.position.subtract([this.radius, 0.05, this.radius]), max: this.position.add([this.radius, 0.05, this.radius]) };
  }
  translate() { this.position = this.position.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) { this.translate(); return this._row([6, ...this.position.elements, this.radius, this.innerRadius], id); }
}
class Hyperboloid extends Object3D {
  constructor(position, p1, p2, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.position = vec(position); this.p1 = vec(p1); this.p2 = vec(p2);
    const r1 = Math.sqrt(el(p1, 1) * el(p1, 1) + el(p1, 2) * el(p1, 2));
    const r2 = Math.sqrt(el(p2, 1) * el(p2, 1) + el(p2, 2) * el(p2, 2));
    this.rMax = Math.max(r1, r2);
    this.zMin = Math.min(el(p1, 3), el(p2, 3));
    this.zMax = Math.max(el(p1, 3), el(p2, 3));
    this._pluginName = 'hyperboloid';
    // ah/ch of ah(x^2+y^2) - ch z^2 = 1 through p2 and an extrapolated point (geometry.js:466-486). The
    // reference loops until ah is finite and can spin forever; this build stops after 20 tries and throws.
    if (this.p2.e(3) === 0) { const t = this.p1; this.p1 = this.p2; this.p2 = t; }
    let pp = this.p1, n = 0;
    do {
      pp = pp.add(this.p2.subtract(this.p1).x(2));
      const xy1 = pp.e(1) * pp.e(1) + pp.e(2) * pp.e(2);
      const xy2 = this.p2.e(1) * this.p2.e(1) + this.p2.e(2) * this.p2.e(2);
      const z1 = pp.e(3), z2 = this.p2.e(3);
      this.ah = (1 / xy1 - (z1 * z1) / (xy1 * z2 * z2)) / (1 - (xy2 * z1 * z1) / (xy1 * z2 * z2));
      this.ch = (this.ah * xy2 - 1) / (z2 * z2);
      n++;
    } while (!isFinite(this.ah) && n < 20);
    if (!isFinite(this.ah)) throw new Error('the p1,p2 of hyperboloid is illegal');
  }
  boundbox() {
    return { min: this.position.subtract([this.rMax, -this.zMin, this.rMax]), max: this.position.add([this.rMax, this.zMax, this.rMax]) };
  }
  translate() { this.position = this.position.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) {
    this.translate();
    return this._row([7, ...this.position.elements, ...this.p1.elements, ...this.p2.elements, this.ah, this.ch], id);
  }
}
class Paraboloid extends Object3D {
  constructor(position, z0, z1, radius, material, texture, emission, reverseNormal) {
    super(material, texture, emission, reverseNormal);
    this.position = vec(position); this.z0 = z0; this.z1 = z1; this.radius = radius;
    this.zMin = Math.min(z0, z1); this.zMax = Math.max(z0, z1);
    this._pluginName = 'paraboloid';
  }
  boundbox() {
    return { min: this.position.subtract([this.radius, -this.zMin, this.radius]), max: this.position.add([this.radius, this.zMax, this.radius]) };
  }
  translate() { this.position = this.position.add(this.temporaryTranslation); super.translate(); }
  gen(id = this.texparamID) { this.translate(); return this._row([8, ...this.position.elements, this.z0, this.z1, this.radius], id); }
}
class Cornellbox extends Object3D {
  constructor(min = [0, 0, -5], max = [5.560, 5.488, 5.592]) {
    super(new Matte(1), Color.BLACK);
    this.min = vec(min); this.max = vec(max); this._pluginName = 'cornellbox';
  }
  scale(k) { this.min = this.min.x(k); this.max = this.max.x(k); }
  boundbox() { return { min: this.min, max: this.max }; }
  gen(id = this.texparamID) { return this._row([9, ...this.min.elements, ...this.max.elements], id); }
}

// ---- lights (src/scene/light.js) ----------------------------------------------------------------------------
class Light {
  constructor(emission) { this.emission = vec(emission); this._pluginName = ''; }
  get pluginName() { return this._pluginName; }
  set pluginName(n) {}
  gen(data) { return pad(data.concat(this.emission.elements), LIGHTS_LENGTH); }
}
class GeometryLight extends Light {
  constructor(geometry, emission) { super(emission); geometry.emission = vec(emission); this._geometry = geometry; }
  get geometry() { return (typeof this.index !== 'undefined') ? this._geometry : undefined; }
  set geometry(g) { this._geometry = g; }
  getGeometry(index) { this.index = index; return this._geometry; }
  gen(data) {
    if (typeof this.index === 'undefined') throw new Error("can't find index of AreaLight's geometry");
    return super.gen(data.concat([this.index]));
  }
}
class AreaLight extends GeometryLight {
  constructor(geometry, emission) { super(geometry, emission); this._pluginName = 'area'; }
  gen() { return super.gen([0]); }
}
class PointLight extends Light {
  constructor(from, emission) { super(emission); this.from = vec(from); this._pluginName = 'point'; }
  gen() { return super.gen([1, ...this.from.elements]); }
}
class SpotLight extends Light {
  constructor(from, coneangle, conedelta, emission) {
    super(emission);
    this.cosTotalWidth = Math.cos(coneangle / 180 * Math.PI);
    this.cosFalloffStart = Math.cos((coneangle - conedelta) / 180 * Math.PI);
    this.from = vec(from);
    this._pluginName = 'spot';
  }
  gen() { return super.gen([2, this.cosTotalWidth, this.cosFalloffStart, ...this.from.elements]); }
}

// ---- camera (src/scene/camera.js) ----------------------------------------------------------------------------
class Camera {
  constructor(eye, center, up = [0, 1, 0]) {
    this.eye = vec(eye); this.center = vec(center); this.up = vec(up);
    this.makePerspective();
    this.makeLookAt();
  }
  makePerspective(fovy = 55, aspect = 1, znear = 1, zfar = 100) {
    const top = znear * Math.tan(fovy * Math.PI / 360.0), bottom = -top;
    const left = bottom * aspect, right = top * aspect;
    const X = 2 * znear / (right - left), Y = 2 * znear / (top - bottom);
    const A = (right + left) / (right - left), B = (top + bottom) / (top - bottom);
    const C = -(zfar + znear) / (zfar - znear), D = -2 * zfar * znear / (zfar - znear);
    this.fovy = fovy; this.aspect = aspect; this.znear = znear; this.zfar = zfar;
    this.projection = new Matrix([[X, 0, A, 0], [0, Y, B, 0], [0, 0, C, D], [0, 0, -1, 0]]);
  }
  makeLookAt() {
    const z = this.eye.subtract(this.center).toUnitVector();
    let x = this.up.cross(z).toUnitVector();
    const y = z.cross(x).toUnitVector();
    x = x.x(-1);
    const m = new Matrix([[x.e(1), x.e(2), x.e(3), 0], [y.e(1), y.e(2), y.e(3), 0], [z.e(1), z.e(2), z.e(3), 0], [0, 0, 0, 1]]);
    const t = new Matrix([[1, 0, 0, -this.eye.e(1)], [0, 1, 0, -this.eye.e(2)], [0, 0, 1, -this.eye.e(3)], [0, 0, 0, 1]]);
    this.modelview = m.x(t);
  }
  update() { this.makeLookAt(); }
}

// ---- scene (src/scene/scene.js) ----------------------------------------------------------------------------------
const FILTERS = ['color', 'gamma', 'box', 'gaussian', 'mitchell', 'sinc', 'triangle', 'normal', 'position', 'wavelet', 'tonemapping'];
const TRACES = ['path'];

class Scene {
  constructor() {
    this.camera = {};
    this.objects = [];
    this.lights = [];
    this.sampleCount = 0;
    this._trace = new PluginParams('path');
    this._filter = new PluginParams('color');
    this.select = null;
    this.moving = false;
  }
  set filter(p) { if (FILTERS.includes(p)) this._filter.name = p; }
  get filter() { return this._filter; }
  set trace(p) { if (TRACES.includes(p)) this._trace.name = p; }
  get trace() { return this._trace; }
  get mat() { return this.camera.projection.x(this.camera.modelview); }
  set mat(m) {}
  get eye() { return this.camera.eye; }
  set eye(e) {}
  add(thing) {
    if (thing instanceof Camera) this.camera = thing;
    else if (thing instanceof Object3D) this.objects.push(thing);
    else if (thing instanceof Light) {
      if (thing instanceof GeometryLight) this.objects.push(thing.getGeometry(this.objects.length));
      this.lights.push(thing);
    }
  }
  // the reference resets a global `scene` here (scene.js:65-68); this build resets this scene
  update() { this.camera.update(); this.sampleCount = 0; }
  tracerConfig() {
    const cfg = { shape: [], light: [], material: [], texture: [], trace: this.trace };
    const seen = { shape: [], light: [], material: [], texture: [] };
    const note = (kind, name) => {
      if (name && !seen[kind].includes(name)) { cfg[kind].push(new PluginParams(name)); seen[kind].push(name); }
    };
    for (const ob of this.objects) {
      note('shape', ob.pluginName);
      note('material', ob.material.pluginName);
      note('texture', ob.texture.pluginName);
    }
    for (const l of this.lights) note('light', l.pluginName);
    return cfg;
  }
  rendererConfig() { return { filter: this.filter }; }
  // serialisation exactly as Tracer.update does it (tracer.js:45-52)
  serialize() {
    const objects = [], texparams = [], lights = [];
    for (const ob of this.objects) {
      objects.push(...ob.gen(texparams.length / TEXPARAMS_LENGTH));
      texparams.push(...ob.genTexparams());
    }
    for (const l of this.lights) lights.push(...l.gen());
    return {
      objects: new Float32Array(objects), texparams: new Float32Array(texparams), lights: new Float32Array(lights),
      n: Math.floor(objects.length / OBJECTS_LENGTH), tn: Math.floor(texparams.length / TEXPARAMS_LENGTH),
      ln: Math.floor(lights.length / LIGHTS_LENGTH),
    };
  }
  serializeObjects() {  // Tracer.updateObjects (tracer.js:25-40): object rows with their existing texparam ids
    const objects = [];
    for (const ob of this.objects) objects.push(...ob.gen());
    return new Float32Array(objects);
  }
}

module.exports = {
  PluginParams, Material, Matte, Mirror, Metal, Glass, Texture, UniformColor, Checkerboard, Checkerboard2, Bilerp,
  Mix, Scale, UV, Color, Object3D, Cube, Sphere, Rectangle, Cone, Cylinder, Disk, Hyperboloid, Paraboloid,
  Cornellbox, Light, GeometryLight, AreaLight, PointLight, SpotLight, Camera, Scene, FILTERS,
  OBJECTS_LENGTH, TEXPARAMS_LENGTH, LIGHTS_LENGTH,
};
