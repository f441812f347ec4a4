'use strict';
// Sail.Control / Pickup (reference src/core/control.js, src/core/pickup.js): mouse orbit, zoom, pick and drag.
// The orbit/zoom/drag arithmetic is the reference's host-side f64 JavaScript. pick() is the one piece that
// moved: instead of the reference's CPU intersect() per object (geometry.js, whose Rectangle test uses the
// wrong plane), the ray goes to the GPU through sail_pick and is answered by the trace kernel's own
// primitive sweep, so a click selects exactly the object the rendered pixel shows.
const { Vector } = require('./la');

const MINVALUE = 1e-4;   // pickup.js / geometry.js
const MAXVALUE = 1e5;

class Ray {
  constructor(origin, dir) { this.origin = origin; this.dir = dir; }
  // pickup.js:11-14: inverse(P*MV) * (x, y, 0, 1), divided by w, minus the eye (not normalised)
  static generate(eye, inmp, x, y) {
    const dir = inmp.multiply(new Vector([x, y, 0, 1])).divideByW().ensure3().subtract(eye);
    return new Ray(eye, dir);
  }
  intersectBoundBox(boundbox) {  // pickup.js:31-42
    const tMin = boundbox.min.subtract(this.origin).componentDivide(this.dir);
    const tMax = boundbox.max.subtract(this.origin).componentDivide(this.dir);
    const t1 = Vector.min(tMin, tMax), t2 = Vector.max(tMin, tMax);
    const tNear = t1.maxComponent(), tFar = t2.minComponent();
    if (tNear > MINVALUE && tNear < tFar) return tNear;
    else if (tNear < tFar) return tFar;
    return MAXVALUE;
  }
}

class Pickup {
  constructor(scene, renderer = null) {
    this.scene = scene;
    this.renderer = renderer;
  }
  _size() {
    const r = this.renderer || this.scene.renderer;
    return r ? [r.width, r.height] : [512, 512];
  }
  _ray(x, y) {
    const [W, H] = this._size();
    return Ray.generate(this.scene.eye, this.scene.mat.inverse(), (x / W) * 2 - 1, 1 - (y / H) * 2);
  }
  // pickup.js:46-66, answered on the GPU
  pick(x, y) {
    const r = this.renderer || this.scene.renderer;
    if (!r) throw new Error('Pickup.pick needs a Renderer that has been updated with this scene');
    const ray = this._ray(x, y);
    const hit = r.pick(ray.origin.elements, ray.dir.elements);
    this.scene.select = hit.index >= 0 ? this.scene.objects[hit.index] : null;
    return hit.index >= 0;
  }
  // pickup.js:68-96: start dragging the selection along the face of its bounding box under the cursor
  movingBegin(x, y) {
    const boundbox = this.scene.select.boundbox();
    const ray = this._ray(x, y);
    const t = ray.intersectBoundBox(boundbox);
    if (t < MAXVALUE) {
      const hit = ray.origin.add(ray.dir.x(t));
      const e = hit.elements, mn = boundbox.min.elements, mx = boundbox.max.elements;
      if (Math.abs(e[0] - mn[0]) < MINVALUE) this.movementNormal = new Vector([-1, 0, 0]);
      else if (Math.abs(e[0] - mx[0]) < MINVALUE) this.movementNormal = new Vector([1, 0, 0]);
      else if (Math.abs(e[1] - mn[1]) < MINVALUE) this.movementNormal = new Vector([0, -1, 0]);
      else if (Math.abs(e[1] - mx[1]) < MINVALUE) this.movementNormal = new Vector([0, 1, 0]);
      else if (Math.abs(e[2] - mn[2]) < MINVALUE) this.movementNormal = new Vector([0, 0, -1]);
      else this.movementNormal = new Vector([0, 0, 1]);
      this.movementDistance = this.movementNormal.dot(hit);
      this.originalHit = hit;
      this.scene.moving = true;
      return true;
    }
    return false;
  }
  _planeHit(x, y) {
    const ray = this._ray(x, y);
    const t = (this.movementDistance - this.movementNormal.dot(ray.origin)) / this.movementNormal.dot(ray.dir);
    return ray.origin.add(ray.dir.multiply(t));
  }
  moving(x, y) {  // pickup.js:98-109
    const hit = this._planeHit(x, y);
    this.scene.select.temporaryTranslate(hit.subtract(this.originalHit));
    this.originalHit = hit;
  }
  movingEnd(x, y) {  // pickup.js:111-123
    const hit = this._planeHit(x, y);
    this.scene.select.temporaryTranslate(hit.subtract(this.originalHit));
    this.scene.moving = false;
  }
}

// control.js: orbit (drag on empty space), zoom (wheel), pick + drag (click on an object). The handlers
// are exposed as plain methods taking canvas-relative mouse positions so a Node host can drive them; init()
// binds them to DOM events when a document is present.
class Control {
  static init(canvas) {
    Control.canvas = canvas;
    if (typeof document !== 'undefined' && document.addEventListener) {
      const pos = (ev) => {
        const r = canvas.getBoundingClientRect();
        return { x: ev.clientX - r.left, y: ev.clientY - r.top };
      };
      document.addEventListener('mousedown', (ev) => { const p = pos(ev); Control.mousedown(p.x, p.y); }, false);
      document.addEventListener('mousemove', (ev) => { const p = pos(ev); Control.mousemove(p.x, p.y); }, false);
      document.addEventListener('mouseup', (ev) => { const p = pos(ev); Control.mouseup(p.x, p.y); }, false);
      document.addEventListener('wheel', (ev) => { Control.wheel(ev.deltaY > 0); ev.preventDefault(); }, { passive: false });
    }
  }
  static update(scene) {  // control.js:58-69
    Control.scene = scene;
    Control.pick = new Pickup(scene);
    Control.mouseDown = false;
    const cam = scene.camera;
    Control.R = cam.eye.distanceFrom(cam.center);
    Control.angleX = Math.asin((cam.eye.e(2) - cam.center.e(2)) / Control.R);
    Control.angleY = Math.acos((cam.eye.e(3) - cam.center.e(3)) / (Control.R * Math.cos(Control.angleX)));
    if (cam.eye.e(1) - cam.center.e(1) < 0) Control.angleY = -Control.angleY;
  }
  static _size() {
    const r = Control.scene && Control.scene.renderer;
    return r ? [r.width, r.height] : [512, 512];
  }
  static _orbit() {
    const cam = Control.scene.camera;
    cam.eye = new Vector([
      Control.R * Math.sin(Control.angleY) * Math.cos(Control.angleX),
      Control.R * Math.sin(Control.angleX),
      Control.R * Math.cos(Control.angleY) * Math.cos(Control.angleX),
    ]).add(cam.center);
  }
  static mousedown(x, y) {  // control.js:71-87
    Control.oldX = x; Control.oldY = y;
    const [W, H] = Control._size();
    if (x >= 0 && x < W && y >= 0 && y < H) {
      Control.mouseDown = true;
      if (Control.scene.select !== null) Control.mouseDown = !Control.pick.movingBegin(x, y);
      if (Control.mouseDown) Control.mouseDown = !Control.pick.pick(x, y);
    }
    return true;
  }
  static mousemove(x, y) {  // control.js:89-114
    if (Control.mouseDown) {
      Control.angleY += -(Control.oldX - x) * 0.01;
      Control.angleX += -(Control.oldY - y) * 0.01;
      Control.angleX = Math.max(Control.angleX, -Math.PI / 2 + 0.01);
      Control.angleX = Math.min(Control.angleX, Math.PI / 2 - 0.01);
      Control._orbit();
      Control.oldX = x; Control.oldY = y;
      Control.scene.update();
    } else if (Control.scene.moving) {
      Control.pick.moving(x, y);
    }
  }
  static mouseup(x, y) {  // control.js:116-125
    Control.mouseDown = false;
    if (Control.scene.moving) Control.pick.movingEnd(x, y);
  }
  static wheel(down) {  // control.js:127-154
    Control.R *= down ? 1.1 : 0.9;
    Control._orbit();
    Control.scene.update();
  }
}

module.exports = { Control, Pickup, Ray };
