'use strict';
// The Sail public object (reference index.js:15-46), backed by libsail_hip.so on MI355X.
// require('sail_amd/js') in Node; in a browser-like global it is also published as window.Sail.
const scene = require('./src/scene');
const { Vector, Matrix } = require('./src/la');
const { Renderer } = require('./src/renderer');

const { Control } = require('./src/control');  // mouse orbit / zoom / GPU pick + drag (control.js, pickup.js)

const Sail = {
  Renderer,
  Scene: scene.Scene,
  Cube: scene.Cube,
  Sphere: scene.Sphere,
  Rectangle: scene.Rectangle,
  Cone: scene.Cone,
  Cylinder: scene.Cylinder,
  Disk: scene.Disk,
  Hyperboloid: scene.Hyperboloid,
  Paraboloid: scene.Paraboloid,
  AreaLight: scene.AreaLight,
  PointLight: scene.PointLight,
  SpotLight: scene.SpotLight,
  Cornellbox: scene.Cornellbox,
  Camera: scene.Camera,
  Control,
  Matte: scene.Matte,
  Mirror: scene.Mirror,
  Metal: scene.Metal,
  Glass: scene.Glass,
  UniformColor: scene.UniformColor,
  Checkerboard: scene.Checkerboard,
  Checkerboard2: scene.Checkerboard2,
  Bilerp: scene.Bilerp,
  Mix: scene.Mix,
  Scale: scene.Scale,
  UV: scene.UV,
  Color: scene.Color,
  Matrix,
  Vector,
};

if (typeof window !== 'undefined') {
  window.Sail = Sail;
  window.$V = Matrix;  // the reference's aliases (index.js:48-49)
  window.$M = Vector;
}
module.exports = Sail;
