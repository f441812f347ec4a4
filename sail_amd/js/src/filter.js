'use strict';
// Display-filter configuration: Scene.filter (a PluginParams) -> the libsail_hip.so filter call.
// The 4x4 window-weight tables follow the reference's host-side generators (src/shader/filter/box.js,
// gaussian.js, mitchell.js, sinc.js, triangle.js; windowWidth = 4, shader.filter.js:31): weights are
// sampled at ((j+.5) r_x/4, (i+.5) r_y/4) from the one-decimal getParam() values, while the window radius
// itself is the raw FILTER_WINDOW_RADIUS text (e.g. "vec2(2.0,2.0)") evaluated as GLSL would.

const KIND = { color: 0, gamma: 1, tonemapping: 2, window: 3, wavelet: 4, normal: 5, position: 6 };
const WINDOW = 4;

function gaussianW(d, expv, alpha) { return Math.max(0.0, Math.exp(-alpha * d * d) - expv); }
function mitchellW(x, B, C) {
  x = Math.abs(2 * x);
  if (x > 1) return ((-B - 6 * C) * x * x * x + (6 * B + 30 * C) * x * x + (-12 * B - 48 * C) * x + (8 * B + 24 * C)) * (1.0 / 6.0);
  return ((12 - 9 * B - 6 * C) * x * x * x + (-18 + 12 * B + 6 * C) * x * x + (6 - 2 * B)) * (1.0 / 6.0);
}
function sinc(x) { x = Math.abs(x); return x < 1e-5 ? 1.0 : Math.sin(Math.PI * x) / (Math.PI * x); }
function windowedSinc(x, radius, tau) { x = Math.abs(x); return x > radius ? 0.0 : sinc(x) * sinc(x / tau); }
function triangleW(d, radius) { return Math.max(0.0, radius - d); }

// weight table in the reference's row order (offset = i*4 + j); doubles
function windowWeights(pp) {
  const name = pp.name;
  const r = pp.getParam('r');
  const w = [];
  for (let i = 0; i < WINDOW; i++) {
    for (let j = 0; j < WINDOW; j++) {
      if (name === 'box') { w.push(1.0); continue; }
      const px = (j + 0.5) * r[0] / WINDOW, py = (i + 0.5) * r[1] / WINDOW;
      if (name === 'gaussian') {
        const alpha = pp.getParam('alpha')[0];
        const ex = Math.exp(-alpha * r[0] * r[0]), ey = Math.exp(-alpha * r[1] * r[1]);
        w.push(gaussianW(px, ex, alpha) * gaussianW(py, ey, alpha));
      } else if (name === 'mitchell') {
        const b = pp.getParam('b')[0], c = pp.getParam('c')[0];
        w.push(mitchellW(px / r[0], b, c) * mitchellW(py / r[1], b, c));
      } else if (name === 'sinc') {
        const tau = pp.getParam('tau')[0];
        w.push(windowedSinc(px, r[0], tau) * windowedSinc(py, r[1], tau));
      } else if (name === 'triangle') {
        w.push(triangleW(px, r[0]) * triangleW(py, r[1]));
      }
    }
  }
  return w;
}

// "vec2(2.0,2.0)" / "vec2(1.5)" / "2.0" -> [x, y] as the GLSL compiler evaluates FILTER_WINDOW_RADIUS
function glslVec2(text) {
  const nums = String(text).match(/-?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?/g) || [];
  const v = nums.map(parseFloat);
  if (v.length === 0) throw new Error(`filter radius "${text}" has no value`);
  return v.length === 1 ? [v[0], v[0]] : [v[0], v[1]];
}

function filterConfig(pp) {
  switch (pp.name) {
    case 'color': return { kind: KIND.color, weights: null, rx: 0, ry: 0, gamma: 1 };
    case 'tonemapping': return { kind: KIND.tonemapping, weights: null, rx: 0, ry: 0, gamma: 1 };
    case 'gamma': {
      if (pp.params.c === undefined) throw new Error("gamma filter needs scene.filter.addParam('c', '<float>')");
      return { kind: KIND.gamma, weights: null, rx: 0, ry: 0, gamma: parseFloat(pp.params.c) };
    }
    case 'box': case 'gaussian': case 'mitchell': case 'sinc': case 'triangle': {
      if (pp.params.r === undefined) throw new Error(`${pp.name} filter needs scene.filter.addParam('r', 'vec2(x,y)')`);
      const [rx, ry] = glslVec2(pp.params.r);
      const w64 = windowWeights(pp);
      return { kind: KIND.window, weights: Float32Array.from(w64), weights64: w64, rx, ry, gamma: 1 };
    }
    // the AOV filters (normal.glsl, position.glsl, wavelet.glsl) need a Renderer created with aov: true
    case 'normal': case 'position': return { kind: KIND[pp.name], aov: true, weights: null, rx: 0, ry: 0, gamma: 1 };
    case 'wavelet': {
      if (pp.params.r === undefined) throw new Error("wavelet filter needs scene.filter.addParam('r', 'vec2(x,y)')");
      const [rx, ry] = glslVec2(pp.params.r);  // FILTER_WAVELET_R (wavelet.glsl:42-44)
      return { kind: KIND.wavelet, aov: true, weights: null, rx, ry, gamma: 1 };
    }
    default: throw new Error(`filter "${pp.name}" is not a Sail display filter`);
  }
}

module.exports = { filterConfig, windowWeights, glslVec2, KIND };
