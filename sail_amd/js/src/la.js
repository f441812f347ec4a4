'use strict';
// Sail.Vector / Sail.Matrix: the small double-precision linear-algebra surface of the reference's public
// API (index.js:44-45, src/utils/matrix.js). Results that feed the GPU (camera P*MV, the jittered inverse)
// must equal the reference's to the last bit, so the reductions keep its evaluation order:
// Vector.dot sums from the last component down (matrix.js:97-103), Matrix.multiply accumulates from 0 in
// column order (:324-350), inverse is Gauss elimination without pivoting on [M | I] followed by back
// substitution (:391-419, :501-527). Checked against tests/golden/fixtures.json by tests/test_js_host.py.

class Vector {
  constructor(elements) { this.setElements(elements); }
  setElements(els) { this.elements = Array.from(els.elements || els); return this; }
  e(i) { return (i < 1 || i > this.elements.length) ? null : this.elements[i - 1]; }
  dimensions() { return this.elements.length; }
  dup() { return new Vector(this.elements); }
  map(fn) { return new Vector(this.elements.map((x, i) => fn(x, i + 1))); }
  each(fn) { this.elements.forEach((x, i) => fn(x, i + 1)); }
  dot(v) {
    const b = v.elements || v;
    if (b.length !== this.elements.length) return null;
    let p = 0;
    for (let n = this.elements.length; n >= 1; n--) p += this.elements[n - 1] * b[n - 1];
    return p;
  }
  modulus() { return Math.sqrt(this.dot(this)); }
  length() { return this.modulus(); }
  toUnitVector() { const r = this.modulus(); return r === 0 ? this.dup() : this.map((x) => x / r); }
  eql(v) {
    const b = v.elements || v;
    if (b.length !== this.elements.length) return false;
    return this.elements.every((x, i) => Math.abs(x - b[i]) <= 1e-5);
  }
  add(v) { const b = v.elements || v; return this.map((x, i) => x + b[i - 1]); }
  subtract(v) { const b = v.elements || v; return this.map((x, i) => x - b[i - 1]); }
  multiply(k) { return this.map((x) => x * k); }
  x(k) { return this.multiply(k); }
  divide(k) { return this.map((x) => x / k); }
  componentDivide(v) { const b = v.elements || v; return this.map((x, i) => x / b[i - 1]); }
  cross(v) {
    const A = this.elements, B = v.elements || v;
    if (A.length !== 3 || B.length !== 3) return null;
    return new Vector([(A[1] * B[2]) - (A[2] * B[1]), (A[2] * B[0]) - (A[0] * B[2]), (A[0] * B[1]) - (A[1] * B[0])]);
  }
  divideByW() { const w = this.elements[this.elements.length - 1]; return this.map((x) => x / w); }
  ensure3() { return new Vector(this.elements.slice(0, 3)); }
  maxComponent() { return Math.max(...this.elements); }
  minComponent() { return Math.min(...this.elements); }
  flatten() { return this.elements.slice(); }
  distanceFrom(v) { return this.subtract(v).modulus(); }
  static get i() { return new Vector([1, 0, 0]); }
  static get j() { return new Vector([0, 1, 0]); }
  static get k() { return new Vector([0, 0, 1]); }
  static Zero(n) { return new Vector(new Array(n).fill(0)); }
  static min(a, b) { return a.map((x, i) => Math.min(x, b.e(i))); }
  static max(a, b) { return a.map((x, i) => Math.max(x, b.e(i))); }
}

class Matrix {
  constructor(elements) { this.setElements(elements); }
  setElements(els) {
    const rows = els.elements || els;
    this.elements = (typeof rows[0] === 'number') ? rows.map((x) => [x]) : rows.map((r) => Array.from(r.elements || r));
    return this;
  }
  e(i, j) { return this.elements[i - 1] ? this.elements[i - 1][j - 1] : null; }
  rows() { return this.elements.length; }
  cols() { return this.elements[0].length; }
  dup() { return new Matrix(this.elements); }
  map(fn) { return new Matrix(this.elements.map((r, i) => r.map((x, j) => fn(x, i + 1, j + 1)))); }
  row(i) { return new Vector(this.elements[i - 1]); }
  col(j) { return new Vector(this.elements.map((r) => r[j - 1])); }
  isSquare() { return this.elements.length === this.elements[0].length; }
  add(m) { const b = m.elements || m; return this.map((x, i, j) => x + b[i - 1][j - 1]); }
  subtract(m) { const b = m.elements || m; return this.map((x, i, j) => x - b[i - 1][j - 1]); }
  transpose() { return new Matrix(this.elements[0].map((_, j) => this.elements.map((r) => r[j]))); }
  multiply(m) {
    if (typeof m === 'number') return this.map((x) => x * m);
    const isVec = m instanceof Vector;
    let B = m.elements || m;
    if (typeof B[0] === 'number') B = B.map((x) => [x]);
    const n = this.elements.length, p = B[0].length, q = this.elements[0].length;
    if (q !== B.length) return null;
    const out = [];
    for (let i = 0; i < n; i++) {
      out.push([]);
      for (let j = 0; j < p; j++) {
        let sum = 0;
        for (let c = 0; c < q; c++) sum += this.elements[i][c] * B[c][j];
        out[i].push(sum);
      }
    }
    const M = new Matrix(out);
    return isVec ? M.col(1) : M;
  }
  x(m) { return this.multiply(m); }
  // Gauss elimination without pivoting; a zero pivot borrows (adds) the first later row with a non-zero
  static _triangulate(rows) {
    const n = rows.length, kp = rows[0].length;
    for (let i = 0; i < n; i++) {
      if (rows[i][i] === 0) {
        for (let j = i + 1; j < n; j++) {
          if (rows[j][i] !== 0) { rows[i] = rows[i].map((x, p) => x + rows[j][p]); break; }
        }
      }
      if (rows[i][i] !== 0) {
        for (let j = i + 1; j < n; j++) {
          const mul = rows[j][i] / rows[i][i];
          rows[j] = rows[j].map((x, p) => (p <= i ? 0 : x - rows[i][p] * mul));
        }
      }
    }
    return rows;
  }
  toRightTriangular() { return new Matrix(Matrix._triangulate(this.elements.map((r) => r.slice()))); }
  determinant() {
    if (!this.isSquare()) return null;
    const T = Matrix._triangulate(this.elements.map((r) => r.slice()));
    let det = T[0][0];
    for (let i = 1; i < T.length; i++) det = det * T[i][i];
    return det;
  }
  det() { return this.determinant(); }
  isSingular() { return this.isSquare() && this.determinant() === 0; }
  inverse() {
    if (!this.isSquare() || this.isSingular()) return null;
    const n = this.elements.length;
    const A = Matrix._triangulate(this.elements.map((r, i) => r.concat(r.map((_, j) => (i === j ? 1 : 0)))));
    const inv = [];
    for (let i = n - 1; i >= 0; i--) {
      const d = A[i][i];
      A[i] = A[i].map((x) => x / d);
      inv[i] = A[i].slice(n);
      for (let j = 0; j < i; j++) {
        const f = A[j][i];
        A[j] = A[j].map((x, p) => x - A[i][p] * f);
      }
    }
    return new Matrix(inv);
  }
  inv() { return this.inverse(); }
  flatten() {  // column-major, as uniformMatrix4fv expects
    const out = [];
    for (let j = 0; j < this.elements[0].length; j++) for (let i = 0; i < this.elements.length; i++) out.push(this.elements[i][j]);
    return out;
  }
  static I(n) { return new Matrix(Array.from({ length: n }, (_, i) => Array.from({ length: n }, (_, j) => (i === j ? 1 : 0)))); }
  static Zero(n, m) { return new Matrix(Array.from({ length: n }, () => new Array(m).fill(0))); }
  static Diagonal(els) { const M = Matrix.I(els.length); els.forEach((x, i) => { M.elements[i][i] = x; }); return M; }
  static Translation(v) {
    const e = v.elements || v;
    const M = Matrix.I(e.length + 1);
    for (let i = 0; i < e.length; i++) M.elements[i][e.length] = e[i];
    if (e.length === 2) {  // 2-D form of the reference stores the offset in the last row
      const R = Matrix.I(3); R.elements[2][0] = e[0]; R.elements[2][1] = e[1]; return R;
    }
    return M;
  }
  static Scale(v) { const e = v.elements || v; const M = Matrix.I(e.length === 2 ? 3 : 4); e.forEach((x, i) => { M.elements[i][i] = x; }); return M; }
  static RotationX(t) { const c = Math.cos(t), s = Math.sin(t); return new Matrix([[1, 0, 0], [0, c, -s], [0, s, c]]); }
  static RotationY(t) { const c = Math.cos(t), s = Math.sin(t); return new Matrix([[c, 0, s], [0, 1, 0], [-s, 0, c]]); }
  static RotationZ(t) { const c = Math.cos(t), s = Math.sin(t); return new Matrix([[c, -s, 0], [s, c, 0], [0, 0, 1]]); }
}

module.exports = { Vector, Matrix };
