'use strict';
// Image output for the Node host (SURVEY §8(f) row 3): the browser build paints the filtered frame into a
// canvas (fsrender.glsl -> putImageData); headless renders go to files instead.
//   PFM  — the float mean image (or any W x H x 4 float map), little-endian, rows bottom-to-top, which is
//          exactly the GL row order the renderer already holds, so no flip.
//   PNG  — the display-filtered RGBA8 canvas pixels (top-to-bottom rows, so the GL rows are flipped).
//   EXR  — the float mean image as a single-part scanline OpenEXR file: channels B, G, R (the format sorts them by
//          name) of 32-bit FLOAT, NO_COMPRESSION, one scanline per chunk, INCREASING_Y line order; EXR's y grows
//          downwards, so the GL rows are flipped like the PNG's.
const fs = require('fs');
const zlib = require('zlib');

function toPFM(W, H, rgba) {
  const header = Buffer.from(`PF\n${W} ${H}\n-1.0\n`, 'ascii');  // negative scale = little-endian
  const body = Buffer.alloc(W * H * 3 * 4);
  for (let i = 0, o = 0; i < W * H; i++) {
    for (let c = 0; c < 3; c++, o += 4) body.writeFloatLE(rgba[4 * i + c], o);
  }
  return Buffer.concat([header, body]);
}

const CRC_TABLE = (() => {
  const t = new Uint32Array(256);
  for (let n = 0; n < 256; n++) {
    let c = n;
    for (let k = 0; k < 8; k++) c = (c & 1) ? (0xEDB88320 ^ (c >>> 1)) : (c >>> 1);
    t[n] = c >>> 0;
  }
  return t;
})();
function crc32(buf) {
  let c = 0xFFFFFFFF;
  for (let i = 0; i < buf.length; i++) c = CRC_TABLE[(c ^ buf[i]) & 0xFF] ^ (c >>> 8);
  return (c ^ 0xFFFFFFFF) >>> 0;
}
function chunk(type, data) {
  const len = Buffer.alloc(4);
  len.writeUInt32BE(data.length, 0);
  const td = Buffer.concat([Buffer.from(type, 'ascii'), data]);
  const crc = Buffer.alloc(4);
  crc.writeUInt32BE(crc32(td), 0);
  return Buffer.concat([len, td, crc]);
}
// rgba8: W*H*4 bytes in GL order (row 0 = bottom)
function toPNG(W, H, rgba8) {
  const raw = Buffer.alloc(H * (1 + W * 4));
  for (let y = 0; y < H; y++) {
    const src = (H - 1 - y) * W * 4;
    const dst = y * (1 + W * 4);
    raw[dst] = 0;  // filter type: none
    Buffer.from(rgba8.buffer, rgba8.byteOffset + src, W * 4).copy(raw, dst + 1);
  }
  const ihdr = Buffer.alloc(13);
  ihdr.writeUInt32BE(W, 0);
  ihdr.writeUInt32BE(H, 4);
  ihdr[8] = 8;   // bit depth
  ihdr[9] = 6;   // colour type RGBA
  ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
  return Buffer.concat([Buffer.from([0x89, 0x50, 0x4E, 0x47, 0x0D, 0x0A, 0x1A, 0x0A]), chunk('IHDR', ihdr),
    chunk('IDAT', zlib.deflateSync(raw)), chunk('IEND', Buffer.alloc(0))]);
}

// ---- OpenEXR (uncompressed scanline float) ----
function exrAttr(name, type, value) {
  const size = Buffer.alloc(4);
  size.writeInt32LE(value.length, 0);
  return Buffer.concat([Buffer.from(name + '\0' + type + '\0', 'ascii'), size, value]);
}
function i32s(...v) { const b = Buffer.alloc(4 * v.length); v.forEach((x, i) => b.writeInt32LE(x, 4 * i)); return b; }
function f32s(...v) { const b = Buffer.alloc(4 * v.length); v.forEach((x, i) => b.writeFloatLE(x, 4 * i)); return b; }
const EXR_FLOAT = 2;
// rgba: W*H*4 floats in GL order (row 0 = bottom); the alpha slot (a sample count or 1) is not written
function toEXR(W, H, rgba) {
  const names = ['B', 'G', 'R'];            // chlist order is alphabetical; data follows it per scanline
  const src = { R: 0, G: 1, B: 2 };
  const chlist = Buffer.concat([...names.map((n) => Buffer.concat([Buffer.from(n + '\0', 'ascii'),
    i32s(EXR_FLOAT), Buffer.from([0, 0, 0, 0]), i32s(1, 1)])), Buffer.from([0])]);
  const header = Buffer.concat([
    Buffer.from([0x76, 0x2f, 0x31, 0x01]), i32s(2),   // magic, version 2 (single-part scanline)
    exrAttr('channels', 'chlist', chlist),
    exrAttr('compression', 'compression', Buffer.from([0])),
    exrAttr('dataWindow', 'box2i', i32s(0, 0, W - 1, H - 1)),
    exrAttr('displayWindow', 'box2i', i32s(0, 0, W - 1, H - 1)),
    exrAttr('lineOrder', 'lineOrder', Buffer.from([0])),
    exrAttr('pixelAspectRatio', 'float', f32s(1)),
    exrAttr('screenWindowCenter', 'v2f', f32s(0, 0)),
    exrAttr('screenWindowWidth', 'float', f32s(1)),
    Buffer.from([0])]);
  const lineBytes = W * names.length * 4;
  const chunkBytes = 8 + lineBytes;
  const table = Buffer.alloc(8 * H);
  const body = Buffer.alloc(chunkBytes * H);
  const base = header.length + table.length;
  for (let y = 0; y < H; y++) {
    table.writeBigUInt64LE(BigInt(base + y * chunkBytes), 8 * y);
    let o = y * chunkBytes;
    body.writeInt32LE(y, o);
    body.writeInt32LE(lineBytes, o + 4);
    o += 8;
    const row = (H - 1 - y) * W;
    for (const n of names) {
      for (let x = 0; x < W; x++, o += 4) body.writeFloatLE(rgba[4 * (row + x) + src[n]], o);
    }
  }
  return Buffer.concat([header, table, body]);
}

function writePFM(path, W, H, rgba) { fs.writeFileSync(path, toPFM(W, H, rgba)); }
function writePNG(path, W, H, rgba8) { fs.writeFileSync(path, toPNG(W, H, rgba8)); }
function writeEXR(path, W, H, rgba) { fs.writeFileSync(path, toEXR(W, H, rgba)); }

module.exports = { toPFM, toPNG, toEXR, writePFM, writePNG, writeEXR, crc32 };
