'use strict';
// Image output for the Node host (SURVEY §8(f) row 3): the browser build paints the filtered frame into a
// canvas (fsrender.glsl -> putImageData); headless renders go to files instead.
//   PFM  — the float mean image (or any W x H x 4 float map), little-endian, rows bottom-to-top, which is
//          exactly the GL row order the renderer already holds, so no flip.
//   PNG  — the display-filtered RGBA8 canvas pixels (top-to-bottom rows, so the GL rows are flipped).
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

function writePFM(path, W, H, rgba) { fs.writeFileSync(path, toPFM(W, H, rgba)); }
function writePNG(path, W, H, rgba8) { fs.writeFileSync(path, toPNG(W, H, rgba8)); }

module.exports = { toPFM, toPNG, writePFM, writePNG, crc32 };
