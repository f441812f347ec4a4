"""Output formats and the headless CLI: PFM/PNG writers (CPU), the scene-script CLI
failing loudly without a device (CPU) and rendering bit-exactly against the oracle (GPU)."""
import json
import os
import shutil
import struct
import subprocess
import zlib

import numpy as np
import pytest

import oracle
from sail_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node") or shutil.which("nodejs")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _node(code, *args):
    return subprocess.run([NODE, "-e", code, *args], cwd=ROOT, capture_output=True, check=True).stdout


def read_png(buf):
    assert buf[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, W = 8, b"", None
    while pos < len(buf):
        ln, typ = struct.unpack(">I4s", buf[pos:pos + 8])
        data = buf[pos + 8:pos + 8 + ln]
        assert struct.unpack(">I", buf[pos + 8 + ln:pos + 12 + ln])[0] == zlib.crc32(typ + data)
        if typ == b"IHDR":
            W, H, depth, ctype = struct.unpack(">IIBB", data[:10])
            assert (depth, ctype) == (8, 6)
        elif typ == b"IDAT":
            idat += data
        pos += 12 + ln
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(H, 1 + W * 4)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(H, W, 4)


def read_pfm(buf):
    parts = buf.split(b"\n", 3)
    assert parts[0] == b"PF"
    W, H = map(int, parts[1].split())
    assert float(parts[2]) < 0  # little-endian
    return np.frombuffer(parts[3], "<f4").reshape(H, W, 3)


def read_exr(buf):
    """Single-part scanline OpenEXR reader (the file-format spec, independent of the writer): header
    attributes, the line offset table, then uncompressed FLOAT chunks. Returns (rows top-down, attributes)."""
    assert buf[:4] == b"\x76\x2f\x31\x01" and struct.unpack("<i", buf[4:8])[0] == 2
    pos, attrs = 8, {}
    while buf[pos] != 0:
        end = buf.index(b"\0", pos)
        name = buf[pos:end].decode()
        tend = buf.index(b"\0", end + 1)
        typ = buf[end + 1:tend].decode()
        size = struct.unpack("<i", buf[tend + 1:tend + 5])[0]
        attrs[name] = (typ, buf[tend + 5:tend + 5 + size])
        pos = tend + 5 + size
    pos += 1
    for req in ("channels", "compression", "dataWindow", "displayWindow", "lineOrder", "pixelAspectRatio",
                "screenWindowCenter", "screenWindowWidth"):
        assert req in attrs, req
    assert attrs["compression"] == ("compression", b"\0") and attrs["lineOrder"] == ("lineOrder", b"\0")
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    chl, names, cp = attrs["channels"][1], [], 0
    while chl[cp] != 0:
        end = chl.index(b"\0", cp)
        names.append(chl[cp:end].decode())
        ptype, _, xs, ys = struct.unpack("<iB3xii", chl[end + 1:end + 17])
        assert (ptype, xs, ys) == (2, 1, 1)
        cp = end + 17
    assert names == sorted(names)
    offsets = struct.unpack(f"<{H}Q", buf[pos:pos + 8 * H])
    img = np.zeros((H, W, len(names)), np.float32)
    for off in offsets:
        y, n = struct.unpack("<ii", buf[off:off + 8])
        assert n == W * len(names) * 4
        line = np.frombuffer(buf[off + 8:off + 8 + n], "<f4").reshape(len(names), W)
        img[y - y0] = line.T
    return img, names


def test_png_and_pfm_writers():
    W, H = 7, 5
    rng = np.random.default_rng(0)
    px = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    fl = rng.normal(size=(H, W, 4)).astype(np.float32)
    code = """
const { toPNG, toPFM, toEXR } = require('./sail_amd/js/src/image');
const [W, H, a, b] = process.argv.slice(1);
const px = Uint8Array.from(Buffer.from(a, 'hex')), fb = Buffer.from(b, 'hex'), fl = new Float32Array(fb.buffer.slice(fb.byteOffset, fb.byteOffset + fb.length));
process.stdout.write(JSON.stringify({ png: toPNG(+W, +H, px).toString('base64'), pfm: toPFM(+W, +H, fl).toString('base64'),
  exr: toEXR(+W, +H, fl).toString('base64') }));
"""
    import base64
    out = json.loads(_node(code, str(W), str(H), px.tobytes().hex(), fl.tobytes().hex()))
    png = read_png(base64.b64decode(out["png"]))
    assert np.array_equal(png, px[::-1])              # GL rows (bottom-up) -> PNG rows (top-down)
    pfm = read_pfm(base64.b64decode(out["pfm"]))
    assert np.array_equal(pfm, fl[..., :3])           # PFM rows are bottom-up, like GL
    exr, names = read_exr(base64.b64decode(out["exr"]))
    assert names == ["B", "G", "R"]
    assert np.array_equal(exr[..., ::-1].view(np.uint32), fl[::-1, :, :3].view(np.uint32))  # EXR y grows down


def test_cli_fails_loudly_without_device(tmp_path):
    if capi.device_count() > 0:
        pytest.skip("device present")
    r = subprocess.run([NODE, "sail_amd/js/cli.js", "sail_amd/js/examples/cornell.js", "--width", "8", "--height", "8",
                        "--spp", "1", "--png", str(tmp_path / "x.png")], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 1 and "sail:" in r.stderr
    assert not (tmp_path / "x.png").exists()


def test_cli_rejects_bad_script(tmp_path):
    bad = tmp_path / "bad.js"
    bad.write_text("let x = 1;\n")
    r = subprocess.run([NODE, "sail_amd/js/cli.js", str(bad)], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 1 and ("Sail.Scene" in r.stderr or "HIP" in r.stderr or "device" in r.stderr)


@pytest.mark.gpu
def test_cli_renders_bit_exact(tmp_path, fixtures):
    if capi.device_count() < 1:
        pytest.skip("no HIP device")
    W, H, spp, B = 40, 30, 4, 5
    pfm, png, exr = tmp_path / "c.pfm", tmp_path / "c.png", tmp_path / "c.exr"
    r = subprocess.run([NODE, "sail_amd/js/cli.js", "sail_amd/js/examples/cornell.js", "--width", str(W), "--height", str(H),
                        "--spp", str(spp), "--bounces", str(B), "--deterministic", "--pfm", str(pfm), "--png", str(png), "--exr", str(exr),
                        "--stats"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["segments"] == W * H * spp * B  # closed box: every path runs all bounces
    got = read_pfm(pfm.read_bytes())
    sc = fixtures["scenes"]["C1"]
    inv, seeds = capi.schedule(np.array(sc["mvp_rowmajor"]), W, H, 0, spp)
    acc = oracle.render(sc, capi.plugin_masks(sc["plugins"]), W, H, inv, seeds, sc["eye"], B)
    want = acc[..., :3] / acc[..., 3:4]
    assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32))
    ex, _ = read_exr(exr.read_bytes())
    assert np.array_equal(ex[::-1, :, ::-1].view(np.uint32), want.astype(np.float32).view(np.uint32))
    img = read_png(png.read_bytes())
    assert img.shape == (H, W, 4) and (img[..., 3] == 255).all()
