"""Output path (rt_image.cpp): the RGBA8 frame written as PPM /
PNG in place of the reference's WebGL texture upload (wasm/wasm.cpp:216-218).
Host-only: checked byte for byte against the oracle's RGBA8 frame, the PNG
decoded with the standard library's zlib (CRCs, Adler-32, stored blocks)."""
import struct
import zlib

import numpy as np
import pytest


def read_ppm(path):
    data = open(path, "rb").read()
    magic, w, h, mx, rest = data.split(maxsplit=4)
    assert magic == b"P6" and mx == b"255"
    w, h = int(w), int(h)
    return np.frombuffer(rest, np.uint8).reshape(h, w, 3)


def read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body), typ
        chunks.setdefault(typ, b"")
        chunks[typ] += body
        pos += 12 + n
    w, h, depth, ctype, comp, filt, inter = struct.unpack(">IIBBBBB", chunks[b"IHDR"])
    assert (depth, ctype, comp, filt, inter) == (8, 6, 0, 0, 0) and b"IEND" in chunks
    raw = zlib.decompress(chunks[b"IDAT"])  # checks the Adler-32 too
    rows = np.frombuffer(raw, np.uint8).reshape(h, 4 * w + 1)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(h, w, 4)


@pytest.mark.parametrize("W,H", [(48, 40), (1, 1), (300, 90)])  # 300x90: more than one stored block
def test_ppm_and_png_hold_the_oracle_frame(rt, orc, tmp_path, W, H):
    o = orc.scene_builtin(1).prefix(16)
    _, cur, _ = orc.render(o, orc.camera(o, W, H), W, H, frames=2, max_bounce=4)
    img = np.ascontiguousarray(cur.reshape(H, W).astype(np.uint32))
    rgba = img.view(np.uint8).reshape(H, W, 4)  # r | g << 8 | b << 16 | a << 24, little endian
    for flip in (True, False):
        want = rgba[::-1] if flip else rgba
        rt.write_image(img, tmp_path / "f.ppm", flip_y=flip)
        assert np.array_equal(read_ppm(tmp_path / "f.ppm"), want[:, :, :3])
        rt.write_image(img, tmp_path / "f.png", flip_y=flip)
        assert np.array_equal(read_png(tmp_path / "f.png"), want)


def test_writer_rejects_bad_images(rt, tmp_path):
    import ctypes
    img = rt.RtImage(None, 4, 4, rt.RT_FORMAT_R8G8B8A8_U32)
    assert rt.lib().rt_image_write_ppm(ctypes.byref(img), str(tmp_path / "x.ppm").encode(), 0) == -22
    buf = np.zeros((4, 4, 4), np.float32)
    img = rt.RtImage(buf.ctypes.data, 4, 4, rt.RT_FORMAT_R32B32G32A32_F32)  # the f32 accumulation is not RGBA8
    assert rt.lib().rt_image_write_png(ctypes.byref(img), str(tmp_path / "x.png").encode(), 0) == -22
    img = rt.RtImage(buf.ctypes.data, 4, 4, rt.RT_FORMAT_R8G8B8A8_U32)
    assert rt.lib().rt_image_write_ppm(ctypes.byref(img), b"/nonexistent-dir/x.ppm", 0) == -5
