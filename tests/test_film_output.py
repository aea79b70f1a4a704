"""Film output: the reference's tonemap and image writers.

The 8-bit pixels follow rgbPixels (Image.hs:317-331): getPixel (XYZ / W, splat weight 1 on an
empty splat buffer), xyzToRgb (Spectrum.hs:162-168), gamma 2.2 as Float `**`, clamp with GHC's
min / max, * 255, `round` half to even.  The restatement here is numpy binary32; libm powf and
numpy's float32 power may differ by an ulp, which can move a value across a .5 rounding edge, so
<= 0.1 % of channels may differ by 1 (parity of the formula, not of one libm).
The PNG container is checked by decoding it with zlib; the HDR by decoding RGBE.
"""
import os
import struct
import zlib

import numpy as np

from bling_amd import film


def _film(rng, w, h):
    f = np.zeros((h, w, 4), np.float32)
    f[..., 0] = rng.uniform(0.5, 4.0, (h, w))
    f[..., 1:] = rng.uniform(-0.05, 1.5, (h, w, 3)) * f[..., :1]
    f[0, 0] = 0.0                        # an empty pixel (W == 0 -> black)
    f[0, 1, 1:] = np.nan                 # NaN -> clamped to 0 by GHC max
    return f.reshape(-1)


def _rgb_ref(f, w, h):
    f = f.reshape(h, w, 4).astype(np.float32)
    W = f[..., 0]
    with np.errstate(divide="ignore", invalid="ignore"):
        iw = np.where(W != 0, np.float32(1) / W, np.float32(0)).astype(np.float32)
    x = np.where(W != 0, np.float32(0) * np.float32(0) + f[..., 1] * iw, 0).astype(np.float32)
    y = np.where(W != 0, np.float32(0) * np.float32(0) + f[..., 2] * iw, 0).astype(np.float32)
    z = np.where(W != 0, np.float32(0) * np.float32(0) + f[..., 3] * iw, 0).astype(np.float32)
    c = lambda v: np.float32(v)
    r = c(3.240479) * x - c(1.537150) * y - c(0.498535) * z
    g = c(-0.969256) * x + c(1.875991) * y + c(0.041556) * z
    b = c(0.055648) * x - c(0.204043) * y + c(1.057311) * z
    return np.stack([r, g, b], -1).astype(np.float32)


def _pixels_ref(rgb):
    with np.errstate(invalid="ignore"):
        gm = np.power(rgb, np.float32(1) / np.float32(2.2)).astype(np.float32)
    mx = np.where(np.float32(0) <= gm, gm, np.float32(0))          # max 0 v (NaN -> 0)
    mn = np.where(np.float32(1) <= mx, np.float32(1), mx)          # min 1 v
    return np.round((mn * np.float32(255)).astype(np.float32)).astype(np.uint8)   # half to even


def test_to_rgb_matches_getpixel_xyztorgb():
    rng = np.random.default_rng(1)
    w, h = 37, 23
    f = _film(rng, w, h)
    got = film.to_rgb(f, w, h)
    ref = _rgb_ref(f, w, h)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    np.testing.assert_array_equal(got[ok], ref[ok])


def test_rgb_pixels_match_rgbpixels_formula():
    rng = np.random.default_rng(2)
    w, h = 64, 48
    f = _film(rng, w, h)
    got = film.rgb_pixels(f, w, h).astype(int)
    ref = _pixels_ref(_rgb_ref(f, w, h)).astype(int)
    diff = np.abs(got - ref)
    assert diff.max() <= 1
    assert (diff > 0).mean() <= 1e-3
    assert (got[0, 0] == 0).all() and (got[0, 1] == 0).all()


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, ihdr = 8, b"", None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF, typ
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype = ihdr[:4]
    assert depth == 8 and ctype == 2
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 3 * w + 1)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 3)


def test_write_png_holds_rgb_pixels(tmp_path):
    rng = np.random.default_rng(3)
    w, h = 300, 250                       # > 65535 raw bytes: several stored deflate blocks
    f = _film(rng, w, h)
    p = str(tmp_path / "pass-00001.png")
    film.write_png(p, f, w, h)
    np.testing.assert_array_equal(_read_png(p), film.rgb_pixels(f, w, h))


def test_write_hdr_rgbe_roundtrip(tmp_path):
    rng = np.random.default_rng(4)
    w, h = 20, 10
    f = _film(rng, w, h)
    f[4:8] = [1.0, 0.5, 0.5, 0.5]
    p = str(tmp_path / "x.hdr")
    film.write_hdr(p, f, w, h)
    data = open(p, "rb").read()
    head, body = data.split(b"\n\n", 1)
    assert head.startswith(b"#?RADIANCE")
    dims, body = body.split(b"\n", 1)
    assert dims == f"-Y {h} +X {w}".encode()
    e = np.frombuffer(body, np.uint8).reshape(h, w, 4).astype(np.float64)
    dec = np.where(e[..., 3:] > 0, (e[..., :3] + 0.0) * np.ldexp(1.0, (e[..., 3:] - 136).astype(int)), 0.0)
    rgb = np.maximum(np.nan_to_num(film.to_rgb(f, w, h), nan=0.0), 0)
    big = rgb.max(-1, keepdims=True) > 1e-3
    rel = np.abs(dec - rgb) / np.maximum(rgb.max(-1, keepdims=True), 1e-9)
    assert (rel[big[..., 0]] <= 1 / 128).all()


def test_progress_writer_writes_numbered_pass_files(tmp_path):
    from bling_amd.render import Progress
    w, h = 8, 4
    rep = film.progress_writer(str(tmp_path / "out"), w, h)
    assert rep(Progress("Started"))
    assert rep(Progress("PassDone", 3, _film(np.random.default_rng(5), w, h)))
    assert os.path.exists(tmp_path / "out-00003.png") and os.path.exists(tmp_path / "out-00003.hdr")
