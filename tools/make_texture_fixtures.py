#!/usr/bin/env python3
"""Writes the synthetic texture images of feature scene X14 (fixtures/scenes/image-textures.bling).

The reference ships no texture image or environment map (its example scenes name .hdr files that are
not in the repository), so these are generated here, deterministically, with small independent
encoders (numpy, zlib, struct) that exercise every decoder path of bling_amd/csrc/host/image_io.h:
  textures/checker-rgb.png     24 x 16 RGB8, every PNG row filter (0..4 in turn)
  textures/tiles-rgba-i.png    13 x 11 RGBA8, Adam7 interlaced, rows filtered 4, 1, 2, 3, 0, ...
  textures/palette.png         10 x 10 palette (8 colours)
  textures/height-y8.png       32 x 32 greyscale (Y8), the bump map
  envmaps/sky-synth.hdr        64 x 32 Radiance RGBE: run-length scanlines except rows 5 and 17
                               (flat); a sky gradient, a ground and a bright sun patch
tests/test_image_io.py decodes the same files with an independent numpy reader and checks the
loader's texel tables against it.

  python tools/make_texture_fixtures.py [--out fixtures/scenes]
"""
import argparse
import os
import struct
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- PNG encoder
def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def _filter_rows(img: np.ndarray, bpp: int, filt) -> bytes:
    """img: (h, w*bpp) uint8; filt(y) -> filter type of row y."""
    h, stride = img.shape
    out = bytearray()
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        row = img[y].astype(np.int32)
        a = np.concatenate([np.zeros(bpp, np.int32), row[:-bpp]])
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        f = filt(y)
        if f == 0:
            r = row
        elif f == 1:
            r = row - a
        elif f == 2:
            r = row - prev
        elif f == 3:
            r = row - ((a + prev) >> 1)
        else:
            r = row - _paeth(a, prev, c)
        out.append(f)
        out += (r & 0xFF).astype(np.uint8).tobytes()
        prev = row
    return bytes(out)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def write_png(path: str, px: np.ndarray, ctype: int, palette=None, interlace=False, filt=lambda y: y % 5):
    """px: (h, w, c) uint8 samples as stored (palette: (h, w, 1) indices)."""
    h, w, c = px.shape
    if interlace:
        raw = b""
        k = 0
        for x0, y0, dx, dy in ADAM7:
            sub = px[y0::dy, x0::dx]
            if sub.size == 0:
                continue
            raw += _filter_rows(sub.reshape(sub.shape[0], -1), c, lambda y, k=k: (y + k) % 5)
            k += 1
    else:
        raw = _filter_rows(px.reshape(h, -1), c, filt)
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 1 if interlace else 0))
    if palette is not None:
        data += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    comp = zlib.compress(raw, 9)
    data += _chunk(b"IDAT", comp[: len(comp) // 2]) + _chunk(b"IDAT", comp[len(comp) // 2:])   # split IDAT
    data += _chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(data)


# ---------------------------------------------------------------- Radiance RGBE encoder
def to_rgbe(rgb: np.ndarray) -> np.ndarray:
    v = rgb.max(axis=-1)
    out = np.zeros(rgb.shape[:-1] + (4,), np.uint8)
    ok = v >= 1e-32
    m, e = np.frexp(v[ok])
    scale = m * 256.0 / v[ok]
    out[ok, :3] = np.floor(rgb[ok] * scale[:, None]).astype(np.uint8)
    out[ok, 3] = (e + 128).astype(np.uint8)
    return out


def _rle_plane(b: np.ndarray) -> bytes:
    out = bytearray()
    i, n = 0, len(b)
    while i < n:
        j = i
        while j < n and j - i < 127 and b[j] == b[i]:
            j += 1
        if j - i >= 3:
            out += bytes([128 + j - i, int(b[i])])
            i = j
            continue
        j = i                                       # literal run up to the next run of >= 3
        while j < n and j - i < 128 and not (j + 2 < n and b[j] == b[j + 1] == b[j + 2]):
            j += 1
        out += bytes([j - i]) + bytes(b[i:j].tolist())
        i = j
    return bytes(out)


def write_hdr(path: str, e: np.ndarray, flat_rows=()):
    """e: (h, w, 4) RGBE bytes."""
    h, w, _ = e.shape
    data = bytearray(b"#?RADIANCE\n# synthetic fixture (tools/make_texture_fixtures.py)\nFORMAT=32-bit_rle_rgbe\n\n")
    data += f"-Y {h} +X {w}\n".encode()
    for y in range(h):
        row = e[y]
        if y in flat_rows:
            assert not (row[0, 0] == 2 and row[0, 1] == 2) and not (row[:, :3] == 1).all(axis=1).any()
            data += row.tobytes()
            continue
        data += bytes([2, 2, w >> 8, w & 0xFF])
        for c in range(4):
            data += _rle_plane(row[:, c])
    with open(path, "wb") as fh:
        fh.write(bytes(data))


# ---------------------------------------------------------------- the images
def images():
    """name -> (pixel array as stored, PNG colour type or 'hdr', extra): the fixtures' exact contents."""
    rng = np.random.default_rng(0x7E47)
    out = {}
    # checker with a colour ramp (RGB8)
    y, x = np.mgrid[0:16, 0:24]
    chk = ((x // 4 + y // 4) & 1).astype(np.int32)
    rgb = np.stack([40 + 200 * chk + (x * 3) % 16, 60 + 120 * (1 - chk) + y * 4, 30 + (x * 7 + y * 5) % 200], -1)
    out["textures/checker-rgb.png"] = (np.clip(rgb, 0, 255).astype(np.uint8), 2, None)
    # tiles, RGBA, Adam7
    y, x = np.mgrid[0:11, 0:13]
    rgba = np.stack([(x * 19) % 256, (y * 23) % 256, ((x + y) * 11 + 90) % 256, 128 + (x * y) % 128], -1)
    out["textures/tiles-rgba-i.png"] = (rgba.astype(np.uint8), 6, "interlace")
    # palette image
    pal = rng.integers(0, 256, (8, 3)).astype(np.uint8)
    idx = ((np.arange(10)[:, None] * 3 + np.arange(10)[None, :]) % 8).astype(np.uint8)[..., None]
    out["textures/palette.png"] = (idx, 3, pal)
    # greyscale height map: smooth bumps
    y, x = np.mgrid[0:32, 0:32] / 32.0
    hm = 0.5 + 0.25 * np.sin(2 * np.pi * 3 * x) * np.cos(2 * np.pi * 2 * y) + 0.2 * rng.random((32, 32))
    out["textures/height-y8.png"] = (np.clip(hm * 255, 0, 255).astype(np.uint8)[..., None], 0, None)
    # environment: sky gradient over a ground, a sun patch (RGBE, mostly run-length rows)
    h, w = 32, 64
    v, u = (np.mgrid[0:h, 0:w] + 0.5) / np.array([h, w])[:, None, None]
    sky = np.stack([0.3 + 0.5 * v, 0.45 + 0.4 * v, 0.9 + 0.2 * v], -1) * 0.8
    ground = np.stack([0.25 + 0 * v, 0.2 + 0 * v, 0.15 + 0 * v], -1)
    env = np.where((v > 0.5)[..., None], sky, ground)
    env[(np.abs(u - 0.3) < 0.04) & (np.abs(v - 0.75) < 0.06)] = (60.0, 55.0, 45.0)
    env[20:22, 40:48] = 0.0                                         # exact zeros (e = 0 pixels)
    out["envmaps/sky-synth.hdr"] = (to_rgbe(env.astype(np.float32)), "hdr", (5, 17))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "fixtures", "scenes"))
    args = ap.parse_args()
    for name, (px, kind, extra) in images().items():
        path = os.path.join(args.out, name)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        if kind == "hdr":
            write_hdr(path, px, flat_rows=extra)
        elif kind == 3:
            write_png(path, px, 3, palette=extra)
        else:
            write_png(path, px, kind, interlace=extra == "interlace")
        print("wrote", path)


if __name__ == "__main__":
    main()
