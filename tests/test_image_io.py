"""Texture images and image environment maps (feature scenes X14 / X15): the loader's PNG and
Radiance RGBE readers (bling_amd/csrc/host/image_io.h, restating what JuicyPixels' readImage /
decodeImage hand the reference: IO/Bitmap.hs:13-29, Texture.hs:87-126), the texel tables folded at
parse time, and the oracle's lookups through the 2d mappings (Texture.hs:91-108, 128-129, 164-179)
and rgbfToTexMap (IO/Bitmap.hs:22-29).

The images are the synthetic fixtures of tools/make_texture_fixtures.py; its images() returns their
exact pixel contents, so every decoder path (all five PNG row filters, Adam7, palette, greyscale,
run-length and flat RGBE scanlines, e = 0 pixels) is checked against known data, and the texels
against independent numpy restatements of pixelSpectrum (rgbToSpectrumRefl . unGamma) and
rgbToSpectrumIllum (Spectrum.hs:118-159).  JuicyPixels itself is absent (a Hackage dependency), so
the decoders are pinned by these round trips, not by the reference's own outputs.
"""
import ctypes as C
import os
import re
import sys

import numpy as np
import pytest

import oracle_py
from bling_amd.scene import Job, ParseError, load_config
from scene_desc import arr, desc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import make_texture_fixtures as mtf  # noqa: E402

f32 = np.float32
fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
SCENES = os.path.join(ROOT, "fixtures", "scenes")


def _table(name):
    text = open(os.path.join(ROOT, "bling_amd", "csrc", "common", "spectral_data.h")).read()
    body = re.search(name + r"\[[^=]*=\s*\{(.*?)\};", text, re.S).group(1)
    return np.array([float.fromhex(x.rstrip("f")) for x in re.findall(r"-?0x[0-9a-fA-F.]+p[+-]?\d+f?", body)], f32)


def rgb_to_spectrum(bands, r, g, b):
    """rgbToSpectrum (Spectrum.hs:146-159) in binary32, bases r, g, b, c, m, y, w."""
    rb, gb, bb, cb, mb, yb, wb = bands.reshape(7, 16)
    r, g, b = f32(r), f32(g), f32(b)

    def ss(base, k):
        return (base * f32(k)).astype(f32)

    def add(a, c):
        return (a + c).astype(f32)
    if r <= g and r <= b:
        return add(ss(wb, r), add(ss(cb, g - r), ss(bb, b - g)) if g <= b else add(ss(cb, b - r), ss(gb, g - b)))
    if g <= r and g <= b:
        return add(ss(wb, g), add(ss(mb, r - g), ss(bb, b - r)) if r <= b else add(ss(mb, b - g), ss(rb, r - b)))
    return add(ss(wb, b), add(ss(yb, r - b), ss(gb, g - r)) if r <= b else add(ss(yb, g - b), ss(rb, r - g)))


def ungamma_lut():
    """unGamma of fromIntegral c / 255 (Texture.hs:88-89, Spectrum.hs:118-120): (c / 255) ** 2.2 in
    binary32, the power correctly rounded (binary64 pow rounded once)."""
    x = (np.arange(256, dtype=f32) / f32(255)).astype(f32)
    return np.power(x.astype(np.float64), float(f32(2.2))).astype(f32)


def pixel_rgb8(name):
    px, kind, extra = mtf.images()[name]
    if kind == 3:
        return extra[px[..., 0]]                      # palette -> RGB8
    return px[..., :3]                                # RGBA: dropTransparency


def rgbe_to_rgbf(e):
    """Radiance RGBE -> RGBF: c * 2^(e - 136), e = 0 -> 0."""
    s = np.where(e[..., 3] == 0, 0.0, np.ldexp(1.0, e[..., 3].astype(np.int32) - 136))
    return (e[..., :3].astype(np.float64) * s[..., None]).astype(f32)


def image_texels(d, k):
    im = d.images[k]
    n = im.width * im.height * im.channels
    return np.ctypeslib.as_array(im.texels, shape=(n,)).copy().reshape(im.height, im.width, im.channels)


@pytest.fixture(scope="module")
def x14():
    job = load_config("X14")
    return job, desc(job)


def find_image(d, w, h, ch):
    for k in range(d.num_images):
        im = d.images[k]
        if (im.width, im.height, im.channels) == (w, h, ch):
            return k
    raise KeyError((w, h, ch))


@pytest.mark.parametrize("name", ["textures/checker-rgb.png", "textures/tiles-rgba-i.png", "textures/palette.png"])
def test_png_spectral_texels(x14, name):
    """RGB8 (all five row filters), interlaced RGBA8 and palette PNGs -> pixelSpectrum texels."""
    _, d = x14
    rgb = pixel_rgb8(name)
    h, w, _ = rgb.shape
    tx = image_texels(d, find_image(d, w, h, 16))
    lut = ungamma_lut()
    refl = _table("BLING_RGB_REFL_BANDS")
    for y in range(h):
        for x in range(w):
            r, g, b = (lut[int(c)] for c in rgb[y, x])
            np.testing.assert_array_equal(tx[y, x], rgb_to_spectrum(refl, r, g, b), err_msg=f"{name} ({x}, {y})")


def test_png_greyscale_texels(x14):
    """A Y8 PNG as getPixelScalar values c / 255 (Texture.hs:103-108)."""
    _, d = x14
    px = mtf.images()["textures/height-y8.png"][0][..., 0]
    tx = image_texels(d, find_image(d, 32, 32, 1))[..., 0]
    np.testing.assert_array_equal(tx, (px.astype(f32) / f32(255)).astype(f32))


def test_hdr_env_texels_and_dist(x14):
    """The RGBE map (run-length and flat scanlines, e = 0 pixels) as rgbToSpectrumIllum texels, and
    mkInfiniteAreaLight's Dist2D function sY (eval (x / w, y / h)) over them (Light.hs:72-82)."""
    _, d = x14
    L = d.lights[0]
    assert (L.kind, L.env_kind, L.env_w, L.env_h) == (2, 2, 64, 32)
    rgbf = rgbe_to_rgbf(mtf.images()["envmaps/sky-synth.hdr"][0])
    assert (rgbf == 0).all(axis=-1).sum() == 16 and rgbf.max() > 40
    tx = np.ctypeslib.as_array(L.env_texels, shape=(64 * 32 * 16,)).reshape(32, 64, 16)
    illum = _table("BLING_RGB_ILLUM_BANDS")
    for y in range(32):
        for x in range(64):
            np.testing.assert_array_equal(tx[y, x], rgb_to_spectrum(illum, *rgbf[y, x]), err_msg=f"({x}, {y})")
    # Dist2D: nu x nv = texSize; func[v][u] = sY of the texel of Cartesian (u / 64, v / 32)
    assert (L.dist_nu, L.dist_nv) == (64, 32)
    func = np.ctypeslib.as_array(L.dist_func, shape=(64 * 32,)).reshape(32, 64)
    text = open(os.path.join(ROOT, "bling_amd", "csrc", "common", "spectral_data.h")).read()
    ybands = _table("BLING_CIE_Y_BANDS")
    ysum = f32(float.fromhex(re.search(r"BLING_CIE_Y_SUM = (\S+)f;", text).group(1)))
    for v in range(32):
        for u in range(64):
            x = min(63, max(0, int(np.floor(f32(f32(1) - f32(f32(u) / f32(64))) * f32(64)))))
            y = min(31, max(0, int(np.floor(f32(f32(1) - f32(f32(v) / f32(32))) * f32(32)))))
            acc = f32(0)
            for i in range(16):
                acc = f32(acc + f32(tx[y, x, i] * ybands[i]))
            assert func[v, u] == f32(acc / ysum), (u, v)


def texel_index(w, h, s, t):
    """getPixel's wrapped pixel (Texture.hs:91-101): mod' (floor (u w)) w, mod' (floor (-v h)) h."""
    x = int(np.floor(f32(f32(s) * f32(w)))) % w
    y = int(np.floor(f32(f32(-f32(t)) * f32(h)))) % h
    return x, y


def test_image_texture_lookup(x14):
    """imageTexture through uvMapping (negative offsets wrap) and planarMapping, at the oracle."""
    job, d = x14
    orc = oracle_py.Oracle(job)
    lib = oracle_py.lib()
    rng = np.random.default_rng(5)
    checked = 0
    for ti in range(d.num_textures):
        t = d.textures[ti]
        if t.kind != 5:
            continue
        im = d.images[t.tex1]
        tx = image_texels(d, t.tex1)
        for _ in range(300):
            p = rng.uniform(-6, 6, 3).astype(f32)
            u, v = (f32(x) for x in rng.uniform(-1.5, 2.5, 2))
            if t.tex2 == 0:                                            # uv su sv ou ov
                m = arr(t.uv_map)
                s, tt = f32(f32(m[0] * u) + m[2]), f32(f32(m[1] * v) + m[3])
            else:                                                      # planar vu vv ou ov
                m = arr(t.value)[:8]
                s = f32(f32(f32(f32(p[0] * m[0]) + f32(p[1] * m[1])) + f32(p[2] * m[2])) + m[6])
                tt = f32(f32(f32(f32(p[0] * m[3]) + f32(p[1] * m[4])) + f32(p[2] * m[5])) + m[7])
            x, y = texel_index(im.width, im.height, s, tt)
            out = np.zeros(16, f32)
            lib.oracle_spectrum_probe(orc.h, ti, fp(p), u, v, fp(out))
            np.testing.assert_array_equal(out, tx[y, x], err_msg=f"texture {ti} at {p} ({u}, {v})")
            checked += 1
    assert checked >= 900                                              # uv, planar RGBA, palette, planar checker


def test_image_scalar_lookup(x14):
    """The bump map's scale 0 0.05 over a uv-mapped Y8 image (scaleTexture, Texture.hs:185)."""
    job, d = x14
    orc = oracle_py.Oracle(job)
    lib = oracle_py.lib()
    ks = [k for k in range(d.num_scalar_textures) if d.scalar_textures[k].kind == 6]
    assert len(ks) == 1
    img = d.scalar_textures[ks[0]]
    top = next(k for k in range(d.num_scalar_textures)
               if d.scalar_textures[k].kind == 1 and d.scalar_textures[k].child == ks[0])
    sc = d.scalar_textures[top]
    tx = image_texels(d, img.child)[..., 0]
    m = arr(img.w2t)
    rng = np.random.default_rng(6)
    for _ in range(300):
        p = rng.uniform(-3, 3, 3).astype(f32)
        u, v = (f32(x) for x in rng.uniform(-1, 2, 2))
        x, y = texel_index(32, 32, f32(f32(m[0] * u) + m[2]), f32(f32(m[1] * v) + m[3]))
        want = f32(f32(sc.a) + f32(f32(sc.s) * tx[y, x]))
        assert lib.oracle_stex_probe_uv(orc.h, top, fp(p), u, v) == want


def test_env_image_lookup(x14):
    """le of the image map at Cartesian (u, v): rgbfToTexMap's clamped pixel (IO/Bitmap.hs:22-29)."""
    job, d = x14
    orc = oracle_py.Oracle(job)
    lib = oracle_py.lib()
    L = d.lights[0]
    tx = np.ctypeslib.as_array(L.env_texels, shape=(64 * 32 * 16,)).reshape(32, 64, 16)
    for u in np.linspace(-0.1, 1.1, 41, dtype=f32):
        for v in np.linspace(-0.1, 1.1, 29, dtype=f32):
            x = min(63, max(0, int(np.floor(f32(f32(1) - u) * f32(64)))))
            y = min(31, max(0, int(np.floor(f32(f32(1) - v) * f32(32)))))
            out = np.zeros(16, f32)
            lib.oracle_env_probe(orc.h, 0, u, v, fp(out))
            np.testing.assert_array_equal(out, tx[y, x])


def test_x15_profile_and_features():
    """X15 runs the env map on a profile without per-hit textures (FT_ENV_IMG, no FT_PROCTEX)."""
    f = load_config("X15").counts()["features"]
    assert f & (1 << 20) and not f & (1 << 18) and not f & (1 << 7)
    f14 = load_config("X14").counts()["features"]
    assert f14 & (1 << 20) and f14 & (1 << 18) and f14 & (1 << 17)


def test_multi_light_feature_bit():
    """FT_MULTI_LIGHT (scene_features.h, bit 21) marks scenes with more than one light: the cornell
    kernel profile reads light 0 with wave-uniform scalar loads (dev_scene.h one_light), so only
    one-light scenes may run on it.  C2 (one area light) keeps the cornell profile's bits; X1 and X4
    (three lights) carry the bit and run on a profile that indexes lights per lane."""
    c2 = load_config("C2").counts()
    assert c2["lights"] == 1 and not c2["features"] & (1 << 21) and c2["features"] == 0x1041
    for name in ("X1", "X4"):
        k = load_config(name).counts()
        assert k["lights"] > 1 and k["features"] & (1 << 21)


def _scene_with(tmp_path, body):
    import shutil
    for sub in ("textures", "envmaps"):
        shutil.copytree(os.path.join(SCENES, sub), tmp_path / sub, dirs_exist_ok=True)
    p = tmp_path / "t.bling"
    p.write_text("imageSize 8 8\n" + body + "\nprim { shape { sphere radius 1 } }\n")
    return str(p)


@pytest.mark.parametrize("body,msg", [
    ('light { infinite { identity } l { rgbeFile "envmaps/sky-synth.hdr" } }', "unknown map type rgbeFile"),
    ('light { infinite { identity } l { file "textures/checker-rgb.png" } }', "can't convert image format"),
    ('material { matte kd { image { file "textures/height-y8.png" map { uv 1 1 0 0 } } } sigma { constant 0 } }',
     "unsupported image type"),
    ('material { bumpMap bump { image { file "textures/palette.png" map { uv 1 1 0 0 } } } matte kd { constant rgbR 1 1 1 } '
     'sigma { constant 0 } }', "unsupported image type"),
    ('material { matte kd { image { file "textures/missing.png" map { uv 1 1 0 0 } } } sigma { constant 0 } }',
     "cannot open"),
    ('material { matte kd { image { file "textures/checker-rgb.png" map { spherical } } } sigma { constant 0 } }',
     "unknown 2d mapping"),
])
def test_image_errors(tmp_path, body, msg):
    """Inputs the reference refuses (pDiscSpectrumMap2d's `fail`, readTexture's Left, decodeImage's
    `error "unsupported image type"`) are refused at load with the reason."""
    with pytest.raises(ParseError, match=re.escape(msg)):
        Job(_scene_with(tmp_path, body))


def test_png_bad_bytes(tmp_path):
    """Truncated and 16-bit PNGs, JPEG and unknown files are refused by the reader."""
    src = open(os.path.join(SCENES, "textures", "checker-rgb.png"), "rb").read()
    ihdr16 = bytearray(src)
    ihdr16[24] = 16                                                     # bit depth byte of IHDR
    cases = {"trunc.png": src[:60], "deep.png": bytes(ihdr16), "x.jpg": b"\xff\xd8\xff\xe0" + b"\0" * 40,
             "x.bin": b"hello world"}
    for fn, data in cases.items():
        (tmp_path / fn).write_bytes(data)
        p = tmp_path / "t.bling"
        p.write_text(f'imageSize 8 8\nmaterial {{ matte kd {{ image {{ file "{fn}" map {{ uv 1 1 0 0 }} }} }} '
                     'sigma { constant 0 } }\nprim { shape { sphere radius 1 } }\n')
        with pytest.raises(ParseError):
            Job(str(p))


def _refix_ihdr(buf: bytearray):
    import zlib
    crc = zlib.crc32(bytes(buf[12:29])) & 0xFFFFFFFF                    # IHDR type + 13 data bytes
    buf[29:33] = crc.to_bytes(4, "big")
    return buf


@pytest.mark.parametrize("what,msg", [("interlace", "unknown PNG interlace method"), ("crc", "PNG chunk CRC mismatch")])
def test_png_rejects_bad_interlace_and_crc(tmp_path, what, msg):
    """An IHDR interlace method other than 0 / 1 (PNG spec 11.2.2) and a chunk whose CRC does not
    match are refused with their reason, not decoded (image_io.h)."""
    buf = bytearray(open(os.path.join(SCENES, "textures", "checker-rgb.png"), "rb").read())
    if what == "interlace":
        buf[28] = 2                                                     # interlace byte of IHDR
        _refix_ihdr(buf)
    else:
        buf[30] ^= 0xFF                                                 # IHDR CRC
    (tmp_path / "bad.png").write_bytes(bytes(buf))
    p = tmp_path / "t.bling"
    p.write_text('imageSize 8 8\nmaterial { matte kd { image { file "bad.png" map { uv 1 1 0 0 } } } '
                 'sigma { constant 0 } }\nprim { shape { sphere radius 1 } }\n')
    with pytest.raises(ParseError, match=re.escape(msg)):
        Job(str(p))
