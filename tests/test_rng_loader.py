"""Sampler RNG specification and scene-loader invariants (CPU only).

* The counter RNG (bling_amd/csrc/common/counter_rng.h, DESIGN.md "Sampler RNG") is restated here in
  pure Python and checked word-for-word against the oracle's build of the same header; the device
  includes that header unchanged, so the three agree by construction and by this test.
* Stratification properties the reference's Sampling.hs guarantees for every pixel (stratified1D /
  stratified2D strata, Sampling.hs:157-171, shuffled per pixel, :294-311) hold for the counter-RNG
  sampler.  The reference's own tests hold only `prop_rndIn01` and `prop_shuffle_retains`
  (L/Main/Tests.hs:24-41): their counterparts are test_u01_range and test_permute_is_bijection.
* Loader: the five BASELINE configs parse to the primitive counts and camera-sample counts of
  SURVEY.md 8(a)/(d) (C3 carries trap T15)."""
import numpy as np
import pytest

import oracle_py
from bling_amd.scene import CONFIGS, ParseError, load_config, parse_job

M = 0xFFFFFFFF


def rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & M


def mix(h, k):
    k = (k * 0xcc9e2d51) & M
    k = rotl(k, 15)
    k = (k * 0x1b873593) & M
    h ^= k
    h = rotl(h, 13)
    return (h * 5 + 0xe6546b64) & M


def fmix(h):
    h ^= h >> 16
    h = (h * 0x85ebca6b) & M
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & M
    h ^= h >> 16
    return h


def hash5(seed, pss, pixel, sample, dim):
    """Specification version 2 (counter_rng.h): pixel key, sample key, dimension key."""
    pkey = mix(mix(seed, pss), pixel)
    skey = fmix(pkey ^ ((sample * 0x9E3779B9) & M))
    return fmix(skey ^ fmix(dim ^ 0x2C1B3C6D))


def permute(i, l, p):
    if l <= 1:
        return 0
    w = l - 1
    for s in (1, 2, 4, 8, 16):
        w |= w >> s
    while True:
        i ^= p; i = (i * 0xe170893d) & M; i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8
        i = (i * 0x0929eb3f) & M; i ^= p >> 23; i ^= (i & w) >> 1; i = (i * (1 | p >> 27)) & M
        i = (i * 0x6935fa69) & M; i ^= (i & w) >> 11; i = (i * 0x74dcb303) & M; i ^= (i & w) >> 2
        i = (i * 0x9e501cc3) & M; i ^= (i & w) >> 2; i = (i * 0xc860a3df) & M; i &= w; i ^= i >> 5
        if i < l:
            break
    return (i + p) % l


def test_hash5_matches_spec():
    rng = np.random.default_rng(5)
    for _ in range(2000):
        k = [int(v) for v in rng.integers(0, 2**32, 5, dtype=np.uint64)]
        assert oracle_py.hash5(*k) == hash5(*k)


def test_permute_matches_spec():
    rng = np.random.default_rng(6)
    for _ in range(2000):
        l = int(rng.integers(1, 5000))
        i = int(rng.integers(0, l))
        p = int(rng.integers(0, 2**32, dtype=np.uint64))
        assert oracle_py.permute(i, l, p) == permute(i, l, p)


def _permute24(i, l, p):
    """counter_rng.h permute_w as the device computes it: every product through v_mul_u32_u24, the low
    32 bits of (a mod 2^24)(c mod 2^24)."""
    def m24(a, c):
        return ((a & 0xFFFFFF) * (c & 0xFFFFFF)) & M
    if l <= 1:
        return 0
    w = l - 1
    for s in (1, 2, 4, 8, 16):
        w |= w >> s
    while True:
        i ^= p; i = m24(i, 0xe170893d); i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8
        i = m24(i, 0x0929eb3f); i ^= p >> 23; i ^= (i & w) >> 1; i = m24(i, 1 | p >> 27)
        i = m24(i, 0x6935fa69); i ^= (i & w) >> 11; i = m24(i, 0x74dcb303); i ^= (i & w) >> 2
        i = m24(i, 0x9e501cc3); i ^= (i & w) >> 2; i = m24(i, 0xc860a3df); i &= w; i ^= i >> 5
        if i < l:
            break
    return (i + p) % l


def test_permute_mul24_is_the_32bit_permute():
    """The device's permutation multiplies with 24-bit operands (full rate on gfx950); every product
    is masked to l - 1's bit width (<= 24 bits) before use, so for l <= 2^24 it is Kensler's 32-bit
    permutation bit for bit (the spec: counter_rng.h permute_w)."""
    rng = np.random.default_rng(8)
    for l in [2, 3, 64, 100, 1024, 4097, 1 << 16, (1 << 20) + 3, 1 << 24]:
        for _ in range(300):
            i = int(rng.integers(0, l))
            p = int(rng.integers(0, 2**32, dtype=np.uint64))
            assert _permute24(i, l, p) == permute(i, l, p) == oracle_py.permute(i, l, p), (i, l, p)


@pytest.mark.parametrize("l", [1, 2, 3, 4, 9, 64, 100, 256, 1000, 1024])
def test_permute_is_bijection(l):
    for p in (0, 1, 0xDEADBEEF, 0x0B11A6):
        img = sorted(oracle_py.permute(i, l, p) for i in range(l))
        assert img == list(range(l))


def test_u01_range():
    vals = [(hash5(0x0B11A6, 0, px, 0, 7) >> 8) / 16777216.0 for px in range(20000)]
    assert min(vals) >= 0.0 and max(vals) < 1.0


@pytest.fixture(scope="module")
def c1():
    job = load_config("C1", "image=32,32")
    return job, oracle_py.Oracle(job)


def test_stratified_1d_dims_cover_strata(c1):
    job, orc = c1
    spp = job.spp
    for dim in (0, 1, 5, 11):
        for (px, py) in ((0, 0), (7, 3), (31, 31)):
            v = np.array([orc.sampler_probe(px, py, n, 0, dim)[0] for n in range(spp)])
            assert ((v >= 0) & (v < 1)).all()
            assert sorted(np.floor(v * spp).astype(int)) == list(range(spp)), (dim, px, py, v)


def test_pixel_offsets_stratified_in_index_order(c1):
    """Camera offsets: sample n lies in stratum (u, v) = n `quotRem` nu (Sampling.hs:167-171)."""
    job, orc = c1
    nu = nv = 2
    for n in range(job.spp):
        ox, oy, lu, lv = orc.sampler_probe(5, 6, n, 2)
        assert int(np.floor(ox * nu)) == n // nu and int(np.floor(oy * nv)) == n % nu, (n, ox, oy)
        assert 0 <= lu < 1 and 0 <= lv < 1


def test_samples_differ_across_passes_and_seeds(c1):
    _, orc = c1
    a = orc.sampler_probe(3, 3, 1, 0, 2, seed=1, pass_index=0)[0]
    b = orc.sampler_probe(3, 3, 1, 0, 2, seed=1, pass_index=1)[0]
    c = orc.sampler_probe(3, 3, 1, 0, 2, seed=2, pass_index=0)[0]
    assert len({a, b, c}) == 3


# ---------------------------------------------------------------- loader
EXPECT = {  # SURVEY.md 8(a) a3/a10/a11 and 8(d); C3: T15 drops the last material run of ducky.obj
    "C1": dict(triangles=30, shapes=1, fractal=0, prims=31, lights=1, samples=272484, tiles=289),
    "C2": dict(triangles=30, shapes=1, fractal=0, prims=31, lights=1, samples=67765824, tiles=4225),
    "C3": dict(triangles=13456, shapes=1, fractal=0, prims=13457, lights=1, samples=536230144, tiles=8228),
    "C4": dict(triangles=0, shapes=4, fractal=0, prims=4, lights=1, samples=2157982208, tiles=16641),
    "C5": dict(triangles=0, shapes=1, fractal=1, prims=2, lights=1, samples=17221837824, tiles=66049),
}


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_config_counts(name):
    job = load_config(name)
    e = EXPECT[name]
    c = job.counts()
    for k in ("triangles", "shapes", "fractal", "prims", "lights"):
        assert c[k] == e[k], (k, c[k], e[k])
    assert job.camera_samples() == e["samples"]
    assert job.num_tiles() == e["tiles"]


def test_extent_matches_oracle():
    job = load_config("C1")
    orc = oracle_py.Oracle(job)
    ext, nt = orc.extent()
    assert tuple(ext) == job.extent() == (-2, 258, -2, 258)
    assert nt == job.num_tiles()


def test_parse_error_is_reported(tmp_path):
    bad = tmp_path / "bad.bling"
    bad.write_text("imageSize 10 10\ncamera { perspective fov }\n")
    with pytest.raises(ParseError):
        parse_job(str(bad))


def _fastdiv(d):
    """FastDiv::make (bling_amd/csrc/core/dev_scene.h), restated."""
    if d == 1:
        return None
    l = (d - 1).bit_length()                      # ceil(log2 d)
    m = ((((1 << l) - d) << 32) // d + 1) & 0xFFFFFFFF
    return m, l - 1


def test_fastdiv_is_exact():
    """The device's exact division by spp / nu (FastDiv) agrees with // for every divisor up to 4096
    and numerators spanning the whole 32-bit range (the (i + p) % spp of permute wraps)."""
    rng = np.random.default_rng(5)
    n = np.concatenate([np.arange(0, 5000, dtype=np.uint64), rng.integers(0, 2**32, 20000, dtype=np.uint64),
                        np.array([2**32 - 1, 2**32 - 2, 2**31, 2**31 - 1], dtype=np.uint64)])
    for d in list(range(1, 4097)) + [65536, 1 << 20, 1000003]:
        f = _fastdiv(d)
        if f is None:
            q = n
        else:
            m, s = f
            t = (np.uint64(m) * n) >> np.uint64(32)
            q = (t + ((n - t) >> np.uint64(1))) >> np.uint64(s)
        np.testing.assert_array_equal(q, n // np.uint64(d), err_msg=f"d={d}")


# ---------------------------------------------------------------- substrate, scalar textures, bumpMap
@pytest.mark.parametrize("name,bits", [("X7", 1 << 16), ("X8", 1 << 16), ("X9", 1 << 17), ("X10", 1 << 18),
                                       ("X11", 1 << 18), ("X12", 1 << 18), ("X13", 1 << 19),
                                       ("X14", 1 << 20), ("X15", 1 << 20)])
def test_loader_feature_bits_substrate_and_bump(name, bits):
    """pSubstrateMaterial with fbm / perlin / scale scalar textures (X7 and the reference's
    substrate.bling, X8) and pBumpMap (the reference's bumpmap.bling, X9) load and report their feature bit
    (scene_features.h: SUBSTRATE = 1 << 16, BUMP = 1 << 17), which selects the kernel profile."""
    info = load_config(name).counts()
    assert info["features"] & bits
    assert info["shapes"] >= 1 and info["lights"] >= 1


@pytest.mark.parametrize("tex,err", [
    ("blend tex1 { blend tex1 { constant rgbR 1 1 1 } tex2 { constant rgbR 0 0 0 } f { constant 0.5 } } "
     "tex2 { constant rgbR 0 0 0 } f { constant 0.5 }", "top of a material"),
    ("gradient f { constant 0.5 } steps { }", "empty list given to mkGradient"),
    ("gradient f { cellNoise taxicab map { identity { scale 1 1 1 } } } steps { 0 rgbR 1 1 1 }",
     "unknown distance function taxicab"),
])
def test_loader_rejects_bad_computed_textures(tmp_path, tex, err):
    """Computed spectrum textures sit at the top of a material's slot (their children are stored
    spectra), mkGradient refuses an empty list, cellNoise knows four distances (MaterialParser.hs:124-133)."""
    p = tmp_path / "t.bling"
    p.write_text("imageSize 8 8\ntransform { lookAt { pos 0 0 -5 look 0 0 0 up 0 1 0 } }\n"
                 "camera { perspective fov 45 lensRadius 0 focalDistance 10 }\n"
                 "material { matte kd { " + tex + " } sigma { constant 0 } }\n"
                 "prim { shape { sphere radius 1 } }\n")
    with pytest.raises(ParseError, match=err):
        parse_job(str(p))


@pytest.mark.parametrize("depth,ok", [(8, True), (9, False)])
def test_loader_bounds_nested_scale_textures(tmp_path, depth, ok):
    """A chain of nested `scale` scalar textures deeper than BLING_STEX_MAX_SCALE (8, the depth the
    device's eval_stex unwinds) is refused at load time instead of being evaluated differently by
    the device and the oracle (which recurses without a limit)."""
    import os
    from bling_amd.scene import SCENES, Job, ParseError
    src = open(os.path.join(SCENES, "bumpmap.bling")).read()
    inner = "fbm octaves 5 omega 0.5 map {\n      identity { scale 2 2 2 }\n   }"
    old = "bump { scale 0.1 0.1 tex { " + inner + "}}"
    assert old in src
    nest = inner
    for _ in range(depth):
        nest = "scale 0.1 0.1 tex { " + nest + " }"
    scene = tmp_path / "nested.bling"
    scene.write_text(src.replace(old, "bump { " + nest + " }"))
    if ok:
        Job(str(scene))
    else:
        with pytest.raises(ParseError, match="nested"):
            Job(str(scene))
