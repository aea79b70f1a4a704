"""Known-answer tests of the computed textures, restated here from the Haskell
source alone and compared BIT FOR BIT with the oracle (which the HIP core is checked against):

  * Worley cellNoise, all four distances        Texture.hs:256-315 (lcg, hash, prob, cellPoints)
  * spectrumBlend                               Texture.hs:135-145
  * gradient (mkGradient: stable sort by pos)   Texture.hs:225-250
  * checkerBoard over a graphPaper child        Texture.hs:191-219

Haskell Int is 64-bit with wrap-around (restated with Python ints reduced mod 2^64); Float
arithmetic is numpy binary32 in GHC's left-to-right order.  The scenes: the reference's own
cellnoise.bling (X10, as shipped) and this repository's procedural-textures.bling (X11)."""
import ctypes
import math

import numpy as np
import pytest

import oracle_py
from bling_amd.scene import load_config
from scene_desc import arr, desc
from test_kat_hotpath import fp, trans_point

f32 = np.float32
M32 = 4294967296
BLEND, GRADIENT, CHECKER, GRAPHPAPER, CONST = 2, 3, 4, 1, 0
S_CONST, S_SCALE, S_CELL = 0, 1, 4


def wrap64(x):                                            # Haskell Int arithmetic
    return ((x + (1 << 63)) % (1 << 64)) - (1 << 63)


def rem(a, b):                                            # `rem`: truncates toward zero
    r = abs(a) % b
    return r if a >= 0 else -r


def lcg(x):                                               # Texture.hs:298-299
    return rem(wrap64(1103515245 * x + 12345), M32)


def hash3(x, y, z):                                       # Texture.hs:301-302
    h = wrap64(wrap64(x * 73856093) ^ wrap64(y * 19349663) ^ wrap64(z * 83492791))
    return rem(wrap64(abs(h)), M32)


PROB = [393325350, 1022645910, 1861739990, 2700834071, 3372109335, 3819626178, 4075350088, 4203212043]


def prob(v):                                              # Texture.hs:305-315
    for k, t in enumerate(PROB):
        if v < t:
            return k + 1
    return 9


def ghc_min(a, b):
    return a if a <= b else b


def ghc_max(a, b):
    return b if a <= b else a


def dist_fn(kind, a, b):                                  # Texture.hs:259-271 (sqLen = x*x + y*y + z*z)
    d = (f32(a[0] - b[0]), f32(a[1] - b[1]), f32(a[2] - b[2]))
    if kind in (0, 1):
        q = f32(f32(f32(d[0] * d[0]) + f32(d[1] * d[1])) + f32(d[2] * d[2]))
        return q if kind == 1 else f32(np.sqrt(q))
    ad = [f32(abs(v)) for v in d]
    if kind == 2:
        return f32(f32(ad[0] + ad[1]) + ad[2])
    return ghc_max(ghc_max(ad[0], ad[1]), ad[2])           # maximum = foldl1 max


def cell_noise(kind, p):                                  # cellNoise dist m dg, Texture.hs:274-296
    o = [math.floor(float(v)) for v in p]
    pts = []
    for x in (-1, 0, 1):
        for y in (-1, 0, 1):
            for z in (-1, 0, 1):
                cx, cy, cz = x + o[0], y + o[1], z + o[2]
                u = lcg(hash3(cx, cy, cz))
                for _ in range(prob(u)):                  # take n $ tail $ iterate go (undefined, us)
                    u1 = lcg(u)
                    u2 = lcg(u1)
                    u3 = lcg(u2)
                    pts.append((f32(f32(cx) + f32(f32(u1) / f32(M32))), f32(f32(cy) + f32(f32(u2) / f32(M32))),
                                f32(f32(cz) + f32(f32(u3) / f32(M32)))))
                    u = u3
    ds = [dist_fn(kind, p, q) for q in pts]
    m = ds[0]
    for d in ds[1:]:                                      # minimum = foldl1 min
        m = ghc_min(m, d)
    return m


def stex_value(d, ti, p, orc):
    """A scalar texture: cellNoise restated here, a scale chain restated over it; other leaves (fBm,
    Perlin, pinned by tests/test_heightmap.py) taken from the oracle."""
    t = d.scalar_textures[ti]
    if t.kind == S_CONST:
        return f32(t.value)
    if t.kind == S_SCALE:
        return f32(f32(t.a) + f32(f32(t.s) * stex_value(d, t.child, p, orc)))
    if t.kind == S_CELL:
        return cell_noise(t.octaves, trans_point(arr(t.w2t), p))
    return f32(oracle_py.lib().oracle_stex_probe(orc.h, ti, fp(p)))


def graph_paper(d, ti, u, v):                             # Texture.hs:191-207 (properFraction)
    while d.textures[ti].kind == GRAPHPAPER:
        t = d.textures[ti]
        x = f32(f32(f32(t.uv_map[0]) * u) + f32(t.uv_map[2]))
        z = f32(f32(f32(t.uv_map[1]) * v) + f32(t.uv_map[3]))
        xf, zf = f32(abs(f32(x - f32(math.trunc(float(x)))))), f32(abs(f32(z - f32(math.trunc(float(z))))))
        lo = f32(f32(t.line_width) / f32(2))
        hi = f32(f32(1) - lo)
        ti = t.tex2 if (xf < lo or zf < lo or xf > hi or zf > hi) else t.tex1
    return arr(d.textures[ti].value)


def spectrum_value(d, ti, p, u, v, orc):
    t = d.textures[ti]
    if t.kind == BLEND:                                   # spectrumBlend
        v1, v2 = graph_paper(d, t.tex1, u, v), graph_paper(d, t.tex2, u, v)
        x = stex_value(d, t.stex, p, orc)
        if x <= 0:
            return v1
        if x >= 1:
            return v2
        return (v1 * f32(f32(1) - x)).astype(np.float32) + (v2 * x).astype(np.float32)
    if t.kind == GRADIENT:                                # gradient (steps sorted at load)
        f = stex_value(d, t.stex, p, orc)
        steps = [(f32(d.textures[t.tex1 + k].line_width), arr(d.textures[t.tex1 + k].value)) for k in range(t.tex2)]
        ps = [s[0] for s in steps]
        if f <= min(ps):
            return steps[0][1]
        if f >= max(ps):
            return steps[-1][1]
        idx = next(k for k, s in enumerate(steps) if s[0] > f)
        (p0, c0), (p1, c1) = steps[idx - 1], steps[idx]
        w = f32(f32(f - p0) / f32(p1 - p0))
        return (c0 * f32(f32(1) - w)).astype(np.float32) + (c1 * w).astype(np.float32)
    if t.kind == CHECKER:                                 # checkerBoard: floor (x * sx) + ... `mod` 2
        s = sum(math.floor(float(f32(p[a] * f32(t.uv_map[a])))) for a in range(3))
        return graph_paper(d, t.tex1 if s % 2 == 0 else t.tex2, u, v)
    return graph_paper(d, ti, u, v)


@pytest.mark.parametrize("name", ["X10", "X11"])
def test_cell_noise_kat(name):
    job = load_config(name)
    d = desc(job)
    orc = oracle_py.Oracle(job)
    rng = np.random.default_rng(5)
    cells = [i for i in range(d.num_scalar_textures) if d.scalar_textures[i].kind == S_CELL]
    kinds = {d.scalar_textures[i].octaves for i in cells}
    assert kinds == {0, 1, 2, 3}                          # euclidian, euclidian2, manhattan, chebyshev
    pts = rng.uniform(-6, 6, size=(120, 3)).astype(np.float32)
    pts[:8] = np.floor(pts[:8])                           # points on cell corners
    for ti in cells:
        for p in pts:
            got = f32(oracle_py.lib().oracle_stex_probe(orc.h, ti, fp(p)))
            want = stex_value(d, ti, p, orc)
            assert got.tobytes() == want.tobytes(), (name, ti, p, got, want)


def test_computed_spectra_kat():
    job = load_config("X11")
    d = desc(job)
    orc = oracle_py.Oracle(job)
    rng = np.random.default_rng(6)
    comp = [i for i in range(d.num_textures) if d.textures[i].kind >= BLEND]
    assert {d.textures[i].kind for i in comp} == {BLEND, GRADIENT, CHECKER}
    interior = 0
    for ti in comp:
        for _ in range(150):
            p = rng.uniform(-4, 4, size=3).astype(np.float32)
            u, v = rng.uniform(0, 1, size=2).astype(np.float32)
            out = np.zeros(16, np.float32)
            oracle_py.lib().oracle_spectrum_probe(orc.h, ti, fp(p), u, v, fp(out))
            want = spectrum_value(d, ti, p, u, v, orc)
            np.testing.assert_array_equal(out, want, err_msg=f"texture {ti} at {p} ({u}, {v})")
            t = d.textures[ti]
            if t.kind in (BLEND, GRADIENT):
                x = stex_value(d, t.stex, p, orc)
                lo, hi = (0, 1) if t.kind == BLEND else (d.textures[t.tex1].line_width,
                                                         d.textures[t.tex1 + t.tex2 - 1].line_width)
                interior += int(lo < x < hi)
    assert interior > 100                                 # the interpolating branches were exercised


def test_gradient_steps_sorted_stably():
    """mkGradient sorts the steps by position (sortBy, stable); X11's plastic kd lists 0.6, 0, 0.3."""
    d = desc(load_config("X11"))
    grads = [d.textures[i] for i in range(d.num_textures) if d.textures[i].kind == GRADIENT]
    pos = [[d.textures[g.tex1 + k].line_width for k in range(g.tex2)] for g in grads]
    assert [0.0, pytest.approx(0.3), pytest.approx(0.6)] == pos[0]
    assert all(p == sorted(p) for p in pos)
    assert [len(p) for p in pos] == [3, 2, 1]


# ---------------------------------------------------------------- quasiCrystal (Texture.hs:317-338)
_libm = ctypes.CDLL("libm.so.6")
for _fn in ("cosf", "sinf"):
    getattr(_libm, _fn).restype = ctypes.c_float
    getattr(_libm, _fn).argtypes = [ctypes.c_float]
S_CRYSTAL = 5


def crystal_angles(o):
    """take o $ enumFromThen 0 (pi / fromIntegral o), GHC's numericEnumFromThen n m = n : (m, m+m-n)."""
    a0, a1 = f32(0), f32(f32(np.pi) / f32(o))
    out = []
    for _ in range(o):
        out.append(a0)
        a0, a1 = a1, f32(f32(a1 + a1) - a0)
    return out


def quasi_crystal(t, rec, p):
    m = arr(t.w2t)
    x = f32(f32(f32(f32(p[0] * m[0]) + f32(p[1] * m[1])) + f32(p[2] * m[2])) + m[6])   # planarMapping
    y = f32(f32(f32(f32(p[0] * m[3]) + f32(p[1] * m[4])) + f32(p[2] * m[5])) + m[7])
    s = f32(0)
    for (c, sn) in rec:                                   # sum . sequence (map wave angles), foldl (+) 0
        arg = f32(f32(c * x) + f32(sn * y))
        w = f32(f32(f32(oracle_py.cr_eval("cos", np.array([arg], np.float32))[0]) + f32(1)) / f32(2))   # cr_math.h's cos
        s = f32(s + w)
    k = math.trunc(float(s))                              # properFraction, aux, wrap
    v = f32(s - f32(k))
    if v < 0:
        k, v = k - 1, f32(f32(1) + v)
    return f32(f32(1) - v) if k % 2 else v


def test_quasi_crystal_kat():
    job = load_config("X12")
    d = desc(job)
    orc = oracle_py.Oracle(job)
    cr = [i for i in range(d.num_scalar_textures) if d.scalar_textures[i].kind == S_CRYSTAL]
    assert len(cr) == 1                                   # the ground of crystal.bling
    rng = np.random.default_rng(8)
    for ti in cr:
        t = d.scalar_textures[ti]
        assert t.octaves == 17
        ang = crystal_angles(t.octaves)
        rec = [(f32(d.scalar_textures[t.child + k].a), f32(d.scalar_textures[t.child + k].s)) for k in range(t.octaves)]
        assert rec == [(f32(_libm.cosf(float(a))), f32(_libm.sinf(float(a)))) for a in ang]   # GHC cos / sin = libm
        for _ in range(300):
            p = rng.uniform(-12, 12, size=3).astype(np.float32)
            got = f32(oracle_py.lib().oracle_stex_probe(orc.h, ti, fp(p)))
            want = quasi_crystal(t, rec, p)
            assert got.tobytes() == want.tobytes(), (ti, p, got, want)


@pytest.mark.parametrize("name", ["X9", "X10"])
def test_bump_kat(name):
    """bump (Reflection.hs:347-377), restated in numpy binary32 from the Haskell: the displacement at
    p, p + du dpdu and p + dv dpdv (du = dv = 0.01), dpdu / dpdv tilted along the shading normal by the
    finite differences, the new normal normalize (cross dpdu' dpdv') faced to the geometric normal.
    X9 = the reference's bumpmap.bling (fBm bump on metal), X10 = its cellnoise.bling (cellNoise
    bumps); the displacement values come from stex_value (cellNoise restated above, fBm pinned by
    tests/test_heightmap.py).  Bit-exact against the oracle, which the HIP core is checked against."""
    from test_kat_hotpath import cross, dot, normalize, V
    job = load_config(name)
    d = desc(job)
    orc = oracle_py.Oracle(job)
    bumps = sorted({d.materials[m].stex[3] for m in range(d.num_materials) if d.materials[m].stex[3] >= 0})
    assert bumps, name
    rng = np.random.default_rng(11)
    du = f32(0.01)
    n_checked = 0
    for ti in bumps:
        for _ in range(64):
            p = rng.uniform(-3, 3, 3).astype(np.float32)
            ng = normalize(rng.normal(size=3).astype(np.float32))
            dpdu = rng.normal(size=3).astype(np.float32)
            dpdv = rng.normal(size=3).astype(np.float32)
            ns = normalize(cross(dpdu, dpdv))
            if rng.uniform() < 0.5:
                ns = (-ns).astype(np.float32)
            add = lambda a, b: np.array([f32(a[k] + b[k]) for k in range(3)], np.float32)
            smul = lambda s, v: np.array([f32(s * v[k]) for k in range(3)], np.float32)
            u_disp = stex_value(d, ti, add(p, smul(du, dpdu)), orc)
            v_disp = stex_value(d, ti, add(p, smul(du, dpdv)), orc)
            disp = stex_value(d, ti, p, orc)
            vscale = f32(f32(v_disp - disp) / du)
            dpdv2 = add(dpdv, smul(vscale, ns))
            uscale = f32(f32(u_disp - disp) / du)
            dpdu2 = add(dpdu, smul(uscale, ns))
            nn1 = normalize(cross(dpdu2, dpdv2))
            n2 = (-nn1).astype(np.float32) if dot(nn1, ng) < 0 else nn1     # faceForward nn' (dgN dgg)
            inp = np.concatenate([ng, p, ns, dpdu, dpdv]).astype(np.float32)
            out = np.zeros(9, np.float32)
            oracle_py.lib().oracle_bump_probe(orc.h, ti, fp(inp), fp(out))
            want = np.concatenate([n2, dpdu2, dpdv2]).astype(np.float32)
            assert out.tobytes() == want.tobytes(), (name, ti, out, want)
            n_checked += 1
    assert n_checked >= 64
