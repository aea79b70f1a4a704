"""Known-answer tests of the C2 hot path's formulas.

Each formula is restated here from the Haskell source alone, in numpy binary32 with GHC's
left-to-right evaluation and no fused multiply-add, and compared BIT FOR BIT with what the oracle
(oracle/oracle.cpp) or the loader (the flattened bling_scene_desc) computes.  Transcendentals:
GHC's Float `sin`, `cos`, `tan`, `acos`, `exp`, `**` are C sinf ... powf (libm binary32); the loader
keeps them for what it evaluates once per scene (camera, initSky, sunSpectrum'), while the
per-sample path (oracle and device alike) evaluates them in binary64 rounded once (common/cr_math.h,
round 3), whose departure from libm binary32 tests/test_cr_math.py measures:

  * Moller-Trumbore triangle hit / miss          TriangleMesh.hs:160-207
  * fromSpd band averaging of cornell's SPDs      Spectrum.hs:199-207, 291-335, ParserCore.hs:164-167
  * lookAt / perspective / invert / mkProjective  Transform.hs:37-101, 150-238; Camera.hs:108-147
    and fireRay (pinhole and thin lens)           Camera.hs:49-76, Montecarlo.hs:160-177
  * Oren-Nayar (sigma 0.5, cornell's white)       Reflection/Diffuse.hs:29-66
  * the quad area light's sampleShape' / shapePdf Shape.hs:157-171, 312-409; Light.hs:122-160, 215-229
    (trap T6: sampled normal -z, hit normal +z)
  * Blinn microfacet D / pdf / sample (plastic)   Reflection/Microfacet.hs:19-54, 113-195
  * Perez sky, initSky, sunSpectrum'              SunSky.hs:12-125, Spectrum.hs:143-168, 229-250

The oracle in turn is what the HIP core is checked against (tests/test_gpu_parity.py)."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

import oracle_py
from bling_amd.scene import SCENES, load_config
from scene_desc import arr, desc

f32 = np.float32
ONE, ZERO, TWO = f32(1), f32(0), f32(2)
PI = f32(np.pi)
_m = ctypes.CDLL("libm.so.6")
for _fn in ("sinf", "cosf", "tanf", "acosf", "expf", "atanf"):
    getattr(_m, _fn).restype = ctypes.c_float
    getattr(_m, _fn).argtypes = [ctypes.c_float]
_m.powf.restype = ctypes.c_float
_m.powf.argtypes = [ctypes.c_float, ctypes.c_float]


# GHC's Float transcendentals: libm binary32 -- what the host loader evaluates once per scene
# (camera construction, initSky, sunSpectrum'), unchanged from the reference
def sinf32(x): return f32(_m.sinf(float(x)))
def cosf32(x): return f32(_m.cosf(float(x)))
def tanf32(x): return f32(_m.tanf(float(x)))
def acosf32(x): return f32(_m.acosf(float(x)))
def expf32(x): return f32(_m.expf(float(x)))
def powf32(x, y): return f32(_m.powf(float(x), float(y)))


# the per-sample path's transcendentals (device and oracle, common/cr_math.h): binary64 rounded once
# to binary32 -- the correctly rounded value -- except exp, log, sinh, sin, cos, acos: faithful binary32
# algorithms (round 5), taken here from the shared implementation itself (tests/test_cr_math.py
# measures both kinds against binary64 libm and the departure from libm binary32)
def sinf(x): return f32(oracle_py.cr_eval("sin", np.array([x], np.float32))[0])
def cosf(x): return f32(oracle_py.cr_eval("cos", np.array([x], np.float32))[0])
def tanf(x): return f32(math.tan(float(x)))
def acosf(x): return f32(oracle_py.cr_eval("acos", np.array([x], np.float32))[0])
def expf(x): return f32(oracle_py.cr_eval("exp", np.array([x], np.float32))[0])
def powf(x, y): return f32(math.pow(float(x), float(y)))
def sqrtf(x): return f32(np.sqrt(f32(x)))


def fp(a):
    return np.ascontiguousarray(a, np.float32).ctypes.data_as(oracle_py.f32p)


# ---------------------------------------------------------------- Math.hs vector algebra (binary32)
def V(x, y, z):
    return np.array([x, y, z], np.float32)


def dot(a, b):                                          # Math.hs:341-343: x*a + y*b + z*c
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def cross(u, w):                                        # Math.hs:336-339
    return V(f32(u[1] * w[2]) - f32(u[2] * w[1]), -(f32(u[0] * w[2]) - f32(u[2] * w[0])),
             f32(u[0] * w[1]) - f32(u[1] * w[0]))


def sqlen(v):
    return dot(v, v)


def vlen(v):
    return sqrtf(sqlen(v))


def normalize(v):                                       # Math.hs:349-353: v * (1 / len v)
    if sqlen(v) != 0:
        return (v * (ONE / vlen(v))).astype(np.float32)
    return V(0, 1, 0)


def scale(v, s):
    return (v * f32(s)).astype(np.float32)


def lerp(t, a, b):                                      # Math.hs:108-110
    t, a, b = f32(t), f32(a), f32(b)
    return f32(f32(f32(ONE - t) * a) + f32(t * b))


def ghc_max(x, y):                                      # GHC Ord max/min on Float
    return y if x <= y else x


def ghc_min(x, y):
    return x if x <= y else y


# ---------------------------------------------------------------- triangles (TriangleMesh.hs:160-207)
def tri_intersect(p1, p2, p3, ro, rd, tmin, tmax):
    e1, e2 = p2 - p1, p3 - p1
    s1 = cross(rd, e2)
    divisor = dot(s1, e1)
    if divisor == 0:
        return None
    inv = ONE / divisor
    d = ro - p1
    b1 = f32(dot(d, s1) * inv)
    s2 = cross(d, e1)
    b2 = f32(dot(rd, s2) * inv)
    t = f32(dot(e2, s2) * inv)
    if b1 < 0 or b1 > 1:
        return None
    if b2 < 0 or f32(b1 + b2) > 1:
        return None
    if t < tmin or t > tmax:
        return None
    return t, b1, b2


def _tri_cases():
    rng = np.random.default_rng(5)
    cases = []
    for _ in range(400):
        p = rng.uniform(-10, 10, (3, 3)).astype(np.float32)
        c = (p.sum(0) / 3).astype(np.float32)
        o = rng.uniform(-30, 30, 3).astype(np.float32)
        aim = (c + rng.normal(0, 3, 3)).astype(np.float32)
        d = normalize((aim - o).astype(np.float32))
        cases.append((p, o, d, f32(0), f32(np.inf)))
    # exact edge cases: through a vertex (b1 = b2 = 0), parallel to the plane (divisor == 0), behind
    # the origin, clipped by tmin / tmax, on an edge (b1 + b2 == 1)
    p = np.array([[0, 0, 5], [4, 0, 5], [0, 4, 5]], np.float32)
    cases += [(p, V(0, 0, 0), V(0, 0, 1), f32(0), f32(np.inf)),
              (p, V(1, 1, 0), V(1, 0, 0), f32(0), f32(np.inf)),
              (p, V(1, 1, 10), V(0, 0, 1), f32(0), f32(np.inf)),
              (p, V(1, 1, 0), V(0, 0, 1), f32(6), f32(np.inf)),
              (p, V(1, 1, 0), V(0, 0, 1), f32(0), f32(4)),
              (p, V(2, 2, 0), V(0, 0, 1), f32(0), f32(np.inf)),
              (p, V(4, 0, 0), V(0, 0, 1), f32(0), f32(np.inf))]
    return cases


def test_triangle_hit_and_miss():
    lib = oracle_py.lib()
    hits = misses = 0
    for p, o, d, tmin, tmax in _tri_cases():
        out = np.zeros(3, np.float32)
        got = lib.oracle_tri_probe(fp(p.reshape(-1)), fp(np.r_[o, d, tmin, tmax]), fp(out))
        want = tri_intersect(p[0], p[1], p[2], o, d, tmin, tmax)
        assert bool(got) == (want is not None), (p, o, d)
        if want is not None:
            hits += 1
            assert tuple(out) == want, (out, want)
        else:
            misses += 1
    assert hits > 50 and misses > 50


# ---------------------------------------------------------------- SPDs (Spectrum.hs:291-335)
def avg_spd_irregular(ls, vs, l0, l1):
    if l1 <= ls[0]:
        return vs[0]
    if l0 >= ls[-1]:
        return vs[-1]
    i0 = next((i for i, l in enumerate(ls) if l >= l0), 0)
    i1 = next((i for i, l in enumerate(ls) if l >= l1), len(vs) - 1)
    acc = ZERO
    for v in vs[i0:i1 + 1]:                             # V.sum = foldl' (+) 0
        acc = f32(acc + v)
    return f32(acc / f32(i1 - i0 + 1))


def from_spd(pairs):
    pairs = sorted(pairs, key=lambda p: p[0])           # mkSpd: stable sortBy on lambda
    ls = [f32(a) for a, _ in pairs]
    vs = [f32(b) for _, b in pairs]
    out = np.zeros(16, np.float32)
    for i in range(16):
        l0 = lerp(f32(i) / f32(16), 400, 700)
        l1 = lerp(f32(i + 1) / f32(16), 400, 700)
        out[i] = avg_spd_irregular(ls, vs, l0, l1)
    return out


def scene_spds(name):
    text = open(os.path.join(SCENES, name)).read()
    text = "\n".join(line.split("#")[0] for line in text.splitlines())
    spds = []
    for body in re.findall(r"spd\s*\{([^}]*)\}", text):
        pairs = [tuple(float(x) for x in item.split()) for item in body.split(",") if item.strip()]
        spds.append(pairs)
    return spds


def test_from_spd_cornell_bands():
    """Every `spd { ... }` of cornell-box.bling becomes, band for band, a spectrum the loader put in
    the flattened scene (material textures and the area light's radiance)."""
    job = load_config("C2")
    d = desc(job)
    have = [arr(d.textures[i].value) for i in range(d.num_textures)]
    have += [arr(d.lights[i].radiance) for i in range(d.num_lights)]
    spds = scene_spds("cornell-box.bling")
    assert len(spds) >= 4                               # white, red, green, the light's emission
    for pairs in spds:
        want = from_spd(pairs)
        assert any(np.array_equal(want, h) for h in have), (pairs[:3], want)
    # the light: spd { 400 0, 500 8, 600 15.6, 700 18.4 } averaged over 18.75-nm bands
    light = arr(d.lights[0].radiance)
    assert np.array_equal(light, from_spd([(400, 0), (500, 8), (600, 15.6), (700, 18.4)]))


# ---------------------------------------------------------------- Transform.hs
def mat(rows):
    return np.array(rows, np.float32).reshape(16)


IDENT = mat([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])


def mul(m1, m2):                                        # Transform.hs:99-102: element (i, j) = sum_k m1[k][j] m2[i][k]
    out = np.zeros(16, np.float32)
    for n in range(16):
        i, j = divmod(n, 4)
        acc = ZERO                                      # sum = foldl (+) 0
        for k in range(4):
            acc = f32(acc + f32(m1[k * 4 + j] * m2[i * 4 + k]))
        out[n] = acc
    return out


def invert(m):                                          # Transform.hs:42-85, Gauss-Jordan on idx r c = c*4 + r
    minv = [f32(x) for x in m]
    ipiv = [0, 1, 2, 3]
    indx = []

    def idx(r, c):
        return c * 4 + r
    for _ in range(4):
        best, bv = None, None
        for j in ipiv:                                  # maximumBy (compare `on` snd): last maximum wins
            for k in ipiv:
                v = abs(minv[idx(j, k)])
                if best is None or not (bv > v):
                    best, bv = (j, k), v
        irow, icol = best
        ipiv = [i for i in ipiv if i != icol]
        if irow != icol:
            for k in range(4):
                a, b = idx(irow, k), idx(icol, k)
                minv[a], minv[b] = minv[b], minv[a]
        pivinv = f32(ONE / minv[idx(icol, icol)])
        minv[idx(icol, icol)] = ONE
        for j in range(4):
            minv[idx(icol, j)] = f32(minv[idx(icol, j)] * pivinv)
        for j in range(4):
            if j != icol:
                save = minv[idx(j, icol)]
                minv[idx(j, icol)] = ZERO
                for k in range(4):
                    minv[idx(j, k)] = f32(minv[idx(j, k)] - f32(minv[idx(icol, k)] * save))
        indx.append((irow, icol))
    for ir, ic in reversed(indx):
        if ir != ic:
            for k in range(4):
                a, b = idx(k, ir), idx(k, ic)
                minv[a], minv[b] = minv[b], minv[a]
    return np.array(minv, np.float32)


class Xf:
    def __init__(self, m, i):
        self.m, self.i = m, i

    def __matmul__(self, o):                            # a <> b = concatTrans a b (a applies first)
        return Xf(mul(self.m, o.m), mul(o.i, self.i))

    def inverse(self):
        return Xf(self.i, self.m)


IDX = Xf(IDENT, IDENT)


def translate(dx, dy, dz):
    dx, dy, dz = f32(dx), f32(dy), f32(dz)
    return Xf(mat([[1, 0, 0, dx], [0, 1, 0, dy], [0, 0, 1, dz], [0, 0, 0, 1]]),
              mat([[1, 0, 0, -dx], [0, 1, 0, -dy], [0, 0, 1, -dz], [0, 0, 0, 1]]))


def xscale(sx, sy, sz):
    sx, sy, sz = f32(sx), f32(sy), f32(sz)
    return Xf(mat([[sx, 0, 0, 0], [0, sy, 0, 0], [0, 0, sz, 0], [0, 0, 0, 1]]),
              mat([[ONE / sx, 0, 0, 0], [0, ONE / sy, 0, 0], [0, 0, ONE / sz, 0], [0, 0, 0, 1]]))


def radians(x):
    return f32(f32(f32(x) / f32(180)) * PI)


def perspective(fov, n, f):                             # Transform.hs:207-219
    n, f = f32(n), f32(f)
    ita = f32(ONE / tanf32(f32(radians(fov) / TWO)))
    m = mat([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, f32(f / f32(f - n)), -f32(f32(f * n) / f32(f - n))], [0, 0, 1, 0]])
    return xscale(ita, ita, 1) @ Xf(m, invert(m))


def look_at(p, l, up):                                  # Transform.hs:222-235
    p, l, up = V(*p), V(*l), V(*up)
    d = normalize(l - p)
    left = normalize(cross(normalize(up), d))
    u = cross(d, left)
    m = mat([[left[0], u[0], d[0], p[0]], [left[1], u[1], d[1], p[1]], [left[2], u[2], d[2], p[2]], [0, 0, 0, 1]])
    return Xf(m, invert(m))


def trans_point(m, p):                                  # Transform.hs:247-256
    r = [f32(f32(f32(f32(m[4 * a] * p[0]) + f32(m[4 * a + 1] * p[1])) + f32(m[4 * a + 2] * p[2])) + m[4 * a + 3])
         for a in range(4)]
    if r[3] == 1:
        return V(r[0], r[1], r[2])
    return V(f32(r[0] / r[3]), f32(r[1] / r[3]), f32(r[2] / r[3]))


def trans_vector(m, v):                                 # Transform.hs:259-264
    return V(*[f32(f32(f32(m[4 * a] * v[0]) + f32(m[4 * a + 1] * v[1])) + f32(m[4 * a + 2] * v[2])) for a in range(3)])


def mk_perspective_camera(c2w, lr, fd, fov, sx, sy):   # Camera.hs:108-147
    sx, sy = f32(sx), f32(sy)
    p = perspective(fov, 1e-2, 1000)
    aspect = f32(sx / sy)
    if aspect > 1:
        s0, s1, s2, s3 = -aspect, aspect, f32(-1), ONE
    else:
        s0, s1, s2, s3 = f32(-1), ONE, f32(f32(-1) / aspect), f32(ONE / aspect)
    st1 = xscale(sx, sy, 1)
    st2 = xscale(ONE / f32(s1 - s0), ONE / f32(s2 - s3), 1)
    t = translate(-s0, -s3, 0)
    s2r = t @ (st2 @ st1)                               # <> is infixr 6
    r2c = s2r.inverse() @ p.inverse()
    return c2w, r2c


def concentric_disk(u1, u2):                            # Montecarlo.hs:160-177
    sx, sy = f32(f32(u1) * TWO) - ONE, f32(f32(u2) * TWO) - ONE
    if sx == 0 and sy == 0:
        return ZERO, ZERO
    if sx >= -sy:
        if sx > sy:
            r, th = (sx, f32(sy / sx)) if sy > 0 else (sx, f32(f32(8) + f32(sy / sx)))
        else:
            r, th = sy, f32(TWO - f32(sx / sy))
    elif sx <= sy:
        r, th = -sx, f32(f32(4) - f32(sy / -sx))
    else:
        r, th = -sy, f32(f32(6) + f32(sx / -sy))
    theta = f32(f32(th * PI) / f32(4))
    return f32(r * cosf(theta)), f32(r * sinf(theta))


def fire_ray(c2w, r2c, lr, fd, ix, iy, lu, lv):        # Camera.hs:49-76
    p_cam = trans_point(r2c.m, V(ix, iy, 0))
    o, d = V(0, 0, 0), normalize(p_cam)
    if lr > 0:
        du, dv = concentric_disk(lu, lv)
        ro = V(f32(du * lr), f32(dv * lr), 0)
        t = f32(f32(fd) / d[2])
        focus = (o + (d * t).astype(np.float32)).astype(np.float32)
        o, d = ro, normalize((focus - ro).astype(np.float32))
    return trans_point(c2w.m, o), trans_vector(c2w.m, d)


CAMERAS = {  # config: (lookAt pos, look, up, fov, lensRadius, focalDistance) as in the scene files
    "C2": ((278.0, 273.0, -800.0), (278.0, 273.0, 0.0), (0.0, 1.0, 0.0), 37.5, 0.0, 10.0),
    "C3": ((0, 235, -500), (0, 30, 0), (0, 1, 0), 35.0, 0.0, 10.0),
    "C4": ((1, 5, -5), (0, 0, -1), (0, 1, 0), 65.0, 0.0, 7.0),
    "C5": ((-1, 0, -0.5), (2, 1.5, -0.5), (0, 1, 0), 40.0, 0.001, 0.425),
}


@pytest.mark.parametrize("cfg", sorted(CAMERAS))
def test_mk_projective_and_fire_ray(cfg):
    """The loader's camera matrices equal lookAt / perspective / mkProjective restated here (the
    parsed transform is `lookAt <> identity` composed onto the identity state, TransformParser.hs
    :15-25), and the oracle's fireRay gives the same corner and centre rays, with the thin lens for
    C5 (lensRadius 0.001)."""
    job = load_config(cfg)
    d = desc(job)
    pos, look, up, fov, lr, fd = CAMERAS[cfg]
    c2w = (look_at(pos, look, up) @ IDX) @ IDX
    c2w, r2c = mk_perspective_camera(c2w, lr, fd, fov, job.width, job.height)
    cam = d.camera
    np.testing.assert_array_equal(arr(cam.c2w), c2w.m)
    np.testing.assert_array_equal(arr(cam.c2w_inv), c2w.i)
    np.testing.assert_array_equal(arr(cam.r2c), r2c.m)
    np.testing.assert_array_equal(arr(cam.r2c_inv), r2c.i)
    assert cam.lens_radius == f32(lr) and cam.focal_distance == f32(fd)
    orc = oracle_py.Oracle(job)
    w, h = job.width, job.height
    rng = np.random.default_rng(3)
    pts = [(0, 0), (w, 0), (0, h), (w, h), (w / 2, h / 2), (0.25, 0.75), (w - 0.5, h - 0.25)]
    pts += [tuple(rng.uniform(-2, w + 2, 1).tolist() + rng.uniform(-2, h + 2, 1).tolist()) for _ in range(40)]
    for ix, iy in pts:
        lu, lv = (f32(x) for x in rng.uniform(0, 1, 2))
        out = np.zeros(6, np.float32)
        oracle_py.lib().oracle_fire_ray_probe(orc.h, f32(ix), f32(iy), lu, lv, fp(out))
        o, dd = fire_ray(c2w, r2c, f32(lr), f32(fd), f32(ix), f32(iy), lu, lv)
        np.testing.assert_array_equal(out[:3], o, err_msg=f"{cfg} origin at {(ix, iy)}")
        np.testing.assert_array_equal(out[3:], dd, err_msg=f"{cfg} direction at {(ix, iy)}")


# ---------------------------------------------------------------- Reflection.hs helpers
INV_PI = f32(ONE / PI)
INV_TWO_PI = f32(ONE / f32(TWO * PI))


def clamp(v, lo, hi):                                   # Math.hs:78-87
    return lo if v < lo else (hi if v > hi else v)


def sin_theta(w):
    return sqrtf(ghc_max(ZERO, f32(ONE - f32(w[2] * w[2]))))


def cos_phi(w):
    s = sin_theta(w)
    return ONE if s == 0 else clamp(f32(w[0] / s), f32(-1), ONE)


def sin_phi(w):
    s = sin_theta(w)
    return ZERO if s == 0 else clamp(f32(w[1] / s), f32(-1), ONE)


def same_hemi(a, b):
    return f32(a[2] * b[2]) > 0


def cosine_hemisphere(u1, u2):                          # Montecarlo.hs:146-149
    x, y = concentric_disk(u1, u2)
    return V(x, y, sqrtf(ghc_max(ZERO, f32(f32(ONE - f32(x * x)) - f32(y * y)))))


def to_same_hemi(wo, wi):
    return V(wi[0], wi[1], -wi[2]) if wo[2] < 0 else wi


def cos_pdf(wo, wi):
    return f32(INV_PI * abs(wi[2])) if same_hemi(wo, wi) else ZERO


def oren_nayar(r, sig, wo, wi):                         # Diffuse.hs:29-66
    sg = clamp(f32(sig), ZERO, ONE)
    sig2 = f32(sg * sg)
    a = f32(ONE - f32(sig2 / f32(TWO * f32(sig2 + f32(0.33)))))
    b = f32(f32(f32(0.45) * sig2) / f32(sig2 + f32(0.09)))
    sinti, sinto = sin_theta(wi), sin_theta(wo)
    if abs(wi[2]) > abs(wo[2]):
        sina, tanb = sinto, f32(sinti / abs(wi[2]))
    else:
        sina, tanb = sinti, f32(sinto / abs(wo[2]))
    maxcos = ZERO
    if sinti > f32(1e-4) and sinto > f32(1e-4):
        maxcos = ghc_max(ZERO, f32(f32(cos_phi(wi) * cos_phi(wo)) + f32(sin_phi(wi) * sin_phi(wo))))
    return (r * f32(a + f32(f32(f32(b * maxcos) * sina) * tanb))).astype(np.float32)


def probe_bxdf(orc, mat_i, comp, wo, wi, u):
    out = np.zeros(37, np.float32)
    n = oracle_py.lib().oracle_bxdf_probe(orc.h, mat_i, comp, fp(wo), fp(wi), fp(np.array(u, np.float32)), fp(out))
    return n, out


def random_dirs(rng, n, upper=True):
    out = []
    for _ in range(n):
        w = normalize(rng.normal(size=3).astype(np.float32))
        if upper and w[2] < 0:
            w = V(w[0], w[1], -w[2])
        out.append(w)
    return out


def test_oren_nayar_cornell_white():
    """cornell's white material: matte, kd = the white SPD, sigma 0.5 -> one Oren-Nayar lobe."""
    job = load_config("C2")
    d = desc(job)
    mats = [i for i in range(d.num_materials) if d.materials[i].kind == 1 and d.materials[i].scalar[0] == f32(0.5)]
    assert mats, "no sigma-0.5 matte in cornell-box.bling"
    mi = mats[0]
    r = arr(d.textures[d.materials[mi].tex[0]].value)
    orc = oracle_py.Oracle(job)
    rng = np.random.default_rng(17)
    wos, wis = random_dirs(rng, 64), random_dirs(rng, 64)
    wis[0] = V(0, 0, 1)                                 # sin theta = 0 branches
    wos[1] = V(0, 0, 1)
    for wo, wi in zip(wos, wis):
        u = rng.uniform(0, 1, 2).astype(np.float32)
        n, out = probe_bxdf(orc, mi, 0, wo, wi, u)
        assert n == 1
        np.testing.assert_array_equal(out[:16], (oren_nayar(r, 0.5, wo, wi) * f32(INV_PI * abs(wo[2]))).astype(np.float32))
        assert out[16] == cos_pdf(wo, wi)
        ws = to_same_hemi(wo, cosine_hemisphere(u[0], u[1]))
        np.testing.assert_array_equal(out[33:36], ws)
        if same_hemi(wo, ws):
            np.testing.assert_array_equal(out[17:33], oren_nayar(r, 0.5, wo, ws))
            assert out[36] == cos_pdf(wo, ws)
        else:
            assert out[36] == 0 and not out[17:33].any()


# ---------------------------------------------------------------- Microfacet.hs: Blinn (ducky's plastic)
def fr_dielectric(etai, etat, cosi):                    # Fresnel.hs (frDielectric / frDiel')
    etai, etat, cosi = f32(etai), f32(etat), f32(cosi)
    c = ghc_max(ZERO, f32(ONE - f32(cosi * cosi)))
    costp = f32(c / f32(etat * etat)) if cosi > 0 else f32(c * f32(etat * etat))
    cost = sqrtf(f32(ONE - clamp(costp, ZERO, ONE)))
    ci = abs(cosi)
    eta = f32(etat / etai)
    rparl_ = f32(eta * ci)
    rparl = f32(f32(cost - rparl_) / f32(cost + rparl_))
    rperp_ = f32(eta * cost)
    rperp = f32(f32(ci - rperp_) / f32(ci + rperp_))
    return f32(f32(f32(rparl * rparl) + f32(rperp * rperp)) * f32(0.5))


def mf_g(wo, wi, wh):                                   # Microfacet.hs:113-120
    nwh, nwo, nwi = abs(wh[2]), abs(wo[2]), abs(wi[2])
    wowh = abs(dot(wo, wh))
    return ghc_min(ONE, ghc_min(f32(f32(f32(TWO * nwh) * nwo) / wowh), f32(f32(f32(TWO * nwh) * nwi) / wowh)))


def blinn_d(e, wh):
    return f32(f32(f32(e + TWO) * INV_TWO_PI) * powf(abs(wh[2]), e))


def blinn_pdf(e, wh):
    return f32(f32(f32(e + ONE) * powf(abs(wh[2]), e)) * INV_TWO_PI)


def blinn_sample(e, u1, u2):
    cost = powf(u1, f32(ONE / f32(e + ONE)))
    sint = sqrtf(ghc_max(ZERO, f32(ONE - f32(cost * cost))))
    phi = f32(f32(u2 * TWO) * PI)
    wh = V(f32(sint * cosf(phi)), f32(sint * sinf(phi)), cost)      # sphericalDirection
    fv = f32(powf(cost, e) * INV_TWO_PI)
    return wh, f32(f32(e + TWO) * fv), f32(f32(e + ONE) * fv)


def microfacet_blinn(r, e, wo, wi, u):
    """(eval, pdf, (f, wi, pdf)) of mkMicrofacet (Blinn e) (frDielectric 1 1.5) r."""
    costo, costi = abs(wo[2]), abs(wi[2])
    whp = (wi + wo).astype(np.float32)
    if costi == 0 or costo == 0 or not whp.any():
        ev = np.zeros(16, np.float32)
    else:
        wh = normalize(whp)
        if wh[2] < 0:
            ev = np.zeros(16, np.float32)
        else:
            x = f32(f32(blinn_d(e, wh) * mf_g(wo, wi, wh)) / f32(f32(4) * costi))
            ev = ((r * fr_dielectric(1, 1.5, dot(wi, wh))).astype(np.float32) * x).astype(np.float32)
    whq = (wo + wi).astype(np.float32)
    if sqlen(whq) == 0:
        pdf = ZERO
    else:
        wh = normalize(whq)
        pdf = ZERO if wh[2] < 0 else f32(blinn_pdf(e, wh) / f32(f32(4) * abs(dot(wo, wh))))
    whs, dd, pp = blinn_sample(e, u[0], u[1])
    wh = -whs if whs[2] < 0 else whs
    ws = ((wh * f32(TWO * dot(wo, wh))).astype(np.float32) - wo).astype(np.float32)
    cos_h = dot(wo, wh)
    if same_hemi(wo, ws):
        fact = f32(f32(f32(dd * abs(cos_h)) / pp) * mf_g(wo, ws, wh))
        fs = ((r * fr_dielectric(1, 1.5, cos_h)).astype(np.float32) * f32(fact / abs(ws[2]))).astype(np.float32)
        samp = (fs, ws, f32(pp / f32(f32(4) * abs(cos_h))))
    else:
        samp = (np.zeros(16, np.float32), wo, ZERO)
    return ev, pdf, samp


def test_blinn_microfacet_ducky_plastic():
    """ducky's plastic: Lambert + mkMicrofacet (mkBlinn (1 / rough)) (frDielectric 1 1.5) ks."""
    job = load_config("C3")
    d = desc(job)
    mats = [i for i in range(d.num_materials) if d.materials[i].kind == 2]
    assert mats
    mi = mats[0]
    m = d.materials[mi]
    ks = arr(d.textures[m.tex[1]].value)
    e = f32(ONE / f32(m.scalar[0]))
    e = f32(10000) if (e > 10000 or np.isnan(e)) else e                # fixExponent
    orc = oracle_py.Oracle(job)
    rng = np.random.default_rng(23)
    checked = 0
    wos, wis = random_dirs(rng, 96), random_dirs(rng, 96)
    for k in range(48):                                  # near-mirror pairs: inside e = 1 / rough's lobe
        wh = normalize(V(*rng.normal(0, 0.02, 2), 1))
        wis[k] = ((wh * f32(TWO * dot(wos[k], wh))).astype(np.float32) - wos[k]).astype(np.float32)
    for wo, wi in zip(wos, wis):
        u = rng.uniform(0, 1, 2).astype(np.float32)
        n, out = probe_bxdf(orc, mi, 1, wo, wi, u)
        assert n == 2
        ev, pdf, (fs, ws, ps) = microfacet_blinn(ks, e, wo, wi, u)
        np.testing.assert_array_equal(out[:16], ev)
        assert out[16] == pdf
        np.testing.assert_array_equal(out[17:33], fs)
        np.testing.assert_array_equal(out[33:36], ws)
        assert out[36] == ps
        checked += int(ev.any())
    assert checked > 30


# ---------------------------------------------------------------- the quad area light (cornell)
def quad_intersect(sx, sy, ro, rd, tmin, tmax):         # Shape.hs:157-171
    if abs(rd[2]) < f32(1e-7):
        return None
    t = f32(-ro[2] / rd[2])
    if t < tmin or t > tmax:
        return None
    p = (ro + (rd * t).astype(np.float32)).astype(np.float32)
    if abs(p[0]) > sx or abs(p[1]) > sy:
        return None
    n = normalize(cross(V(sx, 0, 0), V(0, sy, 0)))     # mkDg: normalize (dpdu x dpdv)
    return t, p, n


def quad_pdf(sx, sy, p, wi):                            # shapePdf -> generalPdf (Shape.hs:333-350)
    h = quad_intersect(sx, sy, p, wi, f32(1e-3), f32(np.inf))
    if h is None:
        return ZERO
    t, ph, n = h
    area = f32(f32(f32(4) * sx) * sy)
    pd = f32(sqlen((p - ph).astype(np.float32)) / f32(abs(dot(n, -wi)) * area))
    return ZERO if np.isinf(pd) else pd


def area_light_sample(s, radiance, pw, eps, u1, u2):    # Light.hs:150-158 with sampleShape' Quad (:405-406)
    sx, sy = f32(s.params[0]), f32(s.params[1])
    o2w, w2o = arr(s.o2w), arr(s.w2o)
    p = trans_point(w2o, pw)
    ps, ns = V(lerp(u1, -sx, sx), lerp(u2, -sy, sy), 0), V(0, 0, -1)
    wi = normalize((ps - p).astype(np.float32))
    li = radiance if dot(ns, wi) < 0 else np.zeros(16, np.float32)
    pd = quad_pdf(sx, sy, p, wi)
    tmax = f32(vlen((ps - p).astype(np.float32)) - eps)
    return li, trans_vector(o2w, wi), pd, trans_point(o2w, p), trans_vector(o2w, wi), eps, tmax


def test_quad_light_sample_and_pdf():
    """cornell's light: quad 65 x 52.2 under rotateX -90 translate 278 548.7 279.5."""
    job = load_config("C2")
    d = desc(job)
    L = d.lights[0]
    assert L.kind == 1
    s = d.shapes[L.shape]
    assert s.kind == 1 and s.params[0] == f32(65) and s.params[1] == f32(52.2)
    rad = arr(L.radiance)
    orc = oracle_py.Oracle(job)
    lib = oracle_py.lib()
    rng = np.random.default_rng(29)
    lit = 0
    for _ in range(200):
        pw = rng.uniform([0, 0, 0], [556, 548, 559]).astype(np.float32)
        eps = f32(rng.uniform(1e-3, 1e-1))
        u1, u2 = (f32(x) for x in rng.uniform(0, 1, 2))
        out = np.zeros(28, np.float32)
        lib.oracle_light_sample_probe(orc.h, 0, fp(pw), eps, u1, u2, fp(out))
        li, wiw, pd, ro, rd, tmin, tmax = area_light_sample(s, rad, pw, eps, u1, u2)
        np.testing.assert_array_equal(out[:16], li)
        np.testing.assert_array_equal(out[16:19], wiw)
        assert out[19] == pd
        np.testing.assert_array_equal(out[20:23], ro)
        np.testing.assert_array_equal(out[23:26], rd)
        assert out[26] == tmin and out[27] == tmax
        lit += int(li.any())
        # Light.pdf (Light.hs:228): shapePdf in the light's space
        wq = normalize(rng.normal(size=3).astype(np.float32))
        got = lib.oracle_light_pdf_probe(orc.h, 0, fp(pw), fp(wq))
        want = quad_pdf(f32(s.params[0]), f32(s.params[1]), trans_point(arr(s.w2o), pw), trans_vector(arr(s.w2o), wq))
        assert f32(got) == want
    # trap T6: points below the downward-facing light see it (sampled normal -z), points above do not
    assert lit > 100


# ---------------------------------------------------------------- SunSky.hs
def _table(name):
    text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "bling_amd", "csrc", "common", "spectral_data.h")).read()
    body = re.search(name + r"\[[^=]*=\s*\{(.*?)\};", text, re.S).group(1)
    return np.array([float.fromhex(x.rstrip("f")) for x in re.findall(r"-?0x[0-9a-fA-F.]+p[+-]?\d+f?", body)],
                    np.float32)


def coordinate_system2(w, v):                          # Math.hs:427-432 coordinateSystem'
    w2 = normalize(w)
    u = normalize(cross(v, w2))
    return u, cross(w2, u), w2


def init_sky(east, sdw, t):                             # SunSky.hs:12-24, 45-65
    t = f32(t)
    bs, bt, bn = coordinate_system2(normalize(V(0, 1, 0)), normalize(V(*east)))
    sdw = normalize(V(*sdw))
    sd = normalize(V(dot(sdw, bs), dot(sdw, bt), dot(sdw, bn)))
    st = acosf32(clamp(sd[2], f32(-1), ONE))
    st2, st3, t2 = f32(st * st), f32(f32(st * st) * st), f32(t * t)
    chi = f32(f32(f32(f32(4) / f32(9)) - f32(t / f32(120))) * f32(PI - f32(TWO * st)))

    def lin(a, b):        # a * t + b with Haskell's unary minus on the product (negate (a' * t))
        return f32(f32(f32(a) * t) + f32(b))
    pY = [lin(0.17872, -1.46303), lin(-0.35540, 0.42749), lin(-0.02266, 5.32505), lin(0.12064, -2.57705),
          lin(-0.06696, 0.37027)]
    px = [lin(-0.01925, -0.25922), lin(-0.06651, 0.00081), lin(-0.00041, 0.21247), lin(-0.06409, -0.89887),
          lin(-0.00325, 0.04517)]
    py = [lin(-0.01669, -0.26078), lin(-0.09495, 0.00921), lin(-0.00792, 0.21023), lin(-0.04405, -1.65369),
          lin(-0.01092, 0.05291)]
    zY = f32(f32(f32(f32(f32(f32(f32(4.04530) * t) - f32(4.97100)) * tanf32(chi)) - f32(f32(0.2155) * t))
                 + f32(2.4192)) * f32(1000))

    def cubic(a3, a2, a1, a0):
        return f32(f32(f32(f32(f32(a3) * st3) + f32(f32(a2) * st2)) + f32(f32(a1) * st)) + f32(a0))
    zx = f32(f32(f32(cubic(0.00165, -0.00374, 0.00208, 0) * t2) + f32(cubic(-0.02902, 0.06377, -0.03202, 0.00394) * t))
             + cubic(0.11693, -0.21196, 0.06052, 0.25885))
    zy = f32(f32(f32(cubic(0.00275, -0.00610, 0.00316, 0) * t2) + f32(cubic(-0.04212, 0.08970, -0.04153, 0.00515) * t))
             + cubic(0.15346, -0.26756, 0.06669, 0.26688))
    return dict(sd=sd, st=st, pY=pY, px=px, py=py, zY=zY, zx=zx, zy=zy, basis=(bs, bt, bn))


def eval_regular(l0, l1, amps, lam):                    # Spectrum.hs:271-280 evalSpd RegularSpd
    if lam <= l0:
        return amps[0]
    if lam >= l1:
        return amps[-1]
    d1 = f32(ONE / f32(f32(f32(l1) - f32(l0)) / f32(len(amps) - 1)))
    x = f32(f32(lam - f32(l0)) * d1)
    b0 = int(np.floor(x))
    b1 = min(b0 + 1, len(amps) - 1)
    dx = f32(x - f32(b0))
    return f32(f32(f32(ONE - dx) * amps[b0]) + f32(dx * amps[b1]))


def eval_irregular(ls, vs, lam):                        # Spectrum.hs:258-269 evalSpd IrregularSpd
    if lam <= ls[0]:
        return vs[0]
    if lam >= ls[-1]:
        return vs[-1]
    lo, hi = 0, len(ls) - 1
    while True:
        mid = (lo + hi) // 2
        if lo == mid:
            break
        if ls[mid] == lam:
            lo = mid
            break
        if ls[mid] < lam:
            lo = mid
        else:
            hi = mid
    t = f32(f32(lam - ls[lo]) / f32(ls[lo + 1] - ls[lo]))
    return lerp(t, vs[lo], vs[lo + 1])


def sun_spectrum(st, turb):                             # SunSky.hs:96-125 sunSpectrum'
    turb = f32(turb)
    sol = _table("BLING_SOL_CURVE_380_750")
    ko = (_table("BLING_KO_LAMBDA"), _table("BLING_KO_VALUE"))
    kg = (_table("BLING_KG_LAMBDA"), _table("BLING_KG_VALUE"))
    kwa = (_table("BLING_KWA_LAMBDA"), _table("BLING_KWA_VALUE"))

    def sf(lam):
        m = f32(ONE / f32(cosf32(st) + f32(f32(0.000940) * powf32(f32(f32(1.6386) - st), f32(-1.253)))))
        tR = expf32(-f32(f32(m * f32(0.008735)) * powf32(f32(lam / f32(1000)), f32(-4.08))))
        beta = f32(f32(f32(0.04608365822050) * turb) - f32(0.04586025928522))
        tA = expf32(-f32(f32(m * beta) * powf32(f32(lam / f32(1000)), -f32(1.3))))
        tO = expf32(-f32(f32(m * eval_irregular(*ko, lam)) * f32(0.35)))
        k_g = eval_irregular(*kg, lam)
        tG = expf32(-f32(f32(f32(f32(1.41) * k_g) * m) / powf32(f32(ONE + f32(f32(f32(118.93) * k_g) * m)), f32(0.45))))
        k_w = eval_irregular(*kwa, lam)
        w = TWO
        tWA = expf32(-f32(f32(f32(f32(f32(0.2385) * k_w) * w) * m) /
                        powf32(f32(ONE + f32(f32(f32(f32(20.07) * k_w) * w) * m)), f32(0.45))))
        s = eval_regular(380, 750, sol, lam)
        return f32(f32(f32(f32(f32(s * tR) * tA) * tO) * tG) * tWA)
    out = np.zeros(16, np.float32)
    for i in range(16):                                 # fromSpd (mkSpdFunc sf): avgSpd = (f l0 + f l1) * 0.5
        l0 = lerp(f32(i) / f32(16), 400, 700)
        l1 = lerp(f32(i + 1) / f32(16), 400, 700)
        out[i] = f32(f32(sf(l0) + sf(l1)) * f32(0.5))
    return out


def perez(p, sun_t, t, g, lvz):                         # SunSky.hs:81-86
    csg, cst = cosf(g), cosf(sun_t)
    num = f32(f32(f32(ONE + f32(p[0] * expf(f32(p[1] / cosf(t))))) * f32(ONE + f32(p[2] * expf(f32(p[3] * g)))))
              + f32(f32(p[4] * csg) * csg))
    den = f32(f32(f32(ONE + f32(p[0] * expf(p[1]))) * f32(ONE + f32(p[2] * expf(f32(p[3] * sun_t)))))
              + f32(f32(p[4] * cst) * cst))
    return f32(f32(lvz * num) / den)


def sky_spectrum(L, dirv):                              # SunSky.hs:67-79 + xyzToSpectrum (Spectrum.hs:143-168, 357-358)
    dz = -dirv[2]
    if dz < f32(1e-4):
        return np.zeros(16, np.float32)
    sd = arr(L.sun_dir_local)
    theta = acosf(dz)
    gamma = acosf(clamp(dot(dirv, sd), f32(-1), ONE))
    st = f32(L.sun_theta)
    x = perez(arr(L.perez_x), st, theta, gamma, f32(L.zenith_x))
    y = perez(arr(L.perez_y), st, theta, gamma, f32(L.zenith_y))
    yy = f32(perez(arr(L.perez_Y), st, theta, gamma, f32(L.zenith_Y)) * f32(1e-4))
    den = f32(f32(f32(0.0241) + f32(f32(0.2562) * x)) - f32(f32(0.7341) * y))
    m1 = f32(f32(f32(f32(-1.3515) - f32(f32(1.7703) * x)) + f32(f32(5.9114) * y)) / den)
    m2 = f32(f32(f32(f32(0.03) - f32(f32(31.4424) * x)) + f32(f32(30.0717) * y)) / den)
    S = _table("BLING_S_XYZ").reshape(3, 3)
    cx = f32(f32(S[0, 0] + f32(m1 * S[1, 0])) + f32(m2 * S[2, 0]))
    cy = f32(f32(S[0, 1] + f32(m1 * S[1, 1])) + f32(m2 * S[2, 1]))
    cz = f32(f32(S[0, 2] + f32(m1 * S[1, 2])) + f32(m2 * S[2, 2]))
    X, Y, Z = f32(f32(cx * yy) / cy), yy, f32(f32(cz * yy) / cy)
    r = f32(f32(f32(f32(3.240479) * X) - f32(f32(1.537150) * Y)) - f32(f32(0.498535) * Z))
    g = f32(f32(f32(f32(-0.969256) * X) + f32(f32(1.875991) * Y)) + f32(f32(0.041556) * Z))
    b = f32(f32(f32(f32(0.055648) * X) - f32(f32(0.204043) * Y)) + f32(f32(1.057311) * Z))
    rb, gb, bb, cb, mb, yb, wb = _table("BLING_RGB_ILLUM_BANDS").reshape(7, 16)

    def ss(base, k):
        return (base * f32(k)).astype(np.float32)

    def add(a, c):
        return (a + c).astype(np.float32)
    if r <= g and r <= b:
        return add(ss(wb, r), add(ss(cb, g - r), ss(bb, b - g)) if g <= b else add(ss(cb, b - r), ss(gb, g - b)))
    if g <= r and g <= b:
        return add(ss(wb, g), add(ss(mb, r - g), ss(bb, b - r)) if r <= b else add(ss(mb, b - g), ss(rb, r - b)))
    return add(ss(wb, b), add(ss(yb, r - b), ss(gb, g - r)) if r <= b else add(ss(yb, g - b), ss(rb, r - g)))


SUNSKY = {"C4": ((0, 0, 1), (0, 0.3, 1), 12), "C5": ((0, 0, 1), (2, 0.5, -1), 3)}


@pytest.mark.parametrize("cfg", sorted(SUNSKY))
def test_sun_sky_model(cfg):
    """initSky's Perez coefficients, zenith values and sun direction, sunSpectrum' (the solar curve
    through Rayleigh / aerosol / ozone / gas / water attenuation, band averaged) as precomputed by the
    loader, and the oracle's sky + sun lookups at a grid of map coordinates."""
    east, sdw, turb = SUNSKY[cfg]
    job = load_config(cfg)
    d = desc(job)
    L = next(d.lights[i] for i in range(d.num_lights) if d.lights[i].kind == 2 and d.lights[i].env_kind == 1)
    k = init_sky(east, sdw, turb)
    np.testing.assert_array_equal(arr(L.sun_dir_local), k["sd"])
    assert f32(L.sun_theta) == k["st"]
    np.testing.assert_array_equal(arr(L.perez_Y), np.array(k["pY"], np.float32))
    np.testing.assert_array_equal(arr(L.perez_x), np.array(k["px"], np.float32))
    np.testing.assert_array_equal(arr(L.perez_y), np.array(k["py"], np.float32))
    assert (f32(L.zenith_Y), f32(L.zenith_x), f32(L.zenith_y)) == (k["zY"], k["zx"], k["zy"])
    np.testing.assert_array_equal(arr(L.sun_radiance), sun_spectrum(k["st"], turb))
    orc = oracle_py.Oracle(job)
    li = next(i for i in range(d.num_lights) if d.lights[i].kind == 2)
    stm = sqrtf(ghc_max(ZERO, f32(ONE - f32(f32(6.955e5) / f32(1.496e8)))))
    sd = arr(L.sun_dir_local)
    nsky = 0
    for u in np.linspace(0, 1, 23, dtype=np.float32):
        for v in np.linspace(0, 1, 19, dtype=np.float32):
            out = np.zeros(16, np.float32)
            oracle_py.lib().oracle_env_probe(orc.h, li, u, v, fp(out))
            phi, th = f32(f32(u * TWO) * PI), f32(v * PI)
            sth = sinf(th)
            dirv = V(f32(sth * cosf(phi)), f32(sth * sinf(phi)), cosf(th))
            want = sky_spectrum(L, dirv)
            dsun = dot(V(sd[0], sd[1], -sd[2]), dirv)
            if dsun > stm:
                want = (want + arr(L.sun_radiance)).astype(np.float32)
            np.testing.assert_array_equal(out, want, err_msg=f"{cfg} sky at u={u} v={v}")
            nsky += int(want.any())
    assert nsky > 50


# ---------------------------------------------------------------- point / directional lights (X13)
def test_delta_lights_sample_and_pdf():
    """Light.sample of a directional and a point light (Light.hs:143-150) and their Light.pdf = 0
    (:225, 229), against the oracle, from numpy binary32.  mkDirectional normalises its normal at
    parse time (:52-54); the point light's visibility ray keeps the unnormalised p' - p and no upper
    bound (trap T19).  The oracle probe passes the shading normal (0, 0, 1)."""
    job = load_config("X13")
    d = desc(job)
    orc = oracle_py.Oracle(job)
    lib = oracle_py.lib()
    kinds = [d.lights[i].kind for i in range(d.num_lights)]
    assert kinds[:2] == [4, 3]                            # parsed lights, reverse parse order: directional, point
    ldir, lpt = d.lights[0], d.lights[1]
    np.testing.assert_array_equal(arr(ldir.delta_vec), normalize(V(0.3, 1, -0.5)))
    np.testing.assert_array_equal(arr(lpt.delta_vec), V(2, 4, -2))
    rng = np.random.default_rng(13)
    n = V(0, 0, 1)
    for _ in range(64):
        pw = rng.uniform(-4, 4, 3).astype(np.float32)
        eps = f32(rng.uniform(1e-4, 1e-2))
        for li, L in ((0, ldir), (1, lpt)):
            out = np.zeros(28, np.float32)
            lib.oracle_light_sample_probe(orc.h, li, fp(pw), eps, f32(0.3), f32(0.7), fp(out))
            v = arr(L.delta_vec)
            if li == 0:
                want_li = (arr(L.radiance) * f32(abs(dot(n, v)))).astype(np.float32)
                want_wi, ro, rd = v, pw, v
            else:
                dv = (v - pw).astype(np.float32)
                want_li = (arr(L.radiance) * f32(ONE / sqlen(dv))).astype(np.float32)
                want_wi, ro, rd = normalize(dv), pw, dv
            np.testing.assert_array_equal(out[:16], want_li)
            np.testing.assert_array_equal(out[16:19], want_wi)
            assert out[19] == ONE
            np.testing.assert_array_equal(out[20:23], ro)
            np.testing.assert_array_equal(out[23:26], rd)
            assert out[26] == eps and out[27] == np.inf
            wq = normalize(rng.normal(size=3).astype(np.float32))
            assert lib.oracle_light_pdf_probe(orc.h, li, fp(pw), fp(wq)) == 0.0
