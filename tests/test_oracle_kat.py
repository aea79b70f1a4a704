"""Known-answer tests pinning the CPU oracle.

Each check restates a reference formula independently in numpy binary32 (left-to-right evaluation,
no FMA -- GHC's order) and compares it with the oracle's C++ restatement, which the HIP core is in
turn checked against (tests/test_gpu_parity.py).  The reference's own test suite pins no hot-path
value (L/Main/Tests.hs only checks rnd in [0,1) and that shuffle permutes), so these formula KATs
plus the committed golden vectors (tests/golden/) are the parity anchor."""
import ctypes
import math

import numpy as np
import pytest

import oracle_py
from bling_amd.scene import load_config

f32 = np.float32


# ---------------------------------------------------------------- Math.hs:124-139 solveQuadric
def solve_quadric(a, b, c):
    a, b, c = f32(a), f32(b), f32(c)
    discrim = f32(b * b) - f32(f32(4) * a) * c
    if discrim < 0:
        return None
    root = f32(np.sqrt(discrim))
    q = f32(-0.5) * (b - root) if b < 0 else f32(-0.5) * (b + root)
    t0, t1 = f32(q / a), f32(c / q)
    return (min(t0, t1), max(t0, t1))


@pytest.mark.parametrize("abc", [(1, -3, 2), (1, 2, 1), (2, 0, -8), (1, 0, 1), (0.5, -7.25, 1e-3),
                                 (3.0, 1e4, -2.5), (1, 1e-20, -1e-20), (4.0, -4.0, 1.0)])
def test_solve_quadric(abc):
    out = np.zeros(2, np.float32)
    ok = oracle_py.lib().oracle_solve_quadric(*abc, oracle_py._fp(out))
    want = solve_quadric(*abc)
    assert bool(ok) == (want is not None)
    if want is not None:
        assert out[0] == want[0] and out[1] == want[1]


def test_solve_quadric_roots_are_roots():
    t = solve_quadric(1, -3, 2)
    assert t == (1.0, 2.0)


# ---------------------------------------------------------------- Montecarlo.hs:160-177
def concentric_disk(u1, u2):
    sx, sy = f32(f32(u1) * f32(2)) - f32(1), f32(f32(u2) * f32(2)) - f32(1)
    if sx == 0 and sy == 0:
        return 0.0, 0.0
    if sx >= -sy:
        if sx > sy:
            r, th = (sx, sy / sx) if sy > 0 else (sx, f32(8) + f32(sy / sx))
        else:
            r, th = sy, f32(2) - f32(sx / sy)
    elif sx <= sy:
        r, th = -sx, f32(4) - f32(sy / -sx)
    else:
        r, th = -sy, f32(6) + f32(sx / -sy)
    theta = f32(f32(th) * f32(math.pi)) / f32(4)
    # cos / sin: the shared cr_math.h functions (faithful binary32 since round 5)
    c, sn = (oracle_py.cr_eval(k, np.array([theta], np.float32))[0] for k in ("cos", "sin"))
    return float(f32(r) * f32(c)), float(f32(r) * f32(sn))


@pytest.mark.parametrize("u", [(0.5, 0.5), (1.0, 0.5), (0.5, 1.0), (0.0, 0.5), (0.5, 0.0), (0.9, 0.7),
                               (0.1, 0.2), (0.3, 0.95), (0.75, 0.25), (0.0, 0.0)])
def test_concentric_disk(u):
    out = np.zeros(2, np.float32)
    oracle_py.lib().oracle_concentric_disk(u[0], u[1], oracle_py._fp(out))
    want = concentric_disk(*u)
    # cos / sin shared with the oracle (common/cr_math.h): bit-exact
    np.testing.assert_array_equal(out, np.array(want, np.float32))
    assert float(np.hypot(out[0], out[1])) <= 1.0 + 1e-6


# ---------------------------------------------------------------- Fresnel.hs:17-70
def fr_dielectric(etai, etat, cosi):
    etai, etat, cosi = f32(etai), f32(etat), f32(cosi)
    c = max(f32(0), f32(1) - f32(cosi * cosi))
    costp = f32(c / f32(etat * etat)) if cosi > 0 else f32(c * f32(etat * etat))
    cost = f32(np.sqrt(f32(1) - min(max(costp, f32(0)), f32(1))))
    ci = abs(cosi)
    eta = f32(etat / etai)
    rparl_ = f32(eta * ci)
    rparl = f32(cost - rparl_) / f32(cost + rparl_)
    rperp_ = f32(eta * cost)
    rperp = f32(ci - rperp_) / f32(ci + rperp_)
    return f32(f32(f32(rparl * rparl) + f32(rperp * rperp)) * f32(0.5))


@pytest.mark.parametrize("args", [(1.0, 1.5, 1.0), (1.0, 1.5, 0.5), (1.0, 1.5, -0.3), (1.0, 1.5, 0.01),
                                  (1.0, 1.33, 0.9), (1.0, 1.5, -0.95)])
def test_fr_dielectric(args):
    out = np.zeros(16, np.float32)
    oracle_py.lib().oracle_fr_dielectric(*args, oracle_py._fp(out))
    want = fr_dielectric(*args)
    assert (out == want).all(), (out[0], want)


def test_fr_dielectric_normal_incidence_value():
    # ((n - 1) / (n + 1))^2 = 0.04 at n = 1.5
    assert abs(float(fr_dielectric(1.0, 1.5, 1.0)) - 0.04) < 1e-7


def fr_conductor(eta, k, cosi):
    eta, k = eta.astype(np.float32), k.astype(np.float32)
    a = abs(f32(cosi))
    tmpF = (eta * eta + k * k).astype(np.float32)
    tmp = (tmpF * f32(a * a)).astype(np.float32)
    ec2 = (eta * f32(f32(2) * a)).astype(np.float32)
    a2 = f32(a * a)
    rper2 = ((tmpF - ec2 + a2) / (tmpF + ec2 + a2)).astype(np.float32)
    rpar2 = ((tmp - ec2 + f32(1)) / (tmp + ec2 + f32(1))).astype(np.float32)
    return ((rper2 + rpar2) / f32(2)).astype(np.float32)


@pytest.mark.parametrize("cosi", [1.0, 0.7, -0.2, 0.05])
def test_fr_conductor(cosi):
    rng = np.random.default_rng(11)
    eta = rng.uniform(0.1, 3.0, 16).astype(np.float32)
    k = rng.uniform(0.5, 5.0, 16).astype(np.float32)
    out = np.zeros(16, np.float32)
    oracle_py.lib().oracle_fr_conductor(oracle_py._fp(eta), oracle_py._fp(k), cosi, oracle_py._fp(out))
    np.testing.assert_array_equal(out, fr_conductor(eta, k, cosi))


# ---------------------------------------------------------------- Filter.hs:75-84, Image.hs:48-61
def mitchell_table(w, h, b, c):
    b, c, w, h = f32(b), f32(c), f32(w), f32(h)

    def m1d(xp):
        x = abs(f32(f32(2) * xp))
        if x > 1:
            y = f32(f32(f32(f32(-b) - f32(f32(6) * c)) * x) * x) * x
            y = f32(y + f32(f32(f32(f32(6) * b) + f32(f32(30) * c)) * x) * x)
            y = f32(y + f32(f32(f32(f32(-12) * b) - f32(f32(48) * c)) * x))
            y = f32(y + f32(f32(f32(8) * b) + f32(f32(24) * c)))
        else:
            y = f32(f32(f32(f32(f32(f32(12) - f32(f32(9) * b)) - f32(f32(6) * c)) * x) * x) * x)
            y = f32(y + f32(f32(f32(f32(f32(-18) + f32(f32(12) * b)) + f32(f32(6) * c)) * x) * x))
            y = f32(y + f32(f32(6) - f32(f32(2) * b)))
        return f32(y * f32(f32(1) / f32(6)))

    iw, ih = f32(f32(1) / w), f32(f32(1) / h)
    t = np.zeros((16, 16), np.float32)
    for y in range(16):
        fy = f32(f32(f32(y) + f32(0.5)) * h) / f32(16)
        for x in range(16):
            fx = f32(f32(f32(x) + f32(0.5)) * w) / f32(16)
            t[y, x] = f32(m1d(f32(fx * iw)) * m1d(f32(fy * ih)))
    return t


def test_mitchell_table_matches_loader():
    job = load_config("C1")
    assert job.filter_size == (2.0, 2.0)
    want = mitchell_table(2.0, 2.0, 0.333333, 0.333333)
    np.testing.assert_array_equal(job.filter_table(), want)


def test_mitchell_table_c3_width3():
    job = load_config("C3")
    want = mitchell_table(3.0, 3.0, 0.333333, 0.333333)
    np.testing.assert_array_equal(job.filter_table(), want)


# ---------------------------------------------------------------- Microfacet.hs:56-84, 185-192 substrate
INV_TWO_PI = f32(f32(1) / f32(f32(2) * f32(math.pi)))
PI32 = f32(math.pi)
_libm = ctypes.CDLL("libm.so.6")
_libm.powf.restype = ctypes.c_float
_libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]


def powf(x, y):
    """GHC's (**) on Float is C powf; the per-sample path evaluates it in binary64 and rounds once
    (common/cr_math.h), which tests/test_cr_math.py compares with libm's powf."""
    return f32(math.pow(float(x), float(y)))


def aniso_d(ex, ey, wh):
    ex, ey = f32(ex), f32(ey)
    costh = f32(abs(wh[2]))
    d = f32(f32(1) - f32(costh * costh))
    if d == 0:
        return f32(0)
    e = f32(f32(f32(f32(ex * wh[0]) * wh[0]) + f32(f32(ey * wh[1]) * wh[1])) / d)
    return f32(f32(f32(np.sqrt(f32(f32(ex + f32(2)) * f32(ey + f32(2))))) * INV_TWO_PI) * powf(costh, e))


def normalize32(v):
    n = f32(np.sqrt(f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))))
    s = f32(f32(1) / n)
    return np.array([f32(v[0] * s), f32(v[1] * s), f32(v[2] * s)], np.float32)


def fblend_eval(wo, wi, rd, rs, ex, ey):
    """mkFresnelBlend's e wo wi with depth 0 (no absorption): diff + spec, GHC's evaluation order."""
    costi, costo = f32(abs(wi[2])), f32(abs(wo[2]))
    one = f32(1)
    p5 = lambda x: powf(x, 5.0)   # noqa: E731
    wd = f32(f32(f32(f32(f32(costo * f32(28)) / f32(23)) * PI32) * f32(one - p5(f32(one - f32(f32(0.5) * costi))))) *
             f32(one - p5(f32(one - f32(f32(0.5) * costo)))))
    wh = normalize32(wi + wo)
    if wh[2] < 0:
        wh = -wh
    costih = f32(abs(f32(f32(f32(wi[0] * wh[0]) + f32(wi[1] * wh[1])) + f32(wi[2] * wh[2]))))
    mx = costo if costi <= costo else costi                                     # GHC max
    ws = f32(f32(aniso_d(ex, ey, wh) * costo) / f32(f32(f32(4) * costih) * mx))
    sk = p5(f32(one - costih))
    diff = ((rd * (one - rs)).astype(np.float32) * wd).astype(np.float32)      # white * rd * (white - rs)
    schlick = (rs + ((one - rs) * sk).astype(np.float32)).astype(np.float32)
    return (diff + (schlick * ws).astype(np.float32)).astype(np.float32)


@pytest.mark.parametrize("ex,ey", [(20.0, 20.0), (200.0, 5000.0), (50.0, 10.0)])
def test_fresnel_blend_eval(ex, ey):
    rng = np.random.default_rng(int(ex + ey))
    rd = rng.uniform(0, 1, 16).astype(np.float32)
    rs = rng.uniform(0, 1, 16).astype(np.float32)
    ra = rng.uniform(0, 1, 16).astype(np.float32)
    L = oracle_py.lib()
    for _ in range(16):
        wo = normalize32(rng.normal(size=3).astype(np.float32))
        wi = normalize32(rng.normal(size=3).astype(np.float32))
        wo[2], wi[2] = abs(wo[2]), abs(wi[2])
        wh = normalize32(wi + wo)
        assert f32(L.oracle_aniso_d(ex, ey, oracle_py._fp(wh))) == aniso_d(ex, ey, wh)
        out = np.zeros(16, np.float32)
        L.oracle_fblend_eval(oracle_py._fp(wo), oracle_py._fp(wi), oracle_py._fp(rd), oracle_py._fp(rs),
                             oracle_py._fp(ra), oracle_py._fp(np.array([ex, ey, 0.0], np.float32)), oracle_py._fp(out))
        np.testing.assert_array_equal(out, fblend_eval(wo, wi, rd, rs, ex, ey))
        # depth > 0 multiplies the diffuse term by exp(-ra depth (ci + co) / (ci co)) and nothing else
        out_a = np.zeros(16, np.float32)
        L.oracle_fblend_eval(oracle_py._fp(wo), oracle_py._fp(wi), oracle_py._fp(rd), oracle_py._fp(rs),
                             oracle_py._fp(ra), oracle_py._fp(np.array([ex, ey, 0.5], np.float32)), oracle_py._fp(out_a))
        assert np.all(out_a <= out + 1e-6)
