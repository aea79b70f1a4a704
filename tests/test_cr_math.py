"""How far the shared transcendentals depart from the reference's.

The per-sample path -- oracle and device alike -- evaluates every binary32 tan / asin / atan / atan2 /
pow with one shared binary64 algorithm rounded once, and exp / log / sinh / sin / cos / acos with
shared binary32 algorithms within one ulp (bling_amd/csrc/common/cr_math.h): checked here against
binary64 libm, and the same bits on the device (checked on the GPU).  GHC's Float primops, which the reference
calls, are libm's binary32 functions instead.  Both are within about one ulp of the exact value,
so they differ only where libm's binary32 result is not the correctly rounded one.  These tests
measure that departure, at two levels, and pin it:

  * per function, over the argument ranges the path uses: how many results differ, and by at most
    one ulp (two for glibc's sinhf);
  * per path: the oracle re-run with libm's binary32 functions (oracle_set_libm32) against its
    default, on the C5 trace golden's rays (the Mandelbulb march) and on per-sample radiance of C2 and
    C5 -- the reference-arithmetic uncertainty of every golden, "parity unpinned" at that level.

CPU only; the numbers are printed and written to gpurun_out/parity_metrics.jsonl (report).
"""
import ctypes
import math
import os

import numpy as np
import pytest

import oracle_py
from bling_amd.scene import load_config
from parity_util import random_samples, report, spectra_mismatch

f32 = np.float32
_m = ctypes.CDLL("libm.so.6")
for _fn in ("sinf", "cosf", "tanf", "acosf", "asinf", "atanf", "expf", "logf", "sinhf"):
    getattr(_m, _fn).restype = ctypes.c_float
    getattr(_m, _fn).argtypes = [ctypes.c_float]
for _fn in ("powf", "atan2f"):
    getattr(_m, _fn).restype = ctypes.c_float
    getattr(_m, _fn).argtypes = [ctypes.c_float, ctypes.c_float]

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SEED = 0x0B11A6

# (libm binary32 name, binary64 function, argument sampler) over the ranges the path evaluates
CASES = {
    "sinf": (math.sin, lambda r, n: r.uniform(-2 * np.pi, 2 * np.pi, n)),      # warps, lens, sky map
    "cosf": (math.cos, lambda r, n: r.uniform(-2 * np.pi, 2 * np.pi, n)),
    "tanf": (math.tan, lambda r, n: r.uniform(-1.5, 1.5, n)),                   # Oren-Nayar, anisotropic phi
    "acosf": (math.acos, lambda r, n: r.uniform(-1, 1, n)),                     # sky theta / gamma, sphere v
    "atanf": (math.atan, lambda r, n: r.uniform(-50, 50, n)),
    "expf": (math.exp, lambda r, n: r.uniform(-30, 10, n)),                     # Perez, DE step
    "logf": (math.log, lambda r, n: r.uniform(1.2, 1e8, n)),                    # Mandelbulb potential
    "sinhf": (math.sinh, lambda r, n: r.uniform(1e-6, 3, n)),                   # DE step
}
N_ARGS = 1 << 15


def _ulps(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


@pytest.mark.parametrize("name", sorted(CASES))
def test_unary_departure_at_most_one_ulp(name):
    f64, gen = CASES[name]
    x = gen(np.random.default_rng(3), N_ARGS).astype(np.float32)
    lib = getattr(_m, name)
    l32 = np.array([lib(float(v)) for v in x], np.float32)
    cr = np.array([f64(float(v)) for v in x]).astype(np.float32)
    d = _ulps(l32, cr)
    report(f"cr_math[{name}]", args=len(x), differ=int((d > 0).sum()), max_ulps=int(d.max()))
    # glibc documents sinhf within 2 ulps (measured: 26 % of the DE-step arguments differ, by <= 2);
    # the others within 1 (measured 0.01 % (logf) .. 8 % (acosf) of the arguments)
    assert d.max() <= (2 if name == "sinhf" else 1)


def test_pow_atan2_departure_at_most_one_ulp():
    r = np.random.default_rng(4)
    x = r.uniform(0, 1, N_ARGS).astype(np.float32)          # powf(cos, e): Blinn, anisotropic
    y = r.uniform(0.01, 2000, N_ARGS).astype(np.float32)
    l32 = np.array([_m.powf(float(a), float(b)) for a, b in zip(x, y)], np.float32)
    cr = np.array([math.pow(float(a), float(b)) for a, b in zip(x, y)]).astype(np.float32)
    dp = _ulps(l32, cr)
    u = r.uniform(-1, 1, N_ARGS).astype(np.float32)
    v = r.uniform(-1, 1, N_ARGS).astype(np.float32)
    l32 = np.array([_m.atan2f(float(a), float(b)) for a, b in zip(u, v)], np.float32)
    cr = np.array([math.atan2(float(a), float(b)) for a, b in zip(u, v)]).astype(np.float32)
    da = _ulps(l32, cr)
    report("cr_math[powf,atan2f]", args=len(x), pow_differ=int((dp > 0).sum()), pow_max_ulps=int(dp.max()),
           atan2_differ=int((da > 0).sum()), atan2_max_ulps=int(da.max()))
    assert dp.max() <= 1 and da.max() <= 1


def _inputs(name: str, n: int, seed: int):
    """Arguments over the ranges the path uses plus edge values (zeros, axes, near-boundaries)."""
    r = np.random.default_rng(seed)
    ranges = {"sin": (-30, 30), "cos": (-30, 30), "tan": (-1.5, 1.5), "asin": (-1, 1), "acos": (-1, 1),
              "atan": (-60, 60), "exp": (-110, 90), "sinh": (-12, 12), "atan2": (-2, 2)}
    name = {"sincos_s": "sin", "sincos_c": "cos"}.get(name, name)
    if name == "log":
        x = np.exp(r.uniform(-100, 88, n))
    elif name == "pow":
        x = r.uniform(0, 1.2, n)
    else:
        x = r.uniform(*ranges[name], n)
    edges = {"sin": [0, -0.0, 1e-30, np.pi / 2, np.pi, 6e5, -7e6], "cos": [0, np.pi / 4, 1e5, 3e6],
             "tan": [0, 1e-20, 1.5707963], "asin": [1, -1, 0, -0.0, 0.9999999], "acos": [1, -1, 0, -0.0, 0.9999999],
             "atan": [0, -0.0, 1e30, -1e30, np.inf, -np.inf, 1, 0.2679492], "exp": [0, 88.72, 89, -87, -103, -150, -200],
             "log": [1, 1e-45, 3.4e38, 0.5, 2, 0.9999999], "sinh": [0, -0.0, 1e-30, 1, -1, 89, 95]}
    x = np.concatenate([np.array(edges.get(name, []), np.float64), x]).astype(np.float32)[:n]
    y = None
    if name == "atan2":
        y = np.concatenate([np.array([0, -0.0, 1, -1, 0, -0.0], np.float32), r.uniform(-2, 2, n)]).astype(np.float32)[:n]
        x[:6] = np.array([0, 0, 0, 0, -0.0, -0.0], np.float32)
    if name == "pow":
        y = r.uniform(0.01, 2000, n).astype(np.float32)
        y[:4] = np.array([0, 1, 2, 0.5], np.float32)
    return x, y


_F64 = {"sin": math.sin, "cos": math.cos, "tan": math.tan, "asin": math.asin, "acos": math.acos, "atan": math.atan,
        "exp": math.exp, "log": math.log, "sinh": math.sinh, "atan2": math.atan2, "pow": math.pow,
        "sincos_s": math.sin, "sincos_c": math.cos}


def _cr_ref(name, x, y):
    """binary64 libm, rounded once (the correctly rounded binary32 value but for ties within 2^-29 ulp)"""
    f = _F64[name]
    out = []
    for i, a in enumerate(x):
        try:
            v = f(float(a), float(y[i])) if y is not None else f(float(a))
        except OverflowError:
            v = math.inf
        except ValueError:
            v = math.nan
        out.append(v)
    with np.errstate(over="ignore"):
        return np.array(out).astype(np.float32)


# exp, log, sinh, sin, cos and acos are faithful binary32 algorithms (round 5, cr_math.h exp_f /
# log_f / sincos_f / acosf): within one ulp of the exact value, the correctly rounded one for most
# arguments -- the share that is not, over these arguments, at most (twice the measured 5.5 %,
# 0.55 %, 20.6 %, 5.4 %, 5.5 %, 7.5 %)
FAITHFUL = {"exp": 0.11, "log": 0.011, "sinh": 0.42, "sin": 0.11, "cos": 0.11, "sincos_s": 0.11, "sincos_c": 0.11,
            "acos": 0.15}


@pytest.mark.parametrize("name", oracle_py.CR_FUNCS)
def test_shared_functions_are_correctly_rounded(name):
    """cr_math.h's binary64 algorithms, rounded to binary32, against binary64 libm rounded once;
    the binary32 exp / log / sinh within one ulp of it."""
    x, y = _inputs(name, 1 << 16, 7)
    got = oracle_py.cr_eval(name, x, y)
    want = _cr_ref(name, x, y)
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    d = _ulps(got, want)
    d = np.where(np.isfinite(got) & np.isfinite(want), d, 0)
    report(f"cr_math_accuracy[{name}]", args=len(x), differ=int((~same).sum()), max_ulps=int(d.max()))
    assert d.max() <= 1
    assert ((np.isnan(got) == np.isnan(want)) & (np.isinf(got) == np.isinf(want))).all()
    if name in FAITHFUL:
        assert (~same).sum() <= FAITHFUL[name] * len(x)
    else:
        # the series are cut at ~1e-13 relative: about 1 in 10^5 results may round the other way
        assert (~same).sum() <= 4
    np.testing.assert_array_equal(np.signbit(got[got == 0]), np.signbit(want[got == 0]))   # signed zeros


def test_sincos_is_sin_and_cos():
    """sincosf (one range reduction) returns sinf's and cosf's bits, huge and special arguments included."""
    x, _ = _inputs("sin", 1 << 16, 13)
    x = np.concatenate([x, np.array([np.nan, np.inf, -np.inf, 3e38, -1e10, 524288.0, 524289.0], np.float32)])
    for a, b in (("sincos_s", "sin"), ("sincos_c", "cos")):
        got, want = oracle_py.cr_eval(a, x), oracle_py.cr_eval(b, x)
        assert ((got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))).all(), a


@pytest.mark.gpu
@pytest.mark.parametrize("name", oracle_py.CR_FUNCS)
def test_device_equals_host(name):
    """The same source on gfx950 (libbling_mathcheck.so) and on the host: identical bits."""
    lib = ctypes.CDLL(os.path.join(os.path.dirname(GOLD), "..", "bling_amd", "_lib", "libbling_mathcheck.so"))
    x, y = _inputs(name, 1 << 20, 11)
    out = np.zeros_like(x)
    fp = ctypes.POINTER(ctypes.c_float)
    lib.bling_cr_eval_device.argtypes = [ctypes.c_int, fp, fp, fp, ctypes.c_size_t]
    rc = lib.bling_cr_eval_device(oracle_py.CR_FUNCS.index(name), x.ctypes.data_as(fp),
                                  None if y is None else y.ctypes.data_as(fp), out.ctypes.data_as(fp), len(x))
    assert rc == 0
    host = oracle_py.cr_eval(name, x, y)
    same = (out.view(np.uint32) == host.view(np.uint32)) | (np.isnan(out) & np.isnan(host))
    report(f"cr_math_device[{name}]", args=len(x), mismatch=int((~same).sum()))
    assert same.all()


@pytest.fixture
def libm32():
    yield lambda on: oracle_py.lib().oracle_set_libm32(1 if on else 0)
    oracle_py.lib().oracle_set_libm32(0)


def test_march_departure_on_c5_golden(libm32):
    """The Mandelbulb march (Fractal.hs:37-137) under GHC's libm binary32 log / exp / sinh against the
    committed C5 trace golden (binary64-once): how many of its 1 024 rays change hit or distance."""
    g = np.load(os.path.join(GOLD, "trace_C5.npz"))
    orc = oracle_py.Oracle(load_config("C5", str(g["overrides"]) or None))
    t0, p0, _, _ = orc.trace(g["rays"])
    libm32(True)
    t1, p1, _, _ = orc.trace(g["rays"])
    libm32(False)
    np.testing.assert_array_equal(t0, g["t"])                 # default mode = the golden
    fin = np.isfinite(t0) & np.isfinite(t1)
    rel = np.abs(t1[fin] - t0[fin]) / np.maximum(np.abs(t0[fin]), 1e-6)
    rec = report("cr_math_departure[C5 march]", rays=len(t0), prim_changed=int((p0 != p1).sum()),
                 t_changed=int((t0[fin] != t1[fin]).sum()), t_over_1e_3=int((rel > 1e-3).sum()),
                 t_max_rel=float(rel.max(initial=0)))
    # measured: 295 of the 1 024 distances change, two by more than 1e-3 (305 on round 5's golden
    # rays; 143 and one with the round-4 correctly rounded exp / log / sinh; the parity of every
    # fractal golden with the reference's own arithmetic is unpinned at this level)
    assert rec["prim_changed"] <= 16 and rec["t_over_1e_3"] <= 16


@pytest.mark.parametrize("cfg", ["C2", "C5"])
def test_path_departure_per_sample(libm32, cfg):
    """Per-sample radiance of the oracle under libm binary32 vs its default: the share of samples a
    last-ulp difference of the transcendentals moves by more than 1e-4 (relative L1)."""
    job = load_config(cfg)
    orc = oracle_py.Oracle(job)
    smp = random_samples(orc, job, 512, seed=5)
    L0, _, _ = orc.sample_li_batch(smp, seed=SEED, pass_index=1)
    libm32(True)
    L1, _, _ = orc.sample_li_batch(smp, seed=SEED, pass_index=1)
    libm32(False)
    bad, exact, worst, _ = spectra_mismatch(L1, L0)
    report(f"cr_math_departure[{cfg} samples]", samples=len(smp), mismatch=bad, exact=exact)
    # measured: C2 0 of 512 (466 bit-exact); C5 169 of 512 -- the Mandelbulb's paths are chaotic in
    # the last ulp, which is why C5's device-vs-oracle agreement needs identical transcendentals.
    # History of the C5 count ("speed / parity trade"): 97 with round 4's
    # correctly rounded binary64 exp / log / sinh, 159 with round 5's faithful binary32 ones, 169 with
    # the same functions on round 6's sampler (counter_rng.h version 2: another set of 512 samples).
    # The bar is the measured count plus 11 (~7 %): a larger departure is a decision to record, not to
    # absorb.
    assert bad <= (8 if cfg == "C2" else 180)
