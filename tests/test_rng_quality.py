"""Statistical quality of the counter RNG (bling_amd/csrc/common/counter_rng.h, specification version 2).

The sampler draws every value as a hash of (seed, pass, pixel, sample, dimension), so its quality
is the hash's: the values of one sample across its dimensions, of one pixel across its samples and
of neighbouring pixels must look like independent uniforms.  The reference draws them from MWC256
streams (Random.hs:56-96), which are independent by construction; tests/test_mwc_sampler.py checks
that the two samplers' estimators converge to the same film.  Here, on 2^20 keys each, in numpy
(the restatement of tests/test_rng_loader.py, checked there word for word against the oracle):

* 1D uniformity of u01 (4 096 bins);
* pairwise 2D uniformity (64 x 64 bins) and correlation for dimension pairs of one vertex, for
  consecutive samples of one pixel and for neighbouring pixels;
* bit balance of the XOR of two dimensions' words (a differential check of the finaliser).

A chi-square bar of df + 6 sqrt(2 df) rejects with probability ~1e-9 under independence.  The
checks have power: the same bars reject a one-round multiply-xorshift finaliser (corr ~0.1,
test_checks_reject_a_weak_finaliser)."""
import numpy as np
import pytest

U = np.uint32
SEED = 0x0B11A6
N = 1 << 20


def _rotl(x, r):
    return (x << U(r)) | (x >> U(32 - r))


def _mix(h, k):
    k = (k * U(0xcc9e2d51)).astype(U)
    k = _rotl(k, 15)
    k = (k * U(0x1b873593)).astype(U)
    h = h ^ k
    h = _rotl(h, 13)
    return (h * U(5) + U(0xe6546b64)).astype(U)


def _fmix(h):
    h = h ^ (h >> U(16)); h = (h * U(0x85ebca6b)).astype(U)
    h = h ^ (h >> U(13)); h = (h * U(0xc2b2ae35)).astype(U)
    return h ^ (h >> U(16))


def hash5(seed, pss, pixel, sample, dim, fin=_fmix):
    """counter_rng.h hash5 over arrays: draw(sample_key(pixel_key(seed, pass, pixel), sample), dim)."""
    with np.errstate(over="ignore"):
        seed, pss, pixel, sample, dim = (np.asarray(v, dtype=np.uint64).astype(U) for v in (seed, pss, pixel, sample, dim))
        pkey = _mix(_mix(np.broadcast_to(seed, pixel.shape).copy(), pss), pixel)
        skey = _fmix(pkey ^ (sample * U(0x9E3779B9)).astype(U))
        return fin(skey ^ _fmix(dim ^ U(0x2C1B3C6D)))


def _u(h):
    return (h >> U(8)).astype(np.float64) / 16777216.0


def _chi2_bar(df):
    return df + 6.0 * np.sqrt(2.0 * df)


def _chi2_2d(a, b, bins=64):
    i = np.floor(_u(a) * bins).astype(np.int64) * bins + np.floor(_u(b) * bins).astype(np.int64)
    h = np.bincount(i, minlength=bins * bins)
    e = len(a) / (bins * bins)
    return float(((h - e) ** 2 / e).sum()), bins * bins - 1


def _keys(rng):
    pixel = rng.integers(0, 1 << 20, N, dtype=np.uint64)
    sample = rng.integers(0, 64, N, dtype=np.uint64)
    return pixel, sample


# the dimension codes one path vertex at depth d draws (dev_shade.h rnd1 / rnd2, wavefront.h shade_vertex):
# RR 3 + 4d, the continuation's 2D 3d (two words), the light's 2D and the BSDF-MIS 2D
def _vertex_dims(d=4):
    f1, f2 = 0x7000, 0x8000
    return [f1 + 3 + 4 * d, f2 + 2 * (3 * d), f2 + 2 * (3 * d) + 1, f2 + 2 * (3 * d + 1), f2 + 2 * (3 * d + 1) + 1,
            f2 + 2 * (3 * d + 2), f2 + 2 * (3 * d + 2) + 1, 0x4000 + 1, 0x6000 + 2]


def _pairs_ok(a, b):
    chi, df = _chi2_2d(a, b)
    r = np.corrcoef(_u(a), _u(b))[0, 1]
    x = a ^ b
    bias = max(abs(float(((x >> U(k)) & U(1)).mean()) - 0.5) for k in range(8, 32))
    return chi < _chi2_bar(df) and abs(r) < 6.0 / np.sqrt(len(a)) and bias < 6.0 * 0.5 / np.sqrt(len(a)), (chi, r, bias)


def test_u01_is_uniform():
    rng = np.random.default_rng(11)
    pixel, sample = _keys(rng)
    h = hash5(SEED, 3, pixel, sample, 0x7000 + 7)
    u = _u(h)
    assert u.min() >= 0.0 and u.max() <= 1.0 - 2.0 ** -24
    cnt = np.bincount(np.floor(u * 4096).astype(np.int64), minlength=4096)
    e = N / 4096
    chi = float(((cnt - e) ** 2 / e).sum())
    assert chi < _chi2_bar(4095), chi


def test_dimensions_of_one_sample_are_independent():
    rng = np.random.default_rng(12)
    pixel, sample = _keys(rng)
    dims = _vertex_dims()
    words = [hash5(SEED, 1, pixel, sample, d) for d in dims]
    for i in range(len(dims)):
        for j in range(i + 1, len(dims)):
            ok, m = _pairs_ok(words[i], words[j])
            assert ok, (hex(dims[i]), hex(dims[j]), m)


def test_consecutive_samples_and_neighbouring_pixels_are_independent():
    rng = np.random.default_rng(13)
    pixel, sample = _keys(rng)
    for dim in (0x7000 + 3, 0x8000 + 1, 0x4000):
        a = hash5(SEED, 2, pixel, sample, dim)
        ok, m = _pairs_ok(a, hash5(SEED, 2, pixel, sample + 1, dim))
        assert ok, ("samples", hex(dim), m)
        ok, m = _pairs_ok(a, hash5(SEED, 2, pixel + 1, sample, dim))
        assert ok, ("pixels", hex(dim), m)
        ok, m = _pairs_ok(a, hash5(SEED, 3, pixel, sample, dim))
        assert ok, ("passes", hex(dim), m)


def test_checks_reject_a_weak_finaliser():
    """Power of the checks above: a single multiply-xorshift round in place of fmix fails them."""
    def weak(y):
        y = y ^ (y >> U(16)); y = (y * U(0x7feb352d)).astype(U)
        return y ^ (y >> U(15))
    rng = np.random.default_rng(12)
    pixel, sample = _keys(rng)
    dims = _vertex_dims()
    words = [hash5(SEED, 1, pixel, sample, d, fin=weak) for d in dims]
    fails = sum(not _pairs_ok(words[i], words[j])[0] for i in range(len(dims)) for j in range(i + 1, len(dims)))
    assert fails > 0


def test_numpy_restatement_is_the_oracles():
    import oracle_py
    rng = np.random.default_rng(14)
    k = rng.integers(0, 2**32, (5, 500), dtype=np.uint64)
    got = hash5(k[0], k[1], k[2], k[3], k[4])
    want = [oracle_py.hash5(*(int(v) for v in k[:, i])) for i in range(500)]
    assert [int(x) for x in got] == want
