"""SPPM renderer (Renderer/SPPM.hs), SURVEY.md 8(f) row f4: the second consumer of the trace core.

CPU: the loader's `sppm` block and overrides, the oracle against its committed golden vectors
(tests/golden/sppm_X5.npz: cornell-box as shipped; sppm_X6.npz: sun-sky as shipped -- infinite
sun/sky photons and glass eye trees; sppm_X13.npz: delta-lights.bling switched to SPPM -- photons
from a point and a directional light next to an area light, sample' Light.hs:181-213), and
properties read off the reference source (statsUpdate, getPixel with splats).
GPU: the HIP pass (k_sppm_eye / hash / k_sppm_photon / k_sppm_stats) against the same goldens.

Parity anchor: the reference's tests hold no SPPM vectors, and its MWC streams are entropy-seeded,
so the eye and photon samples are keyed by the counter RNG; the goldens are
oracle-generated -- parity unpinned beyond the restated source.

GPU tolerances (the sums run through float atomics in another order, libm vs ocml ulps):
  * hit points, eye rays: within 0.5 %; photons emitted: exact; photon rays within 1 %;
    (photon, hit point) pairs within 2 %;
  * eye-pass film: image relative L2 of XYZ/W <= 1e-2; splat: relative L2 <= 3e-2;
  * pixel radii after two passes: >= 97 % of the extent pixels within 1e-5 relative.
"""
import os

import numpy as np
import pytest

from bling_amd.scene import load_config
from oracle_py import OracleSppm

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x0B11A6


def golden(name):
    return np.load(os.path.join(HERE, "golden", f"sppm_{name}.npz"))


# ------------------------------------------------------------------ loader
def test_loader_reads_sppm_blocks_as_shipped():
    c = load_config("X5").config                       # cornell-box.bling:24
    assert c.renderer == 2                             # BLING_RENDERER_SPPM: the last renderer block (T1)
    assert (c.sppm_photons, c.max_depth) == (20000, 10)
    assert c.sppm_radius == np.float32(10) and c.sppm_alpha == np.float32(0.9)
    assert c.sppm_threads == 8                         # default numCapabilities of the modelled run
    s = load_config("X6").config                       # sun-sky.bling: alpha omitted -> option 0.8
    assert s.renderer == 2 and (s.sppm_photons, s.max_depth) == (50000, 10)
    assert s.sppm_radius == np.float32(0.2) and s.sppm_alpha == np.float32(0.8)


def test_sppm_overrides():
    c = load_config("C1", "sppm=1000,3,2.5;sppm_threads=3;image=16,16").config
    assert c.renderer == 2 and (c.sppm_photons, c.max_depth, c.sppm_threads) == (1000, 3, 3)
    assert c.sppm_radius == np.float32(2.5) and c.sppm_alpha == np.float32(0.8)
    assert load_config("X5", "force_path=1;stratified=2,2;path=5,2").config.renderer == 0


# ------------------------------------------------------------------ oracle
def _digest(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["X5", "X6", "X13", "X13q"])
def test_oracle_matches_goldens(name):
    g = golden(name)
    job = load_config(name.rstrip("q"), str(g["overrides"]))
    o = OracleSppm(job)
    w, h = job.width, job.height
    film = np.zeros(w * h * 4, np.float32)
    splat = np.zeros(w * h * 3, np.float32)
    for p in range(1, len(g["stats"]) + 1):
        film, splat, st = o.render_pass(seed=SEED, pass_index=p, film=film, splat=splat)
        got = [st.hitpoints, st.photons, st.photon_rays, st.photon_hits, st.cam_rays, st.dropped]
        assert got == list(g["stats"][p - 1])
        r2, n = o.pixel_stats()
        assert np.array_equal(r2, g["r2"][p - 1]) and np.array_equal(n, g["n"][p - 1])
    if "film" in g:
        assert np.array_equal(film.reshape(h, w, 4), g["film"])
        assert np.array_equal(splat.reshape(h, w, 3), g["splat"])
    else:
        assert _digest(film.reshape(h, w, 4)) == str(g["film_sha256"])
        assert _digest(splat.reshape(h, w, 3)) == str(g["splat_sha256"])


def test_tree_lookup_bound_drops_pairs_on_x13q():
    """treeLookup (SPPM.hs:391-404) prunes a subtree with the node's mr, which mixes pivots' r2 and
    leaves' r (mkKdTree, :363-389).  Once radii are below 1 and differ per pixel, a pivot whose r
    exceeds every mr above it can be skipped although the photon lies within its radius.  The X13q
    golden reaches that case: the literal lookup finds fewer pairs than the all-within-radius query
    in a later pass (never more), and some pixels' radii then differ."""
    g = golden("X13q")
    pairs, pairs_all = g["stats"][:, 3], g["pairs_all_within"]
    assert pairs[0] == pairs_all[0]                     # pass 1: one radius everywhere, mr = r
    assert (pairs <= pairs_all).all() and (pairs < pairs_all).any()
    assert (g["r2"][-1] < 1).all() and len(np.unique(g["r2"][-1])) > 100
    assert (g["r2"][-1] != g["r2_all_within"][-1]).sum() >= 1


@pytest.mark.parametrize("name", ["X5", "X6", "X13"])
def test_stats_update_properties(name):
    """statsUpdate (SPPM.hs:272-291): n' = n + a m, r2' = r2 n' / (n + m) -- radii never grow and
    pixels without photon hits keep both values."""
    g = golden(name)
    job = load_config(name, str(g["overrides"]))
    a, r0 = np.float32(job.config.sppm_alpha), np.float32(job.config.sppm_radius)
    r2, n = g["r2"], g["n"]
    assert (r2[0] <= r0 * r0).all() and (r2[1] <= r2[0]).all()
    assert (n[1] >= n[0]).all() and (n[0] >= 0).all()
    ch = n[1] != n[0]
    assert ch.any()
    m = np.rint((n[1][ch] - n[0][ch]) / a)             # the merged photon count of the pass
    assert (m >= 1).all()
    n2 = (n[0][ch] + a * m.astype(np.float32)).astype(np.float32)
    assert np.array_equal(n2, n[1][ch])
    ratio = (n2 / (n[0][ch] + m.astype(np.float32))).astype(np.float32)
    assert np.array_equal((r2[0][ch] * ratio).astype(np.float32), r2[1][ch])
    assert np.array_equal(r2[1][~ch], r2[0][~ch])


def test_photon_count_is_threads_times_sn_squared():
    g = golden("X5")
    # photonCount 20000 over 4 samplers: sn = ceiling (sqrt (20000 / 4)) = 71 (SPPM.hs:474)
    assert int(g["stats"][0][1]) == 4 * 71 * 71


def test_film_splat_to_rgb_matches_getpixel():
    """bling_host_film_splat_to_rgb restates getPixel (Image.hs:301-314) + xyzToRgb."""
    import ctypes as C
    from bling_amd import _ffi
    lib = _ffi.host()
    lib.bling_host_film_splat_to_rgb.argtypes = [_ffi.c_f32p, _ffi.c_f32p, C.c_float, C.c_int, C.c_int, _ffi.c_f32p]
    rng = np.random.default_rng(3)
    w, h = 7, 5
    film = rng.uniform(0, 2, (h * w, 4)).astype(np.float32)
    film[::3, 0] = 0.0
    splat = rng.uniform(0, 5, (h * w, 3)).astype(np.float32)
    sw = np.float32(1 / 4096)
    out = np.zeros(h * w * 3, np.float32)
    lib.bling_host_film_splat_to_rgb(_ffi.f32ptr(film.reshape(-1)), _ffi.f32ptr(splat.reshape(-1)), float(sw), w, h,
                                     _ffi.f32ptr(out))
    f32 = np.float32
    W = film[:, 0]
    iw = np.where(W == 0, f32(0), f32(1) / np.where(W == 0, f32(1), W)).astype(f32)
    xyz = (sw * splat).astype(f32)
    xyz = np.where(W[:, None] == 0, xyz, (xyz + film[:, 1:] * iw[:, None]).astype(f32))
    x, y, z = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    r = f32(3.240479) * x - f32(1.537150) * y - f32(0.498535) * z
    gg = f32(-0.969256) * x + f32(1.875991) * y + f32(0.041556) * z
    b = f32(0.055648) * x - f32(0.204043) * y + f32(1.057311) * z
    assert np.array_equal(out.reshape(-1, 3), np.stack([r, gg, b], 1).astype(f32))


# ------------------------------------------------------------------ GPU
def _rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["X5", "X6", "X13"])
def test_gpu_sppm_matches_goldens(name):
    from bling_amd.render import Context
    g = golden(name)
    job = load_config(name, str(g["overrides"]))
    w, h = job.width, job.height
    ctx = Context(0)
    ctx.upload(job)
    film = np.zeros(w * h * 4, np.float32)
    splat = np.zeros(w * h * 3, np.float32)
    for p in (1, 2):
        film, splat, st = ctx.sppm_pass(seed=SEED, pass_index=p, film=film, splat=splat)
        gs = g["stats"][p - 1]
        assert st.photons == gs[1]
        assert abs(int(st.hitpoints) - int(gs[0])) <= 0.005 * gs[0] + 1, (st.hitpoints, gs[0])
        assert abs(int(st.cam_rays) - int(gs[4])) <= 0.005 * gs[4] + 1, (st.cam_rays, gs[4])
        assert abs(int(st.photon_rays) - int(gs[2])) <= 0.01 * gs[2] + 1, (st.photon_rays, gs[2])
        assert abs(int(st.photon_hits) - int(gs[3])) <= 0.02 * gs[3] + 1, (st.photon_hits, gs[3])
    r2, n = ctx.sppm_pixel_stats()
    ok = np.abs(r2 - g["r2"][1]) <= 1e-5 * g["r2"][1]
    assert ok.mean() >= 0.97, ok.mean()
    f = film.reshape(h, w, 4)
    gf = g["film"]
    hasw = (gf[..., 0] > 0) & (f[..., 0] > 0)
    xg = f[..., 1:][hasw] / f[..., :1][hasw]
    xo = gf[..., 1:][hasw] / gf[..., :1][hasw]
    assert np.isfinite(f).all() and _rel_l2(xg, xo) <= 1e-2
    assert np.isfinite(splat).all() and _rel_l2(splat.reshape(h, w, 3), g["splat"]) <= 3e-2
    ctx.close()


@pytest.mark.gpu
def test_gpu_sppm_tree_lookup_matches_oracle():
    """X13q: radii below 1 that differ per pixel, where treeLookup's mixed r / r2 bound drops pairs
    (test_tree_lookup_bound_drops_pairs_on_x13q).  The device's per-bucket kd-trees (k_sppm_kd) and
    lookup against the oracle's over three passes: hit points, photons, eye and photon rays, photon /
    hit-point pairs and every pixel's radius exact in every pass.
    History: in round 5 (old sampler, radius 0.5) passes 2-3 differed by 3 and 23 pairs of ~10^5 while
    hit points, trees and photon rays agreed, and the bar was loosened to 5e-4.  Round 6 found that
    the device skipped the reference's first query step, kdTreePrimitive's intersectAABB against the
    kd-tree's bounds (tests/test_kd_root.py): a photon ray that grazes the bounds where a primitive's
    edge lies on them hits on the device only, splats, and if the walk then ends (Russian roulette)
    the photon ray counts still agree.  The device now makes that test.  With round 6's sampler the
    case does not recur at radius 0.5 or 0.8 with or without the test (gpurun_out/r06h: every pass
    exact both ways), so the cause of the round-5 pairs is this candidate, not proven; the bar is
    exact again (measured on MI355X: gpurun_out/r06g)."""
    from bling_amd.render import Context
    from parity_util import report
    g = golden("X13q")
    job = load_config("X13", str(g["overrides"]))
    w, h = job.width, job.height
    ctx = Context(0)
    ctx.upload(job)
    film = np.zeros(w * h * 4, np.float32)
    splat = np.zeros(w * h * 3, np.float32)
    for p in range(1, len(g["stats"]) + 1):
        film, splat, st = ctx.sppm_pass(seed=SEED, pass_index=p, film=film, splat=splat)
        gs = [int(x) for x in g["stats"][p - 1]]
        r2, n = ctx.sppm_pixel_stats()
        r2_exact = float(np.mean(r2 == g["r2"][p - 1]))
        report(f"sppm_x13q_pass{p}", hitpoints=int(st.hitpoints), hitpoints_oracle=gs[0], photon_rays=int(st.photon_rays),
               photon_rays_oracle=gs[2], pairs=int(st.photon_hits), pairs_oracle=gs[3], r2_exact_frac=r2_exact)
        assert [st.hitpoints, st.photons, st.cam_rays, st.dropped] == [gs[0], gs[1], gs[4], gs[5]], (p, gs)
        assert st.photon_rays == gs[2], (p, st.photon_rays, gs[2])
        assert st.photon_hits == gs[3] and r2_exact == 1.0, (p, st.photon_hits, gs[3], r2_exact)
    ctx.close()


@pytest.mark.gpu
def test_gpu_sppm_is_deterministic_and_resets():
    from bling_amd.render import Context
    job = load_config("X5", "image=64,64")
    ctx = Context(0)
    ctx.upload(job)
    f1, s1, st1 = ctx.sppm_pass(seed=SEED, pass_index=1)
    r2a, _ = ctx.sppm_pixel_stats()
    ctx.sppm_reset()
    r2r, nr = ctx.sppm_pixel_stats()
    assert (r2r == np.float32(100.0)).all() and (nr == 0).all()
    f2, s2, st2 = ctx.sppm_pass(seed=SEED, pass_index=1)
    r2b, _ = ctx.sppm_pixel_stats()
    assert st1.hitpoints == st2.hitpoints and st1.photon_rays == st2.photon_rays
    assert st1.photon_hits == st2.photon_hits and np.array_equal(r2a, r2b)
    assert _rel_l2(f1, f2) <= 1e-6 and _rel_l2(s1, s2) <= 1e-5     # float-atomic order only
    ctx.close()


@pytest.mark.gpu
def test_gpu_sppm_as_shipped_cornell_pass():
    """cornell-box.bling as shipped (480 x 480, 20000 photons, maxDepth 10): one pass, sane output."""
    from bling_amd.render import Context
    job = load_config("X5")
    ctx = Context(0)
    ctx.upload(job)
    film, splat, st = ctx.sppm_pass(seed=SEED, pass_index=1)
    assert st.photons == 8 * 50 * 50 and st.hitpoints > 0.9 * 484 * 484
    assert np.isfinite(film).all() and np.isfinite(splat).all() and splat.sum() > 0
    ctx.close()


@pytest.mark.gpu
def test_gpu_sppm_refuses_computed_textures():
    """SPPM keeps each hit point's BSDF between its eye and photon passes; computed spectra (blend /
    gradient / checker) and cellNoise exist only while one thread shades (FT_PROCTEX), so
    bling_sppm_pass refuses such scenes with BLING_EUNSUPPORTED instead of rendering them wrongly."""
    from bling_amd.render import Context
    job = load_config("X11", "sppm=2000,3,1")
    ctx = Context(0)
    ctx.upload(job)
    with pytest.raises(Exception, match="SPPM"):
        ctx.sppm_pass(seed=SEED, pass_index=1)
    ctx.close()
