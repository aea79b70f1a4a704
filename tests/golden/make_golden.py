#!/usr/bin/env python3
"""Generate the committed golden vectors from the CPU oracle.

The reference (Haskell) cannot be built here and its tests hold no hot-path vectors, so these
fixtures are produced by the oracle at a fixed seed and committed; tests/test_golden.py re-derives
them (oracle drift = failure) and tests/test_gpu_parity.py checks the HIP core against them.

  python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from bling_amd.scene import load_config  # noqa: E402
from oracle_py import Oracle, OracleSppm  # noqa: E402

SEED = 0x0B11A6
# per config: small image override, ray-box for random rays
TRACE_CASES = {
    "C1": ("image=64,64", [5, 5, 5], [550, 540, 555]),
    "C3": ("image=96,54", [-200, -80, -200], [200, 200, 200]),
    "C4": ("image=64,64", [-4, 0.1, -4], [4, 3, 4]),
    "C5": ("image=64,64", [-1.5, -1.5, -1.5], [1.5, 1.5, 1.5]),
    "X1": ("", [-6, 0.05, -6], [6, 8, 6]),          # disk / cylinder / box, transMatte, shinyMetal
    "X2": ("", [-4, 0.5, -4], [4, 5, 4]),           # heightMap mesh with shading normals
    "X3": ("", [-1.6, -0.9, -1.6], [1.6, 1.6, 1.6]), # quaternion Julia fractal
    "X4": ("", [-5, 0.05, -4], [5, 6, 5]),          # directLighting scene: spheres, mirror, box
    "X7": ("", [-5, 0.05, -4], [5, 5, 4]),          # substrate spheres
    "X10": ("", [-8, 0.05, -8], [8, 8, 8]),         # cellnoise.bling: spheres on boxes (cellNoise bumps)
    "X11": ("", [-5, 0.05, -4], [5, 6, 4]),         # computed-texture spheres
    "X12": ("", [-10, 0.05, -10], [10, 10, 10]),    # crystal.bling: glass sphere, quasiCrystal ground
    "X13": ("", [-5, 0.05, -4], [5, 5, 5]),          # point + directional lights next to an area light
    "X14": ("", [-5, 0.05, -4], [5, 5, 4]),          # image textures, image env map
    "X15": ("", [-5, 0.05, -4], [5, 5, 4]),          # image env map over constant materials
    "X16": ("", [-4, 0.05, -3], [4, 3, 3]),          # Bezier patches tessellated at load
}
N_CAM = 16     # camera rays per side  -> 256
N_RAND = 768   # random rays           -> 1024 rays per config


def camera_batch(orc, job, rng):
    xs = np.linspace(0, job.width - 1, N_CAM).astype(int)
    ys = np.linspace(0, job.height - 1, N_CAM).astype(int)
    rays = []
    for y in ys:
        for x in xs:
            r = orc.camera_ray(int(x), int(y), int(rng.integers(0, job.spp)), seed=SEED)
            rays.append([r[2], r[3], r[4], r[5], r[6], r[7], 0.0, np.inf])
    return np.array(rays, np.float32).T


def random_batch(lo, hi, rng):
    o = rng.uniform(lo, hi, size=(N_RAND, 3)).astype(np.float32)
    d = rng.normal(size=(N_RAND, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tmax = np.where(rng.uniform(size=N_RAND) < 0.25, rng.uniform(0.1, 300, N_RAND), np.inf).astype(np.float32)
    return np.concatenate([o.T, d.T, np.zeros((1, N_RAND), np.float32), tmax[None]], 0).astype(np.float32)


def trace_golden(name):
    over, lo, hi = TRACE_CASES[name]
    job = load_config(name, over or None)
    orc = Oracle(job)
    rng = np.random.default_rng(1234)
    rays = np.ascontiguousarray(np.concatenate([camera_batch(orc, job, rng), random_batch(lo, hi, rng)], 1))
    t, prim, bary, _ = orc.trace(rays)
    _, occ, _, _ = orc.trace(rays, any_hit=True)
    return dict(overrides=over, rays=rays, t=t, prim=prim, bary=bary, occluded=occ)


def sample_golden(name="C1", over="image=64,64"):
    job = load_config(name, over)
    orc = Oracle(job)
    rng = np.random.default_rng(99)
    (x0, x1, y0, y1), _ = orc.extent()
    k = 256
    smp = np.stack([rng.integers(x0, x1 + 1, k), rng.integers(y0, y1 + 1, k), rng.integers(0, job.spp, k)],
                   1).astype(np.int32)
    L = np.zeros((k, 16), np.float32)
    img = np.zeros((k, 2), np.float32)
    for i, (x, y, n) in enumerate(smp):
        L[i], img[i], _ = orc.sample_li(int(x), int(y), int(n), seed=SEED)
    return dict(overrides=over, samples=smp, L=L, img=img)


def film_golden():
    job = load_config("C1", "image=48,48")
    film, st = Oracle(job).render(seed=SEED, pass_index=0, threads=1)
    return dict(overrides="image=48,48", film=film.reshape(48, 48, 4),
                counts=np.array([st.samples, st.rays_camera, st.rays_continuation, st.rays_mis, st.rays_shadow],
                                np.int64))


# SPPM (Renderer/SPPM.hs) feature scenes as shipped, small images, 4 photon samplers, 2 passes; X13
# (delta-lights.bling) switched to SPPM: photons from point and directional lights (Light.hs:181-213).
# X13q: the same scene at radius 0.8 (0.5 before the round-6 sampler) with alpha 0.1 over three passes, so the radii fall below 1 and
# differ per pixel and treeLookup's bound (r2 at pivots, r at leaves, SPPM.hs:363-404) drops pairs an
# all-within-radius query would find (recorded as `pairs_all_within`); its films are kept as digests.
SPPM_CASES = {"X5": "image=40,40;sppm_threads=4", "X6": "image=48,27;sppm_threads=4",
              "X13": "image=48,36;sppm=20000,6,0.25;sppm_threads=4",
              "X13q": "image=128,96;sppm=200000,6,0.8,0.1;sppm_threads=4"}
SPPM_PASSES = {"X13q": 3}


def sppm_run(name, all_within=False):
    over = SPPM_CASES[name]
    job = load_config(name.rstrip("q"), over)
    OracleSppm.set_lookup(all_within)
    try:
        o = OracleSppm(job)
        w, h = job.width, job.height
        film = np.zeros(w * h * 4, np.float32)
        splat = np.zeros(w * h * 3, np.float32)
        stats, r2s, ns = [], [], []
        for p in range(1, SPPM_PASSES.get(name, 2) + 1):
            film, splat, st = o.render_pass(seed=SEED, pass_index=p, film=film, splat=splat)
            stats.append([st.hitpoints, st.photons, st.photon_rays, st.photon_hits, st.cam_rays, st.dropped])
            r2, n = o.pixel_stats()
            r2s.append(r2)
            ns.append(n)
    finally:
        OracleSppm.set_lookup(False)
    return over, film.reshape(h, w, 4), splat.reshape(h, w, 3), np.stack(r2s), np.stack(ns), np.array(stats, np.int64)


def digest(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def sppm_golden(name):
    over, film, splat, r2, n, stats = sppm_run(name)
    if name.endswith("q"):
        _, _, _, r2a, _, stats_a = sppm_run(name, all_within=True)
        return dict(overrides=over, film_sha256=digest(film), splat_sha256=digest(splat), r2=r2, n=n, stats=stats,
                    pairs_all_within=stats_a[:, 3], r2_all_within=r2a)
    return dict(overrides=over, film=film, splat=splat, r2=r2, n=n, stats=stats)


def main():
    only = set(sys.argv[1:])          # e.g. `make_golden.py X1`: regenerate only these cases
    for name in TRACE_CASES:
        if not only or name in only:
            np.savez_compressed(os.path.join(HERE, f"trace_{name}.npz"), **trace_golden(name))
    if not only or "C1" in only:
        np.savez_compressed(os.path.join(HERE, "sample_li_C1.npz"), **sample_golden())
        np.savez_compressed(os.path.join(HERE, "film_C1_48.npz"), **film_golden())
    for name in ("X1", "X2", "X3", "X4", "X7", "X8", "X9", "X10", "X11", "X12", "X13", "X14", "X15", "X16"):
        if not only or name in only:
            np.savez_compressed(os.path.join(HERE, f"sample_li_{name}.npz"), **sample_golden(name, ""))
    for name in SPPM_CASES:
        if not only or name in only:
            np.savez_compressed(os.path.join(HERE, f"sppm_{name}.npz"), **sppm_golden(name))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
