#!/usr/bin/env python3
"""SPPM probe (GPU box): device pass vs the CPU oracle on the same scene, per-pass timing, and a PNG.

  python tools/sppm_probe.py --config X5 --over "image=128,128" --passes 3 --png gpurun_out/x5.png
  python tools/sppm_probe.py --config X5 --passes 8 --oracle-passes 1 --photons 2000000

Prints one JSON line per pass (device stats + rays/s) and, for the passes the oracle also runs, the
parity figures (hit-point count, eye film relative L2 of XYZ/W, splat relative L2, radius agreement).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from bling_amd import _ffi  # noqa: E402
from bling_amd.render import Context  # noqa: E402
from bling_amd.scene import load_config  # noqa: E402

SEED = 0x0B11A6


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="X5")
    ap.add_argument("--over", default="")
    ap.add_argument("--photons", type=int, default=0, help="override photonCount (keeps the file's depth/radius)")
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--oracle-passes", type=int, default=0)
    ap.add_argument("--oracle-threads", type=int, default=16)
    ap.add_argument("--png", default="")
    a = ap.parse_args()
    over = a.over
    if a.photons:
        c = load_config(a.config, over or None).config
        over = ";".join(x for x in (over, f"sppm={a.photons},{c.max_depth},{c.sppm_radius},{c.sppm_alpha}") if x)
    job = load_config(a.config, over or None)
    w, h = job.width, job.height
    ctx = Context(0)
    ctx.upload(job)
    orc = None
    if a.oracle_passes:
        from oracle_py import OracleSppm
        orc = OracleSppm(job)
    film = np.zeros(w * h * 4, np.float32)
    splat = np.zeros(w * h * 3, np.float32)
    ofilm = np.zeros_like(film)
    osplat = np.zeros_like(splat)
    cfg = job.config
    sn = max(1, int(np.ceil(np.sqrt(np.float32(cfg.sppm_photons) / np.float32(max(1, cfg.sppm_threads))))))
    for p in range(1, a.passes + 1):
        t0 = time.perf_counter()
        film, splat, st = ctx.sppm_pass(seed=SEED, pass_index=p, film=film, splat=splat)
        wall = (time.perf_counter() - t0) * 1e3
        rays = st.cam_rays + st.photon_rays
        line = {"pass": p, "config": a.config, "over": over, "image": [w, h], **st.as_dict(), "wall_ms": round(wall, 3),
                "Mrays_per_s": round(rays / (st.ms_total * 1e-3) / 1e6, 2)}
        if orc is not None and p <= a.oracle_passes:
            ofilm, osplat, ost = orc.render_pass(seed=SEED, pass_index=p, threads=a.oracle_threads, film=ofilm,
                                                  splat=osplat)
            f, of = film.reshape(-1, 4), ofilm.reshape(-1, 4)
            m = (f[:, 0] > 0) & (of[:, 0] > 0)
            r2, _ = ctx.sppm_pixel_stats()
            or2, _ = orc.pixel_stats()
            line["oracle"] = {"hitpoints": ost.hitpoints, "cam_rays": ost.cam_rays, "photon_rays": ost.photon_rays,
                              "photon_hits": ost.photon_hits, "seconds": round(ost.seconds, 4),
                              "cpu_Mrays_per_s": round((ost.cam_rays + ost.photon_rays) / ost.seconds / 1e6, 3),
                              "film_rel_l2": rel_l2(f[m, 1:] / f[m, :1], of[m, 1:] / of[m, :1]),
                              "splat_rel_l2": rel_l2(splat, osplat),
                              "r2_agree": float((np.abs(r2 - or2) <= 1e-5 * or2).mean()),
                              "r2_exact_px": int((r2 == or2).sum()), "r2_px": int(r2.size),
                              "r2_below_1": float((or2 < 1).mean()), "r2_distinct": int(len(np.unique(or2)))}
        print(json.dumps(line), flush=True)
    if a.png:
        sw = 1.0 / (max(1, cfg.sppm_threads) * a.passes * sn * sn)
        _ffi.host().bling_host_write_png_splat.argtypes = [_ffi.C.c_char_p, _ffi.c_f32p, _ffi.c_f32p, _ffi.C.c_float,
                                                           _ffi.C.c_int, _ffi.C.c_int]
        _ffi.host().bling_host_write_png_splat(a.png.encode(), _ffi.f32ptr(film), _ffi.f32ptr(splat), sw, w, h)
    ctx.close()


if __name__ == "__main__":
    main()
