#!/usr/bin/env python3
"""SPPM device vs oracle, per pass: the hit-point sets (by key pixel << 24 | eye-tree node: keys on
one side only, position / radius^2 bit mismatches), photon rays and photon / hit-point pairs.

  python tools/sppm_hp_compare.py --config X13 --over "image=128,96;sppm=200000,6,0.5,0.1;sppm_threads=4" --passes 3
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from bling_amd.render import Context  # noqa: E402
from bling_amd.scene import load_config  # noqa: E402
from oracle_py import OracleSppm  # noqa: E402

SEED = 0x0B11A6


def pivots(n):
    """positions of the kd-tree's pivots in a bucket of n entries (mkKdTree's median split)"""
    out, st = [], [(0, n)]
    while st:
        l, u = st.pop()
        if u - l <= 5:
            continue
        m = l + (u - l) // 2
        out.append(m)
        st += [(l, m), (m + 1, u)]
    return np.array(sorted(out), np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="X13")
    ap.add_argument("--over", default="image=128,96;sppm=200000,6,0.5,0.1;sppm_threads=4")
    ap.add_argument("--passes", type=int, default=3)
    a = ap.parse_args()
    job = load_config(a.config, a.over)
    w, h = job.width, job.height
    ctx = Context(0)
    ctx.upload(job)
    orc = OracleSppm(job)
    film = np.zeros(w * h * 4, np.float32); splat = np.zeros(w * h * 3, np.float32)
    ofilm = np.zeros_like(film); osplat = np.zeros_like(splat)
    for p in range(1, a.passes + 1):
        film, splat, st = ctx.sppm_pass(seed=SEED, pass_index=p, film=film, splat=splat)
        ofilm, osplat, ost = orc.render_pass(seed=SEED, pass_index=p, film=ofilm, splat=osplat)
        dp, dk = ctx.sppm_hitpoints()
        op, ok = orc.hitpoints()
        di, oi = np.argsort(dk, kind="stable"), np.argsort(ok, kind="stable")
        dk, dp, ok, op = dk[di], dp[di], ok[oi], op[oi]
        only_d = np.setdiff1d(dk, ok).size
        only_o = np.setdiff1d(ok, dk).size
        common, ia, ib = np.intersect1d(dk, ok, return_indices=True)
        bad = ~np.all(dp[ia].view(np.uint32) == op[ib].view(np.uint32), axis=1)
        r2, _ = ctx.sppm_pixel_stats()
        or2, _ = orc.pixel_stats()
        rec = {"pass": p, "hitpoints": [int(st.hitpoints), int(ost.hitpoints)], "keys_only_device": int(only_d),
               "keys_only_oracle": int(only_o), "pos_r2_mismatch": int(bad.sum()),
               "photon_rays": [int(st.photon_rays), int(ost.photon_rays)], "pairs": [int(st.photon_hits), int(ost.photon_hits)],
               "r2_pixels_differ": int((r2 != or2).sum())}
        # the kd-tree buckets: device and oracle hit point indices differ (append order), so compare
        # by key; entries per bucket in kd order and the mr at each position
        dbs, dit, dmr = ctx.sppm_buckets()
        obs, oit, omr = orc.buckets()
        dkey_of = ctx.sppm_hitpoints()[1]
        okey_of = orc.hitpoints()[1]
        nbd = nbm = 0
        first_b = None
        for b in range(min(len(dbs), len(obs)) - 1):
            dk_b = dkey_of[dit[dbs[b]:dbs[b + 1]]]
            ok_b = okey_of[oit[obs[b]:obs[b + 1]]]
            if len(dk_b) != len(ok_b) or not np.array_equal(dk_b, ok_b):
                nbd += 1
                if first_b is None:
                    first_b = {"bucket": b, "n": [int(len(dk_b)), int(len(ok_b))], "device": dk_b[:12].tolist(), "oracle": ok_b[:12].tolist()}
            else:
                pv = pivots(len(dk_b))
                if pv.size and not np.array_equal(dmr[dbs[b] + pv].view(np.uint32), omr[obs[b] + pv].view(np.uint32)):
                    nbm += 1
        rec["buckets"] = [int(len(dbs) - 1), int(len(obs) - 1)]
        rec["bucket_order_differs"] = nbd
        rec["bucket_mr_differs"] = nbm
        if first_b is not None:
            rec["first_bucket"] = first_b
        if bad.any():
            k = int(common[np.argmax(bad)])
            rec["first_mismatch"] = {"key": k, "pixel": k >> 24, "node": k & 0xFFFFFF,
                                     "device": dp[ia][bad][0].tolist(), "oracle": op[ib][bad][0].tolist()}
        print(json.dumps(rec), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
