#!/usr/bin/env python3
"""Find the camera sample(s) behind a film test's ray-count difference and name their first
diverging operation.

test_film_parity_config_tiles renders every stride-th tile of a full-size pass on the device and on
the oracle; a continuation or BSDF-MIS ray count that differs means some path went another way, which
summation order cannot cause.  This tool
  1. renders each kept tile alone on both sides (shard = (m, tiles)) and compares the ray counts;
  2. for each tile that differs, runs all of its camera samples through bling_sample_li_vertices
     (the BLING_DEBUG_VERTEX build) and oracle_sample_li_vertices, and reports every sample whose
     per-vertex records differ: the first differing field in the order a vertex computes them
     (tools/vertex_divergence.py GROUPS), both values and their ulp distance.

  BLING_HIP_VARIANT=dbg python tools/film_divergence.py --config C2 --stride 16 --out gpurun_out/x.json

Test infrastructure (loads the oracle); needs a GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from vertex_divergence import GROUPS, first_divergence, ulps  # noqa: E402

SEED = 0x0B11A6


def kept_tiles(extent, stride):
    """The tiles a pass with tile_stride keeps, in splitWindow order (core.hip pass_tiles)."""
    x0, x1, y0, y1 = extent
    out, k = [], 0
    for y in range(y0, y1 + 1, 16):
        for x in range(x0, x1 + 1, 16):
            if k % stride == 0:
                out.append((x, min(x + 15, x1), y, min(y + 15, y1)))
            k += 1
    return out


def counts(st):
    return {"camera": int(st.rays_camera), "continuation": int(st.rays_continuation), "mis": int(st.rays_mis),
            "shadow": int(st.rays_shadow)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--stride", type=int, default=16)
    ap.add_argument("--pass-index", type=int, default=0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from bling_amd.render import Context
    from bling_amd.scene import load_config
    from oracle_py import Oracle
    job = load_config(args.config)
    orc = Oracle(job)
    ctx = Context(0)
    ctx.upload(job)
    ext, _ = orc.extent()
    tiles = kept_tiles(ext, args.stride)
    T = len(tiles)
    _, sg = ctx.render_pass(seed=SEED, pass_index=args.pass_index, tile_stride=args.stride)
    _, so = orc.render(seed=SEED, pass_index=args.pass_index, tile_stride=args.stride)
    whole = {"device": counts(sg), "oracle": counts(so)}
    bad_tiles = []
    for m in range(T):
        _, a = ctx.render_pass(seed=SEED, pass_index=args.pass_index, tile_stride=args.stride, shard=(m, T))
        _, b = orc.render(seed=SEED, pass_index=args.pass_index, tile_stride=args.stride, shard=(m, T))
        ca, cb = counts(a), counts(b)
        if ca != cb:
            bad_tiles.append({"tile": m, "window": tiles[m], "device": ca, "oracle": cb})
    samples = []
    for bt in bad_tiles:
        tx0, tx1, ty0, ty1 = bt["window"]
        xs, ys, ns = np.meshgrid(np.arange(tx0, tx1 + 1), np.arange(ty0, ty1 + 1), np.arange(job.spp), indexing="ij")
        smp = np.stack([xs.ravel(), ys.ravel(), ns.ravel()], 1).astype(np.int32)
        Lg, vg = ctx.sample_li_vertices(smp, seed=SEED, pass_index=args.pass_index)
        Lo, vo = orc.sample_li_vertices(smp, seed=SEED, pass_index=args.pass_index)
        for k in range(len(smp)):
            fd = first_divergence(vg[k], vo[k])
            if fd is None:
                continue
            d, name, f, a, b = fd
            samples.append({"tile": bt["tile"], "sample": smp[k].tolist(), "depth": d, "field": name, "index": f,
                            "device": a, "oracle": b, "ulps": ulps(a, b),
                            "L_device": float(np.sum(Lg[k])), "L_oracle": float(np.sum(Lo[k])),
                            "records_device": vg[k, :d + 2].tolist(), "records_oracle": vo[k, :d + 2].tolist()})
    out = {"config": args.config, "stride": args.stride, "pass_index": args.pass_index, "tiles": T,
           "whole_pass": whole, "tiles_with_ray_delta": bad_tiles, "diverging_samples": samples,
           "fields": [g for g, _ in GROUPS]}
    s = json.dumps(out, indent=1)
    print(json.dumps({k: out[k] for k in ("config", "tiles", "whole_pass", "tiles_with_ray_delta")}, indent=1))
    for smp in samples:
        print({k: smp[k] for k in ("tile", "sample", "depth", "field", "device", "oracle", "ulps")})
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        open(args.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
