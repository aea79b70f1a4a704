#!/usr/bin/env python3
"""First-divergence analysis of per-sample parity.

Runs the same camera samples through the device (the BLING_DEBUG_VERTEX build,
BLING_HIP_VARIANT=dbg) and the oracle, both recording one BLING_DV_FIELDS record per path vertex
(include/bling.h), and names, for every sample, the first vertex and the first field (in the order
the vertex computes them) where the two disagree bit for bit.  The tally over the samples whose
spectra mismatch is the cause table DESIGN.md section 2 cites.

  BLING_HIP_VARIANT=dbg python tools/vertex_divergence.py --config C5 [--n 8192] [--out file.json]

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

SEED = 0x0B11A6
# field groups in the order a vertex computes them (include/bling.h BLING_DV_*)
GROUPS = [("ray_o", [0, 1, 2]), ("ray_d", [3, 4, 5]), ("hit_t", [6]), ("p", [7, 8, 9]), ("n", [10, 11, 12]),
          ("eps", [13]), ("light_wi", [14, 15, 16]), ("light_pdf", [17]), ("mis_wi", [18, 19, 20]),
          ("mis_pdf", [21]), ("rr_pc", [26]), ("rr_u", [27]), ("cont_wi", [22, 23, 24]), ("cont_pdf", [25]),
          ("occluded", [28]), ("mis_t", [29]), ("lhere", [30]), ("L", [31])]


def same_bits(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Elementwise: equal bit patterns, or both NaN (not reached on either side)."""
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def ulps(a: float, b: float) -> int | None:
    if not (np.isfinite(a) and np.isfinite(b)):
        return None
    ia = int(np.float32(a).view(np.int32))
    ib = int(np.float32(b).view(np.int32))
    ia = ia if ia >= 0 else -(ia & 0x7FFFFFFF)
    ib = ib if ib >= 0 else -(ib & 0x7FFFFFFF)
    return abs(ia - ib)


def first_divergence(vg: np.ndarray, vo: np.ndarray):
    """(depth, group, field, device value, oracle value) of the first differing field, or None."""
    for d in range(vg.shape[0]):
        eq = same_bits(vg[d], vo[d])
        if eq.all():
            continue
        for name, fields in GROUPS:
            for f in fields:
                if not eq[f]:
                    return d, name, f, float(vg[d, f]), float(vo[d, f])
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--sample-seed", type=int, default=11)   # test_sample_li_full_config's samples
    ap.add_argument("--pass-index", type=int, default=1)
    ap.add_argument("--out", default="")
    ap.add_argument("--examples", type=int, default=12)
    args = ap.parse_args()

    from bling_amd.render import Context
    from bling_amd.scene import load_config
    from oracle_py import Oracle
    from parity_util import random_samples, spectra_mismatch

    job = load_config(args.config)
    orc = Oracle(job)
    ctx = Context(0)
    ctx.upload(job)
    smp = random_samples(orc, job, args.n, seed=args.sample_seed)
    Lg, vg = ctx.sample_li_vertices(smp, seed=SEED, pass_index=args.pass_index)
    Lo, vo = orc.sample_li_vertices(smp, seed=SEED, pass_index=args.pass_index)
    bad, exact, worst, rel = spectra_mismatch(Lg, Lo)
    mism = ~(rel <= 1e-4)

    tally_bad: dict[str, int] = {}
    tally_all: dict[str, int] = {}
    depth_bad: dict[int, int] = {}
    examples = []
    diverged = 0
    for k in range(len(smp)):
        fd = first_divergence(vg[k], vo[k])
        if fd is None:
            continue
        diverged += 1
        d, name, f, a, b = fd
        tally_all[name] = tally_all.get(name, 0) + 1
        if mism[k]:
            tally_bad[name] = tally_bad.get(name, 0) + 1
            depth_bad[d] = depth_bad.get(d, 0) + 1
            if len(examples) < args.examples:
                examples.append({"sample": smp[k].tolist(), "depth": d, "field": name, "index": f, "device": a,
                                 "oracle": b, "ulps": ulps(a, b), "rel_L1": float(rel[k])})
    no_div_but_bad = int(sum(1 for k in range(len(smp)) if mism[k] and first_divergence(vg[k], vo[k]) is None))
    out = {"config": args.config, "samples": len(smp), "spectra_mismatch": bad, "spectra_exact": exact,
           "records_diverged": diverged, "mismatch_without_record_divergence": no_div_but_bad,
           "first_divergence_of_mismatching": dict(sorted(tally_bad.items(), key=lambda x: -x[1])),
           "first_divergence_all": dict(sorted(tally_all.items(), key=lambda x: -x[1])),
           "depth_of_first_divergence_mismatching": {str(k): v for k, v in sorted(depth_bad.items())},
           "examples": examples}
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
