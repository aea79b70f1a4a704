"""Shared measurement helpers of the GPU parity tests: every comparison reports what it measured
(mismatch counts, worst errors) on stdout and in gpurun_out/parity_metrics.jsonl, so the bars in
the tests can be set from observed values ("Tolerances")."""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def report(test: str, **metrics):
    rec = {"test": test}
    for k, v in metrics.items():
        rec[k] = v.item() if isinstance(v, np.generic) else v
    line = json.dumps(rec)
    print("PARITY " + line)
    out = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_metrics.jsonl"), "a") as f:
            f.write(line + "\n")
    except OSError:
        pass
    return rec


def spectra_mismatch(Lg: np.ndarray, Lo: np.ndarray, tol: float = 1e-4):
    """Per-sample relative L1 over the 16 bands.  A sample mismatches when rel > tol (two black
    spectra match).  Returns (n_mismatch, n_exact, worst rel among matches, rel array)."""
    den = np.abs(Lo).astype(np.float64).sum(1)
    num = np.abs(Lg.astype(np.float64) - Lo.astype(np.float64)).sum(1)
    both_black = (den == 0) & (np.abs(Lg).sum(1) == 0)
    rel = np.where(both_black, 0.0, num / np.maximum(den, 1e-30))
    rel = np.where(np.isnan(Lg).any(1) & np.isnan(Lo).any(1), 0.0, rel)   # NaN samples on both sides
    bad = ~(rel <= tol)
    exact = (Lg == Lo).all(1) | both_black
    worst_ok = float(rel[~bad].max()) if (~bad).any() else 0.0
    return int(bad.sum()), int(exact.sum()), worst_ok, rel


def film_errors(fg: np.ndarray, fo: np.ndarray):
    """Film comparison: filter-weight error, per-pixel XYZ/W relative errors, image relative L2."""
    fg, fo = fg.reshape(-1, 4).astype(np.float64), fo.reshape(-1, 4).astype(np.float64)
    w_abs = float(np.abs(fg[:, 0] - fo[:, 0]).max())
    w_rel = float((np.abs(fg[:, 0] - fo[:, 0]) / np.maximum(np.abs(fo[:, 0]), 1e-12)).max())
    m = fo[:, 0] != 0
    xo = fo[m, 1:] / fo[m, :1]
    xg = fg[m, 1:] / np.where(fg[m, :1] == 0, 1.0, fg[m, :1])
    pix = np.linalg.norm(xg - xo, axis=1) / (np.linalg.norm(xo, axis=1) + 1e-6)
    l2 = float(np.linalg.norm(xg - xo) / max(np.linalg.norm(xo), 1e-30))
    return {"w_abs": w_abs, "w_rel": w_rel, "rel_l2": l2, "pix_over_1e-3": int((pix > 1e-3).sum()),
            "pix_over_1e-5": int((pix > 1e-5).sum()), "pixels": int(m.sum()), "pix_max": float(pix.max(initial=0.0))}


def random_samples(orc, job, k: int, seed: int):
    """k random (x, y, n) camera samples over the whole sample extent and sample range."""
    rng = np.random.default_rng(seed)
    (x0, x1, y0, y1), _ = orc.extent()
    return np.stack([rng.integers(x0, x1 + 1, k), rng.integers(y0, y1 + 1, k),
                     rng.integers(0, job.spp, k)], 1).astype(np.int32)
