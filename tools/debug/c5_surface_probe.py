"""Debug probe: secondary rays leaving the Mandelbulb surface, GPU bling_trace vs oracle_trace."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
from bling_amd.scene import load_config
from oracle_py import Oracle
SEED = 0x0B11A6
job = load_config("C5", "image=64,64")
orc = Oracle(job)
gpu = len(sys.argv) < 2 or sys.argv[1] != "cpu"
if gpu:
    from bling_amd.render import Context
    ctx = Context(0); ctx.upload(job)
rng = np.random.default_rng(5)
rays = []
for y in range(0, 64, 2):
    for x in range(0, 64, 2):
        r = orc.camera_ray(x, y, int(rng.integers(0, 1024)), seed=SEED)
        rays.append([r[2], r[3], r[4], r[5], r[6], r[7], 0.0, np.inf])
cam = np.array(rays, np.float32).T.copy()
t, prim, _, _ = orc.trace(cam)
fr = (prim == 0) & np.isfinite(t)     # prim 0 = the fractal in mandelbulb.bling
print("camera rays", cam.shape[1], "prims", np.unique(prim, return_counts=True))
eps = np.float32(1e-4 * 2)
o = cam[0:3, fr] + cam[3:6, fr] * t[fr]
n = o.shape[1]
d = rng.normal(size=(3, n)).astype(np.float32); d /= np.linalg.norm(d, axis=0)
sec = np.concatenate([o, d, np.full((1, n), eps, np.float32), np.full((1, n), np.inf, np.float32)], 0).astype(np.float32)
t_o, p_o, _, _ = orc.trace(sec)
print("secondary", n, "oracle prims", np.unique(p_o, return_counts=True))
if gpu:
    t_g, p_g, _ = ctx.trace(sec)
    print("gpu prims", np.unique(p_g, return_counts=True))
    same = p_g == p_o
    print("prim agree", same.mean())
    fin = same & np.isfinite(t_o) & np.isfinite(t_g)
    rel = np.abs(t_g[fin] - t_o[fin]) / np.maximum(np.abs(t_o[fin]), 1e-6)
    print("t rel: median", np.median(rel), "p99", np.quantile(rel, 0.99), "frac<=1e-3", (rel <= 1e-3).mean())
    print("nan t gpu", np.isnan(t_g).sum(), "oracle", np.isnan(t_o).sum())
    bad = np.where(~same)[0][:10]
    for i in bad: print(i, p_o[i], t_o[i], p_g[i], t_g[i])
