"""Debug probe: C5 (mandelbulb) per-sample parity, GPU vs oracle (run on the GPU box)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
from bling_amd.scene import load_config
from bling_amd.render import Context
from oracle_py import Oracle
SEED = 0x0B11A6
job = load_config("C5", "image=4,4")
orc = Oracle(job)
ctx = Context(0); ctx.upload(job)
f_o, st_o = orc.render(seed=SEED)
f_g, st_g = ctx.render_pass(seed=SEED, pass_index=0)
for nm in ("rays_camera", "rays_continuation", "rays_mis", "rays_shadow", "dropped_samples"):
    print(nm, getattr(st_g, nm), getattr(st_o, nm if nm != "dropped_samples" else "dropped"))
rng = np.random.default_rng(3)
(x0, x1, y0, y1), _ = orc.extent()
k = 400
smp = np.stack([rng.integers(x0, x1 + 1, k), rng.integers(y0, y1 + 1, k), rng.integers(0, job.spp, k)], 1).astype(np.int32)
Lg, img_g, stg = ctx.sample_li(smp, seed=SEED)
Lo = np.zeros_like(Lg); rays_o = np.zeros(4, np.int64)
for i, (x, y, n) in enumerate(smp):
    L, xy, st = orc.sample_li(int(x), int(y), int(n), seed=SEED)
    Lo[i] = L
    rays_o += [st.rays_camera, st.rays_continuation, st.rays_mis, st.rays_shadow]
print("sample rays gpu", stg.rays_camera, stg.rays_continuation, stg.rays_mis, stg.rays_shadow, "oracle", rays_o)
rel = np.abs(Lg - Lo).sum(1) / (np.abs(Lo).sum(1) + 1e-12)
zero = (np.abs(Lo).sum(1) == 0) & (np.abs(Lg).sum(1) == 0)
print("close 1e-4:", ((rel <= 1e-4) | zero).mean(), "close 1e-2:", ((rel <= 1e-2) | zero).mean())
print("mean Y gpu/oracle", Lg.sum(), Lo.sum())
bad = np.where(~((rel <= 1e-2) | zero))[0][:15]
for i in bad:
    print(smp[i], Lg[i].sum(), Lo[i].sum())
