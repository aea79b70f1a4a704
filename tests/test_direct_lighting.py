"""DirectLighting surface integrator (Integrator/DirectLighting.hs:14-57), SURVEY.md 8(f) row f4:
loader fields and the oracle's restatement of the recursion, on the X4 feature scene
(fixtures/scenes/direct-lighting.bling).  The HIP side (k_shade_dl) is checked against the same
oracle in test_gpu_parity.py (sample_li golden X4, film parity X4).

Parity anchor: the reference's test suite holds no DirectLighting vectors, so these are
properties read off the reference source -- parity unpinned beyond them.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from bling_amd.scene import load_config  # noqa: E402
from oracle_py import Oracle  # noqa: E402

SEED = 0x0B11A6


def test_loader_reads_direct_lighting_block():
    job = load_config("X4")
    assert job.config.integrator == 1          # BLING_INTEGRATOR_DIRECT
    assert job.config.max_depth == 5           # integrator { directLighting maxDepth 5 }
    assert job.config.renderer == 0            # the sampler renderer
    assert "direct md=5" in job.summary()


def test_overrides_switch_integrator():
    p = load_config("X4", "path=4,2").config
    assert (p.integrator, p.max_depth, p.sample_depth) == (0, 4, 2)
    d = load_config("C1", "direct=3;image=16,16").config
    assert (d.integrator, d.max_depth) == (1, 3)


def test_max_depth_one_has_no_continuations():
    """cont at d + 1 == maxDepth returns black without sampling: no specular rays are traced."""
    job = load_config("X4", "direct=1;image=24,18")
    _, st = Oracle(job).render(seed=SEED, threads=4)
    assert st.rays_continuation == 0
    assert st.rays_camera == st.samples > 0
    job5 = load_config("X4", "image=24,18")
    _, st5 = Oracle(job5).render(seed=SEED, threads=4)
    assert st5.rays_continuation > 0            # glass / mirror / shinyMetal spawn specular children


def _escaping_samples(orc, job, want=8):
    """(x, y, n) samples whose camera ray hits nothing."""
    out = []
    for y in range(0, job.height, 2):
        for x in range(0, job.width, 2):
            r = orc.camera_ray(x, y, 0, seed=SEED)
            rays = np.array([[r[2]], [r[3]], [r[4]], [r[5]], [r[6]], [r[7]], [0.0], [np.inf]], np.float32)
            _, prim, _, _ = orc.trace(rays)
            if prim[0] == 0xFFFFFFFF:
                out.append((x, y))
                if len(out) == want:
                    return out
    return out


def test_escaped_camera_rays_add_black():
    """`maybe (return black) ls (scIntersect s r)` (DirectLighting.hs:23): a camera ray that escapes
    adds nothing even under an infinite light, where Path adds that light's Le (Path.hs:44)."""
    job = load_config("X4", "image=32,24")
    orc = Oracle(job)
    esc = _escaping_samples(orc, job)
    assert esc, "the X4 view has sky pixels"
    path = Oracle(load_config("X4", "image=32,24;path=5,3"))
    for x, y in esc:
        L, _, st = orc.sample_li(x, y, 0, seed=SEED)
        assert np.all(L == 0.0) and st.rays_camera == 1 and st.rays_shadow == 0
        Lp, _, _ = path.sample_li(x, y, 0, seed=SEED)
        assert np.all(Lp > 0.0)


def test_direct_lighting_differs_from_path_but_agrees_on_first_vertex_light():
    """Same scene, same seed: DirectLighting and Path both sample one light at the first vertex, but
    draw it from different sampler dimensions (2d vs 1 + 4d) -- the films differ, the mean
    brightness is of the same order (no indirect diffuse in DirectLighting)."""
    fd, _ = Oracle(load_config("X4", "image=32,24")).render(seed=SEED, threads=4)
    fp, _ = Oracle(load_config("X4", "image=32,24;path=5,3")).render(seed=SEED, threads=4)
    yd = fd.reshape(-1, 4)[:, 2].sum() / fd.reshape(-1, 4)[:, 0].sum()
    yp = fp.reshape(-1, 4)[:, 2].sum() / fp.reshape(-1, 4)[:, 0].sum()
    assert not np.array_equal(fd, fp)
    assert 0.3 < yd / yp < 1.05, (yd, yp)
