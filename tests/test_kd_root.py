"""The reference tests every query against the kd-tree's bounds first (kdTreePrimitive's
`intersectAABB b r >>= trav`, KdTree.hs:236-244; AABB.hs:79-94), and the device mirrors that test
(dev_trace.h kd_root) ahead of its padded BVH.

Found by tools/film_divergence.py on MI355X after the round-6 sampler change (gpurun_out/r06c,
profiles/r06_c2_film_divergence.json): C2 sample (1, 1026, 13) fires a camera ray that meets the floor
exactly on its front edge, y = z = 0, which is also an edge of the scene's bounds.  Moller-Trumbore
reports the hit (t = 887.6492), but intersectAABB's entry t (887.6492, the z slab) exceeds its exit t
(887.6491, the y slab) by one ulp, so the reference never reaches the floor: the camera ray misses and
the path ends.  Before kd_root the device's padded BVH found the floor and traced five more rays.

CPU: the ray's binary32 bits, the oracle's miss, the floor hit of a numpy binary32 Moller-Trumbore
(tests/test_kat_hotpath.py tri_intersect), and the numpy restatement of intersectAABB.
GPU: bling_trace misses the same ray, and a ray one ulp inside still hits the floor."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bling_amd.scene import load_config  # noqa: E402
from scene_desc import desc  # noqa: E402
from test_kat_hotpath import tri_intersect  # noqa: E402

f32 = np.float32
# origin (278, 273, -800), direction of C2 sample (1, 1026, 13), pass 0, seed 0x0B11A6 (sampler v2)
DIR_BITS = [0xbe9c430a, 0xbe9d77b6, 0x3f66b8c7]


def _ray():
    ro = np.array([278, 273, -800], f32)
    rd = np.array(DIR_BITS, np.uint32).view(f32)
    return ro, rd


def _soa(ro, rd):
    return np.array([[ro[0]], [ro[1]], [ro[2]], [rd[0]], [rd[1]], [rd[2]], [0], [np.inf]], f32)


def _hmax(a, b):
    return b if a <= b else a


def _hmin(a, b):
    return a if a <= b else b


def intersect_aabb(mn, mx, ro, rd, tmin=f32(0), tmax=f32(np.inf)):
    """AABB.hs:79-94 in binary32, Haskell max / min."""
    near, far = f32(tmin), f32(tmax)
    for a in range(3):
        if near > far:
            return None
        dinv = f32(1) / rd[a]
        tn, tf = f32((mn[a] - ro[a]) * dinv), f32((mx[a] - ro[a]) * dinv)
        n2, f2 = (tf, tn) if tn > tf else (tn, tf)
        near, far = _hmax(near, n2), _hmin(far, f2)
    return None if near > far else (near, far)


def _mesh(job):
    d = desc(job)
    nv, nt = d.num_vertices, d.num_triangles
    verts = np.ctypeslib.as_array(d.vertices, shape=(3 * nv,)).reshape(nv, 3).astype(f32)
    idx = np.ctypeslib.as_array(d.tri_indices, shape=(3 * nt,)).reshape(nt, 3)
    return verts, idx


def test_the_reference_misses_a_ray_through_the_bounds_edge():
    from oracle_py import Oracle
    job = load_config("C2")
    orc = Oracle(job)
    ro, rd = _ray()
    cam = orc.camera_ray(1, 1026, 13, seed=0x0B11A6, pass_index=0)
    assert np.array_equal(cam[5:8].astype(f32).view(np.uint32), np.array(DIR_BITS, np.uint32))
    t, prim, _, _ = orc.trace(_soa(ro, rd))
    assert not np.isfinite(t[0]) and prim[0] == 0xFFFFFFFF          # the oracle's kd-tree: a miss
    verts, idx = _mesh(job)
    hits = [(k, tri_intersect(verts[idx[k, 0]], verts[idx[k, 1]], verts[idx[k, 2]], ro, rd, f32(0), f32(np.inf)))
            for k in range(len(idx))]
    hits = [(k, h) for k, h in hits if h is not None]
    assert len(hits) == 1 and abs(float(hits[0][1][0]) - 887.6492) < 1e-3   # the floor, on its front edge
    # the scene bounds (the triangles' and the light quad's; the quad lies inside) reject the ray by one ulp
    mn, mx = verts.min(0), verts.max(0)
    assert mn[1] == 0 and mn[2] == 0
    assert intersect_aabb(mn, mx, ro, rd) is None
    tz = f32((mn[2] - ro[2]) * (f32(1) / rd[2]))
    ty = f32((mn[1] - ro[1]) * (f32(1) / rd[1]))
    assert tz == np.nextafter(ty, f32(np.inf))                     # entry one ulp past the exit


@pytest.mark.gpu
def test_device_misses_it_too():
    from bling_amd.render import Context
    job = load_config("C2")
    ctx = Context(0)
    ctx.upload(job)
    ro, rd = _ray()
    t, prim, _ = ctx.trace(_soa(ro, rd))
    assert not np.isfinite(t[0]) and prim[0] == 0xFFFFFFFF, (t, prim)
    # aimed a little further into the room (one ulp up in z), the ray enters the bounds and hits the floor
    rd2 = rd.copy()
    rd2[2] = np.nextafter(rd[2], f32(1))
    t2, prim2, _ = ctx.trace(_soa(ro, rd2))
    from oracle_py import Oracle
    to, po, _, _ = Oracle(job).trace(_soa(ro, rd2))
    assert t2[0] == to[0] and prim2[0] == po[0], (t2, prim2, to, po)
    ctx.close()
