"""Bezier patch primitives (`prim { bezier subdivs n p { 48 floats } ... }`, PrimitiveParser.hs:32-37,
121-128): the loader tessellates each bicubic patch into (n + 1)^2 vertices and 2 n^2 triangles with
shading normals dpdu x dpdv and (u, v) = (i / n, j / n) (tesselateBezier / onePatch / evalPatch,
Primitive/Bezier.hs:50-105).  The device and the oracle then see an ordinary shading-normal mesh,
so GPU parity is the mesh path's (feature scene X16, test_gpu_parity.py).

Here: a numpy binary32 restatement of onePatch, in GHC's operation order, against the loader's
triangles for the fixture's first patch; the reference's own gumbo.bling (51 patches, subdivs 16)
and the other scenes whose environment map the reference does not ship, with this repo's synthetic
.hdr substituted.  Parity unpinned beyond these: the reference ships
no tessellated output.
"""
import ctypes as C
import os
import re
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bling_amd.scene import ParseError, load_config, parse_job  # noqa: E402

f32 = np.float32
REF_EXAMPLES = "/root/reference/examples"
HDR = os.path.join(ROOT, "fixtures", "scenes", "envmaps", "sky-synth.hdr")


class DescHead(C.Structure):     # leading fields of bling_scene_desc (include/bling_scene.h)
    _fields_ = [("num_vertices", C.c_uint32), ("vertices", C.POINTER(C.c_float)),
                ("num_triangles", C.c_uint32), ("tri_indices", C.POINTER(C.c_uint32)),
                ("tri_material", C.POINTER(C.c_int32)), ("tri_uvs", C.POINTER(C.c_float)),
                ("tri_normals", C.POINTER(C.c_float))]


def bern(u, x):                  # bernstein (Bezier.hs:27-35), left to right
    i = f32(1) - u
    return [lambda: f32(f32(f32(1) * i) * i) * i, lambda: f32(f32(f32(3) * u) * i) * i,
            lambda: f32(f32(f32(3) * u) * u) * i, lambda: f32(f32(f32(1) * u) * u) * u][x]()


def bern_d(u, x):                # bernsteinDeriv (Bezier.hs:39-47)
    i = f32(1) - u
    return [lambda: f32(3) * -(i * i),
            lambda: f32(3) * f32(i * i - f32(f32(2) * u) * i),
            lambda: f32(3) * f32(f32(f32(2) * u) * i - u * u),
            lambda: f32(3) * (u * u)][x]()


def ev(c, bj, bi):               # evalPatch's ev: sum = foldl (+) 0 over i then j
    out = []
    for o in range(3):
        acc = f32(0)
        for i in range(4):
            for j in range(4):
                acc = f32(acc + f32(f32(c[i * 12 + j * 3 + o] * bj[j]) * bi[i]))
        out.append(acc)
    return np.array(out, np.float32)


def cross(u, v):                 # Math.hs:336-339
    return np.array([u[1] * v[2] - u[2] * v[1], -(u[0] * v[2] - u[2] * v[0]), u[0] * v[1] - u[1] * v[0]], np.float32)


def one_patch(c, n):
    step = f32(1) / f32(n)
    ps, ns, uvs = [], [], []
    for i in range(n + 1):
        for j in range(n + 1):
            u, v = f32(i) * step, f32(j) * step
            bu, bdu = [bern(u, k) for k in range(4)], [bern_d(u, k) for k in range(4)]
            bv, bdv = [bern(v, k) for k in range(4)], [bern_d(v, k) for k in range(4)]
            ps.append(ev(c, bu, bv))
            ns.append(cross(ev(c, bdu, bv), ev(c, bu, bdv)))
            uvs.append((u, v))
    tris = []
    vs = n + 1
    for i in range(n):
        for j in range(n):
            v00, v10, v01, v11 = i * vs + j, (i + 1) * vs + j, i * vs + j + 1, (i + 1) * vs + j + 1
            tris += [(v00, v10, v01), (v10, v11, v01)]
    return np.array(ps), np.array(ns), np.array(uvs, np.float32), tris


def test_fixture_patch_matches_numpy_restatement():
    text = open(os.path.join(ROOT, "fixtures", "scenes", "bezier.bling")).read()
    block = re.search(r"bezier\s+subdivs\s+(\d+)\s+p\s*\{([^}]*)\}", text)
    n = int(block.group(1))
    c = np.array([float(x) for x in block.group(2).replace(",", " ").split()], np.float32)
    assert c.size == 48
    job = load_config("X16")
    d = C.cast(C.c_void_p(job.desc), C.POINTER(DescHead)).contents
    assert d.num_triangles == 2 * 6 * 6 + 2 * 5 * 5                  # subdivs 6 and 5
    verts = np.ctypeslib.as_array(d.vertices, shape=(3 * d.num_vertices,)).reshape(-1, 3)
    idx = np.ctypeslib.as_array(d.tri_indices, shape=(3 * d.num_triangles,)).reshape(-1, 3)
    uvs = np.ctypeslib.as_array(d.tri_uvs, shape=(6 * d.num_triangles,)).reshape(-1, 3, 2)
    nrm = np.ctypeslib.as_array(d.tri_normals, shape=(9 * d.num_triangles,)).reshape(-1, 3, 3)
    ps, ns, uv, tris = one_patch(c, n)                                # first patch: identity transform
    assert len(tris) == 2 * n * n
    for t, tri in enumerate(tris):
        for k, vi in enumerate(tri):
            np.testing.assert_array_equal(verts[idx[t, k]], ps[vi], err_msg=f"p tri {t} vertex {k}")
            np.testing.assert_array_equal(nrm[t, k], ns[vi], err_msg=f"n tri {t} vertex {k}")
            np.testing.assert_array_equal(uvs[t, k], uv[vi], err_msg=f"uv tri {t} vertex {k}")


def test_patch_needs_48_values():
    text = open(os.path.join(ROOT, "fixtures", "scenes", "bezier.bling")).read()
    bad = re.sub(r"(p \{ )([-0-9.]+), ", r"\1", text, count=1)   # drop one value of the first patch
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "bad.bling")
        open(p, "w").write(bad)
        with pytest.raises(ParseError, match="48 values"):
            parse_job(p)


@pytest.mark.skipif(not os.path.isdir(REF_EXAMPLES), reason="reference examples absent (GPU box)")
@pytest.mark.parametrize("name,tris", [("gumbo", 51 * 2 * 16 * 16), ("environment", 0), ("crystal", 0)])
def test_reference_scenes_load_with_the_fixture_map(name, tris):
    """environment.bling reads an .hdr from its author's home directory; gumbo.bling and crystal.bling
    read envmaps/studio015.hdr through `rgbeFile`, a map keyword the reference's own parser does not
    have (MaterialParser.hs:258-264 knows `file`).  With `file "<fixture>.hdr"` substituted, all
    three load; gumbo's 51 Bezier patches tessellate to 26 112 triangles."""
    text = open(os.path.join(REF_EXAMPLES, f"{name}.bling")).read()
    text = re.sub(r'^(\s*l\s*\{\s*)(?:file|rgbeFile)\s+"[^"]*"', lambda m: m.group(1) + f'file "{HDR}"', text,
                  flags=re.M)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, f"{name}.bling")
        open(p, "w").write(text)
        job = parse_job(p, "force_path=1")
    assert job.counts()["triangles"] == tris
    assert job.counts()["lights"] >= 1
