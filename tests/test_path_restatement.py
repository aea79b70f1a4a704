"""An independent restatement of the path composition for the cornell profile, bit for bit against
the oracle.

The reference ships no fixtures, so the goldens follow the oracle.  A misreading of
Path.hs / Scene.hs shared by the oracle and the device would pass every golden.  This file restates
the per-sample radiance of the C1 configuration (cornell-box.bling, stratified 2 x 2, path maxDepth
15 sampleDepth 3) in numpy binary32 from the Haskell sources alone, and compares 64 samples with the
oracle's sample_li bit for bit:

* Integrator/Path.hs:25-87 nextVertex: the dimension layout (rnd' 1+4d / 2+4d / 3+4d / 0+4d, rnd2D'
  1+3d / 2+3d / 0+3d), intLe on specular bounces, l + t * lHere, Russian roulette from depth 8 with
  pc = min 0.75 (sY t), t' = sScale (f * t) (1 / pc), the end at maxDepth;
* Scene.hs:61-118 sampleOneLight / estimateDirect / sampleLightMis / sampleBsdfMis (guard order,
  power heuristic, l' == l, intLe (-wi): trap T6), Scene.hs:45-51 with kdTreePrimitive's root test
  (KdTree.hs:236-244, tests/test_kd_root.py intersect_aabb) and Primitive.near's fold (T11);
* Reflection.hs:201-332 mkBsdf / sampleBsdf'' / evalBsdf (T7: the flipped eval) / bsdfPdf over one
  Lambertian or Oren-Nayar lobe (Diffuse.hs, Material.hs mkMatte);
* TriangleMesh.hs:160-207 (hit, uv partials, mkDgTri) and Shape.hs quad + Geometry.hs transDg for the
  light; Light.hs area-light sample / pdf / lEmit;
* the sampler: common/counter_rng.h version 2 (tests/test_rng_loader.py hash5 / permute, restated).

Leaf formulas come from tests/test_kat_hotpath.py (each pinned there against the Haskell); the
scene's spectra and matrices from the loader (pinned there too).  CPU only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import oracle_py  # noqa: E402
from bling_amd.scene import load_config  # noqa: E402
from scene_desc import arr, desc  # noqa: E402
from test_kat_hotpath import (INV_PI, ONE, ZERO, V, area_light_sample, cosine_hemisphere, cross, dot,  # noqa: E402
                              fire_ray, ghc_max, ghc_min, normalize, oren_nayar, quad_intersect, quad_pdf, sqrtf,
                              to_same_hemi, trans_point, trans_vector, tri_intersect)
from test_kd_root import intersect_aabb  # noqa: E402
from test_rng_loader import hash5, permute  # noqa: E402

f32 = np.float32
SEED = 0x0B11A6
ALMOST_ONE = f32.fromhex("0x1.fffffep-1") if hasattr(f32, "fromhex") else np.float32(float.fromhex("0x1.fffffep-1"))
BLACK = np.zeros(16, np.float32)
DIM_PIX, DIM_1D_PERM, DIM_1D_J, DIM_2D_PERM, DIM_2D_J = 0x1000, 0x3000, 0x4000, 0x5000, 0x6000
DIM_FRESH1D, DIM_FRESH2D, ALL = 0x7000, 0x8000, 0xFFFFFFFF


def _cie_y():
    from test_kat_hotpath import _table
    text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bling_amd", "csrc",
                             "common", "spectral_data.h")).read()
    import re
    ysum = float.fromhex(re.search(r"BLING_CIE_Y_SUM = (-?0x[0-9a-fA-F.]+p[+-]?\d+)f", text).group(1))
    return _table("BLING_CIE_Y_BANDS").astype(np.float32), f32(ysum)


def s_y(t, cy, ysum):                                        # Spectrum.hs:371-373
    acc = ZERO
    for i in range(16):                                      # V.sum = foldl' (+) 0
        acc = f32(acc + f32(t[i] * cy[i]))
    return f32(acc / ysum)


def sscale(s, k):
    return (s * f32(k)).astype(np.float32)


def is_black(s):
    return bool((s == 0).all())


def power_heuristic(f, g):                                   # Montecarlo.hs:113-116, nf = ng = 1
    f, g = f32(f32(1) * f32(f)), f32(f32(1) * f32(g))
    return f32(f32(f * f) / f32(f32(f * f) + f32(g * g)))


def ray_at(o, d, t):
    return (o + (d * f32(t)).astype(np.float32)).astype(np.float32)


def trans_normal(inv, n):                                    # Transform.hs:267-272 (mi m r c = m[4 r + c] of the inverse)
    return V(*[f32(f32(f32(inv[c] * n[0]) + f32(inv[4 + c] * n[1])) + f32(inv[8 + c] * n[2])) for c in range(3)])


def local(cs, v):                                            # worldToLocal (Math.hs:439-441)
    sn, tn, nn = cs
    return V(dot(v, sn), dot(v, tn), dot(v, nn))


def world(cs, v):                                            # localToWorld (Math.hs:443-449)
    sn, tn, nn = cs
    return V(*[f32(f32(f32(sn[a] * v[0]) + f32(tn[a] * v[1])) + f32(nn[a] * v[2])) for a in range(3)])


class Scene:
    def __init__(self, job):
        d = desc(job)
        self.d = d
        nv, nt = d.num_vertices, d.num_triangles
        self.verts = np.ctypeslib.as_array(d.vertices, shape=(3 * nv,)).reshape(nv, 3).astype(np.float32)
        self.idx = np.ctypeslib.as_array(d.tri_indices, shape=(3 * nt,)).reshape(nt, 3)
        self.uvs = np.ctypeslib.as_array(d.tri_uvs, shape=(6 * nt,)).reshape(nt, 6).astype(np.float32)
        self.tri_mat = np.ctypeslib.as_array(d.tri_material, shape=(nt,))
        self.prims = [(d.prim_kind[i], d.prim_index[i]) for i in range(d.num_prims)]
        lo = np.full(3, np.inf, np.float32)
        hi = np.full(3, -np.inf, np.float32)
        for kind, i in self.prims:                           # the kd-tree's bounds: union of primitive bounds
            pts = self.verts[self.idx[i]] if kind == 0 else self._shape_corners(d.shapes[i])
            lo, hi = np.minimum(lo, pts.min(0)), np.maximum(hi, pts.max(0))
        self.lo, self.hi = lo, hi
        assert d.num_lights == 1 and d.lights[0].kind == 1
        self.light = d.lights[0]
        self.light_shape = d.shapes[self.light.shape]
        self.radiance = arr(self.light.radiance)

    @staticmethod
    def _shape_corners(s):                                   # transBox o2w (objectBounds (Shape.hs:299-311), quad)
        sx, sy = f32(s.params[0]), f32(s.params[1])
        o2w = arr(s.o2w)
        return np.array([trans_point(o2w, V(x, y, 0)) for x in (-sx, sx) for y in (-sy, sy)], np.float32)

    def material(self, mi):
        m = self.d.materials[mi]
        assert m.kind == 1                                   # matte
        return arr(self.d.textures[m.tex[0]].value), f32(m.scalar[0])

    # ---------------------------------------------------------------- intersection
    def _tri_hit(self, k, ro, rd, tmin, tmax):
        p1, p2, p3 = (self.verts[j] for j in self.idx[k])
        h = tri_intersect(p1, p2, p3, ro, rd, tmin, tmax)
        if h is None:
            return None
        t, b1, b2 = h
        uv = self.uvs[k]
        du1, du2 = f32(uv[0] - uv[4]), f32(uv[2] - uv[4])
        dv1, dv2 = f32(uv[1] - uv[5]), f32(uv[3] - uv[5])
        dp1, dp2 = (p1 - p3).astype(np.float32), (p2 - p3).astype(np.float32)
        det = f32(f32(du1 * dv2) - f32(dv1 * du2))
        assert det != 0
        inv = f32(ONE / det)
        dpdu = ((dv2 * dp1).astype(np.float32) - (dv1 * dp2).astype(np.float32)).astype(np.float32) * inv
        dpdv = ((-du2 * dp1).astype(np.float32) + (du1 * dp2).astype(np.float32)).astype(np.float32) * inv
        dpdu, dpdv = dpdu.astype(np.float32), dpdv.astype(np.float32)
        n = normalize(cross(dpdu, dpdv))                     # mkDgTri
        return dict(t=t, p=ray_at(ro, rd, t), n=n, dpdu=dpdu, eps=f32(f32(1e-3) * t), mat=int(self.tri_mat[k]),
                    light=False)

    def _quad_hit(self, s, ro, rd, tmin, tmax):
        w2o, o2w = arr(s.w2o), arr(s.o2w)
        oo, od = trans_point(w2o, ro), trans_vector(w2o, rd)  # transRay w2o
        h = quad_intersect(f32(s.params[0]), f32(s.params[1]), oo, od, tmin, tmax)
        if h is None:
            return None
        t, p, n = h
        return dict(t=t, p=trans_point(o2w, p), n=normalize(trans_normal(w2o, n)),   # transDg o2w
                    dpdu=trans_vector(o2w, V(s.params[0], 0, 0)), eps=f32(f32(5e-4) * t), mat=s.material,
                    light=s.light >= 0)

    def intersect(self, ro, rd, tmin, tmax=f32(np.inf)):
        if intersect_aabb(self.lo, self.hi, ro, rd, tmin, tmax) is None:
            return None
        best = None
        for kind, i in self.prims:                           # Primitive.near: rayMax = the hit so far (T11)
            h = self._tri_hit(i, ro, rd, tmin, tmax) if kind == 0 else self._quad_hit(self.d.shapes[i], ro, rd, tmin, tmax)
            if h is not None:
                best, tmax = h, h["t"]
        return best

    def occluded(self, ro, rd, tmin, tmax):
        if intersect_aabb(self.lo, self.hi, ro, rd, tmin, tmax) is None:
            return False
        for kind, i in self.prims:
            if kind == 0:
                p1, p2, p3 = (self.verts[j] for j in self.idx[i])
                if tri_intersect(p1, p2, p3, ro, rd, tmin, tmax) is not None:
                    return True
            elif self._quad_hit(self.d.shapes[i], ro, rd, tmin, tmax) is not None:
                return True
        return False

    # ---------------------------------------------------------------- the area light (Light.hs)
    def light_sample(self, p, eps, u1, u2):
        li, wi, pd, ro, rd, tmin, tmax = area_light_sample(self.light_shape, self.radiance, p, eps, u1, u2)
        return li, wi, pd, (ro, rd, tmin, tmax)

    def light_pdf(self, p, wi):
        s = self.light_shape
        w2o = arr(s.w2o)
        return quad_pdf(f32(s.params[0]), f32(s.params[1]), trans_point(w2o, p), trans_vector(w2o, wi))


class Bsdf:
    """mkMatte -> mkBsdf' [Lambertian r | OrenNayar r sigma] dgg dgs (no shading normals: dgs = dgg)."""

    def __init__(self, r, sigma, hit):
        self.r, self.sigma = r, sigma
        nn = hit["n"]
        sn = normalize(hit["dpdu"])
        self.cs = (sn, cross(nn, sn), nn)
        self.ng, self.p = hit["n"], hit["p"]

    def _eval(self, wo, wi):                                 # bxdfEval of the lobe (Diffuse.hs)
        if self.sigma == 0:
            return sscale(self.r, f32(INV_PI * abs(wo[2])))
        return sscale(oren_nayar(self.r, self.sigma, wo, wi), f32(INV_PI * abs(wo[2])))

    def _pdf(self, wo, wi):                                  # cosPdf
        return f32(INV_PI * abs(wi[2])) if f32(wo[2] * wi[2]) > 0 else ZERO

    def eval(self, wo_w, wi_w):                              # evalBsdf False (Reflection.hs:306-320)
        cos_wo = dot(wo_w, self.ng)
        side = f32(dot(wi_w, self.ng) / cos_wo)
        if side == 0 or abs(cos_wo) < f32(1e-5):
            return BLACK.copy()
        if side < 0:                                         # a reflection lobe only
            return BLACK.copy()
        wo, wi = local(self.cs, wo_w), local(self.cs, wi_w)
        return (BLACK + self._eval(wi, wo)).astype(np.float32)   # flip (bxdfEval b): trap T7; V.sum from 0

    def pdf(self, wo_w, wi_w):                               # bsdfPdf
        return f32(f32(ZERO + self._pdf(local(self.cs, wo_w), local(self.cs, wi_w))) / f32(1))

    def sample(self, wo_w, uc, u1, u2):                      # sampleBsdf'' False bxdfAll, one lobe
        wo = local(self.cs, wo_w)
        wi = to_same_hemi(wo, cosine_hemisphere(u1, u2))
        same = f32(wo[2] * wi[2]) > 0
        if self.sigma == 0:
            f, pdf = (self.r.copy(), self._pdf(wo, wi)) if same else (BLACK.copy(), ZERO)
        else:
            f, pdf = (oren_nayar(self.r, self.sigma, wo, wi), self._pdf(wo, wi)) if same else (BLACK.copy(), ZERO)
        wi_w = world(self.cs, wi)
        side = f32(dot(wi_w, self.ng) / dot(wo_w, self.ng))
        if pdf == 0 or side == 0 or side < 0:                # emptyBsdfSample; not (flt bxdf)
            return ZERO, BLACK.copy(), V(0, 1, 0)
        return pdf, f, wi_w


class Sampler:
    """runSample's stratified sampler under the counter RNG (counter_rng.h v2; dev_shade.h rnd1 / rnd2)."""

    def __init__(self, job, ix, iy, n):
        c = job.config
        self.nu, self.nv, self.spp = c.nu, c.nv, c.spp
        self.n1d, self.n2d = 4 * c.sample_depth, 3 * c.sample_depth
        x0, x1, y0, _ = job.extent()
        self.pixel = (iy - y0) * (x1 - x0 + 1) + (ix - x0)
        self.n = n

    def h(self, sample, dim):
        return hash5(SEED, 0, self.pixel, sample, dim)

    @staticmethod
    def u01(w):
        return f32(f32(w >> 8) * f32(1.0 / 16777216.0))

    def rnd1(self, dim):
        if dim < self.n1d:
            j = permute(self.n, self.spp, self.h(ALL, DIM_1D_PERM + dim))
            jit = self.u01(self.h(self.n, DIM_1D_J + dim))
            return ghc_min(ALMOST_ONE, f32(f32(f32(j) + jit) * f32(ONE / f32(self.spp))))
        return self.u01(self.h(self.n, DIM_FRESH1D + dim))

    def rnd2(self, dim):
        if dim < self.n2d:
            j = permute(self.n, self.spp, self.h(ALL, DIM_2D_PERM + dim))
            ju, jv = self.u01(self.h(self.n, DIM_2D_J + 2 * dim)), self.u01(self.h(self.n, DIM_2D_J + 2 * dim + 1))
            u, v = divmod(j, self.nu)                        # quotRem j nu (trap T5)
            return (ghc_min(ALMOST_ONE, f32(f32(f32(u) + ju) * f32(ONE / f32(self.nu)))),
                    ghc_min(ALMOST_ONE, f32(f32(f32(v) + jv) * f32(ONE / f32(self.nv)))))
        return self.u01(self.h(self.n, DIM_FRESH2D + 2 * dim)), self.u01(self.h(self.n, DIM_FRESH2D + 2 * dim + 1))

    def camera(self):                                        # pixel offsets: stratum n quotRem nu
        u, v = divmod(self.n, self.nu)
        ju, jv = self.u01(self.h(self.n, DIM_PIX)), self.u01(self.h(self.n, DIM_PIX + 1))
        return (ghc_min(ALMOST_ONE, f32(f32(f32(u) + ju) * f32(ONE / f32(self.nu)))),
                ghc_min(ALMOST_ONE, f32(f32(f32(v) + jv) * f32(ONE / f32(self.nv)))))


class _M:
    def __init__(self, m):
        self.m = m


def sample_li(sc, job, ix, iy, n, cy, ysum):
    """Path.li for camera sample (ix, iy, n): nextVertex (Path.hs:41-87) as a loop."""
    smp = Sampler(job, ix, iy, n)
    ox, oy = smp.camera()
    cam = sc.d.camera
    ro, rd = fire_ray(_M(arr(cam.c2w)), _M(arr(cam.r2c)), f32(cam.lens_radius), f32(cam.focal_distance),
                      f32(f32(ix) + ox), f32(f32(iy) + oy), ZERO, ZERO)
    md = job.config.max_depth
    hit = sc.intersect(ro, rd, ZERO)
    depth, spec, t, l = 0, True, np.ones(16, np.float32), BLACK.copy()
    while True:
        if hit is None:                                      # area lights: le = black
            return (l + (t * BLACK).astype(np.float32)).astype(np.float32) if spec else l
        if depth == md:
            return l
        l_num = smp.rnd1(1 + 4 * depth)                      # one light: not used past lc == 1
        lu1, lu2 = smp.rnd2(1 + 3 * depth)
        bc = smp.rnd1(2 + 4 * depth)
        bu1, bu2 = smp.rnd2(2 + 3 * depth)
        del l_num
        intl = BLACK.copy()
        if spec and hit["light"] and dot(hit["n"], rd) > 0:   # intLe int rd (lEmit: n . wo > 0), trap T6
            intl = sc.radiance.copy()
        wo = (-rd).astype(np.float32)
        r, sigma = sc.material(hit["mat"])
        bsdf = Bsdf(r, sigma, hit)
        p, eps = bsdf.p, hit["eps"]
        # sampleLightMis
        li, wi, lpdf, (sro, srd, stmin, stmax) = sc.light_sample(p, eps, lu1, lu2)
        ls = BLACK.copy()
        if not (lpdf == 0 or is_black(li)):
            f = bsdf.eval(wo, wi)
            if not is_black(f) and not sc.occluded(sro, srd, stmin, stmax):
                w = power_heuristic(lpdf, bsdf.pdf(wo, wi))
                ls = sscale((f * li).astype(np.float32), f32(w / lpdf))
        # sampleBsdfMis
        bpdf, bf, bwi = bsdf.sample(wo, bc, bu1, bu2)
        bs = BLACK.copy()
        if not (bpdf == 0 or is_black(bf)):
            lp = sc.light_pdf(p, bwi)
            w = power_heuristic(bpdf, lp)
            lint = sc.intersect(p, bwi, eps)
            if lint is None:
                bs = sscale((bf * BLACK).astype(np.float32), w)
            elif lint["light"]:                              # l' == l: intLe (-wi)
                le = sc.radiance if dot(lint["n"], (-bwi).astype(np.float32)) > 0 else BLACK
                bs = sscale((bf * le).astype(np.float32), w)
        lhere = (intl + (ls + bs).astype(np.float32)).astype(np.float32)
        l = (l + (t * lhere).astype(np.float32)).astype(np.float32)
        pc = ONE if depth <= 7 else ghc_min(f32(0.75), s_y(t, cy, ysum))
        x = smp.rnd1(3 + 4 * depth)
        if x > pc:
            return l
        uc = smp.rnd1(0 + 4 * depth)
        ud1, ud2 = smp.rnd2(0 + 3 * depth)
        cpdf, cf, cwi = bsdf.sample(wo, uc, ud1, ud2)
        t = sscale((cf * t).astype(np.float32), f32(ONE / pc))
        if cpdf == 0 or is_black(cf):
            return l
        depth, spec, rd = depth + 1, False, cwi
        hit = sc.intersect(p, cwi, eps)


def test_path_restatement_matches_the_oracle_bit_for_bit():
    job = load_config("C1")
    sc = Scene(job)
    cy, ysum = _cie_y()
    orc = oracle_py.Oracle(job)
    rng = np.random.default_rng(21)
    smp = np.stack([rng.integers(0, job.width, 64), rng.integers(0, job.height, 64),
                    rng.integers(0, job.config.spp, 64)], 1).astype(np.int32)
    smp[:8, 0] = 128                                         # a few down the middle column (the light above)
    want, _, _ = orc.sample_li_batch(smp, seed=SEED, pass_index=0)
    got = np.array([sample_li(sc, job, int(x), int(y), int(n), cy, ysum) for x, y, n in smp], np.float32)
    same = [np.array_equal(got[k], want[k]) for k in range(len(smp))]
    bad = [(tuple(smp[k]), got[k][:3], want[k][:3]) for k in range(len(smp)) if not same[k]]
    assert not bad, bad[:4]
    assert (want.sum(1) > 0).sum() >= 32                     # most samples carry light
