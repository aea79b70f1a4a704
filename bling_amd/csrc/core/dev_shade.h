// dev_shade.h -- per-vertex shading of Integrator.Path on the device: BSDF construction and
// sampling (Reflection.hs:201-332 with Diffuse/Specular/Microfacet/Fresnel/Material.hs), light
// sampling and MIS (Light.hs:85-229, Scene.hs:61-118), the counter-RNG sampler (Sampling.hs:101-221)
// and the perspective camera (Camera.hs:49-76).  Expression order follows the Haskell sources.
#pragma once
#include "../common/perlin.h"
#include "../common/cellnoise.h"
#include "../common/cr_math.h"
#include "../common/sky_model.h"
#include "../common/image_tex.h"
#include "dev_common.h"
#include "dev_scene.h"
#include "dev_shapes.h"

namespace bd {

// ================================================================ sampler (counter RNG)
// skey: the sample's key (common/counter_rng.h sample_key), pkey: the pixel's (the stratified
// dimensions' permutation key sample_key(pkey, ALL_SAMPLES) is formed where one is drawn).
struct SampleKey { uint32_t pkey; uint32_t skey; uint32_t n; };

DEV SampleKey sample_key(uint32_t seed, uint32_t pass, uint32_t pixel, uint32_t n) {
  const uint32_t pk = brng::pixel_key(seed, pass, pixel);
  return SampleKey{pk, brng::sample_key(pk, n), n};
}
DEV float draw01(const SampleKey& k, uint32_t dim) { return brng::u01(brng::draw(k.skey, dim)); }

// brng::permute with the spp-specific mask and modulus precomputed (DevScene::fd_spp): the same
// cycle-walking bijection, bit for bit
DEV uint32_t permute_spp(const DevScene& S, uint32_t i, uint32_t p) {
  if (S.spp <= 1) return 0;
#if defined(BLING_RNG_COST_EXPERIMENT) || defined(BLING_RNG_PERM_EXPERIMENT)   // measurement-only builds
  return S.fd_spp.mod(i + p);
#endif
  return S.fd_spp.mod(brng::permute_w(i, (uint32_t)S.spp, S.perm_mask_spp, p) + p);
}
// stratum of sample k.n in the pixel's shuffled strata of dimension code `perm`
DEV uint32_t stratum(const DevScene& S, const SampleKey& k, uint32_t perm) {
  return permute_spp(S, k.n, brng::draw(brng::sample_key(k.pkey, brng::ALL_SAMPLES), perm));
}

// rnd' (Sampling.hs:203-211): stratified dimension below n1d, else a fresh draw
DEV float rnd1(const DevScene& S, const SampleKey& k, int dim) {
  if (S.sampler == BLING_SAMPLER_STRATIFIED && dim < S.n1d) {
    const uint32_t j = stratum(S, k, brng::DIM_1D_PERM + dim);
    const float jit = draw01(k, brng::DIM_1D_J + dim);
    return fminf(ALMOST_ONE, ((float)j + jit) * S.inv_spp);
  }
  return draw01(k, brng::DIM_FRESH1D + dim);
}
DEV void rnd2(const DevScene& S, const SampleKey& k, int dim, float* a, float* b) {
  if (S.sampler == BLING_SAMPLER_STRATIFIED && dim < S.n2d) {
    const uint32_t j = stratum(S, k, brng::DIM_2D_PERM + dim);
    const float ju = draw01(k, brng::DIM_2D_J + 2 * dim);
    const float jv = draw01(k, brng::DIM_2D_J + 2 * dim + 1);
    const uint32_t uq = S.fd_nu.div(j);
    int u = (int)uq, v = (int)(j - uq * (uint32_t)S.nu);            // quotRem i nu (trap T5)
    *a = fminf(ALMOST_ONE, ((float)u + ju) * S.inv_nu);
    *b = fminf(ALMOST_ONE, ((float)v + jv) * S.inv_nv);
    return;
  }
  *a = draw01(k, brng::DIM_FRESH2D + 2 * dim);
  *b = draw01(k, brng::DIM_FRESH2D + 2 * dim + 1);
}
DEV void camera_sample(const DevScene& S, const SampleKey& k, float* ox, float* oy, float* lu, float* lv) {
  if (S.sampler == BLING_SAMPLER_STRATIFIED) {
    float du = S.inv_nu, dv = S.inv_nv;
    const uint32_t nq = S.fd_nu.div(k.n);
    int u = (int)nq, v = (int)(k.n - nq * (uint32_t)S.nu);
    float ju = draw01(k, brng::DIM_PIX), jv = draw01(k, brng::DIM_PIX + 1);
    *ox = fminf(ALMOST_ONE, ((float)u + ju) * du);
    *oy = fminf(ALMOST_ONE, ((float)v + jv) * dv);
    const uint32_t j = stratum(S, k, brng::DIM_LENS_PERM);
    float lj = draw01(k, brng::DIM_LENS_J), lk = draw01(k, brng::DIM_LENS_J + 1);
    const uint32_t jq = S.fd_nu.div(j);
    int lu_i = (int)jq, lv_i = (int)(j - jq * (uint32_t)S.nu);
    *lu = fminf(ALMOST_ONE, ((float)lu_i + lj) * du);
    *lv = fminf(ALMOST_ONE, ((float)lv_i + lk) * dv);
    return;
  }
  *ox = draw01(k, brng::DIM_RAND_CAM);
  *oy = draw01(k, brng::DIM_RAND_CAM + 1);
  *lu = draw01(k, brng::DIM_RAND_CAM + 2);
  *lv = draw01(k, brng::DIM_RAND_CAM + 3);
}

// fireRay (Camera.hs:49-76)
DEV Ray fire_ray(const bling_camera& cam, float ix, float iy, float lu, float lv) {
  if (cam.kind == BLING_CAM_ENVIRONMENT) {
    float t = PI * iy / cam.yres, p = 2.f * PI * ix / cam.xres;
    const bcr::SinCos st = bcr::sincosf(t), sp = bcr::sincosf(p);
    V3 d = mk(st.s * sp.c, st.c, st.s * sp.s);
    return Ray{xpoint(cam.c2w, mk(0.f, 0.f, 0.f)), xvector(cam.c2w, d), 0.f, INFINITY};
  }
  V3 pc = xpoint(cam.r2c, mk(ix, iy, 0.f));
  Ray r{mk(0.f, 0.f, 0.f), normalize(pc), 0.f, INFINITY};
  if (cam.lens_radius > 0.f) {
    float dx, dy;
    concentric_sample_disk(lu, lv, &dx, &dy);
    V3 ro = mk(dx * cam.lens_radius, dy * cam.lens_radius, 0.f);
    V3 pf = ray_at(r, cam.focal_distance / r.d.z);
    r = Ray{ro, normalize(pf - ro), 0.f, INFINITY};
  }
  return Ray{xpoint(cam.c2w, r.o), xvector(cam.c2w, r.d), r.tmin, r.tmax};
}

// ================================================================ hit reconstruction
struct DG { V3 p, n; float u, v; V3 dpdu, dpdv; };

// triangleIntersect's DG (TriangleMesh.hs:169-205) from (t, b1, b2)
// The shading frame of one triangle (mkDgTri, TriangleMesh.hs:140-158): everything the hit's
// differential geometry takes from the triangle alone -- dpdu, dpdv (or the coordinate system of
// the face normal when the uv determinant is 0) and the normal normalize(dpdu x dpdv) -- plus its
// uvs, as 4 float4 {dpdu, uv00 | dpdv, uv01 | n, uv10 | uv11, uv20, uv21, 0}.  k_tri_frames
// (core.hip) runs it once per triangle at upload with these operations in this order, so tri_dg
// returns the bits the per-hit computation returned: a hit reads 64 B instead of 15 scattered
// floats and skips two normalisations, a division and three cross products.
DEV void tri_frame_build(const float* P, const float* uv, float4* out) {
  V3 p1 = mk(P[0], P[1], P[2]), p2 = mk(P[3], P[4], P[5]), p3 = mk(P[6], P[7], P[8]);
  float uv00 = uv[0], uv01 = uv[1], uv10 = uv[2], uv11 = uv[3], uv20 = uv[4], uv21 = uv[5];
  V3 e1 = p2 - p1, e2 = p3 - p1;
  V3 n = normalize(cross(e1, e2));
  float du1 = uv00 - uv20, du2 = uv10 - uv20, dv1 = uv01 - uv21, dv2 = uv11 - uv21;
  V3 dp1 = p1 - p3, dp2 = p2 - p3;
  float det = du1 * dv2 - dv1 * du2;
  V3 dpdu, dpdv;
  if (det == 0.f) { LC c = coordinate_system(n); dpdu = c.s; dpdv = c.t; }
  else {
    float idet = 1.f / det;
    dpdu = sm(idet, sm(dv2, dp1) - sm(dv1, dp2));
    dpdv = sm(idet, sm(-du2, dp1) + sm(du1, dp2));
  }
  const V3 gn = normalize(cross(dpdu, dpdv));
  out[0] = make_float4(dpdu.x, dpdu.y, dpdu.z, uv00);
  out[1] = make_float4(dpdv.x, dpdv.y, dpdv.z, uv01);
  out[2] = make_float4(gn.x, gn.y, gn.z, uv10);
  out[3] = make_float4(uv11, uv20, uv21, 0.f);
}
DEV DG tri_dg(const DevScene& S, uint32_t tri, const Ray& r, float t, float b1, float b2) {
  const float4 f0 = gen(S.tri_frame[4 * tri]), f1 = gen(S.tri_frame[4 * tri + 1]);
  const float4 f2 = gen(S.tri_frame[4 * tri + 2]), f3 = gen(S.tri_frame[4 * tri + 3]);
  float b0 = 1.f - b1 - b2;
  DG g;
  g.p = ray_at(r, t);
  g.u = b0 * f0.w + b1 * f2.w + b2 * f3.y;
  g.v = b0 * f1.w + b1 * f3.x + b2 * f3.z;
  g.dpdu = mk(f0.x, f0.y, f0.z); g.dpdv = mk(f1.x, f1.y, f1.z);
  g.n = mk(f2.x, f2.y, f2.z);
  return g;
}

// Object-space normal of a disk / cylinder / box hit at p (Shape.hs:96-98, 136-140, 155)
DEV V3 shape2_normal(const DevShape& s, const Ray& r, V3 p) {
  if (s.kind == BLING_SHAPE_DISK) return mk(0.f, 0.f, -1.f);
  if (s.kind == BLING_SHAPE_CYLINDER) {
    const float phimax = s.params[3];
    V3 dpdu = mk(-(phimax * p.y), phimax * p.x, 0.f), dpdv = mk(0.f, 0.f, s.params[2] - s.params[1]);
    return normalize(cross(dpdu, dpdv));
  }
  float t0, t1;
  int ax = 0;
  box_slabs(s.params, r, &t0, &t1, &ax);
  const float half = (s.params[ax] + s.params[3 + ax]) / 2.f;
  const float dir = v3c(p, ax) > half ? 1.f : -1.f;
  return normalize(mk(ax == 0 ? dir : 0.f, ax == 1 ? dir : 0.f, ax == 2 ? dir : 0.f));
}

// Quad / Sphere DG in object space (Shape.hs:157-229), then transDg o2w (DifferentialGeometry.hs:72-81)
template <uint32_t F>
DEV DG shape_dg(const DevShape& s, const Ray& rw, float t) {
  Ray r{xpoint(s.w2o, rw.o), xvector(s.w2o, rw.d), rw.tmin, rw.tmax};
  V3 p = ray_at(r, t);
  DG g;
  if ((F & FT_SHAPES2) && s.kind >= BLING_SHAPE_DISK) {
    // disk / cylinder / box: mkDg' p n (DifferentialGeometry.hs:53-56), dpdu dpdv from coordinateSystem n
    V3 n = shape2_normal(s, r, p);
    LC c = coordinate_system(n);
    g.p = p; g.n = n; g.u = 0.f; g.v = 0.f; g.dpdu = c.s; g.dpdv = c.t;
    DG w;
    w.p = xpoint(s.o2w, g.p);
    w.n = normalize(xnormal(s.w2o, g.n));
    w.u = 0.f; w.v = 0.f;
    w.dpdu = xvector(s.o2w, g.dpdu);
    w.dpdv = xvector(s.o2w, g.dpdv);
    return w;
  }
  if (!(F & FT_NONQUAD) || s.kind == BLING_SHAPE_QUAD) {
    float sx = s.params[0], sy = s.params[1];
    g.u = (sx + p.x) / (2.f * sx); g.v = (sy + p.y) / (2.f * sy);
    g.dpdu = mk(sx, 0.f, 0.f); g.dpdv = mk(0.f, sy, 0.f);
  } else {
    float rad = s.params[0];
    const float thetaMin = PI, thetaMax = 0.f, phiMax = TWO_PI;
    float phi = atan2p(p.y, p.x);
    g.u = phi / phiMax;
    float theta = bcr::acosf(clampf(p.z / rad, -1.f, 1.f));
    g.v = (theta - thetaMin) / (thetaMax - thetaMin);
    float zr = sqrtf(p.x * p.x + p.y * p.y);
    float izr = 1.f / zr;
    float cosphi = p.x * izr, sinphi = p.y * izr;
    g.dpdu = mk(-(phiMax * p.y), phiMax * p.x, 0.f);
    g.dpdv = vs(mk(p.z * cosphi, p.z * sinphi, -(rad * bcr::sinf(theta))), thetaMax - thetaMin);
  }
  g.p = p;
  g.n = normalize(cross(g.dpdu, g.dpdv));
  DG w;
  w.p = xpoint(s.o2w, g.p);
  w.n = normalize(xnormal(s.w2o, g.n));
  w.u = g.u; w.v = g.v;
  w.dpdu = xvector(s.o2w, g.dpdu);
  w.dpdv = xvector(s.o2w, g.dpdv);
  return w;
}

// ================================================================ textures / BSDF
template <uint32_t F>
DEV const float* eval_texture(const DevScene& S, int ti, float u, float v) {            // Texture.hs:191-207
  if (!(F & FT_GRAPHPAPER)) return gen(S.textures[ti]).value;
  for (int guard = 0; guard < 16; ++guard) {
    const bling_texture& t = gen(S.textures[ti]);
    if (t.kind == BLING_TEX_CONST) return t.value;
    float x = t.uv_map[0] * u + t.uv_map[2], z = t.uv_map[1] * v + t.uv_map[3];
    float xf = fabsf(x - (float)(long long)x), zf = fabsf(z - (float)(long long)z);
    float lo = t.line_width / 2.f, hi = 1.0f - lo;
    ti = (xf < lo || zf < lo || xf > hi || zf > hi) ? t.tex2 : t.tex1;
  }
  return gen(S.textures[ti]).value;
}

enum : int { F_REFL = 1, F_TRANS = 2, F_DIFF = 4, F_GLOSSY = 8, F_SPEC = 16 };
enum : int { K_LAMB = 0, K_OREN = 1, K_MICRO = 2, K_SREFL = 3, K_STRANS = 4, K_FBLEND = 5 };
// K_FBLEND (mkFresnelBlend, Microfacet.hs:56-105) reuses the fields: r = rd, eta = rs, k = ra,
// e = ex, A = ey (the anisotropic exponents), B = depth
enum : int { FR_NOOP = 0, FR_DIEL = 1, FR_COND = 2 };

// A BxDF keeps pointers to its (constant-texture) spectra instead of 16-register copies.
struct BxDF {
  int kind, flags, fr;
  const float* r;         // reflectance / transmittance (NULL = white)
  const float* eta;       // conductor eta / k
  const float* k;
  float A, B, e, ei, et;
  bool clamp01;
  bool btdf;              // brdfToBtdf (Reflection.hs:188-195): wi mirrored to the other hemisphere
};
struct Bsdf { int n; BxDF b[2]; LC cs; V3 p, ng; };

// The lobe bs.b[second ? 1 : 0], selected field by field: a select of the two array elements'
// addresses kept the whole lobe array in scratch memory (112 B per lane in the two-lobe profiles).
DEV BxDF pick_lobe(const Bsdf& bs, bool second) {
  const BxDF& a = bs.b[0];
  const BxDF& b = bs.b[1];
  BxDF r;
  r.kind = second ? b.kind : a.kind; r.flags = second ? b.flags : a.flags; r.fr = second ? b.fr : a.fr;
  r.r = second ? b.r : a.r; r.eta = second ? b.eta : a.eta; r.k = second ? b.k : a.k;
  r.A = second ? b.A : a.A; r.B = second ? b.B : a.B; r.e = second ? b.e : a.e;
  r.ei = second ? b.ei : a.ei; r.et = second ? b.et : a.et;
  r.clamp01 = second ? b.clamp01 : a.clamp01; r.btdf = second ? b.btdf : a.btdf;
  return r;
}

DEV Sp refl(const BxDF& b) {
  if (!b.r) return sconst(1.f);
  Sp s = sload(b.r);
  return b.clamp01 ? sclamp01(s) : s;
}
DEV float cos_t(V3 w) { return w.z; }
DEV float abs_cos_t(V3 w) { return fabsf(w.z); }
DEV float sin_t2(V3 w) { return hmax(0.f, 1.f - w.z * w.z); }
DEV float sin_t(V3 w) { return sqrtf(sin_t2(w)); }
DEV float cos_phi(V3 w) { float s = sin_t(w); return s == 0.f ? 1.f : clampf(w.x / s, -1.f, 1.f); }
DEV float sin_phi(V3 w) { float s = sin_t(w); return s == 0.f ? 0.f : clampf(w.y / s, -1.f, 1.f); }
DEV bool same_hemi(V3 a, V3 b) { return a.z * b.z > 0.f; }

DEV float fr_diel_scalar(float etai, float etat, float cosi) {                         // Fresnel.hs:21-56
  float c = hmax(0.f, 1.f - cosi * cosi);
  float costp = cosi > 0.f ? c / (etat * etat) : c * (etat * etat);
  float cost = sqrtf(1.f - clampf(costp, 0.f, 1.f));
  float ci = fabsf(cosi);
  float eta = etat / etai;
  float rpa_p = eta * ci;
  float rpa = (cost - rpa_p) / (cost + rpa_p);
  float rpe_p = eta * cost;
  float rpe = (ci - rpe_p) / (ci + rpe_p);
  return (rpa * rpa + rpe * rpe) * 0.5f;
}
DEV Sp fr_conductor(const float* eta, const float* k, float cosi) {                   // Fresnel.hs:58-70
  float ac = fabsf(cosi);
  Sp r;
  SP_LOOP {
    float e = eta[i], kk = k[i];
    float tmpF = e * e + kk * kk;
    float ec2 = e * (2.f * ac);
    float tmp = (e * e + kk * kk) * (ac * ac);
    float c2 = ac * ac;
    float rper2 = (tmpF - ec2 + c2) / (tmpF + ec2 + c2);
    float rpar2 = (tmp - ec2 + 1.f) / (tmp + ec2 + 1.f);
    r.v[i] = (rper2 + rpar2) / 2.f;
  }
  return r;
}
template <uint32_t F>
DEV Sp fresnel(const BxDF& b, float c) {
  if (!(F & (FT_TWO_LOBES | FT_COND)) || b.fr == FR_NOOP) return sconst(1.f);
  if (!(F & FT_COND) || b.fr == FR_DIEL) return sconst(fr_diel_scalar(b.ei, b.et, c));
  return fr_conductor(b.eta, b.k, c);
}

// Blinn's D and pdf share |cos theta_h| ^ e (Microfacet.hs:146-147, 194-195): for one direction
// pair the evaluation and the pdf of the same lobe see the same half vector (wo + wi), so a caller
// that needs both passes the power from one to the other (dp; NaN = not computed)
DEV float blinn_pow(float e, V3 wh) { return bcr::powf(abs_cos_t(wh), e); }
DEV float blinn_pdf_p(float e, float pw) { return (e + 1.f) * pw * INV_TWO_PI; }
DEV float blinn_D_p(float e, float pw) { return (e + 2.f) * INV_TWO_PI * pw; }
DEV float mf_G(V3 wo, V3 wi, V3 wh) {                                                              // :113-120
  float nwh = abs_cos_t(wh), nwo = abs_cos_t(wo), nwi = abs_cos_t(wi), wowh = fabsf(dot(wo, wh));
  return hmin(1.f, hmin(2.f * nwh * nwo / wowh, 2.f * nwh * nwi / wowh));
}

// Anisotropic distribution (Microfacet.hs:136-192)
DEV float aniso_pdf(float ex, float ey, V3 wh) {                                                   // :140-144
  float costh = abs_cos_t(wh);
  float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / hmax(0.f, 1.f - costh * costh);
  return sqrtf((ex + 1.f) * (ey + 1.f)) * INV_TWO_PI * bcr::powf(costh, e);
}
DEV float aniso_D(float ex, float ey, V3 wh) {                                                     // :185-192
  float costh = abs_cos_t(wh);
  float d = 1.f - costh * costh;
  if (d == 0.f) return 0.f;
  float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / d;
  return sqrtf((ex + 2.f) * (ey + 2.f)) * INV_TWO_PI * bcr::powf(costh, e);
}
DEV void aniso_quadrant(float ex, float ey, float u1p, float u2, float* p, float* c) {             // smpFirstQuadrand
  *p = ex == ey ? PI * u1p * 0.5f : bcr::atanf(sqrtf((ex + 1.f) / (ey + 1.f)) * bcr::tanf(PI * u1p * 0.5f));
  const bcr::SinCos sc = bcr::sincosf(*p);
  const float cp = sc.c, sp = sc.s;
  *c = bcr::powf(u2, 1.f / (ex * cp * cp + ey * sp * sp + 1.f));
}
DEV V3 aniso_sample(float ex, float ey, float u1, float u2, float* pdf) {                         // :151-172
  float p, cost, phi;
  if (u1 < 0.25f) { aniso_quadrant(ex, ey, 4.f * u1, u2, &p, &cost); phi = p; }
  else if (u1 < 0.5f) { aniso_quadrant(ex, ey, 4.f * (0.5f - u1), u2, &p, &cost); phi = PI - p; }
  else if (u1 < 0.75f) { aniso_quadrant(ex, ey, 4.f * (u1 - 0.5f), u2, &p, &cost); phi = p + PI; }
  else { aniso_quadrant(ex, ey, 4.f * (1.f - u1), u2, &p, &cost); phi = TWO_PI - p; }
  float sint = sqrtf(hmax(0.f, 1.f - cost * cost));
  const bcr::SinCos sc = bcr::sincosf(phi);
  V3 wh = mk(sint * sc.c, sint * sc.s, cost);                                                                 // sphericalDirection
  float ds = 1.f - cost * cost;
  float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / ds;
  float f = INV_TWO_PI * bcr::powf(cost, e);
  *pdf = sqrtf((ex + 1.f) * (ey + 1.f)) * f;
  return wh;
}
DEV V3 fblend_half(V3 wo, V3 wi) { V3 h = normalize(wi + wo); return h.z < 0.f ? -h : h; }
// mkFresnelBlend's e wo wi (Microfacet.hs:64-84): the |cos| factor rides on wo (costo)
DEV Sp fblend_eval(const BxDF& b, V3 wo, V3 wi) {
  float costi = abs_cos_t(wi), costo = abs_cos_t(wo);
  const Sp rd = sload(b.r), rs = sload(b.eta);
  Sp a = sconst(1.f);
  if (b.B > 0.f) {                                                                                // absorption
    const float x = -(b.B * (costi + costo) / (costi * costo));
    const Sp ra = sload(b.k);
    SP_LOOP a.v[i] = bcr::expf(ra.v[i] * x);
  }
  const float wd = (costo * 28.f / 23.f * PI) * (1.f - bcr::powf(1.f - 0.5f * costi, 5.f)) * (1.f - bcr::powf(1.f - 0.5f * costo, 5.f));
  V3 wh = fblend_half(wo, wi);
  float costih = fabsf(dot(wi, wh));
  const float ws = aniso_D(b.e, b.A, wh) * costo / (4.f * costih * hmax(costi, costo));
  const float sk = bcr::powf(1.f - costih, 5.f);
  Sp r;
  SP_LOOP {
    const float diff = a.v[i] * rd.v[i] * (1.f - rs.v[i]) * wd;
    const float schlick = rs.v[i] + (1.f - rs.v[i]) * sk;
    r.v[i] = diff + schlick * ws;
  }
  return r;
}

DEV float oren_factor(const BxDF& b, V3 wo, V3 wi) {                                  // Diffuse.hs:53-65
  float sinti = sin_t(wi), sinto = sin_t(wo);
  float sina, tanb;
  if (abs_cos_t(wi) > abs_cos_t(wo)) { sina = sinto; tanb = sinti / abs_cos_t(wi); }
  else { sina = sinti; tanb = sinto / abs_cos_t(wo); }
  float maxcos = 0.f;
  if (sinti > 1e-4f && sinto > 1e-4f) {
    float sinpi = sin_phi(wi), cospi = cos_phi(wi), sinpo = sin_phi(wo), cospo = cos_phi(wo);
    maxcos = hmax(0.f, cospi * cospo + sinpi * sinpo);
  }
  return b.A + b.B * maxcos * sina * tanb;
}

// bxdfEval with the |cos| of the FIRST argument (evalBsdf False calls it as (wi, wo): trap T7)
template <uint32_t F>
DEV Sp bxdf_eval(const BxDF& b, V3 wo, V3 wi, float* dp = nullptr) {
  if ((F & FT_TRANSMATTE) && b.btdf) wi.z = -wi.z;                                   // e wo wi = bxdfEval brdf wo (otherHemisphere wi)
  if ((F & FT_DIFFUSE) && b.kind == K_LAMB) return sscale(refl(b), INV_PI * abs_cos_t(wo));
  if ((F & FT_OREN) && b.kind == K_OREN) return sscale(sscale(refl(b), oren_factor(b, wo, wi)), INV_PI * abs_cos_t(wo));
  if ((F & FT_MICRO) && b.kind == K_MICRO) {
    float costo = abs_cos_t(wo), costi = abs_cos_t(wi);
    if (costi == 0.f || costo == 0.f) return sconst(0.f);
    V3 whp = wi + wo;
    if (whp.x == 0.f && whp.y == 0.f && whp.z == 0.f) return sconst(0.f);
    V3 wh = normalize(whp);
    if (cos_t(wh) < 0.f) return sconst(0.f);
    float costh = dot(wi, wh);
    const float pw = blinn_pow(b.e, wh);
    if (dp) *dp = pw;
    float x = blinn_D_p(b.e, pw) * mf_G(wo, wi, wh) / (4.f * costi);
    return sscale(refl(b) * fresnel<F>(b, costh), x);
  }
  if ((F & FT_SUBSTRATE) && b.kind == K_FBLEND) return fblend_eval(b, wo, wi);
  return sconst(0.f);
}
template <uint32_t F>
DEV float bxdf_pdf(const BxDF& b, V3 wo, V3 wi, float dp = __builtin_nanf("")) {
  if ((F & FT_TRANSMATTE) && b.btdf) wi.z = -wi.z;
  if ((F & FT_DIFFUSE) && (b.kind == K_LAMB || b.kind == K_OREN)) return same_hemi(wo, wi) ? INV_PI * abs_cos_t(wi) : 0.f;
  if ((F & FT_MICRO) && b.kind == K_MICRO) {
    V3 whp = wo + wi;
    if (sqlen(whp) == 0.f) return 0.f;
    V3 wh = normalize(whp);
    if (cos_t(wh) < 0.f) return 0.f;
    const float pw = dp == dp ? dp : blinn_pow(b.e, wh);              // shared with bxdf_eval
    return blinn_pdf_p(b.e, pw) / (4.f * fabsf(dot(wo, wh)));
  }
  if ((F & FT_SUBSTRATE) && b.kind == K_FBLEND) {                                      // Microfacet.hs:101-105
    if (!same_hemi(wo, wi)) return 0.f;
    V3 wh = fblend_half(wo, wi);
    return 0.5f * (abs_cos_t(wi) * INV_PI + aniso_pdf(b.e, b.A, wh) / (4.f * fabsf(dot(wo, wh))));
  }
  return 0.f;
}
// ADJ = bxdfSample True (the adjoint of photon paths, SPPM.hs:232): |cos wo / cos wi| on diffuse
// lobes, |cos wo| in the microfacet denominator, the adjoint transmission weight (Specular.hs:52-57)
template <uint32_t F, bool ADJ = false>
DEV Sp bxdf_sample(const BxDF& b, V3 wo, float u1, float u2, V3* wi, float* pdf) {
  if ((F & FT_DIFFUSE) && (b.kind == K_LAMB || b.kind == K_OREN)) {                                          // Diffuse.hs:14-22, 38-42
    V3 w = cosine_sample_hemisphere(u1, u2);
    if (wo.z < 0.f) w.z = -w.z;                                                       // toSameHemisphere
    const float flip = ((F & FT_TRANSMATTE) && b.btdf) ? -1.f : 1.f;                 // brdfToBtdf: (f, otherHemisphere wi, pdf)
    if (same_hemi(wo, w)) {
      *wi = mk(w.x, w.y, flip * w.z); *pdf = INV_PI * abs_cos_t(w);
      Sp fv = b.kind == K_LAMB ? refl(b) : sscale(refl(b), oren_factor(b, wo, w));
      return ADJ ? sscale(fv, fabsf(cos_t(wo) / cos_t(w))) : fv;
    }
    V3 w0 = b.kind == K_LAMB ? wo : w;
    *wi = mk(w0.x, w0.y, flip * w0.z); *pdf = 0.f;
    return sconst(0.f);
  }
  if ((F & FT_MICRO) && b.kind == K_MICRO) {                                            // Microfacet.hs:42-54
    float cost = bcr::powf(u1, 1.f / (b.e + 1.f));
    float sint = sqrtf(hmax(0.f, 1.f - cost * cost));
    float phi = u2 * 2.f * PI;
    const bcr::SinCos sc = bcr::sincosf(phi);
    V3 whp = mk(sint * sc.c, sint * sc.s, cost);
    float f = bcr::powf(cost, b.e) * INV_TWO_PI;
    float d = (b.e + 2.f) * f, p = (b.e + 1.f) * f;
    V3 wh = cos_t(whp) < 0.f ? -whp : whp;
    V3 w = sm(2.f * dot(wo, wh), wh) - wo;
    float costH = dot(wo, wh);
    if (!same_hemi(wo, w)) { *wi = wo; *pdf = 0.f; return sconst(0.f); }
    float fact = d * fabsf(costH) / p * mf_G(wo, w, wh);
    Sp fp = refl(b) * fresnel<F>(b, costH);
    *wi = w; *pdf = p / (4.f * fabsf(costH));
    return sscale(fp, fact / abs_cos_t(ADJ ? wo : w));
  }
  if ((F & FT_SUBSTRATE) && b.kind == K_FBLEND) {                                      // Microfacet.hs:86-99
    float pp;
    V3 wh, w;
    if (u1 < 0.5f) {
      w = cosine_sample_hemisphere(u1 * 2.f, u2);
      if (wo.z < 0.f) w.z = -w.z;                                                      // toSameHemisphere
      wh = fblend_half(wo, w);
      pp = aniso_pdf(b.e, b.A, wh);
    } else {
      wh = aniso_sample(b.e, b.A, 2.f * (u1 - 0.5f), u2, &pp);
      w = sm(2.f * dot(wo, wh), wh) - wo;
    }
    *wi = w;
    if (pp == 0.f) { *pdf = 0.f; return sconst(0.f); }
    float p = 0.5f * (abs_cos_t(w) * INV_PI + pp / (4.f * fabsf(dot(wo, wh))));
    *pdf = p;
    return sscale(ADJ ? fblend_eval(b, w, wo) : fblend_eval(b, wo, w), 1.f / p);
  }
  if ((F & FT_SREFL) && b.kind == K_SREFL) {                              // Specular.hs:11-26
    *wi = mk(-wo.x, -wo.y, wo.z); *pdf = 1.f;
    return refl(b) * fresnel<F>(b, cos_t(wo));
  }
  if (!(F & FT_GLASS) || b.kind != K_STRANS) { *wi = wo; *pdf = 0.f; return sconst(0.f); }
  // K_STRANS (Specular.hs:28-57)
  bool entering = cos_t(wo) > 0.f;
  float ei = entering ? b.ei : b.et, et = entering ? b.et : b.ei;
  float sini2 = sin_t2(wo);
  float eta = ei / et, eta2 = eta * eta;
  float sint2 = eta2 * sini2;
  if (sint2 >= 1.f) { *wi = wo; *pdf = 0.f; return sconst(0.f); }
  float c = sqrtf(hmax(0.f, 1.f - sint2));
  float cost = entering ? -c : c;
  *wi = mk(eta * (-wo.x), eta * (-wo.y), cost);
  float fr = fr_diel_scalar(ei, et, ADJ ? cos_t(wo) : cost);
  Sp t = refl(b);
  Sp fp;
  SP_LOOP fp.v[i] = (1.f - fr) * t.v[i];
  *pdf = 1.f;
  return ADJ ? sscale(fp, fabsf(cos_t(wo) / cost)) : sscale(fp, eta2);
}

DEV float fix_exponent(float e) { return (e > 10000.f || __builtin_isnan(e)) ? 10000.f : e; }

// Scalar texture at the shading point (pScalarTexture, MaterialParser.hs:115-156): a chain of
// scaleTexture a s (Texture.hs:185) over a constant, fbm or perlin leaf (Texture.hs:340-385) on
// identityMapping3d (transPoint w2t p, :152-156).  The chain is unwound innermost-first, so each
// a + s * t is formed in the reference's order.
template <uint32_t F>
DEV float eval_stex(const DevScene& S, int ti, V3 p, float du, float dv) {
  float ca[BLING_STEX_MAX_SCALE], cs[BLING_STEX_MAX_SCALE];
  int n = 0;
  for (;;) {                     // the loader bounds a scale chain by BLING_STEX_MAX_SCALE
    const bling_scalar_texture& t = gen(S.stex[ti]);
    if (t.kind != BLING_STEX_SCALE || n == BLING_STEX_MAX_SCALE) break;
    ca[n] = t.a; cs[n] = t.s; ++n;
    ti = t.child;
  }
  const bling_scalar_texture& t = gen(S.stex[ti]);
  float v;
  if (t.kind == BLING_STEX_CONST) v = t.value;
  else if ((F & FT_PROCTEX) && t.kind == BLING_STEX_IMAGE) {        // imageTexture of a Y8 map (Texture.hs:103-108, 128-129)
    const bling_image& im = gen(S.images[t.child]);
    float s, tt;
    bimgtex::map2d(t.octaves, t.w2t, p.x, p.y, p.z, du, dv, &s, &tt);
    v = im.texels[bimgtex::texel(im.width, im.height, s, tt)];
  } else if ((F & FT_PROCTEX) && t.kind == BLING_STEX_CRYSTAL) {      // quasiCrystal (Texture.hs:317-338)
    const float* m = t.w2t;
    const float x = (p.x * m[0] + p.y * m[1] + p.z * m[2]) + m[6];  // planarMapping
    const float y = (p.x * m[3] + p.y * m[4] + p.z * m[5]) + m[7];
    float s = 0.f;
    for (int k = 0; k < t.octaves; ++k) {
      const bling_scalar_texture& w = gen(S.stex[t.child + k]);     // (cos th, sin th), host libm
      s = s + (bcr::cosf(w.a * x + w.s * y) + 1.f) / 2.f;
    }
    const float kf = truncf(s);
    float fr = s - kf;                                              // properFraction, then wrap
    long long k = (long long)kf;
    if (fr < 0.f) { k = k - 1; fr = 1.f + fr; }
    v = (k & 1) ? 1.f - fr : fr;
  } else {
    const V3 q = xpoint(t.w2t, p);
    if ((F & FT_PROCTEX) && t.kind == BLING_STEX_CELLNOISE) v = bcell::cell_noise(t.octaves, q.x, q.y, q.z);
    else v = t.kind == BLING_STEX_FBM ? bperlin::fbm(t.octaves, t.omega, q.x, q.y, q.z) : bperlin::perlin3d(q.x, q.y, q.z);
  }
  for (int k = n - 1; k >= 0; --k) v = ca[k] + cs[k] * v;
  return v;
}

// Material closures (Material.hs:32-96) evaluated at the shading DG
// bump (Reflection.hs:347-377): displacement d at p, p + du dpdu and p + dv dpdv (du = dv = 0.01);
// dpdu' = dpdu + ((d_u - d) / du) n, dpdv' likewise, n' = faceForward (normalize (dpdu' x dpdv')) ng.
// The shifted DGs carry u + du / v + dv for uv-mapped (image) displacement textures; their shifted
// normals feed no texture kind.
template <uint32_t F>
DEV DG bump_dg(const DevScene& S, int ti, const DG& dgg, const DG& dgs) {
  const float du = 0.01f, dv = 0.01f;
  const float uDisp = eval_stex<F>(S, ti, dgs.p + sm(du, dgs.dpdu), dgs.u + du, dgs.v);
  const float vDisp = eval_stex<F>(S, ti, dgs.p + sm(dv, dgs.dpdv), dgs.u, dgs.v + dv);
  const float disp = eval_stex<F>(S, ti, dgs.p, dgs.u, dgs.v);
  const float vscale = (vDisp - disp) / dv;
  const V3 dpdv = dgs.dpdv + sm(vscale, dgs.n);
  const float uscale = (uDisp - disp) / du;
  const V3 dpdu = dgs.dpdu + sm(uscale, dgs.n);
  const V3 nn1 = normalize(cross(dpdu, dpdv));
  DG b = dgs;
  b.n = dot(nn1, dgg.n) < 0.f ? -nn1 : nn1;                                 // faceForward nn' (dgN dgg)
  b.dpdu = dpdu; b.dpdv = dpdv;
  return b;
}

// A material's spectrum texture at the shading DG.  Stored spectra (constant, graphPaper) come back
// as pointers into S.textures; the computed kinds of FT_PROCTEX scenes (spectrumBlend, gradient,
// Texture.hs:135-145, 239-250) are formed into tmp (16 floats of the caller's), checkerBoard
// (:215-219) selects a stored child.  Same operations and order as the oracle's eval_spectrum.
template <uint32_t F>
DEV const float* eval_spectrum(const DevScene& S, int ti, const DG& dg, float* tmp) {
  if (F & FT_PROCTEX) {
    const bling_texture& t = gen(S.textures[ti]);
    if (t.kind == BLING_TEX_BLEND) {
      const float* v1 = eval_texture<F>(S, t.tex1, dg.u, dg.v);
      const float* v2 = eval_texture<F>(S, t.tex2, dg.u, dg.v);
      const float x = eval_stex<F>(S, t.stex, dg.p, dg.u, dg.v);
      if (x <= 0.f) return v1;
      if (x >= 1.f) return v2;
      const float y = 1.f - x;
      SP_LOOP tmp[i] = v1[i] * y + v2[i] * x;
      return tmp;
    }
    if (t.kind == BLING_TEX_GRADIENT) {
      const float f = eval_stex<F>(S, t.stex, dg.p, dg.u, dg.v);
      const int n = t.tex2;
      const bling_texture* st = gen(S.textures) + t.tex1;
      if (f <= st[0].line_width) return st[0].value;
      if (f >= st[n - 1].line_width) return st[n - 1].value;
      int idx = 1;                                                          // findIndex ((> f) . fst)
      while (idx < n - 1 && !(st[idx].line_width > f)) ++idx;
      const float p0 = st[idx - 1].line_width;
      const float w = (f - p0) / (st[idx].line_width - p0);
      const float y = 1.f - w;
      const float* c0 = st[idx - 1].value;
      const float* c1 = st[idx].value;
      SP_LOOP tmp[i] = c0[i] * y + c1[i] * w;
      return tmp;
    }
    if (t.kind == BLING_TEX_CHECKER) {
      const long long s = (long long)floorf(dg.p.x * t.uv_map[0]) + (long long)floorf(dg.p.y * t.uv_map[1]) +
                          (long long)floorf(dg.p.z * t.uv_map[2]);
      return eval_texture<F>(S, (s & 1) == 0 ? t.tex1 : t.tex2, dg.u, dg.v);
    }
    if (t.kind == BLING_TEX_IMAGE) {                                        // imageTexture (Texture.hs:96-101, 128-129)
      const bling_image& im = gen(S.images[t.tex1]);
      float s, tt;
      bimgtex::map2d(t.tex2, t.tex2 == BLING_MAP_UV ? t.uv_map : t.value, dg.p.x, dg.p.y, dg.p.z, dg.u, dg.v, &s, &tt);
      return im.texels + 16 * bimgtex::texel(im.width, im.height, s, tt);
    }
  }
  return eval_texture<F>(S, ti, dg.u, dg.v);
}

// tmp: 32 floats of the caller's that hold computed spectra (FT_PROCTEX profiles) while the Bsdf lives
template <uint32_t F>
DEV Bsdf make_bsdf(const DevScene& S, int mi, const DG& dgg, const DG& dgs_in, float* tmp = nullptr) {
  const int bump_tex = (F & FT_BUMP) ? gen(S.materials[mi]).stex[3] : -1;
  const DG dgs = bump_tex >= 0 ? bump_dg<F>(S, bump_tex, dgg, dgs_in) : dgs_in;     // bumpMapped (Reflection.hs:344-345)
  Bsdf bs;
  bs.n = 0;
  V3 nn = dgs.n, sn = normalize(dgs.dpdu);
  bs.cs = LC{sn, cross(nn, sn), nn};
  bs.p = dgs.p;
  bs.ng = dgg.n;
  const bling_material& m = gen(S.materials[mi]);
  BxDF z{};
  z.r = nullptr; z.eta = nullptr; z.k = nullptr; z.clamp01 = false; z.btdf = false;
  // the lobes go into bs.b once, after the material chain: per-branch stores into the two array
  // slots were merged by the compiler into stores through a phi'd address, which kept the whole
  // Bsdf in scratch memory (112 B per lane in the two-lobe profiles)
  BxDF l0 = z, l1 = z;
  int n = 0;
  if ((F & FT_MATTE) && m.kind == BLING_MAT_MATTE) {
    BxDF b = z;
    b.r = eval_spectrum<F>(S, m.tex[0], dgs, tmp + 0);
    b.flags = F_REFL | F_DIFF;
    float s = m.scalar[0];
    if (s == 0.f) b.kind = K_LAMB;
    else {
      b.kind = K_OREN;
      float sg = clampf(s, 0.f, 1.f), sig2 = sg * sg;
      b.A = 1.f - (sig2 / (2.f * (sig2 + 0.33f)));
      b.B = 0.45f * sig2 / (sig2 + 0.09f);
    }
    l0 = b; n = 1;
  } else if ((F & FT_PLASTIC) && m.kind == BLING_MAT_PLASTIC) {
    BxDF d = z; d.kind = K_LAMB; d.flags = F_REFL | F_DIFF; d.r = eval_spectrum<F>(S, m.tex[0], dgs, tmp + 0);
    BxDF g = z; g.kind = K_MICRO; g.flags = F_REFL | F_GLOSSY; g.r = eval_spectrum<F>(S, m.tex[1], dgs, tmp + 16);
    g.e = fix_exponent(1.f / m.scalar[0]); g.fr = FR_DIEL; g.ei = 1.0f; g.et = 1.5f;
    l0 = d; l1 = g; n = 2;
  } else if ((F & FT_GLASS) && m.kind == BLING_MAT_GLASS) {
    float ior = m.scalar[0];
    BxDF rf = z; rf.kind = K_SREFL; rf.flags = F_REFL | F_SPEC; rf.r = eval_spectrum<F>(S, m.tex[0], dgs, tmp + 0);
    rf.clamp01 = true; rf.fr = FR_DIEL; rf.ei = 1.f; rf.et = ior;
    BxDF tr = z; tr.kind = K_STRANS; tr.flags = F_TRANS | F_SPEC; tr.r = eval_spectrum<F>(S, m.tex[1], dgs, tmp + 16);
    tr.clamp01 = true; tr.ei = 1.f; tr.et = ior;
    l0 = rf; l1 = tr; n = 2;
  } else if ((F & FT_METAL) && m.kind == BLING_MAT_METAL) {
    BxDF g = z; g.kind = K_MICRO; g.flags = F_REFL | F_GLOSSY; g.r = nullptr;
    g.e = fix_exponent(1.f / m.scalar[0]); g.fr = FR_COND;
    g.eta = eval_spectrum<F>(S, m.tex[0], dgs, tmp + 0); g.k = eval_spectrum<F>(S, m.tex[1], dgs, tmp + 16);
    l0 = g; n = 1;
  } else if ((F & FT_TRANSMATTE) && m.kind == BLING_MAT_TRANSMATTE) {
    // translucentMatte (Material.hs:43-53): r and t folded on the host (bling_scene.h)
    BxDF rf = z, tr = z;
    rf.r = gen(S.textures[m.tex[0]]).value; tr.r = gen(S.textures[m.tex[1]]).value;
    float s = m.scalar[0];
    if (s == 0.f) { rf.kind = K_LAMB; tr.kind = K_LAMB; }
    else {
      float sg = clampf(s, 0.f, 1.f), sig2 = sg * sg;
      rf.kind = K_OREN; rf.A = 1.f - (sig2 / (2.f * (sig2 + 0.33f))); rf.B = 0.45f * sig2 / (sig2 + 0.09f);
      tr.kind = K_OREN; tr.A = rf.A; tr.B = rf.B;
    }
    rf.flags = F_REFL | F_DIFF;
    tr.flags = F_TRANS | F_DIFF; tr.btdf = true;                                       // bxdfTypeFlip (Refl|Trans)
    l0 = rf; l1 = tr; n = 2;
  } else if ((F & FT_SHINYMETAL) && m.kind == BLING_MAT_SHINYMETAL) {
    // mkShinyMetal (Material.hs:98-109): conductor spectra folded on the host
    BxDF g = z; g.kind = K_MICRO; g.flags = F_REFL | F_GLOSSY; g.r = nullptr;
    g.e = fix_exponent(1.f / m.scalar[0]); g.fr = FR_COND;
    g.eta = gen(S.textures[m.tex[0]]).value; g.k = gen(S.textures[m.tex[1]]).value;
    BxDF sp = z; sp.kind = K_SREFL; sp.flags = F_REFL | F_SPEC; sp.r = nullptr; sp.fr = FR_COND;
    sp.eta = gen(S.textures[m.tex[2]]).value; sp.k = gen(S.textures[m.tex[3]]).value;
    l0 = g; l1 = sp; n = 2;
  } else if ((F & FT_SUBSTRATE) && m.kind == BLING_MAT_SUBSTRATE) {
    // mkSubstrate (Material.hs:111-128): one FresnelBlend lobe, spectra and exponents folded on the host
    BxDF fb = z; fb.kind = K_FBLEND; fb.flags = F_REFL | F_GLOSSY;
    fb.r = gen(S.textures[m.tex[0]]).value; fb.eta = gen(S.textures[m.tex[1]]).value; fb.k = gen(S.textures[m.tex[2]]).value;
    fb.e = m.scalar[0]; fb.A = m.scalar[1]; fb.B = m.scalar[2];
    // per-hit parameters: u / v = max 0 (t dgs), exponents fixExponent (1 / u); depth = td dgs
    if (m.stex[0] >= 0) { const float u = eval_stex<F>(S, m.stex[0], dgs.p, dgs.u, dgs.v); fb.e = fix_exponent(1.f / (0.f <= u ? u : 0.f)); }
    if (m.stex[1] >= 0) { const float v = eval_stex<F>(S, m.stex[1], dgs.p, dgs.u, dgs.v); fb.A = fix_exponent(1.f / (0.f <= v ? v : 0.f)); }
    if (m.stex[2] >= 0) fb.B = eval_stex<F>(S, m.stex[2], dgs.p, dgs.u, dgs.v);
    l0 = fb; n = 1;
  } else if ((F & FT_MIRROR) && m.kind == BLING_MAT_MIRROR) {
    BxDF rf = z; rf.kind = K_SREFL; rf.flags = F_REFL | F_SPEC; rf.r = eval_spectrum<F>(S, m.tex[0], dgs, tmp + 0);
    rf.clamp01 = true; rf.fr = FR_NOOP;
    l0 = rf; n = 1;
  }
  bs.b[0] = l0; bs.b[1] = l1; bs.n = n;
  return bs;
}

DEV bool has_flag(const BxDF& b, int f) { return (b.flags & f) == f; }

template <uint32_t F>
constexpr int max_lobes() { return (F & FT_TWO_LOBES) ? 2 : 1; }

// dps: the microfacet powers eval_bsdf computed for the same direction pair (optional)
template <uint32_t F>
DEV float bsdf_pdf(const Bsdf& bs, V3 woW, V3 wiW, const float* dps = nullptr) {     // Reflection.hs:251-257
  if (bs.n == 0) return 0.f;
  V3 wo = world_to_local(bs.cs, woW), wi = world_to_local(bs.cs, wiW);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < max_lobes<F>(); ++i)
    if (i < bs.n) s = s + bxdf_pdf<F>(bs.b[i], wo, wi, dps ? dps[i] : __builtin_nanf(""));
  return s / (float)bs.n;
}
template <uint32_t F>
DEV Sp eval_bsdf(const Bsdf& bs, V3 woW, V3 wiW, float* dps = nullptr) {             // Reflection.hs:318-332
  float cosWo = dot(woW, bs.ng);
  float side = dot(wiW, bs.ng) / cosWo;
  if (side == 0.f) return sconst(0.f);
  if (fabsf(cosWo) < 1e-5f) return sconst(0.f);
  int flt = side < 0.f ? F_TRANS : F_REFL;
  V3 wo = world_to_local(bs.cs, woW), wi = world_to_local(bs.cs, wiW);
  Sp f = sconst(0.f);
#pragma unroll
  for (int i = 0; i < max_lobes<F>(); ++i)
    if (i < bs.n && has_flag(bs.b[i], flt)) f = f + bxdf_eval<F>(bs.b[i], wi, wo, dps ? dps + i : nullptr);
  return f;
}

// sampleBsdf'' (Reflection.hs:278-316).  Returns the pdf; on pdf == 0 ("no sample") f is black.
// Out-parameters with one exit keep the 16-band f in registers (a returned aggregate with several
// early returns was materialised in scratch).
// ADJ = sampleAdjBsdf (the photon direction): the sampled lobe adjoint, the other lobes evaluated
// unflipped, every result scaled by |sideTest| (fAdj, Reflection.hs:299-316)
template <uint32_t F, bool ADJ = false>
DEV float sample_bsdf(const Bsdf& bs, V3 woW, float uc, float u1, float u2, Sp& f, V3& wiW, int& flags) {
  float pdf = 0.f;
  f = sconst(0.f);
  wiW = mk(0.f, 1.f, 0.f);
  flags = F_REFL | F_DIFF;
  if (bs.n != 0) {
    V3 wo = world_to_local(bs.cs, woW);
    int cntm = bs.n;
    float cntf = (float)cntm, invCnt = 1.f / cntf;
    int sNum = max(0, min(cntm - 1, (int)floorf(uc * cntf)));
    const BxDF b = max_lobes<F>() == 1 ? bs.b[0] : pick_lobe(bs, sNum != 0);
    V3 wi; float pdfp;
    Sp fs = bxdf_sample<F, ADJ>(b, wo, u1, u2, &wi, &pdfp);
    V3 w = local_to_world(bs.cs, wi);
    float side = dot(w, bs.ng) / dot(woW, bs.ng);
    int flt = side < 0.f ? F_TRANS : F_REFL;
    if (!(pdfp == 0.f) && !(side == 0.f) && has_flag(b, flt)) {
      flags = b.flags;
      wiW = w;
      if (has_flag(b, F_SPEC)) {
        pdf = pdfp * invCnt; f = sscale(fs, cntf);
      } else if (max_lobes<F>() == 1 || cntm == 1) {
        pdf = pdfp; f = fs;
      } else {
        float others = 0.f;
        Sp fo = sconst(0.f);
#pragma unroll
        for (int i = 0; i < max_lobes<F>(); ++i) {
          if (i >= bs.n || i == sNum) continue;
          float dp = __builtin_nanf("");
          if (has_flag(bs.b[i], flt)) fo = fo + (ADJ ? bxdf_eval<F>(bs.b[i], wo, wi) : bxdf_eval<F>(bs.b[i], wi, wo, &dp));
          others = others + bxdf_pdf<F>(bs.b[i], wo, wi, dp);
        }
        pdf = (pdfp + others) * invCnt;
        f = sscale(sscale(fs, pdfp) + fo, 1.f / pdf);
      }
      if (ADJ) f = sscale(f, fabsf(side));                          // fAdj of each case
    }
  }
  return pdf;
}

// ---- one diffuse lobe with a texture spectrum r: every f is (r * s1) * s2 ----
// The profiles whose materials are all matte (Lambertian or Oren-Nayar, Diffuse.hs:24-66) build a
// Bsdf of at most one lobe, so sampleBsdf's f is r * s1 and evalBsdf's f is 0 + (r * s1) * s2 for
// scalars s1, s2.  These mirror sample_bsdf / eval_bsdf for that case operation for operation and
// return the scalars, which k_shade stores instead of the 16-band candidates and k_resolve expands
// with the same multiplications (wavefront.h, "factored candidates").
// sampleBsdf'' (Reflection.hs:278-316) with one non-specular diffuse lobe: returns the pdf (0 = no
// sample) and f = r * s1.
template <uint32_t F>
DEV float sample_bsdf_diffuse1(const Bsdf& bs, V3 woW, float u1, float u2, float& s1, V3& wiW) {
  float pdf = 0.f;
  s1 = 0.f;
  wiW = mk(0.f, 1.f, 0.f);
  if (bs.n != 0) {
    const BxDF& b = bs.b[0];
    const V3 wo = world_to_local(bs.cs, woW);
    V3 w = cosine_sample_hemisphere(u1, u2);                                          // Diffuse.hs:14-22, 38-42
    if (wo.z < 0.f) w.z = -w.z;
    V3 wi;
    float pdfp, s;
    if (same_hemi(wo, w)) { wi = w; pdfp = INV_PI * abs_cos_t(w); s = b.kind == K_LAMB ? 1.f : oren_factor(b, wo, w); }
    else { wi = b.kind == K_LAMB ? wo : w; pdfp = 0.f; s = 0.f; }
    const V3 ww = local_to_world(bs.cs, wi);
    const float side = dot(ww, bs.ng) / dot(woW, bs.ng);
    const int flt = side < 0.f ? F_TRANS : F_REFL;
    if (!(pdfp == 0.f) && !(side == 0.f) && has_flag(b, flt)) { wiW = ww; pdf = pdfp; s1 = s; }
  }
  return pdf;
}
// evalBsdf (Reflection.hs:318-332) with one diffuse lobe: false = black, else f = 0 + (r * s1) * s2
template <uint32_t F>
DEV bool eval_bsdf_diffuse1(const Bsdf& bs, V3 woW, V3 wiW, float& s1, float& s2) {
  if (bs.n == 0) return false;
  const float cosWo = dot(woW, bs.ng);
  const float side = dot(wiW, bs.ng) / cosWo;
  if (side == 0.f) return false;
  if (fabsf(cosWo) < 1e-5f) return false;
  const int flt = side < 0.f ? F_TRANS : F_REFL;
  const BxDF& b = bs.b[0];
  if (!has_flag(b, flt)) return false;
  const V3 wo = world_to_local(bs.cs, woW), wi = world_to_local(bs.cs, wiW);
  // bxdf_eval(b, wi, wo): the |cos| of its first argument (trap T7)
  if (b.kind == K_LAMB) { s1 = INV_PI * abs_cos_t(wi); s2 = 1.f; }
  else { s1 = oren_factor(b, wi, wo); s2 = INV_PI * abs_cos_t(wi); }
  return true;
}
DEV Sp diffuse1_f(const float* r, float s1) { return r ? sscale(sload(r), s1) : sconst(s1); }
DEV Sp diffuse1_e(const float* r, float s1, float s2) {
  return sconst(0.f) + sscale(r ? sscale(sload(r), s1) : sconst(1.f * s1), s2);
}

// sampleBsdf' (Specular | side) bsdf wo 0.5 (0.5, 0.5) of DirectLighting's cont
// (DirectLighting.hs:47-57, Reflection.hs:278-316): bsm = the BxDFs whose type lies within the
// filter (bxdfMatches).  A type within {Specular, Reflection} or {Specular, Transmission} is a
// specular lobe, so the sampled lobe always takes the isSpecular branch (pdf' / n, n f).
// With uc, (u1, u2) from the sampler it is SPPM's followCam sample (SPPM.hs:89-103).
template <uint32_t F>
DEV float sample_bsdf_spec(const Bsdf& bs, V3 woW, int side_flag, float uc, float u1, float u2, Sp& f, V3& wiW) {
  const int filt = F_SPEC | side_flag;
  int cntm = 0, first = 0, second = 0;
#pragma unroll
  for (int i = 0; i < max_lobes<F>(); ++i)
    if (i < bs.n && (bs.b[i].flags & filt) == bs.b[i].flags) { if (cntm == 0) first = i; else second = i; ++cntm; }
  float pdf = 0.f;
  f = sconst(0.f);
  wiW = mk(0.f, 1.f, 0.f);
  if (cntm != 0) {
    const float cntf = (float)cntm;
    const int sIdx = max(0, min(cntm - 1, (int)floorf(uc * cntf)));
    const BxDF b = max_lobes<F>() == 1 ? bs.b[0] : pick_lobe(bs, (sIdx == 0 ? first : second) != 0);
    V3 wo = world_to_local(bs.cs, woW);
    V3 wi; float pdfp;
    Sp fs = bxdf_sample<F>(b, wo, u1, u2, &wi, &pdfp);
    V3 w = local_to_world(bs.cs, wi);
    float side = dot(w, bs.ng) / dot(woW, bs.ng);
    int flt = side < 0.f ? F_TRANS : F_REFL;
    if (!(pdfp == 0.f) && !(side == 0.f) && has_flag(b, flt)) {
      wiW = w;
      pdf = pdfp * (1.f / cntf);
      f = sscale(fs, cntf);
    }
  }
  return pdf;
}
template <uint32_t F>
DEV float sample_bsdf_spec(const Bsdf& bs, V3 woW, int side_flag, Sp& f, V3& wiW) {
  return sample_bsdf_spec<F>(bs, woW, side_flag, 0.5f, 0.5f, 0.5f, f, wiW);
}

// ================================================================ lights
// upper_bound (Montecarlo.hs:53-54) with the CDF's guide table (core.hip upload): the first index with cdf[i] >= u lies
// in [g[k], g[k + 1]] for k = floor(u kCdfGuide) (u kCdfGuide is exact: a power-of-two scale), so
// the search over that range returns exactly the whole-range search's index
DEV int upper_bound_guided(const float* cdf, int nv, float u, const uint32_t* g) {
  int lo = 0, hi = nv;
  if (u >= 0.f && u < 1.f) { const int k = (int)(u * (float)kCdfGuide); lo = (int)g[k]; hi = (int)g[k + 1]; }
  while (lo < hi) { int mid = (lo + hi) >> 1; if (cdf[mid] >= u) hi = mid; else lo = mid + 1; }
  int idx = lo < nv ? lo - 1 : nv - 1;
  idx = max(0, idx);
  return min(nv - 2, idx);
}
DEV float sample_c1d(const float* func, const float* cdf, float fi, int n, float u, float* pdf, int* off_out,
                     const uint32_t* guide) {
  int off = upper_bound_guided(cdf, n + 1, u, guide);
  *pdf = fi == 0.f ? 0.f : func[off] / fi;
  float du = (u - cdf[off]) / (cdf[off + 1] - cdf[off]);
  *off_out = off;
  return ((float)off + du) / (float)n;
}
DEV void sample_c2d(const bling_light& L, float u0, float u1, float* u, float* v, float* pdf) {
  int nu = L.dist_nu, nv = L.dist_nv, im, dummy;
  float pdf1, pdf0;
  // device layout (core.hip): each CDF buffer carries its guide tables behind the CDF values
  const uint32_t* mg = reinterpret_cast<const uint32_t*>(L.marg_cdf + nv + 1);
  const uint32_t* rg = reinterpret_cast<const uint32_t*>(L.dist_cdf + (size_t)(nu + 1) * nv);
  *v = sample_c1d(L.marg_func, L.marg_cdf, L.marg_func_int, nv, u1, &pdf1, &im, mg);
  *u = sample_c1d(L.dist_func + (size_t)im * nu, L.dist_cdf + (size_t)im * (nu + 1), L.dist_func_int[im], nu, u0, &pdf0,
                  &dummy, rg + (size_t)im * (kCdfGuide + 1));
  *pdf = pdf0 * pdf1;
}
DEV float pdf_d2d(const bling_light& L, float u, float v) {
  int nu = L.dist_nu, nv = L.dist_nv;
  int iu = max(0, min(nu - 1, (int)floorf(u * (float)nu)));
  int iv = max(0, min(nv - 1, (int)floorf(v * (float)nv)));
  if (L.marg_func_int * L.dist_func_int[iv] == 0.f) return 0.f;
  return (L.dist_func[(size_t)iv * nu + iu] * L.marg_func[iv]) / (L.dist_func_int[iv] * L.marg_func_int);
}
// skySpectrum + sunSpectrum (SunSky.hs:67-94) as bsky::sky_eval, with perez's light-constant
// denominators taken from the upload (host libm, like the oracle's per-call evaluation) and the
// cos of theta / gamma shared by the three Perez channels
DEV void sky_eval_dev(const bling_light& L, const float* den, float dx, float dy, float dz, float* out) {
  float sky[16];
  const float dzn = -dz;
  if (dzn < 1e-4f) {
    for (int i = 0; i < 16; ++i) sky[i] = 0.f;
  } else {
    const float theta = bcr::acosf(dzn);
    const float dd = dx * L.sun_dir_local[0] + dy * L.sun_dir_local[1] + dz * L.sun_dir_local[2];
    const float gamma = bcr::acosf(clampf(dd, -1.f, 1.f));
    const float csg = bcr::cosf(gamma), ct = bcr::cosf(theta);
    auto perez = [&](const float* p, float lvz, float dn) {                         // SunSky.hs:81-86
      const float num = (1.f + p[0] * bcr::expf(p[1] / ct)) * (1.f + p[2] * bcr::expf(p[3] * gamma)) + p[4] * csg * csg;
      return lvz * num / dn;
    };
    const float x = perez(L.perez_x, L.zenith_x, den[0]);
    const float y = perez(L.perez_y, L.zenith_y, den[1]);
    const float yy = perez(L.perez_Y, L.zenith_Y, den[2]) * 1e-4f;
    float cx, cy, cz;
    bsky::chromaticity_to_xyz(x, y, &cx, &cy, &cz);
    bsky::xyz_to_spectrum(cx * yy / cy, yy, cz * yy / cy, sky);
  }
  const float d = L.sun_dir_local[0] * dx + L.sun_dir_local[1] * dy + (L.sun_dir_local[2] * -1.f) * dz;
  const bool sun = d > bsky::sun_theta_max2();
  for (int i = 0; i < 16; ++i) out[i] = sky[i] + (sun ? L.sun_radiance[i] : 0.f);
}
// The sky's radiance at image coordinates (u, v).  BLING_SKY_OUTLINE experiment builds make it one
// out-of-line function instead of a copy at each env_eval site.
#if defined(BLING_SKY_OUTLINE)
#define SKY_FN static __device__ __attribute__((noinline))
#else
#define SKY_FN DEV
#endif
// st, ct, cph, sph: sin / cos of th = v pi and of phi = u 2 pi (the reference's lookup recomputes
// them from (u, v); the light sample, which needs them for its direction too, passes its own)
SKY_FN Sp sky_trig(const bling_light& L, float st, float ct, float cph, float sph) {
  Sp s;
  const float* den = L.marg_cdf + L.dist_nv + 1 + kCdfGuide + 1;     // behind the marginal guide
  sky_eval_dev(L, den, st * cph, st * sph, ct, s.v);
  return s;
}
template <uint32_t F>
DEV Sp env_eval_trig(const bling_light& L, float u, float v, float st, float ct, float cph, float sph) {
  if ((F & FT_ENV_IMG) && L.env_kind == BLING_ENV_IMAGE)                     // rgbfToTexMap (IO/Bitmap.hs:22-29)
    return sload(L.env_texels + 16 * bimgtex::env_texel(L.env_w, L.env_h, u, v));
  if (!(F & FT_ENV_SKY) || L.env_kind == BLING_ENV_CONSTANT) return sload(L.env_const);
  return sky_trig(L, st, ct, cph, sph);
}
template <uint32_t F>
DEV Sp env_eval(const bling_light& L, float u, float v) {
  if ((F & FT_ENV_IMG) && L.env_kind == BLING_ENV_IMAGE)                     // rgbfToTexMap (IO/Bitmap.hs:22-29)
    return sload(L.env_texels + 16 * bimgtex::env_texel(L.env_w, L.env_h, u, v));
  if (!(F & FT_ENV_SKY) || L.env_kind == BLING_ENV_CONSTANT) return sload(L.env_const);
  const float phi = u * 2.f * PI, th = v * PI;
  const bcr::SinCos st = bcr::sincosf(th), sp = bcr::sincosf(phi);
  return sky_trig(L, st.s, st.c, sp.c, sp.s);
}
DEV void dir_to_uv(V3 w, float* u, float* v, float* sint) {
  float p = bcr::atan2f(w.y, w.x);
  if (p < 0.f) p = p + 2.f * PI;
  float th = bcr::acosf(hmax(-1.f, hmin(1.f, w.z)));
  *u = p / (2.f * PI);
  *v = th / PI;
  *sint = bcr::sinf(th);
}
template <uint32_t F>
DEV Sp light_le(const bling_light& L, V3 dir) {                                       // Light.hs:98-106
  if (!(F & FT_INF) || L.kind != BLING_LIGHT_INFINITE) return sconst(0.f);
  V3 wh = normalize(xvector(L.w2l, dir));
  float u, v, st;
  dir_to_uv(wh, &u, &v, &st);
  return env_eval<F>(L, u, v);
}

template <uint32_t F>
DEV bool shape_local_hit(const DevShape& s, const Ray& r, float* t, V3* n) {
  if ((F & FT_SHAPES2) && s.kind >= BLING_SHAPE_DISK) {
    if (!shape2_test(s, r, r.tmax, false, t)) return false;
    *n = shape2_normal(s, r, ray_at(r, *t));
    return true;
  }
  if (!(F & FT_NONQUAD) || s.kind == BLING_SHAPE_QUAD) {
    if (fabsf(r.d.z) < 1e-7f) return false;
    float tt = -(r.o.z) / r.d.z;
    if (tt < r.tmin || tt > r.tmax) return false;
    V3 p = ray_at(r, tt);
    if (fabsf(p.x) > s.params[0] || fabsf(p.y) > s.params[1]) return false;
    *t = tt;
    *n = normalize(cross(mk(s.params[0], 0.f, 0.f), mk(0.f, s.params[1], 0.f)));
    return true;
  }
  float rad = s.params[0];
  float a = sqlen(r.d), b = 2.f * dot(r.o, r.d), c = sqlen(r.o) - (rad * rad);
  float t1, t2;
  if (!solve_quadric(a, b, c, &t1, &t2)) return false;
  if (t1 > r.tmax || t2 < r.tmin) return false;
  float tt = t1 < r.tmin ? t2 : t1;
  if (tt > r.tmax) return false;
  *t = tt;
  // object-space DG normal of the sphere (Shape.hs:173-229)
  V3 p = ray_at(r, tt);
  const float thetaMin = PI, thetaMax = 0.f, phiMax = TWO_PI;
  float theta = bcr::acosf(clampf(p.z / rad, -1.f, 1.f));
  float zr = sqrtf(p.x * p.x + p.y * p.y), izr = 1.f / zr;
  V3 dpdu = mk(-(phiMax * p.y), phiMax * p.x, 0.f);
  V3 dpdv = vs(mk(p.z * (p.x * izr), p.z * (p.y * izr), -(rad * bcr::sinf(theta))), thetaMax - thetaMin);
  *n = normalize(cross(dpdu, dpdv));
  return true;
}
template <uint32_t F>
DEV float shape_area(const DevShape& s) {                                                // Shape.hs:314-328
  if ((F & FT_SHAPES2) && s.kind >= BLING_SHAPE_DISK) {
    const float* P = s.params;
    if (s.kind == BLING_SHAPE_DISK) return PI * (P[1] * P[1] - P[2] * P[2]);
    if (s.kind == BLING_SHAPE_CYLINDER) return 2.f * PI * P[0] * (P[2] - P[1]);
    const float h = P[3] - P[0], w = P[4] - P[1], l = P[5] - P[2];
    return 2.f * (h * w + h * l + w * l);
  }
  return (!(F & FT_NONQUAD) || s.kind == BLING_SHAPE_QUAD) ? 4.f * s.params[0] * s.params[1] : s.params[0] * s.params[0] * 4.f * PI;
}
// sampleShape' of a disk / cylinder / box (Shape.hs:384-403): object-space point and normal
DEV void shape2_sample(const DevShape& s, float u1, float u2, V3* ps, V3* ns) {
  const float* P = s.params;
  if (s.kind == BLING_SHAPE_DISK) {
    float r = lerpf(u1, P[2], P[1]), phi = lerpf(u2, 0.f, P[3]);
    const bcr::SinCos sc = bcr::sincosf(phi);
    *ps = mk(r * sc.c, r * sc.s, P[0]);
    *ns = mk(0.f, 0.f, -1.f);
    return;
  }
  if (s.kind == BLING_SHAPE_CYLINDER) {
    float z = lerpf(u1, P[1], P[2]), phi = lerpf(u2, 0.f, TWO_PI);
    const bcr::SinCos sc = bcr::sincosf(phi);
    *ps = mk(P[0] * sc.c, P[0] * sc.s, z);
    *ns = normalize(mk(ps->x, ps->y, 0.f));
    return;
  }
  // remapRand (Math.hs:113-121)
  int axis = min(2, (int)floorf(u1 * 3.f));
  float u1p = (u1 - (float)axis / 3.f) * 3.f;
  int nf = min(1, (int)floorf(u2 * 2.f));
  float u2p = (u2 - (float)nf / 2.f) * 2.f;
  float nv = (float)nf * 2.f - 1.f;
  *ns = mk(axis == 0 ? nv : 0.f, axis == 1 ? nv : 0.f, axis == 2 ? nv : 0.f);
  const int oa0 = (axis + 1) % 3, oa1 = (axis + 2) % 3;
  float q[3] = {nf == 0 ? P[0] : P[3], nf == 0 ? P[1] : P[4], nf == 0 ? P[2] : P[5]};
  q[oa1] = lerpf(u2p, P[oa1], P[3 + oa1]);
  q[oa0] = lerpf(u1p, P[oa0], P[3 + oa0]);
  *ps = mk(q[0], q[1], q[2]);
}
template <uint32_t F>
DEV float shape_pdf(const DevShape& s, V3 p, V3 wi) {                                 // Shape.hs:333-350
  if ((F & FT_SPHERE) && s.kind == BLING_SHAPE_SPHERE) {
    float r = s.params[0];
    if (!(sqlen(p) - r * r < 1e-4f)) return uniform_cone_pdf(sqrtf(hmax(0.f, 1.f - r * r / sqlen(p))));
  }
  Ray ray{p, wi, 1e-3f, INFINITY};
  float t; V3 n;
  if (!shape_local_hit<F>(s, ray, &t, &n)) return 0.f;
  float pd = sqlen(p - ray_at(ray, t)) / (fabsf(dot(n, -wi)) * shape_area<F>(s));
  return __builtin_isinf(pd) ? 0.f : pd;
}

// Light ln's record and a light's shape record; one-light profiles (dev_scene.h one_light) read
// light 0 and its shape through the constant address space with a wave-uniform address.
template <uint32_t F>
DEV const bling_light& light_rec(const DevScene& S, int ln) {
  if constexpr (one_light<F>()) { (void)ln; return *(const bling_light*)(cptr<bling_light>)S.lights; }
  else return gen(S.lights[ln]);
}
template <uint32_t F>
DEV const DevShape& light_shape(const DevScene& S, const bling_light& L) {
  if constexpr (one_light<F>()) return *(const DevShape*)((cptr<DevShape>)S.shapes + L.shape);
  else return gen(S.shapes[L.shape]);
}

struct LightSample { Sp li; V3 wi; Ray ray; float pdf; bool delta; };

// sample (Light.hs:122-160); nS = the shading normal (bsdfShadingNormal), used by directional lights
template <uint32_t F>
DEV LightSample light_sample(const DevScene& S, const bling_light& L, V3 pW, V3 nS, float eps, float u1, float u2) {
  LightSample ls;
  ls.delta = false;
  if ((F & FT_DELTA) && L.kind >= BLING_LIGHT_POINT) {
    const V3 v = mk(L.delta_vec[0], L.delta_vec[1], L.delta_vec[2]);
    ls.delta = true;
    ls.pdf = 1.f;
    if (L.kind == BLING_LIGHT_DIRECTIONAL) {                                          // Light.hs:143-145
      ls.li = sscale(sload(L.radiance), fabsf(dot(nS, v)));
      ls.wi = v;
      ls.ray = Ray{pW, v, eps, INFINITY};
    } else {                                                                          // Light.hs:147-150
      ls.li = sscale(sload(L.radiance), 1.f / sqlen(v - pW));
      ls.wi = normalize(v - pW);
      ls.ray = Ray{pW, v - pW, eps, INFINITY};      // unnormalised direction, no tmax: trap T19
    }
    return ls;
  }
  if (!(F & FT_INF) || L.kind == BLING_LIGHT_AREA) {                                 // Light.hs:152-160
    const DevShape& s = light_shape<F>(S, L);
    V3 p = xpoint(s.w2o, pW);
    V3 ps, ns;
    if ((F & FT_SHAPES2) && s.kind >= BLING_SHAPE_DISK) {
      shape2_sample(s, u1, u2, &ps, &ns);
    } else if (!(F & FT_NONQUAD) || s.kind == BLING_SHAPE_QUAD) {
      ps = mk(lerpf(u1, -s.params[0], s.params[0]), lerpf(u2, -s.params[1], s.params[1]), 0.f);
      ns = mk(0.f, 0.f, -1.f);                                                        // sampleShape' Quad (trap T6)
    } else {
      float r = s.params[0];
      if (sqlen(p) - r * r < 1e-4f) { V3 q = uniform_sample_sphere(u1, u2); ps = vs(q, r); ns = q; }
      else {
        V3 dn = normalize(-p);
        LC cs = coordinate_system(dn);
        float cosmax = sqrtf(hmax(0.f, 1.f - (r * r) / sqlen(p)));
        V3 dd = uniform_sample_cone(cs, cosmax, u1, u2);
        float t; V3 n;
        ps = shape_local_hit<F>(s, Ray{p, dd, 0.f, INFINITY}, &t, &n) ? ray_at(Ray{p, dd, 0.f, INFINITY}, t) : vs(dn, r);
        ns = normalize(ps);
      }
    }
    V3 wi = normalize(ps - p);
    ls.li = dot(ns, wi) < 0.f ? sload(L.radiance) : sconst(0.f);
    ls.wi = xvector(s.o2w, wi);
    ls.pdf = shape_pdf<F>(s, p, wi);
    ls.ray = Ray{xpoint(s.o2w, p), xvector(s.o2w, wi), eps, len(ps - p) - eps};
    return ls;
  }
  float u, v, mpdf;                                                                   // Light.hs:130-141
  sample_c2d(L, u1, u2, &u, &v, &mpdf);
  float th = v * PI, phi = u * 2.f * PI;
  const bcr::SinCos sct = bcr::sincosf(th);
  float sint = sct.s;
  if (mpdf == 0.f || sint == 0.f) {
    ls.li = sconst(0.f); ls.wi = mk(0.f, 1.f, 0.f); ls.pdf = 0.f;
    ls.ray = Ray{mk(0.f, 0.f, 0.f), mk(0.f, 1.f, 0.f), 0.f, 1.f};
    return ls;
  }
  // one sin / cos each for the radiance lookup and the direction (the same values: env_eval's
  // phi = u 2 pi, th = v pi are these)
  const bcr::SinCos scp = bcr::sincosf(phi);
  const float cth = sct.c, cph = scp.c, sph = scp.s;
  ls.li = env_eval_trig<F>(L, u, v, sint, cth, cph, sph);
  V3 dl = mk(sint * cph, sint * sph, cth);
  ls.wi = xvector(L.l2w, dl);
  ls.ray = Ray{pW, ls.wi, eps, INFINITY};
  ls.pdf = mpdf / (2.f * PI * PI * sint);
  return ls;
}

template <uint32_t F>
DEV float light_pdf(const DevScene& S, const bling_light& L, V3 p, V3 wi) {           // Light.hs:215-229
  if ((F & FT_DELTA) && L.kind >= BLING_LIGHT_POINT) return 0.f;
  if (!(F & FT_INF) || L.kind == BLING_LIGHT_AREA) {
    const DevShape& s = light_shape<F>(S, L);
    return shape_pdf<F>(s, xpoint(s.w2o, p), xvector(s.w2o, wi));
  }
  V3 w = xvector(L.w2l, wi);
  float u, v, st;
  dir_to_uv(w, &u, &v, &st);
  if (st == 0.f) return 0.f;
  return pdf_d2d(L, u, v) / (2.f * PI * PI * st);
}

}  // namespace bd
