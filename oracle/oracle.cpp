// oracle.cpp -- ORACLE (test infrastructure only).  CPU restatement of bling's per-sample path,
// following the Haskell sources of bindingflare/bling (paths relative to src/lib/Graphics/Bling/).
// Product code never links this file; see oracle.h for the parity status.
#include "oracle.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "ocore.h"
#include "../bling_amd/csrc/common/cr_math.h"
#include "../bling_amd/csrc/common/image_tex.h"

using namespace ora;

namespace {

// ======================================================================= scene data
struct AABB { V mn, mx; };
inline AABB empty_box() { return AABB{mk(INF, INF, INF), mk(-INF, -INF, -INF)}; }      // AABB.hs:63-67
inline AABB extend(const AABB& a, const AABB& b) {                                      // AABB.hs:73-80
  return AABB{mk(hmin(a.mn.x, b.mn.x), hmin(a.mn.y, b.mn.y), hmin(a.mn.z, b.mn.z)),
              mk(hmax(a.mx.x, b.mx.x), hmax(a.mx.y, b.mx.y), hmax(a.mx.z, b.mx.z))};
}
inline AABB extend_p(const AABB& a, V p) {                                              // AABB.hs:82-85
  return AABB{mk(hmin(a.mn.x, p.x), hmin(a.mn.y, p.y), hmin(a.mn.z, p.z)),
              mk(hmax(a.mx.x, p.x), hmax(a.mx.y, p.y), hmax(a.mx.z, p.z))};
}
inline int dominant(V v) {                                                              // Math.hs:292-301
  float ax = std::fabs(v.x), ay = std::fabs(v.y), az = std::fabs(v.z);
  if (ax > ay && ax > az) return 0;
  if (ay > az) return 1;
  return 2;
}
inline float surface_area(const AABB& b) {                                              // AABB.hs:68-71
  V d = b.mx - b.mn;
  return 2.f * (d.x * d.y + d.x * d.z + d.y * d.z);
}

// intersectAABB (AABB.hs:79-94) with Haskell max/min semantics
bool intersect_aabb(const AABB& b, const Ray& r, float* n_out, float* f_out) {
  float near = r.tmin, far = r.tmax;
  for (int dim = 0; dim < 3; ++dim) {
    if (near > far) return false;
    float dinv = 1.f / comp(r.d, dim);
    float oc = comp(r.o, dim);
    float tn = (comp(b.mn, dim) - oc) * dinv;
    float tf = (comp(b.mx, dim) - oc) * dinv;
    float n2, f2;
    if (tn > tf) { n2 = tf; f2 = tn; } else { n2 = tn; f2 = tf; }
    near = hmax(near, n2);
    far = hmin(far, f2);
  }
  if (near > far) return false;
  *n_out = near; *f_out = far;
  return true;
}

struct DG {                                                                             // DifferentialGeometry.hs:26-36
  V p, n;
  float u, v;
  V dpdu, dpdv;
  bool has_b;
  float b1, b2;
};
inline DG mk_dg(V p, float u, float v, V dpdu, V dpdv) {                                // DifferentialGeometry.hs:41-50
  return DG{p, normalize(cross(dpdu, dpdv)), u, v, dpdu, dpdv, false, 0.f, 0.f};
}
inline DG mk_dg2(V p, V n) {                                                            // DifferentialGeometry.hs:53-56
  LC c = coordinate_system(n);
  return DG{p, n, 0.f, 0.f, c.s, c.t, false, 0.f, 0.f};
}
inline DG trans_dg(const float* o2w, const float* w2o, const DG& d) {                   // DifferentialGeometry.hs:72-81
  DG r = d;
  r.p = xpoint(o2w, d.p);
  r.n = normalize(xnormal(w2o, d.n));
  r.dpdu = xvector(o2w, d.dpdu);
  r.dpdv = xvector(o2w, d.dpdv);
  return r;
}

struct Hit { float t, eps; DG dg; int prim; };

struct Prim { int kind, index; AABB bounds; };

struct Scene {
  const bling_scene_desc* d;
  std::vector<Prim> prims;
  // kd-tree (KdTree.hs:109-113)
  struct Node { int leaf; int left, right; float sp; int axis; std::vector<int> ps; };
  std::vector<Node> nodes;
  AABB bounds;
  int max_depth_param;
  // extent / tiles
  int ex0, ex1, ey0, ey1;
  struct Tile { int x0, x1, y0, y1; };
  std::vector<Tile> tiles;
  std::string info;
  int rng = 0;                          // ORACLE_RNG_COUNTER (product's sampler) / ORACLE_RNG_MWC
};

// ======================================================================= shapes
// Shape.hs:157-171 (Quad intersect), :266-273 (intersects)
bool quad_intersect(float sx, float sy, const Ray& r, float* t_out, float* eps, DG* dg) {
  if (std::fabs(r.d.z) < 1e-7f) return false;
  float t = -(r.o.z) / r.d.z;
  if (t < r.tmin || t > r.tmax) return false;
  V p = ray_at(r, t);
  if (std::fabs(p.x) > sx || std::fabs(p.y) > sy) return false;
  if (dg) {
    *eps = 5e-4f * t;
    float u = (sx + p.x) / (2.f * sx), v = (sy + p.y) / (2.f * sy);
    *dg = mk_dg(p, u, v, mk(sx, 0.f, 0.f), mk(0.f, sy, 0.f));
  }
  *t_out = t;
  return true;
}

// Shape.hs:173-229 (Sphere intersect)
bool sphere_intersect(float rad, const Ray& r, float* t_out, float* eps, DG* dg) {
  float a = sqlen(r.d), b = 2.f * dot(r.o, r.d), c = sqlen(r.o) - (rad * rad);
  float t1, t2;
  if (!solve_quadric(a, b, c, &t1, &t2)) return false;
  if (t1 > r.tmax) return false;
  if (t2 < r.tmin) return false;
  float t = t1 < r.tmin ? t2 : t1;
  if (t > r.tmax) return false;
  *t_out = t;
  if (dg) {
    *eps = 5e-4f * t;
    V p = ray_at(r, t);
    const float thetaMin = PI, thetaMax = 0.f, phiMax = TWO_PI;
    float phi = atan2p(p.y, p.x);
    float u = phi / phiMax;
    float theta = bcr::acosf(clampf(p.z / rad, -1.f, 1.f));
    float v = (theta - thetaMin) / (thetaMax - thetaMin);
    float zr = std::sqrt(p.x * p.x + p.y * p.y);
    float izr = 1.f / zr;
    float cosphi = p.x * izr, sinphi = p.y * izr;
    V dpdu = mk(-(phiMax * p.y), phiMax * p.x, 0.f);
    V dpdv = vs(mk(p.z * cosphi, p.z * sinphi, -(rad * bcr::sinf(theta))), thetaMax - thetaMin);
    *dg = mk_dg(p, u, v, dpdu, dpdv);
  }
  return true;
}

// Shape.hs:275-284 (Sphere intersects)
bool sphere_intersects(float rad, const Ray& r) {
  float a = sqlen(r.d), b = 2.f * dot(r.o, r.d), c = sqlen(r.o) - (rad * rad);
  float t0, t1;
  if (!solve_quadric(a, b, c, &t0, &t1)) return false;
  if (t0 > r.tmax || t1 < r.tmin) return false;
  if (t0 < r.tmin) return t1 < r.tmax;
  return true;
}

inline V set_comp(int k, float t, V v) { if (k == 0) v.x = t; else if (k == 1) v.y = t; else v.z = t; return v; }

// Shape.hs:142-155 (Disk intersect) / :253-264 (intersects): the same tests
bool disk_intersect(const float* P, const Ray& r, float* t_out, float* eps, DG* dg) {
  float h = P[0], rad = P[1], irad = P[2], phimax = P[3];
  if (std::fabs(r.d.z) < 1e-7f) return false;
  float t = (h - r.o.z) / r.d.z;
  if (t < r.tmin || t > r.tmax) return false;
  V p = ray_at(r, t);
  float d2 = p.x * p.x + p.y * p.y;
  if (d2 > rad * rad || d2 < irad * irad) return false;
  if (atan2p(p.y, p.x) > phimax) return false;
  if (dg) { *eps = 5e-4f * t; *dg = mk_dg2(p, mk(0.f, 0.f, -1.f)); }
  *t_out = t;
  return true;
}
// Shape.hs:113-140 (Cylinder intersect) / :235-251 (intersects)
bool cylinder_hit(const float* P, const Ray& r, bool any, float* t_out, V* p_out) {
  float rad = P[0], zmin = P[1], zmax = P[2], phimax = P[3];
  float a = r.d.x * r.d.x + r.d.y * r.d.y;
  float b = 2.f * (r.d.x * r.o.x + r.d.y * r.o.y);
  float c = r.o.x * r.o.x + r.o.y * r.o.y - rad * rad;
  float t0, t1;
  if (!solve_quadric(a, b, c, &t0, &t1)) return false;
  if (t0 > r.tmax) return false;
  if (t1 < r.tmin) return false;
  V p0 = ray_at(r, t0), p1 = ray_at(r, t1);
  if (t0 > r.tmin && p0.z > zmin && p0.z < zmax && atan2p(p0.y, p0.x) <= phimax) { *t_out = t0; *p_out = p0; return true; }
  bool second = any ? (t1 < r.tmax && p1.z > zmin && p1.z < zmax && atan2p(p1.y, p1.x) <= phimax && t1 <= r.tmax)
                    : (t1 <= r.tmax && p1.z > zmin && p1.z < zmax && atan2p(p1.y, p1.x) <= phimax);
  if (second) { *t_out = t1; *p_out = p1; return true; }
  return false;
}
bool cylinder_intersect(const float* P, const Ray& r, float* t_out, float* eps, DG* dg) {
  V p;
  if (!cylinder_hit(P, r, false, t_out, &p)) return false;
  if (dg) {
    *eps = 5e-4f * *t_out;
    float phimax = P[3];
    V dpdu = mk(-(phimax * p.y), phimax * p.x, 0.f), dpdv = mk(0.f, 0.f, P[2] - P[1]);
    *dg = mk_dg2(p, normalize(cross(dpdu, dpdv)));
  }
  return true;
}
// Shape.hs:86-111 (Box intersect): testSlabs from (-inf, inf) with the axis of the last near increase
bool box_intersect(const float* P, const Ray& r, float* t_out, float* eps, DG* dg) {
  V pmin = mk(P[0], P[1], P[2]), pmax = mk(P[3], P[4], P[5]);
  float n = -INF, f = INF;
  int dd = 0;
  for (int dim = 0; dim < 3; ++dim) {
    if (n > f) return false;
    float oc = comp(r.o, dim), dinv = 1.f / comp(r.d, dim);
    float t1p = (comp(pmax, dim) - oc) * dinv, t2p = (comp(pmin, dim) - oc) * dinv;
    float t1 = t1p > t2p ? t2p : t1p, t2 = t1p > t2p ? t1p : t2p;
    int nd = n < t1 ? dim : dd;
    n = hmax(n, t1); f = hmin(f, t2); dd = nd;
  }
  if (n > f) return false;
  float t0 = hmin(n, f), t1 = hmax(n, f);
  if (t0 > r.tmax || t0 < r.tmin) return false;
  float t = t0 < r.tmin ? t1 : t0;
  if (t > r.tmax) return false;
  if (dg) {
    V p = ray_at(r, t);
    *eps = 5e-4f * t;
    float half = (comp(pmin, dd) + comp(pmax, dd)) / 2.f;
    float dir = comp(p, dd) > half ? 1.f : -1.f;
    *dg = mk_dg2(p, normalize(set_comp(dd, dir, mk(0.f, 0.f, 0.f))));
  }
  *t_out = t;
  return true;
}

float shape_area(const bling_shape& s) {                                                // Shape.hs:314-328
  const float* P = s.params;
  switch (s.kind) {
    case BLING_SHAPE_QUAD: return 4.f * P[0] * P[1];
    case BLING_SHAPE_DISK: return PI * (P[1] * P[1] - P[2] * P[2]);
    case BLING_SHAPE_CYLINDER: return 2.f * PI * P[0] * (P[2] - P[1]);
    case BLING_SHAPE_BOX: {
      float h = P[3] - P[0], w = P[4] - P[1], l = P[5] - P[2];
      return 2.f * (h * w + h * l + w * l);
    }
    default: return P[0] * P[0] * 4.f * PI;
  }
}

bool shape_intersect_local(const bling_shape& s, const Ray& r, float* t, float* eps, DG* dg) {
  switch (s.kind) {
    case BLING_SHAPE_QUAD: return quad_intersect(s.params[0], s.params[1], r, t, eps, dg);
    case BLING_SHAPE_DISK: return disk_intersect(s.params, r, t, eps, dg);
    case BLING_SHAPE_CYLINDER: return cylinder_intersect(s.params, r, t, eps, dg);
    case BLING_SHAPE_BOX: return box_intersect(s.params, r, t, eps, dg);
    default: return sphere_intersect(s.params[0], r, t, eps, dg);
  }
}
bool shape_intersects_local(const bling_shape& s, const Ray& r) {
  float t, n0, f0;
  V p;
  switch (s.kind) {
    case BLING_SHAPE_QUAD: return quad_intersect(s.params[0], s.params[1], r, &t, nullptr, nullptr);
    case BLING_SHAPE_DISK: return disk_intersect(s.params, r, &t, nullptr, nullptr);
    case BLING_SHAPE_CYLINDER: return cylinder_hit(s.params, r, true, &t, &p);
    case BLING_SHAPE_BOX: {                                                              // intersectAABB (mkAABB pmin pmax)
      AABB b{mk(s.params[0], s.params[1], s.params[2]), mk(s.params[3], s.params[4], s.params[5])};
      return intersect_aabb(b, r, &n0, &f0);
    }
    default: return sphere_intersects(s.params[0], r);
  }
}

// ======================================================================= triangles
// TriangleMesh.hs:140-158 (triangleIntersects) / 160-207 (triangleIntersect)
struct TriVerts { V p1, p2, p3; };
TriVerts tri_verts(const bling_scene_desc* d, int t) {
  const uint32_t* ix = d->tri_indices + 3 * t;
  auto P = [&](uint32_t i) { return mk(d->vertices[3 * i], d->vertices[3 * i + 1], d->vertices[3 * i + 2]); };
  return TriVerts{P(ix[0]), P(ix[1]), P(ix[2])};
}

bool tri_intersects(const TriVerts& tv, const Ray& r) {
  V e1 = tv.p2 - tv.p1, e2 = tv.p3 - tv.p1;
  V s1 = cross(r.d, e2);
  float divisor = dot(s1, e1);
  if (divisor == 0.f) return false;
  float inv = 1.f / divisor;
  V dd = r.o - tv.p1;
  float b1 = dot(dd, s1) * inv;
  if (b1 < 0.f || b1 > 1.f) return false;
  V s2 = cross(dd, e1);
  float b2 = dot(r.d, s2) * inv;
  if (b2 < 0.f || b1 + b2 > 1.f) return false;
  float t = dot(e2, s2) * inv;
  if (t < r.tmin || t > r.tmax) return false;
  return true;
}

bool tri_intersect(const bling_scene_desc* d, int tri, const Ray& r, Hit* h) {
  TriVerts tv = tri_verts(d, tri);
  V e1 = tv.p2 - tv.p1, e2 = tv.p3 - tv.p1;
  V s1 = cross(r.d, e2);
  float divisor = dot(s1, e1);
  if (divisor == 0.f) return false;
  float inv = 1.f / divisor;
  V dd = r.o - tv.p1;
  float b1 = dot(dd, s1) * inv;
  if (b1 < 0.f || b1 > 1.f) return false;
  V s2 = cross(dd, e1);
  float b2 = dot(r.d, s2) * inv;
  if (b2 < 0.f || b1 + b2 > 1.f) return false;
  float t = dot(e2, s2) * inv;
  if (t < r.tmin || t > r.tmax) return false;
  const float* uv = d->tri_uvs + 6 * tri;
  float uv00 = uv[0], uv01 = uv[1], uv10 = uv[2], uv11 = uv[3], uv20 = uv[4], uv21 = uv[5];
  V n = normalize(cross(e1, e2));
  float du1 = uv00 - uv20, du2 = uv10 - uv20, dv1 = uv01 - uv21, dv2 = uv11 - uv21;
  V dp1 = tv.p1 - tv.p3, dp2 = tv.p2 - tv.p3;
  float det = du1 * dv2 - dv1 * du2;
  V dpdu, dpdv;
  if (det == 0.f) {
    LC c = coordinate_system(n);                                                        // coordinateSystem''
    dpdu = c.s; dpdv = c.t;
  } else {
    float idet = 1.f / det;
    dpdu = sm(idet, sm(dv2, dp1) - sm(dv1, dp2));
    dpdv = sm(idet, sm(-du2, dp1) + sm(du1, dp2));
  }
  float b0 = 1.f - b1 - b2;
  float tu = b0 * uv00 + b1 * uv10 + b2 * uv20;
  float tvv = b0 * uv01 + b1 * uv11 + b2 * uv21;
  h->t = t;
  h->eps = 1e-3f * t;
  h->dg = DG{ray_at(r, t), normalize(cross(dpdu, dpdv)), tu, tvv, dpdu, dpdv, true, b1, b2};   // mkDgTri
  return true;
}

// ======================================================================= mandelbulb (Fractal.hs)
V bulb_power(V p, int n) {                                                              // Fractal.hs:103-137
  if (n == 8) {
    float x = p.x, y = p.y, z = p.z;
    float x2 = x * x, y2 = y * y, z2 = z * z;
    float x4 = x2 * x2, y4 = y2 * y2, z4 = z2 * z2;
    float k3 = x2 + z2;
    float k2p = std::sqrt(k3 * k3 * k3 * k3 * k3 * k3 * k3);
    if (k2p <= 0.f) return mk(0.f, 0.f, 0.f);
    float k2 = 1.f / k2p;
    float k1 = x4 + y4 + z4 - 6.f * y2 * z2 - 6.f * x2 * y2 + 2.f * z2 * x2;
    float k4 = x2 - y2 + z2;
    float wx = 64.f * x * y * z * (x2 - z2) * k4 * (x4 - 6.f * x2 * z2 + z4) * k1 * k2;
    float wy = -(16.f * y2 * k3 * k4 * k4) + k1 * k1;
    float wz = -(8.f * y * k4 * (x4 * x4 - 28.f * x4 * x2 * z2 + 70.f * x4 * z4 - 28.f * x2 * z2 * z4 + z4 * z4) * k1 * k2);
    return mk(wx, wy, wz);
  }
  float wr = len(p);
  float wo = bcr::acosf(p.y / wr);
  float wi = bcr::atan2f(p.x, p.z);
  float fn = (float)n;
  float wrp = bcr::powf(wr, fn), wop = wo * fn, wip = wi * fn;
  return vs(mk(bcr::sinf(wop) * bcr::sinf(wip), bcr::cosf(wop), bcr::sinf(wop) * bcr::cosf(wip)), wrp);
}
float mandel_potential(int order, int its, V pos) {                                     // Fractal.hs:90-98
  V z = pos;
  for (int n = its + 1;; --n) {
    if (n == 1) return 0.f;
    V zp = bulb_power(z, order) + pos;
    if (sqlen(zp) > 2.5f) {
      long pw = 1;
      for (int k = 0; k < 1 + its - n; ++k) pw *= order;
      return bcr::logf(len(zp)) / (float)pw;
    }
    z = zp;
  }
}
float mandel_dist(int order, int its, float eps, V p, V* g) {                           // Fractal.hs:73-88
  float pot = mandel_potential(order, its, p);
  if (pot == 0.f) { *g = mk(0.f, 1.f, 0.f); return 0.f; }
  V gp = mk(mandel_potential(order, its, p + mk(eps, 0.f, 0.f)), mandel_potential(order, its, p + mk(0.f, eps, 0.f)),
            mandel_potential(order, its, p + mk(0.f, 0.f, eps)));
  *g = vs(gp - mk(pot, pot, pot), 1.f / eps);
  return (0.5f / bcr::expf(pot)) * bcr::sinhf(pot) / len(*g);
}
bool int_sphere(float r2, const Ray& r, float* t_out) {                                 // Fractal.hs:59-70
  float c = sqlen(r.o) - r2;
  if (c <= 0.f) { *t_out = r.tmin; return true; }
  float a = sqlen(r.d), b = 2.f * dot(r.d, r.o);
  float t0, t1;
  if (!solve_quadric(a, b, c, &t0, &t1)) return false;
  if (t0 > r.tmax || t1 < r.tmin) return false;
  *t_out = t0;
  return true;
}
Ray normalize_ray(const Ray& r) {                                                       // Math.hs:399-405
  float l = len(r.d);
  return Ray{r.o, vs(r.d, 1.f / l), r.tmin * l, r.tmax * l};
}
// mandelInter / mandelInters (Fractal.hs:37-57): no rayMax check (trap T10)
bool mandel_march(const bling_fractal& f, const Ray& r, float* d_out, V* p_out, V* n_out) {
  float d;
  if (!int_sphere(2.f, r, &d)) return false;
  Ray rn = normalize_ray(r);
  for (;;) {
    V p = ray_at(rn, d);
    if (sqlen(p) > 2.5f) return false;
    V g;
    float dist = mandel_dist(f.order, f.iterations, f.epsilon, p, &g);
    if (dist < f.epsilon) { *d_out = d; *p_out = p; *n_out = normalize(g); return true; }
    d = d + dist;
  }
}

// ======================================================================= Julia quaternion fractal
// Fractal.hs:148-281: Quaternion r (i, j, k)
struct Q { float r; V i; };
inline Q qadd(Q a, Q b) { return Q{a.r + b.r, a.i + b.i}; }
inline Q qsub(Q a, Q b) { return Q{a.r - b.r, a.i - b.i}; }
inline float qlen(Q q) { return std::sqrt(q.r * q.r + q.i.x * q.i.x + q.i.y * q.i.y + q.i.z * q.i.z); }
inline Q qscale(Q q, float s) { return Q{q.r * s, mk(s * q.i.x, s * q.i.y, s * q.i.z)}; }
inline Q qsq(Q q) { return Q{q.r * q.r - dot(q.i, q.i), mk(2.f * q.r * q.i.x, 2.f * q.r * q.i.y, 2.f * q.r * q.i.z)}; }
inline Q qmul(Q q, Q r) {
  float r1 = q.r, r2 = r.r;
  V c = cross(q.i, r.i);
  return Q{r1 * r2 - dot(q.i, r.i),
           mk(c.x + r1 * r.i.x + r2 * q.i.x, c.y + r1 * r.i.y + r2 * q.i.y, c.z + r1 * r.i.z + r2 * q.i.z)};
}
inline Q qpromote(V p) { return Q{p.x, mk(p.y, p.z, 0.f)}; }
const float kJuliaR2 = 3.f;                                                             // juliaRadius2
// iter (Fractal.hs:236-242): returns the NEXT iterate and its derivative when it stops
void julia_iter(Q q, Q c, int mi, Q* z, Q* zp) {
  Q qp = Q{1.f, mk(0.f, 0.f, 0.f)};                                                     // qzero
  for (int i = mi;; --i) {
    Q q2 = qadd(qsq(q), c), qp2 = qscale(qmul(q, qp), 2.f);
    if (i == 0 || qlen(q) > 4.f) { *z = q2; *zp = qp2; return; }                       // escapeThreashold
    q = q2; qp = qp2;
  }
}
// traverseJulia (Fractal.hs:188-198) on the normalised ray, with prepare (:162-172)
bool julia_march(const bling_fractal& f, const Ray& r0, float* d_out, V* p_out) {
  Ray r = normalize_ray(r0);
  float d;
  {
    float c = sqlen(r.o) - kJuliaR2;
    if (c <= 0.f) d = r.tmin;
    else {
      float a = sqlen(r.d), b = 2.f * dot(r.d, r.o), t0, t1;
      if (!solve_quadric(a, b, c, &t0, &t1)) return false;
      if (t0 > r.tmax || t1 < r.tmin) return false;
      d = t0;
    }
  }
  Q c = Q{f.julia_c[0], mk(f.julia_c[1], f.julia_c[2], f.julia_c[3])};
  for (;;) {
    V o = ray_at(r, d);
    if (sqlen(o) > kJuliaR2 + f.epsilon) return false;
    Q z, zp;
    julia_iter(qpromote(o), c, f.iterations, &z, &zp);
    float nz = qlen(z);
    float dist = (0.5f * nz * bcr::logf(nz)) / qlen(zp);
    if (dist < f.epsilon) {
      if (!(d >= r.tmin && d <= r.tmax)) return false;                                   // onRay
      *d_out = d; *p_out = o;
      return true;
    }
    d = d + dist;
  }
}
// normalJulia (Fractal.hs:203-223): central differences of |z| after exactly mi iterations
V julia_normal(const bling_fractal& f, V p) {
  Q c = Q{f.julia_c[0], mk(f.julia_c[1], f.julia_c[2], f.julia_c[3])};
  Q qp = qpromote(p);
  Q dx = qpromote(mk(f.epsilon, 0.f, 0.f)), dy = qpromote(mk(0.f, f.epsilon, 0.f)), dz = qpromote(mk(0.f, 0.f, f.epsilon));
  Q v[6] = {qsub(qp, dx), qadd(qp, dx), qsub(qp, dy), qadd(qp, dy), qsub(qp, dz), qadd(qp, dz)};
  for (int n = 0; n < f.iterations; ++n)
    for (int k = 0; k < 6; ++k) v[k] = qadd(c, qsq(v[k]));                              // qadd c . qsq
  return normalize(mk(qlen(v[1]) - qlen(v[0]), qlen(v[3]) - qlen(v[2]), qlen(v[5]) - qlen(v[4])));
}
bool fractal_hit(const bling_fractal& f, const Ray& r, float* d, V* p, V* n) {
  if (f.kind == BLING_FRACTAL_JULIA) {
    if (!julia_march(f, r, d, p)) return false;
    *n = julia_normal(f, *p);
    return true;
  }
  return mandel_march(f, r, d, p, n);
}

// ======================================================================= primitives
AABB prim_bounds(const bling_scene_desc* d, int kind, int idx) {
  if (kind == 0) {                                                                      // triangleBounds
    TriVerts tv = tri_verts(d, idx);
    AABB b = empty_box();
    b = extend_p(b, tv.p1); b = extend_p(b, tv.p2); b = extend_p(b, tv.p3);
    return b;
  }
  if (kind == 1) {                                                                      // transBox o2w objectBounds
    const bling_shape& s = d->shapes[idx];
    const float* P = s.params;
    V mn, mx;                                                                           // objectBounds (Shape.hs:299-311)
    if (s.kind == BLING_SHAPE_QUAD) { mn = mk(-P[0], -P[1], 0.f); mx = mk(P[0], P[1], 0.f); }
    else if (s.kind == BLING_SHAPE_DISK) { mn = mk(-P[1], -P[1], P[0]); mx = mk(P[1], P[1], P[0]); }
    else if (s.kind == BLING_SHAPE_CYLINDER) { mn = mk(-P[0], -P[0], P[1]); mx = mk(P[0], P[0], P[2]); }
    else if (s.kind == BLING_SHAPE_BOX) { mn = mk(P[0], P[1], P[2]); mx = mk(P[3], P[4], P[5]); }
    else { float r = P[0]; mn = mk(-r, -r, -r); mx = mk(r, r, r); }
    V c[8] = {mk(mn.x, mn.y, mn.z), mk(mn.x, mn.y, mx.z), mk(mn.x, mx.y, mn.z), mk(mn.x, mx.y, mx.z),
              mk(mx.x, mn.y, mn.z), mk(mx.x, mn.y, mx.z), mk(mx.x, mx.y, mn.z), mk(mx.x, mx.y, mx.z)};
    AABB b = empty_box();
    for (int k = 0; k < 8; ++k) b = extend_p(b, xpoint(s.o2w, c[k]));
    return b;
  }
  if (d->fractal.kind == BLING_FRACTAL_JULIA) {                                         // mkJuliaQuat bounds
    float jr = std::sqrt(kJuliaR2);
    return AABB{mk(-jr, -jr, -jr), mk(jr, jr, jr)};
  }
  return AABB{mk(-2.5f, -2.5f, -2.5f), mk(2.5f, 2.5f, 2.5f)};                              // mkMandelBulb bounds
}

bool prim_intersect(const Scene& Sc, int pi, const Ray& r, Hit* h) {
  const Prim& p = Sc.prims[pi];
  const bling_scene_desc* d = Sc.d;
  if (p.kind == 0) {
    if (!tri_intersect(d, p.index, r, h)) return false;
    h->prim = pi;
    return true;
  }
  if (p.kind == 1) {                                                                    // mkGeom inter (Geometry.hs:33-36)
    const bling_shape& s = d->shapes[p.index];
    Ray ro{xpoint(s.w2o, r.o), xvector(s.w2o, r.d), r.tmin, r.tmax};
    float t, eps;
    DG dg;
    if (!shape_intersect_local(s, ro, &t, &eps, &dg)) return false;
    h->t = t; h->eps = eps; h->dg = trans_dg(s.o2w, s.w2o, dg); h->prim = pi;
    return true;
  }
  float dd; V pp, nn;                                                                   // mkMandelBulb / mkJuliaQuat inter
  if (!fractal_hit(d->fractal, r, &dd, &pp, &nn)) return false;
  h->t = dd; h->eps = d->fractal.epsilon * 2.f; h->dg = mk_dg2(pp, nn); h->prim = pi;
  return true;
}

bool prim_intersects(const Scene& Sc, int pi, const Ray& r) {
  const Prim& p = Sc.prims[pi];
  const bling_scene_desc* d = Sc.d;
  if (p.kind == 0) return tri_intersects(tri_verts(d, p.index), r);
  if (p.kind == 1) {
    const bling_shape& s = d->shapes[p.index];
    Ray ro{xpoint(s.w2o, r.o), xvector(s.w2o, r.d), r.tmin, r.tmax};
    return shape_intersects_local(s, ro);
  }
  float dd; V pp;
  if (d->fractal.kind == BLING_FRACTAL_JULIA) return julia_march(d->fractal, r, &dd, &pp);
  V nn;
  return mandel_march(d->fractal, r, &dd, &pp, &nn);
}

// ======================================================================= kd-tree (KdTree.hs)
const float cT = 1.f, cI = 80.f;

struct Edge { int prim; float t; bool start; };
inline bool edge_lt(const Edge& a, const Edge& b) {                                     // Ord Edge (KdTree.hs:177-180)
  if (a.t == b.t) return a.start && !b.start;
  return a.t < b.t;
}

float kd_cost(const AABB& b, int a0, float t, int nl, int nr) {                         // KdTree.hs:187-208
  V d = b.mx - b.mn;
  int a1 = (a0 + 1) % 3, a2 = (a0 + 2) % 3;
  float dl = t - comp(b.mn, a0), dr = comp(b.mx, a0) - t;
  float sal = 2.f * (comp(d, a1) * comp(d, a2) + dl * (comp(d, a1) + comp(d, a2)));
  float sar = 2.f * (comp(d, a1) * comp(d, a2) + dr * (comp(d, a1) + comp(d, a2)));
  float inv = 1.f / surface_area(b);
  float pl = sal * inv, pr = sar * inv;
  float pI = pl * (float)nl + pr * (float)nr;
  float eb = (nl == 0 || nr == 0) ? 0.5f : 1.f;
  return cT + cI * eb * pI;
}

int kd_build(Scene& Sc, const AABB& bounds, std::vector<int> ps, int depth) {           // buildTree / trySplit
  int me = (int)Sc.nodes.size();
  Sc.nodes.push_back(Scene::Node());
  if (depth == 0 || ps.size() <= 1) {
    Sc.nodes[me].leaf = 1; Sc.nodes[me].ps = ps;
    return me;
  }
  int mext = dominant(bounds.mx - bounds.mn);
  float old_cost = cI * (float)ps.size();
  for (int k = 0; k < 3; ++k) {
    int axis = (mext + k) % 3;
    std::vector<Edge> es;
    for (int p : ps) {
      const AABB& b = Sc.prims[p].bounds;
      es.push_back(Edge{p, comp(b.mn, axis), true});
      es.push_back(Edge{p, comp(b.mx, axis), false});
    }
    std::stable_sort(es.begin(), es.end(), edge_lt);
    // allSplits + filterSplits + bestSplit
    int l = 0, r = (int)es.size() / 2;
    float best = INF; int bi = -1; float bt = 0.f;
    float tmin = comp(bounds.mn, axis), tmax = comp(bounds.mx, axis);
    bool any = false;
    for (int i = 0; i < (int)es.size(); ++i) {
      int nl, nr;
      if (!es[i].start) { r -= 1; nl = l; nr = r; } else { nl = l; nr = r; l += 1; }
      float t = es[i].t;
      if (!(t > tmin && t < tmax)) continue;
      any = true;
      float c = kd_cost(bounds, axis, t, nl, nr);
      if (c < best) { best = c; bi = i; bt = t; }
    }
    if (!any) continue;
    if (best < old_cost) {
      std::vector<int> lp, rp;
      for (int i = 0; i < bi; ++i) if (es[i].start) lp.push_back(es[i].prim);
      for (int i = bi + 1; i < (int)es.size(); ++i) if (!es[i].start) rp.push_back(es[i].prim);
      AABB lb = bounds, rb = bounds;
      setc(lb.mx, axis, bt);
      setc(rb.mn, axis, bt);
      int li = kd_build(Sc, lb, lp, depth - 1);
      int ri = kd_build(Sc, rb, rp, depth - 1);
      Scene::Node& n = Sc.nodes[me];
      n.leaf = 0; n.left = li; n.right = ri; n.sp = bt; n.axis = axis;
      return me;
    }
  }
  Sc.nodes[me].leaf = 1; Sc.nodes[me].ps = ps;
  return me;
}

struct TStats { uint64_t nodes = 0, leaf_prims = 0; };

// traverse (KdTree.hs:223-234): closest hit
void kd_traverse(const Scene& Sc, Ray& r, bool& found, Hit& best, V inv, int node, float tmin, float tmax, TStats& ts) {
  const Scene::Node& n = Sc.nodes[node];
  ts.nodes++;
  if (n.leaf) {                                                                         // nearest' (Primitive.hs:29-43)
    for (int p : n.ps) {
      ts.leaf_prims++;
      Hit h;
      if (prim_intersect(Sc, p, r, &h)) { r.tmax = h.t; best = h; found = true; }
    }
    return;
  }
  if (r.tmax < tmin) return;
  float oa = comp(r.o, n.axis), da = comp(r.d, n.axis);
  float tp = (n.sp - oa) * comp(inv, n.axis);
  bool lf = (oa < n.sp) || (oa == n.sp && da <= 0.f);
  int fc = lf ? n.left : n.right, sc = lf ? n.right : n.left;
  if (tp > tmax || tp <= 0.f) { kd_traverse(Sc, r, found, best, inv, fc, tmin, tmax, ts); return; }
  if (tp < tmin) { kd_traverse(Sc, r, found, best, inv, sc, tmin, tmax, ts); return; }
  kd_traverse(Sc, r, found, best, inv, fc, tmin, tp, ts);
  kd_traverse(Sc, r, found, best, inv, sc, tp, tmax, ts);
}

// traverse' (KdTree.hs:210-221): any hit
bool kd_traverse_any(const Scene& Sc, const Ray& r, V inv, int node, float tmin, float tmax, TStats& ts) {
  const Scene::Node& n = Sc.nodes[node];
  ts.nodes++;
  if (n.leaf) {
    for (int p : n.ps) { ts.leaf_prims++; if (prim_intersects(Sc, p, r)) return true; }
    return false;
  }
  float oa = comp(r.o, n.axis), da = comp(r.d, n.axis);
  float tp = (n.sp - oa) * comp(inv, n.axis);
  bool lf = (oa < n.sp) || (oa == n.sp && da <= 0.f);
  int fc = lf ? n.left : n.right, sc = lf ? n.right : n.left;
  if (tp > tmax || tp <= 0.f) return kd_traverse_any(Sc, r, inv, fc, tmin, tmax, ts);
  if (tp < tmin) return kd_traverse_any(Sc, r, inv, sc, tmin, tmax, ts);
  return kd_traverse_any(Sc, r, inv, fc, tmin, tp, ts) || kd_traverse_any(Sc, r, inv, sc, tp, tmax, ts);
}

// kdTreePrimitive inter / inters (KdTree.hs:236-250)
bool sc_intersect(const Scene& Sc, const Ray& r0, Hit* h, TStats& ts) {
  float n, f;
  if (!intersect_aabb(Sc.bounds, r0, &n, &f)) return false;
  V inv = mk(1.f / r0.d.x, 1.f / r0.d.y, 1.f / r0.d.z);
  Ray r = r0;
  bool found = false;
  kd_traverse(Sc, r, found, *h, inv, 0, n, f, ts);
  return found;
}
bool sc_occluded(const Scene& Sc, const Ray& r, TStats& ts) {
  float n, f;
  if (!intersect_aabb(Sc.bounds, r, &n, &f)) return false;
  V inv = mk(1.f / r.d.x, 1.f / r.d.y, 1.f / r.d.z);
  return kd_traverse_any(Sc, r, inv, 0, n, f, ts);
}

// ======================================================================= textures / materials
// graphPaper (Texture.hs:191-207) with uvMapping (Texture.hs:166-170)
const float* eval_texture(const bling_scene_desc* d, int ti, const DG& dg) {
  for (;;) {
    const bling_texture& t = d->textures[ti];
    if (t.kind == BLING_TEX_CONST) return t.value;
    float x = t.uv_map[0] * dg.u + t.uv_map[2], z = t.uv_map[1] * dg.v + t.uv_map[3];
    float xf = std::fabs(x - (float)(long long)x);                                      // properFraction
    float zf = std::fabs(z - (float)(long long)z);
    float lo = t.line_width / 2.f, hi = 1.0f - lo;
    ti = (xf < lo || zf < lo || xf > hi || zf > hi) ? t.tex2 : t.tex1;
  }
}

enum { B_REFL = 1, B_TRANS = 2, B_DIFF = 4, B_GLOSSY = 8, B_SPEC = 16 };              // Reflection.hs:102-108
enum { K_LAMB, K_OREN, K_MICRO, K_SREFL, K_STRANS, K_FBLEND };
enum { FR_NOOP, FR_DIEL, FR_COND };

struct Fresnel { int kind; float ei, et; S eta, k; };
// K_FBLEND (mkFresnelBlend, Microfacet.hs:56-105): r = rd, rs, ra; e / ey = the anisotropic
// distribution's exponents ex / ey; depth = coating thickness
struct BxDF { int kind, flags; S r; float A, B, e; Fresnel fr; float ei, et; bool btdf; S rs, ra; float ey, depth; };
struct Bsdf { int n; BxDF b[2]; LC cs; V p, ng; };

inline float cos_t(V w) { return w.z; }                                                 // Reflection.hs:48-78
inline float abs_cos_t(V w) { return std::fabs(w.z); }
inline float sin_t2(V w) { return hmax(0.f, 1.f - w.z * w.z); }
inline float sin_t(V w) { return std::sqrt(sin_t2(w)); }
inline float cos_phi(V w) { float s = sin_t(w); return s == 0.f ? 1.f : clampf(w.x / s, -1.f, 1.f); }
inline float sin_phi(V w) { float s = sin_t(w); return s == 0.f ? 0.f : clampf(w.y / s, -1.f, 1.f); }
inline bool same_hemi(V a, V b) { return a.z * b.z > 0.f; }
inline V to_same_hemi(V wo, V wi) { if (wo.z < 0.f) wi.z = -wi.z; return wi; }

// frDielectric (Fresnel.hs:21-56) / frConductor (Fresnel.hs:58-70)
S fr_dielectric(float etai, float etat, float cosi) {
  float c = hmax(0.f, 1.f - cosi * cosi);
  float costp = cosi > 0.f ? c / (etat * etat) : c * (etat * etat);
  float cost = std::sqrt(1.f - clampf(costp, 0.f, 1.f));
  float ci = std::fabs(cosi);
  float eta = etat / etai;                                                              // frDiel: etat / etai (per band)
  float rparl_p = eta * ci;
  float rparl = (cost - rparl_p) / (cost + rparl_p);
  float rperp_p = eta * cost;
  float rperp = (ci - rperp_p) / (ci + rperp_p);
  return sconst((rparl * rparl + rperp * rperp) * 0.5f);
}
S fr_conductor(const S& eta, const S& k, float cosi) {
  float ac = std::fabs(cosi);
  S tmpF = eta * eta + k * k;
  S ec2 = sscale(eta, 2.f * ac);
  S tmp = sscale(eta * eta + k * k, ac * ac);
  S c2 = sconst(ac * ac);
  S rper2 = (tmpF - ec2 + c2) / (tmpF + ec2 + c2);
  S rpar2 = (tmp - ec2 + white()) / (tmp + ec2 + white());
  return (rper2 + rpar2) / sconst(2.f);
}
S fresnel(const Fresnel& f, float c) {
  if (f.kind == FR_NOOP) return white();
  if (f.kind == FR_DIEL) return fr_dielectric(f.ei, f.et, c);
  return fr_conductor(f.eta, f.k, c);
}

// Blinn distribution (Microfacet.hs:146-195)
inline float blinn_pdf(float e, V wh) { return (e + 1.f) * bcr::powf(abs_cos_t(wh), e) * INV_TWO_PI; }
inline float blinn_D(float e, V wh) { return (e + 2.f) * INV_TWO_PI * bcr::powf(abs_cos_t(wh), e); }
inline void blinn_sample(float e, float u1, float u2, V* wh, float* d, float* pdf) {
  float cost = bcr::powf(u1, 1.f / (e + 1.f));
  float sint = std::sqrt(hmax(0.f, 1.f - cost * cost));
  float phi = u2 * 2.f * PI;
  *wh = mk(sint * bcr::cosf(phi), sint * bcr::sinf(phi), cost);
  float f = bcr::powf(cost, e) * INV_TWO_PI;
  *d = (e + 2.f) * f;
  *pdf = (e + 1.f) * f;
}
inline float mf_G(V wo, V wi, V wh) {                                                   // Microfacet.hs:113-120
  float nwh = abs_cos_t(wh), nwo = abs_cos_t(wo), nwi = abs_cos_t(wi), wowh = absdot(wo, wh);
  return hmin(1.f, hmin(2.f * nwh * nwo / wowh, 2.f * nwh * nwi / wowh));
}
inline float fix_exponent(float e) { return (e > 10000.f || std::isnan(e)) ? 10000.f : e; }

// pScalarTexture at the shading point (MaterialParser.hs:115-156): scaleTexture a s t = a + s * t dg
// (Texture.hs:185), fbm / perlin over identityMapping3d = transPoint w2t (dgP dg) (Texture.hs:152-156,
// 340-385; perlin3d / fbm from common/perlin.h, pinned by tests/test_heightmap.py)
// An image scalar texture (pImageScalar, MaterialParser.hs:106-113) reads its Y8 map at the 2d
// mapping of the DG's point / (u, v) (getPixelScalar, Texture.hs:103-108; common/image_tex.h).
float eval_stex(const bling_scene_desc* d, int ti, V p, float u, float v) {
  const bling_scalar_texture& t = d->scalar_textures[ti];
  switch (t.kind) {
    case BLING_STEX_CONST: return t.value;
    case BLING_STEX_SCALE: return t.a + t.s * eval_stex(d, t.child, p, u, v);
    case BLING_STEX_IMAGE: {
      const bling_image& im = d->images[t.child];
      float s, tt;
      bimgtex::map2d(t.octaves, t.w2t, p.x, p.y, p.z, u, v, &s, &tt);
      return im.texels[bimgtex::texel(im.width, im.height, s, tt)];
    }
    case BLING_STEX_CRYSTAL: {                       // quasiCrystal o (planarMapping ...) (Texture.hs:317-338)
      const float* m = t.w2t;
      const float x = (p.x * m[0] + p.y * m[1] + p.z * m[2]) + m[6];    // (p `dot` vu + ou, p `dot` vv + ov)
      const float y = (p.x * m[3] + p.y * m[4] + p.z * m[5]) + m[7];
      float s = 0.f;                                                      // sum = foldl (+) 0
      for (int k = 0; k < t.octaves; ++k) {
        const bling_scalar_texture& w = d->scalar_textures[t.child + k];  // (cos th, sin th)
        s = s + (bcr::cosf(w.a * x + w.s * y) + 1.f) / 2.f;
      }
      float kf = std::trunc(s), v = s - kf;                               // properFraction
      long long k = (long long)kf;
      if (v < 0.f) { k = k - 1; v = 1.f + v; }
      return (k & 1) ? 1.f - v : v;                                       // wrap
    }
    default: {
      V q = xpoint(t.w2t, p);
      if (t.kind == BLING_STEX_CELLNOISE) return bcell::cell_noise(t.octaves, q.x, q.y, q.z);   // Texture.hs:274-315
      return t.kind == BLING_STEX_FBM ? bperlin::fbm(t.octaves, t.omega, q.x, q.y, q.z) : bperlin::perlin3d(q.x, q.y, q.z);
    }
  }
}

// A material's spectrum texture at the shading DG (pSpectrumTexture, IO/MaterialParser.hs:198-226):
// spectrumBlend (Texture.hs:135-145), gradient (:239-250, steps sorted at load = mkGradient) and
// checkerBoard (:215-219) over constant / graphPaper children
S eval_spectrum(const bling_scene_desc* d, int ti, const DG& dg) {
  const bling_texture& t = d->textures[ti];
  if (t.kind == BLING_TEX_BLEND) {
    const S v1 = from_array(eval_texture(d, t.tex1, dg)), v2 = from_array(eval_texture(d, t.tex2, dg));
    const float x = eval_stex(d, t.stex, dg.p, dg.u, dg.v);
    if (x <= 0.f) return v1;
    if (x >= 1.f) return v2;
    return sscale(v1, 1.f - x) + sscale(v2, x);
  }
  if (t.kind == BLING_TEX_GRADIENT) {
    const float f = eval_stex(d, t.stex, dg.p, dg.u, dg.v);
    const bling_texture* st = d->textures + t.tex1;
    const int n = t.tex2;
    if (f <= st[0].line_width) return from_array(st[0].value);           // gradMin = the first position
    if (f >= st[n - 1].line_width) return from_array(st[n - 1].value);   // gradMax = the last
    int idx = 1;                                                          // findIndex ((> f) . fst)
    while (idx < n - 1 && !(st[idx].line_width > f)) ++idx;
    const float w = (f - st[idx - 1].line_width) / (st[idx].line_width - st[idx - 1].line_width);
    return sscale(from_array(st[idx - 1].value), 1.f - w) + sscale(from_array(st[idx].value), w);
  }
  if (t.kind == BLING_TEX_CHECKER) {
    const long long s = (long long)std::floor(dg.p.x * t.uv_map[0]) + (long long)std::floor(dg.p.y * t.uv_map[1]) +
                        (long long)std::floor(dg.p.z * t.uv_map[2]);
    return from_array(eval_texture(d, (s & 1) == 0 ? t.tex1 : t.tex2, dg));   // `mod` 2 == 0
  }
  if (t.kind == BLING_TEX_IMAGE) {                   // imageTexture tm mapping dg = texMapEval tm (mapping dg)
    const bling_image& im = d->images[t.tex1];
    float s, tt;
    bimgtex::map2d(t.tex2, t.tex2 == BLING_MAP_UV ? t.uv_map : t.value, dg.p.x, dg.p.y, dg.p.z, dg.u, dg.v, &s, &tt);
    return from_array(im.texels + 16 * bimgtex::texel(im.width, im.height, s, tt));
  }
  return from_array(eval_texture(d, ti, dg));
}

// Anisotropic distribution (Microfacet.hs:136-192)
inline float aniso_pdf(float ex, float ey, V wh) {                                     // :140-144
  float costh = abs_cos_t(wh);
  float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / hmax(0.f, 1.f - costh * costh);
  return std::sqrt((ex + 1.f) * (ey + 1.f)) * INV_TWO_PI * bcr::powf(costh, e);
}
inline float aniso_D(float ex, float ey, V wh) {                                       // :185-192
  float costh = abs_cos_t(wh);
  float d = 1.f - costh * costh;
  if (d == 0.f) return 0.f;
  float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / d;
  return std::sqrt((ex + 2.f) * (ey + 2.f)) * INV_TWO_PI * bcr::powf(costh, e);
}
inline void aniso_sample(float ex, float ey, float u1, float u2, V* wh, float* d, float* pdf) {   // :151-172
  auto quadrant = [&](float u1p, float* p, float* c) {                                  // smpFirstQuadrand
    *p = ex == ey ? PI * u1p * 0.5f : bcr::atanf(std::sqrt((ex + 1.f) / (ey + 1.f)) * bcr::tanf(PI * u1p * 0.5f));
    float cp = bcr::cosf(*p), sp = bcr::sinf(*p);
    *c = bcr::powf(u2, 1.f / (ex * cp * cp + ey * sp * sp + 1.f));
  };
  float p, cost, phi;
  if (u1 < 0.25f) { quadrant(4.f * u1, &p, &cost); phi = p; }
  else if (u1 < 0.5f) { quadrant(4.f * (0.5f - u1), &p, &cost); phi = PI - p; }
  else if (u1 < 0.75f) { quadrant(4.f * (u1 - 0.5f), &p, &cost); phi = p + PI; }
  else { quadrant(4.f * (1.f - u1), &p, &cost); phi = TWO_PI - p; }
  float sint = std::sqrt(hmax(0.f, 1.f - cost * cost));
  *wh = mk(sint * bcr::cosf(phi), sint * bcr::sinf(phi), cost);                          // sphericalDirection
  float ds = 1.f - cost * cost;
  float e = (ex * wh->x * wh->x + ey * wh->y * wh->y) / ds;
  float f = INV_TWO_PI * bcr::powf(cost, e);
  *d = std::sqrt((ex + 2.f) * (ey + 2.f)) * f;
  *pdf = std::sqrt((ex + 1.f) * (ey + 1.f)) * f;
}
inline V fblend_half(V wo, V wi) { V h = normalize(wi + wo); return h.z < 0.f ? -h : h; }
// mkFresnelBlend's e wo wi (Microfacet.hs:64-84): the |cos| factor rides on wo (costo)
S fblend_eval(const BxDF& b, V wo, V wi) {
  float costi = abs_cos_t(wi), costo = abs_cos_t(wo);
  S a = b.depth > 0.f ? smap_exp(sscale(b.ra, -(b.depth * (costi + costo) / (costi * costo)))) : white();
  S diff = sscale(a * b.r * (white() - b.rs), (costo * 28.f / 23.f * PI) * (1.f - bcr::powf(1.f - 0.5f * costi, 5.f)) *
                                                  (1.f - bcr::powf(1.f - 0.5f * costo, 5.f)));
  V wh = fblend_half(wo, wi);
  float costih = absdot(wi, wh);
  S schlick = b.rs + sscale(white() - b.rs, bcr::powf(1.f - costih, 5.f));
  S spec = sscale(schlick, aniso_D(b.e, b.ey, wh) * costo / (4.f * costih * hmax(costi, costo)));
  return diff + spec;
}

S oren_nayar(const BxDF& b, V wo, V wi) {                                               // Diffuse.hs:53-65
  float sinti = sin_t(wi), sinto = sin_t(wo);
  float sina, tanb;
  if (abs_cos_t(wi) > abs_cos_t(wo)) { sina = sinto; tanb = sinti / abs_cos_t(wi); }
  else { sina = sinti; tanb = sinto / abs_cos_t(wo); }
  float maxcos = 0.f;
  if (sinti > 1e-4f && sinto > 1e-4f) {
    float sinpi = sin_phi(wi), cospi = cos_phi(wi), sinpo = sin_phi(wo), cospo = cos_phi(wo);
    maxcos = hmax(0.f, cospi * cospo + sinpi * sinpo);
  }
  return sscale(b.r, b.A + b.B * maxcos * sina * tanb);
}

// bxdfEval (first argument carries the |cos| factor; evalBsdf False flips the order, trap T7)
S brdf_eval(const BxDF& b, V wo, V wi) {
  switch (b.kind) {
    case K_LAMB: return sscale(b.r, INV_PI * abs_cos_t(wo));                            // Diffuse.hs:26
    case K_OREN: return sscale(oren_nayar(b, wo, wi), INV_PI * abs_cos_t(wo));         // Diffuse.hs:51
    case K_MICRO: {                                                                      // Microfacet.hs:21-32
      float costo = abs_cos_t(wo), costi = abs_cos_t(wi);
      if (costi == 0.f || costo == 0.f) return black();
      V whp = wi + wo;
      if (whp.x == 0.f && whp.y == 0.f && whp.z == 0.f) return black();
      V wh = normalize(whp);
      if (cos_t(wh) < 0.f) return black();
      float costh = dot(wi, wh);
      float x = blinn_D(b.e, wh) * mf_G(wo, wi, wh) / (4.f * costi);
      return sscale(b.r * fresnel(b.fr, costh), x);
    }
    case K_FBLEND: return fblend_eval(b, wo, wi);
    default: return black();                                                             // specular: e = black
  }
}
float brdf_pdf(const BxDF& b, V wo, V wi) {
  switch (b.kind) {
    case K_LAMB: case K_OREN: return same_hemi(wo, wi) ? INV_PI * abs_cos_t(wi) : 0.f;  // cosPdf
    case K_MICRO: {                                                                      // Microfacet.hs:34-40
      V whp = wo + wi;
      if (sqlen(whp) == 0.f) return 0.f;
      V wh = normalize(whp);
      if (cos_t(wh) < 0.f) return 0.f;
      return blinn_pdf(b.e, wh) / (4.f * absdot(wo, wh));
    }
    case K_FBLEND: {                                                                     // Microfacet.hs:101-105
      if (!same_hemi(wo, wi)) return 0.f;
      V wh = fblend_half(wo, wi);
      return 0.5f * (abs_cos_t(wi) * INV_PI + aniso_pdf(b.e, b.ey, wh) / (4.f * absdot(wo, wh)));
    }
    default: return 0.f;
  }
}
// bxdfSample adj -> (f, wi, pdf).  adj (the adjoint, light-to-eye direction of photons) rescales
// the sampled value by |cos wo / cos wi| (diffuse), divides by |cos wo| instead of |cos wi|
// (microfacet), or takes the adjoint transmission weight (Specular.hs:52-57).
S brdf_sample(const BxDF& b, V wo, float u1, float u2, V* wi, float* pdf, bool adj = false) {
  switch (b.kind) {
    case K_LAMB: {                                                                       // cosSample (Diffuse.hs:14-22)
      V w = to_same_hemi(wo, cosine_sample_hemisphere(u1, u2));
      if (same_hemi(wo, w)) {
        *wi = w; *pdf = brdf_pdf(b, wo, w);
        return adj ? sscale(b.r, std::fabs(cos_t(wo) / cos_t(w))) : b.r;
      }
      *wi = wo; *pdf = 0.f; return black();
    }
    case K_OREN: {                                                                       // Diffuse.hs:38-49
      V w = to_same_hemi(wo, cosine_sample_hemisphere(u1, u2));
      *wi = w;
      if (same_hemi(wo, w)) {
        *pdf = brdf_pdf(b, wo, w);
        return adj ? sscale(oren_nayar(b, wo, w), std::fabs(cos_t(wo) / cos_t(w))) : oren_nayar(b, wo, w);
      }
      *pdf = 0.f; return black();
    }
    case K_MICRO: {                                                                      // Microfacet.hs:42-54
      V whp; float d, p;
      blinn_sample(b.e, u1, u2, &whp, &d, &p);
      V wh = cos_t(whp) < 0.f ? -whp : whp;
      V w = sm(2.f * dot(wo, wh), wh) - wo;
      float costH = dot(wo, wh);
      if (!same_hemi(wo, w)) { *wi = wo; *pdf = 0.f; return black(); }
      float fact = d * std::fabs(costH) / p * mf_G(wo, w, wh);
      S fp = b.r * fresnel(b.fr, costH);
      *wi = w; *pdf = p / (4.f * std::fabs(costH));
      return sscale(fp, fact / abs_cos_t(adj ? wo : w));
    }
    case K_SREFL: {                                                                      // Specular.hs:11-26
      *wi = mk(-wo.x, -wo.y, wo.z); *pdf = 1.f;
      return b.r * fresnel(b.fr, cos_t(wo));
    }
    case K_FBLEND: {                                                                     // Microfacet.hs:86-99
      float pp;
      V wh, w;
      if (u1 < 0.5f) {
        w = to_same_hemi(wo, cosine_sample_hemisphere(u1 * 2.f, u2));
        wh = fblend_half(wo, w);
        pp = aniso_pdf(b.e, b.ey, wh);
      } else {
        float dd;
        aniso_sample(b.e, b.ey, 2.f * (u1 - 0.5f), u2, &wh, &dd, &pp);
        w = sm(2.f * dot(wo, wh), wh) - wo;
      }
      *wi = w;
      if (pp == 0.f) { *pdf = 0.f; return black(); }
      float p = 0.5f * (abs_cos_t(w) * INV_PI + pp / (4.f * absdot(wo, wh)));
      *pdf = p;
      return sscale(adj ? fblend_eval(b, w, wo) : fblend_eval(b, wo, w), 1.f / p);
    }
    case K_STRANS: {                                                                     // Specular.hs:28-57
      bool entering = cos_t(wo) > 0.f;
      float ei = entering ? b.ei : b.et, et = entering ? b.et : b.ei;
      float sini2 = sin_t2(wo);
      float eta = ei / et, eta2 = eta * eta;
      float sint2 = eta2 * sini2;
      if (sint2 >= 1.f) { *wi = wo; *pdf = 0.f; return black(); }
      float c = std::sqrt(hmax(0.f, 1.f - sint2));
      float cost = entering ? -c : c;
      *wi = mk(eta * (-wo.x), eta * (-wo.y), cost);
      S fr = fr_dielectric(ei, et, adj ? cos_t(wo) : cost);
      S fp = (white() - fr) * b.r;
      *pdf = 1.f;
      return adj ? sscale(fp, std::fabs(cos_t(wo) / cost)) : sscale(fp, eta2);
    }
  }
  *pdf = 0.f; *wi = wo; return black();
}

// brdfToBtdf (Reflection.hs:188-195): the BTDF mirrors wi into the other hemisphere around the BRDF
inline V other_hemi(V w) { return mk(w.x, w.y, -w.z); }
S bxdf_eval(const BxDF& b, V wo, V wi) { return brdf_eval(b, wo, b.btdf ? other_hemi(wi) : wi); }
float bxdf_pdf(const BxDF& b, V wo, V wi) { return brdf_pdf(b, wo, b.btdf ? other_hemi(wi) : wi); }
S bxdf_sample(const BxDF& b, V wo, float u1, float u2, V* wi, float* pdf, bool adj = false) {
  S f = brdf_sample(b, wo, u1, u2, wi, pdf, adj);
  if (b.btdf) *wi = other_hemi(*wi);
  return f;
}

// material -> Bsdf (Material.hs:32-96, Reflection.hs:209-225)
// bump (Reflection.hs:347-377): dgeu / dgev shift the point and u / v (the shifted normals feed no
// texture kind)
DG bump_dg(const bling_scene_desc* d, int ti, const DG& dgg, const DG& dgs) {
  const float du = 0.01f, dv = 0.01f;
  float uDisp = eval_stex(d, ti, dgs.p + sm(du, dgs.dpdu), dgs.u + du, dgs.v);   // d dgeu
  float vDisp = eval_stex(d, ti, dgs.p + sm(dv, dgs.dpdv), dgs.u, dgs.v + dv);   // d dgev
  float disp = eval_stex(d, ti, dgs.p, dgs.u, dgs.v);
  float vscale = (vDisp - disp) / dv;
  V dpdv = dgs.dpdv + sm(vscale, dgs.n);
  float uscale = (uDisp - disp) / du;
  V dpdu = dgs.dpdu + sm(uscale, dgs.n);
  V nn1 = normalize(cross(dpdu, dpdv));
  DG b = dgs;
  b.n = dot(nn1, dgg.n) < 0.f ? -nn1 : nn1;                                 // faceForward nn' (dgN dgg)
  b.dpdu = dpdu; b.dpdv = dpdv;
  return b;
}

Bsdf make_bsdf(const bling_scene_desc* d, int mi, const DG& dgg, const DG& dgs_in) {
  const DG dgs = d->materials[mi].stex[3] >= 0 ? bump_dg(d, d->materials[mi].stex[3], dgg, dgs_in) : dgs_in;   // bumpMapped
  Bsdf bs;
  bs.n = 0;
  V nn = dgs.n, sn = normalize(dgs.dpdu);
  bs.cs = LC{sn, cross(nn, sn), nn};
  bs.p = dgs.p;
  bs.ng = dgg.n;
  const bling_material& m = d->materials[mi];
  auto tex = [&](int k) { return eval_spectrum(d, m.tex[k], dgs); };
  switch (m.kind) {
    case BLING_MAT_MATTE: {
      S r = tex(0);
      float s = m.scalar[0];
      BxDF b{};
      b.r = r;
      if (s == 0.f) { b.kind = K_LAMB; b.flags = B_REFL | B_DIFF; }
      else {
        b.kind = K_OREN; b.flags = B_REFL | B_DIFF;
        float sg = clampf(s, 0.f, 1.f); float sig2 = sg * sg;
        b.A = 1.f - (sig2 / (2.f * (sig2 + 0.33f)));
        b.B = 0.45f * sig2 / (sig2 + 0.09f);
      }
      bs.b[bs.n++] = b;
      break;
    }
    case BLING_MAT_PLASTIC: {
      BxDF df{}; df.kind = K_LAMB; df.flags = B_REFL | B_DIFF; df.r = tex(0);
      BxDF sp{}; sp.kind = K_MICRO; sp.flags = B_REFL | B_GLOSSY; sp.r = tex(1);
      sp.e = fix_exponent(1.f / m.scalar[0]);
      sp.fr.kind = FR_DIEL; sp.fr.ei = 1.0f; sp.fr.et = 1.5f;
      bs.b[bs.n++] = df; bs.b[bs.n++] = sp;
      break;
    }
    case BLING_MAT_GLASS: {
      float ior = m.scalar[0];
      BxDF rf{}; rf.kind = K_SREFL; rf.flags = B_REFL | B_SPEC; rf.r = sclamp(tex(0), 0.f, 1.f);
      rf.fr.kind = FR_DIEL; rf.fr.ei = 1.f; rf.fr.et = ior;
      BxDF tr{}; tr.kind = K_STRANS; tr.flags = B_TRANS | B_SPEC; tr.r = sclamp(tex(1), 0.f, 1.f);
      tr.ei = 1.f; tr.et = ior;
      bs.b[bs.n++] = rf; bs.b[bs.n++] = tr;
      break;
    }
    case BLING_MAT_METAL: {
      BxDF sp{}; sp.kind = K_MICRO; sp.flags = B_REFL | B_GLOSSY; sp.r = white();
      sp.e = fix_exponent(1.f / m.scalar[0]);
      sp.fr.kind = FR_COND; sp.fr.eta = tex(0); sp.fr.k = tex(1);
      bs.b[bs.n++] = sp;
      break;
    }
    case BLING_MAT_TRANSMATTE: {                       // translucentMatte (Material.hs:43-53)
      S r = tex(0), t = tex(1);                          // sClamp'd kr and sClamp kt * (white - r), folded at load
      float s = m.scalar[0];
      BxDF rf{}, tr{};
      rf.r = r; tr.r = t;
      if (s == 0.f) { rf.kind = K_LAMB; tr.kind = K_LAMB; }
      else {
        float sg = clampf(s, 0.f, 1.f); float sig2 = sg * sg;
        rf.kind = K_OREN; rf.A = 1.f - (sig2 / (2.f * (sig2 + 0.33f))); rf.B = 0.45f * sig2 / (sig2 + 0.09f);
        tr.kind = K_OREN; tr.A = rf.A; tr.B = rf.B;
      }
      rf.flags = B_REFL | B_DIFF;
      tr.flags = B_TRANS | B_DIFF; tr.btdf = true;       // bxdfTypeFlip (Reflection | Transmission)
      bs.b[bs.n++] = rf; bs.b[bs.n++] = tr;
      break;
    }
    case BLING_MAT_SHINYMETAL: {                       // mkShinyMetal (Material.hs:98-109)
      BxDF g{}; g.kind = K_MICRO; g.flags = B_REFL | B_GLOSSY; g.r = white();
      g.e = fix_exponent(1.f / m.scalar[0]);
      g.fr.kind = FR_COND; g.fr.eta = tex(0); g.fr.k = tex(1);        // frApproxEta / K of ks (host-folded)
      BxDF sp{}; sp.kind = K_SREFL; sp.flags = B_REFL | B_SPEC; sp.r = white();
      sp.fr.kind = FR_COND; sp.fr.eta = tex(2); sp.fr.k = tex(3);     // of kr
      bs.b[bs.n++] = g; bs.b[bs.n++] = sp;
      break;
    }
    case BLING_MAT_SUBSTRATE: {                        // mkSubstrate (Material.hs:111-128): one FresnelBlend lobe
      BxDF fb{}; fb.kind = K_FBLEND; fb.flags = B_REFL | B_GLOSSY;
      fb.r = tex(0); fb.rs = tex(1); fb.ra = tex(2);     // sClamp 0 1 kd / ks / ka, folded at load
      fb.e = m.scalar[0]; fb.ey = m.scalar[1];           // mkAnisotropic (1 / u) (1 / v), fixExponent'd at load
      fb.depth = m.scalar[2];
      auto max0 = [](float x) { return 0.f <= x ? x : 0.f; };                 // max 0 (GHC max)
      if (m.stex[0] >= 0) fb.e = fix_exponent(1.f / max0(eval_stex(d, m.stex[0], dgs.p, dgs.u, dgs.v)));
      if (m.stex[1] >= 0) fb.ey = fix_exponent(1.f / max0(eval_stex(d, m.stex[1], dgs.p, dgs.u, dgs.v)));
      if (m.stex[2] >= 0) fb.depth = eval_stex(d, m.stex[2], dgs.p, dgs.u, dgs.v);
      bs.b[bs.n++] = fb;
      break;
    }
    case BLING_MAT_MIRROR: {
      BxDF rf{}; rf.kind = K_SREFL; rf.flags = B_REFL | B_SPEC; rf.r = sclamp(tex(0), 0.f, 1.f);
      rf.fr.kind = FR_NOOP;
      bs.b[bs.n++] = rf;
      break;
    }
    default: break;  // blackbody: no components
  }
  return bs;
}

inline bool has_flag(const BxDF& b, int f) { return (b.flags & f) == f; }             // bxdfIs

// bsdfPdf (Reflection.hs:251-257)
float bsdf_pdf(const Bsdf& bs, V woW, V wiW) {
  if (bs.n == 0) return 0.f;
  V wo = world_to_local(bs.cs, woW), wi = world_to_local(bs.cs, wiW);
  float s = 0.f;
  for (int i = 0; i < bs.n; ++i) s = s + bxdf_pdf(bs.b[i], wo, wi);
  return s / (float)bs.n;
}

// evalBsdf False (Reflection.hs:318-332)
S eval_bsdf(const Bsdf& bs, V woW, V wiW) {
  float cosWo = dot(woW, bs.ng);
  float side = dot(wiW, bs.ng) / cosWo;
  if (side == 0.f) return black();
  if (std::fabs(cosWo) < 1e-5f) return black();
  int flt = side < 0.f ? B_TRANS : B_REFL;
  V wo = world_to_local(bs.cs, woW), wi = world_to_local(bs.cs, wiW);
  S f = black();
  for (int i = 0; i < bs.n; ++i)
    if (has_flag(bs.b[i], flt)) f = f + bxdf_eval(bs.b[i], wi, wo);
  return f;
}

struct BsdfSample { int flags; float pdf; S f; V wi; };

// sampleBsdf'' False flags (Reflection.hs:278-316); bsm = the BxDFs whose type is within `flags`
// (bxdfMatches, :185-186).  sample_bsdf = sampleBsdf (flags = bxdfAll).
// adj = sampleAdjBsdf: the BxDF sampled adjointly, the other lobes evaluated unflipped and the
// result scaled by |sideTest| (fAdj, :299-316).
BsdfSample sample_bsdf_t(const Bsdf& bs, int flags, V woW, float uc, float u1, float u2, bool adj = false) {
  BsdfSample empty{B_REFL | B_DIFF, 0.f, black(), mk(0.f, 1.f, 0.f)};
  int bsm[2], cntm = 0;
  for (int i = 0; i < bs.n; ++i)
    if ((bs.b[i].flags & flags) == bs.b[i].flags) bsm[cntm++] = i;
  if (cntm == 0) return empty;
  V wo = world_to_local(bs.cs, woW);
  float cntf = (float)cntm, invCnt = 1.f / cntf;
  int sIdx = std::max(0, std::min(cntm - 1, (int)std::floor(uc * cntf)));
  int sNum = bsm[sIdx];
  const BxDF& b = bs.b[sNum];
  V wi; float pdfp;
  S fs = bxdf_sample(b, wo, u1, u2, &wi, &pdfp, adj);
  if (pdfp == 0.f) return empty;
  V wiW = local_to_world(bs.cs, wi);
  float side = dot(wiW, bs.ng) / dot(woW, bs.ng);
  if (side == 0.f) return empty;
  int flt = side < 0.f ? B_TRANS : B_REFL;
  if (!has_flag(b, flt)) return empty;
  auto fadj = [&](const S& f) { return adj ? sscale(f, std::fabs(side)) : f; };
  if (has_flag(b, B_SPEC)) return BsdfSample{b.flags, pdfp * invCnt, fadj(sscale(fs, cntf)), wiW};
  if (cntm == 1) return BsdfSample{b.flags, pdfp, fadj(fs), wiW};
  float others = 0.f;
  S fo = black();
  for (int q = 0; q < cntm; ++q) {
    int i = bsm[q];
    if (i == sNum) continue;
    others = others + bxdf_pdf(bs.b[i], wo, wi);
    if (has_flag(bs.b[i], flt)) fo = fo + (adj ? bxdf_eval(bs.b[i], wo, wi) : bxdf_eval(bs.b[i], wi, wo));
  }
  float pdf = (pdfp + others) * invCnt;
  S fsum = sscale(sscale(fs, pdfp) + fo, 1.f / pdf);
  return BsdfSample{b.flags, pdf, fadj(fsum), wiW};
}
constexpr int B_ALL = B_REFL | B_TRANS | B_DIFF | B_GLOSSY | B_SPEC;                    // bxdfAll (:160-161)
BsdfSample sample_bsdf(const Bsdf& bs, V woW, float uc, float u1, float u2) {
  return sample_bsdf_t(bs, B_ALL, woW, uc, u1, u2);
}

// ======================================================================= lights (Light.hs)
struct LightSample { S li; V wi; Ray ray; float pdf; bool delta = false; };

// sampleContinuous1D / 2D (Montecarlo.hs:67-94)
int upper_bound(const float* cdf, int nv, float u) {
  int idx = nv - 1;
  for (int i = 0; i < nv; ++i) if (cdf[i] >= u) { idx = i - 1; break; }
  idx = std::max(0, idx);
  return std::min(nv - 2, idx);
}
float sample_c1d(const float* func, const float* cdf, float fi, int n, float u, float* pdf, int* off_out) {
  int off = upper_bound(cdf, n + 1, u);
  *pdf = fi == 0.f ? 0.f : func[off] / fi;
  float du = (u - cdf[off]) / (cdf[off + 1] - cdf[off]);
  *off_out = off;
  return ((float)off + du) / (float)n;
}
void sample_c2d(const bling_light& L, float u0, float u1, float* u, float* v, float* pdf) {
  int nu = L.dist_nu, nv = L.dist_nv, im, dummy;
  float pdf1, pdf0;
  *v = sample_c1d(L.marg_func, L.marg_cdf, L.marg_func_int, nv, u1, &pdf1, &im);
  *u = sample_c1d(L.dist_func + (size_t)im * nu, L.dist_cdf + (size_t)im * (nu + 1), L.dist_func_int[im], nu, u0, &pdf0, &dummy);
  *pdf = pdf0 * pdf1;
}
float pdf_d2d(const bling_light& L, float u, float v) {                                 // Montecarlo.hs:95-111
  int nu = L.dist_nu, nv = L.dist_nv;
  int iu = std::max(0, std::min(nu - 1, (int)std::floor(u * (float)nu)));
  int iv = std::max(0, std::min(nv - 1, (int)std::floor(v * (float)nv)));
  if (L.marg_func_int * L.dist_func_int[iv] == 0.f) return 0.f;
  return (L.dist_func[(size_t)iv * nu + iu] * L.marg_func[iv]) / (L.dist_func_int[iv] * L.marg_func_int);
}

// texMapEval of the infinite light's map at Cartesian (u, v)
S env_eval(const bling_light& L, float u, float v) {
  if (L.env_kind == BLING_ENV_CONSTANT) return from_array(L.env_const);
  if (L.env_kind == BLING_ENV_IMAGE)                 // rgbfToTexMap (IO/Bitmap.hs:22-29)
    return from_array(L.env_texels + 16 * bimgtex::env_texel(L.env_w, L.env_h, u, v));
  float phi = u * 2.f * PI, th = v * PI;                                                // cartToSph (Types.hs:31-33)
  float st = bcr::sinf(th), ct = bcr::cosf(th);
  V dir = mk(st * bcr::cosf(phi), st * bcr::sinf(phi), ct);                               // sphToDir (Math.hs:146-148)
  // skySpectrum + sunSpectrum (SunSky.hs:67-94)
  S sky = black();
  float dzn = -dir.z;
  if (!(dzn < 1e-4f)) {
    V sd = mk(L.sun_dir_local[0], L.sun_dir_local[1], L.sun_dir_local[2]);
    float theta = bcr::acosf(dzn), gamma = bcr::acosf(clampf(dot(dir, sd), -1.f, 1.f));
    auto perez = [&](const float* p, float lvz) {
      float csg = bcr::cosf(gamma), cst = bcr::cosf(L.sun_theta);
      float num = (1.f + p[0] * bcr::expf(p[1] / bcr::cosf(theta))) * (1.f + p[2] * bcr::expf(p[3] * gamma)) + p[4] * csg * csg;
      float den = (1.f + p[0] * bcr::expf(p[1])) * (1.f + p[2] * bcr::expf(p[3] * L.sun_theta)) + p[4] * cst * cst;
      return lvz * num / den;
    };
    float x = perez(L.perez_x, L.zenith_x), y = perez(L.perez_y, L.zenith_y);
    float yy = perez(L.perez_Y, L.zenith_Y) * 1e-4f;
    float dn = 0.0241f + 0.2562f * x - 0.7341f * y;                                     // chromaticityToXYZ
    float m1 = (-1.3515f - 1.7703f * x + 5.9114f * y) / dn, m2 = (0.03f - 31.4424f * x + 30.0717f * y) / dn;
    float cx = BLING_S_XYZ[0][0] + m1 * BLING_S_XYZ[1][0] + m2 * BLING_S_XYZ[2][0];
    float cy = BLING_S_XYZ[0][1] + m1 * BLING_S_XYZ[1][1] + m2 * BLING_S_XYZ[2][1];
    float cz = BLING_S_XYZ[0][2] + m1 * BLING_S_XYZ[1][2] + m2 * BLING_S_XYZ[2][2];
    float X = cx * yy / cy, Y = yy, Z = cz * yy / cy;
    float r = 3.240479f * X - 1.537150f * Y - 0.498535f * Z;                            // xyzToRgb
    float g = (-0.969256f) * X + 1.875991f * Y + 0.041556f * Z;
    float b = 0.055648f * X - 0.204043f * Y + 1.057311f * Z;
    const float (*B)[16] = BLING_RGB_ILLUM_BANDS;                                       // rgbToSpectrumIllum
    auto bs2 = [&](int k, float f) { return sscale(from_array(B[k]), f); };
    if (r <= g && r <= b) sky = bs2(6, r) + (g <= b ? bs2(3, g - r) + bs2(2, b - g) : bs2(3, b - r) + bs2(1, g - b));
    else if (g <= r && g <= b) sky = bs2(6, g) + (r <= b ? bs2(4, r - g) + bs2(2, b - r) : bs2(4, b - g) + bs2(0, r - b));
    else sky = bs2(6, b) + (r <= b ? bs2(5, r - b) + bs2(1, g - r) : bs2(5, g - b) + bs2(0, r - g));
  }
  float d = (L.sun_dir_local[0] * 1.f) * dir.x + (L.sun_dir_local[1] * 1.f) * dir.y + (L.sun_dir_local[2] * -1.f) * dir.z;
  float stm = std::sqrt(hmax(0.f, 1.f - 6.955e5f / 1.496e8f));
  S sun = d > stm ? from_array(L.sun_radiance) : black();
  return sky + sun;
}

// dirToSph -> sphToCart (Math.hs:150-169, Types.hs:35-39)
inline void dir_to_uv(V w, float* u, float* v, float* sint) {
  float p = bcr::atan2f(w.y, w.x);
  if (p < 0.f) p = p + 2.f * PI;
  float th = bcr::acosf(hmax(-1.f, hmin(1.f, w.z)));
  *u = p / (2.f * PI);
  *v = th / PI;
  *sint = bcr::sinf(th);
}

S light_le(const bling_light& L, const Ray& r) {                                        // Light.hs:98-106
  if (L.kind != BLING_LIGHT_INFINITE) return black();
  V wh = normalize(xvector(L.w2l, r.d));
  float u, v, st;
  dir_to_uv(wh, &u, &v, &st);
  return env_eval(L, u, v);
}

// generalPdf / shapePdf (Shape.hs:333-350)
float shape_pdf(const bling_shape& s, V p, V wi) {
  if (s.kind == BLING_SHAPE_SPHERE) {
    float r = s.params[0];
    if (!(sqlen(p) - r * r < 1e-4f)) {
      float stm2 = r * r / sqlen(p);
      return uniform_cone_pdf(std::sqrt(hmax(0.f, 1.f - stm2)));
    }
  }
  Ray ray{p, wi, 1e-3f, INF};
  float t, eps;
  DG dg;
  if (!shape_intersect_local(s, ray, &t, &eps, &dg)) return 0.f;
  float pd = sqlen(p - ray_at(ray, t)) / (absdot(dg.n, -wi) * shape_area(s));
  return std::isinf(pd) ? 0.f : pd;
}

// remapRand (Math.hs:113-121)
inline void remap_rand(int segs, float u, int* seg, float* up) {
  float segsf = (float)segs;
  *seg = std::min(segs - 1, (int)std::floor(u * segsf));
  *up = (u - (float)*seg / segsf) * segsf;
}

// sampleShape (Shape.hs:362-409)
void sample_shape(const bling_shape& s, V p, float u1, float u2, V* ps, V* ns) {
  const float* P = s.params;
  if (s.kind == BLING_SHAPE_DISK) {                                                    // :400-403
    float r = lerp(u1, P[2], P[1]), phi = lerp(u2, 0.f, P[3]);
    *ps = mk(r * bcr::cosf(phi), r * bcr::sinf(phi), P[0]);
    *ns = mk(0.f, 0.f, -1.f);
    return;
  }
  if (s.kind == BLING_SHAPE_CYLINDER) {                                                // :394-398
    float z = lerp(u1, P[1], P[2]), phi = lerp(u2, 0.f, TWO_PI);
    *ps = mk(P[0] * bcr::cosf(phi), P[0] * bcr::sinf(phi), z);
    *ns = normalize(mk(ps->x, ps->y, 0.f));
    return;
  }
  if (s.kind == BLING_SHAPE_BOX) {                                                     // :384-392
    int axis, nf; float u1p, u2p;
    remap_rand(3, u1, &axis, &u1p);
    remap_rand(2, u2, &nf, &u2p);
    V pmin = mk(P[0], P[1], P[2]), pmax = mk(P[3], P[4], P[5]);
    *ns = set_comp(axis, (float)nf * 2.f - 1.f, mk(0.f, 0.f, 0.f));
    int oa0 = (axis + 1) % 3, oa1 = (axis + 2) % 3;
    V q = nf == 0 ? pmin : pmax;
    q = set_comp(oa1, lerp(u2p, comp(pmin, oa1), comp(pmax, oa1)), q);
    q = set_comp(oa0, lerp(u1p, comp(pmin, oa0), comp(pmax, oa0)), q);
    *ps = q;
    return;
  }
  if (s.kind == BLING_SHAPE_QUAD) {
    *ps = mk(lerp(u1, -s.params[0], s.params[0]), lerp(u2, -s.params[1], s.params[1]), 0.f);
    *ns = mk(0.f, 0.f, -1.f);
    return;
  }
  float r = s.params[0];
  if (sqlen(p) - r * r < 1e-4f) { V q = uniform_sample_sphere(u1, u2); *ps = vs(q, r); *ns = q; return; }
  V dn = normalize(-p);
  LC cs = coordinate_system(dn);
  float cosmax = std::sqrt(hmax(0.f, 1.f - (r * r) / sqlen(p)));
  V dd = uniform_sample_cone(cs, cosmax, u1, u2);
  Ray ray{p, dd, 0.f, INF};
  float t, eps;
  DG dg;
  V q = shape_intersect_local(s, ray, &t, &eps, &dg) ? ray_at(ray, t) : vs(dn, r);
  *ps = q;
  *ns = normalize(q);
}

// sample (Light.hs:122-160); n = the shading normal (bsdfShadingNormal) the directional light's
// cosine uses
LightSample light_sample(const Scene& Sc, const bling_light& L, V pW, V n, float eps, float u1, float u2) {
  LightSample ls;
  if (L.kind == BLING_LIGHT_DIRECTIONAL) {                                              // Light.hs:143-145
    const V d = mk(L.delta_vec[0], L.delta_vec[1], L.delta_vec[2]);
    ls.li = sscale(from_array(L.radiance), std::fabs(dot(n, d)));                        // absDot n d
    ls.wi = d;
    ls.ray = Ray{pW, d, eps, INF};
    ls.pdf = 1.f;
    ls.delta = true;
    return ls;
  }
  if (L.kind == BLING_LIGHT_POINT) {                                                    // Light.hs:147-150
    const V pos = mk(L.delta_vec[0], L.delta_vec[1], L.delta_vec[2]);
    ls.li = sscale(from_array(L.radiance), 1.f / sqlen(pos - pW));
    ls.wi = normalize(pos - pW);
    ls.ray = Ray{pW, pos - pW, eps, INF};     // unnormalised direction, no tmax: trap T19
    ls.pdf = 1.f;
    ls.delta = true;
    return ls;
  }
  if (L.kind == BLING_LIGHT_AREA) {
    const bling_shape& s = Sc.d->shapes[L.shape];
    V p = xpoint(s.w2o, pW);
    V ps, ns;
    sample_shape(s, p, u1, u2, &ps, &ns);
    V wi = normalize(ps - p);
    ls.li = dot(ns, wi) < 0.f ? from_array(L.radiance) : black();
    ls.wi = xvector(s.o2w, wi);
    ls.pdf = shape_pdf(s, p, wi);
    Ray rl{p, wi, eps, len(ps - p) - eps};
    ls.ray = Ray{xpoint(s.o2w, rl.o), xvector(s.o2w, rl.d), rl.tmin, rl.tmax};
    return ls;
  }
  float u, v, mpdf;
  sample_c2d(L, u1, u2, &u, &v, &mpdf);
  float th = v * PI, phi = u * 2.f * PI;
  float sint = bcr::sinf(th);
  if (mpdf == 0.f || sint == 0.f) {
    ls.li = black(); ls.wi = mk(0.f, 1.f, 0.f); ls.ray = Ray{mk(0, 0, 0), mk(0, 1, 0), 0.f, 1.f}; ls.pdf = 0.f;
    return ls;
  }
  ls.li = env_eval(L, u, v);
  V dl = mk(sint * bcr::cosf(phi), sint * bcr::sinf(phi), bcr::cosf(th));
  ls.wi = xvector(L.l2w, dl);
  ls.ray = Ray{pW, ls.wi, eps, INF};
  ls.pdf = mpdf / (2.f * PI * PI * sint);
  return ls;
}

// pdf (Light.hs:215-229)
float light_pdf(const Scene& Sc, const bling_light& L, V p, V wi) {
  if (L.kind == BLING_LIGHT_POINT || L.kind == BLING_LIGHT_DIRECTIONAL) return 0.f;     // Light.hs:225, 229
  if (L.kind == BLING_LIGHT_AREA) {
    const bling_shape& s = Sc.d->shapes[L.shape];
    return shape_pdf(s, xpoint(s.w2o, p), xvector(s.w2o, wi));
  }
  V w = xvector(L.w2l, wi);
  float u, v, st;
  dir_to_uv(w, &u, &v, &st);
  if (st == 0.f) return 0.f;
  return pdf_d2d(L, u, v) / (2.f * PI * PI * st);
}

// intLe (Primitive.hs:68-76) -> lEmit (Light.hs:85-96)
S int_le(const Scene& Sc, const Hit& h, V wo) {
  const Prim& p = Sc.prims[h.prim];
  if (p.kind != 1) return black();
  const bling_shape& s = Sc.d->shapes[p.index];
  if (s.light < 0) return black();
  const bling_light& L = Sc.d->lights[s.light];
  return dot(h.dg.n, wo) > 0.f ? from_array(L.radiance) : black();
}
int hit_light(const Scene& Sc, const Hit& h) {                                          // intLight
  const Prim& p = Sc.prims[h.prim];
  if (p.kind != 1) return -1;
  return Sc.d->shapes[p.index].light;
}

// ======================================================================= sampler (counter RNG)
// One sample's sampler: the job's (sample_ctx), or SPPM's own random 1-spp camera sampler and
// sn x sn stratified photon sampler (SPPM.hs:150, 442).
struct SamplerCfg { int sampler, nu, nv; };

// ----------------------------------------------------------------------- MWC sampler mode
// The reference's own sampler, restated for the statistical convergence test only (the product and
// the per-sample parity checks use the counter RNG above).  Generator: mwc-random's MWC8222
// (Marsaglia's lag-256 multiply-with-carry, a = 1540315826), the third-party package the reference
// takes from Stackage lts-8.13 (/root/reference/stack.yaml:18, mwc-random 0.13.x; not vendored):
// uniformWord32 / wordToFloat / Int = two words high-first, as that package publishes them.  The
// reference seeds every tile of every pass from the system entropy source (ioSeed,
// Rendering.hs:127-128, Random.hs:61-62); here a tile's 256-word state is filled from the counter
// hash of (seed, pass, tile origin), so a run is reproducible.
struct Mwc {
  uint32_t q[256], i = 255, c = 362436;
  Mwc(uint32_t seed, uint32_t pass, uint32_t key) {
    for (uint32_t k = 0; k < 256; ++k) q[k] = hash5(seed, pass, key, k, 0x4D574321u);
  }
  uint32_t word() {                                      // uniformWord32 (MWC8222)
    i = (i + 1) & 255u;
    uint64_t t = 1540315826ull * q[i] + c;
    uint32_t cc = (uint32_t)(t >> 32), x = (uint32_t)t + cc;
    if (x < cc) { x++; cc++; }
    q[i] = x; c = cc;
    return x;
  }
  float uniform() {                                      // wordToFloat: (0, 1], Float arithmetic
    float v = (float)(int32_t)word() * 2.3283064365386962890625e-10f;
    v = v + 0.5f;
    return v + 1.16415321826934814453125e-10f;
  }
  float rnd() { return uniform() - 1.16415321826934814453125e-10f; }  // rnd (Random.hs:92-96)
  int64_t rnd_int() {                                    // rndInt = uniform :: Int (Random.hs:98-100)
    uint64_t hi = word(), lo = word();
    return (int64_t)((hi << 32) | lo);
  }
  template <class T> void shuffle(std::vector<T>& v) {   // shuffle (Random.hs:79-89), modulus n - 1
    int64_t n = (int64_t)v.size();
    if (n < 2) return;
    for (int64_t k = 0; k < n; ++k) {
      int64_t o = rnd_int();
      int64_t a = o < 0 ? (int64_t)(0 - (uint64_t)o) : o;
      std::swap(v[k], v[a % (n - 1)]);
    }
  }
  std::vector<float> stratified1D(int n) {               // Sampling.hs:157-161 (rndVec: no 2^-33 shift)
    std::vector<float> x(n);
    for (int k = 0; k < n; ++k) x[k] = uniform();
    float du = 1.f / (float)n;
    for (int k = 0; k < n; ++k) x[k] = std::min(ALMOST_ONE, ((float)k + x[k]) * du);
    return x;
  }
  std::vector<std::pair<float, float>> stratified2D(int nu, int nv) {   // Sampling.hs:164-171
    int n = nu * nv;
    std::vector<float> ju(n), jv(n);
    for (int k = 0; k < n; ++k) ju[k] = uniform();       // rndVec2D: all u, then all v
    for (int k = 0; k < n; ++k) jv[k] = uniform();
    float du = 1.f / (float)nu, dv = 1.f / (float)nv;
    std::vector<std::pair<float, float>> r(n);
    for (int k = 0; k < n; ++k) {
      int u = k / nu, v = k % nu;                        // quotRem i nu (trap T5)
      r[k] = {std::min(ALMOST_ONE, ((float)u + ju[k]) * du), std::min(ALMOST_ONE, ((float)v + jv[k]) * dv)};
    }
    return r;
  }
};
// One pixel's precomputed stratified sample (runSample Stratified, Sampling.hs:112-132; fill 134-150): pixel
// offsets, shuffled lens strata and the fill'ed v1d / v2d tables, plus the tile's generator for
// every fresh draw past them.
struct MwcPixel {
  Mwc* g;
  std::vector<std::pair<float, float>> ps, lens, v2d;
  std::vector<float> v1d;
};

struct SampleCtx {
  const Scene* S;
  uint32_t seed, pass, pixel, n;
  int n1d, n2d;
  SamplerCfg cfg;
  MwcPixel* mwc = nullptr;
};
float rnd1(const SampleCtx& c, int dim) {                                               // rnd' (Sampling.hs:203-211)
  const SamplerCfg& cfg = c.cfg;
  if (c.mwc) {
    if (cfg.sampler == BLING_SAMPLER_STRATIFIED && dim < c.n1d) return c.mwc->v1d[(size_t)c.n * c.n1d + dim];
    return c.mwc->g->rnd();
  }
  if (cfg.sampler == BLING_SAMPLER_STRATIFIED && dim < c.n1d) {
    uint32_t spp = (uint32_t)(cfg.nu * cfg.nv);
    uint32_t k = permute(c.n, spp, hash5(c.seed, c.pass, c.pixel, ALL_SAMPLES, DIM_1D_PERM + dim));
    float j = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_1D_J + dim));         // jitter: sample key (spec v2)
    return std::min(ALMOST_ONE, ((float)k + j) * (1.f / (float)spp));                   // stratified1D
  }
  return u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_FRESH1D + dim));
}
void rnd2(const SampleCtx& c, int dim, float* a, float* b) {                            // rnd2D' (Sampling.hs:213-221)
  const SamplerCfg& cfg = c.cfg;
  if (c.mwc) {
    if (cfg.sampler == BLING_SAMPLER_STRATIFIED && dim < c.n2d) {
      const auto& p = c.mwc->v2d[(size_t)c.n * c.n2d + dim];
      *a = p.first; *b = p.second;
    } else {
      *a = c.mwc->g->rnd(); *b = c.mwc->g->rnd();                                        // rnd2D (Random.hs:137-139)
    }
    return;
  }
  if (cfg.sampler == BLING_SAMPLER_STRATIFIED && dim < c.n2d) {
    uint32_t spp = (uint32_t)(cfg.nu * cfg.nv);
    uint32_t k = permute(c.n, spp, hash5(c.seed, c.pass, c.pixel, ALL_SAMPLES, DIM_2D_PERM + dim));
    float ju = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_2D_J + 2 * dim));
    float jv = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_2D_J + 2 * dim + 1));
    int u = (int)k / cfg.nu, v = (int)k % cfg.nu;                                        // quotRem i nu (trap T5)
    *a = std::min(ALMOST_ONE, ((float)u + ju) * (1.f / (float)cfg.nu));
    *b = std::min(ALMOST_ONE, ((float)v + jv) * (1.f / (float)cfg.nv));
    return;
  }
  *a = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_FRESH2D + 2 * dim));
  *b = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_FRESH2D + 2 * dim + 1));
}
// camera sample: pixel offsets (unshuffled stratified2D) + shuffled lens strata (runSample, Sampling.hs:112-132)
void camera_sample(const SampleCtx& c, float* ox, float* oy, float* lu, float* lv) {
  const SamplerCfg& cfg = c.cfg;
  if (c.mwc) {
    if (cfg.sampler == BLING_SAMPLER_STRATIFIED) {
      *ox = c.mwc->ps[c.n].first; *oy = c.mwc->ps[c.n].second;
      *lu = c.mwc->lens[c.n].first; *lv = c.mwc->lens[c.n].second;
    } else {                                                                              // Sampling.hs:104-107
      *ox = c.mwc->g->rnd(); *oy = c.mwc->g->rnd(); *lu = c.mwc->g->rnd(); *lv = c.mwc->g->rnd();
    }
    return;
  }
  if (cfg.sampler == BLING_SAMPLER_STRATIFIED) {
    uint32_t spp = (uint32_t)(cfg.nu * cfg.nv);
    float du = 1.f / (float)cfg.nu, dv = 1.f / (float)cfg.nv;
    int u = (int)c.n / cfg.nu, v = (int)c.n % cfg.nu;
    float ju = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_PIX)), jv = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_PIX + 1));
    *ox = std::min(ALMOST_ONE, ((float)u + ju) * du);
    *oy = std::min(ALMOST_ONE, ((float)v + jv) * dv);
    uint32_t k = permute(c.n, spp, hash5(c.seed, c.pass, c.pixel, ALL_SAMPLES, DIM_LENS_PERM));
    float lj = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_LENS_J)), lk = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_LENS_J + 1));
    int lu_i = (int)k / cfg.nu, lv_i = (int)k % cfg.nu;
    *lu = std::min(ALMOST_ONE, ((float)lu_i + lj) * du);
    *lv = std::min(ALMOST_ONE, ((float)lv_i + lk) * dv);
    return;
  }
  *ox = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_RAND_CAM));                          // Random (Sampling.hs:101-110)
  *oy = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_RAND_CAM + 1));
  *lu = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_RAND_CAM + 2));
  *lv = u01(hash5(c.seed, c.pass, c.pixel, c.n, DIM_RAND_CAM + 3));
}

// fireRay (Camera.hs:49-76)
Ray fire_ray(const bling_camera& cam, float ix, float iy, float lu, float lv) {
  if (cam.kind == BLING_CAM_ENVIRONMENT) {
    float t = PI * iy / cam.yres, p = 2.f * PI * ix / cam.xres;
    V d = mk(bcr::sinf(t) * bcr::cosf(p), bcr::cosf(t), bcr::sinf(t) * bcr::sinf(p));
    return Ray{xpoint(cam.c2w, mk(0, 0, 0)), xvector(cam.c2w, d), 0.f, INF};
  }
  V pc = xpoint(cam.r2c, mk(ix, iy, 0.f));
  Ray r{mk(0.f, 0.f, 0.f), normalize(pc), 0.f, INF};
  if (cam.lens_radius > 0.f) {
    float dx, dy;
    concentric_sample_disk(lu, lv, &dx, &dy);
    V ro = mk(dx * cam.lens_radius, dy * cam.lens_radius, 0.f);
    V pf = ray_at(r, cam.focal_distance / r.d.z);
    r = Ray{ro, normalize(pf - ro), 0.f, INF};
  }
  return Ray{xpoint(cam.c2w, r.o), xvector(cam.c2w, r.d), r.tmin, r.tmax};
}

// ======================================================================= integrator (Integrator/Path.hs)
struct Counters { uint64_t cam = 0, cont = 0, mis = 0, shadow = 0; TStats ts; };

// Per-vertex debug record of one sample (oracle_sample_li_vertices; the device's counterpart is
// bling_sample_li_vertices of a BLING_DEBUG_VERTEX build): DV_FIELDS floats per path vertex, in the
// order the vertex computes them, so the first field where device and oracle part names the first
// diverging operation.  Field map: include/bling.h BLING_DV_*.
constexpr int DV_DEPTHS = 16, DV_FIELDS = 32;
thread_local float* g_dv = nullptr;
inline void dvrec(int depth, int f, float v) {
  if (g_dv && depth >= 0 && depth < DV_DEPTHS) g_dv[depth * DV_FIELDS + f] = v;
}
inline void dvrec3(int depth, int f, V v) { dvrec(depth, f, v.x); dvrec(depth, f + 1, v.y); dvrec(depth, f + 2, v.z); }
inline float ssum(const S& s) { float a = 0.f; for (int k = 0; k < 16; ++k) a += s.v[k]; return a; }

// sampleOneLight -> estimateDirect -> sampleLightMis + sampleBsdfMis (Scene.hs:61-118)
S sample_one_light(const Scene& Sc, V p, float eps, V wo, const Bsdf& bsdf, float ulNum, float ul1, float ul2,
                   float ubc, float ub1, float ub2, Counters& C, int dvd = -1) {
  int lc = (int)Sc.d->num_lights;
  if (lc == 0) return black();
  int ln = lc == 1 ? 0 : std::min((int)std::floor(ulNum * (float)lc), lc - 1);
  const bling_light& L = Sc.d->lights[ln];
  // light side
  S ls = black();
  {
    LightSample smp = light_sample(Sc, L, p, bsdf.cs.n, eps, ul1, ul2);
    dvrec3(dvd, 14, smp.wi); dvrec(dvd, 17, smp.pdf);
    if (!(smp.pdf == 0.f) && !is_black(smp.li)) {
      S f = eval_bsdf(bsdf, wo, smp.wi);
      if (!is_black(f)) {
        C.shadow++;
        const bool occl = sc_occluded(Sc, smp.ray, C.ts);
        dvrec(dvd, 28, occl ? 1.f : 0.f);
        if (!occl) {
          if (smp.delta) ls = sscale(f * smp.li, 1.f / smp.pdf);                          // Scene.hs:65
          else {
            float w = power_heuristic(smp.pdf, bsdf_pdf(bsdf, wo, smp.wi));
            ls = sscale(f * smp.li, w / smp.pdf);
          }
        }
      }
    }
  }
  // bsdf side
  S bsd = black();
  {
    BsdfSample bs = sample_bsdf(bsdf, wo, ubc, ub1, ub2);
    dvrec3(dvd, 18, bs.wi); dvrec(dvd, 21, bs.pdf);
    if (!(bs.pdf == 0.f) && !is_black(bs.f)) {
      Ray ray{p, bs.wi, eps, INF};
      C.mis++;
      Hit h;
      const bool mhit = sc_intersect(Sc, ray, &h, C.ts);
      dvrec(dvd, 29, mhit ? h.t : INF);
      if (mhit) {
        int hl = hit_light(Sc, h);
        if (hl >= 0 && L.kind == BLING_LIGHT_AREA && hl == ln) {                         // l' == l (Light.hs:48-50)
          float lpdf = light_pdf(Sc, L, p, bs.wi);
          bsd = sscale(bs.f * int_le(Sc, h, -bs.wi), power_heuristic(bs.pdf, lpdf));
        }
      } else {
        float lpdf = light_pdf(Sc, L, p, bs.wi);
        bsd = sscale(bs.f * light_le(L, ray), power_heuristic(bs.pdf, lpdf));
      }
    }
  }
  S ld = ls + bsd;
  return lc == 1 ? ld : sscale(ld, (float)lc);
}

// shading geometry + material BSDF of a hit (mkIntersection -> shadingGeometry, Primitive.hs:57-65)
Bsdf hit_bsdf(const Scene& Sc, const Hit& h) {
  DG dgs = h.dg;
  const Prim& pr = Sc.prims[h.prim];
  int mat;
  if (pr.kind == 0) {
    mat = Sc.d->tri_material[pr.index];
    if (Sc.d->tri_has_normals && Sc.d->tri_has_normals[pr.index]) {                   // triangleShadingGeometry
      const float* nn = Sc.d->tri_normals + 9 * pr.index;
      float b1 = h.dg.b1, b2 = h.dg.b2, b0 = 1.f - b1 - b2;
      V n0 = mk(nn[0], nn[1], nn[2]), n1 = mk(nn[3], nn[4], nn[5]), n2 = mk(nn[6], nn[7], nn[8]);
      V nsp = sm(b0, n0) + sm(b1, n1) + sm(b2, n2);
      V ns = normalize(nsp);
      V ssp = normalize(h.dg.dpdu);
      V tsp = cross(ssp, ns);
      V ss, ts;
      if (sqlen(tsp) > 0.f) { ss = cross(normalize(tsp), ns); ts = normalize(tsp); }
      else { LC c = coordinate_system(ns); ss = c.s; ts = c.t; }
      dgs.n = ns; dgs.dpdu = ss; dgs.dpdv = ts;
    }
  } else if (pr.kind == 1) mat = Sc.d->shapes[pr.index].material;
  else mat = Sc.d->fractal.material;
  return make_bsdf(Sc.d, mat, h.dg, dgs);
}

// li / nextVertex (Path.hs:30-87), iterative form of the same recursion
S path_li(const Scene& Sc, const SampleCtx& sc, Ray ray, Counters& C) {
  const bling_render_config& cfg = Sc.d->config;
  int md = cfg.max_depth;
  S t = white(), l = black();
  bool spec = true;
  int depth = 0;
  C.cam++;
  Hit h;
  bool hit = sc_intersect(Sc, ray, &h, C.ts);
  for (;;) {
    if (!hit) {
      if (spec) {                                                                        // :44
        S sum = black();
        for (uint32_t i = 0; i < Sc.d->num_lights; ++i) sum = sum + light_le(Sc.d->lights[i], ray);
        return l + t * sum;
      }
      return l;                                                                          // :47
    }
    if (depth == md) return l;                                                           // :51
    dvrec3(depth, 0, ray.o); dvrec3(depth, 3, ray.d); dvrec(depth, 6, h.t);
    float lNumU = rnd1(sc, 1 + 4 * depth);
    float ld1, ld2; rnd2(sc, 1 + 3 * depth, &ld1, &ld2);
    float lBc = rnd1(sc, 2 + 4 * depth);
    float lb1, lb2; rnd2(sc, 2 + 3 * depth, &lb1, &lb2);
    V rd = ray.d;
    S intl = spec ? int_le(Sc, h, rd) : black();                                          // passes rd (trap T6)
    V wo = -rd;
    Bsdf bsdf = hit_bsdf(Sc, h);
    V p = bsdf.p;
    float eps = h.eps;
    dvrec3(depth, 7, p); dvrec3(depth, 10, h.dg.n); dvrec(depth, 13, eps);
    S lhere = intl + sample_one_light(Sc, p, eps, wo, bsdf, lNumU, ld1, ld2, lBc, lb1, lb2, C, depth);
    S lp = l + t * lhere;
    dvrec(depth, 30, ssum(lhere)); dvrec(depth, 31, ssum(lp));
    float pc = depth <= 7 ? 1.f : hmin(0.75f, sY(t));                                    // :68
    float x = rnd1(sc, 3 + 4 * depth);
    dvrec(depth, 26, pc); dvrec(depth, 27, x);
    if (x > pc) return lp;
    float uc = rnd1(sc, 0 + 4 * depth);
    float ud1, ud2; rnd2(sc, 0 + 3 * depth, &ud1, &ud2);
    BsdfSample bs = sample_bsdf(bsdf, wo, uc, ud1, ud2);
    dvrec3(depth, 22, bs.wi); dvrec(depth, 25, bs.pdf);
    if (bs.pdf == 0.f || is_black(bs.f)) return lp;
    Ray nr{p, bs.wi, eps, INF};
    spec = (bs.flags & B_SPEC) == B_SPEC;
    t = sscale(bs.f * t, 1.f / pc);
    l = lp;
    depth += 1;
    ray = nr;
    C.cont++;
    hit = sc_intersect(Sc, ray, &h, C.ts);
  }
}

// directLighting / cont (Integrator/DirectLighting.hs:22-57): at every hit one light sample
// (dimensions 2d and 2d + 1) + Le towards wo, then BOTH specular continuations -- reflection, then
// transmission -- sampled with the fixed uComp 0.5, uDir (0.5, 0.5), down to maxDepth.  An escaped
// ray contributes black (the `maybe black` at :23, even with infinite lights).
S direct_li(const Scene& Sc, const SampleCtx& sc, const Ray& ray, int d, Counters& C) {
  const int md = Sc.d->config.max_depth;
  Hit h;
  if (!sc_intersect(Sc, ray, &h, C.ts)) return black();
  float uln = rnd1(sc, 2 * d);
  float ul1, ul2; rnd2(sc, 2 * d, &ul1, &ul2);
  float ubc = rnd1(sc, 1 + 2 * d);
  float ub1, ub2; rnd2(sc, 1 + 2 * d, &ub1, &ub2);
  Bsdf bsdf = hit_bsdf(Sc, h);
  V p = bsdf.p, wo = -ray.d;
  float e = h.eps;
  S l = sample_one_light(Sc, p, e, wo, bsdf, uln, ul1, ul2, ubc, ub1, ub2, C);
  S cs[2] = {black(), black()};
  const int types[2] = {B_SPEC | B_REFL, B_SPEC | B_TRANS};
  for (int c = 0; c < 2; ++c) {                                                          // cont (:47-57)
    if (d + 1 == md) continue;
    BsdfSample bs = sample_bsdf_t(bsdf, types[c], wo, 0.5f, 0.5f, 0.5f);
    if (bs.pdf == 0.f) continue;
    C.cont++;
    cs[c] = bs.f * direct_li(Sc, sc, Ray{p, bs.wi, e, INF}, d + 1, C);
  }
  return l + cs[0] + cs[1] + int_le(Sc, h, wo);
}

S sample_li(const Scene& Sc, const SampleCtx& sc, const Ray& r, Counters& C) {
  if (Sc.d->config.integrator == BLING_INTEGRATOR_DIRECT) { C.cam++; return direct_li(Sc, sc, r, 0, C); }
  return path_li(Sc, sc, r, C);
}

// sampler dimensions the integrator requests: Path 4 sd / 3 sd (Path.hs:26-28), DirectLighting
// 2 md / 2 md (DirectLighting.hs:17-18)
SampleCtx sample_ctx(const Scene& Sc, uint32_t seed, uint32_t pass) {
  const bling_render_config& cfg = Sc.d->config;
  const SamplerCfg smp{cfg.sampler, cfg.nu, cfg.nv};
  if (cfg.integrator == BLING_INTEGRATOR_DIRECT) return SampleCtx{&Sc, seed, pass, 0, 0, 2 * cfg.max_depth, 2 * cfg.max_depth, smp};
  return SampleCtx{&Sc, seed, pass, 0, 0, 4 * cfg.sample_depth, 3 * cfg.sample_depth, smp};
}

// ======================================================================= film (Image.hs)
struct TileImg { int ox, oy, w, h; std::vector<float> px; };

void add_sample(TileImg& T, const bling_filter& F, float sx, float sy, const S& ss, uint64_t& dropped) {
  if (s_nan(ss) || s_inf(ss)) { dropped++; return; }                                     // Image.hs:253-256
  float smx, smy, smz;
  to_xyz(ss, &smx, &smy, &smz);
  float fw = F.width, fh = F.height;
  float ifw = 1.f / fw, ifh = 1.f / fw;                                                  // trap T12
  float dx = sx - 0.5f, dy = sy - 0.5f;
  int x0 = std::max(T.ox, (int)std::ceil(dx - fw)), x1 = std::min(T.ox + T.w - 1, (int)std::floor(dx + fw));
  int y0 = std::max(T.oy, (int)std::ceil(dy - fh)), y1 = std::min(T.oy + T.h - 1, (int)std::floor(dy + fh));
  if (x1 - x0 < 0 || y1 - y0 < 0) return;
  int ifx[64], ify[64];
  for (int x = x0; x <= x1; ++x) ifx[x - x0] = std::min((int)std::floor(std::fabs(((float)x - dx) * ifw * 16.f)), 15);
  for (int y = y0; y <= y1; ++y) ify[y - y0] = std::min((int)std::floor(std::fabs(((float)y - dy) * ifh * 16.f)), 15);
  for (int y = y0; y <= y1; ++y)
    for (int x = x0; x <= x1; ++x) {
      float* o = &T.px[4 * ((x - T.ox) + (y - T.oy) * T.w)];
      float fltw = F.table[ify[y - y0] * 16 + ifx[x - x0]];
      o[0] = o[0] + fltw;
      o[1] = o[1] + smx * fltw;
      o[2] = o[2] + smy * fltw;
      o[3] = o[3] + smz * fltw;
    }
}

void setup_extent(Scene& Sc) {
  const bling_scene_desc* d = Sc.d;
  float fw = d->filter.width, fh = d->filter.height;
  int W = d->config.width, H = d->config.height;
  Sc.ex0 = (int)std::floor(0.5f - fw);                                                   // Image.hs:162-168
  Sc.ex1 = (int)std::floor(0.5f + (float)W + fw);
  Sc.ey0 = (int)std::floor(0.5f - fh);
  Sc.ey1 = (int)std::floor(0.5f + (float)H + fh);
  Sc.tiles.clear();
  for (int y = Sc.ey0; y <= Sc.ey1; y += 16)                                              // splitWindow (Sampling.hs:55-58)
    for (int x = Sc.ex0; x <= Sc.ex1; x += 16) Sc.tiles.push_back(Scene::Tile{x, std::min(x + 15, Sc.ex1), y, std::min(y + 15, Sc.ey1)});
}

TileImg make_tile(const Scene& Sc, const Scene::Tile& w) {                               // mkImageTile (Image.hs:108-120)
  float fw = Sc.d->filter.width, fh = Sc.d->filter.height;
  TileImg T;
  T.ox = std::max(0, w.x0); T.oy = std::max(0, w.y0);
  T.w = w.x1 - T.ox + (int)std::floor(0.5f + fw);
  T.h = w.y1 - T.oy + (int)std::floor(0.5f + fh);
  T.px.assign((size_t)std::max(0, T.w) * std::max(0, T.h) * 4, 0.f);
  return T;
}

void render_tile(const Scene& Sc, const Scene::Tile& w, uint32_t seed, uint32_t pass, TileImg& T, Counters& C,
                 uint64_t& samples, uint64_t& dropped) {
  const bling_render_config& cfg = Sc.d->config;
  int spp = cfg.spp;
  int extW = Sc.ex1 - Sc.ex0 + 1;
  SampleCtx sc = sample_ctx(Sc, seed, pass);
  std::unique_ptr<Mwc> gen;
  MwcPixel mp;
  if (Sc.rng == ORACLE_RNG_MWC) {
    gen.reset(new Mwc(seed, pass, (uint32_t)((w.y0 - Sc.ey0) * extW + (w.x0 - Sc.ex0))));
    mp.g = gen.get();
    sc.mwc = &mp;
  }
  const bool strat = cfg.sampler == BLING_SAMPLER_STRATIFIED;
  for (int iy = w.y0; iy <= w.y1; ++iy)                                                  // coverWindow: y outer
    for (int ix = w.x0; ix <= w.x1; ++ix) {
      sc.pixel = (uint32_t)((iy - Sc.ey0) * extW + (ix - Sc.ex0));
      if (sc.mwc && strat) {                                         // runSample Stratified, per pixel
        const int nu = cfg.nu, nv = cfg.nv, ns = nu * nv;
        mp.ps = gen->stratified2D(nu, nv);
        mp.lens = gen->stratified2D(nu, nv);
        gen->shuffle(mp.lens);
        mp.v1d.assign((size_t)ns * sc.n1d, 0.f);                     // fill v1d n1d spp (stratified1D spp)
        for (int off = 0; off < sc.n1d; ++off) {
          std::vector<float> rs = gen->stratified1D(ns);
          gen->shuffle(rs);
          for (int k = 0; k < ns; ++k) mp.v1d[(size_t)k * sc.n1d + off] = rs[k];
        }
        mp.v2d.assign((size_t)ns * sc.n2d, {0.f, 0.f});              // fill v2d n2d spp (stratified2D nu nv)
        for (int off = 0; off < sc.n2d; ++off) {
          auto rs = gen->stratified2D(nu, nv);
          gen->shuffle(rs);
          for (int k = 0; k < ns; ++k) mp.v2d[(size_t)k * sc.n2d + off] = rs[k];
        }
      }
      for (int n = 0; n < spp; ++n) {
        sc.n = (uint32_t)n;
        float ox, oy, lu, lv;
        camera_sample(sc, &ox, &oy, &lu, &lv);
        float imx = (float)ix + ox, imy = (float)iy + oy;
        Ray r = fire_ray(Sc.d->camera, imx, imy, lu, lv);
        S L = sample_li(Sc, sc, r, C);
        add_sample(T, Sc.d->filter, imx, imy, L, dropped);
        samples++;
      }
    }
}


// ======================================================================= SPPM (Renderer/SPPM.hs)
// Counter-RNG keys of the SPPM renderer (common/counter_rng.h): the eye pass is a random 1-spp
// sampler whose sequential rnd / rnd2D draws of followCam (SPPM.hs:91-92) are keyed by the heap id
// of the ray-tree child they start (root 1, child 2 id + {0 refl, 1 trans}); the photon pass keys
// "thread" k's sn x sn stratified sampler (SPPM.hs:441-443) with pixel SPPM_PHOTON_PIXEL | k.
constexpr uint32_t DIM_SPPM_1D = 0x100000u, DIM_SPPM_2D = 0x200000u, SPPM_PHOTON_PIXEL = 0x80000000u;

// SPPM.hs:56-62; key = pixel << 24 | heap id of the eye-tree node: a hit point's identity, which
// breaks ties of the kd-tree's median split (sppm_kd_build)
struct HitPoint { Bsdf bsdf; float px, py, r2; V w; S f; uint64_t key; };

inline bool has_non_specular(const Bsdf& b) {                                            // bsdfHasNonSpecular
  for (int i = 0; i < b.n; ++i) if (!has_flag(b.b[i], B_SPEC)) return true;
  return false;
}

// sIdx (SPPM.hs:266-270): row stride xEnd - xStart (one less than the window width) and the
// column/row clamp against that width / height, restated literally
inline int64_t sppm_sidx(const Scene& Sc, float px, float py) {
  int64_t w = Sc.ex1 - Sc.ex0, h = Sc.ey1 - Sc.ey0;
  int64_t ix = std::min<int64_t>(w, (int64_t)px), iy = std::min<int64_t>(h, (int64_t)py);   // truncate
  return w * (iy - Sc.ey0) + (ix - Sc.ex0);
}

struct EyeCtx {
  const Scene* Sc;
  uint32_t seed, pass, pixel;
  float px, py, r2;
  std::vector<HitPoint>* hps;
  uint64_t rays;
};

S trace_cam(EyeCtx& E, const Ray& ray, int depth, uint32_t id, const S& t);

// followCam (SPPM.hs:89-103): sampleBsdf' {prop, Specular}; the child keeps the node's state except
// depth, throughput and ray, so a rejected sample contributes the (always black) incoming csLs
S follow_cam(EyeCtx& E, int prop, const Hit& h, const Bsdf& bsdf, V wo, int depth, uint32_t id, const S& t) {
  const uint32_t cid = 2u * id + (prop == B_TRANS ? 1u : 0u);
  float bc = u01(hash5(E.seed, E.pass, E.pixel, 0u, DIM_SPPM_1D + cid));
  float b1 = u01(hash5(E.seed, E.pass, E.pixel, 0u, DIM_SPPM_2D + 2u * cid));
  float b2 = u01(hash5(E.seed, E.pass, E.pixel, 0u, DIM_SPPM_2D + 2u * cid + 1u));
  BsdfSample bs = sample_bsdf_t(bsdf, prop | B_SPEC, wo, bc, b1, b2);
  if (bs.pdf == 0.f || is_black(bs.f)) return black();
  return trace_cam(E, Ray{bsdf.p, bs.wi, h.eps, INF}, depth + 1, cid, bs.f * t);
}

// traceCam (SPPM.hs:105-131): records a hit point at every hit whose BSDF has a non-specular lobe,
// then follows the specular reflection and transmission children; Le is taken towards the ray
// direction (intLe int (-wo), :122) and an escaped ray adds t * sum (le lights) (:74-75, 116)
S trace_cam(EyeCtx& E, const Ray& ray, int depth, uint32_t id, const S& t) {
  const Scene& Sc = *E.Sc;
  if (depth == Sc.d->config.max_depth) return black();
  E.rays++;
  Hit h;
  TStats ts;
  if (!sc_intersect(Sc, ray, &h, ts)) {
    S sum = black();
    for (uint32_t i = 0; i < Sc.d->num_lights; ++i) sum = sum + light_le(Sc.d->lights[i], ray);
    return black() + t * sum;
  }
  V wo = -ray.d;
  Bsdf bsdf = hit_bsdf(Sc, h);
  S ls = t * int_le(Sc, h, -wo);
  if (has_non_specular(bsdf)) E.hps->push_back(HitPoint{bsdf, E.px, E.py, E.r2, wo, t, (uint64_t)E.pixel << 24 | id});
  S lr = follow_cam(E, B_REFL, h, bsdf, wo, depth, id, t);
  S lt = follow_cam(E, B_TRANS, h, bsdf, wo, depth, id, t);
  return ((black() + lr) + lt) + ls;
}

// sample' (Light.hs:166-213): (Le, ray, normal at the light, pdf)
struct LightRay { S li; Ray ray; V n; float pdf; };
LightRay light_ray(const Scene& Sc, const bling_light& L, float uo1, float uo2, float ud1, float ud2) {
  LightRay r{black(), Ray{mk(0, 0, 0), mk(0, 1, 0), 0.f, 0.f}, mk(0, 1, 0), 0.f};
  if (L.kind == BLING_LIGHT_POINT) {                                // sample' PointLight (Light.hs:210-213)
    const V d = uniform_sample_sphere(ud1, ud2);
    r.li = from_array(L.radiance);
    r.ray = Ray{mk(L.delta_vec[0], L.delta_vec[1], L.delta_vec[2]), d, 0.f, INF};
    r.n = d;
    r.pdf = 1.f / (2.f * PI);              // uniformSpherePdf = 1 / (2 pi) as written (Montecarlo.hs:188-190)
    return r;
  }
  if (L.kind == BLING_LIGHT_DIRECTIONAL) {                          // sample' Directional (Light.hs:181-187)
    const V n = mk(L.delta_vec[0], L.delta_vec[1], L.delta_vec[2]);
    V c = Sc.bounds.mn + vs(Sc.bounds.mx - Sc.bounds.mn, 0.5f);                        // boundingSphere (AABB.hs:62-66)
    float wr = len(Sc.bounds.mx - c);
    LC cs = coordinate_system(n);                                                      // coordinateSystem''
    float d1, d2;
    concentric_sample_disk(uo1, uo2, &d1, &d2);
    V pd = c + vs(vs(cs.s, d1) + vs(cs.t, d2), wr);
    r.li = from_array(L.radiance);
    r.ray = Ray{pd + vs(n, wr), -n, 0.f, INF};
    r.n = -n;
    r.pdf = 1.f / (PI * wr * wr);
    return r;
  }
  if (L.kind == BLING_LIGHT_AREA) {
    const bling_shape& s = Sc.d->shapes[L.shape];
    V ps, ns;
    sample_shape(s, mk(0.f, 0.f, 0.f), uo1, uo2, &ps, &ns);        // sampleShape' (the sphere's full-sphere case)
    V org = xpoint(s.o2w, ps);
    V n = normalize(xnormal(s.w2o, ns));
    float dx, dy;
    concentric_sample_disk(ud1, ud2, &dx, &dy);                       // cosineSampleHemisphere' (Montecarlo.hs:152-158)
    V wi = local_to_world(coordinate_system(n), mk(dx, dy, std::sqrt(hmax(0.f, 1.f - dx * dx - dy * dy))));
    r.pdf = INV_PI * (1.f / shape_area(s)) * absdot(n, wi);
    r.li = from_array(L.radiance);
    r.ray = Ray{org, wi, 1e-3f, INF};
    r.n = n;
    return r;
  }
  float u, v, mpdf;
  sample_c2d(L, ud1, ud2, &u, &v, &mpdf);
  if (mpdf == 0.f) return r;
  r.li = env_eval(L, u, v);
  float th = v * PI, phi = u * 2.f * PI;
  float sint = bcr::sinf(th);
  V d = xvector(L.l2w, mk(sint * bcr::cosf(phi), sint * bcr::sinf(phi), bcr::cosf(th)));
  V c = Sc.bounds.mn + vs(Sc.bounds.mx - Sc.bounds.mn, 0.5f);                            // boundingSphere (AABB.hs:62-66)
  float wr = len(Sc.bounds.mx - c);
  LC cs = coordinate_system(-d);
  float d1, d2;
  concentric_sample_disk(uo1, uo2, &d1, &d2);
  V pd = c + vs(vs(cs.s, d1) + vs(cs.t, d2), wr);
  r.ray = Ray{pd + vs(d, wr), -d, 0.f, INF};
  r.n = d;
  float pdDir = mpdf / (2.f * PI * PI * sint), pdArea = 1.f / (PI * wr * wr);
  r.pdf = sint == 0.f ? 0.f : pdDir * pdArea;
  return r;
}

// sampleLightRay (Scene.hs:121-135)
LightRay sample_light_ray(const Scene& Sc, float ul, float uo1, float uo2, float ud1, float ud2) {
  int lc = (int)Sc.d->num_lights;
  if (lc == 0) return LightRay{black(), Ray{mk(0, 0, 0), mk(0, 1, 0), 0.f, 0.f}, mk(0, 1, 0), 0.f};
  if (lc == 1) return light_ray(Sc, Sc.d->lights[0], uo1, uo2, ud1, ud2);
  int ln = std::min((int)std::floor(ul * (float)lc), lc - 1);
  LightRay r = light_ray(Sc, Sc.d->lights[ln], uo1, uo2, ud1, ud2);
  r.pdf = r.pdf / (float)lc;
  return r;
}

// hash (SPPM.hs:303-305) on 64-bit Int with wrap-around, abs, then `rem cnt` clamped to [0, cnt)
inline int64_t sppm_bucket(int64_t x, int64_t y, int64_t z, int64_t cnt) {
  uint64_t hv = ((uint64_t)x * 73856093ull) ^ ((uint64_t)y * 19349663ull) ^ ((uint64_t)z * 83492791ull);
  int64_t a = (int64_t)hv;
  if (a < 0) a = (int64_t)(0ull - (uint64_t)a);
  return std::max<int64_t>(0, std::min<int64_t>(cnt - 1, a % cnt));
}

// Each bucket's kd-tree (mkKdTree, SPPM.hs:363-389), as an implicit tree over the bucket's list: a
// range [l, u) of more than five hit points is a Node whose pivot is the element of rank (u - l)
// `quot` 2 by the coordinate on axis depth `rem` 3, the smaller ones left ([l, m)), the rest right
// ([m + 1, u)); five or fewer are a Leaf.  The bucket's list is reordered so that the pivot sits at
// m and each side is its subtree's range.  mr[m] is the node's `mr`: max (hpR2 pivot) (max lr rr),
// where a Leaf returns sqrt of its largest r2 and a Node its mr -- r2 at pivots, r at leaves, the
// reference's mix, kept.  The selection (vector-algorithms' introselect, a Stackage lts-8.13
// dependency not vendored here) leaves the order of equal coordinates to its partitioning; here
// ties go by the hit point's key (pixel, eye-tree node), so the tree is a function of the set alone
// and the device builds the same one.  Parity with the reference's own tie order is unpinned.
struct SppmKdItem { float c[3]; uint64_t key; };
inline bool kd_less(const SppmKdItem& a, const SppmKdItem& b, int axis) {
  return a.c[axis] < b.c[axis] || (!(b.c[axis] < a.c[axis]) && a.key < b.key);
}
// returns the subtree's mr (go, SPPM.hs:367-389); v is the bucket's list, mr its per-position values
float sppm_kd_build(std::vector<int>& v, std::vector<float>& mr, const std::vector<HitPoint>& hps, int l, int u, int depth) {
  if (u - l <= 5) {
    float m = 0.f;
    for (int i = l; i < u; ++i) m = hmax(m, hps[(size_t)v[(size_t)i]].r2);        // foldl' (\m hp -> max m r2) 0
    return std::sqrt(m);
  }
  const int median = (u - l) / 2, axis = depth % 3;
  auto item = [&](int id) {
    const HitPoint& h = hps[(size_t)id];
    return SppmKdItem{{h.bsdf.p.x, h.bsdf.p.y, h.bsdf.p.z}, h.key};
  };
  std::sort(v.begin() + l, v.begin() + u, [&](int a, int b) { return kd_less(item(a), item(b), axis); });
  const int m = l + median;
  const float lr = sppm_kd_build(v, mr, hps, l, m, depth + 1);
  const float rr = sppm_kd_build(v, mr, hps, m + 1, u, depth + 1);
  const float r = hmax(hps[(size_t)v[(size_t)m]].r2, hmax(lr, rr));
  mr[(size_t)m] = r;
  return r;
}

// mkHash (SPPM.hs:316-349): cell size 2 r (r = the largest hit-point radius), every hit point
// entered into each cell its own radius overlaps, then a kd-tree per bucket (sppm_kd_build).
struct SppmHash { AABB bounds; float scale; std::vector<std::vector<int>> buckets; std::vector<std::vector<float>> mr; };
SppmHash sppm_hash(const std::vector<HitPoint>& hps) {
  SppmHash H;
  const int64_t cnt = (int64_t)hps.size();
  float r2 = 0.f;
  for (const HitPoint& hp : hps) r2 = (hp.r2 <= r2) ? r2 : hp.r2;                       // max (hpR2 hp) m
  float r = std::sqrt(r2);
  H.scale = 1.f / (2.f * r);
  AABB b = empty_box();
  for (const HitPoint& hp : hps) {
    V p = hp.bsdf.p, lo = p - mk(r, r, r), hi = p + mk(r, r, r);
    b = extend(b, AABB{mk(hmin(lo.x, hi.x), hmin(lo.y, hi.y), hmin(lo.z, hi.z)), mk(hmax(lo.x, hi.x), hmax(lo.y, hi.y), hmax(lo.z, hi.z))});
  }
  H.bounds = b;
  H.buckets.assign((size_t)cnt, {});
  for (int i = 0; i < (int)cnt; ++i) {
    const HitPoint& hp = hps[i];
    if (hp.r2 == 0.f) continue;
    float rp = std::sqrt(hp.r2);
    V p = hp.bsdf.p, pmin = b.mn;
    V a0 = (p - mk(rp, rp, rp)) - pmin, a1 = (p + mk(rp, rp, rp)) - pmin;
    int64_t x0 = (int64_t)(H.scale * std::fabs(a0.x)), y0 = (int64_t)(H.scale * std::fabs(a0.y)), z0 = (int64_t)(H.scale * std::fabs(a0.z));
    int64_t x1 = (int64_t)(H.scale * std::fabs(a1.x)), y1 = (int64_t)(H.scale * std::fabs(a1.y)), z1 = (int64_t)(H.scale * std::fabs(a1.z));
    for (int64_t x = x0; x <= x1; ++x)
      for (int64_t y = y0; y <= y1; ++y)
        for (int64_t z = z0; z <= z1; ++z) H.buckets[(size_t)sppm_bucket(x, y, z, cnt)].push_back(i);
  }
  H.mr.resize(H.buckets.size());
  for (size_t b = 0; b < H.buckets.size(); ++b) {
    H.mr[b].assign(H.buckets[b].size(), 0.f);
    sppm_kd_build(H.buckets[b], H.mr[b], hps, 0, (int)H.buckets[b].size(), 0);
  }
  return H;
}

// Measurement only (oracle_sppm_set_lookup): visit every hit point of the bucket with |p - hp|^2 <=
// r2 (the intended all-within-radius query) instead of treeLookup's pruned walk, to show which
// pairs the reference's mixed r / r2 bound drops.  Off by default; no golden uses it.
inline bool& sppm_all_within() { static bool on = false; return on; }

// treeLookup (SPPM.hs:391-404): a Node tests its pivot, then descends left when pos - mr <= split
// and right when pos + mr >= split (mr the node's own, split the pivot's coordinate on the axis); a
// Leaf tests each of its hit points against its own radius
template <class Fn>
void sppm_kd_lookup(const std::vector<int>& v, const std::vector<float>& mr, const std::vector<HitPoint>& hps, int l, int u,
                    int depth, V p, Fn&& fun) {
  if (u - l <= 5 || sppm_all_within()) {
    for (int i = l; i < u; ++i) {
      const HitPoint& hp = hps[(size_t)v[(size_t)i]];
      if (sqlen(hp.bsdf.p - p) <= hp.r2) fun(hp);
    }
    return;
  }
  const int m = l + (u - l) / 2, axis = depth % 3;
  const HitPoint& hp = hps[(size_t)v[(size_t)m]];
  const float split = axis == 0 ? hp.bsdf.p.x : (axis == 1 ? hp.bsdf.p.y : hp.bsdf.p.z);
  const float pos = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
  const float r = mr[(size_t)m];
  if (sqlen(hp.bsdf.p - p) <= hp.r2) fun(hp);
  if (pos - r <= split) sppm_kd_lookup(v, mr, hps, l, m, depth + 1, p, fun);
  if (pos + r >= split) sppm_kd_lookup(v, mr, hps, m + 1, u, depth + 1, p, fun);
}

struct PhotonOut { std::vector<float> splat; std::vector<int32_t> cnt; uint64_t rays = 0, pairs = 0, dropped = 0; };

// splatSample (Image.hs:201-221)
void splat_sample(const Scene& Sc, std::vector<float>& img, float sx, float sy, const S& s, uint64_t& dropped) {
  int W = Sc.d->config.width, H = Sc.d->config.height;
  int px = (int)std::floor(sx), py = (int)std::floor(sy);
  if (px >= W || py >= H || px < 0 || py < 0) return;
  if (s_nan(s) || s_inf(s)) { dropped++; return; }
  float x, y, z;
  to_xyz(s, &x, &y, &z);
  float* o = &img[3 * ((size_t)px + (size_t)py * W)];
  o[0] = o[0] + x; o[1] = o[1] + y; o[2] = o[2] + z;
}

// tracePhoton / followPhoton (SPPM.hs:181-239): no depth limit; Russian roulette with 0.8 beyond
// depth 7.  (A photon that survived 1 << 16 bounces would be cut; none does at these albedos.)
void trace_photon(const Scene& Sc, const SppmHash& Hs, const std::vector<HitPoint>& hps, const SampleCtx& sc, PhotonOut& O) {
  float ul = rnd1(sc, 0);
  float uo1, uo2, ud1, ud2;
  rnd2(sc, 0, &uo1, &uo2);
  rnd2(sc, 1, &ud1, &ud2);
  LightRay lr = sample_light_ray(Sc, ul, uo1, uo2, ud1, ud2);
  V wi0 = -lr.ray.d;
  if (!(lr.pdf > 0.f)) return;
  S li = sscale(lr.li, absdot(lr.n, wi0) / lr.pdf);
  if (is_black(li)) return;
  Ray ray = lr.ray;
  const int64_t cnt = (int64_t)hps.size();
  for (int d = 0; d < (1 << 16); ++d) {
    V wi = -ray.d;
    Hit h;
    TStats ts;
    O.rays++;
    if (!sc_intersect(Sc, ray, &h, ts)) return;
    Bsdf bsdf = hit_bsdf(Sc, h);
    V p = bsdf.p, ng = bsdf.ng;
    if (has_non_specular(bsdf) && cnt > 0) {                                             // hashLookup (:307-314)
      V q = p - Hs.bounds.mn;
      int64_t x = (int64_t)std::fabs(q.x * Hs.scale), y = (int64_t)std::fabs(q.y * Hs.scale), z = (int64_t)std::fabs(q.z * Hs.scale);
      const size_t b = (size_t)sppm_bucket(x, y, z, cnt);
      sppm_kd_lookup(Hs.buckets[b], Hs.mr[b], hps, 0, (int)Hs.buckets[b].size(), 0, p, [&](const HitPoint& hp) {
        O.pairs++;
        S f = eval_bsdf(hp.bsdf, hp.w, wi);
        S l = sscale(hp.f * f * li, 1.f / (absdot(wi, ng) * hp.r2 * PI));
        splat_sample(Sc, O.splat, hp.px, hp.py, l, O.dropped);
        O.cnt[(size_t)sppm_sidx(Sc, hp.px, hp.py)] += 1;
      });
    }
    float ubc = rnd1(sc, 1 + d * 2);
    float ub1, ub2;
    rnd2(sc, 2 + d, &ub1, &ub2);
    BsdfSample bs = sample_bsdf_t(bsdf, B_ALL, wi, ubc, ub1, ub2, true);                 // sampleAdjBsdf
    float pcont = d > 7 ? 0.8f : 1.f;
    S li2 = sscale(bs.f * li, 1.f / pcont);
    if (bs.pdf == 0.f || is_black(li2)) return;
    if (rnd1(sc, 2 + d * 2) > pcont) return;
    ray = Ray{p, bs.wi, h.eps, INF};
    li = li2;
  }
}

}  // namespace

struct oracle_scene { Scene s; };

extern "C" {

oracle_scene* oracle_build(const bling_scene_desc* d) {
  auto* os = new oracle_scene();
  Scene& Sc = os->s;
  Sc.d = d;
  for (uint32_t i = 0; i < d->num_prims; ++i) {
    Prim p;
    p.kind = d->prim_kind[i];
    p.index = d->prim_index[i];
    p.bounds = prim_bounds(d, p.kind, p.index);
    Sc.prims.push_back(p);
  }
  AABB b = empty_box();                                                                  // mkKdTree (KdTree.hs:187-192)
  for (auto& p : Sc.prims) b = extend(b, p.bounds);
  Sc.bounds = b;
  float lg = std::log((float)Sc.prims.size());
  Sc.max_depth_param = (int)std::lrint(8.f + 3.f * lg);                                   // round (banker's)
  std::vector<int> all;
  for (int i = 0; i < (int)Sc.prims.size(); ++i) all.push_back(i);
  kd_build(Sc, b, all, Sc.max_depth_param);
  setup_extent(Sc);
  int leaves = 0, maxleaf = 0;
  for (auto& n : Sc.nodes) if (n.leaf) { leaves++; maxleaf = std::max(maxleaf, (int)n.ps.size()); }
  char buf[256];
  std::snprintf(buf, sizeof buf, "prims %zu, kd nodes %zu (leaves %d, max leaf %d, depth cap %d), tiles %zu",
                Sc.prims.size(), Sc.nodes.size(), leaves, maxleaf, Sc.max_depth_param, Sc.tiles.size());
  Sc.info = buf;
  return os;
}

void oracle_free(oracle_scene* s) { delete s; }

// 1: the per-sample transcendentals become libm's binary32 functions (GHC's Float primops) instead
// of the correctly rounded binary64-once ones the device shares (common/cr_math.h) -- for measuring
// that departure only (tests/test_cr_math.py); 0 restores the default.  Process-wide.
void oracle_set_libm32(int on) { bcr::libm32_mode() = on != 0; }

// The shared transcendentals (common/cr_math.h) over arrays, for their accuracy tests and the
// device-equals-host check: fn 0 sin, 1 cos, 2 tan, 3 asin, 4 acos, 5 atan, 6 exp, 7 log, 8 sinh,
// 9 atan2(x, y), 10 pow(x, y)
int oracle_cr_eval(int fn, const float* x, const float* y, float* out, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const float a = x[i], b = y ? y[i] : 0.f;
    float r;
    switch (fn) {
      case 0: r = bcr::sinf(a); break;
      case 1: r = bcr::cosf(a); break;
      case 2: r = bcr::tanf(a); break;
      case 3: r = bcr::asinf(a); break;
      case 4: r = bcr::acosf(a); break;
      case 5: r = bcr::atanf(a); break;
      case 6: r = bcr::expf(a); break;
      case 7: r = bcr::logf(a); break;
      case 8: r = bcr::sinhf(a); break;
      case 9: r = bcr::atan2f(a, b); break;
      case 10: r = bcr::powf(a, b); break;
      case 11: r = bcr::sincosf(a).s; break;
      case 12: r = bcr::sincosf(a).c; break;
      default: return -1;
    }
    out[i] = r;
  }
  return 0;
}
const char* oracle_info(const oracle_scene* s) { return s->s.info.c_str(); }

int oracle_extent(const oracle_scene* s, int* o) {
  o[0] = s->s.ex0; o[1] = s->s.ex1; o[2] = s->s.ey0; o[3] = s->s.ey1;
  return (int)s->s.tiles.size();
}

// The tile generator's first n outputs: kind 0 uniformWord32 (as float bit patterns), 1 uniform,
// 2 rnd, 3 a shuffled stratified1D(n) table, 4 the low / high words of n rndInt draws.
int oracle_mwc_probe(uint32_t seed, uint32_t pass, uint32_t key, int kind, int n, uint32_t* out) {
  Mwc g(seed, pass, key);
  if (kind == 3) {
    std::vector<float> v = g.stratified1D(n);
    g.shuffle(v);
    std::memcpy(out, v.data(), sizeof(float) * n);
    return 0;
  }
  for (int k = 0; k < n; ++k) {
    if (kind == 0) out[k] = g.word();
    else if (kind == 1) { float f = g.uniform(); std::memcpy(&out[k], &f, 4); }
    else if (kind == 2) { float f = g.rnd(); std::memcpy(&out[k], &f, 4); }
    else if (kind == 4 && k + 1 < n) { uint64_t v = (uint64_t)g.rnd_int(); out[k] = (uint32_t)v; out[++k] = (uint32_t)(v >> 32); }
    else return -1;
  }
  return 0;
}

int oracle_set_rng(oracle_scene* os, int mode) {
  if (mode != ORACLE_RNG_COUNTER && mode != ORACLE_RNG_MWC) return -1;
  int prev = os->s.rng;
  os->s.rng = mode;
  return prev;
}

int oracle_render(oracle_scene* os, uint32_t seed, uint32_t pass, int tile_stride, int threads, float* film,
                  oracle_stats* st) {
  return oracle_render_shard(os, seed, pass, 0, 1, tile_stride, threads, film, st);
}

int oracle_render_shard(oracle_scene* os, uint32_t seed, uint32_t pass, int shard_rank, int shard_world,
                        int tile_stride, int threads, float* film, oracle_stats* st) {
  Scene& Sc = os->s;
  if (Sc.d->config.renderer != BLING_RENDERER_SAMPLER_PATH) return -1;
  auto t0 = std::chrono::steady_clock::now();
  int nt = (int)Sc.tiles.size();
  if (tile_stride < 1) tile_stride = 1;
  std::vector<int> todo;
  if (shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world) return -1;
  for (int k = 0; k < nt; ++k)                      // interleaved tile shard
    // the stride picks the sub-sample, the shard deals the picked tiles round-robin (core.hip render)
    if (k % tile_stride == 0 && (k / tile_stride) % shard_world == shard_rank) todo.push_back(k);
  std::vector<TileImg> imgs(todo.size());
  std::vector<Counters> cs(todo.size());
  std::vector<uint64_t> smp(todo.size(), 0), drp(todo.size(), 0);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int i = 0; i < (int)todo.size(); ++i) {
    imgs[i] = make_tile(Sc, Sc.tiles[todo[i]]);
    render_tile(Sc, Sc.tiles[todo[i]], seed, pass, imgs[i], cs[i], smp[i], drp[i]);
  }
  // addTile in tile order (Image.hs:178-199)
  int W = Sc.d->config.width, H = Sc.d->config.height;
  for (size_t i = 0; i < todo.size(); ++i) {
    TileImg& T = imgs[i];
    for (int y = 0; y < T.h; ++y)
      for (int x = 0; x < T.w; ++x) {
        int gx = x + T.ox, gy = y + T.oy;
        if (gy >= H || gx >= W) continue;
        float* o = film + 4 * ((size_t)gy * W + gx);
        const float* q = &T.px[4 * ((size_t)y * T.w + x)];
        for (int c = 0; c < 4; ++c) o[c] = o[c] + q[c];
      }
  }
  if (st) {
    std::memset(st, 0, sizeof *st);
    for (size_t i = 0; i < todo.size(); ++i) {
      st->samples += smp[i]; st->dropped += drp[i];
      st->rays_camera += cs[i].cam; st->rays_continuation += cs[i].cont;
      st->rays_mis += cs[i].mis; st->rays_shadow += cs[i].shadow;
      st->kd_nodes += cs[i].ts.nodes; st->kd_leaf_prims += cs[i].ts.leaf_prims;
    }
    st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return 0;
}

// The same shard's tiles as mkImageTile images (Image.hs:108-120), one slot of slot_w x slot_h x 4
// floats per tile in tile order, zero-padded (slot_w = 15 + floor (0.5 + fw), slot_h likewise: the
// largest tile image; pixels past the film stay zero); origins_out: the tile images' (ox, oy).  The multi-rank merge gathers these
// slots and adds them (addTile, Image.hs:178-199) -- the layout bling_render_pass_device writes with
// BLING_PASS_TILE_IMAGES.  Returns the number of tiles, or -1.
int oracle_render_tiles(oracle_scene* os, uint32_t seed, uint32_t pass, int shard_rank, int shard_world,
                        int tile_stride, int threads, float* tiles_out, int* origins_out, oracle_stats* st) {
  Scene& Sc = os->s;
  if (Sc.d->config.renderer != BLING_RENDERER_SAMPLER_PATH) return -1;
  if (tile_stride < 1) tile_stride = 1;
  if (shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world) return -1;
  const int sw = 15 + (int)std::floor(0.5f + Sc.d->filter.width), sh = 15 + (int)std::floor(0.5f + Sc.d->filter.height);
  std::vector<int> todo;
  for (int k = 0; k < (int)Sc.tiles.size(); ++k)
    if (k % tile_stride == 0 && (k / tile_stride) % shard_world == shard_rank) todo.push_back(k);
  std::vector<Counters> cs(todo.size());
  std::vector<uint64_t> smp(todo.size(), 0), drp(todo.size(), 0);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int i = 0; i < (int)todo.size(); ++i) {
    TileImg T = make_tile(Sc, Sc.tiles[todo[i]]);
    render_tile(Sc, Sc.tiles[todo[i]], seed, pass, T, cs[i], smp[i], drp[i]);
    float* slot = tiles_out + (size_t)i * sw * sh * 4;
    std::fill(slot, slot + (size_t)sw * sh * 4, 0.f);
    const int W = Sc.d->config.width, H = Sc.d->config.height;
    for (int y = 0; y < T.h && y < sh && y + T.oy < H; ++y)       // pixels past the film stay zero
      for (int x = 0; x < T.w && x < sw && x + T.ox < W; ++x)
        for (int c = 0; c < 4; ++c) slot[4 * ((size_t)y * sw + x) + c] = T.px[4 * ((size_t)y * T.w + x) + c];
    if (origins_out) { origins_out[2 * i] = T.ox; origins_out[2 * i + 1] = T.oy; }
  }
  if (st) {
    std::memset(st, 0, sizeof *st);
    for (size_t i = 0; i < todo.size(); ++i) {
      st->samples += smp[i]; st->dropped += drp[i];
      st->rays_camera += cs[i].cam; st->rays_continuation += cs[i].cont;
      st->rays_mis += cs[i].mis; st->rays_shadow += cs[i].shadow;
    }
  }
  return (int)todo.size();
}

int oracle_camera_ray(oracle_scene* os, uint32_t seed, uint32_t pass, int px, int py, int n, float* out) {
  Scene& Sc = os->s;
  int extW = Sc.ex1 - Sc.ex0 + 1;
  SampleCtx sc = sample_ctx(Sc, seed, pass);
  sc.pixel = (uint32_t)((py - Sc.ey0) * extW + (px - Sc.ex0));
  sc.n = (uint32_t)n;
  float ox, oy, lu, lv;
  camera_sample(sc, &ox, &oy, &lu, &lv);
  float imx = (float)px + ox, imy = (float)py + oy;
  Ray r = fire_ray(Sc.d->camera, imx, imy, lu, lv);
  out[0] = imx; out[1] = imy;
  out[2] = r.o.x; out[3] = r.o.y; out[4] = r.o.z; out[5] = r.d.x; out[6] = r.d.y; out[7] = r.d.z;
  return 0;
}

int oracle_sample_li(oracle_scene* os, uint32_t seed, uint32_t pass, int px, int py, int n, float* L,
                     float* img_xy, oracle_stats* st) {
  Scene& Sc = os->s;
  int extW = Sc.ex1 - Sc.ex0 + 1;
  SampleCtx sc = sample_ctx(Sc, seed, pass);
  sc.pixel = (uint32_t)((py - Sc.ey0) * extW + (px - Sc.ex0));
  sc.n = (uint32_t)n;
  float ox, oy, lu, lv;
  camera_sample(sc, &ox, &oy, &lu, &lv);
  float imx = (float)px + ox, imy = (float)py + oy;
  Ray r = fire_ray(Sc.d->camera, imx, imy, lu, lv);
  Counters C;
  ora::S li = sample_li(Sc, sc, r, C);
  std::memcpy(L, li.v, sizeof li.v);
  if (img_xy) { img_xy[0] = imx; img_xy[1] = imy; }
  if (st) {
    st->rays_camera += C.cam; st->rays_continuation += C.cont; st->rays_mis += C.mis; st->rays_shadow += C.shadow;
    st->kd_nodes += C.ts.nodes; st->kd_leaf_prims += C.ts.leaf_prims; st->samples += 1;
  }
  return 0;
}

// oracle_sample_li with the per-vertex debug records of the path (Path integrator only): vtx holds
// n x DV_DEPTHS x DV_FIELDS floats, NaN where a vertex or field was not reached.
int oracle_sample_li_vertices(oracle_scene* os, uint32_t seed, uint32_t pass, const int* samples, size_t n, float* L,
                              float* vtx, int threads) {
  if (os->s.d->config.integrator != BLING_INTEGRATOR_PATH) return -1;
  std::fill(vtx, vtx + n * DV_DEPTHS * DV_FIELDS, std::numeric_limits<float>::quiet_NaN());
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (long i = 0; i < (long)n; ++i) {
    g_dv = vtx + (size_t)i * DV_DEPTHS * DV_FIELDS;
    oracle_sample_li(os, seed, pass, samples[3 * i], samples[3 * i + 1], samples[3 * i + 2], L + 16 * i, nullptr, nullptr);
    g_dv = nullptr;
  }
  return 0;
}

// oracle_sample_li over a list of (x, y, n) samples, OpenMP over the list (per-sample parity at the
// BASELINE configs' full sizes); stats sum over the list.
int oracle_sample_li_batch(oracle_scene* os, uint32_t seed, uint32_t pass, const int* samples, size_t n, float* L,
                           float* img_xy, int threads, oracle_stats* st) {
  uint64_t cam = 0, cont = 0, mis = 0, shadow = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : cam, cont, mis, shadow)
#endif
  for (long i = 0; i < (long)n; ++i) {
    oracle_stats s{};
    oracle_sample_li(os, seed, pass, samples[3 * i], samples[3 * i + 1], samples[3 * i + 2], L + 16 * i,
                     img_xy ? img_xy + 2 * i : nullptr, &s);
    cam += s.rays_camera; cont += s.rays_continuation; mis += s.rays_mis; shadow += s.rays_shadow;
  }
  if (st) {
    st->rays_camera += cam; st->rays_continuation += cont; st->rays_mis += mis; st->rays_shadow += shadow;
    st->samples += n;
  }
  return 0;
}

int oracle_trace(oracle_scene* os, const float* rays, size_t n, int any_hit, float* t, uint32_t* prim, float* bary,
                 oracle_stats* st) {
  Scene& Sc = os->s;
  uint64_t nodes = 0, lp = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : nodes, lp)
#endif
  for (long i = 0; i < (long)n; ++i) {
    Ray r{mk(rays[i], rays[n + i], rays[2 * n + i]), mk(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]), rays[6 * n + i],
          rays[7 * n + i]};
    TStats ts;
    if (any_hit) {
      prim[i] = sc_occluded(Sc, r, ts) ? 1u : 0u;
    } else {
      Hit h;
      if (sc_intersect(Sc, r, &h, ts)) {
        if (t) t[i] = h.t;
        prim[i] = (uint32_t)h.prim;
        if (bary) {
          if (h.dg.has_b) { bary[2 * i] = h.dg.b1; bary[2 * i + 1] = h.dg.b2; }
          else { bary[2 * i] = h.dg.u; bary[2 * i + 1] = h.dg.v; }
        }
      } else {
        if (t) t[i] = INF;
        prim[i] = 0xFFFFFFFFu;
        if (bary) { bary[2 * i] = 0.f; bary[2 * i + 1] = 0.f; }
      }
    }
    nodes += ts.nodes; lp += ts.leaf_prims;
  }
  if (st) { st->kd_nodes += nodes; st->kd_leaf_prims += lp; }
  return 0;
}

int oracle_sampler_probe(oracle_scene* os, uint32_t seed, uint32_t pass, int px, int py, int n, int kind, int dim,
                         float* out) {
  Scene& Sc = os->s;
  int extW = Sc.ex1 - Sc.ex0 + 1;
  SampleCtx sc = sample_ctx(Sc, seed, pass);
  sc.pixel = (uint32_t)((py - Sc.ey0) * extW + (px - Sc.ex0));
  sc.n = (uint32_t)n;
  if (kind == 0) out[0] = rnd1(sc, dim);
  else if (kind == 1) rnd2(sc, dim, &out[0], &out[1]);
  else camera_sample(sc, &out[0], &out[1], &out[2], &out[3]);
  return 0;
}

uint32_t oracle_hash5(uint32_t seed, uint32_t pass, uint32_t pixel, uint32_t sample, uint32_t dim) {
  return hash5(seed, pass, pixel, sample, dim);
}
uint32_t oracle_permute(uint32_t i, uint32_t l, uint32_t p) { return permute(i, l, p); }

void oracle_concentric_disk(float u1, float u2, float* o) { concentric_sample_disk(u1, u2, &o[0], &o[1]); }
int oracle_solve_quadric(float a, float b, float c, float* o) { return solve_quadric(a, b, c, &o[0], &o[1]) ? 1 : 0; }
void oracle_fr_dielectric(float ei, float et, float c, float* o) { ora::S s = fr_dielectric(ei, et, c); std::memcpy(o, s.v, 64); }
void oracle_fr_conductor(const float* e, const float* k, float c, float* o) {
  ora::S s = fr_conductor(from_array(e), from_array(k), c);
  std::memcpy(o, s.v, 64);
}
// mkFresnelBlend's e wo wi (Microfacet.hs:64-84) with rd/rs/ra as given; abc = ex, ey, depth
void oracle_fblend_eval(const float* wo, const float* wi, const float* rd, const float* rs, const float* ra,
                        const float* abc, float* o) {
  BxDF b{}; b.kind = K_FBLEND; b.r = from_array(rd); b.rs = from_array(rs); b.ra = from_array(ra);
  b.e = abc[0]; b.ey = abc[1]; b.depth = abc[2];
  ora::S s = fblend_eval(b, mk(wo[0], wo[1], wo[2]), mk(wi[0], wi[1], wi[2]));
  std::memcpy(o, s.v, 64);
}
float oracle_aniso_d(float ex, float ey, const float* wh) { return aniso_D(ex, ey, mk(wh[0], wh[1], wh[2])); }

// ---- formula probes for the known-answer tests (tests/test_kat_hotpath.py)
// triangleIntersect (TriangleMesh.hs:160-207) on explicit vertices p9 = p1 p2 p3 and a ray
// (ox oy oz dx dy dz tmin tmax): 1 = hit, out = t, b1, b2
int oracle_tri_probe(const float* p9, const float* ray8, float* out3) {
  bling_scene_desc d{};
  const uint32_t idx[3] = {0, 1, 2};
  const float uv[6] = {0.f, 0.f, 1.f, 0.f, 1.f, 1.f};
  d.num_vertices = 3; d.vertices = p9; d.num_triangles = 1; d.tri_indices = idx; d.tri_uvs = uv;
  Ray r{mk(ray8[0], ray8[1], ray8[2]), mk(ray8[3], ray8[4], ray8[5]), ray8[6], ray8[7]};
  Hit h;
  if (!tri_intersect(&d, 0, r, &h)) return 0;
  out3[0] = h.t; out3[1] = h.dg.b1; out3[2] = h.dg.b2;
  return 1;
}

// BxDF `comp` of material `mat` built at a hit whose shading frame is the identity (n = +z,
// dpdu = +x), so local = world: out[0..15] = bxdfEval wo wi, [16] = bxdfPdf wo wi, then bxdfSample
// (adj = False) wo u: [17..32] f, [33..35] wi, [36] pdf.  Returns the component count.
int oracle_bxdf_probe(oracle_scene* os, int mat, int comp, const float* wo3, const float* wi3, const float* u2,
                      float* out) {
  const bling_scene_desc* d = os->s.d;
  DG dg = mk_dg(mk(0.f, 0.f, 0.f), 0.5f, 0.5f, mk(1.f, 0.f, 0.f), mk(0.f, 1.f, 0.f));
  Bsdf bs = make_bsdf(d, mat, dg, dg);
  if (comp < 0 || comp >= bs.n) return bs.n;
  const BxDF& b = bs.b[comp];
  V wo = mk(wo3[0], wo3[1], wo3[2]), wi = mk(wi3[0], wi3[1], wi3[2]);
  S e = bxdf_eval(b, wo, wi);
  std::memcpy(out, e.v, 64);
  out[16] = bxdf_pdf(b, wo, wi);
  V ws; float pdf;
  S f = bxdf_sample(b, wo, u2[0], u2[1], &ws, &pdf);
  std::memcpy(out + 17, f.v, 64);
  out[33] = ws.x; out[34] = ws.y; out[35] = ws.z; out[36] = pdf;
  return bs.n;
}

// Light.sample of light `li` seen from world point p (Light.hs:122-160): out = li[16], wi[3], pdf,
// ray o[3] d[3] tmin tmax (28 floats); Light.pdf p wi (Light.hs:215-229) as the return value of
// oracle_light_pdf_probe
void oracle_light_sample_probe(oracle_scene* os, int li, const float* p3, float eps, float u1, float u2, float* out) {
  const Scene& Sc = os->s;
  LightSample ls = light_sample(Sc, Sc.d->lights[li], mk(p3[0], p3[1], p3[2]), mk(0.f, 0.f, 1.f), eps, u1, u2);
  std::memcpy(out, ls.li.v, 64);
  out[16] = ls.wi.x; out[17] = ls.wi.y; out[18] = ls.wi.z; out[19] = ls.pdf;
  out[20] = ls.ray.o.x; out[21] = ls.ray.o.y; out[22] = ls.ray.o.z;
  out[23] = ls.ray.d.x; out[24] = ls.ray.d.y; out[25] = ls.ray.d.z; out[26] = ls.ray.tmin; out[27] = ls.ray.tmax;
}
float oracle_light_pdf_probe(oracle_scene* os, int li, const float* p3, const float* wi3) {
  const Scene& Sc = os->s;
  return light_pdf(Sc, Sc.d->lights[li], mk(p3[0], p3[1], p3[2]), mk(wi3[0], wi3[1], wi3[2]));
}

// the environment map of infinite light `li` at map coordinates (u, v) (texMapEval; the sun / sky
// eval of SunSky.hs:16-19): out16
void oracle_env_probe(oracle_scene* os, int li, float u, float v, float* out16) {
  S s = env_eval(os->s.d->lights[li], u, v);
  std::memcpy(out16, s.v, 64);
}

// a scalar texture at a world point (pScalarTexture), and a spectrum texture at a DG with point p and
// parameters (u, v) (pSpectrumTexture): the texture known-answer tests (tests/test_kat_hotpath.py)
float oracle_stex_probe(oracle_scene* os, int ti, const float* p3) {
  return eval_stex(os->s.d, ti, mk(p3[0], p3[1], p3[2]), 0.f, 0.f);
}
float oracle_stex_probe_uv(oracle_scene* os, int ti, const float* p3, float u, float v) {
  return eval_stex(os->s.d, ti, mk(p3[0], p3[1], p3[2]), u, v);
}
void oracle_spectrum_probe(oracle_scene* os, int ti, const float* p3, float u, float v, float* out16) {
  DG dg{};
  dg.p = mk(p3[0], p3[1], p3[2]);
  dg.u = u; dg.v = v;
  const S s = eval_spectrum(os->s.d, ti, dg);
  std::memcpy(out16, s.v, 64);
}

// bump (Reflection.hs:347-377) with displacement scalar texture ti at a geometric normal ng and a
// shading DG (p, n, dpdu, dpdv): in15 = ng[3] p[3] n[3] dpdu[3] dpdv[3]; out9 = bumped n, dpdu, dpdv
void oracle_bump_probe(oracle_scene* os, int ti, const float* in15, float* out9) {
  DG g{}, s{};
  g.n = mk(in15[0], in15[1], in15[2]);
  s.p = mk(in15[3], in15[4], in15[5]);
  s.n = mk(in15[6], in15[7], in15[8]);
  s.dpdu = mk(in15[9], in15[10], in15[11]);
  s.dpdv = mk(in15[12], in15[13], in15[14]);
  const DG b = bump_dg(os->s.d, ti, g, s);
  out9[0] = b.n.x; out9[1] = b.n.y; out9[2] = b.n.z;
  out9[3] = b.dpdu.x; out9[4] = b.dpdu.y; out9[5] = b.dpdu.z;
  out9[6] = b.dpdv.x; out9[7] = b.dpdv.y; out9[8] = b.dpdv.z;
}

// fireRay (Camera.hs:49-76) for an image position and lens sample: out = o[3], d[3]
void oracle_fire_ray_probe(oracle_scene* os, float ix, float iy, float lu, float lv, float* out6) {
  Ray r = fire_ray(os->s.d->camera, ix, iy, lu, lv);
  out6[0] = r.o.x; out6[1] = r.o.y; out6[2] = r.o.z; out6[3] = r.d.x; out6[4] = r.d.y; out6[5] = r.d.z;
}

// ---- SPPM (Renderer/SPPM.hs)
struct oracle_sppm {
  oracle_scene* os;
  std::vector<float> r2, n;                          // PixelStats psR2 / psN (SPPM.hs:245-257)
  std::vector<HitPoint> last;                        // the last pass's hit points (diagnostics)
  std::vector<uint32_t> bstart, items;               // the last pass's kd-tree buckets (diagnostics)
  std::vector<float> kd_mr;
};

oracle_sppm* oracle_sppm_new(oracle_scene* os) {
  const Scene& Sc = os->s;
  const bling_render_config& cfg = Sc.d->config;
  if (cfg.renderer != BLING_RENDERER_SPPM) return nullptr;
  auto* p = new oracle_sppm();
  p->os = os;
  size_t np = (size_t)(Sc.ex1 - Sc.ex0 + 1) * (size_t)(Sc.ey1 - Sc.ey0 + 1);            // windowPixels
  p->r2.assign(np, cfg.sppm_radius * cfg.sppm_radius);
  p->n.assign(np, 0.f);
  return p;
}
void oracle_sppm_free(oracle_sppm* p) { delete p; }

void oracle_sppm_set_lookup(int all_within) { sppm_all_within() = all_within != 0; }

size_t oracle_sppm_buckets(const oracle_sppm* p, uint32_t* bstart, uint32_t* items, float* mr, size_t* n_items) {
  if (n_items) *n_items = p->items.size();
  if (bstart) std::memcpy(bstart, p->bstart.data(), p->bstart.size() * sizeof(uint32_t));
  if (items) std::memcpy(items, p->items.data(), p->items.size() * sizeof(uint32_t));
  if (mr) std::memcpy(mr, p->kd_mr.data(), p->kd_mr.size() * sizeof(float));
  return p->bstart.size();
}

size_t oracle_sppm_hitpoints(const oracle_sppm* p, float* pos_r2, uint64_t* keys, size_t cap) {
  const size_t k = std::min(cap, p->last.size());
  for (size_t i = 0; i < k; ++i) {
    const HitPoint& h = p->last[i];
    if (pos_r2) { pos_r2[4 * i] = h.bsdf.p.x; pos_r2[4 * i + 1] = h.bsdf.p.y; pos_r2[4 * i + 2] = h.bsdf.p.z; pos_r2[4 * i + 3] = h.r2; }
    if (keys) keys[i] = h.key;
  }
  return p->last.size();
}

int oracle_sppm_pixel_stats(const oracle_sppm* p, float* r2, float* n) {
  if (r2) std::memcpy(r2, p->r2.data(), p->r2.size() * sizeof(float));
  if (n) std::memcpy(n, p->n.data(), p->n.size() * sizeof(float));
  return (int)p->r2.size();
}

// onePass (SPPM.hs:424-460)
int oracle_sppm_pass(oracle_sppm* P, uint32_t seed, uint32_t pass, int threads, float* film, float* splat,
                     oracle_sppm_stats* st) {
  const Scene& Sc = P->os->s;
  const bling_render_config& cfg = Sc.d->config;
  auto t0 = std::chrono::steady_clock::now();
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  // mkHitPoints (:133-164): one random camera sample per extent pixel, tile by tile
  const int nt = (int)Sc.tiles.size(), extW = Sc.ex1 - Sc.ex0 + 1;
  std::vector<TileImg> imgs(nt);
  std::vector<std::vector<HitPoint>> thp(nt);
  std::vector<uint64_t> trays(nt, 0), tdrop(nt, 0);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int t = 0; t < nt; ++t) {
    const Scene::Tile& w = Sc.tiles[t];
    imgs[t] = make_tile(Sc, w);
    for (int iy = w.y0; iy <= w.y1; ++iy)
      for (int ix = w.x0; ix <= w.x1; ++ix) {
        SampleCtx sc{&Sc, seed, pass, (uint32_t)((iy - Sc.ey0) * extW + (ix - Sc.ex0)), 0u, 0, 0,
                     SamplerCfg{BLING_SAMPLER_RANDOM, 1, 1}};
        float ox, oy, lu, lv;
        camera_sample(sc, &ox, &oy, &lu, &lv);
        float px = (float)ix + ox, py = (float)iy + oy;
        Ray ray = fire_ray(Sc.d->camera, px, py, lu, lv);
        EyeCtx E{&Sc, seed, pass, sc.pixel, px, py, P->r2[(size_t)sppm_sidx(Sc, px, py)], &thp[t], 0};
        S ls = trace_cam(E, ray, 0, 1u, white());
        trays[t] += E.rays;
        add_sample(imgs[t], Sc.d->filter, px, py, ls, tdrop[t]);
      }
  }
  const int W = cfg.width, H = cfg.height;
  std::vector<HitPoint> hps;
  uint64_t cam_rays = 0, dropped = 0;
  for (int t = 0; t < nt; ++t) {                                                         // addTile in tile order
    TileImg& T = imgs[t];
    for (int y = 0; y < T.h; ++y)
      for (int x = 0; x < T.w; ++x) {
        int gx = x + T.ox, gy = y + T.oy;
        if (gy >= H || gx >= W) continue;
        float* o = film + 4 * ((size_t)gy * W + gx);
        const float* q = &T.px[4 * ((size_t)y * T.w + x)];
        for (int c = 0; c < 4; ++c) o[c] = o[c] + q[c];
      }
    hps.insert(hps.end(), thp[t].begin(), thp[t].end());
    cam_rays += trays[t]; dropped += tdrop[t];
  }
  SppmHash Hs = sppm_hash(hps);
  P->last = hps;
  P->bstart.assign(1, 0u); P->items.clear(); P->kd_mr.clear();
  for (size_t b = 0; b < Hs.buckets.size(); ++b) {
    for (size_t i = 0; i < Hs.buckets[b].size(); ++i) { P->items.push_back((uint32_t)Hs.buckets[b][i]); P->kd_mr.push_back(Hs.mr[b][i]); }
    P->bstart.push_back((uint32_t)P->items.size());
  }
  // photons: numCapabilities samplers of sn x sn stratified samples (:449-453, 474)
  const int nth = std::max(1, cfg.sppm_threads);
  const int sn = std::max(1, (int)std::ceil(std::sqrt((float)cfg.sppm_photons / (float)nth)));
  std::vector<PhotonOut> outs(nth);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int k = 0; k < nth; ++k) {
    PhotonOut& O = outs[k];
    O.splat.assign((size_t)W * H * 3, 0.f);
    O.cnt.assign(P->r2.size(), 0);
    SampleCtx sc{&Sc, seed, pass, SPPM_PHOTON_PIXEL | (uint32_t)k, 0u, 7, 5, SamplerCfg{BLING_SAMPLER_STRATIFIED, sn, sn}};
    for (int s = 0; s < sn * sn; ++s) { sc.n = (uint32_t)s; trace_photon(Sc, Hs, hps, sc, O); }
  }
  // addTile of the splats and mergeStats in seed order (:451-453), then statsUpdate (:272-291)
  std::vector<int64_t> m(P->r2.size(), 0);
  uint64_t prays = 0, pairs = 0;
  for (int k = 0; k < nth; ++k) {
    const PhotonOut& O = outs[k];
    for (size_t i = 0; i < O.splat.size(); ++i) splat[i] = splat[i] + O.splat[i];
    // mergeStats writes m[i] := m'[i + m[i]] (SPPM.hs:259-262), restated literally; an index past
    // the end (unsafeIndex) reads 0 here
    for (size_t i = 0; i < m.size(); ++i) {
      size_t j = i + (size_t)m[i];
      m[i] = j < O.cnt.size() ? O.cnt[j] : 0;
    }
    prays += O.rays; pairs += O.pairs; dropped += O.dropped;
  }
  const float a = cfg.sppm_alpha;
  for (size_t i = 0; i < m.size(); ++i) {
    if (m[i] > 0) {
      float r2 = P->r2[i], n = P->n[i], mf = (float)m[i];
      float n2 = n + a * mf;
      float ratio = n2 / (n + mf);
      P->r2[i] = r2 * ratio;
      P->n[i] = n2;
    }
  }
  if (st) {
    st->hitpoints = hps.size();
    st->photons = (uint64_t)nth * (uint64_t)sn * (uint64_t)sn;
    st->photon_rays = prays;
    st->photon_hits = pairs;
    st->cam_rays = cam_rays;
    st->dropped = dropped;
    st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return 0;
}

}  // extern "C"
