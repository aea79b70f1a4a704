// dev_shapes.h -- object-space intersection of the disk, cylinder and box shapes (Shape.hs:86-155
// intersect, :233-264 intersects), shared by the traversal kernels (dev_trace.h) and the shading
// code that rebuilds a hit's differential geometry or a light-sample pdf (dev_shade.h).
#pragma once
#include "dev_common.h"
#include "dev_scene.h"

namespace bd {

// ---- disk, cylinder, box (Shape.hs:86-155 intersect, :233-264 intersects); P = bling_shape params
DEV bool disk_test(const float* P, const Ray& r, float tmax, bool any, float* t_out) {
  const float h = P[0], rad = P[1], irad = P[2], phimax = P[3];
  if (fabsf(r.d.z) < 1e-7f) return false;
  float t = (h - r.o.z) / r.d.z;
  if (t < r.tmin || t > tmax) return false;
  V3 p = ray_at(r, t);
  float d2 = p.x * p.x + p.y * p.y;
  if (d2 > rad * rad || d2 < irad * irad) return false;
  if (atan2p(p.y, p.x) > phimax) return false;
  (void)any;
  *t_out = t;
  return true;
}
DEV bool cylinder_test(const float* P, const Ray& r, float tmax, bool any, float* t_out) {
  const float rad = P[0], zmin = P[1], zmax = P[2], phimax = P[3];
  float a = r.d.x * r.d.x + r.d.y * r.d.y;
  float b = 2.f * (r.d.x * r.o.x + r.d.y * r.o.y);
  float c = r.o.x * r.o.x + r.o.y * r.o.y - rad * rad;
  float t0, t1;
  if (!solve_quadric(a, b, c, &t0, &t1)) return false;
  if (t0 > tmax || t1 < r.tmin) return false;
  V3 p0 = ray_at(r, t0);
  if (t0 > r.tmin && p0.z > zmin && p0.z < zmax && atan2p(p0.y, p0.x) <= phimax) { *t_out = t0; return true; }
  V3 p1 = ray_at(r, t1);
  // intersects adds `t1 < tmax` in front of the same test (Shape.hs:245)
  if ((!any || t1 < tmax) && t1 <= tmax && p1.z > zmin && p1.z < zmax && atan2p(p1.y, p1.x) <= phimax) {
    *t_out = t1;
    return true;
  }
  return false;
}
DEV float v3c(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
// Box intersect: testSlabs from (-inf, inf), remembering the axis of the last near-plane increase
DEV bool box_slabs(const float* P, const Ray& r, float* t0o, float* t1o, int* axis) {
  float n = -INFINITY, f = INFINITY;
  int dd = 0;
  for (int k = 0; k < 3; ++k) {
    if (n > f) return false;
    float oc = v3c(r.o, k), dinv = 1.f / v3c(r.d, k);
    float a = (P[3 + k] - oc) * dinv, b = (P[k] - oc) * dinv;
    float t1 = a > b ? b : a, t2 = a > b ? a : b;
    dd = n < t1 ? k : dd;
    n = hmax(n, t1);
    f = hmin(f, t2);
  }
  if (n > f) return false;
  *t0o = hmin(n, f); *t1o = hmax(n, f); *axis = dd;
  return true;
}
DEV bool box_test(const float* P, const Ray& r, float tmax, float* t_out) {
  float t0, t1; int ax;
  if (!box_slabs(P, r, &t0, &t1, &ax)) return false;
  if (t0 > tmax || t0 < r.tmin) return false;
  *t_out = t0;                                    // t = if t0 < tmin then t1 else t0: t0 >= tmin here
  return true;
}
// Box intersects = intersectAABB (AABB.hs:79-94): slabs clipped to [tmin, tmax]
DEV bool box_any(const float* P, const Ray& r) {
  float n = r.tmin, f = r.tmax;
  for (int k = 0; k < 3; ++k) {
    if (n > f) return false;
    float oc = v3c(r.o, k), dinv = 1.f / v3c(r.d, k);
    float tfar = (P[3 + k] - oc) * dinv, tnear = (P[k] - oc) * dinv;
    float nn = tnear > tfar ? tfar : tnear, ff = tnear > tfar ? tnear : tfar;
    n = hmax(n, nn);
    f = hmin(f, ff);
  }
  return !(n > f);
}
// closest (ANY = false, returns t) or any hit of the three shapes against an object-space ray
DEV bool shape2_test(const DevShape& s, const Ray& r, float tmax, bool any, float* t) {
  if (s.kind == BLING_SHAPE_DISK) return disk_test(s.params, r, tmax, any, t);
  if (s.kind == BLING_SHAPE_CYLINDER) return cylinder_test(s.params, r, tmax, any, t);
  if (any) return box_any(s.params, Ray{r.o, r.d, r.tmin, tmax});
  return box_test(s.params, r, tmax, t);
}

}  // namespace bd
