// dev_common.h -- device math for the MI355X core: float3 algebra, 16-band spectra in registers and
// the reference's binary32 evaluation order (built with -ffp-contract=off, no fast-math).
// Formulas restate src/lib/Graphics/Bling/{Math,Spectrum,Montecarlo}.hs of the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../common/counter_rng.h"
#include "../common/spectral_data.h"
#include "../common/cr_math.h"

#define DEV __device__ __forceinline__

namespace bd {

constexpr float PI = 3.14159265358979323846f;
constexpr float TWO_PI = 2.f * PI;
constexpr float INV_PI = 1.f / PI;
constexpr float INV_TWO_PI = 1.f / (2.f * PI);
constexpr float ALMOST_ONE = 0x1.fffffep-1f;

// Haskell default Ord max/min
DEV float hmax(float x, float y) { return x <= y ? y : x; }
DEV float hmin(float x, float y) { return x <= y ? x : y; }
DEV float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
DEV float lerpf(float t, float a, float b) { return (1.f - t) * a + t * b; }

struct V3 { float x, y, z; };
DEV V3 mk(float x, float y, float z) { return V3{x, y, z}; }
DEV V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
DEV V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
DEV V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
DEV V3 sm(float f, V3 v) { return {f * v.x, f * v.y, f * v.z}; }
DEV V3 vs(V3 v, float f) { return {v.x * f, v.y * f, v.z * f}; }
DEV float comp(V3 v, int d) { return d == 0 ? v.x : (d == 1 ? v.y : v.z); }
DEV float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEV V3 cross(V3 u, V3 v) { return {u.y * v.z - u.z * v.y, -(u.x * v.z - u.z * v.x), u.x * v.y - u.y * v.x}; }
DEV float sqlen(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
DEV float len(V3 v) { return sqrtf(sqlen(v)); }
DEV V3 normalize(V3 v) {
  if (sqlen(v) != 0.f) return vs(v, 1.f / len(v));
  return {0.f, 1.f, 0.f};
}

struct Ray { V3 o, d; float tmin, tmax; };
DEV V3 ray_at(const Ray& r, float t) { return r.o + vs(r.d, t); }

struct LC { V3 s, t, n; };
DEV LC coordinate_system(V3 v) {                                   // Math.hs:413-425
  if (fabsf(v.x) > fabsf(v.y)) {
    float il = 1.f / sqrtf(v.x * v.x + v.z * v.z);
    V3 v2 = mk(-v.z * il, 0.f, v.x * il);
    return LC{v2, cross(v, v2), v};
  }
  float il = 1.f / sqrtf(v.y * v.y + v.z * v.z);
  V3 v2 = mk(0.f, v.z * il, -v.y * il);
  return LC{v2, cross(v, v2), v};
}
DEV V3 world_to_local(const LC& c, V3 v) { return {dot(v, c.s), dot(v, c.t), dot(v, c.n)}; }
DEV V3 local_to_world(const LC& c, V3 v) {
  return {c.s.x * v.x + c.t.x * v.y + c.n.x * v.z, c.s.y * v.x + c.t.y * v.y + c.n.y * v.z,
          c.s.z * v.x + c.t.z * v.y + c.n.z * v.z};
}

DEV bool solve_quadric(float a, float b, float c, float* t0, float* t1) {   // Math.hs:124-139
  float discrim = b * b - 4.f * a * c;
  if (discrim < 0.f) return false;
  float rd = sqrtf(discrim);
  float q = b < 0.f ? -0.5f * (b - rd) : -0.5f * (b + rd);
  float x0 = q / a, x1 = c / q;
  *t0 = hmin(x0, x1);
  *t1 = hmax(x0, x1);
  return true;
}
DEV float atan2p(float y, float x) { float a = bcr::atan2f(y, x); return a < 0.f ? a + TWO_PI : a; }

// row-major 4x4 application (Transform.hs:247-272)
DEV V3 xpoint(const float* m, V3 p) {
  float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
  float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
  float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
  float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
  if (wp == 1.f) return {xp, yp, zp};
  return {xp / wp, yp / wp, zp / wp};
}
DEV V3 xvector(const float* m, V3 v) {
  return {m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z, m[8] * v.x + m[9] * v.y + m[10] * v.z};
}
DEV V3 xnormal(const float* inv, V3 n) {
  return {inv[0] * n.x + inv[4] * n.y + inv[8] * n.z, inv[1] * n.x + inv[5] * n.y + inv[9] * n.z,
          inv[2] * n.x + inv[6] * n.y + inv[10] * n.z};
}

// ------------------------------------------------------------ spectra (16 bands in registers)
struct Sp { float v[16]; };
#define SP_LOOP _Pragma("unroll") for (int i = 0; i < 16; ++i)
DEV Sp sconst(float x) { Sp s; SP_LOOP s.v[i] = x; return s; }
DEV Sp sload(const float* p) { Sp s; SP_LOOP s.v[i] = p[i]; return s; }
DEV Sp operator+(const Sp& a, const Sp& b) { Sp r; SP_LOOP r.v[i] = a.v[i] + b.v[i]; return r; }
DEV Sp operator-(const Sp& a, const Sp& b) { Sp r; SP_LOOP r.v[i] = a.v[i] - b.v[i]; return r; }
DEV Sp operator*(const Sp& a, const Sp& b) { Sp r; SP_LOOP r.v[i] = a.v[i] * b.v[i]; return r; }
DEV Sp operator/(const Sp& a, const Sp& b) { Sp r; SP_LOOP r.v[i] = a.v[i] / b.v[i]; return r; }
DEV Sp sscale(const Sp& a, float f) { Sp r; SP_LOOP r.v[i] = a.v[i] * f; return r; }
DEV Sp sclamp01(const Sp& a) { Sp r; SP_LOOP r.v[i] = hmax(0.f, hmin(1.f, a.v[i])); return r; }
DEV bool is_black(const Sp& a) { bool b = true; SP_LOOP b = b && (a.v[i] == 0.f); return b; }
DEV bool s_bad(const Sp& a) { bool b = false; SP_LOOP b = b || __builtin_isnan(a.v[i]) || __builtin_isinf(a.v[i]); return b; }
DEV float sY(const Sp& a) {                                         // Spectrum.hs:371-373
  float acc = 0.f;
  SP_LOOP acc = acc + a.v[i] * BLING_CIE_Y_BANDS[i];
  return acc / BLING_CIE_Y_SUM;
}
DEV void to_xyz(const Sp& a, float* x, float* y, float* z) {       // Spectrum.hs:349-355
  float ax = 0.f, ay = 0.f, az = 0.f;
  SP_LOOP {
    ax = ax + BLING_CIE_X_BANDS[i] * a.v[i];
    ay = ay + BLING_CIE_Y_BANDS[i] * a.v[i];
    az = az + BLING_CIE_Z_BANDS[i] * a.v[i];
  }
  *x = ax / BLING_CIE_Y_SUM; *y = ay / BLING_CIE_Y_SUM; *z = az / BLING_CIE_Y_SUM;
}

// ------------------------------------------------------------ Montecarlo.hs warps
DEV void concentric_sample_disk(float u1, float u2, float* ox, float* oy) {  // :389-406
  float sx = u1 * 2.f - 1.f, sy = u2 * 2.f - 1.f;
  if (sx == 0.f && sy == 0.f) { *ox = 0.f; *oy = 0.f; return; }
  float r, th;
  if (sx >= -sy) {
    if (sx > sy) { if (sy > 0.f) { r = sx; th = sy / sx; } else { r = sx; th = 8.f + sy / sx; } }
    else { r = sy; th = 2.f - sx / sy; }
  } else if (sx <= sy) { r = -sx; th = 4.f - sy / (-sx); }
  else { r = -sy; th = 6.f + sx / (-sy); }
  float theta = th * PI / 4.f;
  const bcr::SinCos sc = bcr::sincosf(theta);
  *ox = r * sc.c;
  *oy = r * sc.s;
}
DEV V3 cosine_sample_hemisphere(float u1, float u2) {
  float x, y;
  concentric_sample_disk(u1, u2, &x, &y);
  return mk(x, y, sqrtf(hmax(0.f, 1.f - x * x - y * y)));
}
DEV float power_heuristic(float fp, float gp) { float f = 1.f * fp, g = 1.f * gp; return (f * f) / (f * f + g * g); }
DEV V3 uniform_sample_cone(const LC& c, float cosmax, float u1, float u2) {
  float ct = lerpf(u1, cosmax, 1.f);
  float st = sqrtf(1.f - ct * ct);
  float phi = u2 * TWO_PI;
  const bcr::SinCos sc = bcr::sincosf(phi);
  return vs(c.s, sc.c * st) + vs(c.t, sc.s * st) + vs(c.n, ct);
}
DEV V3 uniform_sample_sphere(float u1, float u2) {
  float u = u1 * 2.f - 1.f;
  float s = sqrtf(1.f - u * u);
  float om = u2 * 2.f * PI;
  const bcr::SinCos sc = bcr::sincosf(om);
  return mk(s * sc.c, s * sc.s, u);
}
DEV float uniform_cone_pdf(float cosmax) { return cosmax >= 1.f ? 0.f : 1.f / (TWO_PI * (1.f - cosmax)); }

// ------------------------------------------------------------ wave helpers
DEV uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace bd
