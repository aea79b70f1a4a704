// ocore.h -- ORACLE (test infrastructure only; never linked into the product path).
//
// Binary32 restatement of the reference's math, spectrum and sampling primitives, keeping the
// Haskell evaluation order (left folds from 0, no fused multiply-adds: build with
// -ffp-contract=off).  Each function cites the reference file:line it follows; paths are relative
// to src/lib/Graphics/Bling/ of bindingflare/bling.
#pragma once
#include "../bling_amd/csrc/common/perlin.h"
#include "../bling_amd/csrc/common/cellnoise.h"
#include "../bling_amd/csrc/common/cr_math.h"
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>

#include "../bling_amd/csrc/common/spectral_data.h"  // derived CIE / RGB band data (generated)

namespace ora {

const float PI = 3.14159265358979323846f;                 // pi :: Float
const float INF = std::numeric_limits<float>::infinity();
const float INV_PI = 1.f / PI;                             // Math.hs:49-51
const float INV_TWO_PI = 1.f / (2.f * PI);                 // Math.hs:53-55
const float TWO_PI = 2.f * PI;                             // Math.hs:57-59

// Haskell's default Ord max/min: max x y = if x <= y then y else x (NaN-sensitive order matters)
inline float hmax(float x, float y) { return x <= y ? y : x; }
inline float hmin(float x, float y) { return x <= y ? x : y; }
inline float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }  // Math.hs:78-87
inline float lerp(float t, float a, float b) { return (1.f - t) * a + t * b; }                // Math.hs:108-110

struct V { float x, y, z; };
inline V mk(float x, float y, float z) { return V{x, y, z}; }
inline V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V operator*(V a, V b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V operator-(V a) { return {-a.x, -a.y, -a.z}; }
inline V sm(float f, V v) { return {f * v.x, f * v.y, f * v.z}; }       // (*#) f v = vpromote f * v
inline V vs(V v, float f) { return {v.x * f, v.y * f, v.z * f}; }       // v * vpromote f
inline float comp(V v, int d) { return d == 0 ? v.x : (d == 1 ? v.y : v.z); }
inline void setc(V& v, int d, float t) { if (d == 0) v.x = t; else if (d == 1) v.y = t; else v.z = t; }
inline float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }                    // Math.hs:341-343
inline float absdot(V a, V b) { return std::fabs(dot(a, b)); }
inline V cross(V u, V v) { return {u.y * v.z - u.z * v.y, -(u.x * v.z - u.z * v.x), u.x * v.y - u.y * v.x}; }
inline float sqlen(V v) { return v.x * v.x + v.y * v.y + v.z * v.z; }                       // Math.hs:328-330
inline float len(V v) { return std::sqrt(sqlen(v)); }
inline V normalize(V v) {                                                                   // Math.hs:349-353
  if (sqlen(v) != 0.f) return vs(v, 1.f / len(v));
  return {0.f, 1.f, 0.f};
}

struct Ray { V o, d; float tmin, tmax; };
inline V ray_at(const Ray& r, float t) { return r.o + vs(r.d, t); }                         // Math.hs:388-390

struct LC { V s, t, n; };                                                                    // Math.hs:408-411
inline LC coordinate_system(V v) {                                                           // Math.hs:413-425
  if (std::fabs(v.x) > std::fabs(v.y)) {
    float il = 1.f / std::sqrt(v.x * v.x + v.z * v.z);
    V v2 = mk(-v.z * il, 0.f, v.x * il);
    return LC{v2, cross(v, v2), v};
  }
  float il = 1.f / std::sqrt(v.y * v.y + v.z * v.z);
  V v2 = mk(0.f, v.z * il, -v.y * il);
  return LC{v2, cross(v, v2), v};
}
inline V world_to_local(const LC& c, V v) { return {dot(v, c.s), dot(v, c.t), dot(v, c.n)}; }  // :439-441
inline V local_to_world(const LC& c, V v) {                                                  // :443-449
  return {c.s.x * v.x + c.t.x * v.y + c.n.x * v.z,
          c.s.y * v.x + c.t.y * v.y + c.n.y * v.z,
          c.s.z * v.x + c.t.z * v.y + c.n.z * v.z};
}

// solveQuadric (Math.hs:124-139)
inline bool solve_quadric(float a, float b, float c, float* t0, float* t1) {
  float discrim = b * b - 4.f * a * c;
  if (discrim < 0.f) return false;
  float rd = std::sqrt(discrim);
  float q = b < 0.f ? -0.5f * (b - rd) : -0.5f * (b + rd);
  float x0 = q / a, x1 = c / q;
  *t0 = hmin(x0, x1);
  *t1 = hmax(x0, x1);
  return true;
}

inline float atan2p(float y, float x) { float a = bcr::atan2f(y, x); return a < 0.f ? a + TWO_PI : a; }  // Math.hs:69-75

// Transform application with a row-major 4x4 (Transform.hs:247-278)
inline V xpoint(const float* m, V p) {
  float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
  float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
  float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
  float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
  if (wp == 1.f) return {xp, yp, zp};
  return {xp / wp, yp / wp, zp / wp};
}
inline V xvector(const float* m, V v) {
  return {m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
          m[8] * v.x + m[9] * v.y + m[10] * v.z};
}
inline V xnormal(const float* inv, V n) {  // uses the stored inverse, transposed
  return {inv[0] * n.x + inv[4] * n.y + inv[8] * n.z, inv[1] * n.x + inv[5] * n.y + inv[9] * n.z,
          inv[2] * n.x + inv[6] * n.y + inv[10] * n.z};
}

// ------------------------------------------------------------------ Spectrum.hs (16 bands)
struct S { float v[16]; };
inline S sconst(float x) { S s; for (int i = 0; i < 16; ++i) s.v[i] = x; return s; }
inline S black() { return sconst(0.f); }
inline S white() { return sconst(1.f); }
inline S operator+(const S& a, const S& b) { S r; for (int i = 0; i < 16; ++i) r.v[i] = a.v[i] + b.v[i]; return r; }
inline S operator-(const S& a, const S& b) { S r; for (int i = 0; i < 16; ++i) r.v[i] = a.v[i] - b.v[i]; return r; }
inline S operator*(const S& a, const S& b) { S r; for (int i = 0; i < 16; ++i) r.v[i] = a.v[i] * b.v[i]; return r; }
inline S operator/(const S& a, const S& b) { S r; for (int i = 0; i < 16; ++i) r.v[i] = a.v[i] / b.v[i]; return r; }
inline S sscale(const S& a, float f) { S r; for (int i = 0; i < 16; ++i) r.v[i] = a.v[i] * f; return r; }   // :448-450
inline S smap_exp(const S& a) { S r; for (int i = 0; i < 16; ++i) r.v[i] = bcr::expf(a.v[i]); return r; }   // exp = sMap exp (:383-386)
inline S sclamp(const S& a, float lo, float hi) {                                            // :453-456
  S r; for (int i = 0; i < 16; ++i) r.v[i] = hmax(lo, hmin(hi, a.v[i])); return r;
}
inline bool is_black(const S& a) { for (int i = 0; i < 16; ++i) if (!(a.v[i] == 0.f)) return false; return true; }  // :444-446
inline bool s_nan(const S& a) { for (int i = 0; i < 16; ++i) if (std::isnan(a.v[i])) return true; return false; }
inline bool s_inf(const S& a) { for (int i = 0; i < 16; ++i) if (std::isinf(a.v[i])) return true; return false; }
inline float sY(const S& a) {                                                                // :371-373
  float acc = 0.f;
  for (int i = 0; i < 16; ++i) acc = acc + a.v[i] * BLING_CIE_Y_BANDS[i];
  return acc / BLING_CIE_Y_SUM;
}
inline void to_xyz(const S& a, float* x, float* y, float* z) {                              // :349-355
  float ax = 0.f, ay = 0.f, az = 0.f;
  for (int i = 0; i < 16; ++i) {
    ax = ax + BLING_CIE_X_BANDS[i] * a.v[i];
    ay = ay + BLING_CIE_Y_BANDS[i] * a.v[i];
    az = az + BLING_CIE_Z_BANDS[i] * a.v[i];
  }
  *x = ax / BLING_CIE_Y_SUM; *y = ay / BLING_CIE_Y_SUM; *z = az / BLING_CIE_Y_SUM;
}
inline S from_array(const float* p) { S s; std::memcpy(s.v, p, sizeof s.v); return s; }

// ------------------------------------------------------------------ Montecarlo.hs
inline void concentric_sample_disk(float u1, float u2, float* ox, float* oy) {              // :389-406
  float sx = u1 * 2.f - 1.f, sy = u2 * 2.f - 1.f;
  if (sx == 0.f && sy == 0.f) { *ox = 0.f; *oy = 0.f; return; }
  float r, th;
  if (sx >= -sy) {
    if (sx > sy) { if (sy > 0.f) { r = sx; th = sy / sx; } else { r = sx; th = 8.f + sy / sx; } }
    else { r = sy; th = 2.f - sx / sy; }
  } else if (sx <= sy) { r = -sx; th = 4.f - sy / (-sx); }
  else { r = -sy; th = 6.f + sx / (-sy); }
  float theta = th * PI / 4.f;
  *ox = r * bcr::cosf(theta);
  *oy = r * bcr::sinf(theta);
}
inline V cosine_sample_hemisphere(float u1, float u2) {                                      // :375-378
  float x, y;
  concentric_sample_disk(u1, u2, &x, &y);
  return mk(x, y, std::sqrt(hmax(0.f, 1.f - x * x - y * y)));
}
inline float power_heuristic(float fp, float gp) {                                           // :342-345
  float f = 1.f * fp, g = 1.f * gp;
  return (f * f) / (f * f + g * g);
}
inline V uniform_sample_cone(const LC& c, float cosmax, float u1, float u2) {               // :362-373
  float ct = lerp(u1, cosmax, 1.f);
  float st = std::sqrt(1.f - ct * ct);
  float phi = u2 * TWO_PI;
  return vs(c.s, bcr::cosf(phi) * st) + vs(c.t, bcr::sinf(phi) * st) + vs(c.n, ct);
}
inline V uniform_sample_sphere(float u1, float u2) {                                          // :410-415
  float u = u1 * 2.f - 1.f;
  float s = std::sqrt(1.f - u * u);
  float om = u2 * 2.f * PI;
  return mk(s * bcr::cosf(om), s * bcr::sinf(om), u);
}
inline float uniform_cone_pdf(float cosmax) { return cosmax >= 1.f ? 0.f : 1.f / (TWO_PI * (1.f - cosmax)); }  // :356-360

// ------------------------------------------------------------------ counter RNG (oracle copy)
// Restatement of the counter-based sampler RNG that replaces MWC256 (Random.hs:56-96), specification
// version 2 (round 6).  The product's definition is bling_amd/csrc/common/counter_rng.h; tests check
// both agree bit for bit.  value = fmix(fmix(pkey ^ sample * 0x9E3779B9) ^ fmix(dim ^ 0x2C1B3C6D)),
// pkey = mix(mix(seed, pass), pixel).
inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t mmix(uint32_t h, uint32_t k) {
  k *= 0xcc9e2d51u; k = rotl(k, 15); k *= 0x1b873593u;
  h ^= k; h = rotl(h, 13); return h * 5u + 0xe6546b64u;
}
inline uint32_t fmix(uint32_t h) { h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h; }
inline uint32_t hash5(uint32_t seed, uint32_t pass, uint32_t pixel, uint32_t sample, uint32_t dim) {
  const uint32_t pkey = mmix(mmix(seed, pass), pixel);
  const uint32_t skey = fmix(pkey ^ sample * 0x9E3779B9u);
  return fmix(skey ^ fmix(dim ^ 0x2C1B3C6Du));
}
inline float u01(uint32_t h) { return (float)(h >> 8) * (1.f / 16777216.f); }
// Kensler, "Correlated Multi-Jittered Sampling" (Pixar TM 13-01): hashed bijection on [0, l)
inline uint32_t permute(uint32_t i, uint32_t l, uint32_t p) {
  if (l <= 1) return 0;
  uint32_t w = l - 1;
  w |= w >> 1; w |= w >> 2; w |= w >> 4; w |= w >> 8; w |= w >> 16;
  do {
    i ^= p; i *= 0xe170893du; i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8; i *= 0x0929eb3fu; i ^= p >> 23;
    i ^= (i & w) >> 1; i *= 1u | p >> 27; i *= 0x6935fa69u; i ^= (i & w) >> 11; i *= 0x74dcb303u;
    i ^= (i & w) >> 2; i *= 0x9e501cc3u; i ^= (i & w) >> 2; i *= 0xc860a3dfu; i &= w; i ^= i >> 5;
  } while (i >= l);
  return (i + p) % l;
}

enum : uint32_t {
  DIM_PIX = 0x1000u, DIM_LENS_PERM = 0x2000u, DIM_LENS_J = 0x2100u,
  DIM_1D_PERM = 0x3000u, DIM_1D_J = 0x4000u, DIM_2D_PERM = 0x5000u, DIM_2D_J = 0x6000u,
  DIM_FRESH1D = 0x7000u, DIM_FRESH2D = 0x8000u, DIM_RAND_CAM = 0x9000u, ALL_SAMPLES = 0xFFFFFFFFu
};
const float ALMOST_ONE = 0x1.fffffep-1f;                   // Sampling.hs:154-155

}  // namespace ora
