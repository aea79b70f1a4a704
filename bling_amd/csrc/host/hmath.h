// hmath.h -- host-side binary32 math with the reference's evaluation order.
//
// Used by the scene loader (which stands in for the unchanged Haskell parser) to build transforms,
// cameras, spectra and filter tables bit-for-bit as the reference would.  Compile with
// -ffp-contract=off: GHC emits no fused multiply-adds.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

namespace bh {

static const float kPi = 3.14159265358979323846f;   // `pi :: Float`

struct V3 { float x, y, z; };
inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }          // Math.hs:341-343
inline V3 cross(V3 u, V3 v) {                                                          // Math.hs:336-339
  return {u.y * v.z - u.z * v.y, -(u.x * v.z - u.z * v.x), u.x * v.y - u.y * v.x};
}
inline float sqlen(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
inline V3 normalize(V3 v) {                                                            // Math.hs:349-353
  if (sqlen(v) != 0.f) { float il = 1.f / std::sqrt(sqlen(v)); return v * V3{il, il, il}; }
  return {0.f, 1.f, 0.f};
}
inline float radians(float d) { return d / 180.f * kPi; }                              // Math.hs:62-66

// Haskell default Ord max/min (max x y = if x <= y then y else x).
inline float hmax(float x, float y) { return x <= y ? y : x; }
inline float hmin(float x, float y) { return x <= y ? x : y; }

// ---------------------------------------------------------------- Transform.hs
struct M4 { float m[16]; };
inline float mi(const M4& a, int r, int c) { return a.m[r * 4 + c]; }

inline M4 identityM() { M4 r{}; r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.f; return r; }

// `mul m1 m2` (Transform.hs:102-105): element (i,j) = sum_k m1[k][j] * m2[i][k], a left fold from 0.
inline M4 mul(const M4& m1, const M4& m2) {
  M4 r;
  for (int n = 0; n < 16; ++n) {
    int i = n / 4, j = n % 4;
    float s = 0.f;
    for (int k = 0; k < 4; ++k) s = s + mi(m1, k, j) * mi(m2, i, k);
    r.m[n] = s;
  }
  return r;
}

inline M4 transposeM(const M4& a) {
  M4 r;
  for (int n = 0; n < 16; ++n) { int i = n / 4, j = n % 4; r.m[n] = mi(a, j, i); }
  return r;
}

// `invert` (Transform.hs:44-87): Gauss-Jordan with full pivoting, operating on the storage with
// idx r c = c*4 + r; `maximumBy` keeps the LAST maximum.
inline M4 invert(const M4& a) {
  float v[16];
  std::memcpy(v, a.m, sizeof v);
  auto idx = [](int r, int c) { return c * 4 + r; };
  int ipiv[4] = {0, 1, 2, 3};
  int npiv = 4;
  int indx_r[4], indx_c[4];
  for (int it = 0; it < 4; ++it) {
    int irow = -1, icol = -1;
    float best = 0.f;
    bool first = true;
    for (int a1 = 0; a1 < npiv; ++a1)
      for (int b1 = 0; b1 < npiv; ++b1) {
        int j = ipiv[a1], k = ipiv[b1];
        float x = std::fabs(v[idx(j, k)]);
        if (first || !(x < best)) { best = x; irow = j; icol = k; first = false; }  // ties -> later
      }
    // remove icol from ipiv
    int w = 0;
    for (int q = 0; q < npiv; ++q) if (ipiv[q] != icol) ipiv[w++] = ipiv[q];
    npiv = w;
    if (irow != icol)
      for (int k = 0; k < 4; ++k) { float t = v[idx(irow, k)]; v[idx(irow, k)] = v[idx(icol, k)]; v[idx(icol, k)] = t; }
    float pivinv = 1.f / v[idx(icol, icol)];
    v[idx(icol, icol)] = 1.f;
    for (int j = 0; j < 4; ++j) v[idx(icol, j)] = v[idx(icol, j)] * pivinv;
    for (int j = 0; j < 4; ++j) {
      if (j == icol) continue;
      float save = v[idx(j, icol)];
      v[idx(j, icol)] = 0.f;
      for (int k = 0; k < 4; ++k) v[idx(j, k)] = v[idx(j, k)] - v[idx(icol, k)] * save;
    }
    indx_r[it] = irow;
    indx_c[it] = icol;
  }
  for (int it = 3; it >= 0; --it) {
    int ir = indx_r[it], ic = indx_c[it];
    if (ir != ic)
      for (int k = 0; k < 4; ++k) { float t = v[idx(k, ir)]; v[idx(k, ir)] = v[idx(k, ic)]; v[idx(k, ic)] = t; }
  }
  M4 r;
  std::memcpy(r.m, v, sizeof v);
  return r;
}

struct Xf { M4 m, inv; };
inline Xf identityX() { return Xf{identityM(), identityM()}; }
// concatTrans (Transform.hs:241-244): (t1 <> t2) applies t1 first.
inline Xf cat(const Xf& a, const Xf& b) { return Xf{mul(a.m, b.m), mul(b.inv, a.inv)}; }
inline Xf inverseX(const Xf& t) { return Xf{t.inv, t.m}; }

inline M4 mat(float a, float b, float c, float d, float e, float f, float g, float h,
              float i, float j, float k, float l, float m, float n, float o, float p) {
  M4 r; float t[16] = {a, b, c, d, e, f, g, h, i, j, k, l, m, n, o, p};
  std::memcpy(r.m, t, sizeof t); return r;
}

inline Xf translateX(V3 d) {                                                           // :148-160
  return Xf{mat(1, 0, 0, d.x, 0, 1, 0, d.y, 0, 0, 1, d.z, 0, 0, 0, 1),
            mat(1, 0, 0, -d.x, 0, 1, 0, -d.y, 0, 0, 1, -d.z, 0, 0, 0, 1)};
}
inline Xf scaleX(V3 s) {                                                               // :163-174
  return Xf{mat(s.x, 0, 0, 0, 0, s.y, 0, 0, 0, 0, s.z, 0, 0, 0, 0, 1),
            mat(1.f / s.x, 0, 0, 0, 0, 1.f / s.y, 0, 0, 0, 0, 1.f / s.z, 0, 0, 0, 0, 1)};
}
inline Xf rotateXX(float deg) {                                                        // :176-184
  float s = std::sin(radians(deg)), c = std::cos(radians(deg));
  M4 m = mat(1, 0, 0, 0, 0, c, -s, 0, 0, s, c, 0, 0, 0, 0, 1);
  return Xf{m, transposeM(m)};
}
inline Xf rotateYX(float deg) {                                                        // :186-194
  float c = std::cos(radians(deg)), s = std::sin(radians(deg));
  M4 m = mat(c, 0, s, 0, 0, 1, 0, 0, -s, 0, c, 0, 0, 0, 0, 1);
  return Xf{m, transposeM(m)};
}
inline Xf rotateZX(float deg) {                                                        // :196-204
  float s = std::sin(radians(deg)), c = std::cos(radians(deg));
  M4 m = mat(c, -s, 0, 0, s, c, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1);
  return Xf{m, transposeM(m)};
}
inline Xf fromMatrixX(const M4& m) { return Xf{m, invert(m)}; }                        // :140-141
inline Xf perspectiveX(float fov, float n, float f) {                                  // :207-219
  float iTan = 1.f / std::tan(radians(fov) / 2.f);
  M4 m = mat(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, f / (f - n), -(f * n / (f - n)), 0, 0, 1, 0);
  return cat(scaleX(v3(iTan, iTan, 1.f)), Xf{m, invert(m)});
}
inline Xf lookAtX(V3 p, V3 l, V3 up) {                                                 // :222-235
  V3 dir = normalize(l - p);
  V3 left = normalize(cross(normalize(up), dir));
  V3 u = cross(dir, left);
  M4 m = mat(left.x, u.x, dir.x, p.x, left.y, u.y, dir.y, p.y, left.z, u.z, dir.z, p.z, 0, 0, 0, 1);
  return Xf{m, invert(m)};
}

// transPoint / transVector / transNormal (Transform.hs:247-272)
inline V3 xpoint(const M4& m, V3 p) {
  float xp = mi(m, 0, 0) * p.x + mi(m, 0, 1) * p.y + mi(m, 0, 2) * p.z + mi(m, 0, 3);
  float yp = mi(m, 1, 0) * p.x + mi(m, 1, 1) * p.y + mi(m, 1, 2) * p.z + mi(m, 1, 3);
  float zp = mi(m, 2, 0) * p.x + mi(m, 2, 1) * p.y + mi(m, 2, 2) * p.z + mi(m, 2, 3);
  float wp = mi(m, 3, 0) * p.x + mi(m, 3, 1) * p.y + mi(m, 3, 2) * p.z + mi(m, 3, 3);
  if (wp == 1.f) return {xp, yp, zp};
  return {xp / wp, yp / wp, zp / wp};
}
inline V3 xvector(const M4& m, V3 v) {
  return {mi(m, 0, 0) * v.x + mi(m, 0, 1) * v.y + mi(m, 0, 2) * v.z,
          mi(m, 1, 0) * v.x + mi(m, 1, 1) * v.y + mi(m, 1, 2) * v.z,
          mi(m, 2, 0) * v.x + mi(m, 2, 1) * v.y + mi(m, 2, 2) * v.z};
}
inline V3 xnormal(const M4& inv, V3 n) {
  return {mi(inv, 0, 0) * n.x + mi(inv, 1, 0) * n.y + mi(inv, 2, 0) * n.z,
          mi(inv, 0, 1) * n.x + mi(inv, 1, 1) * n.y + mi(inv, 2, 1) * n.z,
          mi(inv, 0, 2) * n.x + mi(inv, 1, 2) * n.y + mi(inv, 2, 2) * n.z};
}

// Haskell `round` for Float -> Int: round half to even.
inline long hround(float x) { return std::lrint(static_cast<double>(x)); }

}  // namespace bh
