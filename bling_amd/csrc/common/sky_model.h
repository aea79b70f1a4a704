// sky_model.h -- Perez sun/sky environment map (SunSky.hs:12-125) and the infinite light's Dist2D
// construction (Light.hs:72-82, Montecarlo.hs:40-104).  Product code shared by the host loader
// (precompute + importance-sampling tables) and the HIP kernels (per-lookup evaluation).
// Evaluation order follows the Haskell expressions; compile with -ffp-contract=off.
#pragma once
#include <stdint.h>
#include "../../../include/bling_scene.h"
#include "spectral_data.h"
#include "cr_math.h"
#include "image_tex.h"

#if defined(__HIPCC__)
#define BLING_HD __host__ __device__ inline
#else
#define BLING_HD inline
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
#include <cmath>
#endif

namespace bsky {

BLING_HD float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }  // Math.hs:78-87

// xyzToRgb (Spectrum.hs:162-168) then rgbToSpectrumIllum (Spectrum.hs:140-159), into out[16]
BLING_HD void xyz_to_spectrum(float x, float y, float z, float* out) {
  float r = 3.240479f * x - 1.537150f * y - 0.498535f * z;
  float g = (-0.969256f) * x + 1.875991f * y + 0.041556f * z;
  float b = 0.055648f * x - 0.204043f * y + 1.057311f * z;
  const float (*B)[16] = BLING_RGB_ILLUM_BANDS;
  // bases: 0 r, 1 g, 2 b, 3 c, 4 m, 5 y, 6 w
  int w1, w2; float a0, a1, a2;
  if (r <= g && r <= b) {
    a0 = r;
    if (g <= b) { w1 = 3; a1 = g - r; w2 = 2; a2 = b - g; } else { w1 = 3; a1 = b - r; w2 = 1; a2 = g - b; }
  } else if (g <= r && g <= b) {
    a0 = g;
    if (r <= b) { w1 = 4; a1 = r - g; w2 = 2; a2 = b - r; } else { w1 = 4; a1 = b - g; w2 = 0; a2 = r - b; }
  } else {
    a0 = b;
    if (r <= b) { w1 = 5; a1 = r - b; w2 = 1; a2 = g - r; } else { w1 = 5; a1 = g - b; w2 = 0; a2 = r - g; }
  }
  for (int i = 0; i < 16; ++i) out[i] = B[6][i] * a0 + (B[w1][i] * a1 + B[w2][i] * a2);
}

// chromaticityToXYZ (Spectrum.hs:229-251)
BLING_HD void chromaticity_to_xyz(float x, float y, float* X, float* Y, float* Z) {
  float den = 0.0241f + 0.2562f * x - 0.7341f * y;
  float m1 = (-1.3515f - 1.7703f * x + 5.9114f * y) / den;
  float m2 = (0.03f - 31.4424f * x + 30.0717f * y) / den;
  *X = BLING_S_XYZ[0][0] + m1 * BLING_S_XYZ[1][0] + m2 * BLING_S_XYZ[2][0];
  *Y = BLING_S_XYZ[0][1] + m1 * BLING_S_XYZ[1][1] + m2 * BLING_S_XYZ[2][1];
  *Z = BLING_S_XYZ[0][2] + m1 * BLING_S_XYZ[1][2] + m2 * BLING_S_XYZ[2][2];
}

// perez (SunSky.hs:81-86)
BLING_HD float perez(const float* p, float sunT, float t, float g, float lvz) {
  float csg = bcr::cosf(g), cst = bcr::cosf(sunT);
  float num = (1.f + p[0] * bcr::expf(p[1] / bcr::cosf(t))) * (1.f + p[2] * bcr::expf(p[3] * g)) + p[4] * csg * csg;
  float den = (1.f + p[0] * bcr::expf(p[1])) * (1.f + p[2] * bcr::expf(p[3] * sunT)) + p[4] * cst * cst;
  return lvz * num / den;
}

// sunThetaMax2 (SunSky.hs:39-43); sint2 is NOT squared (kept as written)
BLING_HD float sun_theta_max2() { return sqrtf(fmaxf(0.f, 1.f - 6.955e5f / 1.496e8f)); }

// texMapEval of mkSunSkyLight for a light-space direction `dir` (= sphToDir (cartToSph uv)):
// skySpectrum ssd dir + sunSpectrum sunLocal sunR dir (SunSky.hs:18-20, 67-94).
BLING_HD void sky_eval(const bling_light* L, float dx, float dy, float dz, float* out) {
  float sky[16];
  float dzn = -dz;
  if (dzn < 1e-4f) {
    for (int i = 0; i < 16; ++i) sky[i] = 0.f;
  } else {
    float theta = bcr::acosf(dzn);
    float dd = dx * L->sun_dir_local[0] + dy * L->sun_dir_local[1] + dz * L->sun_dir_local[2];
    float gamma = bcr::acosf(clampf(dd, -1.f, 1.f));
    float x = perez(L->perez_x, L->sun_theta, theta, gamma, L->zenith_x);
    float y = perez(L->perez_y, L->sun_theta, theta, gamma, L->zenith_y);
    float yy = perez(L->perez_Y, L->sun_theta, theta, gamma, L->zenith_Y) * 1e-4f;
    float cx, cy, cz;
    chromaticity_to_xyz(x, y, &cx, &cy, &cz);
    xyz_to_spectrum(cx * yy / cy, yy, cz * yy / cy, sky);
  }
  // sunSpectrum: d = (sunD * (1,1,-1)) `dot` dir
  float d = L->sun_dir_local[0] * dx + L->sun_dir_local[1] * dy + (L->sun_dir_local[2] * -1.f) * dz;
  bool sun = d > sun_theta_max2();
  for (int i = 0; i < 16; ++i) out[i] = sky[i] + (sun ? L->sun_radiance[i] : 0.f);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// ------------------------------------------------------------------ host-only precompute
BLING_HD float lerpf(float t, float a, float b) { return (1.f - t) * a + t * b; }

inline float eval_regular(float l0, float l1, const float* a, int n, float l) {  // Spectrum.hs:271-280
  if (l <= l0) return a[0];
  if (l >= l1) return a[n - 1];
  float d1 = 1.f / ((l1 - l0) / (float)(n - 1));
  float x = (l - l0) * d1;
  int b0 = (int)floorf(x);
  int b1 = b0 + 1 < n - 1 ? b0 + 1 : n - 1;
  float dx = x - (float)b0;
  return (1.f - dx) * a[b0] + dx * a[b1];
}

inline float eval_irregular(const float* ls, const float* vs, int n, float l) {    // Spectrum.hs:258-269
  if (l <= ls[0]) return vs[0];
  if (l >= ls[n - 1]) return vs[n - 1];
  int lo = 0, hi = n - 1;
  for (;;) {
    int mid = (lo + hi) / 2;
    if (lo == mid) break;
    if (ls[mid] == l) { lo = mid; break; }
    if (ls[mid] < l) lo = mid; else hi = mid;
  }
  float t = (l - ls[lo]) / (ls[lo + 1] - ls[lo]);
  return lerpf(t, vs[lo], vs[lo + 1]);
}

inline void normalize3(float* v) {
  float sl = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  if (sl != 0.f) { float il = 1.f / sqrtf(sl); v[0] *= il; v[1] *= il; v[2] *= il; }
  else { v[0] = 0.f; v[1] = 1.f; v[2] = 0.f; }
}
inline void cross3(const float* u, const float* v, float* r) {
  r[0] = u[1] * v[2] - u[2] * v[1];
  r[1] = -(u[0] * v[2] - u[2] * v[0]);
  r[2] = u[0] * v[1] - u[1] * v[0];
}

// mkSunSkyLight + initSky + sunSpectrum' (SunSky.hs:12-24, 45-65, 96-125)
inline void bling_sky_init_impl(bling_light* L, float ex, float ey, float ez, float sx, float sy, float sz, float t) {
  // basis = coordinateSystem' (normalize up) (normalize east)   (Math.hs:427-432)
  float up[3] = {0.f, 1.f, 0.f};
  normalize3(up);
  float east[3] = {ex, ey, ez};
  normalize3(east);
  float w[3] = {up[0], up[1], up[2]};
  normalize3(w);
  float u[3];
  cross3(east, w, u);
  normalize3(u);
  float v[3];
  cross3(w, u, v);
  for (int i = 0; i < 3; ++i) { L->sky_basis[i] = u[i]; L->sky_basis[3 + i] = v[i]; L->sky_basis[6 + i] = w[i]; }
  float sd[3] = {sx, sy, sz};
  normalize3(sd);
  float sl[3] = {sd[0] * u[0] + sd[1] * u[1] + sd[2] * u[2],
                 sd[0] * v[0] + sd[1] * v[1] + sd[2] * v[2],
                 sd[0] * w[0] + sd[1] * w[1] + sd[2] * w[2]};
  normalize3(sl);
  for (int i = 0; i < 3; ++i) L->sun_dir_local[i] = sl[i];
  float st = acosf(clampf(sl[2], -1.f, 1.f));
  L->sun_theta = st;
  float st2 = st * st, st3 = st * st * st, t2 = t * t;
  const float pi = 3.14159265358979323846f;
  float chi = (4.f / 9.f - t / 120.f) * (pi - 2.f * st);
  float pY[5] = {0.17872f * t - 1.46303f, -(0.35540f * t) + 0.42749f, -(0.02266f * t) + 5.32505f,
                 0.12064f * t - 2.57705f, -(0.06696f * t) + 0.37027f};
  float px[5] = {-(0.01925f * t) - 0.25922f, -(0.06651f * t) + 0.00081f, -(0.00041f * t) + 0.21247f,
                 -(0.06409f * t) - 0.89887f, -(0.00325f * t) + 0.04517f};
  float py[5] = {-(0.01669f * t) - 0.26078f, -(0.09495f * t) + 0.00921f, -(0.00792f * t) + 0.21023f,
                 -(0.04405f * t) - 1.65369f, -(0.01092f * t) + 0.05291f};
  for (int i = 0; i < 5; ++i) { L->perez_Y[i] = pY[i]; L->perez_x[i] = px[i]; L->perez_y[i] = py[i]; }
  L->zenith_Y = ((4.04530f * t - 4.97100f) * tanf(chi) - 0.2155f * t + 2.4192f) * 1000.f;
  L->zenith_x = (0.00165f * st3 - 0.00374f * st2 + 0.00208f * st) * t2 +
                (-(0.02902f * st3) + 0.06377f * st2 - 0.03202f * st + 0.00394f) * t +
                (0.11693f * st3 - 0.21196f * st2 + 0.06052f * st + 0.25885f);
  L->zenith_y = (0.00275f * st3 - 0.00610f * st2 + 0.00316f * st) * t2 +
                (-(0.04212f * st3) + 0.08970f * st2 - 0.04153f * st + 0.00515f) * t +
                (0.15346f * st3 - 0.26756f * st2 + 0.06669f * st + 0.26688f);
  // sunR = sunSpectrum' ssd turb
  if (sl[2] < 0.f) {
    for (int i = 0; i < 16; ++i) L->sun_radiance[i] = 0.f;
  } else {
    auto sf = [&](float l) {
      float m = 1.f / (cosf(st) + 0.000940f * powf(1.6386f - st, -1.253f));
      float tR = expf(-m * 0.008735f * powf(l / 1000.f, -4.08f));
      float alpha = 1.3f;
      float beta = 0.04608365822050f * t - 0.04586025928522f;
      float tA = expf(-m * beta * powf(l / 1000.f, -alpha));
      float tO = expf(-m * eval_irregular(BLING_KO_LAMBDA, BLING_KO_VALUE, (int)(sizeof(BLING_KO_LAMBDA) / 4), l) * 0.35f);
      float kg = eval_irregular(BLING_KG_LAMBDA, BLING_KG_VALUE, (int)(sizeof(BLING_KG_LAMBDA) / 4), l);
      float tG = expf(-(1.41f * kg * m / powf(1.0f + 118.93f * kg * m, 0.45f)));
      float kwa = eval_irregular(BLING_KWA_LAMBDA, BLING_KWA_VALUE, (int)(sizeof(BLING_KWA_LAMBDA) / 4), l);
      float wv = 2.f;
      float tWA = expf(-(0.2385f * kwa * wv * m / powf(1.f + 20.07f * kwa * wv * m, 0.45f)));
      float sol = eval_regular(380.f, 750.f, BLING_SOL_CURVE_380_750, (int)(sizeof(BLING_SOL_CURVE_380_750) / 4), l);
      return sol * tR * tA * tO * tG * tWA;
    };
    for (int i = 0; i < 16; ++i) {
      float l0 = lerpf((float)i / 16.f, 400.f, 700.f);
      float l1 = lerpf((float)(i + 1) / 16.f, 400.f, 700.f);
      L->sun_radiance[i] = (sf(l0) + sf(l1)) * 0.5f;
    }
  }
}
#endif  // host only

BLING_HD float spectrum_y(const float* s) {  // sY (Spectrum.hs:371-373): left fold from 0
  float acc = 0.f;
  for (int i = 0; i < 16; ++i) acc = acc + s[i] * BLING_CIE_Y_BANDS[i];
  return acc / BLING_CIE_Y_SUM;
}

}  // namespace bsky

#if !defined(__HIP_DEVICE_COMPILE__)
#include <vector>
inline void bling_sky_init(bling_light* L, float ex, float ey, float ez, float sx, float sy, float sz, float t) {
  bsky::bling_sky_init_impl(L, ex, ey, ez, sx, sy, sz, t);
}

// mkDist1D (Montecarlo.hs:40-48): appends func/cdf to the given vectors, returns funcInt
inline float bling_dist1d(const std::vector<float>& f, std::vector<float>& cdf_out) {
  int n = (int)f.size();
  std::vector<float> c(n + 1);
  c[0] = 0.f;
  for (int i = 0; i < n; ++i) c[i + 1] = c[i] + f[i] / (float)n;
  float fi = c[n];
  if (fi != 0.f) for (int i = 0; i <= n; ++i) cdf_out.push_back(c[i] / fi);
  else for (int i = 0; i <= n; ++i) cdf_out.push_back((float)i / (float)n);
  return fi;
}

// mkInfiniteAreaLight's Dist2D: mkDist2D (texSize rmap) (sY . eval) (Light.hs:72-82)
inline void bling_sky_build_dist(bling_light* L, std::vector<float>& func, std::vector<float>& cdf,
                                 std::vector<float>& fint, std::vector<float>& mfunc,
                                 std::vector<float>& mcdf) {
  int nu, nv;
  if (L->env_kind == BLING_ENV_CONSTANT) { nu = 1; nv = 1; }
  else if (L->env_kind == BLING_ENV_IMAGE) { nu = L->env_w; nv = L->env_h; }      // texSize of the image
  else { nu = 640; nv = 480; }
  float sx = (float)nu, sy = (float)nv;
  func.assign((size_t)nu * nv, 0.f);
  cdf.clear(); fint.clear(); mfunc.clear(); mcdf.clear();
  for (int v = 0; v < nv; ++v) {
    std::vector<float> row(nu);
    for (int u = 0; u < nu; ++u) {
      float s[16];
      if (L->env_kind == BLING_ENV_CONSTANT) {
        for (int i = 0; i < 16; ++i) s[i] = L->env_const[i];
      } else if (L->env_kind == BLING_ENV_IMAGE) {
        // rgbfToTexMap at Cartesian (u / sx, v / sy) (IO/Bitmap.hs:22-29)
        const float* t = L->env_texels + 16 * bimgtex::env_texel(L->env_w, L->env_h, (float)u / sx, (float)v / sy);
        for (int i = 0; i < 16; ++i) s[i] = t[i];
      } else {
        // cartToSph (Types.hs:31-33) then sphToDir (Math.hs:146-148)
        float cu = (float)u / sx, cv = (float)v / sy;
        float phi = cu * 2.f * 3.14159265358979323846f, th = cv * 3.14159265358979323846f;
        float st = sinf(th), ct = cosf(th);
        bsky::sky_eval(L, st * cosf(phi), st * sinf(phi), ct, s);
      }
      row[u] = bsky::spectrum_y(s);
      func[(size_t)v * nu + u] = row[u];
    }
    fint.push_back(bling_dist1d(row, cdf));
  }
  mfunc = fint;
  L->marg_func_int = bling_dist1d(mfunc, mcdf);
  L->dist_nu = nu; L->dist_nv = nv;
  L->dist_func = func.data(); L->dist_cdf = cdf.data(); L->dist_func_int = fint.data();
  L->marg_func = mfunc.data(); L->marg_cdf = mcdf.data();
}
#endif
