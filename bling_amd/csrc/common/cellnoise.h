// cellnoise.h -- Worley's cell noise of Texture.hs:256-315 (cellNoise, its lcg / hash / prob and the
// four distance functions), shared by the device core (cellNoise scalar textures at a hit) and the CPU
// oracle.  Pinned against an independent pure-Python restatement of the Haskell definitions
// (tests/test_kat_hotpath.py).  Haskell Int is 64-bit with wrap-around; every Float operation keeps
// GHC's order (no FMA).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BCELL_FN __device__ __forceinline__
#else
#include <cmath>
#define BCELL_FN static inline
#endif

namespace bcell {

// lcg x = (1103515245 * x + 12345) `rem` 4294967296 (Int arithmetic wraps; rem truncates)
BCELL_FN int64_t lcg(int64_t x) {
  const int64_t y = (int64_t)((uint64_t)1103515245 * (uint64_t)x + (uint64_t)12345);
  return y % 4294967296LL;
}
// hash (x, y, z) = abs ((x * 73856093) `xor` (y * 19349663) `xor` (z * 83492791)) `rem` 4294967296
BCELL_FN int64_t hash3(int64_t x, int64_t y, int64_t z) {
  const uint64_t h = ((uint64_t)x * 73856093u) ^ ((uint64_t)y * 19349663u) ^ ((uint64_t)z * 83492791u);
  const int64_t s = (int64_t)h;
  const int64_t a = s < 0 ? (int64_t)(0u - h) : s;            // abs (minBound stays minBound)
  return a % 4294967296LL;
}
// prob: the number of feature points of a cell (a Poisson lookup table)
BCELL_FN int prob(int64_t v) {
  return v < 393325350LL ? 1 : v < 1022645910LL ? 2 : v < 1861739990LL ? 3 : v < 2700834071LL ? 4
       : v < 3372109335LL ? 5 : v < 3819626178LL ? 6 : v < 4075350088LL ? 7 : v < 4203212043LL ? 8 : 9;
}

// dist: 0 euclidian (len), 1 euclidian2 (sqLen), 2 manhattan, 3 chebyshev (bling_cell_dist)
BCELL_FN float distance(int dist, float dx, float dy, float dz) {
  if (dist == 2) return fabsf(dx) + fabsf(dy) + fabsf(dz);
  if (dist == 3) {                                   // maximum [|dx|, |dy|, |dz|] = foldl1 max
    float m = fabsf(dx), b = fabsf(dy), c = fabsf(dz);
    m = m <= b ? b : m;
    return m <= c ? c : m;
  }
  const float q = dx * dx + dy * dy + dz * dz;      // sqLen (Math.hs:328-330)
  return dist == 1 ? q : sqrtf(q);
}

// cellNoise dist (identity mapping applied by the caller) at p: minimum over the feature points
// of the 27 cells around floor p of dist p point (minimum = foldl1 min)
BCELL_FN float cell_noise(int dist, float px, float py, float pz) {
  const int64_t ox = (int64_t)floorf(px), oy = (int64_t)floorf(py), oz = (int64_t)floorf(pz);
  float best = 0.f;
  bool first = true;
  for (int i = -1; i <= 1; ++i)
    for (int j = -1; j <= 1; ++j)
      for (int k = -1; k <= 1; ++k) {
        const int64_t x = i + ox, y = j + oy, z = k + oz;
        int64_t u = lcg(hash3(x, y, z));
        const int n = prob(u);
        for (int m = 0; m < n; ++m) {              // take n $ tail $ iterate go (undefined, us)
          const int64_t u1 = lcg(u), u2 = lcg(u1), u3 = lcg(u2);
          const float qx = (float)x + (float)u1 / 4294967296.f;
          const float qy = (float)y + (float)u2 / 4294967296.f;
          const float qz = (float)z + (float)u3 / 4294967296.f;
          const float d = distance(dist, px - qx, py - qy, pz - qz);
          best = (first || !(best <= d)) ? d : best;   // min best d = if best <= d then best else d
          first = false;
          u = u3;
        }
      }
  return best;
}

}  // namespace bcell
