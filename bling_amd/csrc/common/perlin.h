// perlin.h -- Perlin noise and fBm of Texture.hs:341-414 (perlin3d, noiseWeight, grad, noisePerms,
// fbm), shared by the host loader (heightMap elevation, Primitive/Heightmap.hs), the device core
// (fbm / perlin scalar textures at a hit) and the CPU oracle.  Pinned against an independent numpy
// binary32 restatement (tests/test_heightmap.py).  Evaluation order is GHC's (no FMA).
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BPERLIN_FN __device__ __forceinline__
#define BPERLIN_TABLE __constant__ const
#else
#include <cmath>
#define BPERLIN_FN static inline
#define BPERLIN_TABLE static const
#endif

namespace bperlin {

// Ken Perlin's reference permutation (noisePerms = l ++ l, Texture.hs:400-414); i & 255 indexes the
// doubled table for every index the lookups form (< 512)
BPERLIN_TABLE int kNoisePerm[256] = {
  151,160,137,91,90,15,131,13,201,95,96,53,194,233,7,225,140,36,103,30,69,142,8,99,37,240,21,10,23,
  190,6,148,247,120,234,75,0,26,197,62,94,252,219,203,117,35,11,32,57,177,33,88,237,149,56,87,174,20,
  125,136,171,168,68,175,74,165,71,134,139,48,27,166,77,146,158,231,83,111,229,122,60,211,133,230,220,
  105,92,41,55,46,245,40,244,102,143,54,65,25,63,161,1,216,80,73,209,76,132,187,208,89,18,169,200,196,
  135,130,116,188,159,86,164,100,109,198,173,186,3,64,52,217,226,250,124,123,5,202,38,147,118,126,255,
  82,85,212,207,206,59,227,47,16,58,17,182,189,28,42,223,183,170,213,119,248,152,2,44,154,163,70,221,
  153,101,155,167,43,172,9,129,22,39,253,19,98,108,110,79,113,224,232,178,185,112,104,218,246,97,228,
  251,34,242,193,238,210,144,12,191,179,162,241,81,51,145,235,249,14,239,107,49,192,214,31,181,199,106,
  157,184,84,204,176,115,121,50,45,127,4,150,254,138,236,205,93,222,114,67,29,24,72,243,141,128,195,78,
  66,215,61,156,180};

BPERLIN_FN int nperm(int i) { return kNoisePerm[i & 255]; }
BPERLIN_FN float lerp(float t, float a, float b) { return (1.f - t) * a + t * b; }      // Math.hs:108-110
BPERLIN_FN float noise_weight(float t) {                                                // noiseWeight
  float t3 = t * t * t, t4 = t3 * t;
  return 6.f * t4 * t - 15.f * t4 + 10.f * t3;
}
BPERLIN_FN float noise_grad(int x, int y, int z, float dx, float dy, float dz) {       // grad
  int h = nperm(nperm(nperm(x) + y) + z) & 15;
  float up = (h < 8 || h == 12 || h == 13) ? dx : dy;
  float vp = (h < 4 || h == 12 || h == 13) ? dy : dz;
  float u = (h & 1) ? -up : up, v = (h & 2) ? -vp : vp;
  return u + v;
}
BPERLIN_FN float perlin3d(float x, float y, float z) {                                  // perlin3d
  int ixp = (int)floorf(x), iyp = (int)floorf(y), izp = (int)floorf(z);
  float dx = x - (float)ixp, dy = y - (float)iyp, dz = z - (float)izp;
  int ix = ixp & 255, iy = iyp & 255, iz = izp & 255;
  float w000 = noise_grad(ix, iy, iz, dx, dy, dz);
  float w100 = noise_grad(ix + 1, iy, iz, dx - 1.f, dy, dz);
  float w010 = noise_grad(ix, iy + 1, iz, dx, dy - 1.f, dz);
  float w110 = noise_grad(ix + 1, iy + 1, iz, dx - 1.f, dy - 1.f, dz);
  float w001 = noise_grad(ix, iy, iz + 1, dx, dy, dz - 1.f);
  float w101 = noise_grad(ix + 1, iy, iz + 1, dx - 1.f, dy, dz - 1.f);
  float w011 = noise_grad(ix, iy + 1, iz + 1, dx, dy - 1.f, dz - 1.f);
  float w111 = noise_grad(ix + 1, iy + 1, iz + 1, dx - 1.f, dy - 1.f, dz - 1.f);
  float wx = noise_weight(dx), wy = noise_weight(dy), wz = noise_weight(dz);
  float x00 = lerp(wx, w000, w100), x10 = lerp(wx, w010, w110);
  float x01 = lerp(wx, w001, w101), x11 = lerp(wx, w011, w111);
  float y0 = lerp(wy, x00, x10), y1 = lerp(wy, x01, x11);
  return lerp(wz, y0, y1);
}
BPERLIN_FN float fbm(int octaves, float omega, float px, float py, float pz) {         // fbm: sum = foldl (+) 0
  float acc = 0.f, l = 1.f, o = 1.f;
  for (int k = 0; k < octaves; ++k) {
    acc = acc + o * perlin3d(px * l, py * l, pz * l);
    l = 1.99f * l; o = omega * o;                                                        // iterate (1.99 *) 1, iterate (omega *) 1
  }
  return acc;
}

}  // namespace bperlin
