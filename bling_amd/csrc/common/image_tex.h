// image_tex.h -- image texture lookups shared by the device core and the oracle (one definition, so
// both pick the same texel): the 2d texture mappings (Texture.hs:164-179) and getPixel /
// getPixelScalar's wrapped pixel (Texture.hs:91-108).  The texels themselves are folded on the host
// (loader.cpp add_image: bling_image).
#pragma once
#include <stdint.h>
#include "../../../include/bling_scene.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BLING_IT __host__ __device__ inline
#else
#include <cmath>
#define BLING_IT inline
#endif

namespace bimgtex {

// mod' a b (Texture.hs:91-94) with `div` rounding to -infinity: the result lies in [0, b)
BLING_IT long long mod_floor(long long a, long long b) {
  long long r = a % b;
  return r < 0 ? r + b : r;
}

// the texture coordinates of a 2d mapping: uvMapping (su, sv) (ou, ov) = (su u + ou, sv v + ov)
// (Texture.hs:166-170); planarMapping (vu, vv) (ou, ov) = (p . vu + ou, p . vv + ov) (:172-179)
BLING_IT void map2d(int kind, const float* m, float px, float py, float pz, float u, float v, float* s, float* t) {
  if (kind == BLING_MAP_PLANAR) {
    *s = (px * m[0] + py * m[1] + pz * m[2]) + m[6];
    *t = (px * m[3] + py * m[4] + pz * m[5]) + m[7];
  } else {
    *s = m[0] * u + m[2];
    *t = m[1] * v + m[3];
  }
}

// floor to a 64-bit Int; a NaN or a value beyond +-2^62 (where GHC's Float -> Int floor is no
// longer meaningful) maps to 0 on both the device and the oracle
BLING_IT long long floor_int(float a) {
  return (a > -4.6e18f && a < 4.6e18f) ? (long long)floorf(a) : 0;
}

// getPixel's pixel (Texture.hs:96-101): px = mod' (floor (u w)) w, py = mod' (floor (-v h)) h;
// returns the texel index py * w + px
BLING_IT long long texel(int w, int h, float s, float t) {
  const long long x = mod_floor(floor_int(s * (float)w), w);
  const long long y = mod_floor(floor_int(-t * (float)h), h);
  return y * w + x;
}

// rgbfToTexMap's pixel of Cartesian (u, v) (IO/Bitmap.hs:22-29), the environment maps: x = max 0
// (min (w - 1) (floor ((1 - u) * w))), y likewise with v and h; returns the texel index y * w + x
BLING_IT long long env_texel(int w, int h, float u, float v) {
  long long x = floor_int((1.f - u) * (float)w), y = floor_int((1.f - v) * (float)h);
  x = x < 0 ? 0 : (x > w - 1 ? w - 1 : x);
  y = y < 0 ? 0 : (y > h - 1 ? h - 1 : y);
  return y * w + x;
}

}  // namespace bimgtex
