// counter_rng.h -- the sampler RNG of the MI355X core (replaces Graphics.Bling.Random's MWC256
// streams, Random.hs:32-96, seeded per tile per pass from system entropy, Rendering.hs:128).
//
// Every sample value is a pure function of (seed, pass, pixel, sample, dimension), so the device,
// any number of GPUs and the CPU oracle draw identical values regardless of scheduling.
//   hash5     : MurmurHash3-style mixing of the five 32-bit key words + fmix32 finaliser
//   u01       : top 24 bits -> [0, 1 - 2^-24]
//   permute   : Kensler's hashed bijection on [0, l) (Pixar TM 13-01, cycle walking), used where the
//               reference shuffles strata (Sampling.hs:117-120, 134-150)
// Dimension codes partition the key space (see DESIGN.md "Sampler RNG").
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BRNG_HD __host__ __device__ __forceinline__
#else
#define BRNG_HD static inline
#endif

namespace brng {

enum : uint32_t {
  DIM_PIX = 0x1000u, DIM_LENS_PERM = 0x2000u, DIM_LENS_J = 0x2100u,
  DIM_1D_PERM = 0x3000u, DIM_1D_J = 0x4000u, DIM_2D_PERM = 0x5000u, DIM_2D_J = 0x6000u,
  DIM_FRESH1D = 0x7000u, DIM_FRESH2D = 0x8000u, DIM_RAND_CAM = 0x9000u, ALL_SAMPLES = 0xFFFFFFFFu
};

BRNG_HD uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
BRNG_HD uint32_t mix(uint32_t h, uint32_t k) {
  k *= 0xcc9e2d51u; k = rotl(k, 15); k *= 0x1b873593u;
  h ^= k; h = rotl(h, 13); return h * 5u + 0xe6546b64u;
}
BRNG_HD uint32_t fmix(uint32_t h) { h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16; return h; }

// Key prefix shared by every draw of one pixel in one pass.
BRNG_HD uint32_t pixel_key(uint32_t seed, uint32_t pass, uint32_t pixel) { return mix(mix(seed, pass), pixel); }
#if (defined(BLING_RNG_COST_EXPERIMENT) || defined(BLING_RNG_DRAW_EXPERIMENT)) && defined(__HIP_DEVICE_COMPILE__)
// measurement-only experiment builds: what the sampler's hashing costs a kernel (wrong values)
BRNG_HD uint32_t draw(uint32_t pkey, uint32_t sample, uint32_t dim) { return (pkey ^ (sample * 0x9e3779b9u)) + dim * 0x85ebca6bu; }
#else
BRNG_HD uint32_t draw(uint32_t pkey, uint32_t sample, uint32_t dim) { return fmix(mix(mix(pkey, sample), dim) ^ 20u); }
#endif
BRNG_HD uint32_t hash5(uint32_t seed, uint32_t pass, uint32_t pixel, uint32_t sample, uint32_t dim) {
  return draw(pixel_key(seed, pass, pixel), sample, dim);
}
BRNG_HD float u01(uint32_t h) { return (float)(h >> 8) * (1.f / 16777216.f); }

BRNG_HD uint32_t permute(uint32_t i, uint32_t l, uint32_t p) {
  if (l <= 1) return 0;
#if defined(BLING_RNG_COST_EXPERIMENT) && defined(__HIP_DEVICE_COMPILE__)
  return (i + p) % l;
#endif
  uint32_t w = l - 1;
  w |= w >> 1; w |= w >> 2; w |= w >> 4; w |= w >> 8; w |= w >> 16;
  do {
    i ^= p; i *= 0xe170893du; i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8; i *= 0x0929eb3fu; i ^= p >> 23;
    i ^= (i & w) >> 1; i *= 1u | p >> 27; i *= 0x6935fa69u; i ^= (i & w) >> 11; i *= 0x74dcb303u;
    i ^= (i & w) >> 2; i *= 0x9e501cc3u; i ^= (i & w) >> 2; i *= 0xc860a3dfu; i &= w; i ^= i >> 5;
  } while (i >= l);
  return (i + p) % l;
}

}  // namespace brng
