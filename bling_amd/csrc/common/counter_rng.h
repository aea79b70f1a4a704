// counter_rng.h -- the sampler RNG of the MI355X core (replaces Graphics.Bling.Random's MWC256
// streams, Random.hs:32-96, seeded per tile per pass from system entropy, Rendering.hs:128).
//
// Every sample value is a pure function of (seed, pass, pixel, sample, dimension), so the device,
// any number of GPUs and the CPU oracle draw identical values regardless of scheduling.
//
// Specification, version 2 (round 6).  Three keys, each a bijective MurmurHash3 step of the last:
//   pixel_key(seed, pass, pixel)  = mix(mix(seed, pass), pixel)          once per path vertex
//   sample_key(pkey, s)           = fmix(pkey ^ s * 0x9E3779B9)          once per path vertex
//   draw(skey, dim)               = fmix(skey ^ dim_key(dim))            one per sample value
//   dim_key(dim)                  = fmix(dim ^ 0x2C1B3C6D)               wave-uniform (SALU / folded)
//   u01(h)                        = (h >> 8) * 2^-24, in [0, 1 - 2^-24]
//   permute(i, l, p)              = Kensler's hashed bijection on [0, l) (Pixar TM 13-01, cycle
//                                   walking), used where the reference shuffles strata
//                                   (Sampling.hs:117-120, 134-150)
// A sample value therefore costs one xor with a uniform key and one fmix (two 32-bit multiplies);
// version 1 chained two further Murmur mixes per value (draw = fmix(mix(mix(pkey, s), dim) ^ 20),
// three quarter-rate multiplies more, and the compiler held 21 per-dimension keys in VGPRs).  The
// stratified dimensions draw their jitter from the sample's own key (sample n, not its stratum j):
// the strata's jitters are independent uniforms either way, so the sampler's distribution is the
// reference's (tests/test_rng_quality.py checks uniformity and independence across dimensions,
// samples and pixels; tests/test_mwc_sampler.py the convergence to the reference's MWC sampler).
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
// Key shared by every draw of one sample of that pixel (s = ALL_SAMPLES: the pixel's per-dimension
// stratum permutations).
BRNG_HD uint32_t sample_key(uint32_t pkey, uint32_t s) { return fmix(pkey ^ s * 0x9E3779B9u); }
BRNG_HD uint32_t dim_key(uint32_t dim) { return fmix(dim ^ 0x2C1B3C6Du); }
#if (defined(BLING_RNG_COST_EXPERIMENT) || defined(BLING_RNG_DRAW_EXPERIMENT)) && defined(__HIP_DEVICE_COMPILE__)
// measurement-only experiment builds: what the sampler's hashing costs a kernel (wrong values)
BRNG_HD uint32_t draw(uint32_t skey, uint32_t dim) { return skey + dim * 0x85ebca6bu; }
#else
BRNG_HD uint32_t draw(uint32_t skey, uint32_t dim) { return fmix(skey ^ dim_key(dim)); }
#endif
BRNG_HD uint32_t hash5(uint32_t seed, uint32_t pass, uint32_t pixel, uint32_t sample, uint32_t dim) {
  return draw(sample_key(pixel_key(seed, pass, pixel), sample), dim);
}
BRNG_HD float u01(uint32_t h) { return (float)(h >> 8) * (1.f / 16777216.f); }

// Low 32 bits of (a mod 2^24) * (c mod 2^24): one full-rate v_mul_u32_u24 on gfx950 (v_mul_lo_u32
// issues at quarter rate).  Inside permute every product is masked to the low k <= 24 bits
// (l <= 2^24) before it is used, and the low k bits of a product depend only on the low k bits of
// its factors, so permute's value is the 32-bit-multiply one bit for bit
// (tests/test_rng_loader.py::test_permute_mul24_is_the_32bit_permute).
BRNG_HD uint32_t mul24(uint32_t a, uint32_t c) { return (a & 0xFFFFFFu) * (c & 0xFFFFFFu); }

// Kensler's permutation of i in [0, l), l <= 2^24 (callers: spp and photon counts).  w is the
// all-ones mask of l - 1's bit width.
BRNG_HD uint32_t permute_w(uint32_t i, uint32_t l, uint32_t w, uint32_t p) {
  do {
    i ^= p; i = mul24(i, 0xe170893du); i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8; i = mul24(i, 0x0929eb3fu);
    i ^= p >> 23; i ^= (i & w) >> 1; i = mul24(i, 1u | p >> 27); i = mul24(i, 0x6935fa69u); i ^= (i & w) >> 11;
    i = mul24(i, 0x74dcb303u); i ^= (i & w) >> 2; i = mul24(i, 0x9e501cc3u); i ^= (i & w) >> 2;
    i = mul24(i, 0xc860a3dfu); i &= w; i ^= i >> 5;
  } while (i >= l);
  return i;                                         // the caller adds p and reduces mod l
}
BRNG_HD uint32_t permute(uint32_t i, uint32_t l, uint32_t p) {
  if (l <= 1) return 0;
#if defined(BLING_RNG_COST_EXPERIMENT) && defined(__HIP_DEVICE_COMPILE__)
  return (i + p) % l;
#endif
  uint32_t w = l - 1;
  w |= w >> 1; w |= w >> 2; w |= w >> 4; w |= w >> 8; w |= w >> 16;
  return (permute_w(i, l, w, p) + p) % l;
}

}  // namespace brng
