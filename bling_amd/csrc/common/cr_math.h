// cr_math.h -- binary32 transcendentals evaluated in binary64 and rounded once, shared by the device
// core (ocml binary64) and the CPU oracle (glibc binary64): every sin / cos / tan / asin / acos /
// atan / atan2 / pow / exp / log / sinh of a Float that the per-sample path evaluates (sampling
// warps, Oren-Nayar, Blinn / anisotropic microfacets, Fresnel, the sun-sky model, the thin lens,
// the fractal marches, quasiCrystal).
//
// The reference's Float transcendentals are GHC primops over libm's binary32 functions, pinned to
// no version.  The binary32 ocml and glibc versions differ in the last ulp for a
// share of inputs: measured on MI355X with the per-vertex records (tools/vertex_divergence.py,
// profiles/r03_*_divergence.json), 79 % of C2's and 95 % of C5's 8 192 samples had a sampled
// direction a few ulps apart, which the Mandelbulb march (a ray leaving the fractal re-marches from
// its surface) and the DE steps' ~100 summed log / exp / sinh turn into different paths.  Evaluated
// in binary64 and rounded to binary32 once, both sides return the correctly rounded value (the two
// binary64 results differ by at most an ulp of binary64, which changes the binary32 rounding only
// for inputs within 2^-29 ulp of a rounding boundary), so device and oracle agree bit for bit.
// Against GHC's libm binary32 (within 1 ulp of correctly rounded) the departure is measured by
// tests/test_cr_math.py.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BCR_FN __host__ __device__ inline
#else
#include <cmath>
#define BCR_FN static inline
#endif

namespace bcr {

#if defined(__HIPCC__) && defined(BLING_CR32) && BLING_CR32
#define BCR_SEL(f32call, f64call) (f32call)   // measurement build only (make variant DEFS=-DBLING_CR32=1): ocml binary32
#elif defined(__HIPCC__)
#define BCR_SEL(f32call, f64call) (f64call)
#else
// CPU oracle only: the libm binary32 functions GHC calls, switched on by oracle_set_libm32 for the
// measurement of how far the correctly rounded path departs from them (tests/test_cr_math.py)
inline bool& libm32_mode() { static bool on = false; return on; }
#define BCR_SEL(f32call, f64call) (::bcr::libm32_mode() ? (f32call) : (f64call))
#endif

BCR_FN float logf(float x) { return BCR_SEL(::logf(x), (float)::log((double)x)); }
BCR_FN float expf(float x) { return BCR_SEL(::expf(x), (float)::exp((double)x)); }
BCR_FN float sinhf(float x) { return BCR_SEL(::sinhf(x), (float)::sinh((double)x)); }
BCR_FN float cosf(float x) { return BCR_SEL(::cosf(x), (float)::cos((double)x)); }
BCR_FN float sinf(float x) { return BCR_SEL(::sinf(x), (float)::sin((double)x)); }
BCR_FN float tanf(float x) { return BCR_SEL(::tanf(x), (float)::tan((double)x)); }
BCR_FN float asinf(float x) { return BCR_SEL(::asinf(x), (float)::asin((double)x)); }
BCR_FN float acosf(float x) { return BCR_SEL(::acosf(x), (float)::acos((double)x)); }
BCR_FN float atanf(float x) { return BCR_SEL(::atanf(x), (float)::atan((double)x)); }
BCR_FN float atan2f(float y, float x) { return BCR_SEL(::atan2f(y, x), (float)::atan2((double)y, (double)x)); }
BCR_FN float powf(float x, float y) { return BCR_SEL(::powf(x, y), (float)::pow((double)x, (double)y)); }

#undef BCR_SEL
}  // namespace bcr
