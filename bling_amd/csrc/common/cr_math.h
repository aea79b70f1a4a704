// cr_math.h -- binary32 log / exp / sinh / cos evaluated in binary64 and rounded once, shared by
// the device core (ocml binary64) and the CPU oracle (libm binary64), used by the distance-estimator
// fractal marches (Primitive/Fractal.hs:90-98, 130-137, 180-195) and the quasiCrystal texture's
// waves (Texture.hs:335-338), where a last-ulp difference would move a `wrap` boundary.
//
// The march sums ~100 DE steps whose lengths come from `log`, `exp` and `sinh` of Floats; the
// reference's libm logf / expf / sinhf (GHC's Float primops) are pinned to no version (SURVEY.md
// 8c) and the binary32 ocml and glibc versions differ in the last ulp for a share of inputs,
// which the march amplifies into different hit points for about a third of the camera samples.
// Evaluated in binary64 and rounded to binary32 once, both sides return the correctly rounded
// value (the two binary64 results differ by at most an ulp of binary64, which changes the binary32
// rounding only for inputs within 2^-29 ulp of a rounding boundary), so device and oracle march
// identically.  Against a correctly rounded logf the result is the same; glibc's binary32 logf is
// within 1 ulp of it.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BCR_FN __host__ __device__ inline
#else
#include <cmath>
#define BCR_FN static inline
#endif

namespace bcr {

BCR_FN float logf(float x) { return (float)::log((double)x); }
BCR_FN float expf(float x) { return (float)::exp((double)x); }
BCR_FN float sinhf(float x) { return (float)::sinh((double)x); }
BCR_FN float cosf(float x) { return (float)::cos((double)x); }

}  // namespace bcr
