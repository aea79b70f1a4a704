// fast_cr.h -- correctly rounded binary32 reciprocal and square root in fewer instructions than
// the compiler's general IEEE sequences, for the Mandelbulb march's bulbPower (one sqrt and one
// reciprocal per iteration, Fractal.hs:97-111 via dev_trace.h).
//
// Both return exactly what `1.f / x` and `sqrtf(x)` return (binary32, round to nearest even) for
// every input: a fast path covers the operand range where no scaling is needed and everything else
// falls back to the general expression.  The claim is checked exhaustively on gfx950 over all 2^32
// bit patterns by bling_mathcheck (csrc/check/mathcheck.hip, tests/test_gpu_parity.py).
//
//   rcp:  y = v_rcp_f32(x) is faithful (< 1 ulp); one fused Newton correction
//         y + y * (1 - x * y) with the residual exact by fma rounds to RN(1/x).
//   sqrt: s = v_sqrt_f32(x) is faithful; the two neighbours s -/+ 1 ulp are tested with exact
//         fma residuals x - s' * s (the compiler's own correction, without its 2^32 input
//         scaling, which only inputs below 2^-96 need).
#pragma once
#include <hip/hip_runtime.h>

namespace bfast {

// BLING_CR_WAVE: the fast sequences run on every lane and the out-of-range inputs take the IEEE
// operation behind a wave-uniform test (a ballot), instead of an if / else whose two sides the
// compiler either both executes (if-conversion: the whole IEEE division on every call) or wraps in
// exec-mask branches.  Same values either way.
#ifndef BLING_CR_WAVE
#define BLING_CR_WAVE 1
#endif
__device__ __forceinline__ float rcp_cr(float x) {
  const float a = __builtin_fabsf(x);
#if BLING_CR_WAVE
  {
    const float y = __builtin_amdgcn_rcpf(x);
    float r = __builtin_fmaf(__builtin_fmaf(-x, y, 1.f), y, y);
    const bool slow = !(a >= 0x1p-125f && a <= 0x1p125f);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(slow) != 0ull, 0)) { if (slow) r = 1.f / x; }
    return r;
  }
#endif
  if (a >= 0x1p-125f && a <= 0x1p125f) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.f);
    return __builtin_fmaf(e, y, y);
  }
  return 1.f / x;
}

__device__ __forceinline__ float sqrt_cr(float x) {
#if BLING_CR_WAVE
  {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1);
    const float sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    const float t = rm <= 0.f ? sm : s;
    float r = rp > 0.f ? sp : t;
    const bool slow = !(x >= 0x1p-96f && x <= 0x1p126f);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(slow) != 0ull, 0)) { if (slow) r = sqrtf(x); }
    return r;
  }
#endif
  if (x >= 0x1p-96f && x <= 0x1p126f) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1);
    const float sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    const float t = rm <= 0.f ? sm : s;
    return rp > 0.f ? sp : t;
  }
  return sqrtf(x);
}

}  // namespace bfast
