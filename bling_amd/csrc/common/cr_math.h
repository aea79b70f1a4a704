// cr_math.h -- the binary32 transcendentals of the per-sample path (sampling warps, Oren-Nayar,
// Blinn / anisotropic microfacets, Fresnel, the sun-sky model, the thin lens, the fractal marches,
// quasiCrystal), shared by the device core and the CPU oracle so that both return the SAME bits.
//
// The reference's Float transcendentals are GHC primops over libm's binary32 functions, pinned to
// no version; the binary32 ocml and glibc versions differ in the last ulp for a share
// of inputs.  Measured on MI355X with the per-vertex records (tools/vertex_divergence.py,
// profiles/r03_*_divergence.json): with those, 79 % of C2's and 95 % of C5's 8 192 samples had a
// sampled direction a few ulps apart, which the Mandelbulb march and the DE steps' ~100 summed log /
// exp / sinh turn into different paths (C5: 234 samples off).  Every function here is instead one
// written-out algorithm -- since round 5, exp, log, sinh, sin and cos in binary32 arithmetic with
// fused multiply-adds and within one ulp (see exp_f below), the others as follows -- in binary64
// arithmetic -- range reduction, a truncated Taylor series with
// exactly rounded 1/n! or 1/(2k+1) coefficients, reconstruction -- rounded to binary32 once.  The
// operations are plain IEEE binary64 +, -, *, /, sqrt and floor (no fused multiply-add: both sides
// build with -ffp-contract=off), so the host and the device compute them identically.  The series
// are cut where the binary64 result is within ~1e-13 relative of the exact value: the binary32
// result is then the correctly rounded one except for arguments within ~1e-13 of a rounding
// boundary (about 1 in 10^5; tests/test_cr_math.py measures it), and the device still equals the
// host bit for bit, which is what parity needs.  Unlike the ocml / glibc binary64
// functions, these need no large-argument reduction tables or double-double steps, so they stay
// small enough for the shading kernels' register budgets.  tests/test_cr_math.py measures the
// departure from libm binary32 (GHC) and checks the accuracy against binary64 libm; the GPU test
// checks device == host bit for bit.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#include "fast_cr.h"
#define BCR_FN __host__ __device__ inline
#define BCR_OUTLINE static __host__ __device__ __attribute__((noinline))
#if defined(BLING_CR_OUTLINE)
#define BCR_API static __host__ __device__ __attribute__((noinline))
#else
#define BCR_API BCR_FN
#endif
#else
#define BCR_API static inline
#include <cmath>
#define BCR_FN static inline
#define BCR_OUTLINE static __attribute__((noinline))
#endif

namespace bcr {

#if !defined(__HIPCC__)
// CPU oracle only: the libm binary32 functions GHC calls, switched on by oracle_set_libm32 for the
// measurement of how far the shared functions depart from them (tests/test_cr_math.py)
inline bool& libm32_mode() { static bool on = false; return on; }
#define BCR_LIBM32(call) if (::bcr::libm32_mode()) return (call)
#else
#define BCR_LIBM32(call)
#endif
// Measurement-only experiment builds (BCR_FAST_EXPERIMENT): the device calls ocml's binary32
// functions instead, to measure what the shared binary64 algorithms cost a kernel.  Parity with the
// oracle does not hold in such a build; the product build never defines it.
#if defined(BCR_FAST_EXPERIMENT) && defined(__HIP_DEVICE_COMPILE__)
#define BCR_FASTX(call) return (call)
#else
#define BCR_FASTX(call)
#endif

namespace d {

constexpr double PI = 3.141592653589793115997963468544185161590576171875;      // binary64 pi
constexpr double PIO2 = 1.5707963267948965579989817342720925807952880859375;
constexpr double PIO6 = 0.52359877559829881565889309058547951281070709228515625;
constexpr double SQRT3 = 1.732050807568877193176604123436845839023590087890625;
constexpr double TAN_PIO12 = 0.267949192431122695;                              // 2 - sqrt 3
constexpr double LN2_HI = 6.93147180369123816490e-01;    // ln 2 split: hi has 32 significant bits
constexpr double LN2_LO = 1.90821492927058770002e-10;
constexpr double INV_LN2 = 1.44269504088896338700e+00;
constexpr double TWO_OVER_PI = 6.36619772367581382433e-01;
constexpr double PIO2_1 = 1.57079632673412561417e+00;    // pi / 2 split: first 33 bits
constexpr double PIO2_1T = 6.07710050650619224932e-11;   //   the rest

BCR_FN double from_bits(uint64_t b) { return __builtin_bit_cast(double, b); }
BCR_FN uint64_t to_bits(double x) { return __builtin_bit_cast(uint64_t, x); }

// 2^k for -1022 <= k <= 1023
BCR_FN double pow2i(int k) { return from_bits((uint64_t)(k + 1023) << 52); }

// e^x for -745 < x < 709: x = k ln2 + r, |r| <= ln2 / 2, e^r by its Taylor series to r^11 / 11!
// (remainder < 7e-15 relative); callers keep x in range so that 2^k stays a normal binary64
BCR_FN double exp_d(double x) {
  const double k = floor(x * INV_LN2 + 0.5);
  const double r = (x - k * LN2_HI) - k * LN2_LO;
  double p = 1.0 / 39916800.0;                                     // 1 / 11!
  p = p * r + 1.0 / 3628800.0;
  p = p * r + 1.0 / 362880.0;
  p = p * r + 1.0 / 40320.0;
  p = p * r + 1.0 / 5040.0;
  p = p * r + 1.0 / 720.0;
  p = p * r + 1.0 / 120.0;
  p = p * r + 1.0 / 24.0;
  p = p * r + 1.0 / 6.0;
  p = p * r + 0.5;
  p = p * r + 1.0;
  p = p * r + 1.0;
  int ki = (int)k;
  if (ki < -1000) { p *= pow2i(-1000); ki += 1000; }               // subnormal-bound results
  return p * pow2i(ki);
}

// ln x for a positive, finite binary64 x: x = m 2^e with sqrt(1/2) <= m < sqrt 2, ln m = 2 atanh s,
// s = (m - 1) / (m + 1), |s| <= 0.1716, by the series of atanh to s^15 (remainder < 2e-14 relative)
BCR_FN double log_d(double x) {
  uint64_t b = to_bits(x);
  int e = (int)((b >> 52) & 0x7FF);
  if (e == 0) {                                                    // subnormal binary64 (never from binary32)
    x *= 18014398509481984.0;                                      // 2^54
    b = to_bits(x);
    e = (int)((b >> 52) & 0x7FF) - 54;
  }
  e -= 1023;
  double m = from_bits((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);    // [1, 2)
  if (m > 1.4142135623730951) { m *= 0.5; e += 1; }
  const double f = m - 1.0;                                        // exact (Sterbenz)
  const double s = f / (2.0 + f);
  const double z = s * s;
  double p = 1.0 / 15.0;
  p = p * z + 1.0 / 13.0;
  p = p * z + 1.0 / 11.0;
  p = p * z + 1.0 / 9.0;
  p = p * z + 1.0 / 7.0;
  p = p * z + 1.0 / 5.0;
  p = p * z + 1.0 / 3.0;
  const double lm = 2.0 * s + 2.0 * s * (z * p);                   // 2 atanh s
  const double de = (double)e;
  return de * LN2_HI + (lm + de * LN2_LO);
}

// sin and cos of |r| <= pi / 4 + 1e-9 by their Taylor series to r^15 / 15! and r^16 / 16!
// (remainders < 1e-15)
BCR_FN double sin_k(double r) {
  if (fabs(r) < 1e-9) return r;                                    // keeps -0 (and r - r^3 / 6 == r)
  const double z = r * r;
  double p = -1.0 / 1307674368000.0;                               // -1 / 15!
  p = p * z + 1.0 / 6227020800.0;                                  //  1 / 13!
  p = p * z - 1.0 / 39916800.0;
  p = p * z + 1.0 / 362880.0;
  p = p * z - 1.0 / 5040.0;
  p = p * z + 1.0 / 120.0;
  p = p * z - 1.0 / 6.0;
  return r + r * (z * p);
}
BCR_FN double cos_k(double r) {
  const double z = r * r;
  double p = 1.0 / 20922789888000.0;                               //  1 / 16!
  p = p * z - 1.0 / 87178291200.0;                                 // -1 / 14!
  p = p * z + 1.0 / 479001600.0;
  p = p * z - 1.0 / 3628800.0;
  p = p * z + 1.0 / 40320.0;
  p = p * z - 1.0 / 720.0;
  p = p * z + 1.0 / 24.0;
  return (1.0 - 0.5 * z) + (z * z) * p;
}

// Cody-Waite reduction for |x| <= 2^19: x = q pi/2 + r with |r| <= pi/4 (+ rounding); the product
// q * PIO2_1 is exact (|q| < 2^20, PIO2_1 has 33 bits)
BCR_FN double reduce_pio2(double x, int* quadrant) {
  const double q = floor(x * TWO_OVER_PI + 0.5);
  *quadrant = (int)((int64_t)q & 3);
  return (x - q * PIO2_1) - q * PIO2_1T;
}

// huge arguments (|x| > 2^19; quasiCrystal's waves at most): the platform's binary64 functions,
// out of line so their large-argument reduction does not weigh on the callers' register budgets.
// A device unit whose kernels never see such arguments (every profile without computed textures:
// their sin / cos arguments are angles within [-2 pi, 2 pi]) defines BCR_HUGE_ARGS 0 before the
// include: no call -- whose ABI costs the caller register saves and a stack frame even when not
// taken -- is compiled, and a huge argument would give NaN, which the parity tests would report.
#ifndef BCR_HUGE_ARGS
#define BCR_HUGE_ARGS 1
#endif
#if BCR_HUGE_ARGS
BCR_OUTLINE double sin_big(double x) { return ::sin(x); }
BCR_OUTLINE double cos_big(double x) { return ::cos(x); }
#else
BCR_FN double sin_big(double x) { (void)x; return __builtin_nan(""); }
BCR_FN double cos_big(double x) { (void)x; return __builtin_nan(""); }
#endif

BCR_FN double sin_d(double x) {
  if (!(fabs(x) <= 524288.0)) return x != x ? x : sin_big(x);
  int q;
  const double r = reduce_pio2(x, &q);
  switch (q) {
    case 0: return sin_k(r);
    case 1: return cos_k(r);
    case 2: return -sin_k(r);
    default: return -cos_k(r);
  }
}
BCR_FN double cos_d(double x) {
  if (!(fabs(x) <= 524288.0)) return x != x ? x : cos_big(x);
  int q;
  const double r = reduce_pio2(x, &q);
  switch (q) {
    case 0: return cos_k(r);
    case 1: return -sin_k(r);
    case 2: return -cos_k(r);
    default: return sin_k(r);
  }
}

// atan of |t| <= 2 - sqrt 3 by its Taylor series to t^19 / 19 (remainder < 5e-14 relative)
BCR_FN double atan_k(double t) {
  if (fabs(t) < 1e-9) return t;                                    // keeps -0 (and t - t^3 / 3 == t)
  const double z = t * t;
  double p = 1.0 / 19.0;
  p = p * z - 1.0 / 17.0;
  p = p * z + 1.0 / 15.0;
  p = p * z - 1.0 / 13.0;
  p = p * z + 1.0 / 11.0;
  p = p * z - 1.0 / 9.0;
  p = p * z + 1.0 / 7.0;
  p = p * z - 1.0 / 5.0;
  p = p * z + 1.0 / 3.0;
  return t - t * (z * p);
}
// atan of 0 <= a <= inf: arguments above 1 through pi/2 - atan (1/a), those above 2 - sqrt 3
// through pi/6 + atan ((sqrt 3 a - 1) / (sqrt 3 + a))
BCR_FN double atan_pos(double a) {
  const bool inv = a > 1.0;
  if (inv) a = 1.0 / a;
  double r;
  if (a > TAN_PIO12) r = PIO6 + atan_k((SQRT3 * a - 1.0) / (SQRT3 + a));
  else r = atan_k(a);
  return inv ? PIO2 - r : r;
}
BCR_FN double atan_d(double x) { return x == 0.0 ? x : (x < 0.0 ? -atan_pos(-x) : atan_pos(x)); }

// atan2 with C99's signed zeros and axes; both arguments finite (callers route infinities out)
BCR_FN double atan2_d(double y, double x) {
  const bool ny = to_bits(y) >> 63, nx = to_bits(x) >> 63;
  double r;
  if (y == 0.0) r = nx ? PI : 0.0;
  else if (x == 0.0) r = PIO2;
  else {
    const double a = atan_pos(fabs(y) / fabs(x));
    r = nx ? PI - a : a;
  }
  return ny ? -r : r;
}

}  // namespace d

// C99 / glibc atan2 and pow at infinite or zero arguments (neither a NaN), rounded to binary32:
// written out so that no out-of-line call (and its ABI cost) sits in the callers
BCR_FN float atan2_special(float y, float x) {                    // x or y infinite
  float r;
  if (fabsf(y) == __builtin_inff()) r = x == __builtin_inff() ? (float)(0.25 * d::PI)
                                      : (x == -__builtin_inff() ? (float)(0.75 * d::PI) : (float)d::PIO2);
  else r = x == __builtin_inff() ? 0.f : (float)d::PI;           // y finite, x infinite
  return __builtin_copysignf(r, y);
}
BCR_FN bool odd_integer(float y) {
  return fabsf(y) < 16777216.f && floorf(y) == y && ((int64_t)y & 1) != 0;
}
BCR_FN float pow_special(float x, float y) {                      // x == +-0, or x or y infinite
  const float inf = __builtin_inff();
  if (x == 0.f) {
    if (y < 0.f) return odd_integer(y) ? __builtin_copysignf(inf, x) : inf;
    return odd_integer(y) ? x : 0.f;
  }
  if (fabsf(y) == inf) {                                           // x finite nonzero, or infinite
    const float ax = fabsf(x);
    if (ax == 1.f) return 1.f;
    return (ax < 1.f) == (y < 0.f) ? inf : 0.f;
  }
  // x = +-inf, y finite nonzero
  if (x > 0.f) return y > 0.f ? inf : 0.f;
  if (odd_integer(y)) return y > 0.f ? -inf : -0.f;
  return y > 0.f ? inf : 0.f;
}

// exp, log and sinh in binary32 arithmetic with fused multiply-adds (round 5): the Mandelbulb DE
// step evaluates four logs, an exp and a sinh per march step and the sky model two exps per
// channel, and their binary64 series were 11 % of C5's pass (profiles/r05_ab_session.txt r05n).
// These are faithful (within one ulp of the exact value; most results are the correctly rounded
// ones, tests/test_cr_math.py measures the share) instead of correctly rounded.  Only IEEE binary32
// +, -, *, fma, floor and the correctly rounded reciprocal are used, so the host and the device
// still return the same bits.
BCR_FN float fma_f(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
BCR_FN float pow2_f(int k) { return __builtin_bit_cast(float, (uint32_t)(k + 127) << 23); }   // -126 <= k <= 127
#if defined(__HIP_DEVICE_COMPILE__)
BCR_FN float rcp_f(float x) { return bfast::rcp_cr(x); }          // = 1.f / x for every input (fast_cr.h)
#else
BCR_FN float rcp_f(float x) { return 1.f / x; }
#endif

// e^x = 2^k e^r, k = round(x / ln2), r = x - k ln2 by a two-part Cody-Waite reduction (k ln2_hi is
// exact: ln2_hi has 16 significant bits, |k| <= 216), e^r by its Taylor series to r^7 / 7!
// (remainder < 2^-27 relative for |r| <= ln2 / 2); 2^k applied in at most two exact-or-once-rounded
// steps (subnormal and near-overflow results)
BCR_FN float exp_f(float x) {
  const float k = floorf(x * 1.44269502f + 0.5f);
  float r = fma_f(-k, 0.693145752f, x);                           // 0x3f317200
  r = fma_f(-k, 1.42860677e-06f, r);                              // 0x35bfbe8e: ln2 - ln2_hi
  float p = (float)(1.0 / 5040.0);
  p = fma_f(p, r, (float)(1.0 / 720.0));
  p = fma_f(p, r, (float)(1.0 / 120.0));
  p = fma_f(p, r, (float)(1.0 / 24.0));
  p = fma_f(p, r, (float)(1.0 / 6.0));
  p = fma_f(p, r, 0.5f);
  p = fma_f(p, r, 1.f);
  p = fma_f(p, r, 1.f);
  const int ki = (int)k;
  if (ki > 127) return (p * pow2_f(ki - 1)) * 2.f;
  if (ki < -126) return (p * pow2_f(ki + 100)) * pow2_f(-100);
  return p * pow2_f(ki);
}

// ln x = e ln2 + ln(1 + f), x = (1 + f) 2^e with sqrt(1/2) <= 1 + f < sqrt 2; ln(1 + f) =
// f - (hfsq - s (hfsq + R)) with s = f / (2 + f), hfsq = f^2 / 2 and R = 2 s^2 / 3 + 2 s^4 / 5 + ...
// to s^14 (remainder < 1e-12 relative); e ln2 in two parts (fdlibm's e_logf reconstruction)
BCR_FN float log_f(float x) {
  uint32_t ix = __builtin_bit_cast(uint32_t, x);
  int e = 0;
  if (ix < 0x00800000u) { x *= 33554432.f; ix = __builtin_bit_cast(uint32_t, x); e = -25; }   // subnormal: x 2^25
  e += (int)(ix >> 23) - 127;
  float m = __builtin_bit_cast(float, (ix & 0x007FFFFFu) | 0x3F800000u);                  // [1, 2)
  if (m > 1.41421354f) { m *= 0.5f; e += 1; }
  const float f = m - 1.f;                                        // exact
  const float s = f * rcp_f(2.f + f);
  const float z = s * s;
  float R = (float)(2.0 / 15.0);
  R = fma_f(R, z, (float)(2.0 / 13.0));
  R = fma_f(R, z, (float)(2.0 / 11.0));
  R = fma_f(R, z, (float)(2.0 / 9.0));
  R = fma_f(R, z, (float)(2.0 / 7.0));
  R = fma_f(R, z, (float)(2.0 / 5.0));
  R = fma_f(R, z, (float)(2.0 / 3.0));
  R = R * z;
  const float hfsq = 0.5f * f * f;
  const float de = (float)e;
  return de * 6.93138123e-01f - ((hfsq - (s * (hfsq + R) + de * 9.05800061e-06f)) - f);   // 0x3f317180, 0x3717f7d1
}

BCR_API float expf(float x) {
  BCR_LIBM32(::expf(x));
  BCR_FASTX(::expf(x));
  if (x != x) return x;
  if (x > 89.f) return __builtin_inff();
  if (x < -150.f) return 0.f;
  return exp_f(x);
}
BCR_API float logf(float x) {
  BCR_LIBM32(::logf(x));
  BCR_FASTX(::logf(x));
  if (x != x || x < 0.f) return __builtin_nanf("");
  if (x == 0.f) return -__builtin_inff();
  if (x == __builtin_inff()) return x;
  return log_f(x);
}
BCR_API float sinhf(float x) {
  BCR_LIBM32(::sinhf(x));
  BCR_FASTX(::sinhf(x));
  if (x != x || x == 0.f) return x;
  const float a = fabsf(x);
  float r;
  if (a < 1.f) {                                                   // Taylor series to x^13 / 13!
    const float z = a * a;
    float p = (float)(1.0 / 6227020800.0);
    p = fma_f(p, z, (float)(1.0 / 39916800.0));
    p = fma_f(p, z, (float)(1.0 / 362880.0));
    p = fma_f(p, z, (float)(1.0 / 5040.0));
    p = fma_f(p, z, (float)(1.0 / 120.0));
    p = fma_f(p, z, (float)(1.0 / 6.0));
    r = fma_f(a * z, p, a);
  } else if (a <= 88.f) {
    const float e = exp_f(a);
    r = 0.5f * (e - rcp_f(e));
  } else {                                                         // near and past overflow: binary64
    r = a > 90.f ? __builtin_inff() : (float)(0.5 * d::exp_d((double)a));
  }
  return x < 0.f ? -r : r;
}
// sin and cos of one binary32 argument (round 5): the binary64 Cody-Waite reduction above (r to
// ~1e-16), r split into binary32 rh + rl, then binary32 series with fused multiply-adds -- sin to
// r^9 / 9! with rl added in, cos to r^10 / 10! with the -rh rl term (remainders below 3e-9
// relative over |r| <= pi / 4).  Faithful (within one ulp) instead of correctly rounded; sinf and
// cosf are the two halves of sincosf bit for bit.  Huge and non-finite arguments keep the binary64
// functions.
struct SinCos { float s, c; };
BCR_FN SinCos sincos_f(double xd) {
  int q;
  const double rd = d::reduce_pio2(xd, &q);
  const float rh = (float)rd, rl = (float)(rd - (double)rh);
  const float z = rh * rh;
  float ps = (float)(1.0 / 362880.0);
  ps = fma_f(ps, z, (float)(-1.0 / 5040.0));
  ps = fma_f(ps, z, (float)(1.0 / 120.0));
  ps = fma_f(ps, z, (float)(-1.0 / 6.0));
  const float sk = fabsf(rh) < 1e-4f ? rh : rh + fma_f(rh * z, ps, rl);     // tiny r: r itself (keeps -0)
  float pc = (float)(-1.0 / 3628800.0);
  pc = fma_f(pc, z, (float)(1.0 / 40320.0));
  pc = fma_f(pc, z, (float)(-1.0 / 720.0));
  pc = fma_f(pc, z, (float)(1.0 / 24.0));
  pc = fma_f(pc, z, -0.5f);
  const float ck = 1.f + fma_f(z, pc, -(rh * rl));
  switch (q) {
    case 0: return SinCos{sk, ck};
    case 1: return SinCos{ck, -sk};
    case 2: return SinCos{-sk, -ck};
    default: return SinCos{-ck, sk};
  }
}
BCR_API SinCos sincosf(float x) {
  BCR_LIBM32((SinCos{::sinf(x), ::cosf(x)}));
  BCR_FASTX((SinCos{::sinf(x), ::cosf(x)}));
  const double xd = (double)x;
  if (!(fabs(xd) <= 524288.0)) return SinCos{(float)d::sin_d(xd), (float)d::cos_d(xd)};
  return sincos_f(xd);
}
BCR_API float sinf(float x) {
  BCR_LIBM32(::sinf(x));
  BCR_FASTX(::sinf(x));
  const double xd = (double)x;
  if (!(fabs(xd) <= 524288.0)) return (float)d::sin_d(xd);
  return sincos_f(xd).s;
}
BCR_API float cosf(float x) {
  BCR_LIBM32(::cosf(x));
  BCR_FASTX(::cosf(x));
  const double xd = (double)x;
  if (!(fabs(xd) <= 524288.0)) return (float)d::cos_d(xd);
  return sincos_f(xd).c;
}
BCR_API float tanf(float x) {
  BCR_LIBM32(::tanf(x));
  BCR_FASTX(::tanf(x));
  const double xd = (double)x;
  if (!(fabs(xd) <= 524288.0)) return (float)(d::sin_d(xd) / d::cos_d(xd));
  int q;
  const double r = d::reduce_pio2(xd, &q);
  const double s = d::sin_k(r), c = d::cos_k(r);
  return (float)((q & 1) ? -c / s : s / c);
}
BCR_API float atanf(float x) {
  BCR_LIBM32(::atanf(x));
  BCR_FASTX(::atanf(x));
  if (x != x) return x;
  if (x == __builtin_inff()) return (float)d::PIO2;
  if (x == -__builtin_inff()) return (float)-d::PIO2;
  return (float)d::atan_d((double)x);
}
BCR_API float atan2f(float y, float x) {
  BCR_LIBM32(::atan2f(y, x));
  BCR_FASTX(::atan2f(y, x));
  if (x != x || y != y) return x + y;
  if (fabsf(x) == __builtin_inff() || fabsf(y) == __builtin_inff()) return atan2_special(y, x);
  return (float)d::atan2_d((double)y, (double)x);
}
// acos (round 5) in binary32 with fused multiply-adds: pi/2 - asin x, asin a = a + a w P(w), w = a^2,
// P the arcsine series' coefficients to w^11 (remainder < 2e-10 relative for |a| <= 1/2); above 1/2
// through acos a = 2 asin sqrt((1 - a) / 2) (pi minus it below -1/2), with the square root's rounding
// error folded back in, and pi / 2, pi in two parts.  Faithful (within one ulp) instead of correctly
// rounded; host = device.  (asin itself keeps the binary64 algorithm: the same decomposition loses
// up to two ulps to the cancellation in pi/2 - 2 asin just above 1/2, and the path never calls it.)
#if defined(__HIP_DEVICE_COMPILE__)
BCR_FN float sqrt_f(float x) { return bfast::sqrt_cr(x); }        // = sqrtf for every input (fast_cr.h)
#else
BCR_FN float sqrt_f(float x) { return sqrtf(x); }
#endif
constexpr float PIO2_HI_F = 1.57079637f, PIO2_LO_F = -4.37113883e-08f;   // 0x3fc90fdb, pi/2 - it
constexpr float PI_HI_F = 3.14159274f, PI_LO_F = -8.74227766e-08f;       // 0x40490fdb, pi - it
BCR_FN float asin_poly(float w) {                                // sum (2n)! / (4^n n!^2 (2n + 1)) w^(n-1)
  float p = (float)(676039.0 / 104857600.0);
  p = fma_f(p, w, (float)(88179.0 / 12058624.0));
  p = fma_f(p, w, (float)(46189.0 / 5505024.0));
  p = fma_f(p, w, (float)(12155.0 / 1245184.0));
  p = fma_f(p, w, (float)(6435.0 / 557056.0));
  p = fma_f(p, w, (float)(143.0 / 10240.0));
  p = fma_f(p, w, (float)(231.0 / 13312.0));
  p = fma_f(p, w, (float)(63.0 / 2816.0));
  p = fma_f(p, w, (float)(35.0 / 1152.0));
  p = fma_f(p, w, (float)(5.0 / 112.0));
  p = fma_f(p, w, (float)(3.0 / 40.0));
  p = fma_f(p, w, (float)(1.0 / 6.0));
  return p;
}
// asin sqrt(w) for 0 < w <= 1/4 (w = (1 - a) / 2 exactly): s + (s_lo + s w P(w)), s = sqrt(w) rounded,
// s_lo = (w - s^2) / (2 s) its rounding error
BCR_FN float asin_sqrt(float w) {
  const float s = sqrt_f(w);
  const float sl = fma_f(-s, s, w) * rcp_f(2.f * s);
  return s + fma_f(s * w, asin_poly(w), sl);
}
BCR_API float asinf(float x) {
  BCR_LIBM32(::asinf(x));
  BCR_FASTX(::asinf(x));
  if (!(fabsf(x) <= 1.f)) return __builtin_nanf("");
  const double xd = (double)x;
  return (float)d::atan2_d(xd, sqrt((1.0 - xd) * (1.0 + xd)));
}
BCR_API float acosf(float x) {
  BCR_LIBM32(::acosf(x));
  BCR_FASTX(::acosf(x));
  if (!(fabsf(x) <= 1.f)) return __builtin_nanf("");
  const float a = fabsf(x);
  if (a <= 0.5f) {
    const float z = x * x;
    return PIO2_HI_F - (x + fma_f(x * z, asin_poly(z), -PIO2_LO_F));
  }
  const float w = (1.f - a) * 0.5f;
  if (w == 0.f) return x > 0.f ? 0.f : PI_HI_F;
  const float as = asin_sqrt(w);
  return x > 0.f ? 2.f * as : PI_HI_F - (2.f * as - PI_LO_F);
}
BCR_API float powf(float x, float y) {
  BCR_LIBM32(::powf(x, y));
  BCR_FASTX(::powf(x, y));
  if (y == 0.f || x == 1.f) return 1.f;
  if (x != x || y != y) return x + y;
  if (fabsf(x) == __builtin_inff() || fabsf(y) == __builtin_inff() || x == 0.f) return pow_special(x, y);
  double sign = 1.0;
  if (x < 0.f) {                                                   // integer exponents only
    if (floorf(y) != y) return __builtin_nanf("");
    if (fabsf(y) < 16777216.f && ((int64_t)y & 1)) sign = -1.0;
  }
  const double t = (double)y * d::log_d(fabs((double)x));
  if (t > 89.0) return (float)(sign * 1e300);
  if (t < -150.0) return (float)(sign * 0.0);
  return (float)(sign * d::exp_d(t));
}

#undef BCR_LIBM32
#undef BCR_FASTX
}  // namespace bcr
