// mathcheck.hip -- exhaustive check of common/fast_cr.h on the device: for all 2^32 binary32 bit
// patterns, bfast::rcp_cr(x) must equal 1.f / x and bfast::sqrt_cr(x) must equal sqrtf(x) bit for
// bit (any NaN equals any NaN).  Test infrastructure (tests/test_gpu_parity.py), not product code.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../common/cr_math.h"
#include "../common/fast_cr.h"

__device__ __forceinline__ bool same(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__global__ __launch_bounds__(256) void k_mathcheck(uint64_t base, unsigned long long* out) {
  unsigned bad_r = 0, bad_s = 0, first_r = 0xFFFFFFFFu, first_s = 0xFFFFFFFFu;
  for (uint64_t i = base + blockIdx.x * 256ull + threadIdx.x; i < base + (1ull << 30); i += gridDim.x * 256ull) {
    const uint32_t u = (uint32_t)i;
    const float x = __uint_as_float(u);
    if (!same(bfast::rcp_cr(x), 1.f / x)) { ++bad_r; first_r = min(first_r, u); }
    if (!same(bfast::sqrt_cr(x), sqrtf(x))) { ++bad_s; first_s = min(first_s, u); }
  }
  if (bad_r) { atomicAdd(&out[0], (unsigned long long)bad_r); atomicMin(&out[2], (unsigned long long)first_r); }
  if (bad_s) { atomicAdd(&out[1], (unsigned long long)bad_s); atomicMin(&out[3], (unsigned long long)first_s); }
}

// result[0..3] = rcp mismatches, sqrt mismatches, first mismatching rcp input, first sqrt input
// (0xFFFFFFFF.. = none); returns 0 or a HIP error code
extern "C" int bling_mathcheck(unsigned long long* result) {
  unsigned long long* d = nullptr;
  const unsigned long long init[4] = {0, 0, ~0ull, ~0ull};
  hipError_t e = hipMalloc(&d, sizeof(init));
  if (e == hipSuccess) e = hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice);
  for (uint64_t b = 0; e == hipSuccess && b < (1ull << 32); b += 1ull << 30) {
    k_mathcheck<<<4096, 256>>>(b, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(result, d, sizeof(init), hipMemcpyDeviceToHost);
  if (d) (void)hipFree(d);
  return (int)e;
}

// The shared transcendentals of common/cr_math.h on the device over an input array (fn as
// oracle_cr_eval: 0 sin, 1 cos, 2 tan, 3 asin, 4 acos, 5 atan, 6 exp, 7 log, 8 sinh, 9 atan2, 10 pow,
// 11 / 12 the sin / cos of sincosf),
// for tests/test_cr_math.py's device == host check.  Host buffers; returns 0 or a HIP error code.
__global__ __launch_bounds__(256) void k_creval(int fn, const float* x, const float* y, float* out, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const float a = x[i], b = y[i];
    float r;
    switch (fn) {
      case 0: r = bcr::sinf(a); break;
      case 1: r = bcr::cosf(a); break;
      case 2: r = bcr::tanf(a); break;
      case 3: r = bcr::asinf(a); break;
      case 4: r = bcr::acosf(a); break;
      case 5: r = bcr::atanf(a); break;
      case 6: r = bcr::expf(a); break;
      case 7: r = bcr::logf(a); break;
      case 8: r = bcr::sinhf(a); break;
      case 9: r = bcr::atan2f(a, b); break;
      case 11: r = bcr::sincosf(a).s; break;
      case 12: r = bcr::sincosf(a).c; break;
      default: r = bcr::powf(a, b); break;
    }
    out[i] = r;
  }
}

extern "C" int bling_cr_eval_device(int fn, const float* x, const float* y, float* out, size_t n) {
  float *dx = nullptr, *dy = nullptr, *dout = nullptr;
  const size_t b = n * sizeof(float);
  hipError_t e = hipMalloc(&dx, b);
  if (e == hipSuccess) e = hipMalloc(&dy, b);
  if (e == hipSuccess) e = hipMalloc(&dout, b);
  if (e == hipSuccess) e = hipMemcpy(dx, x, b, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = y ? hipMemcpy(dy, y, b, hipMemcpyHostToDevice) : hipMemset(dy, 0, b);
  if (e == hipSuccess) {
    k_creval<<<2048, 256>>>(fn, dx, dy, dout, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, dout, b, hipMemcpyDeviceToHost);
  for (float* p : {dx, dy, dout}) if (p) (void)hipFree(p);
  return (int)e;
}
