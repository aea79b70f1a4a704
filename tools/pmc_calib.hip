// pmc_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns of the traversal kernels (MI355X_MICROARCH.md: only wide coalesced streaming reads are
// calibrated, as a factor 2 on FETCH_SIZE).  Each kernel moves a known number of DRAM bytes over a
// 1 GiB array (4x the 256 MiB MALL, so nothing is served on-die):
//   k_stream_read    float4 per lane, consecutive                       -> 1 GiB read
//   k_gather_read    float4 per lane at a random permutation of records -> 1 GiB read
//   k_gather_read_h  the same, half of the 16-B records of each 64-B line (like sparse path ids) ->
//                    0.5 GiB of records, 1 GiB of lines
//   k_gather_read on mostly-dense slot lists (increasing slots, 85 % / 50 % kept): the path-state
//                    reads of the shading kernel through its resolve queue
//   k_gather_read64  64-B records at an 85 %-dense slot list, AoS (four 16-B pieces per lane, one
//                    instruction each) and plane-major (wavefront.h load_ps)
//   k_stream_write / k_scatter_write: the same for stores
// Build:  hipcc -O3 --offload-arch=gfx950 -o tools/pmc_calib tools/pmc_calib.hip
// Run:    rocprofv3 --pmc FETCH_SIZE -- tools/pmc_calib   (and WRITE_SIZE in a separate run)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CHK(x)                                                                       \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } \
  } while (0)

__global__ void k_stream_read(const float4* __restrict__ a, size_t n, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 123.f) out[0] = s;
}
__global__ void k_gather_read(const float4* __restrict__ a, const uint32_t* __restrict__ idx, size_t n,
                              float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[idx[i]];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 123.f) out[0] = s;
}
// 64-B records (four float4) per lane at listed slots: AoS (record i at 4 i .. 4 i + 3, one
// instruction per float4 covering a 16-B piece of each lane's record) or plane-major (plane q at
// q n + i), as k_shade reads its spectrum streams
__global__ void k_gather_read64(const float4* __restrict__ a, const uint32_t* __restrict__ idx, size_t n, size_t cap,
                                bool planes, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = idx[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = planes ? a[q * cap + r] : a[4 * r + q];
      s += v.x + v.y + v.z + v.w;
    }
  }
  if (s == 123.f) out[0] = s;
}
__global__ void k_stream_write(float4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
__global__ void k_scatter_write(float4* __restrict__ a, const uint32_t* __restrict__ idx, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[idx[i]] = make_float4(1.f, 2.f, 3.f, (float)i);
}

int main() {
  const size_t n = (size_t)1 << 26;                 // 64 Mi float4 = 1 GiB
  float4* a;
  uint32_t *perm, *half;
  float* out;
  CHK(hipMalloc(&a, n * sizeof(float4)));
  CHK(hipMalloc(&perm, n * sizeof(uint32_t)));
  CHK(hipMalloc(&half, n / 2 * sizeof(uint32_t)));
  CHK(hipMalloc(&out, sizeof(float)));
  CHK(hipMemset(a, 0, n * sizeof(float4)));
  std::vector<uint32_t> p(n);
  std::iota(p.begin(), p.end(), 0u);
  std::mt19937_64 rng(7);
  std::shuffle(p.begin(), p.end(), rng);
  CHK(hipMemcpy(perm, p.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
  // half: records 4k and 4k + 1 of every 64-B line (k = line), in random line order
  std::vector<uint32_t> lines(n / 4);
  std::iota(lines.begin(), lines.end(), 0u);
  std::shuffle(lines.begin(), lines.end(), rng);
  std::vector<uint32_t> h(n / 2);
  for (size_t k = 0; k < n / 4; ++k) { h[2 * k] = 4 * lines[k]; h[2 * k + 1] = 4 * lines[k] + 1; }
  CHK(hipMemcpy(half, h.data(), n / 2 * sizeof(uint32_t), hipMemcpyHostToDevice));
  // mostly-dense slot lists, like a resolve queue over the previous launch's entries: slots in
  // increasing order with a fraction dropped at random (kept 85 % / 50 %)
  auto dense_list = [&](double keep, size_t cap) {
    std::vector<uint32_t> v;
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (size_t i = 0; i < cap; ++i)
      if (U(rng) < keep) v.push_back((uint32_t)i);
    return v;
  };
  const std::vector<uint32_t> d85 = dense_list(0.85, n), d50 = dense_list(0.50, n);
  const size_t cap64 = n / 4;                                 // 64-B records in the 1 GiB array
  const std::vector<uint32_t> r85 = dense_list(0.85, cap64);
  uint32_t *dl85, *dl50, *rl85;
  CHK(hipMalloc(&dl85, d85.size() * 4)); CHK(hipMalloc(&dl50, d50.size() * 4)); CHK(hipMalloc(&rl85, r85.size() * 4));
  CHK(hipMemcpy(dl85, d85.data(), d85.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dl50, d50.data(), d50.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(rl85, r85.data(), r85.size() * 4, hipMemcpyHostToDevice));
  const int grid = 256 * 16;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  auto run = [&](const char* name, double bytes, auto&& launch) {
    launch();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%-16s %8.3f ms  %7.1f GB/s  (%.0f MiB of records)\n", name, ms, bytes / ms / 1e6, bytes / 1048576.0);
  };
  run("stream_read", n * 16.0, [&] { k_stream_read<<<grid, 256>>>(a, n, out); });
  run("gather_read", n * 16.0, [&] { k_gather_read<<<grid, 256>>>(a, perm, n, out); });
  run("gather_read_h", n * 8.0, [&] { k_gather_read<<<grid, 256>>>(a, half, n / 2, out); });
  run("dense85_read", d85.size() * 16.0, [&] { k_gather_read<<<grid, 256>>>(a, dl85, d85.size(), out); });
  run("dense50_read", d50.size() * 16.0, [&] { k_gather_read<<<grid, 256>>>(a, dl50, d50.size(), out); });
  run("rec64_aos_d85", r85.size() * 64.0, [&] { k_gather_read64<<<grid, 256>>>(a, rl85, r85.size(), cap64, false, out); });
  run("rec64_planes_d85", r85.size() * 64.0, [&] { k_gather_read64<<<grid, 256>>>(a, rl85, r85.size(), cap64, true, out); });
  run("stream_write", n * 16.0, [&] { k_stream_write<<<grid, 256>>>(a, n); });
  run("scatter_write", n * 16.0, [&] { k_scatter_write<<<grid, 256>>>(a, perm, n); });
  CHK(hipFree(a)); CHK(hipFree(perm)); CHK(hipFree(half)); CHK(hipFree(out));
  CHK(hipFree(dl85)); CHK(hipFree(dl50)); CHK(hipFree(rl85));
  return 0;
}
