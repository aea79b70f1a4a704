// Debug probe: ocml transcendental / denormal behaviour at the edges the Mandelbulb DE reaches.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
__global__ void k(const float* in, float* out, int n) {
  int i = threadIdx.x;
  if (i >= n) return;
  float x = in[i];
  out[6 * i + 0] = sinhf(x);
  out[6 * i + 1] = expf(x);
  out[6 * i + 2] = logf(x);
  out[6 * i + 3] = sqrtf(x * 1e-30f);
  out[6 * i + 4] = (0.5f / expf(x)) * sinhf(x);
  out[6 * i + 5] = x * 1e-40f;
}
int main() {
  const int n = 8;
  float h[n] = {1.f, 10.f, 88.0f, 88.7f, 88.8f, 89.0f, 89.4f, 1e-8f};
  float *d, *o, ho[6 * n];
  hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof ho);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o, n);
  hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) {
    float x = h[i];
    printf("x=%g gpu: sinh=%a exp=%a log=%a sqrt=%a prod=%a den=%a | cpu: sinh=%a exp=%a log=%a sqrt=%a prod=%a den=%a\n", x,
           ho[6*i], ho[6*i+1], ho[6*i+2], ho[6*i+3], ho[6*i+4], ho[6*i+5],
           sinhf(x), expf(x), logf(x), sqrtf(x * 1e-30f), (0.5f / expf(x)) * sinhf(x), x * 1e-40f);
  }
  return 0;
}
