// Chip-wide fp64 vector FMA throughput (v_fma_f64, 8 independent chains per lane; 1-4
// waves per SIMD): the ceiling for the EM-GMM E-step / statistics kernels
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void fma_loop(double* out, int iters) {
  double a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3 + i;
  const double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = fma(a[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int iters = 100000;
  double* out;
  if (hipMalloc(&out, sizeof(double) * 256 * 16 * 256) != hipSuccess) return 1;
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int blocks = 256 * wps, threads = 256;  // wps waves per SIMD (4 waves per block, one block per CU per wps)
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      fma_loop<<<blocks, threads>>>(out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flop = (double)blocks * threads * iters * 8 * 2;
      printf("{\"waves_per_simd\": %d, \"ms\": %.3f, \"fp64_tflops\": %.1f}\n", wps, ms, flop / ms / 1e9);
    }
  }
  return 0;
}
