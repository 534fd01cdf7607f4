// Cycles per back-to-back MFMA on one SIMD (one wave per SIMD, 4 accumulators): the bf16
// 32x32x16 form vs the CDNA3-era 32x32x8 form (would a K = 8 tail step cost half?)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((__vector_size__(8 * sizeof(short)))) short bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(short)))) short bf16x4;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float floatx16;

template <int KIND>
__global__ void mfma_loop(float* out, long long* cyc, int iters) {
  floatx16 acc[4] = {};
  bf16x8 a8, b8;
  bf16x4 a4, b4;
  for (int i = 0; i < 8; ++i) { a8[i] = (short)(threadIdx.x + i); b8[i] = (short)(threadIdx.x * 3 + i); }
  for (int i = 0; i < 4; ++i) { a4[i] = a8[i]; b4[i] = b8[i]; }
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (KIND == 0)
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, acc[q], 0, 0, 0);
      else
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(a4, b4, acc[q], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0;
  for (int q = 0; q < 4; ++q)
    for (int i = 0; i < 16; ++i) s += acc[q][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int iters = 20000, blocks = 256 * 4;
  float* out;
  long long* cyc;
  hipMalloc(&out, sizeof(float) * blocks * 64);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  long long h[1024];
  for (int kind = 0; kind < 2; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (kind == 0) mfma_loop<0><<<blocks, 64>>>(out, cyc, iters);
      else mfma_loop<1><<<blocks, 64>>>(out, cyc, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(h, cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
      double avg = 0;
      for (int b = 0; b < blocks; ++b) avg += h[b];
      avg /= blocks;
      const double flop = (double)blocks * iters * 4 * 32 * 32 * (kind == 0 ? 16 : 8) * 2;
      printf("{\"mfma\": \"%s\", \"cycles_per_mfma\": %.2f, \"ms\": %.3f, \"tflops\": %.1f}\n",
             kind == 0 ? "32x32x16_bf16" : "32x32x8_bf16_1k", avg / (iters * 4.0), ms, flop / ms / 1e9);
    }
  }
  return 0;
}
