#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void k32(const bf16x8* in, float* out, int iters) {
  bf16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
  floatx16 acc = {};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 7; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    a[0] = (__bf16)acc[1];
  }
  float s = 0; for (int q = 0; q < 16; ++q) s += acc[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// same FLOPs: a 32x32 tile over k=112 = four 16x16 tiles x (3 x 16x16x32 + 1 x 16x16x16)
__global__ void k16(const bf16x8* in, float* out, int iters) {
  bf16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
  short4v a4 = {1, 2, 3, 4}, b4 = {5, 6, 7, 8};
  floatx4 acc[4] = {};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int s = 0; s < 3; ++s) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[t], 0, 0, 0);
    }
    a[0] = (__bf16)acc[0][1];
  }
  float s = 0; for (int t = 0; t < 4; ++t) for (int q = 0; q < 4; ++q) s += acc[t][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// 16x16x32 with k padded to 128: four tiles x 4 MFMAs
__global__ void k16p(const bf16x8* in, float* out, int iters) {
  bf16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
  floatx4 acc[4] = {};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[t], 0, 0, 0);
    a[0] = (__bf16)acc[0][1];
  }
  float s = 0; for (int t = 0; t < 4; ++t) for (int q = 0; q < 4; ++q) s += acc[t][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  bf16x8* in; float* out;
  hipMalloc(&in, 128 * sizeof(bf16x8)); hipMalloc(&out, 256 * 2048 * 256 * 4);
  // random-ish operands
  __bf16 h[128 * 8]; for (int i = 0; i < 128 * 8; ++i) h[i] = (__bf16)((float)((i * 2654435761u) % 1000) / 37.f);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000, blocks = 256 * 8;  // 2 waves per SIMD: 8 waves/CU as 2 blocks of 256
  for (int rep = 0; rep < 3; ++rep) {
    for (int v = 0; v < 3; ++v) {
      hipEventRecord(e0);
      if (v == 0) k32<<<blocks, 256>>>(in, out, iters);
      else if (v == 1) k16<<<blocks, 256>>>(in, out, iters);
      else k16p<<<blocks, 256>>>(in, out, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      // useful FLOPs: per wave-iteration a 32x32x112 tile = 2*32*32*112
      double fl = 2.0 * 32 * 32 * 112 * (double)iters * blocks * 4;
      printf("%s %.2f ms  %.0f TFLOP/s (useful k=112)\n", v == 0 ? "32x32x16 x7      " : v == 1 ? "16x16x32x3+16x16x16" : "16x16x32 x4 (k128)", ms, fl / ms / 1e9);
    }
  }
  return 0;
}
