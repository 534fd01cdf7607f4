// Shared helpers for the harp_amd HIP kernels (gfx950 / CDNA4 only).
//
// Every kernel family exposes plain `extern "C"` launchers taking raw device
// pointers plus the caller's hipStream_t; the Python side (harp_amd/ops/_lib.py)
// binds them with ctypes after `import torch`, so the launches go through the
// same HIP runtime (libamdhip64.so.7) that torch loaded.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define HARP_OK 0
#define HARP_EBADARG 1
#define HARP_ELAUNCH 2
#define HARP_EUNSUPPORTED 3

#define HARP_EXPORT extern "C" __attribute__((visibility("default")))

static inline int harp_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? HARP_OK : HARP_ELAUNCH;
}

__device__ __forceinline__ float bf16_to_f32(__bf16 v) { return (float)v; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
