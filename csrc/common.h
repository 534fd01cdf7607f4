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
typedef float floatx2 __attribute__((ext_vector_type(2)));

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

// wave64 fp64 sum on the DPP network: quad_perm [1,0,3,2] and [2,3,0,1], row_ror 4 and 8
// leave every lane of a 16-lane row with the row's sum; the four row sums are then read
// from lanes 0 / 16 / 32 / 48 (v_readlane) and added in one fixed order, so every lane gets
// the same bits. Six dependent ds_bpermute round trips become four DPP moves and eight
// readlanes. Needs the whole wave active (as the __shfl_xor form does).
template <int CTRL>
__device__ __forceinline__ double dpp_mov_d(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double wave_sum_d_dpp(double v) {
  v += dpp_mov_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov_d<0x124>(v);  // row_ror:4
  v += dpp_mov_d<0x128>(v);  // row_ror:8
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// wave64 inclusive prefix sum on the DPP network (no LDS round trips): Hillis-Steele within
// each 16-lane row (row_shr 1, 2, 4, 8), then row_bcast:15 into rows 1 and 3 and
// row_bcast:31 into rows 2 and 3; lanes without a source add 0.
__device__ __forceinline__ float dpp_shift_add(float v, int sel) {
  int t;
  switch (sel) {
    case 0: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false); break;
    case 1: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xf, 0xf, false); break;
    case 2: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xf, 0xf, false); break;
    case 3: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xf, 0xf, false); break;
    case 4: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false); break;
    default: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false); break;
  }
  return v + __int_as_float(t);
}

__device__ __forceinline__ float wave_scan_incl(float v) {
  v = dpp_shift_add(v, 0);
  v = dpp_shift_add(v, 1);
  v = dpp_shift_add(v, 2);
  v = dpp_shift_add(v, 3);
  v = dpp_shift_add(v, 4);
  v = dpp_shift_add(v, 5);
  return v;
}

// wave-uniform total (scalar register), no LDS traffic
__device__ __forceinline__ float wave_total(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wave_scan_incl(v)), 63));
}
