// Test utilities: a bounded "CU hog" that keeps workgroups resident for a fixed wall time,
// to rehearse the cooperative kernels (one-XCD eigensolver, 16-CU SMO) under CU contention
// on one GPU, as RCCL kernels would cause at P > 1 (tests/test_coop_contention_gpu.py).
#include "common.h"

namespace {

// every workgroup holds `lds` bytes of LDS (dynamic) and spins until `ticks` of the 100 MHz
// realtime counter have passed since it started (bounded: the grid always drains)
__global__ __launch_bounds__(256) void spin_kernel(long long ticks, int* __restrict__ done) {
  extern __shared__ int hog_lds[];
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) hog_lds[0] = 1;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(done, hog_lds[0]);
}

}  // namespace

// blocks workgroups of 256 threads, each holding lds bytes of LDS for us microseconds;
// done (one int, zeroed) counts the workgroups that finished
HARP_EXPORT int harp_test_spin(int blocks, int lds, long long us, int* done, hipStream_t s) {
  if (blocks < 1 || lds < 4 || lds > 160 * 1024 || us < 0 || us > 10000000 || !done) return HARP_EBADARG;
  if (lds > 65536 &&
      hipFuncSetAttribute((const void*)spin_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return HARP_ELAUNCH;
  spin_kernel<<<dim3((unsigned)blocks), dim3(256), (size_t)lds, s>>>(us * 100, done);
  return harp_launch_status();
}
