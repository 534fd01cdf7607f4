// Sparse codec for rotating count slabs (gfx950).
//
// Model rotation moves each worker's word-topic block to its ring neighbour once per
// rotation step (reference: ml/java/.../lda/LDAMPCollectiveMapper.java rotates dense
// TopicCountList rows through dymoro/Rotator.java). The blocks are count matrices whose
// rows are mostly zero: a word with t tokens has at most min(K, t) nonzero topics, so a
// 1M-word x 1024-topic int32 model (4 GB) holds at most 1e8 nonzeros at 1e8 tokens. Over
// point-to-point xGMI the dense block is link-bound; this codec sends
//   [row offsets (rows+1) int32][counts cap int32][topics cap uint16]
// with cap = sum over rows of min(cols, tokens of the row), a bound every worker computes
// from the (invariant) per-word token totals, so send and receive sizes agree without a
// size exchange and the encode/decode stay on the device stream (no host sync).
//
// encode: nnz per row (wave per row) -> exclusive scan (torch) -> ballot compaction (wave
// per row, entries in column order). decode: memset the slab, then scatter (wave per row).
#include "common.h"

namespace {

constexpr int kWaves = 4;  // waves (rows) per 256-thread workgroup

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kWaves * 64) void slab_nnz_kernel(const int* __restrict__ slab, int rows, int cols,
                                                              long ld, int* __restrict__ nnz) {
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int* r = slab + (long)row * ld;
  int c = 0;
  for (int j = lane; j < cols; j += 64) c += r[j] != 0;
  c = wave_sum_i(c);
  if (lane == 0) nnz[row] = c;
}

// off[rows + 1] exclusive offsets; entries past cap are dropped and flagged in *overflow
__global__ __launch_bounds__(kWaves * 64) void slab_pack_kernel(const int* __restrict__ slab, int rows, int cols,
                                                               long ld, const int* __restrict__ off, long cap,
                                                               int* __restrict__ counts,
                                                               unsigned short* __restrict__ topics,
                                                               int* __restrict__ overflow) {
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int* r = slab + (long)row * ld;
  long base = off[row];
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int j0 = 0; j0 < cols; j0 += 64) {
    const int j = j0 + lane;
    const int v = j < cols ? r[j] : 0;
    const unsigned long long m = __ballot(v != 0);
    if (v != 0) {
      const long pos = base + __popcll(m & below);
      if (pos < cap) {
        counts[pos] = v;
        topics[pos] = (unsigned short)j;
      } else {
        overflow[0] = 1;
      }
    }
    base += __popcll(m);
  }
}

__global__ __launch_bounds__(kWaves * 64) void slab_unpack_kernel(int* __restrict__ slab, int rows, int cols, long ld,
                                                                 const int* __restrict__ off, long cap,
                                                                 const int* __restrict__ counts,
                                                                 const unsigned short* __restrict__ topics) {
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  int* r = slab + (long)row * ld;
  // a received payload is bounds-checked: offsets clamp to [0, cap], topics to the row
  const long e0 = off[row] > 0 ? off[row] : 0;
  const long e1 = off[row + 1] < cap ? off[row + 1] : cap;
  for (long e = e0 + lane; e < e1; e += 64) {
    const int t = topics[e];
    if (t < cols) r[t] = counts[e];
  }
}

}  // namespace

HARP_EXPORT int harp_slab_nnz(const int* slab, int rows, int cols, long ld, int* nnz, hipStream_t s) {
  if (rows < 0 || cols < 0 || cols > 65536 || ld < cols) return HARP_EBADARG;
  if (rows == 0) return HARP_OK;
  slab_nnz_kernel<<<dim3((rows + kWaves - 1) / kWaves), dim3(kWaves * 64), 0, s>>>(slab, rows, cols, ld, nnz);
  return harp_launch_status();
}

HARP_EXPORT int harp_slab_pack(const int* slab, int rows, int cols, long ld, const int* off, long cap, int* counts,
                               void* topics, int* overflow, hipStream_t s) {
  if (rows < 0 || cols < 0 || cols > 65536 || ld < cols || cap < 0) return HARP_EBADARG;
  if (rows == 0) return HARP_OK;
  slab_pack_kernel<<<dim3((rows + kWaves - 1) / kWaves), dim3(kWaves * 64), 0, s>>>(
      slab, rows, cols, ld, off, cap, counts, (unsigned short*)topics, overflow);
  return harp_launch_status();
}

// slab (rows x cols at stride ld) := decoded payload; zeroes the slab first
HARP_EXPORT int harp_slab_unpack(int* slab, int rows, int cols, long ld, const int* off, long cap,
                                 const int* counts, const void* topics, hipStream_t s) {
  if (rows < 0 || cols < 0 || cols > 65536 || ld < cols || cap < 0) return HARP_EBADARG;
  if (rows == 0) return HARP_OK;
  const size_t n = (size_t)(rows - 1) * (size_t)ld + (size_t)cols;  // a strided view ends at its last row
  if (ld == cols) {
    if (hipMemsetAsync(slab, 0, sizeof(int) * n, s) != hipSuccess) return HARP_ELAUNCH;
  } else if (hipMemset2DAsync(slab, sizeof(int) * ld, 0, sizeof(int) * cols, rows, s) != hipSuccess) {
    return HARP_ELAUNCH;
  }
  slab_unpack_kernel<<<dim3((rows + kWaves - 1) / kWaves), dim3(kWaves * 64), 0, s>>>(
      slab, rows, cols, ld, off, cap, counts, (const unsigned short*)topics);
  return harp_launch_status();
}
