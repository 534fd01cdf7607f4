// Brute-force k-nearest-neighbour selection for gfx950 (MI355X / CDNA4).
//
// Replaces the hot loop of the reference's batch kNN classifier
// (ml/daal/.../daal_knn/ KnnDaalCollectiveMapper -> DAAL kdtree_knn_classification, SURVEY
// §2.9 "kNN distance GEMM + top-k"). A kd-tree is the wrong structure for a GPU: at the
// dimensions the DAAL examples use, exact search is a GEMM plus a selection.
//
//   S = Q . T^T                      hipBLASLt fp32 GEMM (library GEMM, the right tool)
//   d[q, j] = |q|^2 + |t_j|^2 - 2 S  fused into the selection pass below
//   top-k smallest d per query       knn_select_kernel
//
// The selection reads S exactly once (one HBM pass) and never materialises d. It replaces
// torch's distance expression (three elementwise passes over an M x N tile) and its
// radix-select topk (several more passes). Train tiles are merged into a running [M, k]
// state, so N can be any size: each call seeds the lane lists from the previous state.
//
// One wave per query row. Lane l scans columns l, l + 64, ... with coalesced 256-B loads
// (four loads in flight) and keeps a sorted register list of its KK best (distance,
// index) pairs. A candidate that does not beat min(lane's current worst, wave threshold)
// is rejected with one compare; the wave threshold (an upper bound on the k-th best so
// far, carried across train tiles) makes almost every candidate a reject after the first
// tile. An accepted candidate
// is inserted by a branchless compare-exchange sweep over the unrolled list. The 64 lane
// lists are then merged in k rounds: a wave minimum over 64-bit keys (distance bits, then
// column index, so ties resolve to the lower index like a stable sort) names the winning
// lane, which writes the pair out and shifts its list by one.
#include "common.h"

namespace {

template <int KK>
__device__ __forceinline__ void list_insert(float (&dl)[KK], int (&il)[KK], float d, int j) {
  float cd = d;
  int cj = j;
#pragma unroll
  for (int i = 0; i < KK; ++i) {
    const bool s = cd < dl[i] || (cd == dl[i] && cj < il[i]);
    const float td = s ? dl[i] : cd;
    const int tj = s ? il[i] : cj;
    dl[i] = s ? cd : dl[i];
    il[i] = s ? cj : il[i];
    cd = td;
    cj = tj;
  }
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

__device__ __forceinline__ float wave_min_f32(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int KK>
__global__ __launch_bounds__(256) void knn_select_kernel(const float* __restrict__ S, long lds, int M, int N,
                                                         const float* __restrict__ qn, const float* __restrict__ tn,
                                                         int k, int col0, int merge, float* __restrict__ outD,
                                                         int* __restrict__ outI) {
  const int lane = threadIdx.x & 63;
  const long q = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (q >= M) return;  // whole waves exit together (q is wave-uniform)
  float dl[KK];
  int il[KK];
#pragma unroll
  for (int i = 0; i < KK; ++i) {
    dl[i] = __builtin_inff();
    il[i] = 0x7fffffff;
  }
  // thr: an upper bound on the k-th best distance seen so far (strict rejects beyond it).
  // Seeded from the previous tiles' k-th entry, then tightened to the wave minimum of the
  // lane lists' last entries: a lane whose list is full holds KK >= k candidates no worse
  // than its last one. Later columns have higher indices, so dropping ties at thr keeps the
  // lower-index tie order.
  float thr = __builtin_inff();
  if (merge) {
    if (lane < k) {
      const float pd = outD[q * k + lane];
      const int pi = outI[q * k + lane];
      if (pi >= 0) list_insert<KK>(dl, il, pd, pi);
    }
    if (outI[q * k + k - 1] >= 0) thr = outD[q * k + k - 1];
  }
  const float qq = qn[q];
  const float* row = S + q * lds;
  int j = lane;
  for (int it = 0; j + 192 < N; j += 256, ++it) {
    if ((it & 3) == 3) thr = fminf(thr, wave_min_f32(dl[KK - 1]));
    const float s0 = row[j], s1 = row[j + 64], s2 = row[j + 128], s3 = row[j + 192];
    const float t0 = tn[j], t1 = tn[j + 64], t2 = tn[j + 128], t3 = tn[j + 192];
    const float d0 = fmaxf(fmaf(-2.f, s0, qq + t0), 0.f), d1 = fmaxf(fmaf(-2.f, s1, qq + t1), 0.f);
    const float d2 = fmaxf(fmaf(-2.f, s2, qq + t2), 0.f), d3 = fmaxf(fmaf(-2.f, s3, qq + t3), 0.f);
    if (d0 < fminf(dl[KK - 1], thr)) list_insert<KK>(dl, il, d0, col0 + j);
    if (d1 < fminf(dl[KK - 1], thr)) list_insert<KK>(dl, il, d1, col0 + j + 64);
    if (d2 < fminf(dl[KK - 1], thr)) list_insert<KK>(dl, il, d2, col0 + j + 128);
    if (d3 < fminf(dl[KK - 1], thr)) list_insert<KK>(dl, il, d3, col0 + j + 192);
  }
  for (; j < N; j += 64) {
    const float d = fmaxf(fmaf(-2.f, row[j], qq + tn[j]), 0.f);
    if (d < fminf(dl[KK - 1], thr)) list_insert<KK>(dl, il, d, col0 + j);
  }
  // k-round merge of the 64 sorted lane lists
  for (int r = 0; r < k; ++r) {
    const unsigned long long key =
        ((unsigned long long)__float_as_uint(dl[0]) << 32) | (unsigned long long)(unsigned)il[0];
    const unsigned long long m = wave_min_u64(key);
    if (key == m) {
      if (dl[0] == __builtin_inff() && il[0] == 0x7fffffff) {
        outD[q * k + r] = __builtin_inff();
        outI[q * k + r] = -1;
      } else {
        outD[q * k + r] = dl[0];
        outI[q * k + r] = il[0];
      }
#pragma unroll
      for (int i = 0; i + 1 < KK; ++i) {
        dl[i] = dl[i + 1];
        il[i] = il[i + 1];
      }
      dl[KK - 1] = __builtin_inff();
      il[KK - 1] = 0x7fffffff;
    }
  }
}

}  // namespace

// S [M, N] row stride lds (fp32, = Q T^T), qn [M], tn [N] squared norms; out [M, k] running
// state (merge != 0: seeded from outD/outI, index -1 = empty slot). Columns are reported as
// col0 + j. k <= 32 (a 64-entry lane list spills: 256 VGPRs).
HARP_EXPORT int harp_knn_select(const float* S, long lds, int M, int N, const float* qn, const float* tn, int k,
                                int col0, int merge, float* outD, int* outI, hipStream_t s) {
  if (M <= 0) return HARP_OK;
  if (k <= 0 || k > 32 || N < 0 || lds < N) return HARP_EBADARG;
  const long blocks = ((long)M + 3) / 4;
  if (blocks > 0x7fffffffL) return HARP_EBADARG;
  const dim3 g((unsigned)blocks), b(256);
  if (k <= 4) knn_select_kernel<4><<<g, b, 0, s>>>(S, lds, M, N, qn, tn, k, col0, merge, outD, outI);
  else if (k <= 8) knn_select_kernel<8><<<g, b, 0, s>>>(S, lds, M, N, qn, tn, k, col0, merge, outD, outI);
  else if (k <= 16) knn_select_kernel<16><<<g, b, 0, s>>>(S, lds, M, N, qn, tn, k, col0, merge, outD, outI);
  else knn_select_kernel<32><<<g, b, 0, s>>>(S, lds, M, N, qn, tn, k, col0, merge, outD, outI);
  return harp_launch_status();
}
