// Sparse (CSR) K-means E-step + accumulate for gfx950, fp64 like the reference.
//
// Replaces DAAL kmeans DistributedStep1Local on CSR input (ml/daal/.../daal_kmeans/
// allreducecsr/KMeansDaalCollectiveMapper.java; SURVEY §2.9 "kmeans_assign_csr (SpMM +
// argmin)"): per point the argmin over all centroids of |x - c|^2, then the partial sums
// (sum of x, count) of its cluster. The torch path needs three full [n, K] fp64 tensors
// (sparse-dense product, distance expression, one-hot) and a second SpMM for the sums;
// here one wave per CSR row does everything and only the sums leave the kernel.
//
//   * lanes run over centroids: the transposed centroid matrix CT[d][Kp] makes one
//     nonzero (j, v) of the row a 512-B contiguous read CT[j][c0 .. c0+63] per register
//     slot, accumulated in KPL fp64 registers per lane (64 * KPL centroids per pass; K
//     beyond 1024 loops over centroid chunks and re-reads the row from L1).
//   * the row's (col, val) pairs are wave-uniform: one lane-parallel load of 64 of them,
//     then readlane broadcasts, so the inner loop issues no redundant index loads.
//   * dist = |c|^2 - 2 x.c (|x|^2 is row-constant and only enters the objective); wave
//     argmin on (dist, centroid) pairs, ties to the lower centroid like torch.min.
//   * accumulate: the lanes scatter the row's nonzeros into sums[label] with fp64 global
//     atomics (one per nonzero, the row is sparse), lane 0 adds the count.
#include "common.h"

namespace {

__device__ __forceinline__ void wave_argmin_f64(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double w = __shfl_xor(v, o, 64);
    const int wi = __shfl_xor(i, o, 64);
    if (w < v || (w == v && wi < i)) {
      v = w;
      i = wi;
    }
  }
}

__device__ __forceinline__ double readlane_f64(double x, int t) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, t);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), t);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

template <int KPL>
__global__ __launch_bounds__(256) void kmeans_csr_assign_kernel(const long* __restrict__ rowptr,
                                                                const int* __restrict__ col,
                                                                const double* __restrict__ val, long n, int d,
                                                                const double* __restrict__ CT, int K, int Kp,
                                                                const double* __restrict__ cn,
                                                                const double* __restrict__ xn, int* __restrict__ labels,
                                                                double* __restrict__ mind, double* __restrict__ sums,
                                                                double* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += nw) {
    const long a = rowptr[r], b = rowptr[r + 1];
    double best = __builtin_inf();
    int besti = 0;  // a row whose distances are all NaN still lands in a valid cluster
    for (int c0 = 0; c0 < K; c0 += 64 * KPL) {
      double acc[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) acc[i] = 0.0;
      for (long p0 = a; p0 < b; p0 += 64) {
        const int cnt = (int)((b - p0) < 64 ? (b - p0) : 64);
        const int jl = lane < cnt ? col[p0 + lane] : 0;
        const double vl = lane < cnt ? val[p0 + lane] : 0.0;
        for (int t = 0; t < cnt; ++t) {
          const int j = __builtin_amdgcn_readlane(jl, t);
          const double v = readlane_f64(vl, t);
          const double* ct = CT + (long)j * Kp + c0 + lane;
#pragma unroll
          for (int i = 0; i < KPL; ++i)
            if (c0 + 64 * i < Kp) acc[i] = fma(v, ct[64 * i], acc[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const int c = c0 + 64 * i + lane;
        if (c < K) {
          const double dist = fma(-2.0, acc[i], cn[c]);
          if (dist < best) {  // c increases with i: strict < keeps the lower index
            best = dist;
            besti = c;
          }
        }
      }
    }
    wave_argmin_f64(best, besti);
    if (lane == 0) {
      labels[r] = besti;
      const double m = best + xn[r];
      mind[r] = m > 0.0 ? m : 0.0;
      unsafeAtomicAdd(&counts[besti], 1.0);
    }
    double* srow = sums + (long)besti * d;
    for (long p = a + lane; p < b; p += 64) unsafeAtomicAdd(&srow[col[p]], val[p]);
  }
}

}  // namespace

// CSR rows (rowptr int64 [n+1], col int32, val fp64), CT [d][Kp] = centroids transposed
// (Kp >= K, multiple of 64), cn [K] = |c|^2, xn [n] = |x|^2. Writes labels [n] (int32),
// mind [n] (squared distance to the nearest centroid); ADDS into sums [K][d] and counts [K].
HARP_EXPORT int harp_kmeans_csr_assign(const long* rowptr, const int* col, const double* val, long n, int d,
                                       const double* CT, int K, int Kp, const double* cn, const double* xn,
                                       int* labels, double* mind, double* sums, double* counts, hipStream_t s) {
  if (n <= 0) return HARP_OK;
  if (K <= 0 || d <= 0 || Kp < K || (Kp & 63)) return HARP_EBADARG;
  long blocks = (n + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  const dim3 g((unsigned)blocks), bl(256);
  if (Kp <= 64) kmeans_csr_assign_kernel<1><<<g, bl, 0, s>>>(rowptr, col, val, n, d, CT, K, Kp, cn, xn, labels, mind, sums, counts);
  else if (Kp <= 128) kmeans_csr_assign_kernel<2><<<g, bl, 0, s>>>(rowptr, col, val, n, d, CT, K, Kp, cn, xn, labels, mind, sums, counts);
  else if (Kp <= 256) kmeans_csr_assign_kernel<4><<<g, bl, 0, s>>>(rowptr, col, val, n, d, CT, K, Kp, cn, xn, labels, mind, sums, counts);
  else if (Kp <= 512) kmeans_csr_assign_kernel<8><<<g, bl, 0, s>>>(rowptr, col, val, n, d, CT, K, Kp, cn, xn, labels, mind, sums, counts);
  else kmeans_csr_assign_kernel<16><<<g, bl, 0, s>>>(rowptr, col, val, n, d, CT, K, Kp, cn, xn, labels, mind, sums, counts);
  return harp_launch_status();
}
