// Tall-skinny QR panel kernels (fp64) for gfx950: the building blocks of the distributed
// 3-step QR / SVD / SVD-PCA (DAAL svd & qr DistributedStep1Local / Step2Master /
// Step3Local: ml/daal/.../daal_svd/SVDDaalCollectiveMapper.java:149-204,
// daal_qr/QRDaalCollectiveMapper.java:131-153).
//
// Design (MI355X-first):
//  * a workgroup of B = 256 threads factors one B x D row block with Householder
//    reflections, ONE ROW PER THREAD held in registers (D <= 64 fp64 = 128 VGPRs): the
//    column norm is a block reduction, the reflector's dot products with the trailing
//    columns are a [256][D] LDS transpose-reduce, and the rank-1 update is register-local.
//    No LDS copy of the block, no global traffic besides one read and one write of it.
//  * the tree: the stacked R factors of a level are the next level's matrix, factored by
//    the same kernel (B/D R's per block) until one block remains (classical TSQR).
//  * explicit Q: the top level applies its reflectors to [I; 0]; every lower block applies
//    its reflectors to [S_b; 0] where S_b is its D x D slice of the level above's Q, so
//    Q_block * S_b needs no separate GEMM.
#include "common.h"

namespace {

constexpr int TB = 256;  // rows per block = threads per workgroup

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of one value per thread (4 waves); result broadcast to every thread
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum_f64(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// wk[k] = sum over threads of buf[t][k] (k < D): the [TB][D+1] LDS image every thread has
// just written its row of products into (after the barrier here), transposed and reduced
template <int D>
__device__ __forceinline__ void block_colsum(double* buf, double* wk) {
  const int t = threadIdx.x;
  __syncthreads();
  constexpr int PARTS = TB / D;  // threads per column
  const int k = t % D, part = t / D;
  double s = 0.0;
  for (int i = part; i < TB; i += PARTS) s += buf[i * (D + 1) + k];
  __syncthreads();
  buf[t] = s;  // [PARTS][D] partials (reuses the first TB slots)
  __syncthreads();
  if (t < D) {
    double a = 0.0;
    for (int q = 0; q < PARTS; ++q) a += buf[q * D + t];
    wk[t] = a;
  }
  __syncthreads();
}

// Householder QR of rows [b*TB, b*TB + m) of A (m <= TB; missing rows are zero).
// Writes the factored block (R on/above the diagonal, reflector tails below) to V (same
// row layout), tau[b][D] and R[b] (D x D, zeros below the diagonal).
template <int D>
__global__ __launch_bounds__(TB) void house_qr_kernel(const double* __restrict__ A, long lda, long nrows, int d,
                                                      double* __restrict__ V, long ldv, double* __restrict__ tau,
                                                      double* __restrict__ R) {
  __shared__ double buf[TB * (D + 1)];
  __shared__ double red[4];
  __shared__ double wk[D];
  __shared__ double hh[3];  // beta, tau, scale
  const int t = threadIdx.x;
  const long row = (long)blockIdx.x * TB + t;
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = (row < nrows && k < d) ? A[row * lda + k] : 0.0;
  double* taub = tau + (long)blockIdx.x * D;
  // the step loop is NOT unrolled (D^2 code); x[j] with a runtime j is a select chain over
  // the statically indexed registers, so the row never leaves the VGPRs
#pragma unroll 1
  for (int j = 0; j < D; ++j) {
    double xj = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) xj = k == j ? x[k] : xj;
    // reflector for column j over rows j..TB-1
    const double sig = block_sum(t > j ? xj * xj : 0.0, red);
    if (t == j) {
      const double alpha = xj;
      double beta = alpha, tj = 0.0, sc = 0.0;
      if (sig > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + sig), alpha);
        tj = (beta - alpha) / beta;
        sc = 1.0 / (alpha - beta);
      }
      hh[0] = beta;
      hh[1] = tj;
      hh[2] = sc;
    }
    __syncthreads();
    const double beta = hh[0], tj = hh[1], sc = hh[2];
    const double v = t == j ? 1.0 : (t > j ? xj * sc : 0.0);
    __syncthreads();  // the previous step's readers of buf / wk are done
    // w_k = v^T A[:, k] for the trailing columns
#pragma unroll
    for (int k = 0; k < D; ++k) buf[t * (D + 1) + k] = k > j ? v * x[k] : 0.0;
    block_colsum<D>(buf, wk);
    const double nj = t == j ? beta : (t > j ? v : xj);  // reflector tail stored below the diagonal
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = k > j ? x[k] - tj * v * wk[k] : (k == j ? nj : x[k]);
    if (t == 0) taub[j] = tj;
  }
  if (row < nrows) {
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k < d) V[row * ldv + k] = x[k];
  }
  if (t < D) {
    double* Rb = R + (long)blockIdx.x * D * D + (long)t * D;
#pragma unroll
    for (int k = 0; k < D; ++k) Rb[k] = k >= t ? x[k] : 0.0;
  }
}

// Q rows of block b: H_0 H_1 ... H_{D-1} [S_b; 0], S_b = S[b*D .. b*D+D) (identity when
// S is null), written to Q rows [b*TB, b*TB+m).
template <int D>
__global__ __launch_bounds__(TB) void house_apply_kernel(const double* __restrict__ V, long ldv, long nrows, int d,
                                                         const double* __restrict__ tau, const double* __restrict__ S,
                                                         double* __restrict__ Q, long ldq) {
  __shared__ double buf[TB * (D + 1)];
  __shared__ double wk[D];
  const int t = threadIdx.x;
  const long row = (long)blockIdx.x * TB + t;
  double vr[D], y[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    vr[k] = (row < nrows && k < d) ? V[row * ldv + k] : 0.0;
    double s = 0.0;
    if (t < D) s = S ? S[((long)blockIdx.x * D + t) * D + k] : (t == k ? 1.0 : 0.0);
    y[k] = s;
  }
  const double* taub = tau + (long)blockIdx.x * D;
#pragma unroll 1
  for (int jj = 0; jj < D; ++jj) {
    const int j = D - 1 - jj;
    double vj = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) vj = k == j ? vr[k] : vj;
    const double v = t == j ? 1.0 : (t > j ? vj : 0.0);
    const double tj = taub[j];
    __syncthreads();  // the previous step's readers of buf / wk are done
#pragma unroll
    for (int k = 0; k < D; ++k) buf[t * (D + 1) + k] = v * y[k];
    block_colsum<D>(buf, wk);
#pragma unroll
    for (int k = 0; k < D; ++k) y[k] -= tj * v * wk[k];
  }
  if (row < nrows) {
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k < d) Q[row * ldq + k] = y[k];
  }
}

template <int D>
int launch_qr(const double* A, long lda, long nrows, int d, double* V, long ldv, double* tau, double* R,
              hipStream_t s) {
  const long nb = (nrows + TB - 1) / TB;
  house_qr_kernel<D><<<dim3((unsigned)nb), dim3(TB), 0, s>>>(A, lda, nrows, d, V, ldv, tau, R);
  return harp_launch_status();
}

template <int D>
int launch_apply(const double* V, long ldv, long nrows, int d, const double* tau, const double* S, double* Q, long ldq,
                 hipStream_t s) {
  const long nb = (nrows + TB - 1) / TB;
  house_apply_kernel<D><<<dim3((unsigned)nb), dim3(TB), 0, s>>>(V, ldv, nrows, d, tau, S, Q, ldq);
  return harp_launch_status();
}

}  // namespace

// Register width used for d columns (the kernels are instantiated for 8, 16, 32, 64).
HARP_EXPORT int harp_tsqr_width(int d) {
  if (d <= 0 || d > 64) return -1;
  return d <= 8 ? 8 : d <= 16 ? 16 : d <= 32 ? 32 : 64;
}

HARP_EXPORT int harp_tsqr_rows_per_block() { return TB; }

// One level: factor A [nrows, d] in TB-row blocks. V [nrows, >= d] (may alias A), tau
// [nblocks, D], R [nblocks, D, D] with D = harp_tsqr_width(d).
HARP_EXPORT int harp_tsqr_level(const double* A, long lda, long nrows, int d, double* V, long ldv, double* tau,
                                double* R, hipStream_t s) {
  if (nrows <= 0) return HARP_OK;
  if (lda < d || ldv < d) return HARP_EBADARG;
  switch (harp_tsqr_width(d)) {
    case 8: return launch_qr<8>(A, lda, nrows, d, V, ldv, tau, R, s);
    case 16: return launch_qr<16>(A, lda, nrows, d, V, ldv, tau, R, s);
    case 32: return launch_qr<32>(A, lda, nrows, d, V, ldv, tau, R, s);
    case 64: return launch_qr<64>(A, lda, nrows, d, V, ldv, tau, R, s);
    default: return HARP_EUNSUPPORTED;
  }
}

// Explicit Q of one level: Q [nrows, d] = blockdiag(H-products) [S_b; 0] (S: [nblocks*D, D]
// or null for identity).
HARP_EXPORT int harp_tsqr_apply(const double* V, long ldv, long nrows, int d, const double* tau, const double* S,
                                double* Q, long ldq, hipStream_t s) {
  if (nrows <= 0) return HARP_OK;
  if (ldv < d || ldq < d) return HARP_EBADARG;
  switch (harp_tsqr_width(d)) {
    case 8: return launch_apply<8>(V, ldv, nrows, d, tau, S, Q, ldq, s);
    case 16: return launch_apply<16>(V, ldv, nrows, d, tau, S, Q, ldq, s);
    case 32: return launch_apply<32>(V, ldv, nrows, d, tau, S, Q, ldq, s);
    case 64: return launch_apply<64>(V, ldv, nrows, d, tau, S, Q, ldq, s);
    default: return HARP_EUNSUPPORTED;
  }
}
