// EM for Gaussian mixtures (gfx950): fused E-step and sufficient-statistics kernels, fp64.
//
// Reference: ml/daal/src/main/java/edu/iu/daal_em/BatchDense/EMDaalCollectiveMapper.java:146-156
// (DAAL em_gmm batch: E-step responsibilities, M-step weights / means / covariances,
// log-likelihood stopping rule).
//
// E-step (gmm_estep_kernel): with Sigma_k = L_k L_k^T and P_k = L_k^-1 (lower triangular),
// the Mahalanobis term is ||P_k x - c_k||^2 with c_k = P_k mu_k, so
//   log N(x | k) + log w_k = b_k - 0.5 ||P_k x - c_k||^2,  b_k = log w_k - 0.5 (log|Sigma_k| + d log 2 pi)
// Every thread keeps PPT points (D features each) in registers; the K whitening matrices
// stream through LDS in chunks of KC components (packed lower triangles, read as LDS
// broadcasts: one read feeds PPT FMAs). Pass 1 writes log p(x, k) into the n x K output and
// keeps an online log-sum-exp; pass 2 turns the row into responsibilities
// r = exp(log p - lse) in place; the per-point lse (log-likelihood terms) are summed per block.
//
// Statistics (gmm_stats_kernel): with the augmented point x' = [x, 1] every sufficient
// statistic is an entry of sum_n r_nk x'_n x'_n^T: (i, j <= d) the second moments, (i, d)
// the first moments, (d, d) N_k. One GEMM-shaped pass: a workgroup owns a 64-component x
// 128-pair tile and a block of points staged through LDS, each thread a 4 x 8 register
// tile; block partials are added into the fp64 output with atomics.
#include "common.h"

namespace {

constexpr int kT = 256;

template <int D>
constexpr int tri() { return D * (D + 1) / 2; }

template <int D, int PPT, int KC>
__global__ __launch_bounds__(kT) void gmm_estep_kernel(const double* __restrict__ X, long ldx, long n, int d,
                                                       int K, const double* __restrict__ Ptri,
                                                       const double* __restrict__ cvec, const double* __restrict__ bk,
                                                       double* __restrict__ R, long ldr, double* __restrict__ ll_part) {
  constexpr int TRI = tri<D>();
  constexpr int STRIDE = TRI + D + 1;  // packed P, c, b of one component
  __shared__ double sP[KC * STRIDE];
  __shared__ double red[kT / 64];
  const int tid = threadIdx.x;
  double x[PPT][D];
  long pt[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    pt[p] = (long)blockIdx.x * (kT * PPT) + p * kT + tid;
#pragma unroll
    for (int j = 0; j < D; ++j) x[p][j] = (pt[p] < n && j < d) ? X[pt[p] * ldx + j] : 0.0;
  }
  double mx[PPT], sm[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    mx[p] = -__builtin_inf();
    sm[p] = 0.0;
  }
  for (int k0 = 0; k0 < K; k0 += KC) {
    const int kc = K - k0 < KC ? K - k0 : KC;
    __syncthreads();
    for (int e = tid; e < kc * STRIDE; e += kT) {
      const int kk = e / STRIDE, o = e % STRIDE;
      const int k = k0 + kk;
      sP[e] = o < TRI ? Ptri[(long)k * TRI + o] : (o < TRI + D ? cvec[(long)k * D + (o - TRI)] : bk[k]);
    }
    __syncthreads();
    for (int kk = 0; kk < kc; ++kk) {
      const double* P = sP + kk * STRIDE;
      double maha[PPT];
#pragma unroll
      for (int p = 0; p < PPT; ++p) maha[p] = 0.0;
      // rows i of the triangle: a runtime loop (wave-uniform), the columns unrolled so the
      // point coordinates stay in registers; j > i is skipped by a uniform branch
#pragma unroll 1
      for (int i = 0; i < D; ++i) {
        double z[PPT];
        const double ci = P[TRI + i];
        const double* Pi = P + i * (i + 1) / 2;
#pragma unroll
        for (int p = 0; p < PPT; ++p) z[p] = -ci;
#pragma unroll
        for (int j = 0; j < D; ++j) {
          if (j <= i) {
            const double pij = Pi[j];
#pragma unroll
            for (int p = 0; p < PPT; ++p) z[p] = fma(pij, x[p][j], z[p]);
          }
        }
#pragma unroll
        for (int p = 0; p < PPT; ++p) maha[p] = fma(z[p], z[p], maha[p]);
      }
      const double b = P[TRI + D];
      const int k = k0 + kk;
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        if (pt[p] >= n) continue;
        const double lp = b - 0.5 * maha[p];
        R[pt[p] * ldr + k] = lp;
        if (lp > mx[p]) {
          sm[p] = sm[p] * exp(mx[p] - lp) + 1.0;
          mx[p] = lp;
        } else {
          sm[p] += exp(lp - mx[p]);
        }
      }
    }
  }
  double ll = 0.0;
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    if (pt[p] >= n) continue;
    const double lse = mx[p] + log(sm[p]);
    ll += lse;
    double* row = R + pt[p] * ldr;
    for (int k = 0; k < K; ++k) row[k] = exp(row[k] - lse);
  }
  ll = wave_sum_d(ll);
  if ((tid & 63) == 0) red[tid >> 6] = ll;
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kT / 64; ++w) s += red[w];
    ll_part[blockIdx.x] = s;
  }
}

// S[k][q] += sum over the block's points of R[n][k] * x'[n][i_q] * x'[n][j_q], pairs q of
// the augmented point (i_q <= j_q < d + 1, row-major upper triangle), tile 64 k x 128 q.
constexpr int SK = 64, SQ = 128, SP = 32;  // components, pairs per tile; points per LDS stage

__global__ __launch_bounds__(kT) void gmm_stats_kernel(const double* __restrict__ X, long ldx, long n, int d,
                                                       const double* __restrict__ R, long ldr, int K,
                                                       const int* __restrict__ pair_i, const int* __restrict__ pair_j,
                                                       int npairs, long pts_per_block, double* __restrict__ S) {
  __shared__ double sx[SP][65];  // augmented points (d + 1 <= 65)
  __shared__ double sr[SP][SK];
  const int tid = threadIdx.x;
  const int k0 = blockIdx.y * SK, q0 = blockIdx.z * SQ;
  const int tk = (tid / 16) * 4, tq = (tid % 16) * 8;  // this thread's 4 x 8 sub-tile
  int qi[8], qj[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int q = q0 + tq + c;
    qi[c] = q < npairs ? pair_i[q] : d;  // padding pairs read the ones column (discarded)
    qj[c] = q < npairs ? pair_j[q] : d;
  }
  double acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[a][c] = 0.0;
  const long nb = (long)blockIdx.x * pts_per_block;
  const long ne = nb + pts_per_block < n ? nb + pts_per_block : n;
  const int dd = d + 1;
  for (long s0 = nb; s0 < ne; s0 += SP) {
    __syncthreads();
    for (int e = tid; e < SP * dd; e += kT) {
      const int p = e / dd, f = e % dd;
      const long pn = s0 + p;
      sx[p][f] = pn < ne ? (f < d ? X[pn * ldx + f] : 1.0) : 0.0;
    }
    for (int e = tid; e < SP * SK; e += kT) {
      const int p = e / SK, kk = e % SK;
      const long pn = s0 + p;
      sr[p][kk] = (pn < ne && k0 + kk < K) ? R[pn * ldr + k0 + kk] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int p = 0; p < SP; ++p) {
      double r[4], v[8];
#pragma unroll
      for (int a = 0; a < 4; ++a) r[a] = sr[p][tk + a];
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = sx[p][qi[c]] * sx[p][qj[c]];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[a][c] = fma(r[a], v[c], acc[a][c]);
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int k = k0 + tk + a;
    if (k >= K) continue;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int q = q0 + tq + c;
      if (q < npairs) atomicAdd(S + (long)k * npairs + q, acc[a][c]);
    }
  }
}

template <int D, int PPT>
int launch_estep(const double* X, long ldx, long n, int d, int K, const double* P, const double* c, const double* b,
                 double* R, long ldr, double* ll_part, hipStream_t s) {
  constexpr int KC = 8;
  const long blocks = (n + kT * PPT - 1) / (kT * PPT);
  gmm_estep_kernel<D, PPT, KC><<<dim3((unsigned)blocks), dim3(kT), 0, s>>>(X, ldx, n, d, K, P, c, b, R, ldr, ll_part);
  return harp_launch_status();
}

}  // namespace

// blocks of the E-step grid (size of ll_part) for n points of padded width D(d)
HARP_EXPORT int harp_gmm_estep_blocks(long n, int d) {
  const int ppt = d <= 32 ? 2 : 1;
  return (int)((n + kT * ppt - 1) / (kT * ppt));
}

// the padded feature width the E-step expects in P (packed lower triangles of D x D) and c (D)
HARP_EXPORT int harp_gmm_width(int d) { return d <= 8 ? 8 : d <= 16 ? 16 : d <= 32 ? 32 : d <= 64 ? 64 : -1; }

HARP_EXPORT int harp_gmm_estep(const double* X, long ldx, long n, int d, int K, const double* P, const double* c,
                               const double* b, double* R, long ldr, double* ll_part, hipStream_t s) {
  if (n < 0 || d <= 0 || d > 64 || K <= 0 || ldx < d || ldr < K) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  if (d <= 8) return launch_estep<8, 2>(X, ldx, n, d, K, P, c, b, R, ldr, ll_part, s);
  if (d <= 16) return launch_estep<16, 2>(X, ldx, n, d, K, P, c, b, R, ldr, ll_part, s);
  if (d <= 32) return launch_estep<32, 2>(X, ldx, n, d, K, P, c, b, R, ldr, ll_part, s);
  return launch_estep<64, 1>(X, ldx, n, d, K, P, c, b, R, ldr, ll_part, s);
}

// S [K][npairs] (+)= sum_n R[n][k] x'_i x'_j over the given pairs of the augmented point
HARP_EXPORT int harp_gmm_stats(const double* X, long ldx, long n, int d, const double* R, long ldr, int K,
                               const int* pair_i, const int* pair_j, int npairs, double* S, hipStream_t s) {
  if (n < 0 || d <= 0 || d > 64 || K <= 0 || npairs <= 0 || ldx < d || ldr < K) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  // enough point blocks to fill the chip several times over with the (k, pair) tiles
  const int ky = (K + SK - 1) / SK, qz = (npairs + SQ - 1) / SQ;
  long nbx = 2048 / (ky * qz);
  if (nbx < 1) nbx = 1;
  long per = (n + nbx - 1) / nbx;
  per = (per + SP - 1) / SP * SP;
  if (per < 4 * SP) per = 4 * SP;
  nbx = (n + per - 1) / per;
  gmm_stats_kernel<<<dim3((unsigned)nbx, ky, qz), dim3(kT), 0, s>>>(X, ldx, n, d, R, ldr, K, pair_i, pair_j, npairs,
                                                                    per, S);
  return harp_launch_status();
}
