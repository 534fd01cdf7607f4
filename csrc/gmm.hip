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
// (packed lower triangles) are read with scalar loads and used as SGPR operands of the
// FMAs. Pass 1 writes log p(x, k) into the n x K output and
// keeps an online log-sum-exp; pass 2 turns the row into responsibilities
// r = exp(log p - lse) in place; the per-point lse (log-likelihood terms) are summed per block.
//
// Statistics (gmm_stats_kernel): with the augmented point x' = [x, 1] every sufficient
// statistic is an entry of sum_n r_nk x'_n x'_n^T: (i, j <= d) the second moments, (i, d)
// the first moments, (d, d) N_k. One GEMM-shaped pass: a workgroup owns a 64-component x
// 128-pair tile and a block of points staged through LDS, each thread a 4 x 8 register
// tile; block partials are added into the fp64 output with atomics.
#include "common.h"

#include <utility>

namespace {

constexpr int kT = 256;

// The whitening matrices are the same for every point, so they are read with SCALAR loads
// (uniform addresses: s_load through the constant cache into SGPRs) and fed to the fp64
// FMAs as SGPR operands. A component's data is one "augmented" packed triangle, row i =
// [P_i0 .. P_ii, c_i] (row i starts at i (i + 3) / 2), consumed in chunks of 8 doubles:
// chunk C + 1 is loaded before chunk C is computed (software pipeline), and everything is
// generated at compile time (no branch, no per-element LDS read; two partial sums per row
// for independent FMA chains). The first form staged P through LDS and read one broadcast
// double per two FMAs (the LDS return path, 1 KB per wave-instruction): ~7 ms for N = 1e6,
// d = 32, K = 64.
template <int D>
constexpr int aug() { return D * (D + 1) / 2 + D; }
constexpr int row_start(int i) { return i * (i + 3) / 2; }
constexpr int row_of(int e) {
  int i = 0;
  while (row_start(i + 1) <= e) ++i;
  return i;
}
constexpr int kChunk = 8;  // doubles per scalar load group

template <int PPT>
struct TriAcc {
  double za[PPT], zb[PPT], maha[PPT];
};

// Pins the accumulators at this point of the instruction stream (the FMAs before it retire
// into them) and orders later loads after it: without it the compiler issued all of a
// component's scalar loads first, then the FMAs, and spilled the SGPRs it could not hold
// through v_writelane / v_readlane (3,300 lane moves per component at d = 32)
template <int PPT>
__device__ __forceinline__ void pin(TriAcc<PPT>& a) {
#pragma unroll
  for (int p = 0; p < PPT; ++p) asm volatile("" : "+v"(a.za[p]), "+v"(a.zb[p]), "+v"(a.maha[p])::"memory");
}

// element E of the augmented triangle with value v
template <int D, int PPT, int E>
__device__ __forceinline__ void tri_elem(double v, const double (&x)[PPT][D], TriAcc<PPT>& a) {
  if constexpr (E < aug<D>()) {
    constexpr int i = row_of(E), j = E - row_start(i);
    if constexpr (j <= i) {
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        if constexpr (j == 0)
          a.za[p] = v * x[p][0];
        else if constexpr (j == 1)
          a.zb[p] = v * x[p][1];
        else if constexpr (j % 2 == 0)
          a.za[p] = fma(v, x[p][j], a.za[p]);
        else
          a.zb[p] = fma(v, x[p][j], a.zb[p]);
      }
    } else {  // c_i closes row i
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        const double z = (i == 0 ? a.za[p] : a.za[p] + a.zb[p]) - v;
        a.maha[p] = fma(z, z, a.maha[p]);
      }
    }
  }
}

template <int D, int PPT, int C, int... Us>
__device__ __forceinline__ void tri_chunk(const double (&v)[kChunk], const double (&x)[PPT][D], TriAcc<PPT>& a,
                                          std::integer_sequence<int, Us...>) {
  (tri_elem<D, PPT, C * kChunk + Us>(v[Us], x, a), ...);
}

template <int D, int PPT, int C>
__device__ __forceinline__ void tri_pipe(const double* __restrict__ P, const double (&cur)[kChunk],
                                         const double (&x)[PPT][D], TriAcc<PPT>& a) {
  constexpr int NC = (aug<D>() + kChunk - 1) / kChunk;
  if constexpr (C < NC) {
    double nxt[kChunk];
    if constexpr (C + 1 < NC) {
#pragma unroll
      for (int u = 0; u < kChunk; ++u) nxt[u] = P[(C + 1) * kChunk + u];
    }
    tri_chunk<D, PPT, C>(cur, x, a, std::make_integer_sequence<int, kChunk>{});
    pin<PPT>(a);
    tri_pipe<D, PPT, C + 1>(P, nxt, x, a);
  }
}

template <int D, int PPT>
__global__ __launch_bounds__(kT) void gmm_estep_kernel(const double* __restrict__ X, long ldx, long n, int d, int K,
                                                       const double* __restrict__ Paug, const double* __restrict__ bk,
                                                       double* __restrict__ R, long ldr, double* __restrict__ ll_part) {
  constexpr int A = aug<D>();
  __shared__ double red[kT / 64];
  const int tid = threadIdx.x;
  double x[PPT][D];
  long pt[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    pt[p] = (long)blockIdx.x * (kT * PPT) + p * kT + tid;
    // unconditional clamped loads (no per-element exec masks), padding columns zeroed
    const double* xr = X + (pt[p] < n ? pt[p] : n - 1) * ldx;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const double v = xr[j < d ? j : d - 1];
      x[p][j] = j < d ? v : 0.0;
    }
  }
  double mx[PPT], sm[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    mx[p] = -__builtin_inf();
    sm[p] = 0.0;
  }
  for (int k = 0; k < K; ++k) {
    const double* __restrict__ P = Paug + (long)k * A;
    TriAcc<PPT> acc;
#pragma unroll
    for (int p = 0; p < PPT; ++p) {
      acc.za[p] = acc.zb[p] = 0.0;
      acc.maha[p] = 0.0;
    }
    double first[kChunk];
#pragma unroll
    for (int u = 0; u < kChunk; ++u) first[u] = P[u];
    tri_pipe<D, PPT, 0>(P, first, x, acc);
    double maha[PPT];
#pragma unroll
    for (int p = 0; p < PPT; ++p) maha[p] = acc.maha[p];
    const double b = bk[k];
#pragma unroll
    for (int p = 0; p < PPT; ++p) {
      if (pt[p] >= n) continue;
      const double lp = b - 0.5 * maha[p];
      R[(long)k * ldr + pt[p]] = lp;  // component-major: consecutive points, coalesced
      if (lp > mx[p]) {
        sm[p] = sm[p] * exp(mx[p] - lp) + 1.0;
        mx[p] = lp;
      } else {
        sm[p] += exp(lp - mx[p]);
      }
    }
  }
  double ll = 0.0;
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    if (pt[p] >= n) continue;
    const double lse = mx[p] + log(sm[p]);
    ll += lse;
    for (int k = 0; k < K; ++k) R[(long)k * ldr + pt[p]] = exp(R[(long)k * ldr + pt[p]] - lse);
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
      const int kk = e / SP, p = e % SP;  // consecutive threads: consecutive points
      const long pn = s0 + p;
      sr[p][kk] = (pn < ne && k0 + kk < K) ? R[(long)(k0 + kk) * ldr + pn] : 0.0;
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

// Full-covariance statistics by 4 x 4 coordinate blocks: the augmented point x' = [x, 1, 0..]
// is padded to DP = 4 NB coordinates, and pair-block (bi <= bj) holds the 16 products
// x'_{4bi+u} x'_{4bj+v}. A workgroup owns 64 components x 16 pair-blocks; a thread 4
// components x one pair-block (64 accumulators): per point it reads 4 responsibilities and
// 8 coordinates (six ds_read_b128) for 16 products and 64 FMAs. (The pair-list kernel read
// two coordinates per pair, 20 LDS reads per 32 FMAs, and was bound by the LDS return path.)
// S[k][pb][16] += over the block's points; diagonal blocks are computed whole.
constexpr int BSK = 64, BPB = 16, BSP = 32, MAXDP = 68;

__global__ __launch_bounds__(kT) void gmm_stats_blk_kernel(const double* __restrict__ X, long ldx, long n, int d,
                                                           const double* __restrict__ R, long ldr, int K, int nbk,
                                                           long pts_per_block, double* __restrict__ S) {
  __shared__ __attribute__((aligned(16))) double sx[BSP][MAXDP];
  __shared__ __attribute__((aligned(16))) double sr[BSP][BSK];
  const int tid = threadIdx.x;
  const int npb = nbk * (nbk + 1) / 2;
  const int k0 = blockIdx.y * BSK, tk = (tid >> 4) * 4;
  const int pb = blockIdx.z * BPB + (tid & 15);
  int bi = 0, rem = pb < npb ? pb : 0;
  while (rem >= nbk - bi) {
    rem -= nbk - bi;
    ++bi;
  }
  const int bj = bi + rem;
  double acc[4][16];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[a][q] = 0.0;
  const long nb = (long)blockIdx.x * pts_per_block;
  const long ne = nb + pts_per_block < n ? nb + pts_per_block : n;
  const int dp = nbk * 4;
  for (long s0 = nb; s0 < ne; s0 += BSP) {
    __syncthreads();
    for (int e = tid; e < BSP * dp; e += kT) {
      const int p = e / dp, f = e % dp;
      const long pn = s0 + p;
      sx[p][f] = pn < ne ? (f < d ? X[pn * ldx + f] : (f == d ? 1.0 : 0.0)) : 0.0;
    }
    for (int e = tid; e < BSP * BSK; e += kT) {
      const int kk = e / BSP, p = e % BSP;  // consecutive threads: consecutive points
      const long pn = s0 + p;
      sr[p][kk] = (pn < ne && k0 + kk < K) ? R[(long)(k0 + kk) * ldr + pn] : 0.0;
    }
    __syncthreads();
#pragma unroll 2
    for (int p = 0; p < BSP; ++p) {
      double r[4], xi[4], xj[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) r[a] = sr[p][tk + a];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xi[u] = sx[p][bi * 4 + u];
        xj[u] = sx[p][bj * 4 + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const double pr = xi[u] * xj[v];
#pragma unroll
          for (int a = 0; a < 4; ++a) acc[a][u * 4 + v] = fma(r[a], pr, acc[a][u * 4 + v]);
        }
    }
  }
  if (pb >= npb) return;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int k = k0 + tk + a;
    if (k >= K) continue;
#pragma unroll
    for (int q = 0; q < 16; ++q) atomicAdd(S + ((long)k * npb + pb) * 16 + q, acc[a][q]);
  }
}

template <int D, int PPT>
int launch_estep(const double* X, long ldx, long n, int d, int K, const double* P, const double* b, double* R,
                 long ldr, double* ll_part, hipStream_t s) {
  const long blocks = (n + kT * PPT - 1) / (kT * PPT);
  gmm_estep_kernel<D, PPT><<<dim3((unsigned)blocks), dim3(kT), 0, s>>>(X, ldx, n, d, K, P, b, R, ldr, ll_part);
  return harp_launch_status();
}

}  // namespace

// blocks of the E-step grid (size of ll_part) for n points of padded width D(d)
HARP_EXPORT int harp_gmm_estep_blocks(long n, int d) {
  const int ppt = 1;
  return (int)((n + kT * ppt - 1) / (kT * ppt));
}

// the padded feature width D the E-step expects, and the length of one component's
// augmented packed triangle (rows [P_i0 .. P_ii, c_i], i < D); the array needs kChunk
// doubles of padding after the last component
HARP_EXPORT int harp_gmm_width(int d) { return d <= 8 ? 8 : d <= 16 ? 16 : d <= 32 ? 32 : d <= 64 ? 64 : -1; }
HARP_EXPORT int harp_gmm_aug_len(int d) {
  const int D = harp_gmm_width(d);
  return D < 0 ? -1 : D * (D + 1) / 2 + D;
}
HARP_EXPORT int harp_gmm_aug_pad() { return kChunk; }

// R is component-major: R[k * ldr + i] (ldr >= n)
HARP_EXPORT int harp_gmm_estep(const double* X, long ldx, long n, int d, int K, const double* P, const double* b,
                               double* R, long ldr, double* ll_part, hipStream_t s) {
  if (n < 0 || d <= 0 || d > 64 || K <= 0 || ldx < d || ldr < n) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  // one point per thread: more resident waves hide the scalar-load waits better than two
  // points' FMAs per load (d = 32: 2.71 vs 3.45 ms, profiles/r3_gmm)
  if (d <= 8) return launch_estep<8, 1>(X, ldx, n, d, K, P, b, R, ldr, ll_part, s);
  if (d <= 16) return launch_estep<16, 1>(X, ldx, n, d, K, P, b, R, ldr, ll_part, s);
  if (d <= 32) return launch_estep<32, 1>(X, ldx, n, d, K, P, b, R, ldr, ll_part, s);
  return launch_estep<64, 1>(X, ldx, n, d, K, P, b, R, ldr, ll_part, s);
}

// S [K][npairs] (+)= sum_n R[k][n] x'_i x'_j over the given pairs of the augmented point
// (R component-major, R[k * ldr + i], ldr >= n)
HARP_EXPORT int harp_gmm_stats(const double* X, long ldx, long n, int d, const double* R, long ldr, int K,
                               const int* pair_i, const int* pair_j, int npairs, double* S, hipStream_t s) {
  if (n < 0 || d <= 0 || d > 64 || K <= 0 || npairs <= 0 || ldx < d || ldr < n) return HARP_EBADARG;
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

// Full-covariance statistics by 4 x 4 coordinate blocks (gmm_stats_blk_kernel): S [K][npb][16]
// (+)= sum_n R[k][n] x'_{4bi+u} x'_{4bj+v} for pair-blocks pb = (bi <= bj) of the augmented
// point padded to 4 nbk coordinates (nbk = harp_gmm_coord_blocks(d)); R component-major.
HARP_EXPORT int harp_gmm_coord_blocks(int d) { return d <= 0 || d > 64 ? -1 : (d + 1 + 3) / 4; }

HARP_EXPORT int harp_gmm_stats_blocks(const double* X, long ldx, long n, int d, const double* R, long ldr, int K,
                                      double* S, hipStream_t s) {
  if (n < 0 || d <= 0 || d > 64 || K <= 0 || ldx < d || ldr < n) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  const int nbk = harp_gmm_coord_blocks(d), npb = nbk * (nbk + 1) / 2;
  const int ky = (K + BSK - 1) / BSK, qz = (npb + BPB - 1) / BPB;
  long nbx = 2048 / (ky * qz);
  if (nbx < 1) nbx = 1;
  long per = (n + nbx - 1) / nbx;
  per = (per + BSP - 1) / BSP * BSP;
  if (per < 4 * BSP) per = 4 * BSP;
  nbx = (n + per - 1) / per;
  gmm_stats_blk_kernel<<<dim3((unsigned)nbx, ky, qz), dim3(kT), 0, s>>>(X, ldx, n, d, R, ldr, K, nbk, per, S);
  return harp_launch_status();
}
