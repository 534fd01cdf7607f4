// Eigenvectors of a symmetric tridiagonal matrix on gfx950: Cuppen divide and conquer with
// Gu-Eisenstat (Loewner) vectors, every merge of a tree level in the same launches.
//
// Reference: the PCA step of the DAAL correlation method returns eigenvalues AND
// eigenvectors, ml/daal/src/main/java/edu/iu/daal_pca/cordensedistr/PCADaalCollectiveMapper.java:136-154.
// The host reference (same tree, deflation, root finder and vectors, step for step) is
// harp_amd/ops/tridiag_dc.py; its docstring has the derivation.
//
// Per tree level (merges (lo, mid, hi), bottom-up; 1 x 1 leaves):
//  1. dc_prep_kernel, one workgroup per merge: z from the last row of the left block and the
//     first row of the right block of Q, the merged ascending order (rank by counting),
//     rho, and deflation. Small-z deflation is decided in parallel; the rotation deflation of
//     close neighbours is a dependent chain, so one thread walks it -- unless no neighbour
//     pair passes the rotation test, which every thread checks first (the common case).
//     Deflation rotations are applied to Q's columns in the same launch (rows in parallel).
//  2. dc_secular_kernel, ONE WAVE PER ROOT: the k roots of 1/rho + sum z_j^2/(d_j - lambda)
//     in coordinates shifted to the nearer pole; the lanes split the sums, so an iteration
//     costs k/64 terms per lane plus four wave reductions (a thread per root: ~30x longer
//     at k = 1000). Two-pole rational model steps inside a bisection bracket.
//  3. dc_loewner_kernel, one wave per kept j: zhat_j as a product of ratios over the roots.
//  4. dc_vectors_kernel, one wave per root: the normalised column of U.
//  5. dc_gemm_kernel: Q_new[block] = Q[block rows, kept columns] x U (64 x 64 tiles over
//     LDS, fp64 FMA), deflated columns copied; Q ping-pongs between two buffers.
// Eigenvalues are carried as (origin pole, tau) while the vectors are formed, so every
// difference d_j - lambda_i is computed as (d_j - d_o) - tau without cancellation.
#include "common.h"

namespace {

constexpr int kMaxN = 4096;
constexpr double kEps = 2.220446049250313e-16;

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_prod_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v *= __shfl_xor(v, o, 64);
  return v;
}

// block reductions (1024 threads), result in every thread
__device__ __forceinline__ double block_sum_1k(double v, double* red) {
  v = wave_sum_d_dpp(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}
__device__ __forceinline__ double block_max_1k(double v, double* red) {
  v = wave_max_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s = fmax(s, red[w]);
  return s;
}

// merge holding position c (merges sorted by lo, nm of them)
__device__ __forceinline__ int find_merge(const int* __restrict__ mg, int nm, int c) {
  int a = 0, b = nm - 1;
  while (a < b) {
    const int m = (a + b + 1) >> 1;
    if (mg[3 * m] <= c) a = m;
    else b = m - 1;
  }
  return a;
}

struct DcWs {
  double *dd, *zz, *tau, *zh, *rho, *U, *rotc, *rots, *sortbuf;
  int *colsrc, *org, *kcnt, *rotp, *rotq;
  long ldu;  // U of the merge at lo starts at lo * ldu (ldu >= the level's largest block)
};

// ---------------------------------------------------------------------------------------
// 1. z, sort, rho, deflation (+ rotations applied to Q). Q: n x n column-major (ldq).
__global__ __launch_bounds__(1024) void dc_prep_kernel(double* __restrict__ Q, long ldq, double* __restrict__ D,
                                                       const double* __restrict__ e, const int* __restrict__ mg,
                                                       DcWs w) {
  extern __shared__ double sm[];
  const int lo = mg[3 * blockIdx.x], mid = mg[3 * blockIdx.x + 1], hi = mg[3 * blockIdx.x + 2];
  const int s = hi - lo, s1 = mid - lo;
  double* sd = sm;                 // [s] eigenvalues (raw, then sorted)
  double* sz = sm + s;             // [s] z (raw, then sorted)
  int* src = (int*)(sm + 2 * s);   // [s] local source column of sorted position
  int* keep = src + s;             // [s]
  int* defl = keep + s;            // [s]
  __shared__ double red[16];
  __shared__ int s_k, s_nd, s_nrot, s_serial;
  const int tid = threadIdx.x, T = blockDim.x;
  const double beta = e[mid - 1];
  const double sgn = beta < 0.0 ? -1.0 : 1.0;
  // raw values: left block's last row, right block's first row (sign of beta folded in)
  for (int j = tid; j < s; j += T) {
    sd[j] = D[lo + j];
    sz[j] = j < s1 ? Q[(long)(lo + j) * ldq + (mid - 1)] : sgn * Q[(long)(lo + j) * ldq + mid];
  }
  __syncthreads();
  // ranks (ties by index) -> the sorted lists go through global scratch (3 s doubles at 3 lo)
  double* tmp = w.sortbuf + 3L * lo;
  for (int j = tid; j < s; j += T) {
    const double v = sd[j];
    int r = 0;
    for (int i = 0; i < s; ++i) {
      const double u = sd[i];
      r += (u < v) || (u == v && i < j);
    }
    tmp[r] = v;
    tmp[s + r] = sz[j];
    ((int*)(tmp + 2 * s))[r] = j;
  }
  __threadfence_block();
  __syncthreads();
  for (int j = tid; j < s; j += T) {
    sd[j] = tmp[j];
    sz[j] = tmp[s + j];
    src[j] = ((int*)(tmp + 2 * s))[j];
  }
  __syncthreads();
  double nz2 = 0.0, dmax = 0.0;
  for (int j = tid; j < s; j += T) {
    nz2 = fma(sz[j], sz[j], nz2);
    dmax = fmax(dmax, fabs(sd[j]));
  }
  nz2 = block_sum_1k(nz2, red);
  dmax = block_max_1k(dmax, red);
  const double rho = fabs(beta) * nz2;
  const double inz = nz2 > 0.0 ? 1.0 / sqrt(nz2) : 0.0;
  double zmax = 0.0;
  for (int j = tid; j < s; j += T) {
    sz[j] *= inz;
    zmax = fmax(zmax, fabs(sz[j]));
  }
  zmax = block_max_1k(zmax, red);
  const double tol = 8.0 * kEps * fmax(dmax, rho * zmax);
  // parallel pre-check: does any pair of consecutive small-z survivors pass the rotation
  // test? If not, the walk below reduces to a compaction (done in parallel)
  if (tid == 0) s_serial = 0;
  __syncthreads();
  if (rho > 0.0) {
    for (int j = tid; j < s; j += T) {
      if (rho * fabs(sz[j]) <= tol) continue;
      int p = j - 1;
      while (p >= 0 && rho * fabs(sz[p]) <= tol) --p;
      if (p < 0) continue;
      const double ss = sz[p], cc = sz[j];
      const double t2 = hypot(cc, ss);
      if (fabs((sd[j] - sd[p]) * (cc / t2) * (ss / t2)) <= tol) s_serial = 1;  // benign race: any writer sets 1
    }
  }
  __syncthreads();
  if (rho == 0.0) {  // decoupled halves: everything deflates, in sorted order
    for (int j = tid; j < s; j += T) defl[j] = j;
    if (tid == 0) {
      s_k = 0;
      s_nd = s;
      s_nrot = 0;
    }
  } else if (!s_serial) {
    // compaction: keep = survivors, defl = small z, both ascending (wave ballots in order)
    if (tid < 64) {
      int kk = 0, nd = 0;
      for (int b = 0; b < s; b += 64) {
        const int j = b + tid;
        const bool in = j < s;
        const bool dj = in && rho * fabs(sz[j]) <= tol;
        const unsigned long long mk = __ballot(in && !dj), md = __ballot(dj);
        const unsigned long long below = (1ull << tid) - 1ull;
        if (in && !dj) keep[kk + __popcll(mk & below)] = j;
        if (dj) defl[nd + __popcll(md & below)] = j;
        kk += __popcll(mk);
        nd += __popcll(md);
      }
      if (tid == 0) {
        s_k = kk;
        s_nd = nd;
        s_nrot = 0;
      }
    }
  } else if (tid == 0) {
    // the dependent walk (LAPACK dlaed2 order): a rotated pair keeps d_pj c^2 + d_j s^2 at
    // pj (deflated) and continues with j
    int kk = 0, nd = 0, nr = 0, pj = -1;
    for (int j = 0; j < s; ++j) {
      if (rho * fabs(sz[j]) <= tol) {
        defl[nd++] = j;
        continue;
      }
      if (pj < 0) {
        pj = j;
        continue;
      }
      double ss = sz[pj], cc = sz[j];
      const double t2 = hypot(cc, ss);
      const double t = sd[j] - sd[pj];
      cc /= t2;
      ss = -ss / t2;
      if (fabs(t * cc * ss) <= tol) {
        sz[j] = t2;
        sz[pj] = 0.0;
        w.rotp[lo + nr] = lo + src[pj];
        w.rotq[lo + nr] = lo + src[j];
        w.rotc[lo + nr] = cc;
        w.rots[lo + nr] = ss;
        ++nr;
        const double tt = sd[pj] * cc * cc + sd[j] * ss * ss;
        sd[j] = sd[pj] * ss * ss + sd[j] * cc * cc;
        sd[pj] = tt;
        defl[nd++] = pj;
        pj = j;
      } else {
        keep[kk++] = pj;
        pj = j;
      }
    }
    if (pj >= 0) keep[kk++] = pj;
    s_k = kk;
    s_nd = nd;
    s_nrot = nr;
  }
  __threadfence_block();
  __syncthreads();
  const int k = s_k, nd = s_nd, nrot = s_nrot;
  // deflation rotations on Q's columns, in order (each row independent)
  if (nrot) {
    for (int r = lo + tid; r < hi; r += T) {
      for (int q = 0; q < nrot; ++q) {
        double* x = Q + (long)w.rotp[lo + q] * ldq + r;
        double* y = Q + (long)w.rotq[lo + q] * ldq + r;
        const double c = w.rotc[lo + q], sn = w.rots[lo + q];
        const double xv = *x, yv = *y;
        *x = c * xv + sn * yv;
        *y = c * yv - sn * xv;
      }
    }
  }
  for (int i = tid; i < k; i += T) {
    const int j = keep[i];
    w.dd[lo + i] = sd[j];
    w.zz[lo + i] = sz[j];
    w.colsrc[lo + i] = lo + src[j];
  }
  for (int t = tid; t < nd; t += T) {
    const int j = defl[t];
    w.colsrc[lo + k + t] = lo + src[j];
    D[lo + k + t] = sd[j];  // final for this merge
  }
  if (tid == 0) {
    w.kcnt[lo] = k;
    w.rho[lo] = rho;
  }
}

// ---------------------------------------------------------------------------------------
// 2. secular roots: one wave per root; 4 roots per 256-thread workgroup over positions
__global__ __launch_bounds__(256) void dc_secular_kernel(const int* __restrict__ mg, int nm, int n, double* __restrict__ D,
                                                         DcWs w) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= n) return;
  const int m = find_merge(mg, nm, c);
  const int lo = mg[3 * m];
  if (c < lo || c >= mg[3 * m + 2]) return;  // position not merged at this level
  const int i = c - lo;
  const int k = w.kcnt[lo];
  if (i >= k) return;
  const double rho = w.rho[lo];
  const double irho = 1.0 / rho;
  const double* dd = w.dd + lo;
  const double* zz = w.zz + lo;
  int o;
  double lo_t, hi_t;
  if (i < k - 1) {
    const double mid = 0.5 * (dd[i + 1] - dd[i]);
    double f = 0.0;
    for (int j = lane; j < k; j += 64) f += zz[j] * zz[j] / ((dd[j] - dd[i]) - mid);
    f = wave_sum_d_dpp(f) + irho;
    if (f >= 0.0) {
      o = i;
      lo_t = 0.0;
      hi_t = mid;
    } else {
      o = i + 1;
      lo_t = -mid;
      hi_t = 0.0;
    }
  } else {
    double z2 = 0.0;
    for (int j = lane; j < k; j += 64) z2 += zz[j] * zz[j];
    o = i;
    lo_t = 0.0;
    hi_t = rho * wave_sum_d_dpp(z2);
  }
  const double dor = dd[o];
  double tau = 0.5 * (lo_t + hi_t);
  for (int it = 0; it < 64; ++it) {
    double psi = 0.0, phi = 0.0, dpsi = 0.0, dphi = 0.0;
    for (int j = lane; j < k; j += 64) {
      const double r = 1.0 / ((dd[j] - dor) - tau);
      const double t = zz[j] * zz[j] * r;
      if (j <= i) {
        psi += t;
        dpsi = fma(t, r, dpsi);
      } else {
        phi += t;
        dphi = fma(t, r, dphi);
      }
    }
    psi = wave_sum_d_dpp(psi);
    phi = wave_sum_d_dpp(phi);
    dpsi = wave_sum_d_dpp(dpsi);
    dphi = wave_sum_d_dpp(dphi);
    const double f = irho + psi + phi;
    const double erretm = 2.0 * kEps * (irho + fabs(psi) + fabs(phi));
    if (fabs(f) <= erretm || hi_t - lo_t <= 2.0 * kEps * fmax(fabs(lo_t), fabs(hi_t))) break;
    if (f < 0.0) lo_t = tau;
    else hi_t = tau;
    const double D1 = (dd[i] - dor) - tau;
    const double b1 = dpsi * D1 * D1;
    double cc = irho + (psi - b1 / D1);
    double eta = 0.0;
    bool ok = false;
    if (i < k - 1) {
      const double D2 = (dd[i + 1] - dor) - tau;
      const double b2 = dphi * D2 * D2;
      cc += phi - b2 / D2;
      const double B = cc * (D1 + D2) + b1 + b2;
      const double C = D1 * D2 * f;
      const double sq = sqrt(fmax(B * B - 4.0 * cc * C, 0.0));
      double r1 = 0.0, r2 = 0.0;
      int nr = 0;
      if (cc != 0.0) {
        const double q = 0.5 * (B + copysign(sq, B));
        if (q != 0.0) {
          r1 = q / cc;
          r2 = C / q;
          nr = 2;
        }
      } else if (B != 0.0) {
        r1 = C / B;
        nr = 1;
      }
      for (int q = 0; q < nr; ++q) {
        const double cand = q == 0 ? r1 : r2;
        const double nt = tau + cand;
        if (isfinite(nt) && nt > lo_t && nt < hi_t && (!ok || fabs(cand) < fabs(eta))) {
          eta = cand;
          ok = true;
        }
      }
    } else {
      cc += phi;
      if (cc != 0.0) {
        const double cand = D1 + b1 / cc;
        const double nt = tau + cand;
        if (isfinite(nt) && nt > lo_t && nt < hi_t) {
          eta = cand;
          ok = true;
        }
      }
    }
    if (!ok) {
      tau = 0.5 * (lo_t + hi_t);
    } else {
      tau += eta;
      if (fabs(eta) <= 2.0 * kEps * fabs(tau)) break;
    }
  }
  if (lane == 0) {
    w.org[lo + i] = o;
    w.tau[lo + i] = tau;
    D[lo + i] = dor + tau;
  }
}

// 3. zhat_j^2 = (lambda_j - d_j)/rho * prod_{i != j} (lambda_i - d_j)/(d_i - d_j)
__global__ __launch_bounds__(256) void dc_loewner_kernel(const int* __restrict__ mg, int nm, int n, DcWs w) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= n) return;
  const int m = find_merge(mg, nm, c);
  const int lo = mg[3 * m];
  if (c < lo || c >= mg[3 * m + 2]) return;
  const int j = c - lo;
  const int k = w.kcnt[lo];
  if (j >= k) return;
  const double* dd = w.dd + lo;
  const double dj = dd[j];
  double p = 1.0;
  for (int i = lane; i < k; i += 64) {
    const double num = (dd[w.org[lo + i]] - dj) + w.tau[lo + i];
    p *= i == j ? num / w.rho[lo] : num / (dd[i] - dj);
  }
  p = wave_prod_d(p);
  if (lane == 0) w.zh[lo + j] = copysign(sqrt(fmax(p, 0.0)), w.zz[lo + j]);
}

// 4. U[:, i] = zhat / (d - lambda_i), normalised (column-major k x k at lo * ldu)
__global__ __launch_bounds__(256) void dc_vectors_kernel(const int* __restrict__ mg, int nm, int n, DcWs w) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= n) return;
  const int m = find_merge(mg, nm, c);
  const int lo = mg[3 * m];
  if (c < lo || c >= mg[3 * m + 2]) return;
  const int i = c - lo;
  const int k = w.kcnt[lo];
  if (i >= k) return;
  const double* dd = w.dd + lo;
  const double dor = dd[w.org[lo + i]], tau = w.tau[lo + i];
  double* U = w.U + (long)lo * w.ldu + (long)i * k;
  double s2 = 0.0;
  for (int j = lane; j < k; j += 64) {
    const double u = w.zh[lo + j] / ((dd[j] - dor) - tau);
    U[j] = u;
    s2 = fma(u, u, s2);
  }
  const double inv = 1.0 / sqrt(wave_sum_d_dpp(s2));
  for (int j = lane; j < k; j += 64) U[j] *= inv;
}

// 5. Qn[lo.., lo + c] = sum_j Q[lo.., colsrc[j]] U[j, c] (c < k), Q[lo.., colsrc[c]] (c >= k)
constexpr int TM = 64, TK = 16;
__global__ __launch_bounds__(256) void dc_gemm_kernel(const double* __restrict__ Q, double* __restrict__ Qn, long ldq,
                                                      const int* __restrict__ mg, DcWs w) {
  __shared__ double sA[TK][TM + 1];
  __shared__ double sB[TK][TM + 1];
  const int lo = mg[3 * blockIdx.y], hi = mg[3 * blockIdx.y + 2];
  const int s = hi - lo;
  const int tiles = (s + TM - 1) / TM;
  if ((int)blockIdx.x >= tiles * tiles) return;
  const int r0 = (blockIdx.x % tiles) * TM, c0 = (blockIdx.x / tiles) * TM;
  const int k = w.kcnt[lo];
  const int tid = threadIdx.x;
  const int tr = (tid & 15) * 4, tc = (tid >> 4) * 4;  // 4 x 4 outputs per thread
  const int* cs = w.colsrc + lo;
  if (c0 >= k) {  // deflated columns only: copies
    for (int q = tid; q < TM * TM; q += 256) {
      const int r = r0 + (q & 63), c = c0 + (q >> 6);
      if (r < s && c < s) Qn[(long)(lo + c) * ldq + lo + r] = Q[(long)cs[c] * ldq + lo + r];
    }
    return;
  }
  double acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
  const double* U = w.U + (long)lo * w.ldu;
  for (int j0 = 0; j0 < k; j0 += TK) {
    for (int q = tid; q < TK * TM; q += 256) {
      {  // A: rows r0.. (consecutive threads, consecutive rows), inner j0.. (column gather)
        const int jj = q / TM, rr = q % TM;
        const int j = j0 + jj, r = r0 + rr;
        sA[jj][rr] = (j < k && r < s) ? Q[(long)cs[j] * ldq + lo + r] : 0.0;
      }
      {  // B: inner j0.. (consecutive threads along a column of U), columns c0..
        const int jj = q % TK, cc = q / TK;
        const int j = j0 + jj, c = c0 + cc;
        sB[jj][cc] = (j < k && c < k) ? U[(long)c * k + j] : 0.0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < TK; ++jj) {
      double a[4], b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[q] = sA[jj][tr + q];
        b[q] = sB[jj][tc + q];
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = fma(a[x], b[y], acc[x][y]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    const int c = c0 + tc + y;
    if (c >= s) continue;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int r = r0 + tr + x;
      if (r >= s) continue;
      Qn[(long)(lo + c) * ldq + lo + r] = c < k ? acc[x][y] : Q[(long)cs[c] * ldq + lo + r];
    }
  }
}

// the merged blocks of Qn back into Q (positions not merged at this level keep theirs)
__global__ __launch_bounds__(256) void dc_copyback_kernel(const double* __restrict__ Qn, double* __restrict__ Q, long ldq,
                                                          const int* __restrict__ mg) {
  const int lo = mg[3 * blockIdx.y], hi = mg[3 * blockIdx.y + 2];
  const int s = hi - lo;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < (long)s * s; q += gridDim.x * 256L) {
    const int r = (int)(q % s), c = (int)(q / s);
    Q[(long)(lo + c) * ldq + lo + r] = Qn[(long)(lo + c) * ldq + lo + r];
  }
}

size_t prep_lds(int smax) { return (size_t)smax * (2 * sizeof(double) + 3 * sizeof(int)); }

}  // namespace

HARP_EXPORT int harp_dc_max_n() { return kMaxN; }

// doubles of the workspace for size n: Qb n^2, U n^2, dd/zz/tau/zh/rho/rotc/rots 7 n, sort
// scratch 3 n; ints (colsrc/org/kcnt/rotp/rotq 5 n) follow as 3 n doubles
HARP_EXPORT long harp_dc_ws_doubles(int n) { return 2L * n * n + 10L * n + 3L * n + 16; }

// Eigen-decomposition of the symmetric tridiagonal (dmod, e): dmod is the diagonal with
// |e[mid - 1]| already subtracted at d[mid - 1] and d[mid] for every merge (harp_amd/ops/eig.py),
// overwritten by the (unsorted) eigenvalues. Q: n x n column-major, = I on entry, holds the
// eigenvectors on exit (columns in the order of dmod). merges: (lo, mid, hi) int32 triples
// of all levels, bottom level first; level_off[l] .. level_off[l + 1]: level l's merges
// (host array), level_smax[l]: its largest block. ws: harp_dc_ws_doubles(n) doubles, zeroed.
HARP_EXPORT int harp_dc_tridiag(double* dmod, const double* e, int n, double* Q, const int* merges,
                                const int* level_off, const int* level_smax, int nlevels, double* ws, hipStream_t st) {
  if (n < 1 || n > kMaxN || !dmod || !Q || !ws || (nlevels > 0 && (!merges || !level_off || !level_smax)))
    return HARP_EBADARG;
  const long nn = (long)n * n;
  double* Qb = ws;
  DcWs w;
  w.U = ws + nn;
  double* p = ws + 2 * nn;
  w.dd = p;
  w.zz = p + n;
  w.tau = p + 2 * n;
  w.zh = p + 3 * n;
  w.rho = p + 4 * n;
  w.rotc = p + 5 * n;
  w.rots = p + 6 * n;
  w.sortbuf = p + 7 * n;
  int* ip = (int*)(p + 10 * n);
  w.colsrc = ip;
  w.org = ip + n;
  w.kcnt = ip + 2 * n;
  w.rotp = ip + 3 * n;
  w.rotq = ip + 4 * n;
  for (int l = 0; l < nlevels; ++l) {
    const int m0 = level_off[l], nm = level_off[l + 1] - m0;
    const int smax = level_smax[l];
    if (nm <= 0) continue;
    if (smax < 2 || smax > n) return HARP_EBADARG;
    w.ldu = smax;
    const int* mg = merges + 3 * m0;
    const size_t lds = prep_lds(smax);
    // set per launch (a host-side attribute call, no process-wide cache to race on)
    if (lds > 65536 && hipFuncSetAttribute((const void*)dc_prep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds) != hipSuccess)
      return HARP_ELAUNCH;
    const int threads = smax >= 512 ? 1024 : smax >= 128 ? 256 : 64;
    dc_prep_kernel<<<dim3((unsigned)nm), dim3(threads), lds, st>>>(Q, n, dmod, e, mg, w);
    const unsigned wg = (unsigned)((n + 3) / 4);
    dc_secular_kernel<<<dim3(wg), dim3(256), 0, st>>>(mg, nm, n, dmod, w);
    dc_loewner_kernel<<<dim3(wg), dim3(256), 0, st>>>(mg, nm, n, w);
    dc_vectors_kernel<<<dim3(wg), dim3(256), 0, st>>>(mg, nm, n, w);
    const int tiles = (smax + TM - 1) / TM;
    dc_gemm_kernel<<<dim3((unsigned)(tiles * tiles), (unsigned)nm), dim3(256), 0, st>>>(Q, Qb, n, mg, w);
    const long per = (long)smax * smax;
    const unsigned cb = (unsigned)((per + 256 * 4 - 1) / (256 * 4));
    dc_copyback_kernel<<<dim3(cb, (unsigned)nm), dim3(256), 0, st>>>(Qb, Q, n, mg);
    const int s_ = harp_launch_status();
    if (s_ != HARP_OK) return s_;
  }
  return harp_launch_status();
}
