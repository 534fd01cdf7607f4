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
//     LDS, fp64 MFMA, each half's rows over that half's columns only), deflated columns
//     copied; Q ping-pongs between two buffers.
//  6. dc_wave_merge_kernel: levels of merges <= 64 rows, steps 1-5 in one wave per merge.
// Eigenvalues are carried as (origin pole, tau) while the vectors are formed, so every
// difference d_j - lambda_i is computed as (d_j - d_o) - tau without cancellation.
#include <stdlib.h>

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

// workgroup barrier for LDS traffic only (__syncthreads() also drains outstanding global loads)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// LDS ordering within one wave (its lanes run in lockstep: no barrier)
__device__ __forceinline__ void lds_sync_wave() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
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

// diagnostic: thread 0 of the last launch's first merge records s_memtime at its phase ends
// (harp_dc_prep_stamps)
__device__ long long g_prep_t[10];
#define PREP_MARK(i) \
  do {                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_prep_t[i] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

// phase stamps of block 0 of the last dc_wave_merge_kernel launch (harp_dc_wave_stamps)
__device__ long long g_wave_t[8];
__device__ int g_wave_it;
#define WAVE_MARK(i) \
  do {                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_wave_t[i] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

struct DcWs {
  double *dd, *zz, *tau, *zh, *rho, *U, *rotc, *rots, *sortbuf;
  int *colsrc, *org, *kcnt, *rotp, *rotq;
  // kept secular positions whose Q column has entries in the upper (lower) half of the
  // merge: jl / jr (ascending, at lo), counts kl / kr at [lo]. A column is one-sided unless
  // a deflation rotation mixed it with a column of the other half.
  int *jl, *jr, *kl, *kr;
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
  int* hm = defl + s;              // [s] halves holding the column's entries (bit 0 upper, bit 1 lower)
  __shared__ double red[16];
  __shared__ int s_k, s_nd, s_nrot, s_serial;
  __shared__ unsigned long long passm[kMaxN / 64];
  const int tid = threadIdx.x, T = blockDim.x;
  PREP_MARK(0);
  const double beta = e[mid - 1];
  const double sgn = beta < 0.0 ? -1.0 : 1.0;
  // raw values: left block's last row, right block's first row (sign of beta folded in)
  for (int j = tid; j < s; j += T) {
    sd[j] = D[lo + j];
    sz[j] = j < s1 ? Q[(long)(lo + j) * ldq + (mid - 1)] : sgn * Q[(long)(lo + j) * ldq + mid];
  }
  __syncthreads();
  PREP_MARK(1);
  // sort (value, index) pairs ascending, ties by index. Each half is the output of a child
  // merge: its kept roots ascending, then its deflated values ascending -- at most one descent
  // per half, so the input is at most four sorted runs and every element's sorted position is
  // its offset in its run plus a binary-search count in each other run (a few dependent LDS
  // reads per thread). Any other input (not produced here) takes the bitonic network.
  __shared__ int s_nb[2], s_pb[2];
  if (tid < 2) {
    s_nb[tid] = 0;
    s_pb[tid] = tid == 0 ? s1 : s;
  }
  __syncthreads();
  for (int j = tid; j < s; j += T) {
    if (j != 0 && j != s1 && sd[j] < sd[j - 1]) {
      const int h = j >= s1;
      atomicAdd(&s_nb[h], 1);
      s_pb[h] = j;
    }
  }
  __syncthreads();
  if (s_nb[0] <= 1 && s_nb[1] <= 1) {
    const int rb[5] = {0, s_pb[0], s1, s_pb[1], s};
    for (int j = tid; j < s; j += T) {
      const double v = sd[j];
      int r = 0;
      while (j >= rb[r + 1]) ++r;
      int pos = j - rb[r];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q == r) continue;
        // runs before r hold smaller indices (a tie counts), runs after r larger ones (it does not)
        int a = rb[q], b = rb[q + 1];
        const int base = a;
        while (a < b) {
          const int m = (a + b) >> 1;
          const double x = sd[m];
          if (x < v || (q < r && x == v)) a = m + 1;
          else b = m;
        }
        pos += a - base;
      }
      keep[pos] = __double2loint(v);
      defl[pos] = __double2hiint(v);
      hm[pos] = j;
    }
    __syncthreads();
    for (int j = tid; j < s; j += T) {
      sd[j] = __hiloint2double(defl[j], keep[j]);
      src[j] = hm[j];
    }
    __syncthreads();
  } else {
    // bitonic network in the all-ascending (flip) form, in place in LDS: a comparator always
    // keeps the smaller key at the lower position, so the positions past s act as +inf and
    // are never touched (no padding storage)
    for (int j = tid; j < s; j += T) src[j] = j;
    __syncthreads();
    int P2 = 1;
    while (P2 < s) P2 <<= 1;
    auto cmpswap = [&](int i, int l) {
      if (l >= s) return;
      const double a = sd[i], b = sd[l];
      const int ai = src[i], bi = src[l];
      if (b < a || (b == a && bi < ai)) {
        sd[i] = b;
        sd[l] = a;
        src[i] = bi;
        src[l] = ai;
      }
    };
    for (int lp = 1; (1 << lp) <= P2; ++lp) {  // blocks of p = 2^lp (shifts, no integer divides)
      const int hm1 = (1 << (lp - 1)) - 1;
      for (int c = tid; c < (P2 >> 1); c += T) {  // flip: i <-> mirror within the block of p
        const int base = (c >> (lp - 1)) << lp, o = c & hm1;
        cmpswap(base + o, base + (1 << lp) - 1 - o);
      }
      lds_sync();
      for (int lq = lp - 2; lq >= 0; --lq) {  // half-cleaners at distance q = 2^lq
        const int qm1 = (1 << lq) - 1;
        for (int c = tid; c < (P2 >> 1); c += T) {
          const int i = ((c >> lq) << (lq + 1)) + (c & qm1);
          cmpswap(i, i + (1 << lq));
        }
        lds_sync();
      }
    }
  }
  PREP_MARK(2);
  // z in the sorted order, through keep / defl (free until the deflation) as 32-bit halves
  for (int j = tid; j < s; j += T) {
    const double z = sz[src[j]];
    keep[j] = __double2loint(z);
    defl[j] = __double2hiint(z);
  }
  lds_sync();
  for (int j = tid; j < s; j += T) {
    sz[j] = __hiloint2double(defl[j], keep[j]);
    hm[j] = src[j] < s1 ? 1 : 2;
  }
  __syncthreads();
  PREP_MARK(3);
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
  PREP_MARK(4);
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
  PREP_MARK(5);
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
  } else {
    // the dependent walk (LAPACK dlaed2 order): a rotated pair keeps d_pj c^2 + d_j s^2 at
    // pj (deflated) and continues with j. A pair whose first member was not rotated into
    // sees its original values, so its test is precomputed in parallel (passm bits); the
    // one-thread walk jumps between set bits and evaluates only inside rotation chains.
    if (tid < 64) {  // survivors (large z) in order -> keep[0 .. ns)
      int kk = 0;
      for (int b = 0; b < s; b += 64) {
        const int j = b + tid;
        const bool sv = j < s && rho * fabs(sz[j]) > tol;
        const unsigned long long mk = __ballot(sv);
        if (sv) keep[kk + __popcll(mk & ((1ull << tid) - 1ull))] = j;
        kk += __popcll(mk);
      }
      if (tid == 0) s_k = kk;
    }
    __syncthreads();
    const int ns = s_k;
    for (int b = (tid >> 6) * 64; b < ns; b += T) {  // one 64-pair word per wave
      const int i = b + (tid & 63);
      bool ps = false;
      if (i >= 1 && i < ns) {
        const int pj = keep[i - 1], j = keep[i];
        const double ss = sz[pj], cc = sz[j];
        const double t2 = hypot(cc, ss);
        ps = fabs((sd[j] - sd[pj]) * (cc / t2) * (-ss / t2)) <= tol;
      }
      const unsigned long long m = __ballot(ps);
      if ((tid & 63) == 0) passm[b >> 6] = m;
    }
    __syncthreads();
    if (tid == 0) {
      const int nw = (ns + 63) >> 6;
      int nr = 0, i = 1;
      bool chain = false;  // keep[i - 1] was rotated into at the previous step
      while (i < ns) {
        if (!chain) {  // next precomputed rotation
          int wi = i >> 6;
          unsigned long long m = passm[wi] & (~0ull << (i & 63));
          while (!m && ++wi < nw) m = passm[wi];
          if (!m) break;
          i = (wi << 6) + __builtin_ctzll(m);
          if (i >= ns) break;
        }
        const int pj = keep[i - 1], j = keep[i];
        double ss = sz[pj], cc = sz[j];
        const double t2 = hypot(cc, ss);
        const double t = sd[j] - sd[pj];
        cc /= t2;
        ss = -ss / t2;
        if (fabs(t * cc * ss) <= tol) {
          sz[j] = t2;
          sz[pj] = 0.0;
          hm[j] |= hm[pj];
          hm[pj] |= 4;  // rotated away: deflated
          w.rotp[lo + nr] = lo + src[pj];
          w.rotq[lo + nr] = lo + src[j];
          w.rotc[lo + nr] = cc;
          w.rots[lo + nr] = ss;
          ++nr;
          const double tt = sd[pj] * cc * cc + sd[j] * ss * ss;
          sd[j] = sd[pj] * ss * ss + sd[j] * cc * cc;
          sd[pj] = tt;
          chain = true;
        } else {
          chain = false;
        }
        ++i;
      }
      s_nrot = nr;
    }
    __syncthreads();
    if (tid < 64) {  // keep = survivors not rotated away (in place), defl = the rest in j order
      int kk = 0, nd = 0;
      const unsigned long long below = (1ull << tid) - 1ull;
      for (int b = 0; b < ns; b += 64) {
        const int i = b + tid;
        const int j = i < ns ? keep[i] : 0;
        const bool kp = i < ns && !(hm[j] & 4);
        const unsigned long long mk = __ballot(kp);
        if (kp) keep[kk + __popcll(mk & below)] = j;
        kk += __popcll(mk);
      }
      for (int b = 0; b < s; b += 64) {
        const int j = b + tid;
        const bool dj = j < s && (rho * fabs(sz[j]) <= tol || (hm[j] & 4));
        const unsigned long long md = __ballot(dj);
        if (dj) defl[nd + __popcll(md & below)] = j;
        nd += __popcll(md);
      }
      if (tid == 0) {
        s_k = kk;
        s_nd = nd;
      }
    }
  }
  __threadfence_block();
  __syncthreads();
  PREP_MARK(6);
  const int k = s_k, nd = s_nd, nrot = s_nrot;
  // deflation rotations on Q's columns, in order (each row independent). A column takes part
  // in at most two rotations, consecutive ones (y of step q = x of step q + 1, a chain), so
  // the chained value stays in a register and every other operand can be loaded ahead: the
  // loads of a batch of 16 rotations are in flight together (one round trip per batch, not
  // one per rotation).
  if (nrot) {
    constexpr int kRB = 16;
    for (int r = lo + tid; r < hi; r += T) {
      double carry = 0.0;
      int cy = -1;
      for (int q0 = 0; q0 < nrot; q0 += kRB) {
        double xv[kRB], yv[kRB];
#pragma unroll
        for (int u = 0; u < kRB; ++u) {
          if (q0 + u < nrot) {
            xv[u] = Q[(long)w.rotp[lo + q0 + u] * ldq + r];
            yv[u] = Q[(long)w.rotq[lo + q0 + u] * ldq + r];
          }
        }
#pragma unroll
        for (int u = 0; u < kRB; ++u) {
          const int q = q0 + u;
          if (q < nrot) {
            const int xc = w.rotp[lo + q], yc = w.rotq[lo + q];
            const double c = w.rotc[lo + q], sn = w.rots[lo + q];
            const double xo = xc == cy ? carry : xv[u];
            Q[(long)xc * ldq + r] = c * xo + sn * yv[u];
            carry = c * yv[u] - sn * xo;
            cy = yc;
            if (!(q + 1 < nrot && w.rotp[lo + q + 1] == yc)) Q[(long)yc * ldq + r] = carry;
          }
        }
      }
    }
  }
  PREP_MARK(7);
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
  if (tid < 64) {  // one-sided lists, in kept order (ballots)
    int nl = 0, nr2 = 0;
    const unsigned long long below = (1ull << tid) - 1ull;
    for (int b = 0; b < k; b += 64) {
      const int i = b + tid;
      const int h = i < k ? hm[keep[i]] : 0;
      const unsigned long long ml = __ballot(h & 1), mr = __ballot(h & 2);
      if (h & 1) w.jl[lo + nl + __popcll(ml & below)] = i;
      if (h & 2) w.jr[lo + nr2 + __popcll(mr & below)] = i;
      nl += __popcll(ml);
      nr2 += __popcll(mr);
    }
    if (tid == 0) {
      w.kl[lo] = nl;
      w.kr[lo] = nr2;
    }
  }
  PREP_MARK(8);
  if (tid == 0) {
    w.kcnt[lo] = k;
    w.rho[lo] = rho;
  }
}

// ---------------------------------------------------------------------------------------
// 2. secular roots: one wave per root; 4 roots per 256-thread workgroup over positions.
// For k <= 64 kSecR the wave keeps d_j - d_o and z_j^2 in registers for the whole solve
// (the iterations re-read them from L2 otherwise) and forms 1 / (d_j - d_o - tau) with
// v_rcp_f64 + two Newton steps instead of the IEEE divide chain.
constexpr int kSecR = 16;
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}

// Initial tau of root i < k - 1 (LAPACK dlaed4's two-pole start): f0 is the secular function
// at the gap's midpoint, c = f0 without the two nearest poles' terms, and the root of
// c + z_i^2 / (d_i - l) + z_{i+1}^2 / (d_{i+1} - l) in the half f0's sign selects (origin d_i:
// tau in (0, mid); origin d_{i+1}: tau in (-mid, 0)); the bracket's midpoint if that is not
// strictly inside it. Saves the first iterations of the rational steps from the midpoint.
__device__ __forceinline__ double secular_init(double f0, double mid, double zi2, double zj2, bool left, double lo_t,
                                               double hi_t) {
  const double del = 2.0 * mid;
  const double c = f0 + (zi2 - zj2) / mid;
  double tau;
  if (left) {
    const double a = c * del + zi2 + zj2, b = zi2 * del;
    const double sq = sqrt(fabs(a * a - 4.0 * b * c));
    tau = a > 0.0 ? 2.0 * b / (a + sq) : (a - sq) / (2.0 * c);
  } else {
    const double a = c * del - zi2 - zj2, b = zj2 * del;
    const double sq = sqrt(fabs(a * a + 4.0 * b * c));
    tau = a < 0.0 ? 2.0 * b / (a - sq) : -(a + sq) / (2.0 * c);
  }
  return (isfinite(tau) && tau > lo_t && tau < hi_t) ? tau : 0.5 * (lo_t + hi_t);
}

template <bool kReg>
__device__ __forceinline__ void secular_solve(int i, int k, int lane, double rho, const double* __restrict__ dd,
                                              const double* __restrict__ zz, int& o_out, double& tau_out) {
  const double irho = 1.0 / rho;
  double dr[kReg ? kSecR : 1], z2r[kReg ? kSecR : 1];
  if (kReg) {
#pragma unroll
    for (int q = 0; q < kSecR; ++q) {
      const int j = lane + 64 * q;
      dr[q] = j < k ? dd[j] : 0.0;
      z2r[q] = j < k ? zz[j] * zz[j] : 0.0;
    }
  }
  int o;
  double lo_t, hi_t, tau0 = 0.0;
  bool init = false;
  const double ddi = dd[i];
  if (i < k - 1) {
    const double mid = 0.5 * (dd[i + 1] - ddi);
    double f = 0.0;
    if (kReg) {
#pragma unroll
      for (int q = 0; q < kSecR; ++q)
        if (lane + 64 * q < k) f += z2r[q] / ((dr[q] - ddi) - mid);
    } else {
      for (int j = lane; j < k; j += 64) f += zz[j] * zz[j] / ((dd[j] - ddi) - mid);
    }
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
    tau0 = secular_init(f, mid, zz[i] * zz[i], zz[i + 1] * zz[i + 1], f >= 0.0, lo_t, hi_t);
    init = true;
  } else {
    double z2 = 0.0;
    if (kReg) {
#pragma unroll
      for (int q = 0; q < kSecR; ++q) z2 += z2r[q];
    } else {
      for (int j = lane; j < k; j += 64) z2 += zz[j] * zz[j];
    }
    o = i;
    lo_t = 0.0;
    hi_t = rho * wave_sum_d_dpp(z2);
  }
  const double dor = dd[o];
  if (kReg) {
#pragma unroll
    for (int q = 0; q < kSecR; ++q) dr[q] -= dor;
  }
  const double D1o = ddi - dor, D2o = i < k - 1 ? dd[i + 1] - dor : 0.0;
  double tau = init ? tau0 : 0.5 * (lo_t + hi_t);
  for (int it = 0; it < 64; ++it) {
    double psi = 0.0, phi = 0.0, dpsi = 0.0, dphi = 0.0;
    if (kReg) {
#pragma unroll
      for (int q = 0; q < kSecR; ++q) {
        const int j = lane + 64 * q;
        if (j < k) {
          const double r = rcp_nr(dr[q] - tau);
          const double t = z2r[q] * r;
          if (j <= i) {
            psi += t;
            dpsi = fma(t, r, dpsi);
          } else {
            phi += t;
            dphi = fma(t, r, dphi);
          }
        }
      }
    } else {
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
    const double D1 = D1o - tau;
    const double b1 = dpsi * D1 * D1;
    double cc = irho + (psi - b1 / D1);
    double eta = 0.0;
    bool ok = false;
    if (i < k - 1) {
      const double D2 = D2o - tau;
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
  o_out = o;
  tau_out = tau;
}

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
  int o;
  double tau;
  if (k <= 64 * kSecR)
    secular_solve<true>(i, k, lane, w.rho[lo], w.dd + lo, w.zz + lo, o, tau);
  else
    secular_solve<false>(i, k, lane, w.rho[lo], w.dd + lo, w.zz + lo, o, tau);
  if (lane == 0) {
    w.org[lo + i] = o;
    w.tau[lo + i] = tau;
    D[lo + i] = w.dd[lo + o] + tau;
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

// 5. Qn[lo.., lo + c] = sum_j Q[lo.., colsrc[j]] U[j, c] (c < k), Q[lo.., colsrc[c]] (c >= k).
// Q is block diagonal before the merge: a tile of upper-half rows sums only over the kept
// columns with upper entries (jl), a lower tile over jr -- about half the products skipped,
// every skipped one an exact zero (same sums in the same order).
// fp64 MFMA (v_mfma_f64_16x16x4_f64) on 64 x 64 output tiles, 4 waves of 32 x 32. The product
// is formed transposed, Qn^T = U^T Q^T, so the accumulator's lane index runs along Q's rows
// and the stores are coalesced. Row tiles start at 0 and at the split s1 (no tile straddles
// the two halves, so every tile sums over its own half's list only). Per slab of TK inner
// indices every thread loads 16 + 16 values one slab ahead into registers (the gathers'
// index lists live in LDS), so the global round trip overlaps the MFMAs of the current slab.
// LDS: sA[k][r] rows of kPA doubles (2-way banks for the B-operand reads), sBt[c][k] rows of
// kPB (the A-operand reads; the transposed stores stay contiguous).
constexpr int TM = 64, TK = 64, kFetch = TK * TM / 256, kPA = TM + 16, kPB = TK + 4;
constexpr size_t kGemmTileLds = sizeof(double) * (size_t)(TK * kPA + TM * kPB);
typedef double dc_d4 __attribute__((ext_vector_type(4)));
typedef double dc_d2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void dc_gemm_kernel(const double* __restrict__ Q, double* __restrict__ Qn, long ldq,
                                                      const int* __restrict__ mg, DcWs w, int rtm) {
  extern __shared__ double gsm[];
  double* sA = gsm;              // [TK][kPA]: Q[rows r0.., list entry j0 + k]
  double* sBt = gsm + TK * kPA;  // [TM][kPB]: U[list entry j0 + k, column c0 + c]
  int* sidx = (int*)(sBt + TM * kPB);  // [smax] Q column, [smax] U row of list entry t
  const int lo = mg[3 * blockIdx.y], mid = mg[3 * blockIdx.y + 1], hi = mg[3 * blockIdx.y + 2];
  const int s = hi - lo, s1 = mid - lo;
  const int nu = (s1 + TM - 1) / TM, rtiles = nu + (s - s1 + TM - 1) / TM, ctiles = (s + TM - 1) / TM;
  const int rt = (int)blockIdx.x % rtm, ct = (int)blockIdx.x / rtm;
  if (rt >= rtiles || ct >= ctiles) return;
  const bool upper = rt < nu;
  const int r0 = upper ? rt * TM : s1 + (rt - nu) * TM;
  const int rend = upper ? (r0 + TM < s1 ? r0 + TM : s1) : (r0 + TM < s ? r0 + TM : s);
  const int c0 = ct * TM;
  const int k = w.kcnt[lo];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int* cs = w.colsrc + lo;
  if (c0 >= k) {  // deflated columns only: copies
    for (int q = tid; q < TM * TM; q += 256) {
      const int r = r0 + (q & 63), c = c0 + (q >> 6);
      if (r < rend && c < s) Qn[(long)(lo + c) * ldq + lo + r] = Q[(long)cs[c] * ldq + lo + r];
    }
    return;
  }
  const int* jlist = upper ? w.jl + lo : w.jr + lo;
  const int kk = upper ? w.kl[lo] : w.kr[lo];
  int* sJ = sidx;
  int* sU = sidx + s;
  for (int t = tid; t < kk; t += 256) {
    const int j = jlist[t];
    sU[t] = j;
    sJ[t] = cs[j];
  }
  __syncthreads();
  const double* U = w.U + (long)lo * w.ldu;
  double ra[kFetch], rb[kFetch];
  auto fetch = [&](int j0) {
#pragma unroll
    for (int i = 0; i < kFetch; ++i) {
      const int q = tid + 256 * i;
      {  // A: rows r0.. (consecutive threads, consecutive rows), inner j0.. (column gather)
        const int t = j0 + q / TM, r = r0 + q % TM;
        ra[i] = (t < kk && r < rend) ? Q[(long)sJ[t] * ldq + lo + r] : 0.0;
      }
      {  // B: inner j0.. (consecutive threads along a column of U), columns c0..
        const int t = j0 + q % TK, c = c0 + q / TK;
        rb[i] = (t < kk && c < k) ? U[(long)c * k + sU[t]] : 0.0;
      }
    }
  };
  dc_d4 acc[2][2];
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = dc_d4{0.0, 0.0, 0.0, 0.0};
  const int wr = wv & 1, wc = wv >> 1;  // this wave's 32 x 32: rows wr 32.., columns wc 32..
  const int l15 = lane & 15, l4 = lane >> 4;
  fetch(0);
  for (int j0 = 0; j0 < kk; j0 += TK) {
#pragma unroll
    for (int i = 0; i < kFetch; ++i) {
      const int q = tid + 256 * i;
      sA[(q / TM) * kPA + q % TM] = ra[i];
      sBt[(q / TK) * kPB + q % TK] = rb[i];
    }
    __syncthreads();
    if (j0 + TK < kk) fetch(j0 + TK);  // in flight under this slab's MFMAs
#pragma unroll
    for (int kq = 0; kq < TK / 4; ++kq) {
      const int kb = 4 * kq + l4;
      double av[2], bv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        av[h] = sBt[(wc * 32 + 16 * h + l15) * kPB + kb];  // A' = U^T: row c, inner k
        bv[h] = sA[kb * kPA + wr * 32 + 16 * h + l15];      // B' = Q^T: inner k, column r
      }
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[bi], bv[bj], acc[bi][bj], 0, 0, 0);
    }
    __syncthreads();
  }
  // D[i][j]: i = column c (row of the accumulator tile) = l4 + 4 reg, j = row r = lane & 15
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = c0 + wc * 32 + 16 * bi + l4 + 4 * g;
        const int r = r0 + wr * 32 + 16 * bj + l15;
        if (c < s && r < rend) Qn[(long)(lo + c) * ldq + lo + r] = c < k ? acc[bi][bj][g] : Q[(long)cs[c] * ldq + lo + r];
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

// ---------------------------------------------------------------------------------------
// 6. Levels whose merges have at most kWaveMerge rows: ONE wave per merge does all of steps
// 1-5 in a single launch (lane = row / sorted position): the merge's block of Q staged in LDS,
// register bitonic sort over the wave, deflation by ballots (+ the one-lane walk when a
// rotation applies), one LANE per secular root (sequential sums over k <= 64), Loewner z-hat,
// U in LDS, and the block product written straight back to Q (no Qb round trip). The six
// launches of the level kernels cost ~50 us per level at these sizes (dc_kernels_after.txt)
// for work of a few microseconds.
constexpr int kWaveMerge = 64, kWaveMergeDefault = 64;


__device__ __forceinline__ double quad_sum_d(double v) {
  v += dpp_mov_d<0xB1>(v);  // quad_perm [1,0,3,2]
  return v + dpp_mov_d<0x4E>(v);  // quad_perm [2,3,0,1]: the same bits in all four lanes
}
__device__ __forceinline__ double quad_prod_d(double v) {
  v *= dpp_mov_d<0xB1>(v);
  return v * dpp_mov_d<0x4E>(v);
}

// Root i of the secular equation by the four lanes of a quad (part = lane & 3 holds the terms
// j = part + 4 q, q < NT, in registers); the quad's sums are bit-identical in its lanes, so
// its control flow is uniform. Same iteration as secular_solve.
template <int NT>
__device__ int secular_quad(int i, int part, int k, double rho, const double* dd, const double* zz, int& o_out,
                            double& tau_out) {
  const double irho = 1.0 / rho;
  double dr[NT], z2r[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const int j = part + 4 * q;
    dr[q] = j < k ? dd[j] : 1e300;  // absent terms: z^2 = 0 over a finite pole, an exact 0
    z2r[q] = j < k ? zz[j] * zz[j] : 0.0;
  }
  int o;
  double lo_t, hi_t, tau0 = 0.0;
  bool init = false;
  const double ddi = dd[i];
  if (i < k - 1) {
    const double mid = 0.5 * (dd[i + 1] - ddi);
    double f = 0.0;
#pragma unroll
    for (int q = 0; q < NT; ++q) f += z2r[q] / ((dr[q] - ddi) - mid);
    f = quad_sum_d(f) + irho;
    if (f >= 0.0) {
      o = i;
      lo_t = 0.0;
      hi_t = mid;
    } else {
      o = i + 1;
      lo_t = -mid;
      hi_t = 0.0;
    }
    tau0 = secular_init(f, mid, zz[i] * zz[i], zz[i + 1] * zz[i + 1], f >= 0.0, lo_t, hi_t);
    init = true;
  } else {
    double z2 = 0.0;
#pragma unroll
    for (int q = 0; q < NT; ++q) z2 += z2r[q];
    o = i;
    lo_t = 0.0;
    hi_t = rho * quad_sum_d(z2);
  }
  const double dor = dd[o];
#pragma unroll
  for (int q = 0; q < NT; ++q) dr[q] -= dor;
  const double D1o = ddi - dor, D2o = i < k - 1 ? dd[i + 1] - dor : 0.0;
  double tau = init ? tau0 : 0.5 * (lo_t + hi_t);
  int it = 0;
  for (; it < 64; ++it) {
    double psi = 0.0, phi = 0.0, dpsi = 0.0, dphi = 0.0;
#pragma unroll
    for (int q = 0; q < NT; ++q) {  // branch-free: the split j <= i as selects
      const bool left = part + 4 * q <= i;
      const double r = rcp_nr(dr[q] - tau);
      const double t = z2r[q] * r;
      const double tl = left ? t : 0.0, tg = left ? 0.0 : t;
      psi += tl;
      dpsi = fma(tl, r, dpsi);
      phi += tg;
      dphi = fma(tg, r, dphi);
    }
    psi = quad_sum_d(psi);
    phi = quad_sum_d(phi);
    dpsi = quad_sum_d(dpsi);
    dphi = quad_sum_d(dphi);
    const double f = irho + psi + phi;
    const double erretm = 2.0 * kEps * (irho + fabs(psi) + fabs(phi));
    if (fabs(f) <= erretm || hi_t - lo_t <= 2.0 * kEps * fmax(fabs(lo_t), fabs(hi_t))) break;
    if (f < 0.0) lo_t = tau;
    else hi_t = tau;
    const double D1 = D1o - tau;
    const double b1 = dpsi * D1 * D1;
    double cc = irho + (psi - b1 / D1);
    double eta = 0.0;
    bool ok = false;
    if (i < k - 1) {
      const double D2 = D2o - tau;
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
#pragma unroll
      for (int q = 0; q < 2; ++q) {  // straight-line: candidate q valid when q < nr
        const double cand = q == 0 ? r1 : r2;
        const double nt = tau + cand;
        const bool good = q < nr && isfinite(nt) && nt > lo_t && nt < hi_t && (!ok || fabs(cand) < fabs(eta));
        eta = good ? cand : eta;
        ok = ok || good;
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
  o_out = o;
  tau_out = tau;
  return it;
}

template <int NC>
__global__ __launch_bounds__(256) void dc_wave_merge_kernel(double* __restrict__ Q, long ldq, double* __restrict__ D,
                                                             const double* __restrict__ e, const int* __restrict__ mg,
                                                             int S) {
  constexpr int NT = NC / 4;  // secular / Loewner / U terms per lane (quad per root), GEMM columns per wave
  extern __shared__ double sm[];
  double* Ut = sm;            // [S][NC] U row-major: Ut[j NC + c] = U(j, c), NC >= S a power of 2
  double* sQ = Ut + S * NC;   // [S][S] the merge's block of Q: sQ[c S + r] = Q(lo + r, lo + c)
  double* sd = sQ + S * S;    // [64] each: sorted d, z (walk scratch), secular d, z, tau, z-hat,
  double* sz = sd + 64;       // rotation cosines and sines
  double* dd = sz + 64;
  double* zz = dd + 64;
  double* st = zz + 64;
  double* zh = st + 64;
  double* rc = zh + 64;
  double* rsn = rc + 64;
  int* keep = (int*)(rsn + 64);  // [64] each: survivors, halves bits, secular origin, block
  int* hm = keep + 64;           // column of secular / deflated position, rotation columns
  int* org = hm + 64;
  int* cs = org + 64;
  int* rp = cs + 64;
  int* rq = rp + 64;
  __shared__ int s_nrot, s_k;
  __shared__ double s_rho;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lo = mg[3 * blockIdx.x], mid = mg[3 * blockIdx.x + 1], hi = mg[3 * blockIdx.x + 2];
  const int s = hi - lo, s1 = mid - lo;
  const unsigned long long below = (1ull << lane) - 1ull;
  const double beta = e[mid - 1];
  const double sgn = beta < 0.0 ? -1.0 : 1.0;
  WAVE_MARK(0);
  {  // stage the block: up to 16 loads in flight per thread (one round trip for s <= 64)
    const int tot = s * s;
    for (int q0 = 0; q0 < tot; q0 += 256 * 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int q = q0 + 256 * u + tid;
        v[u] = q < tot ? Q[(long)(lo + q / s) * ldq + lo + q % s] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int q = q0 + 256 * u + tid;
        if (q < tot) sQ[(q / s) * S + q % s] = v[u];
      }
    }
  }
  __syncthreads();
  WAVE_MARK(1);
  if (wv == 0) {  // sort, deflation, rotations: wave 0, lane = sorted position
    // z: the left block's last row, the right block's first row (sign of beta folded in)
    double zr = 0.0, key = __builtin_inf();
    int id = lane;
    if (lane < s) {
      zr = lane < s1 ? sQ[lane * S + s1 - 1] : sgn * sQ[lane * S + s1];
      key = D[lo + lane];
    }
    // bitonic sort of (d, index) across the wave, in registers; lanes >= s are +inf
    const int p2 = s <= 2 ? 2 : 1 << (32 - __builtin_clz(s - 1));  // lanes >= p2 are already in place
    for (int kk = 2; kk <= p2; kk <<= 1) {
      for (int j = kk >> 1; j > 0; j >>= 1) {
        const double ok = __shfl_xor(key, j);
        const int oi = __shfl_xor(id, j);
        const bool oless = ok < key || (ok == key && oi < id);
        if ((((lane & j) == 0) == ((lane & kk) == 0)) ? oless : !oless) {
          key = ok;
          id = oi;
        }
      }
    }
    double dv = key, zv = __shfl(zr, id);
    const int srcv = id;
    int hv = id < s1 ? 1 : 2;
    const bool in = lane < s;
    const double nz2 = wave_sum_d_dpp(in ? zv * zv : 0.0);
    const double dmax = wave_max_d(in ? fabs(dv) : 0.0);
    const double rho = fabs(beta) * nz2;
    zv *= nz2 > 0.0 ? 1.0 / sqrt(nz2) : 0.0;
    const double zmax = wave_max_d(in ? fabs(zv) : 0.0);
    const double tol = 8.0 * kEps * fmax(dmax, rho * zmax);
    int nrot = 0;
    if (rho > 0.0) {
      // does a pair of consecutive survivors pass the rotation test (the level kernels' pre-check)?
      const bool sv = in && rho * fabs(zv) > tol;
      const unsigned long long msv = __ballot(sv);
      const unsigned long long pb = msv & below;
      const int p = pb ? 63 - __builtin_clzll(pb) : 0;
      const double zp = __shfl(zv, p), dp = __shfl(dv, p);
      bool pass = false;
      if (sv && pb) {
        const double t2 = hypot(zv, zp);
        pass = fabs((dv - dp) * (zv / t2) * (zp / t2)) <= tol;
      }
      const unsigned long long mpass = __ballot(pass);
      if (mpass) {
        // dependent walk (one lane, the level kernels' order) over the survivors in LDS; a
        // pair whose first member was not rotated into sees its original values (mpass bits)
        sd[lane] = dv;
        sz[lane] = zv;
        hm[lane] = hv;
        if (sv) keep[__popcll(pb)] = lane;
        lds_sync_wave();
        if (lane == 0) {
          const int ns = __popcll(msv);
          int nr = 0, i = 1;
          bool chain = false;
          while (i < ns) {
            const int pj = keep[i - 1], j = keep[i];
            if (!chain && !((mpass >> j) & 1ull)) {
              ++i;
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
              hm[j] |= hm[pj];
              hm[pj] |= 4;
              rp[nr] = pj;
              rq[nr] = j;
              rc[nr] = cc;
              rsn[nr] = ss;
              ++nr;
              const double tt = sd[pj] * cc * cc + sd[j] * ss * ss;
              sd[j] = sd[pj] * ss * ss + sd[j] * cc * cc;
              sd[pj] = tt;
              chain = true;
            } else {
              chain = false;
            }
            ++i;
          }
          s_nrot = nr;
        }
        lds_sync_wave();
        nrot = s_nrot;
        dv = sd[lane];
        zv = sz[lane];
        hv = hm[lane];
      }
    }
    // kept = survivors not rotated away (in sorted order), deflated = the rest (in sorted order)
    const bool dj = in && (rho == 0.0 || rho * fabs(zv) <= tol || (hv & 4));
    const bool kp = in && !dj;
    const unsigned long long mk = __ballot(kp), md = __ballot(dj);
    const int k = __popcll(mk);
    if (nrot && lane < s) {  // rotations on the block's columns (sorted positions -> source columns)
      for (int q = 0; q < nrot; ++q) {
        const int xc = __shfl(srcv, rp[q]), yc = __shfl(srcv, rq[q]);
        const double xv = sQ[xc * S + lane], yv = sQ[yc * S + lane];
        sQ[xc * S + lane] = rc[q] * xv + rsn[q] * yv;
        sQ[yc * S + lane] = rc[q] * yv - rsn[q] * xv;
      }
    }
    if (kp) {
      const int t = __popcll(mk & below);
      dd[t] = dv;
      zz[t] = zv;
      cs[t] = srcv;
    }
    if (dj) {
      const int t = k + __popcll(md & below);
      cs[t] = srcv;
      D[lo + t] = dv;
    }
    if (lane == 0) {
      s_k = k;
      s_rho = rho;
    }
  }
  __syncthreads();
  WAVE_MARK(2);
  const int k = s_k;
  const double rho = s_rho;
  const int i4 = tid >> 2, part = tid & 3;
  WAVE_MARK(3);
  int its = 0;
  if (i4 < k) {  // secular root i4 by a quad
    int o;
    double tau;
    its = secular_quad<NT>(i4, part, k, rho, dd, zz, o, tau);
    if (part == 0) {
      org[i4] = o;
      st[i4] = tau;
      D[lo + i4] = dd[o] + tau;
    }
  }
  if (blockIdx.x == 0 && wv == 0) {  // iterations of the slowest of roots 0-15 (harp_dc_wave_stamps)
    const int mx = (int)wave_max_d((double)its);
    if (lane == 0) g_wave_it = mx;
  }
  __syncthreads();
  WAVE_MARK(4);
  if (i4 < k) {  // Loewner z-hat of position i4 by a quad
    const double dl = dd[i4];
    double pr = 1.0;
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int i = part + 4 * q;
      if (i < k) {
        const double num = (dd[org[i]] - dl) + st[i];
        pr *= i == i4 ? num / rho : num / (dd[i] - dl);
      }
    }
    pr = quad_prod_d(pr);
    if (part == 0) zh[i4] = copysign(sqrt(fmax(pr, 0.0)), zz[i4]);
  }
  __syncthreads();
  WAVE_MARK(5);
  if (i4 < k) {  // column i4 of U, normalised, by a quad
    const double dor = dd[org[i4]], tau = st[i4];
    double u[NT];
    double s2 = 0.0;
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int j = part + 4 * q;
      u[q] = j < k ? zh[j] / ((dd[j] - dor) - tau) : 0.0;
      s2 = fma(u[q], u[q], s2);
    }
    const double inv = 1.0 / sqrt(quad_sum_d(s2));
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int j = part + 4 * q;
      if (j < k) Ut[j * NC + i4] = u[q] * inv;
    }
  }
  __syncthreads();
  WAVE_MARK(6);
  // Q(lo + r, lo + c) = sum_j sQ(r, cs[j]) U(j, c) for c < k, sQ(r, cs[c]) for c >= k: lane = row,
  // wave wv owns columns wv NT .. wv NT + NT - 1 (accumulators in registers; U rows are
  // wave-uniform LDS reads)
  if (lane < s) {
    double* qo = Q + (long)lo * ldq + lo + lane;
    const int c0 = wv * NT;
    if (c0 < k) {
      double acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = 0.0;
      for (int j = 0; j < k; ++j) {
        const double qv = sQ[cs[j] * S + lane];
        const double* u = Ut + j * NC + c0;
#pragma unroll
        for (int t = 0; t < NT; t += 2) {
          const dc_d2 uv = *(const dc_d2*)(u + t);
          acc[t] = fma(qv, uv.x, acc[t]);
          acc[t + 1] = fma(qv, uv.y, acc[t + 1]);
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (c0 + t < k) qo[(long)(c0 + t) * ldq] = acc[t];
    }
    for (int c = k + wv; c < s; c += 4) qo[(long)c * ldq] = sQ[cs[c] * S + lane];
  }
  WAVE_MARK(7);
}

int wave_merge_nc(int S) { return S <= 8 ? 8 : S <= 16 ? 16 : S <= 32 ? 32 : 64; }

size_t wave_merge_lds(int S) {
  return sizeof(double) * ((size_t)S * S + (size_t)S * wave_merge_nc(S) + 8 * 64) + sizeof(int) * 6 * 64;
}

template <int NC>
int launch_wave_merge(double* Q, long ldq, double* D, const double* e, const int* mg, int nm, int S, hipStream_t st) {
  const size_t lds = wave_merge_lds(S);
  if (lds > 65536 && hipFuncSetAttribute((const void*)dc_wave_merge_kernel<NC>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return HARP_ELAUNCH;
  dc_wave_merge_kernel<NC><<<dim3((unsigned)nm), dim3(256), lds, st>>>(Q, ldq, D, e, mg, S);
  return harp_launch_status();
}

// largest merge of the levels on dc_wave_merge_kernel: HARP_DC_WAVE_MERGE (0 = every level on
// the level kernels; A/B and tests), at most kWaveMerge
int wave_merge_max() {
  static const int m = [] {
    const char* v = getenv("HARP_DC_WAVE_MERGE");
    const int x = v ? atoi(v) : kWaveMergeDefault;
    return x < 0 ? 0 : x > kWaveMerge ? kWaveMerge : x;
  }();
  return m;
}

// Inputs of the D&C in one launch (they were ten small torch ops ahead of the first level, ~130
// us of the critical path after the reduction): dmod = d with |e[p]| subtracted at p and p + 1
// for every split point p + 1 (the tree splits down to single rows, so every p in [1, n) is a
// split: dmod[p] = (d[p] - |e[p]|) - |e[p - 1]|, the order of the former two index_add_), Q = I
// (column-major), the workspace zeroed, perm = the identity (for dc_order_kernel).
__global__ __launch_bounds__(256) void dc_setup_kernel(const double* __restrict__ d, const double* __restrict__ e, int n,
                                                       double* __restrict__ dmod, double* __restrict__ Q,
                                                       double* __restrict__ ws, long wsn, long* __restrict__ perm) {
  const long nn = (long)n * n;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nn || i < wsn; i += stride) {
    if (i < nn) Q[i] = i % (n + 1) == 0 ? 1.0 : 0.0;
    if (i < wsn) ws[i] = 0.0;
    if (i < n) {
      const int p = (int)i;
      double v = d[p];
      if (p + 1 < n) v -= fabs(e[p]);
      if (p >= 1) v -= fabs(e[p - 1]);
      dmod[p] = v;
      perm[p] = p;
    }
  }
}

// Ascending order of the D&C's eigenvalues (ties by position): rank_j = the number of
// (d_i, i) < (d_j, j). Workgroup b ranks positions 64 b .. 64 b + 63 with its four waves
// counting over quarters of all n values (in LDS, n <= kMaxN: 32 KB). perm is the identity
// from dc_setup_kernel, so a NaN (no strict order, colliding ranks) cannot leave an index
// unwritten. Replaces a torch argsort + gather (~7 small kernels) after the top merge.
__global__ __launch_bounds__(256) void dc_order_kernel(const double* __restrict__ dmod, int n, double* __restrict__ w,
                                                       long* __restrict__ perm) {
  __shared__ double sv[kMaxN];
  __shared__ int part[4][64];
  for (int j = threadIdx.x; j < n; j += 256) sv[j] = dmod[j];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const double v = j < n ? sv[j] : 0.0;
  const int q = (n + 3) / 4, i0 = wv * q, i1 = i0 + q < n ? i0 + q : n;
  int r = 0;
#pragma unroll 8
  for (int i = i0; i < i1; ++i) {
    const double x = sv[i];
    r += (x < v || (x == v && i < j)) ? 1 : 0;
  }
  part[wv][lane] = r;
  __syncthreads();
  if (wv == 0 && j < n) {
    r = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    w[r] = v;
    perm[r] = j;
  }
}

size_t prep_lds(int smax) { return (size_t)smax * (2 * sizeof(double) + 4 * sizeof(int)); }

}  // namespace

HARP_EXPORT int harp_dc_max_n() { return kMaxN; }
HARP_EXPORT int harp_dc_wave_stamps(long long* out) {
  int it = 0;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), sizeof(long long) * 8) != hipSuccess ||
      hipMemcpyFromSymbol(&it, HIP_SYMBOL(g_wave_it), sizeof(int)) != hipSuccess)
    return HARP_ELAUNCH;
  out[8] = it;
  return HARP_OK;
}

HARP_EXPORT int harp_dc_prep_stamps(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prep_t), sizeof(long long) * 9) == hipSuccess ? HARP_OK : HARP_ELAUNCH;
}

// doubles of the workspace for size n: Qb n^2, U n^2, dd/zz/tau/zh/rho/rotc/rots 7 n, sort
// scratch 3 n; ints (colsrc/org/kcnt/rotp/rotq/jl/jr/kl/kr 9 n) follow as 5 n doubles
HARP_EXPORT long harp_dc_ws_doubles(int n) { return 2L * n * n + 10L * n + 5L * n + 16; }

// dmod, Q (n x n, column-major) and ws (harp_dc_ws_doubles(n)) for harp_dc_tridiag from the
// tridiagonal (d, e): see dc_setup_kernel (the tree of ops/tridiag_dc.py tree_levels, which
// splits every position 1 .. n - 1). e: n - 1 entries (any pointer when n == 1).
HARP_EXPORT int harp_dc_setup(const double* d, const double* e, int n, double* dmod, double* Q, double* ws,
                              long* perm, hipStream_t st) {
  if (n < 1 || n > kMaxN || !d || !dmod || !Q || !ws || !perm || (n > 1 && !e)) return HARP_EBADARG;
  const long wsn = harp_dc_ws_doubles(n);
  const long work = wsn > (long)n * n ? wsn : (long)n * n;
  long blocks = (work + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  dc_setup_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>(d, e, n, dmod, Q, ws, wsn, perm);
  return harp_launch_status();
}

// w = dmod ascending, perm[r] = the position of the r-th smallest (ties by position), for
// n <= harp_dc_max_n(): dc_order_kernel. perm: int64 (a torch index), the identity on entry
// (harp_dc_setup writes it).
HARP_EXPORT int harp_dc_order(const double* dmod, int n, double* w, long* perm, hipStream_t st) {
  if (n < 1 || n > kMaxN || !dmod || !w || !perm) return HARP_EBADARG;
  dc_order_kernel<<<dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st>>>(dmod, n, w, perm);
  return harp_launch_status();
}

// Eigen-decomposition of the symmetric tridiagonal (dmod, e): dmod is the diagonal with
// |e[mid - 1]| already subtracted at d[mid - 1] and d[mid] for every merge (harp_amd/ops/eig.py),
// overwritten by the (unsorted) eigenvalues. Q: n x n column-major, = I on entry, holds the
// eigenvectors on exit (columns in the order of dmod). merges: (lo, mid, hi) int32 triples
// of all levels, bottom level first; level_off[l] .. level_off[l + 1]: level l's merges
// (host array), level_smax[l]: its largest block, level_full[l] (host, may be null): its
// merges cover all n rows. ws: harp_dc_ws_doubles(n) doubles, zeroed.
HARP_EXPORT int harp_dc_tridiag(double* dmod, const double* e, int n, double* Q, const int* merges,
                                const int* level_off, const int* level_smax, const int* level_full, int nlevels,
                                double* ws, hipStream_t st) {
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
  w.jl = ip + 5 * n;
  w.jr = ip + 6 * n;
  w.kl = ip + 7 * n;
  w.kr = ip + 8 * n;
  // a level whose merges cover every row writes its products to the other buffer and the two
  // swap roles (no copy-back); Q's off-block entries are zero in both buffers throughout
  double* cur = Q;
  double* oth = Qb;
  for (int l = 0; l < nlevels; ++l) {
    const int m0 = level_off[l], nm = level_off[l + 1] - m0;
    const int smax = level_smax[l];
    if (nm <= 0) continue;
    if (smax < 2 || smax > n) return HARP_EBADARG;
    w.ldu = smax;
    const int* mg = merges + 3 * m0;
    if (smax <= wave_merge_max()) {
      const int nc = wave_merge_nc(smax);
      const int s_ = nc == 8    ? launch_wave_merge<8>(cur, n, dmod, e, mg, nm, smax, st)
                     : nc == 16 ? launch_wave_merge<16>(cur, n, dmod, e, mg, nm, smax, st)
                     : nc == 32 ? launch_wave_merge<32>(cur, n, dmod, e, mg, nm, smax, st)
                                : launch_wave_merge<64>(cur, n, dmod, e, mg, nm, smax, st);
      if (s_ != HARP_OK) return s_;
      continue;
    }
    const size_t lds = prep_lds(smax);
    // set per launch (a host-side attribute call, no process-wide cache to race on)
    if (lds > 65536 && hipFuncSetAttribute((const void*)dc_prep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds) != hipSuccess)
      return HARP_ELAUNCH;
    const int threads = smax >= 512 ? 1024 : smax >= 128 ? 256 : 64;
    dc_prep_kernel<<<dim3((unsigned)nm), dim3(threads), lds, st>>>(cur, n, dmod, e, mg, w);
    const unsigned wg = (unsigned)((n + 3) / 4);
    dc_secular_kernel<<<dim3(wg), dim3(256), 0, st>>>(mg, nm, n, dmod, w);
    dc_loewner_kernel<<<dim3(wg), dim3(256), 0, st>>>(mg, nm, n, w);
    dc_vectors_kernel<<<dim3(wg), dim3(256), 0, st>>>(mg, nm, n, w);
    const int tiles = (smax + TM - 1) / TM, rtm = tiles + 1;  // row tiles: + 1 for the split
    const size_t glds = kGemmTileLds + 2 * sizeof(int) * (size_t)smax;
    if (glds > 65536 && hipFuncSetAttribute((const void*)dc_gemm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)glds) != hipSuccess)
      return HARP_ELAUNCH;
    dc_gemm_kernel<<<dim3((unsigned)(rtm * tiles), (unsigned)nm), dim3(256), glds, st>>>(cur, oth, n, mg, w, rtm);
    if (level_full && level_full[l]) {
      double* t = cur;
      cur = oth;
      oth = t;
    } else {
      const long per = (long)smax * smax;
      const unsigned cb = (unsigned)((per + 256 * 4 - 1) / (256 * 4));
      dc_copyback_kernel<<<dim3(cb, (unsigned)nm), dim3(256), 0, st>>>(oth, cur, n, mg);
    }
    const int s_ = harp_launch_status();
    if (s_ != HARP_OK) return s_;
  }
  if (cur != Q && hipMemcpyAsync(Q, cur, sizeof(double) * nn, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return HARP_ELAUNCH;
  return harp_launch_status();
}
