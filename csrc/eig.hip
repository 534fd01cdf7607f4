// Eigenvalues of a symmetric fp64 matrix on gfx950: Householder tridiagonalisation on the
// CUs of ONE XCD (cooperative kernel), then multisection on the tridiagonal.
//
// Reference: the PCA step 3 eigen-decomposition of the correlation matrix,
// ml/daal/src/main/java/edu/iu/daal_pca/cordensedistr/PCADaalCollectiveMapper.java:121-147
// (DAAL pca correlation method, eigenvalues + eigenvectors).
//
// Why: rocSOLVER's dsyevd takes ~21 ms for the 1000 x 1000 correlation matrix of the PCA
// pass (its Jacobi forms 157 ms; profiles/r3_eig), 17 % of a one-GPU pass and ~60 % at the
// 8-GPU share. The unblocked reduction (LAPACK dsytd2: per column k a Householder vector v,
// p = tau A v, w = p - (tau p.v / 2) v, A -= v w^T + w v^T) is a chain of n small
// matrix-vector steps: launch-bound as separate kernels, but cheap as ONE kernel whose
// workgroups all sit on one XCD and synchronise through that XCD's L2 (two arrivals per
// column; no L2 write-back is needed since no other XCD touches the matrix):
//  * participants read HW_REG_XCC_ID and claim a slot only on XCD 0 (as the cooperative SMO
//    of svm.hip); 32 workgroups x 16 waves, each workgroup a 64-row super tile of the
//    trailing m x m block split by columns over its waves, the same tile in both phases;
//  * phase 1: p = tau A v per tile row, the waves' partials summed in LDS and added into p
//    with one fp64 atomic per row and workgroup (and p.v likewise); phase 2: the rank-2
//    update of the tile, which also accumulates the next column's squared norm (the next
//    Householder step needs no extra pass);
//  * the matrix is read past the CU's L1 (other CUs wrote it one step earlier).
// The default reduction is the fused look-ahead form (sytrd_fused_kernel below: one pass over
// the trailing block and ONE arrival per column, 14.4 -> ~11 ms at n = 1000,
// profiles/r3_eig_fused); the two-pass form above keeps the per-phase cycle stamps.
// Multisection (tridiag_multisect_kernel): 16 lanes per eigenvalue evaluate Sturm counts at
// 16 points of its interval, so each round narrows it 17-fold (~13 rounds to machine
// precision instead of ~53 bisections).
#include "common.h"

namespace {

constexpr int kT = 1024, kW = kT / 64;
constexpr int kMaxNB = 32;
constexpr int kMaxN = 4096;  // v and w staged in LDS (2 x 32 KB)
// ws (int32, zeroed by the host): [0] claims [1] arrivals [2] error
constexpr int kWsInts = 16;
constexpr int kU = 8;  // columns per batch of loads in flight

__device__ __forceinline__ double ld_agent(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_agent(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_nt(const double* p) { return __builtin_nontemporal_load(p); }

// this thread's stores are complete, then thread 0 arrives and waits for all NB
__device__ __forceinline__ bool arrive(int* cnt, int target, int* err, int* s_ok) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(cnt, 1);
    int ok = 1;
    long spin = 0;
    while (ld_agent(cnt) < target) {
      if (++spin > (1L << 22) || ld_agent(err)) {
        ok = 0;
        atomicExch(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

// block-wide sum, the result in every thread
template <int T = kT>
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum_d_dpp(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < T / 64; ++w) s += red[w];
  __syncthreads();
  return s;
}

// A: n x n symmetric, column-major (lda), overwritten. d[n], e[n-1]: the tridiagonal.
// wsd (doubles, zeroed): p[2][n], then pv[2], sigma[2].
__global__ __launch_bounds__(kT) void sytrd_coop_kernel(double* __restrict__ A, long lda, int n,
                                                        double* __restrict__ dout, double* __restrict__ eout, int NB,
                                                        int* __restrict__ ws, double* __restrict__ wsd,
                                                        long long* __restrict__ stamps) {
  extern __shared__ double smem[];
  double* sv = smem;      // Householder vector of this step (m entries)
  double* sw = smem + n;  // w = p + K v
  __shared__ double red[kW];
  __shared__ double spart[kW][64];  // per-wave partial p of the super tile's 64 rows
  __shared__ int s_b, s_ok;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) {
    int b = -1;
    if ((__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf) == 0) b = atomicAdd(ws, 1);  // HW_REG_XCC_ID
    s_b = b;
  }
  __syncthreads();
  const int b = s_b;
  if (b < 0 || b >= NB) return;
  int* err = ws + 2;
  double* pbuf0 = wsd;
  double* pbuf1 = wsd + n;
  double* scal = wsd + 2 * (long)n;  // pv[2], sigma[2]
  int syncs = 0;
  // diagnostic: workgroup 0 / thread 0 sums the cycles of each phase into stamps[0..5]
  long long st_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, st_t = 0;
  const bool stamp = stamps != nullptr && b == 0 && tid == 0;
#define STAMP(i)                                    \
  if (stamp) {                                      \
    const long long now = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += now - st_t;                        \
    st_t = now;                                     \
  }
  if (stamp) st_t = __builtin_amdgcn_s_memtime();
  // squared norm of column 0 below the subdiagonal (every workgroup, no sync)
  double s0 = 0.0;
  for (int i = 2 + tid; i < n; i += kT) {
    const double x = A[i];
    s0 += x * x;
  }
  s0 = block_sum(s0, red);
  for (int k = 0; k + 2 < n; ++k) {
    const int par = k & 1, off = k + 1, m = n - off;
    double* pcur = par ? pbuf1 : pbuf0;
    double* pnext = par ? pbuf0 : pbuf1;
    const double alpha = ld_nt(A + off + k * lda);
    const double sig = k == 0 ? s0 : ld_agent(scal + 2 + par);
    double beta = alpha, tau = 0.0, scl = 0.0;
    if (sig != 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sig), alpha);
      tau = (beta - alpha) / beta;
      scl = 1.0 / (alpha - beta);
    }
    if (b == 0 && tid == 0) {
      dout[k] = ld_nt(A + k + k * lda);
      eout[k] = beta;
      // next step's accumulators (read by every workgroup one step ago, before the last arrival)
      scal[par ^ 1] = 0.0;
      scal[2 + (par ^ 1)] = 0.0;
    }
    if (b == 0)
      for (int i = tid; i < n; i += kT) pnext[i] = 0.0;
    for (int i = tid; i < m; i += kT) sv[i] = i == 0 ? 1.0 : ld_nt(A + off + i + k * lda) * scl;
    __syncthreads();
    STAMP(0)
    // super tiles: 64 rows x cps columns of the trailing block per workgroup, each wave
    // cpw of those columns (re-cut every step, so the work stays balanced as m shrinks; the
    // matrix is therefore read with agent-scope loads, past the CU's L1, which does not see
    // other workgroups' writes of the last step -- plain, workgroup-scope and plain after
    // `buffer_inv sc0` loads all returned stale lines). The 16 waves' partial p are summed in
    // LDS, so p takes one fp64 atomic per row and workgroup. Measured alternatives
    // (profiles/r3_eig): non-temporal loads 15.7 ms; a fixed element-to-workgroup ownership
    // with plain loads (64-row groups: 27.6 ms; cyclic 16-row chunks: 24.3 ms) balanced or
    // issued worse. What remains is latency: a batch of loads takes ~2.7 us past L1.
    const int RG = (m + 63) / 64;
    const int CSG = NB / RG > 0 ? NB / RG : 1;
    const int cps = (m + CSG - 1) / CSG;
    const int cpw = (cps + kW - 1) / kW;
    const int ST = RG * CSG;
    if (tau != 0.0) {
      double pvp = 0.0;
      for (int st = b; st < ST; st += NB) {
        const int r = (st % RG) * 64 + lane;
        const int cs0 = (st / RG) * cps, cs1 = cs0 + cps < m ? cs0 + cps : m;
        const int c0 = cs0 + wv * cpw, c1 = c0 + cpw < cs1 ? c0 + cpw : cs1;
        double a0 = 0.0, a1 = 0.0;
        if (r < m && c0 < c1) {
          const double* col = A + off + r + (long)(off + c0) * lda;
          int c = c0;
          for (; c + kU <= c1; c += kU, col += kU * lda) {  // kU columns' loads in flight
            double x[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) x[u] = ld_agent(col + u * lda);
#pragma unroll
            for (int u = 0; u < kU; u += 2) {
              a0 = fma(x[u], sv[c + u], a0);
              a1 = fma(x[u + 1], sv[c + u + 1], a1);
            }
          }
          for (; c < c1; ++c, col += lda) a0 = fma(ld_agent(col), sv[c], a0);
        }
        STAMP(6)
        spart[wv][lane] = a0 + a1;
        __syncthreads();
        STAMP(7)
        if (wv == 0 && r < m) {
          double acc = 0.0;
#pragma unroll
          for (int q = 0; q < kW; ++q) acc += spart[q][lane];
          const double pp = tau * acc;
          atomicAdd(pcur + r, pp);
          pvp = fma(pp, sv[r], pvp);
        }
        STAMP(8)
        __syncthreads();
      }
      if (wv == 0) {
        pvp = wave_sum_d_dpp(pvp);
        if (lane == 0 && pvp != 0.0) atomicAdd(scal + par, pvp);
      }
    }
    STAMP(1)
    if (!arrive(ws + 1, NB * ++syncs, err, &s_ok)) return;
    STAMP(2)
    if (tau != 0.0) {
      const double K = -0.5 * tau * ld_agent(scal + par);
      for (int i = tid; i < m; i += kT) sw[i] = ld_agent(pcur + i) + K * sv[i];
      __syncthreads();
    }
    STAMP(3)
    // rank-2 update of the same tiles; column off (local 0) rows >= 2 give the next sigma
    double sp = 0.0;
    for (int st = b; st < ST; st += NB) {
      const int r = (st % RG) * 64 + lane;
      const int cs0 = (st / RG) * cps, cs1 = cs0 + cps < m ? cs0 + cps : m;
      const int c0 = cs0 + wv * cpw, c1 = c0 + cpw < cs1 ? c0 + cpw : cs1;
      if (r >= m || c0 >= c1) continue;
      if (tau != 0.0) {
        const double vr = sv[r], wr = sw[r];
        double* col = A + off + r + (long)(off + c0) * lda;
        int c = c0;
        for (; c + kU <= c1; c += kU, col += kU * lda) {
          double x[kU];
#pragma unroll
          for (int u = 0; u < kU; ++u) x[u] = ld_agent(col + u * lda);
#pragma unroll
          for (int u = 0; u < kU; ++u) {
            const double a = x[u] - (vr * sw[c + u] + wr * sv[c + u]);
            col[u * lda] = a;
            if (c + u == 0 && r >= 2) sp = fma(a, a, sp);
          }
        }
        for (; c < c1; ++c, col += lda) {
          const double a = ld_agent(col) - (vr * sw[c] + wr * sv[c]);
          *col = a;
          if (c == 0 && r >= 2) sp = fma(a, a, sp);
        }
      } else if (c0 == 0 && r >= 2) {
        const double a = ld_agent(A + off + r + (long)off * lda);
        sp = fma(a, a, sp);
      }
    }
    sp = wave_sum_d_dpp(sp);
    if (lane == 0 && sp != 0.0) atomicAdd(scal + 2 + (par ^ 1), sp);
    STAMP(4)
    if (!arrive(ws + 1, NB * ++syncs, err, &s_ok)) return;
    STAMP(5)
  }
  if (stamp)
    for (int i = 0; i < 9; ++i) stamps[i] = st_acc[i];
#undef STAMP
  if (b == 0 && tid == 0) {
    if (n >= 2) {
      dout[n - 2] = ld_nt(A + (n - 2) + (long)(n - 2) * lda);
      eout[n - 2] = ld_nt(A + (n - 1) + (long)(n - 2) * lda);
    }
    dout[n - 1] = ld_nt(A + (n - 1) + (long)(n - 1) * lda);
  }
}

// ---------------------------------------------------------------------------------------
// Fused form (look-ahead): ONE pass over the trailing block and ONE arrival per column.
// After step k's p_k = tau_k A_k v_k is complete, every workgroup forms w_k and -- from the
// column k+1 of A_k, updated on the fly (a_i = A_k[i][k+1] - v_i w_0 - w_i v_0) -- the next
// Householder vector v_{k+1} and tau_{k+1} itself (redundantly, ~2 m loads + two block
// sums), so the rank-2 update of the trailing block can fold in the next product:
// a = x - (v_r w_c + w_r v_c) is stored AND multiplied by v_{k+1}[c] in the same pass, and
// p_{k+1} is complete at the step's single arrival. Same arithmetic as dsytd2; the column
// update is done once per workgroup instead of read back from memory.

// Householder vector of the column held in c[0..L): c[0] = alpha, sigma = sum c[1..]^2;
// c becomes v (v[0] = 1). Returns tau; beta in *beta. Every thread of the block calls it.
template <int T = kT>
__device__ __forceinline__ double house_lds(double* c, int L, double* red, double* beta) {
  __syncthreads();  // c[] was written by other threads
  double s = 0.0;
  for (int i = 1 + (int)threadIdx.x; i < L; i += T) s = fma(c[i], c[i], s);
  const double sig = block_sum<T>(s, red);  // its barriers also order the c[] writes before this read
  const double alpha = c[0];
  double b = alpha, tau = 0.0, scl = 0.0;
  if (sig != 0.0) {
    b = -copysign(sqrt(alpha * alpha + sig), alpha);
    tau = (b - alpha) / b;
    scl = 1.0 / (alpha - b);
  }
  for (int i = 1 + (int)threadIdx.x; i < L; i += T) c[i] *= scl;
  __syncthreads();  // everyone has read c[0] (alpha) before it becomes 1
  if (threadIdx.x == 0) c[0] = 1.0;
  __syncthreads();
  *beta = b;
  return tau;
}

// One pass over the mm x mm block at (base, base): if upd, x -= vu[r] wu[c] + wu[r] vu[c]
// (vu, wu indexed from the block's first row) and stored; if tn != 0, pn[r] += tn * sum_c
// x * vn[c]. Super tiles of 64 rows x cps columns, re-cut every step (see sytrd_coop_kernel).
template <int KU>
__device__ __forceinline__ void fused_pass(double* __restrict__ A, long lda, int base, int mm, int b, int NB,
                                           bool upd, const double* vu, const double* wu, double tn,
                                           const double* vn, double* __restrict__ pn, double (*spart)[64]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int RG = (mm + 63) / 64;
  const int CSG = NB / RG > 0 ? NB / RG : 1;
  const int cps = (mm + CSG - 1) / CSG;
  const int cpw = (cps + kW - 1) / kW;
  const int ST = RG * CSG;
  const bool mv = tn != 0.0;
  if (!upd && !mv) return;
  for (int st = b; st < ST; st += NB) {
    const int r = (st % RG) * 64 + lane;
    const int cs0 = (st / RG) * cps, cs1 = cs0 + cps < mm ? cs0 + cps : mm;
    const int c0 = cs0 + wv * cpw, c1 = c0 + cpw < cs1 ? c0 + cpw : cs1;
    double a0 = 0.0, a1 = 0.0;
    if (r < mm && c0 < c1) {
      const double vr = upd ? vu[r] : 0.0, wr = upd ? wu[r] : 0.0;
      double* col = A + base + r + (long)(base + c0) * lda;
      int c = c0;
      for (; c + KU <= c1; c += KU, col += KU * lda) {  // KU columns' loads in flight
        double x[KU];
#pragma unroll
        for (int u = 0; u < KU; ++u) x[u] = ld_agent(col + u * lda);
        if (upd) {
#pragma unroll
          for (int u = 0; u < KU; ++u) {
            x[u] -= vr * wu[c + u] + wr * vu[c + u];
            col[u * lda] = x[u];
          }
        }
#pragma unroll
        for (int u = 0; u < KU; u += 2) {
          a0 = fma(x[u], vn[c + u], a0);
          a1 = fma(x[u + 1], vn[c + u + 1], a1);
        }
      }
      for (; c < c1; ++c, col += lda) {
        double x = ld_agent(col);
        if (upd) {
          x -= vr * wu[c] + wr * vu[c];
          *col = x;
        }
        a0 = fma(x, vn[c], a0);
      }
    }
    if (mv) {
      spart[wv][lane] = a0 + a1;
      __syncthreads();
      if (wv == 0 && r < mm) {
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < kW; ++q) acc += spart[q][lane];
        if (acc != 0.0) atomicAdd(pn + r, tn * acc);
      }
      __syncthreads();
    }
  }
}

// A: n x n symmetric, column-major (lda), overwritten. d[n], e[n-1]: the tridiagonal.
// wsd (doubles, zeroed): p[3][n] (p_k, p_{k+1}, and the buffer zeroed for p_{k+2}).
template <int KU>
// vout / tauout (nullable): the Householder vectors (column k = v_k, v_k[k + 1] = 1 and
// zeros above, n x n column-major, zeroed by the host) and their factors, written by
// workgroup 0 for the eigenvector back-transform
__global__ __launch_bounds__(kT) void sytrd_fused_kernel(double* __restrict__ A, long lda, int n,
                                                         double* __restrict__ dout, double* __restrict__ eout, int NB,
                                                         int* __restrict__ ws, double* __restrict__ wsd,
                                                         double* __restrict__ vout, double* __restrict__ tauout,
                                                         long long* __restrict__ stamps) {
  extern __shared__ double smem[];
  double* sv = smem;          // v_k
  double* sw = smem + n;      // w_k
  double* sn = smem + 2 * n;  // v_{k+1}
  __shared__ double red[kW];
  __shared__ double spart[kW][64];
  __shared__ int s_b, s_ok;
  const int tid = threadIdx.x;
  if (tid == 0) {
    int b = -1;
    if ((__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf) == 0) b = atomicAdd(ws, 1);  // HW_REG_XCC_ID
    s_b = b;
  }
  __syncthreads();
  const int b = s_b;
  if (b < 0 || b >= NB) return;
  int* err = ws + 2;
  const bool lead = b == 0 && tid == 0;
  if (n < 3) {
    if (lead) {
      dout[0] = A[0];
      if (n == 2) {
        eout[0] = A[1];
        dout[1] = A[1 + lda];
      }
    }
    return;
  }
  int syncs = 0;
  // prologue: v_0 from column 0 (rows 1..n-1), p_0 = tau_0 A[1.., 1..] v_0
  for (int i = tid; i < n - 1; i += kT) sn[i] = A[1 + i];
  double beta;
  double tn = house_lds(sn, n - 1, red, &beta);
  if (lead) {
    dout[0] = A[0];
    eout[0] = beta;
  }
  if (vout && b == 0) {
    for (int i = tid; i < n - 1; i += kT) vout[1 + i] = sn[i];
    if (tid == 0) tauout[0] = tn;
  }
  fused_pass<KU>(A, lda, 1, n - 1, b, NB, false, nullptr, nullptr, tn, sn, wsd, spart);
  if (!arrive(ws + 1, NB * ++syncs, err, &s_ok)) return;
  // diagnostic (stamps != nullptr): workgroup 0 / thread 0 sums the cycles of each phase
  const bool stamp = stamps != nullptr && b == 0 && tid == 0;
  long long ph[4] = {0, 0, 0, 0}, t_last = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {
    if (stamp) {
      const long long now = (long long)__builtin_amdgcn_s_memtime();
      ph[i] += now - t_last;
      t_last = now;
    }
  };
  for (int k = 0; k + 2 < n; ++k) {
    const int off = k + 1, m = n - off;
    const double tk = tn;
    double* t = sv;  // v_k <- the look-ahead vector; the old v_{k-1} buffer takes v_{k+1}
    sv = sn;
    sn = t;
    double* pk = wsd + (long)(k % 3) * n;
    double* pn = wsd + (long)((k + 1) % 3) * n;
    double* pz = wsd + (long)((k + 2) % 3) * n;
    // w_k = p_k - (tau_k p_k.v_k / 2) v_k (every workgroup; w = 0 when tau_k = 0)
    // p_k and column off of A_k are loaded together (one latency); m <= kMaxN = 4 kT
    constexpr int R = kMaxN / kT;
    double pr[R], cr[R];
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = tid + q * kT;
      pr[q] = i < m && tk != 0.0 ? ld_agent(pk + i) : 0.0;
      cr[q] = i < m ? ld_agent(A + off + i + (long)off * lda) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = tid + q * kT;
      if (i < m) s = fma(pr[q], sv[i], s);
    }
    const double K = -0.5 * tk * block_sum(s, red);
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = tid + q * kT;
      if (i < m) sw[i] = fma(K, sv[i], pr[q]);
    }
    if (b == 0)  // p_{k-1}'s buffer: read by every workgroup before the last arrival
      for (int i = tid; i < n; i += kT) pz[i] = 0.0;
    __syncthreads();
    // column off of A_{k+1}: rows off.. updated on the fly; its diagonal is d[k+1], the
    // rest gives v_{k+1} (or, at the last step, the final subdiagonal entry)
    const double v0 = sv[0], w0 = sw[0];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = tid + q * kT;
      if (i >= m) break;
      const double a = cr[q] - (sv[i] * w0 + sw[i] * v0);
      if (i == 0) {
        if (lead) dout[k + 1] = a;
      } else {
        sn[i - 1] = a;
      }
    }
    __syncthreads();
    mark(0);
    if (k + 3 < n) {
      tn = house_lds(sn, m - 1, red, &beta);
      if (lead) eout[k + 1] = beta;
      if (vout && b == 0) {
        double* vc = vout + (long)(k + 1) * n + (k + 2);
        for (int i = tid; i < m - 1; i += kT) vc[i] = sn[i];
      }
    } else {
      tn = 0.0;
      if (lead) eout[k + 1] = sn[0];
    }
    if (vout && lead) tauout[k + 1] = tn;
    mark(1);
    // trailing block of the next step: update by (v_k, w_k) and p_{k+1} in one pass
    fused_pass<KU>(A, lda, off + 1, m - 1, b, NB, tk != 0.0, sv + 1, sw + 1, tn, sn, pn, spart);
    mark(2);
    if (!arrive(ws + 1, NB * ++syncs, err, &s_ok)) return;
    mark(3);
  }
  if (stamp)
    for (int i = 0; i < 4; ++i) stamps[i] = ph[i];
  if (lead) dout[n - 1] = ld_agent(A + (n - 1) + (long)(n - 1) * lda);
}

// number of eigenvalues of the tridiagonal (d, e^2) below x (Sturm sequence)
__device__ __forceinline__ int sturm_count(const double* d, const double* e2, int n, double x, double pivmin) {
  double q = d[0] - x;
  int c = q < 0.0;
  for (int j = 1; j < n; ++j) {
    if (fabs(q) < pivmin) q = -pivmin;
    q = d[j] - x - e2[j - 1] / q;
    c += q < 0.0;
  }
  return c;
}

// eigenvalue i (ascending) of the tridiagonal per 16-lane group: each round the 16 lanes
// count at 16 interior points of [lo, hi] and the group keeps the sub-interval holding i
__global__ __launch_bounds__(256) void tridiag_multisect_kernel(const double* __restrict__ d,
                                                                const double* __restrict__ e, int n,
                                                                double* __restrict__ w) {
  extern __shared__ double sm[];
  double* sd = sm;
  double* se2 = sm + n;
  __shared__ double red[8];
  const int tid = threadIdx.x;
  double glo = __builtin_inf(), ghi = -__builtin_inf(), emax = 0.0;
  for (int j = tid; j < n; j += 256) {
    const double dj = d[j];
    const double el = j > 0 ? fabs(e[j - 1]) : 0.0, er = j + 1 < n ? fabs(e[j]) : 0.0;
    sd[j] = dj;
    if (j + 1 < n) se2[j] = e[j] * e[j];
    glo = fmin(glo, dj - el - er);
    ghi = fmax(ghi, dj + el + er);
    emax = fmax(emax, er);
  }
  // Gershgorin bounds and the pivot floor (block reductions through LDS)
  for (int o = 32; o > 0; o >>= 1) {
    glo = fmin(glo, __shfl_xor(glo, o, 64));
    ghi = fmax(ghi, __shfl_xor(ghi, o, 64));
    emax = fmax(emax, __shfl_xor(emax, o, 64));
  }
  if ((tid & 63) == 0) {
    red[tid >> 6] = glo;
    red[4 + (tid >> 6)] = ghi;
  }
  __syncthreads();
  glo = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
  ghi = fmax(fmax(red[4], red[5]), fmax(red[6], red[7]));
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = emax;
  __syncthreads();
  emax = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  const double scale = fmax(fabs(glo), fabs(ghi));
  const double eps = 2.220446049250313e-16;
  const double pivmin = 2.2250738585072014e-308 * fmax(1.0, emax * emax);
  glo -= 2.0 * eps * scale * n + pivmin;
  ghi += 2.0 * eps * scale * n + pivmin;
  const int i = (int)((blockIdx.x * 256 + tid) >> 4), sl = tid & 15;
  double lo = glo, hi = ghi;
  const double tol = 2.0 * eps * scale;
  for (int round = 0; round < 40 && hi - lo > tol; ++round) {
    const double step = (hi - lo) / 17.0;
    const double x = lo + step * (sl + 1);
    const int cnt = i < n ? sturm_count(sd, se2, n, x, pivmin) : n;
    // the first point whose count exceeds i bounds the eigenvalue from above
    const unsigned long long above = __ballot(cnt > i);
    const int base = (int)(threadIdx.x & 48);  // this group's first lane within the wave
    const unsigned grp = (unsigned)((above >> base) & 0xffffull);
    const int j = grp ? __builtin_ctz(grp) : 16;  // uniform within the group
    const double nlo = lo + step * j, nhi = j < 16 ? lo + step * (j + 1) : hi;
    lo = nlo;
    hi = nhi;
  }
  if (i < n && sl == 0) w[i] = 0.5 * (lo + hi);
}

}  // namespace

// Fused look-ahead reduction (sytrd_fused_kernel) + multisection; wsd: zeroed 3 n doubles.
static long long* g_fused_stamps = nullptr;  // diagnostic phase cycles (harp_eig_fused_stamps)
template <int KU>
static int launch_fused(double* A, long lda, int n, double* d, double* e, int NB, int* ws, double* wsd, hipStream_t s,
                        double* V = nullptr, double* tau = nullptr) {
  const size_t lds1 = sizeof(double) * 3 * (size_t)n;
  if (lds1 > 32 * 1024 && hipFuncSetAttribute((const void*)sytrd_fused_kernel<KU>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1) != hipSuccess)
    return HARP_ELAUNCH;
  sytrd_fused_kernel<KU><<<dim3((unsigned)(NB * 8)), dim3(kT), lds1, s>>>(A, lda, n, d, e, NB, ws, wsd, V, tau,
                                                                      g_fused_stamps);
  return harp_launch_status();
}

HARP_EXPORT int harp_eig_sym_fused(double* A, long lda, int n, double* d, double* e, double* w, int nb_max, int* ws,
                                   double* wsd, hipStream_t s) {
  if (n < 1 || n > kMaxN || lda < n || nb_max < 1 || nb_max > kMaxNB || !ws || !wsd) return HARP_EBADARG;
  const int NB = nb_max;
  // 8 columns per batch of loads: 16 and 32 spill at 16 waves per CU (profiles/r3_eig_fused)
  int st = launch_fused<8>(A, lda, n, d, e, NB, ws, wsd, s);
  if (st != HARP_OK) return st;
  const size_t lds2 = sizeof(double) * 2 * (size_t)n;
  if (lds2 > 32 * 1024 &&
      hipFuncSetAttribute((const void*)tridiag_multisect_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds2) != hipSuccess)
    return HARP_ELAUNCH;
  tridiag_multisect_kernel<<<dim3((unsigned)((n * 16 + 255) / 256)), dim3(256), lds2, s>>>(d, e, n, w);
  return harp_launch_status();
}

// Tridiagonalisation only, keeping the reflectors: A = Q T Q^T with Q = H_0 H_1 ... H_{n-3},
// H_k = I - tau_k v_k v_k^T, v_k = V[:, k] (n x n column-major, zeroed by the caller; tau:
// n doubles). d, e: the tridiagonal. Same cooperative contract as harp_eig_sym_fused.
HARP_EXPORT int harp_sytrd_fused(double* A, long lda, int n, double* d, double* e, double* V, double* tau, int nb_max,
                                 int* ws, double* wsd, hipStream_t s) {
  if (n < 1 || n > kMaxN || lda < n || nb_max < 1 || nb_max > kMaxNB || !ws || !wsd || !V || !tau) return HARP_EBADARG;
  return launch_fused<8>(A, lda, n, d, e, nb_max, ws, wsd, s, V, tau);
}

// Eigenvalues (ascending) of the tridiagonal (d, e) by multisection into w (n doubles).
HARP_EXPORT int harp_tridiag_eigvals(const double* d, const double* e, int n, double* w, hipStream_t s) {
  if (n < 1 || n > kMaxN || !d || !e || !w) return HARP_EBADARG;
  const size_t lds2 = sizeof(double) * 2 * (size_t)n;
  if (lds2 > 32 * 1024 &&
      hipFuncSetAttribute((const void*)tridiag_multisect_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds2) != hipSuccess)
    return HARP_ELAUNCH;
  tridiag_multisect_kernel<<<dim3((unsigned)((n * 16 + 255) / 256)), dim3(256), lds2, s>>>(d, e, n, w);
  return harp_launch_status();
}

// diagnostic: the next fused launches sum workgroup 0's cycles per phase into stamps[0..3]
// (w + column update, Householder vector, trailing pass, arrival); nullptr turns it off
HARP_EXPORT void harp_eig_fused_stamps(long long* stamps) { g_fused_stamps = stamps; }
HARP_EXPORT int harp_eig_ws_ints() { return kWsInts; }
HARP_EXPORT int harp_eig_max_n() { return kMaxN; }
// workgroups the reduction uses (all nb_max of XCD 0; the tiles are re-cut every step)
HARP_EXPORT int harp_eig_workgroups(int n, int nb_max) { return n < 1 || nb_max < 1 || nb_max > kMaxNB ? -1 : nb_max; }

// Eigenvalues (ascending) of the n x n symmetric fp64 matrix A (column-major, lda; destroyed)
// into w. d, e: n-double scratch (the tridiagonal). ws: zeroed harp_eig_ws_ints() int32;
// wsd: zeroed 2 n + 4 doubles. harp_eig_workgroups(n, nb_max) workgroups of XCD 0 take part;
// afterwards ws[0] >= that count and ws[2] == 0 mean the reduction ran cooperatively
// (otherwise d / e / w are invalid).
// stamps: optional (NULL) 9 int64 cycle totals of workgroup 0's phases (diagnostics)
HARP_EXPORT int harp_eig_sym(double* A, long lda, int n, double* d, double* e, double* w, int nb_max, int* ws,
                             double* wsd, long long* stamps, hipStream_t s) {
  if (n < 1 || n > kMaxN || lda < n || nb_max < 1 || nb_max > kMaxNB || !ws || !wsd) return HARP_EBADARG;
  const int NB = harp_eig_workgroups(n, nb_max);
  if (NB < 1) return HARP_EUNSUPPORTED;
  const size_t lds1 = sizeof(double) * 2 * (size_t)n;
  if (lds1 > 32 * 1024 &&
      hipFuncSetAttribute((const void*)sytrd_coop_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1) !=
          hipSuccess)
    return HARP_ELAUNCH;
  sytrd_coop_kernel<<<dim3((unsigned)(NB * 8)), dim3(kT), lds1, s>>>(A, lda, n, d, e, NB, ws, wsd, stamps);
  int st = harp_launch_status();
  if (st != HARP_OK) return st;
  const size_t lds2 = sizeof(double) * 2 * (size_t)n;
  if (lds2 > 32 * 1024 &&
      hipFuncSetAttribute((const void*)tridiag_multisect_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds2) != hipSuccess)
    return HARP_ELAUNCH;
  const int blocks = (n * 16 + 255) / 256;
  tridiag_multisect_kernel<<<dim3((unsigned)blocks), dim3(256), lds2, s>>>(d, e, n, w);
  return harp_launch_status();
}
