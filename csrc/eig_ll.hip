// Householder tridiagonalisation of a symmetric fp64 matrix (n <= 1024) spread over the
// whole chip, with the matrix resident in registers and ONE data-tagged exchange per column.
//
// Reference: the PCA step-3 eigen-decomposition on the master,
// ml/daal/src/main/java/edu/iu/daal_pca/cordensedistr/PCADaalCollectiveMapper.java:121-154.
//
// Why a second reduction next to csrc/eig.hip's one-XCD form: that kernel streams the trailing
// block through L2 every column and pays ~10 us per column in block reductions, barriers and
// its arrival (profiles/r4_eigh: 10 ms of the 11.2 ms eigh at n = 1000). Here:
//  * workgroup b (256 threads, one wave per SIMD) keeps rows [RW b, RW b + RW) of the
//    panel-start matrix in VGPRs; thread i owns indices 4 i .. 4 i + 3 of every vector, and
//    every workgroup carries the whole vector state (x, v, w and the panel's V / W columns)
//    redundantly, so only two n-vectors cross workgroups per column;
//  * the two-sided update is deferred over panels of NBP columns (LAPACK dlatrd): p = tau
//    (A_ps v - V (W^T v) - W (V^T v)), and the next column is A_ps[:, k+1] minus the panel's
//    corrections, so no workgroup waits for another's rank-2 update;
//  * v = scl x + gamma e_{k+1} is affine in the column x, so EVERY per-column reduction (the
//    Householder norm, the panel dots W^T x / V^T x and this workgroup's RW row dots A_ps x)
//    is ONE 16-slot butterfly per wave (v_permlane32_swap / v_permlane16_swap, then DPP
//    mirrors) and one LDS pass -- two __syncthreads per column in all;
//  * the exchange is the data itself: each p_k[r] (and each workgroup's partial p.v) is
//    written as two 8-byte {tag = k + 1, 32 data bits} granules by single agent-scope (sc1)
//    stores, and consumers poll exactly the granules they need with agent-scope loads -- no
//    counter, no flag, no fence (cdna_hip_programming.md Guideline 16, R2). Owners publish
//    the next panel's columns of A_ps the same way a panel ahead of their use.
// Workgroups whose rows are all reduced leave early; the last one writes d, e, tau and the
// reflectors (vout row k = v_k, for the compact-WY back-transform of ops/eig.py).
#include "common.h"

namespace {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;

constexpr int kT = 256;         // threads per workgroup: one wave per SIMD
constexpr int kIPT = 4;         // vector indices per thread (contiguous)
constexpr int kN = kT * kIPT;   // largest n
constexpr int kMaxWG = 256;     // granule slots for the per-workgroup partial p.v
constexpr int kSlots = 16;      // butterfly width
constexpr long kSpinLimit = 1L << 21;

// granule area (u64 words), zeroed by the host before every call
constexpr long kOffP = 0;                          // [2][kN][2]  p_k, parity k & 1
constexpr long kOffPV = kOffP + 2L * kN * 2;       // [2][kMaxWG][2]  partial p.v per workgroup
constexpr long kOffCol = kOffPV + 2L * kMaxWG * 2; // [2][NBP][kN][2]  published A_ps rows
constexpr long gran_words(int nbp) { return kOffCol + 2L * nbp * kN * 2; }

__device__ __forceinline__ u64 gload(const gu64* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(gu64* g, u64 v) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one fp64 value as two granules {tag, low word} {tag, high word}
__device__ __forceinline__ void put_d(gu64* g, unsigned tag, double v) {
  const u64 u = __builtin_bit_cast(u64, v);
  gstore(g, ((u64)tag << 32) | (u & 0xffffffffull));
  gstore(g + 1, ((u64)tag << 32) | (u >> 32));
}
__device__ __forceinline__ bool tagged(u64 lo, u64 hi, unsigned tag) {
  return (unsigned)(lo >> 32) == tag && (unsigned)(hi >> 32) == tag;
}
__device__ __forceinline__ double join_d(u64 lo, u64 hi) {
  return __builtin_bit_cast(double, ((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull));
}

// fp64 pair exchange across lane halves (gfx950 permlane swaps, both 32-bit halves)
__device__ __forceinline__ void swap32(double& a, double& b) {
  const u64 ua = __builtin_bit_cast(u64, a), ub = __builtin_bit_cast(u64, b);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = __builtin_bit_cast(double, ((u64)hi[0] << 32) | lo[0]);
  b = __builtin_bit_cast(double, ((u64)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ void swap16(double& a, double& b) {
  const u64 ua = __builtin_bit_cast(u64, a), ub = __builtin_bit_cast(u64, b);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = __builtin_bit_cast(double, ((u64)hi[0] << 32) | lo[0]);
  b = __builtin_bit_cast(double, ((u64)hi[1] << 32) | lo[1]);
}

// Transposed wave sum of 16 slots: afterwards lane l holds the wave total of slot
// 8 b5 + 4 b4 + 2 b3 + b2 (b_i = bit i of l); lanes l, l^1, l^2, l^3 hold the same bits.
// Pairings: xor 32 (permlane32 swap), xor 16 (permlane16 swap), xor 15 (row_mirror),
// xor 7 (row_half_mirror), xor 2, xor 1 (quad_perm) -- together they span all 64 lanes.
__device__ __forceinline__ double butterfly16(double (&s)[kSlots], int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    swap32(s[i], s[i + 8]);
    s[i] += s[i + 8];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    swap16(s[i], s[i + 4]);
    s[i] += s[i + 4];
  }
  const bool b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double keep = b3 ? s[i + 2] : s[i], send = b3 ? s[i] : s[i + 2];
    s[i] = keep + dpp_mov_d<0x140>(send);  // row_mirror
  }
  {
    const double keep = b2 ? s[1] : s[0], send = b2 ? s[0] : s[1];
    s[0] = keep + dpp_mov_d<0x141>(send);  // row_half_mirror
  }
  s[0] += dpp_mov_d<0x4E>(s[0]);  // quad_perm [2,3,0,1]
  s[0] += dpp_mov_d<0xB1>(s[0]);  // quad_perm [1,0,3,2]
  return s[0];
}
__device__ __forceinline__ int butterfly_slot(int lane) {
  return ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
}

// 1 / x by v_rcp_f64 and two Newton steps (the IEEE divide is a ~10-instruction dependent chain)
__device__ __forceinline__ double rcp_d(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}

// workgroup barrier for LDS traffic only: __syncthreads() also drains vmcnt, i.e. waits for
// the granule stores and for the column prefetch issued a phase earlier
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ bool spin_fail(long& spins, int* err) {
  if (++spins > kSpinLimit) {
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  if ((spins & 63) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
  if (spins > 32) __builtin_amdgcn_s_sleep(1);
  return false;
}

// A: n x n symmetric (lda; read only). d[n], e[n-1]: the tridiagonal; vout (nullable, n x ldv
// row-major, zeroed): row k = v_k (v_k[k + 1] = 1, zeros before); tauout (nullable, zeroed).
// ws[2]: error word (zeroed); gran: gran_words(NBP) u64, zeroed. Grid: ceil(n / RW) workgroups.
template <int RW, int NBP>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(1, 1))) void sytrd_ll_kernel(
    const double* __restrict__ A, long lda, int n, double* __restrict__ dout, double* __restrict__ eout,
    double* __restrict__ vout, long ldv, double* __restrict__ tauout, int* __restrict__ ws, u64* __restrict__ gran_,
    long long* __restrict__ stamps, long long* __restrict__ trace) {
  static_assert(1 + RW + 2 * (NBP - 1) <= kSlots, "butterfly slots");
  constexpr int kBc = 1 + RW + 2 * NBP;  // alpha, A_ps[r][k+1] (own rows), V[k+1][l], W[k+1][l]
  __shared__ double sP[2][kT / 64][kSlots];  // parity: no barrier separates a column's read from the next write
  __shared__ double sBc[2][kBc];
  __shared__ double sB2[2 + 2 * RW];    // p.v total, p[k+1], then p and v of the own rows
  __shared__ double sRow[RW][NBP][2];   // V / W of the own rows over the panel
  gu64* gran = (gu64*)gran_;
  int* err = ws + 2;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x, NB = gridDim.x;
  const int r0 = b * RW;
  const bool last = b == NB - 1;
  const int t0 = tid * kIPT;
  if (n < 3) {
    if (last && tid == 0) {
      dout[0] = A[0];
      if (n == 2) {
        eout[0] = A[1];
        dout[1] = A[1 + lda];
      }
    }
    return;
  }
  // registers: own rows of A_ps, the panel's V / W at own indices, the current column x'
  double a[RW][kIPT], Vw[NBP][kIPT], Ww[NBP][kIPT], x[kIPT];
#pragma unroll
  for (int i = 0; i < RW; ++i)
#pragma unroll
    for (int m = 0; m < kIPT; ++m) {
      const int r = r0 + i, t = t0 + m;
      a[i][m] = r < n && t < n ? A[t + (long)r * lda] : 0.0;
    }
#pragma unroll
  for (int l = 0; l < NBP; ++l)
#pragma unroll
    for (int m = 0; m < kIPT; ++m) Vw[l][m] = Ww[l][m] = 0.0;
#pragma unroll
  for (int m = 0; m < kIPT; ++m) {
    const int t = t0 + m;
    x[m] = t >= 1 && t < n ? A[t] : 0.0;  // column 0 below the diagonal
  }
  if (last && tid == 0) dout[0] = A[0];
  // diagnostic (stamps != nullptr): thread 0 of the last workgroup sums cycles per phase and
  // its poll iterations: [0] local sums + butterfly, [1] sync + p, [2] exchange, [3] S4,
  // [4] panel end, [5] poll iterations
  const bool stamp = stamps != nullptr && last && tid == 0;
  long long ph[6] = {0, 0, 0, 0, 0, 0}, t_last = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {
    if (stamp) {
      const long long now = (long long)__builtin_amdgcn_s_memtime();
      ph[i] += now - t_last;
      t_last = now;
    }
  };

  // diagnostic (trace != nullptr): thread 0 of every workgroup records the chip-wide 100 MHz
  // clock at four points of every 64th column: trace[(k / 64) NB 4 + b 4 + {start, p stored,
  // exchange done, step done}]
  const bool tr = trace != nullptr && tid == 0;
  auto tmark = [&](int k, int i) {
    if (tr && (k & 63) == 0) trace[((long)(k >> 6) * NB + b) * 4 + i] = (long long)__builtin_amdgcn_s_memrealtime();
  };

  // A_ps[k+1][own indices] for the coming step, prefetched one step ahead as raw granule pairs
  // (checked only in that step's exchange, so the loads fly under its local phase)
  u64 clo[kIPT], chi[kIPT];
  auto prefetch_col = [&](int kk) {
    const int pn = kk / NBP, jn = kk % NBP;
    const gu64* gc = gran + kOffCol + ((long)(pn & 1) * NBP + jn) * kN * 2;
#pragma unroll
    for (int m = 0; m < kIPT; ++m) {
      const int t = t0 + m;
      clo[m] = chi[m] = 0;
      if (pn > 0 && t >= kk + 1 && t < n) {
        clo[m] = gload(gc + 2 * t);
        chi[m] = gload(gc + 2 * t + 1);
      }
    }
  };
  prefetch_col(0);
  // the loop's first uses of a / x must not look like they wait on loads still in flight
  // (the waitcnt pass merges the loop header conservatively: one drain here, none per column)
  __builtin_amdgcn_s_waitcnt(0);

  for (int k = 0; k + 2 < n; ++k) {
    const int j = k % NBP, panel = k / NBP, par = k & 1;
    if (r0 + RW - 1 < k + 1 && !last) return;  // every own row reduced: nobody polls us again
    tmark(k, 0);
    const int k1 = k + 1;
    // ---- S1: the owner of index k+1 posts alpha, A_ps[own rows][k+1], V / W[k+1][l < j]
    if (tid == k1 / kIPT) {
      const int mk = k1 % kIPT;
#pragma unroll
      for (int m = 0; m < kIPT; ++m)
        if (m == mk) {
          sBc[par][0] = x[m];
#pragma unroll
          for (int i = 0; i < RW; ++i) sBc[par][1 + i] = a[i][m];
#pragma unroll
          for (int l = 0; l < NBP; ++l) {
            sBc[par][1 + RW + 2 * l] = Vw[l][m];
            sBc[par][2 + RW + 2 * l] = Ww[l][m];
          }
        }
    }
    // local slot sums: 0 sigma (t >= k+2), 1..RW row dots A_ps[r] . x', then W_l . x', V_l . x'
    if (4 * (wv * 64 + 63) + 3 >= k1) {
      double s[kSlots];
#pragma unroll
      for (int q = 0; q < kSlots; ++q) s[q] = 0.0;
#pragma unroll
      for (int m = 0; m < kIPT; ++m) {
        const double xm = x[m];
        if (t0 + m >= k1 + 1) s[0] = fma(xm, xm, s[0]);
#pragma unroll
        for (int i = 0; i < RW; ++i) s[1 + i] = fma(a[i][m], xm, s[1 + i]);
#pragma unroll
        for (int l = 0; l < NBP - 1; ++l)
          if (l < j) {
            s[1 + RW + 2 * l] = fma(Ww[l][m], xm, s[1 + RW + 2 * l]);
            s[2 + RW + 2 * l] = fma(Vw[l][m], xm, s[2 + RW + 2 * l]);
          }
      }
      const double tot = butterfly16(s, lane);
      if ((lane & 3) == 0) sP[par][wv][butterfly_slot(lane)] = tot;
    } else if (lane < kSlots) {
      sP[par][wv][lane] = 0.0;
    }
    mark(0);
    lds_barrier();
    double tot = 0.0;
    if (lane < kSlots) tot = (sP[par][0][lane] + sP[par][1][lane]) + (sP[par][2][lane] + sP[par][3][lane]);
    const double sigma = readlane_d(tot, 0);
    const double alpha = sBc[par][0];
    double beta = alpha, tau = 0.0, scl = 0.0;
    if (sigma != 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
      tau = (beta - alpha) * rcp_d(beta);
      scl = rcp_d(alpha - beta);
    }
    const double gam = sigma != 0.0 ? -beta * scl : 1.0;  // v = scl x' + gam e_{k+1}
    double v[kIPT];
#pragma unroll
    for (int m = 0; m < kIPT; ++m) {
      const int t = t0 + m;
      v[m] = t == k1 ? 1.0 : (t > k1 ? scl * x[m] : 0.0);
      Vw[j][m] = v[m];
    }
    // ---- S1 finish: p for the own rows (threads owning indices r0 .. r0 + RW - 1)
    constexpr int kOwn = RW / kIPT;
    const int h = tid - r0 / kIPT;
    if (h >= 0 && h < kOwn) {
      // uniform across the owning lanes: g_l = W_l . v, u_l = V_l . v
      double gW[NBP], gV[NBP];
#pragma unroll
      for (int l = 0; l < NBP - 1; ++l) {
        gW[l] = gV[l] = 0.0;
        if (l < j) {
          gW[l] = fma(scl, readlane_d(tot, 1 + RW + 2 * l), gam * sBc[par][2 + RW + 2 * l]);
          gV[l] = fma(scl, readlane_d(tot, 2 + RW + 2 * l), gam * sBc[par][1 + RW + 2 * l]);
        }
      }
      double pv = 0.0;
      gu64* gp = gran + kOffP + (long)par * kN * 2;
#pragma unroll
      for (int m = 0; m < kIPT; ++m) {
        double q = 0.0;
#pragma unroll
        for (int hh = 0; hh < kOwn; ++hh)
          if (hh == h) q = readlane_d(tot, 1 + hh * kIPT + m);
        const int r = r0 + h * kIPT + m;
        q = fma(scl, q, gam * sBc[par][1 + h * kIPT + m]);
#pragma unroll
        for (int l = 0; l < NBP - 1; ++l)
          if (l < j) q -= fma(Vw[l][m], gW[l], Ww[l][m] * gV[l]);
        const double p = tau * q;
        sB2[2 + h * kIPT + m] = p;
        sB2[2 + RW + h * kIPT + m] = v[m];
        sRow[h * kIPT + m][j][0] = v[m];
        if (r >= k1 && r < n) {
          put_d(gp + 2L * r, (unsigned)k1, p);
          pv = fma(p, v[m], pv);
        }
      }
      // partial p.v of this workgroup: the kOwn owner lanes are adjacent (kOwn <= 4)
      if (kOwn >= 2) pv += dpp_mov_d<0xB1>(pv);
      if (kOwn >= 4) pv += dpp_mov_d<0x4E>(pv);
      if (h == 0) put_d(gran + kOffPV + (long)par * kMaxWG * 2 + 2L * b, (unsigned)k1, pv);
    }
    mark(1);
    tmark(k, 1);
    // ---- S3: the exchange. p_k at own indices, A_ps[k+1][own indices], partial p.v sums
    double p[kIPT], col[kIPT];
    {
      const gu64* gp = gran + kOffP + (long)par * kN * 2;
      const gu64* gc = gran + kOffCol + ((long)(panel & 1) * NBP + j) * kN * 2;
      const gu64* gv = gran + kOffPV + (long)par * kMaxWG * 2;
      const int blo = k1 / RW;
      double pvs = 0.0, pvq[kMaxWG / 64];
      // what this lane still waits for (bit m: p[m], bit 4 + m: col[m], bit 8 + q: partial q);
      // a granule pair once seen with its tag is kept and never re-read
      unsigned need = 0;
#pragma unroll
      for (int m = 0; m < kIPT; ++m) {
        const int t = t0 + m;
        p[m] = col[m] = 0.0;
        if (t >= k1 && t < n) {
          need |= 1u << m;
          if (panel == 0)
            col[m] = A[t + (long)k1 * lda];
          else if (tagged(clo[m], chi[m], (unsigned)panel + 1))
            col[m] = join_d(clo[m], chi[m]);
          else
            need |= 1u << (4 + m);
        }
      }
      if (wv == 0) {  // wave 0 sums the partial p.v of every live workgroup
#pragma unroll
        for (int q = 0; q < kMaxWG / 64; ++q) {
          pvq[q] = 0.0;
          const int bb = lane + 64 * q;
          if (bb >= blo && bb < NB) need |= 1u << (8 + q);
        }
      }
      long spins = 0;
      for (;;) {
#pragma unroll
        for (int m = 0; m < kIPT; ++m) {
          const int t = t0 + m;
          if (need & (1u << m)) {
            const u64 lo = gload(gp + 2 * t), hi = gload(gp + 2 * t + 1);
            if (tagged(lo, hi, (unsigned)k1)) {
              p[m] = join_d(lo, hi);
              need &= ~(1u << m);
            }
          }
          if (need & (1u << (4 + m))) {
            const u64 lo = gload(gc + 2 * t), hi = gload(gc + 2 * t + 1);
            if (tagged(lo, hi, (unsigned)panel + 1)) {
              col[m] = join_d(lo, hi);
              need &= ~(1u << (4 + m));
            }
          }
        }
        if (wv == 0) {
#pragma unroll
          for (int q = 0; q < kMaxWG / 64; ++q) {
            if (need & (1u << (8 + q))) {
              const int bb = lane + 64 * q;
              const u64 lo = gload(gv + 2 * bb), hi = gload(gv + 2 * bb + 1);
              if (tagged(lo, hi, (unsigned)k1)) {
                pvq[q] = join_d(lo, hi);
                need &= ~(1u << (8 + q));
              }
            }
          }
        }
        const bool ok = need == 0;
        if (stamp) ++ph[5];
        if (__all(ok)) break;
        if (spin_fail(spins, err)) return;
      }
      if (wv == 0) {
#pragma unroll
        for (int q = 0; q < kMaxWG / 64; ++q) pvs += pvq[q];
        pvs = wave_sum_d_dpp(pvs);
        if (lane == 0) sB2[0] = pvs;
      }
      if (tid == k1 / kIPT) {
#pragma unroll
        for (int m = 0; m < kIPT; ++m)
          if (t0 + m == k1) sB2[1] = p[m];
      }
    }
    mark(2);
    tmark(k, 2);
    // (measured: letting every wave poll the partial sums itself to drop this barrier on
    // non-panel columns cost more polling traffic than the barrier: 6.8 -> 7.8 ms)
    lds_barrier();
    const double c = 0.5 * tau * sB2[0];
#pragma unroll
    for (int m = 0; m < kIPT; ++m) Ww[j][m] = t0 + m >= k1 ? fma(-c, v[m], p[m]) : 0.0;
    if (h >= 0 && h < kOwn) {
#pragma unroll
      for (int m = 0; m < kIPT; ++m) sRow[h * kIPT + m][j][1] = fma(-c, v[m], sB2[2 + h * kIPT + m]);
    }
    // ---- S4: column k+1 of A_{k+1} = A_ps[:, k+1] - sum_{l <= j} (V_l W[k+1][l] + W_l V[k+1][l])
    double Vk[NBP], Wk[NBP];
#pragma unroll
    for (int l = 0; l < NBP; ++l) {
      Vk[l] = l < j ? sBc[par][1 + RW + 2 * l] : 0.0;
      Wk[l] = l < j ? sBc[par][2 + RW + 2 * l] : 0.0;
    }
#pragma unroll
    for (int l = 0; l < NBP; ++l)
      if (l == j) {
        Vk[l] = 1.0;
        Wk[l] = fma(-c, 1.0, sB2[1]);
      }
    double xn[kIPT];
#pragma unroll
    for (int m = 0; m < kIPT; ++m) {
      double y = col[m];
#pragma unroll
      for (int l = 0; l < NBP; ++l)
        if (l <= j) y -= fma(Vw[l][m], Wk[l], Ww[l][m] * Vk[l]);
      xn[m] = t0 + m >= k1 ? y : 0.0;
    }
    if (last) {
      if (tid == 0) {
        eout[k] = beta;
        if (tauout) tauout[k] = tau;
      }
#pragma unroll
      for (int m = 0; m < kIPT; ++m) {
        const int t = t0 + m;
        if (t == k1) dout[k1] = xn[m];
        if (vout && t >= k1 && t < n) vout[(long)k * ldv + t] = v[m];
      }
    }
    mark(3);
    tmark(k, 3);
    if (k + 3 >= n) {  // last Householder step: e[n-2] = x[n-1], d[n-1] from A_ps
      if (last) {
#pragma unroll
        for (int m = 0; m < kIPT; ++m) {
          const int t = t0 + m;
          if (t == n - 1) {
            eout[n - 2] = xn[m];
            double dd = 0.0;
#pragma unroll
            for (int i = 0; i < RW; ++i)
              if (r0 + i == n - 1) dd = a[i][m];
#pragma unroll
            for (int l = 0; l < NBP; ++l)
              if (l <= j) dd -= 2.0 * Vw[l][m] * Ww[l][m];
            dout[n - 1] = dd;
          }
        }
      }
      break;
    }
#pragma unroll
    for (int m = 0; m < kIPT; ++m) x[m] = t0 + m >= k1 + 1 ? xn[m] : 0.0;
    // ---- panel end: A_ps -= V W^T + W V^T on the own rows, then publish the next panel's rows
    if (j == NBP - 1) {
      const int k0n = k + 1;  // first column of the next panel
      if (r0 + RW - 1 >= k0n) {
#pragma unroll
        for (int i = 0; i < RW; ++i) {
          if (r0 + i < k0n) continue;
          double rv[NBP], rw[NBP];
#pragma unroll
          for (int l = 0; l < NBP - 1; ++l) {
            rv[l] = sRow[i][l][0];
            rw[l] = sRow[i][l][1];
          }
          // this column's pair: sRow[i][j][1] is being written in this phase by its owner
          rv[NBP - 1] = sB2[2 + RW + i];
          rw[NBP - 1] = fma(-c, sB2[2 + RW + i], sB2[2 + i]);
#pragma unroll
          for (int m = 0; m < kIPT; ++m) {
            double y = a[i][m];
#pragma unroll
            for (int l = 0; l < NBP; ++l) y -= fma(rv[l], Ww[l][m], rw[l] * Vw[l][m]);
            a[i][m] = y;
          }
        }
        // columns k0n + 1 .. k0n + NBP of the new A_ps at this workgroup's rows (by symmetry
        // the rows the consumers need): posted by the threads owning those column indices,
        // RW values each, so no workgroup bursts a whole row
        const int np = panel + 1;
        gu64* gc = gran + kOffCol + (long)(np & 1) * NBP * kN * 2;
#pragma unroll
        for (int m = 0; m < kIPT; ++m) {
          const int c = t0 + m, jj = c - (k0n + 1);
          if (jj < 0 || jj >= NBP || c >= n) continue;
#pragma unroll
          for (int i = 0; i < RW; ++i) {
            const int r = r0 + i;
            if (r >= c && r < n) put_d(gc + ((long)jj * kN + r) * 2, (unsigned)np + 1, a[i][m]);
          }
        }
      }
    }
    prefetch_col(k + 1);
    mark(4);
  }
  if (stamp)
    for (int i = 0; i < 6; ++i) stamps[i] = ph[i];
}

template <int RW, int NBP>
int launch_ll(const double* A, long lda, int n, double* d, double* e, double* V, long ldv, double* tau, int* ws,
              u64* gran, long long* stamps, long long* trace, hipStream_t s) {
  const int nb = (n + RW - 1) / RW;
  if (nb > kMaxWG) return HARP_EUNSUPPORTED;
  sytrd_ll_kernel<RW, NBP><<<dim3((unsigned)nb), dim3(kT), 0, s>>>(A, lda, n, d, e, V, ldv, tau, ws, gran, stamps,
                                                                                          trace);
  return harp_launch_status();
}

}  // namespace

constexpr int kLLRW = 8, kLLNBP = 4;
static long long* g_ll_stamps = nullptr;  // diagnostic phase cycles (harp_sytrd_ll_stamps)
static long long* g_ll_trace = nullptr;   // diagnostic per-workgroup clock marks (harp_sytrd_ll_trace)
// diagnostic: the next launches record every workgroup's 100 MHz clock at four points of every
// 64th column (ceil((n - 2) / 64) x workgroups x 4 int64)
HARP_EXPORT void harp_sytrd_ll_trace(long long* trace) { g_ll_trace = trace; }
// diagnostic: the next launches sum the last workgroup's cycles per phase into stamps[0..5]
HARP_EXPORT void harp_sytrd_ll_stamps(long long* stamps) { g_ll_stamps = stamps; }

HARP_EXPORT int harp_sytrd_ll_max_n() { return kN; }
// zeroed u64 words of granule state the reduction needs per call
HARP_EXPORT long harp_sytrd_ll_gran_words() { return gran_words(kLLNBP); }
HARP_EXPORT int harp_sytrd_ll_workgroups(int n) { return n < 1 ? 0 : (n + kLLRW - 1) / kLLRW; }

// Tridiagonalisation A = Q T Q^T with Q = H_0 ... H_{n-3}, H_k = I - tau_k v_k v_k^T; V (nullable):
// n x ldv row-major, zeroed, row k = v_k; tau (nullable): n doubles, zeroed. A is not modified.
// ws: zeroed harp_eig_ws_ints() int32 (ws[2] != 0 afterwards: a workgroup timed out waiting,
// the outputs are invalid); gran: zeroed harp_sytrd_ll_gran_words() u64. All
// harp_sytrd_ll_workgroups(n) workgroups must be co-resident (one per CU).
HARP_EXPORT int harp_sytrd_ll(const double* A, long lda, int n, double* d, double* e, double* V, long ldv, double* tau,
                              int* ws, unsigned long long* gran, hipStream_t s) {
  if (n < 1 || n > kN || lda < n || !ws || !gran || !d || !e || (V && ldv < n)) return HARP_EBADARG;
  return launch_ll<kLLRW, kLLNBP>(A, lda, n, d, e, V, ldv, tau, ws, gran, g_ll_stamps, g_ll_trace, s);
}
