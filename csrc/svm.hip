// Device-resident SMO for C-SVC (gfx950): every step of every binary machine runs on the
// GPU, no host round trip until the machine has converged.
//
// Reference: ml/daal/.../daal_svm/MultiClassDenseBatch/SVMDaalCollectiveMapper.java:179
// (DAAL svm training, boser SMO, inside multi_class_classifier one-against-one) and the
// libsvm-trained cascade of contrib/.../svm/SVMMapper.java:174-222.
//
// Algorithm: SMO with second-order working-set selection (WSS-2, Fan, Chen & Lin 2005),
// the same arithmetic as the PyTorch solver in harp_amd/models/svm.py (the test oracle):
//   i = argmax_{t in I_up} -y_t G_t,  stop if m(a) - M(a) < eps
//   j = argmin_{t in I_low, -y_t G_t < m} -(m + y_t G_t)^2 / max(K_ii + K_tt - 2 K_it, tau)
//   delta clipped to the box, a_i += y_i delta, a_j -= y_j delta,
//   G += y (y_i da_i K_i + y_j da_j K_j)
// Ties resolve to the lowest index (torch argmax / argmin). Products and sums are rounded
// one by one (no FMA contraction) so the trajectory follows the oracle's.
//
// Design: ONE workgroup per binary machine (one-vs-one machines of a multiclass problem run
// concurrently, one per CU): 1024 threads x <= 8 elements up to 8192 rows, else 512
// threads x <= 64 elements (n <= 32768). Thread t owns elements t + T k: their gradient G
// lives in registers for the whole solve and the box-state bits (a < C, a > 0, y > 0) in
// three bit masks; a machine's column list (multiclass) and, when it fits, its kernel
// diagonal sit in LDS. A step touches global memory only for the two kernel rows (gathered
// from the shared Gram matrix, L2/HBM: with the diagonal in LDS all of a thread's row-i
// loads are in flight at once, else 8-16 at a time) and the owners' two alphas, which are
// fetched under the reductions. Three block reductions per step (i; j; the broadcast of
// the update), whose operands the owners publish from registers. Measured (profiles/r3_svm): the first form, with the
// gradient in global memory and one element's gathers in flight at a time, spent ~44 us per
// step at n = 20k in serialized memory round trips.
#include "common.h"

#include <type_traits>

namespace {


struct ArgMax {
  double v;
  int i;
};

// better(a, b): a larger value, or an equal value at a lower index
__device__ __forceinline__ bool better_max(double va, int ia, double vb, int ib) {
  return va > vb || (va == vb && ia < ib);
}
__device__ __forceinline__ bool better_min(double va, int ia, double vb, int ib) {
  return va < vb || (va == vb && ia < ib);
}

// Wave reductions without the LDS crossbar: DPP inside each 16-lane row (row_ror 8, 4, then
// the two quad permutations: every lane ends with its row's result), then the four row
// results through v_readlane. (__shfl_xor compiles to ds_bpermute: six dependent LDS round
// trips per reduction, ~0.4 us, and a step runs six of them.)
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = dpp_i<CTRL>((int)(b & 0xffffffffll)), hi = dpp_i<CTRL>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_d(double x, int l) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <bool MAX>
__device__ __forceinline__ void arg_take(double& v, int& i, double ov, int oi) {
  if (MAX ? better_max(ov, oi, v, i) : better_min(ov, oi, v, i)) {
    v = ov;
    i = oi;
  }
}

template <bool MAX, int CTRL>
__device__ __forceinline__ void arg_dpp(double& v, int& i) {
  arg_take<MAX>(v, i, dpp_d<CTRL>(v), dpp_i<CTRL>(i));
}

template <bool MAX>
__device__ __forceinline__ void row_arg(double& v, int& i) {
  arg_dpp<MAX, 0x128>(v, i);  // row_ror:8
  arg_dpp<MAX, 0x124>(v, i);  // row_ror:4
  arg_dpp<MAX, 0x4E>(v, i);   // quad_perm [2,3,0,1]
  arg_dpp<MAX, 0xB1>(v, i);   // quad_perm [1,0,3,2]
}

// (value, index) arg-max / arg-min over the wave, ties to the lower index; uniform result
template <bool MAX>
__device__ __forceinline__ void wave_arg(double& v, int& i) {
  row_arg<MAX>(v, i);
  double r = readlane_d(v, 0);
  int ri = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
  for (int q = 16; q < 64; q += 16) arg_take<MAX>(r, ri, readlane_d(v, q), __builtin_amdgcn_readlane(i, q));
  v = r;
  i = ri;
}

__device__ __forceinline__ double row_min(double v) {
  v = fmin(v, dpp_d<0x128>(v));
  v = fmin(v, dpp_d<0x124>(v));
  v = fmin(v, dpp_d<0x4E>(v));
  return fmin(v, dpp_d<0xB1>(v));
}

__device__ __forceinline__ double wave_min(double v) {
  v = row_min(v);
  return fmin(fmin(readlane_d(v, 0), readlane_d(v, 16)), fmin(readlane_d(v, 32), readlane_d(v, 48)));
}

// block arg-reduction: each wave's result through LDS, then EVERY wave reduces the <= 16
// partials itself (one row of lanes), so no second barrier; the arrays are not written
// again before the step's closing barrier
template <bool MAX, int T>
__device__ __forceinline__ void block_arg(double& v, int& i, double* sv, int* si, int lane, int wv) {
  wave_arg<MAX>(v, i);
  if (lane == 0) {
    sv[wv] = v;
    si[wv] = i;
  }
  __syncthreads();
  const double id = MAX ? -__builtin_inf() : __builtin_inf();
  v = lane < T / 64 ? sv[lane] : id;
  i = lane < T / 64 ? si[lane] : 0x7fffffff;
  row_arg<MAX>(v, i);
  v = readlane_d(v, 0);
  i = __builtin_amdgcn_readlane(i, 0);
}

// Thread t owns elements t + T k (k < EPT): gradient G and three box-state bit masks in
// registers (IDENT: the machine is the whole matrix, column = element; else the columns in
// LDS). Gathers are issued GRP elements at a time, unconditionally, so a phase costs a few
// memory round trips, not one per element (the first form waited on every element's
// loads: ~28 us per step at n = 20k).
// elements whose gathers are in flight together: 8 at 1024 threads (128 registers), 16 at
// 512 threads (256 registers)
template <int T>
constexpr int grp() { return T >= 1024 ? 8 : 16; }

// KDL: the machine's kernel diagonal is staged once in LDS (when 8 n bytes fit beside the
// column list), so the j phase gathers only K row i and issues all of a thread's loads
// together (one memory round trip instead of three at 24 elements per thread)
template <int T, bool KDL, int EPT>
constexpr int grp2() { return KDL ? (EPT <= 16 ? EPT : 12) : grp<T>(); }

template <int EPT, bool IDENT, int T, bool KDL>
__global__ __launch_bounds__(T) void smo_kernel(const double* __restrict__ Kfull, long ldk,
                                                       const int* __restrict__ ids_all, const long* __restrict__ moff,
                                                       const double* __restrict__ y_all,
                                                       const double* __restrict__ kd_all, double* __restrict__ a_all,
                                                       double* __restrict__ g_all, int* __restrict__ iters, double C,
                                                       double eps, double tau, int max_iter, int kd_off) {
  __shared__ double s_v1[16], s_w1[16], s_v2[16];  // partials of the i and j reductions
  __shared__ int s_i1[16], s_i2[16];
  __shared__ double s_bc[8];
  constexpr int GRP = grp<T>();
  constexpr int GRP2 = grp2<T, KDL, EPT>();
  const int m = blockIdx.x;
  const long base = moff[m];
  const int n = (int)(moff[m + 1] - base);
  const int* ids = ids_all + base;
  const double* y = y_all + base;
  const double* kd = kd_all + base;
  double* a = a_all + base;
  double* g = g_all + base;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const double NEG = -__builtin_inf(), POS = __builtin_inf();

  double G[EPT];
  // machine-local column indices (not IDENT) and, with KDL, the diagonal (from byte
  // kd_off): staged once in LDS, read per phase
  extern __shared__ int s_col[];
  double* s_kd = reinterpret_cast<double*>(reinterpret_cast<char*>(s_col) + kd_off);
  // bit k: element tid + T k (64-bit masks past 32 elements per thread)
  using Mask = typename std::conditional<(EPT > 32), unsigned long long, unsigned>::type;
  constexpr Mask ONE = 1;
  Mask ypos = 0, ltC = 0, gt0 = 0;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int t = tid + T * k;
    G[k] = -1.0;
    if (t < n) {
      const double at = a[t];
      if (y[t] > 0) ypos |= ONE << k;
      if (at < C) ltC |= ONE << k;
      if (at > 0) gt0 |= ONE << k;
      G[k] = g[t];
      if constexpr (!IDENT) s_col[t] = ids[t];
      if constexpr (KDL) s_kd[t] = kd[t];
    }
  }
  __syncthreads();
#define COL(k, t) (IDENT ? (t) : s_col[t])
  int it = 0;
  for (; it < max_iter; ++it) {
    // an opaque copy of the thread id: keeps the per-element addresses from being hoisted
    // out of the step loop (EPT x 64-bit registers each) -- they are cheap to recompute
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    // ---- i = argmax over I_up of mg = -y G; Mv = min over I_low of mg (registers only)
    double bv = NEG, lo = POS;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int t = tid + T * k;
      if (t < n) {
        const bool yp = (ypos >> k) & 1, lc = (ltC >> k) & 1, g0 = (gt0 >> k) & 1;
        const double mg = yp ? -G[k] : G[k];
        const bool up = (yp && lc) || (!yp && g0);
        const bool low = (yp && g0) || (!yp && lc);
        if (up && better_max(mg, t, bv, bi)) {
          bv = mg;
          bi = t;
        }
        if (low) lo = fmin(lo, mg);
      }
    }
    lo = wave_min(lo);
    if (lane == 0) s_w1[wv] = lo;
    block_arg<true, T>(bv, bi, s_v1, s_i1, lane, wv);
    lo = lane < T / 64 ? s_w1[lane] : POS;
    const double mval = bv, Mv = readlane_d(row_min(lo), 0);
    const int i = bi;
    if (!(mval - Mv >= eps) || i >= n) break;  // converged (or no candidate: NaN-safe)
    // the owner of i fetches a_i now; it lands while the j phase runs (an element's alpha
    // is only ever read and written by its owner thread)
    double ai_pf = 0.0;
    if (tid == (i & (T - 1))) ai_pf = a[i];
    // ---- j: second-order selection over K row i
    const double* Ki = Kfull + (long)(IDENT ? i : ids[i]) * ldk;
    const double kii = KDL ? s_kd[i] : kd[i];
    double sv = POS, sat = 1.0;  // best candidate and its a_t (for the publish)
    int sj = 0x7fffffff;
    // gathers issued GRP elements at a time, unconditionally (clamped index), so they are
    // in flight together; the selection is predicated afterwards
    asm volatile("" : "+v"(tid));  // per-phase address recomputation (not kept live across phases)
#pragma unroll
    for (int k0 = 0; k0 < EPT; k0 += GRP2) {
      double kit[GRP2], kdt[GRP2];
#pragma unroll
      for (int u = 0; u < GRP2; ++u) {
        const int k = k0 + u;
        if (k < EPT) {
          const int t = tid + T * k, tc = t < n ? t : n - 1;
          kit[u] = Ki[COL(k, tc)];
          if constexpr (!KDL) kdt[u] = kd[tc];
        }
      }
#pragma unroll
      for (int u = 0; u < GRP2; ++u) {
        const int k = k0 + u;
        const int t = tid + T * k;
        if (k >= EPT || t >= n) continue;
        const bool yp = (ypos >> k) & 1, lc = (ltC >> k) & 1, g0 = (gt0 >> k) & 1;
        const double mg = yp ? -G[k] : G[k];
        const bool low = (yp && g0) || (!yp && lc);
        if (low && mg < mval) {
          const double bt = __dsub_rn(mval, mg);
          const double kdu = KDL ? s_kd[t] : kdt[u];
          double at = __dsub_rn(__dadd_rn(kii, kdu), __dmul_rn(2.0, kit[u]));
          if (!(at > 0)) at = tau;
          const double sc = -__ddiv_rn(__dmul_rn(bt, bt), at);
          if (better_min(sc, t, sv, sj)) {
            sv = sc;
            sj = t;
            sat = at;
          }
        }
      }
    }
    if (tid == (i & (T - 1))) {  // landed during the j phase; read after the publish barrier
      s_bc[6] = ai_pf;
      s_bc[7] = ((ypos >> (i / T)) & 1) ? 1.0 : -1.0;
    }
    // a thread's best candidate is the only one of its elements that can win: fetch its
    // alpha now, it lands during the reduction
    double aj_pf = 0.0;
    if (sj < n) aj_pf = a[sj];
    block_arg<false, T>(sv, sj, s_v2, s_i2, lane, wv);
    const int j = sj;
    if (j >= n) break;  // no admissible j (cannot happen while m - M >= eps)
    // ---- the owner of j publishes what the update needs, from registers: j is its own best
    // candidate (same order and tie rule), whose a_t was kept; y from the sign mask
    if (tid == (j & (T - 1))) {
      const int kj = j / T;
      double gj = 0.0;
#pragma unroll
      for (int q = 0; q < EPT; ++q)
        if (q == kj) gj = G[q];
      const bool yp = (ypos >> kj) & 1;
      s_bc[2] = __dsub_rn(mval, yp ? -gj : gj);  // bt_j
      s_bc[3] = sat;                               // at_j
      s_bc[4] = aj_pf;
      s_bc[5] = yp ? 1.0 : -1.0;
    }
    __syncthreads();
    const double btj = s_bc[2], atj = s_bc[3], aj = s_bc[4], yj = s_bc[5], ai = s_bc[6], yi = s_bc[7];
    double delta = __ddiv_rn(btj, atj);
    const double lim_i = yi > 0 ? __dsub_rn(C, ai) : ai;
    const double lim_j = yj > 0 ? aj : __dsub_rn(C, aj);
    delta = fmax(0.0, fmin(delta, fmin(lim_i, lim_j)));
    const double dai = __dmul_rn(yi, delta), daj = -__dmul_rn(yj, delta);
    const double nai = __dadd_rn(ai, dai), naj = __dadd_rn(aj, daj);
    // owners refresh the box bits (i != j: j has mg < m = mg_i)
    if (tid == (i & (T - 1))) {
      const int k = i / T;
      ltC = nai < C ? ltC | (ONE << k) : ltC & ~(ONE << k);
      gt0 = nai > 0 ? gt0 | (ONE << k) : gt0 & ~(ONE << k);
      a[i] = nai;
    }
    if (tid == (j & (T - 1))) {
      const int k = j / T;
      ltC = naj < C ? ltC | (ONE << k) : ltC & ~(ONE << k);
      gt0 = naj > 0 ? gt0 | (ONE << k) : gt0 & ~(ONE << k);
      a[j] = naj;
    }
    // ---- G += y (yi dai K_i + yj daj K_j)
    const double ci = __dmul_rn(yi, dai), cj = __dmul_rn(yj, daj);
    const double* Kj = Kfull + (long)(IDENT ? j : ids[j]) * ldk;
    asm volatile("" : "+v"(tid));
#pragma unroll
    for (int k0 = 0; k0 < EPT; k0 += GRP) {
      double ki[GRP], kj[GRP];
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int k = k0 + u;
        if (k < EPT) {
          const int t = tid + T * k, tc = t < n ? t : n - 1;
          const int c = COL(k, tc);
          ki[u] = Ki[c];
          kj[u] = Kj[c];
        }
      }
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int k = k0 + u;
        const int t = tid + T * k;
        if (k >= EPT || t >= n) continue;
        const double v = __dadd_rn(__dmul_rn(ci, ki[u]), __dmul_rn(cj, kj[u]));
        const double yt = ((ypos >> k) & 1) ? 1.0 : -1.0;
        G[k] = __dadd_rn(G[k], __dmul_rn(yt, v));
      }
    }
    __syncthreads();  // s_bc and the partial arrays are rewritten by the next step
  }
#undef COL
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int t = tid + T * k;
    if (t < n) g[t] = G[k];
  }
  if (tid == 0) iters[m] = it;
}

constexpr int kLdsMax = 160 * 1024 - 1024;  // dynamic LDS per workgroup (static arrays aside)

template <int EPT, bool IDENT, int T, bool KDL>
int run_smo(const double* K, long ldk, const int* ids, const long* moff, int nm, const double* y, const double* kd,
            double* a, double* g, int* iters, double C, double eps, double tau, int max_iter, int kd_off, int bytes,
            hipStream_t s) {
  const void* fn = (const void*)smo_kernel<EPT, IDENT, T, KDL>;
  if (bytes > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
    return HARP_ELAUNCH;
  smo_kernel<EPT, IDENT, T, KDL><<<dim3(nm), dim3(T), bytes, s>>>(K, ldk, ids, moff, y, kd, a, g, iters, C, eps, tau,
                                                                  max_iter, kd_off);
  return harp_launch_status();
}

// LDS: the column list (not ident; n ints), then the diagonal if it fits (n doubles, 8-aligned)
template <int EPT, int T>
int launch_smo(const double* K, long ldk, const int* ids, const long* moff, int nm, int max_n, const double* y,
               const double* kd, double* a, double* g, int* iters, double C, double eps, double tau, int max_iter,
               bool ident, hipStream_t s) {
  const int col_bytes = ident ? 0 : (int)sizeof(int) * max_n;
  const int kd_off = (col_bytes + 7) & ~7;
  const int kd_bytes = kd_off + (int)sizeof(double) * max_n;
  const bool kdl = T >= 1024 && kd_bytes <= kLdsMax;  // (512-thread forms run n > 24576: never fits)
#define RUN(ID, KL, BYTES) \
  return run_smo<EPT, ID, T, KL>(K, ldk, ids, moff, nm, y, kd, a, g, iters, C, eps, tau, max_iter, kd_off, BYTES, s)
  if constexpr (T >= 1024) {
    if (kdl) {
      if (ident) RUN(true, true, kd_bytes);
      RUN(false, true, kd_bytes);
    }
  }
  if (ident) RUN(true, false, 0);
  RUN(false, false, col_bytes);
#undef RUN
}

// ---- large machines over several CUs of ONE XCD each (cooperative SMO) ----------------
// A single machine on one CU is bound by that CU: its 160 KB kernel-row gathers, three
// block reductions and the fp64 candidate arithmetic of every element (~21 us per step at
// n = 20k, profiles/r3_svm). Here NB workgroups (one per CU) share the machine: thread g of
// participant b owns elements b T + g + NB T k (k < 4), with its gradient, alpha, diagonal
// AND its slice of kernel row i in registers (row i is gathered once per step; only row j is read
// in the update). A step has two cross-workgroup arg-reductions: each workgroup reduces its
// candidates, writes the winner (with everything the update needs from its owner: alpha,
// diagonal, label, b_t, a_t) to a slot, and arrives on a counter; every workgroup then reads
// all NB slots and reduces them identically, so all of them take the same decisions.
// Machines: XCD x trains machines x, x + 8, ... one after another (up to 8 at once, one
// per XCD). Coherence: a machine's participants all run on its XCD (workgroups read
// HW_REG_XCC_ID and claim a participant index in that XCD's own workspace), so its slots
// and counters live in one L2; stores complete (s_waitcnt) before the arrival, slots and
// counters are read with agent-scope loads that bypass the CU's L1. Slot sets are reused
// one step later, after a sync every participant must have passed after reading them.
// A wait gives up after ~1 s and raises the XCD's error word; the host checks it, and that
// all NB participants were claimed on every XCD that had a machine.
constexpr int kCoopT = 1024;
constexpr int kCoopMaxNB = 16;
// ws (int32, zeroed by the host), one block per XCD: [0] claims [1] arrivals i [2] arrivals
// j [3] error, then at int 16: 10 x 16 doubles of slots, then 2 x 16 ints
constexpr int kCoopXcdInts = 16 + 10 * 16 * 2 + 2 * 16;
constexpr int kCoopWsInts = 8 * kCoopXcdInts;

__device__ __forceinline__ double ld_agent(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_agent(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every thread's slot stores are complete, then thread 0 arrives and waits for all NB
__device__ __forceinline__ bool coop_arrive(int* cnt, int target, int* err, int* s_ok) {
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

template <int EPT, bool IDENT>
__global__ __launch_bounds__(kCoopT) void smo_coop_kernel(const double* __restrict__ Kfull, long ldk,
                                                          const int* __restrict__ ids_all,
                                                          const long* __restrict__ moff, int nm,
                                                          const double* __restrict__ y_all,
                                                          const double* __restrict__ kd_all,
                                                          double* __restrict__ a_all, double* __restrict__ g_all,
                                                          int* __restrict__ iters, double C, double eps, double tau,
                                                          int max_iter, int NB, int* ws_all) {
  constexpr int T = kCoopT;
  __shared__ double s_v1[16], s_w1[16], s_v2[16];
  __shared__ int s_i1[16], s_i2[16];
  __shared__ int s_b, s_ok;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int x = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7;  // HW_REG_XCC_ID
  if (x >= nm) return;  // no machine for this XCD
  int* ws = ws_all + x * kCoopXcdInts;
  if (tid == 0) s_b = atomicAdd(ws, 1);
  __syncthreads();
  const int b = s_b;
  if (b >= NB) return;
  int* err = ws + 3;
  double* sl = reinterpret_cast<double*>(ws + 16);
  double *A_v = sl, *A_lo = sl + 16, *A_a = sl + 32, *A_kd = sl + 48, *A_y = sl + 64;
  double *B_sc = sl + 80, *B_bt = sl + 96, *B_at = sl + 112, *B_a = sl + 128, *B_y = sl + 144;
  int* A_i = reinterpret_cast<int*>(sl + 160);
  int* B_j = A_i + 16;
  const int S = NB * T, g0 = b * T + tid;
  const double NEG = -__builtin_inf(), POS = __builtin_inf();
  int na = 0, nb = 0;  // this XCD's completed syncs on each counter (uniform over its participants)
  for (int m = x; m < nm; m += 8) {
  const long base = moff[m];
  const int n = (int)(moff[m + 1] - base);
  const int* ids = ids_all + base;
  const double* y = y_all + base;
  const double* kd = kd_all + base;
  double* a = a_all + base;
  double* g = g_all + base;
  double G[EPT], A[EPT], KD[EPT], KI[EPT];
  unsigned ypos = 0, ltC = 0, gt0 = 0;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int t = g0 + S * k;
    G[k] = -1.0;
    A[k] = 0.0;
    KD[k] = 1.0;
    if (t < n) {
      A[k] = a[t];
      G[k] = g[t];
      KD[k] = kd[t];
      if (y[t] > 0) ypos |= 1u << k;
      if (A[k] < C) ltC |= 1u << k;
      if (A[k] > 0) gt0 |= 1u << k;
    }
  }
#define COLC(t) (IDENT ? (t) : ids[t])
  int it = 0;
  for (; it < max_iter; ++it) {
    // ---- i: block arg-max of mg over I_up (and min over I_low), then across participants
    double bv = NEG, lo = POS;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int t = g0 + S * k;
      if (t < n) {
        const bool yp = (ypos >> k) & 1, lc = (ltC >> k) & 1, z0 = (gt0 >> k) & 1;
        const double mg = yp ? -G[k] : G[k];
        if (((yp && lc) || (!yp && z0)) && better_max(mg, t, bv, bi)) {
          bv = mg;
          bi = t;
        }
        if ((yp && z0) || (!yp && lc)) lo = fmin(lo, mg);
      }
    }
    lo = wave_min(lo);
    if (lane == 0) s_w1[wv] = lo;
    block_arg<true, T>(bv, bi, s_v1, s_i1, lane, wv);
    lo = lane < T / 64 ? s_w1[lane] : POS;
    lo = readlane_d(row_min(lo), 0);
    if (tid == 0) {
      A_v[b] = bv;
      A_lo[b] = lo;
      A_i[b] = bi;
    }
    if (bi < n && bi % S == g0) {  // the owner of this workgroup's candidate
      const int k = bi / S;
      A_a[b] = A[k];
      A_kd[b] = KD[k];
      A_y[b] = ((ypos >> k) & 1) ? 1.0 : -1.0;
    }
    if (!coop_arrive(ws + 1, NB * ++na, err, &s_ok)) return;
    double mval, Mv, ai, kii, yi;
    int i;
    {
      double v = NEG, w = POS, fa = 0.0, fk = 0.0, fy = 0.0;
      int ii = 0x7fffffff;
      if (lane < NB) {
        v = ld_agent(A_v + lane);
        w = ld_agent(A_lo + lane);
        ii = ld_agent(A_i + lane);
        fa = ld_agent(A_a + lane);
        fk = ld_agent(A_kd + lane);
        fy = ld_agent(A_y + lane);
      }
      row_arg<true>(v, ii);
      mval = readlane_d(v, 0);
      i = __builtin_amdgcn_readlane(ii, 0);
      Mv = readlane_d(row_min(w), 0);
      const int wb = i < n ? (i % S) / T : 0;
      ai = readlane_d(fa, wb);
      kii = readlane_d(fk, wb);
      yi = readlane_d(fy, wb);
    }
    if (!(mval - Mv >= eps) || i >= n) break;  // converged (the same decision everywhere)
    // ---- j: row i gathered once (kept for the update), second-order selection
    const double* Ki = Kfull + (long)(IDENT ? i : ids[i]) * ldk;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int t = g0 + S * k, tc = t < n ? t : n - 1;
      KI[k] = Ki[COLC(tc)];
    }
    double sv = POS, sat = 1.0, sbt = 0.0;
    int sj = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int t = g0 + S * k;
      if (t >= n) continue;
      const bool yp = (ypos >> k) & 1, lc = (ltC >> k) & 1, z0 = (gt0 >> k) & 1;
      const double mg = yp ? -G[k] : G[k];
      if (((yp && z0) || (!yp && lc)) && mg < mval) {
        const double bt = __dsub_rn(mval, mg);
        double at = __dsub_rn(__dadd_rn(kii, KD[k]), __dmul_rn(2.0, KI[k]));
        if (!(at > 0)) at = tau;
        const double sc = -__ddiv_rn(__dmul_rn(bt, bt), at);
        if (better_min(sc, t, sv, sj)) {
          sv = sc;
          sj = t;
          sat = at;
          sbt = bt;
        }
      }
    }
    const int my_j = sj;
    const double my_at = sat, my_bt = sbt;
    block_arg<false, T>(sv, sj, s_v2, s_i2, lane, wv);
    if (tid == 0) {
      B_sc[b] = sv;
      B_j[b] = sj;
    }
    if (sj < n && my_j == sj) {  // the owner of this workgroup's candidate
      const int k = sj / S;
      B_bt[b] = my_bt;
      B_at[b] = my_at;
      B_a[b] = A[k];
      B_y[b] = ((ypos >> k) & 1) ? 1.0 : -1.0;
    }
    if (!coop_arrive(ws + 2, NB * ++nb, err, &s_ok)) return;
    double btj, atj, aj, yj;
    int j;
    {
      double v = POS, fb = 0.0, ft = 1.0, fa = 0.0, fy = 0.0;
      int jj = 0x7fffffff;
      if (lane < NB) {
        v = ld_agent(B_sc + lane);
        jj = ld_agent(B_j + lane);
        fb = ld_agent(B_bt + lane);
        ft = ld_agent(B_at + lane);
        fa = ld_agent(B_a + lane);
        fy = ld_agent(B_y + lane);
      }
      row_arg<false>(v, jj);
      j = __builtin_amdgcn_readlane(jj, 0);
      const int wb = j < n ? (j % S) / T : 0;
      btj = readlane_d(fb, wb);
      atj = readlane_d(ft, wb);
      aj = readlane_d(fa, wb);
      yj = readlane_d(fy, wb);
    }
    if (j >= n) break;
    // ---- update (identical arithmetic in every thread), owners refresh alpha and box bits
    double delta = __ddiv_rn(btj, atj);
    const double lim_i = yi > 0 ? __dsub_rn(C, ai) : ai;
    const double lim_j = yj > 0 ? aj : __dsub_rn(C, aj);
    delta = fmax(0.0, fmin(delta, fmin(lim_i, lim_j)));
    const double dai = __dmul_rn(yi, delta), daj = -__dmul_rn(yj, delta);
    const double nai = __dadd_rn(ai, dai), naj = __dadd_rn(aj, daj);
    if (i % S == g0) {
      const int k = i / S;
#pragma unroll
      for (int q = 0; q < EPT; ++q)
        if (q == k) A[q] = nai;
      ltC = nai < C ? ltC | (1u << k) : ltC & ~(1u << k);
      gt0 = nai > 0 ? gt0 | (1u << k) : gt0 & ~(1u << k);
    }
    if (j % S == g0) {
      const int k = j / S;
#pragma unroll
      for (int q = 0; q < EPT; ++q)
        if (q == k) A[q] = naj;
      ltC = naj < C ? ltC | (1u << k) : ltC & ~(1u << k);
      gt0 = naj > 0 ? gt0 | (1u << k) : gt0 & ~(1u << k);
    }
    const double ci = __dmul_rn(yi, dai), cj = __dmul_rn(yj, daj);
    const double* Kj = Kfull + (long)(IDENT ? j : ids[j]) * ldk;
    double KJ[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int t = g0 + S * k, tc = t < n ? t : n - 1;
      KJ[k] = Kj[COLC(tc)];
    }
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const double v = __dadd_rn(__dmul_rn(ci, KI[k]), __dmul_rn(cj, KJ[k]));
      const double yt = ((ypos >> k) & 1) ? 1.0 : -1.0;
      G[k] = __dadd_rn(G[k], __dmul_rn(yt, v));
    }
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int t = g0 + S * k;
    if (t < n) {
      g[t] = G[k];
      a[t] = A[k];
    }
  }
  if (b == 0 && tid == 0) iters[m] = it;
  // the last step may have ended after the i sync: every participant has read those slots
  // before the next machine rewrites them
  if (!coop_arrive(ws + 2, NB * ++nb, err, &s_ok)) return;
  }
#undef COLC
}

template <int EPT>
int launch_coop(const double* K, long ldk, const int* ids, const long* moff, int nm, const double* y, const double* kd,
                double* a, double* g, int* iters, double C, double eps, double tau, int max_iter, int NB, bool ident,
                int* ws, hipStream_t s) {
  // NB x 8 workgroups: round-robin dispatch puts NB of them on each XCD
  const dim3 grid((unsigned)(NB * 8)), blk(kCoopT);
  if (ident)
    smo_coop_kernel<EPT, true><<<grid, blk, 0, s>>>(K, ldk, ids, moff, nm, y, kd, a, g, iters, C, eps, tau, max_iter,
                                                    NB, ws);
  else
    smo_coop_kernel<EPT, false><<<grid, blk, 0, s>>>(K, ldk, ids, moff, nm, y, kd, a, g, iters, C, eps, tau,
                                                     max_iter, NB, ws);
  return harp_launch_status();
}

}  // namespace

HARP_EXPORT int harp_svm_max_rows() { return 512 * 64; }

// nm binary machines; machine m owns entries [moff[m], moff[m+1]) of ids (row/col indices
// into the n x ldk fp64 Gram K), y (+-1), kd (the machine's K diagonal), a (alphas, in/out:
// usually zeros) and g (gradient, in/out: usually -1). max_n = the largest machine.
// `ident`: one machine whose ids are 0..n-1 (columns need no indirection).
HARP_EXPORT int harp_svm_smo(const double* K, long ldk, const int* ids, const long* moff, int nm, int max_n,
                             const double* y, const double* kd, double* a, double* g, int* iters, double C, double eps,
                             double tau, int max_iter, int ident, hipStream_t s) {
  if (nm <= 0 || max_n <= 0 || max_n > 512 * 64 || !(C > 0) || max_iter < 0) return HARP_EBADARG;
  if (ident && nm != 1) return HARP_EBADARG;
  // up to 24576 rows: 1024 threads x <= 24 elements (<= 128 registers); beyond: 512
  // threads with up to 64 elements each (256 registers per lane, the gradient still in registers)
#define SMO(E, TT) \
  return launch_smo<E, TT>(K, ldk, ids, moff, nm, max_n, y, kd, a, g, iters, C, eps, tau, max_iter, ident != 0, s)
  const int e1 = (max_n + 1023) / 1024;
  if (e1 <= 1) SMO(1, 1024);
  if (e1 <= 2) SMO(2, 1024);
  if (e1 <= 4) SMO(4, 1024);
  if (e1 <= 8) SMO(8, 1024);
  if (e1 <= 16) SMO(16, 1024);
  if (e1 <= 24) SMO(24, 1024);
  const int e2 = (max_n + 511) / 512;
  if (e2 <= 32) SMO(32, 512);
  if (e2 <= 40) SMO(40, 512);
  if (e2 <= 48) SMO(48, 512);
  SMO(64, 512);
#undef SMO
}

// nm machines (same layout as harp_svm_smo), each over NB (<= 16) CUs of one XCD
// (smo_coop_kernel; XCD x trains machines x, x + 8, ...). ws: a zeroed device int32 buffer
// of harp_svm_coop_ws_ints() words (8 blocks of harp_svm_coop_xcd_ints()); afterwards, for
// every XCD x < min(nm, 8), block x word 0 >= NB (all participants ran) and word 3 == 0
// (no wait gave up) mean its machines' results are valid.
HARP_EXPORT int harp_svm_coop_ws_ints() { return kCoopWsInts; }
HARP_EXPORT int harp_svm_coop_xcd_ints() { return kCoopXcdInts; }
HARP_EXPORT int harp_svm_coop_max_rows(int NB) { return NB * kCoopT * 4; }

HARP_EXPORT int harp_svm_smo_coop(const double* K, long ldk, const int* ids, const long* moff, int nm, int max_n,
                                  const double* y, const double* kd, double* a, double* g, int* iters, double C,
                                  double eps, double tau, int max_iter, int NB, int ident, int* ws, hipStream_t s) {
  if (nm <= 0 || max_n <= 0 || NB < 1 || NB > kCoopMaxNB || !(C > 0) || max_iter < 0 || !ws || !ids ||
      (ident && nm != 1))
    return HARP_EBADARG;
  const int e = (max_n + NB * kCoopT - 1) / (NB * kCoopT);
#define COOP(E) \
  return launch_coop<E>(K, ldk, ids, moff, nm, y, kd, a, g, iters, C, eps, tau, max_iter, NB, ident != 0, ws, s)
  if (e <= 1) COOP(1);
  if (e <= 2) COOP(2);
  if (e <= 3) COOP(3);
  if (e <= 4) COOP(4);  // (more elements per thread spill: 10 registers each plus addresses)
#undef COOP
  return HARP_EUNSUPPORTED;
}
