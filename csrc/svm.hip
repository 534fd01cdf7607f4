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
// three bit masks; a machine's column list (multiclass) sits in LDS. A step touches
// global memory only for the two kernel rows (gathered from the shared Gram matrix,
// L2/HBM, 8 elements' loads in flight at a time) and the diagonal. Three block
// reductions per step (i; j; the broadcast of the update). Measured (profiles/r3_svm): the first form, with the
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

template <bool MAX>
__device__ __forceinline__ void wave_arg(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (MAX ? better_max(ov, oi, v, i) : better_min(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
}

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
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

template <int EPT, bool IDENT, int T>
__global__ __launch_bounds__(T) void smo_kernel(const double* __restrict__ Kfull, long ldk,
                                                       const int* __restrict__ ids_all, const long* __restrict__ moff,
                                                       const double* __restrict__ y_all,
                                                       const double* __restrict__ kd_all, double* __restrict__ a_all,
                                                       double* __restrict__ g_all, int* __restrict__ iters, double C,
                                                       double eps, double tau, int max_iter) {
  __shared__ double s_v[16], s_w[16];
  __shared__ int s_i[16];
  __shared__ double s_bc[8];
  __shared__ int s_ic[4];
  constexpr int GRP = grp<T>();
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
  // machine-local column indices (not IDENT): staged once in LDS, read per phase
  extern __shared__ int s_col[];
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
    wave_arg<true>(bv, bi);
    lo = wave_min(lo);
    if (lane == 0) {
      s_v[wv] = bv;
      s_i[wv] = bi;
      s_w[wv] = lo;
    }
    __syncthreads();
    if (wv == 0) {
      double v = lane < (T / 64) ? s_v[lane] : NEG, w = lane < (T / 64) ? s_w[lane] : POS;
      int i = lane < (T / 64) ? s_i[lane] : 0x7fffffff;
      wave_arg<true>(v, i);
      w = wave_min(w);
      if (lane == 0) {
        s_bc[0] = v;
        s_bc[1] = w;
        s_ic[0] = i;
      }
    }
    __syncthreads();
    const double mval = s_bc[0], Mv = s_bc[1];
    const int i = s_ic[0];
    if (!(mval - Mv >= eps) || i >= n) break;  // converged (or no candidate: NaN-safe)
    // ---- j: second-order selection over K row i
    const double* Ki = Kfull + (long)(IDENT ? i : ids[i]) * ldk;
    const double kii = kd[i];
    double sv = POS;
    int sj = 0x7fffffff;
    // gathers issued GRP elements at a time, unconditionally (clamped index), so they are
    // in flight together; the selection is predicated afterwards
    asm volatile("" : "+v"(tid));  // per-phase address recomputation (not kept live across phases)
#pragma unroll
    for (int k0 = 0; k0 < EPT; k0 += GRP) {
      double kit[GRP], kdt[GRP];
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int k = k0 + u;
        if (k < EPT) {
          const int t = tid + T * k, tc = t < n ? t : n - 1;
          kit[u] = Ki[COL(k, tc)];
          kdt[u] = kd[tc];
        }
      }
#pragma unroll
      for (int u = 0; u < GRP; ++u) {
        const int k = k0 + u;
        const int t = tid + T * k;
        if (k >= EPT || t >= n) continue;
        const bool yp = (ypos >> k) & 1, lc = (ltC >> k) & 1, g0 = (gt0 >> k) & 1;
        const double mg = yp ? -G[k] : G[k];
        const bool low = (yp && g0) || (!yp && lc);
        if (low && mg < mval) {
          const double bt = __dsub_rn(mval, mg);
          double at = __dsub_rn(__dadd_rn(kii, kdt[u]), __dmul_rn(2.0, kit[u]));
          if (!(at > 0)) at = tau;
          const double sc = -__ddiv_rn(__dmul_rn(bt, bt), at);
          if (better_min(sc, t, sv, sj)) {
            sv = sc;
            sj = t;
          }
        }
      }
    }
    wave_arg<false>(sv, sj);
    if (lane == 0) {
      s_v[wv] = sv;
      s_i[wv] = sj;
    }
    __syncthreads();
    if (wv == 0) {
      double v = lane < (T / 64) ? s_v[lane] : POS;
      int j = lane < (T / 64) ? s_i[lane] : 0x7fffffff;
      wave_arg<false>(v, j);
      if (lane == 0) s_ic[1] = j;
    }
    __syncthreads();
    const int j = s_ic[1];
    if (j >= n) break;  // no admissible j (cannot happen while m - M >= eps)
    // ---- the two owners publish what the update needs
    if (tid == (j & (T - 1))) {
      const int kj = j / T;
      double gj = 0.0;
#pragma unroll
      for (int q = 0; q < EPT; ++q)
        if (q == kj) gj = G[q];
      const bool yp = (ypos >> kj) & 1;
      const double mg = yp ? -gj : gj;
      double at = __dsub_rn(__dadd_rn(kii, kd[j]), __dmul_rn(2.0, Ki[IDENT ? j : ids[j]]));
      if (!(at > 0)) at = tau;
      s_bc[2] = __dsub_rn(mval, mg);  // bt_j
      s_bc[3] = at;                   // at_j
      s_bc[4] = a[j];
      s_bc[5] = y[j];
    }
    if (tid == (i & (T - 1))) {
      s_bc[6] = a[i];
      s_bc[7] = y[i];
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
    __syncthreads();  // s_bc / s_ic are rewritten by the next step
  }
#undef COL
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int t = tid + T * k;
    if (t < n) g[t] = G[k];
  }
  if (tid == 0) iters[m] = it;
}

template <int EPT, int T>
int launch_smo_attr() {
  const int bytes = (int)sizeof(int) * EPT * T;
  if (bytes <= 64 * 1024) return HARP_OK;
  return hipFuncSetAttribute((const void*)smo_kernel<EPT, false, T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             bytes) == hipSuccess ? HARP_OK : HARP_ELAUNCH;
}

template <int EPT, int T>
int launch_smo(const double* K, long ldk, const int* ids, const long* moff, int nm, const double* y, const double* kd,
               double* a, double* g, int* iters, double C, double eps, double tau, int max_iter, bool ident,
               hipStream_t s) {
  if (ident)
    smo_kernel<EPT, true, T><<<dim3(nm), dim3(T), 0, s>>>(K, ldk, ids, moff, y, kd, a, g, iters, C, eps, tau,
                                                          max_iter);
  else if (launch_smo_attr<EPT, T>() != HARP_OK)
    return HARP_ELAUNCH;
  else  // the machines' column lists live in LDS: EPT * T ints (<= 128 KB)
    smo_kernel<EPT, false, T><<<dim3(nm), dim3(T), sizeof(int) * EPT * T, s>>>(K, ldk, ids, moff, y, kd, a, g,
                                                                               iters, C, eps, tau, max_iter);
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
#define SMO(E, TT) return launch_smo<E, TT>(K, ldk, ids, moff, nm, y, kd, a, g, iters, C, eps, tau, max_iter, ident != 0, s)
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
