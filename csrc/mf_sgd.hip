// Matrix-factorisation SGD kernels for gfx950 (MI355X / CDNA4).
//
// Replaces the reference's SGD hot loop (ml/java/.../sgd/SGDMPTask.java:46-77: for each
// rating e = w.h - v; w -= eps*(e*h + lam*w); h -= eps*(e*w + lam*h), both from the old
// values) and its RMSE task (RMSETask.java:91-103); the DAAL-exp variant runs the same
// update lock-free inside a mapper (experimental/.../daal_sgd), which is the execution
// model used here.
//
// Design (MI355X-first):
//  * one 16-lane subgroup = one sequential update stream; r/16 factors per lane, so a dot
//    product is 16/r FMAs per lane + a 4-step xor reduction inside the subgroup; a wave runs
//    four independent streams.
//  * each stream owns a contiguous run of the slice's ratings sorted by USER: the user's
//    w row stays in registers while its ratings stream past and is written back once per
//    run; H rows are read and written per rating, lock-free across streams (Hogwild, as
//    DAAL-SGD).
//  * the next rating's (row, col, value) and H row are prefetched while the current one
//    updates, so the dependent-load latency of the chain is overlapped.
//  * XCD blocking (mf_sgd_xcd_kernel): the 8 XCDs have private, mutually non-coherent L2s.
//    A flat Hogwild launch lets every XCD cache its own copy of hot H rows, so concurrent
//    updates of one item from different XCDs overwrite each other at write-back, and every
//    H access is served from the Infinity Fabric / MALL. The blocked layout cuts the
//    resident slice into 8 x 8 (user block, item block) cells; in sub-step s the blocks of
//    one XCD (blockIdx.x % 8 == x: blocks are dealt round-robin over the XCDs) train cell
//    (x, (x + s) mod 8). The 8 cells of a sub-step share no user and no item, so each H
//    block (~1/8 of the slice, well inside one XCD's 4 MB L2) is updated by one XCD only,
//    and the kernel boundary between sub-steps publishes it — the Harp rotation schedule
//    (dymoro), applied one level down, across the XCDs of a GPU.
#include "common.h"

namespace {

template <int EPL>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&x)[EPL]) {
  if constexpr (EPL % 4 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const floatx4 v = *(const floatx4*)(p + k);
      x[k] = v[0]; x[k + 1] = v[1]; x[k + 2] = v[2]; x[k + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = p[k];
  }
}

// H rows are shared by the concurrent streams of an XCD: read them from L2 (nt loads skip
// the CU's vector L1, which is never refreshed by other CUs' stores, nor by this CU's own
// write-through stores), so each update sees the newest value of the row in the XCD.
template <int EPL>
__device__ __forceinline__ void load_row_l2(const float* __restrict__ p, float (&x)[EPL]) {
  if constexpr (EPL % 4 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const floatx4 v = __builtin_nontemporal_load((const floatx4*)(p + k));
      x[k] = v[0]; x[k + 1] = v[1]; x[k + 2] = v[2]; x[k + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = __builtin_nontemporal_load(p + k);
  }
}

template <int EPL>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&x)[EPL]) {
  if constexpr (EPL % 4 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) *(floatx4*)(p + k) = floatx4{x[k], x[k + 1], x[k + 2], x[k + 3]};
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) p[k] = x[k];
  }
}

__device__ __forceinline__ float sub16_sum(float v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}

// One update stream: ratings [i0, i1) in order, run by the 16-lane subgroup holding lane `sl`.
template <int R>
__device__ __forceinline__ void sgd_stream(const int* __restrict__ rows, const int* __restrict__ cols,
                                           const float* __restrict__ vals, long i0, long i1, int sl,
                                           float* __restrict__ W, int ldw, float* __restrict__ H, int ldh, float lr,
                                           float lam) {
  constexpr int EPL = R / 16;
  float w[EPL], h[EPL], hn[EPL];
  int cur = rows[i0];
  load_row<EPL>(W + (long)cur * ldw + sl * EPL, w);
  int col = cols[i0];
  float v = vals[i0];
  load_row_l2<EPL>(H + (long)col * ldh + sl * EPL, h);
  for (long i = i0; i < i1; ++i) {
    // prefetch the next rating and its H row
    int nrow = cur, ncol = col;
    float nv = 0.f;
    const bool more = i + 1 < i1;
    if (more) {
      nrow = rows[i + 1];
      ncol = cols[i + 1];
      nv = vals[i + 1];
      load_row_l2<EPL>(H + (long)ncol * ldh + sl * EPL, hn);
    }
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) dot = fmaf(w[k], h[k], dot);
    const float err = sub16_sum(dot) - v;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      const float wk = w[k], hk = h[k];
      w[k] = wk - lr * fmaf(err, hk, lam * wk);
      h[k] = hk - lr * fmaf(err, wk, lam * hk);
    }
    store_row<EPL>(H + (long)col * ldh + sl * EPL, h);
    if (!more) break;
    if (ncol == col) {
      // same item again: use the row just written, not the stale prefetch
#pragma unroll
      for (int k = 0; k < EPL; ++k) hn[k] = h[k];
    }
    if (nrow != cur) {
      store_row<EPL>(W + (long)cur * ldw + sl * EPL, w);
      cur = nrow;
      load_row<EPL>(W + (long)cur * ldw + sl * EPL, w);
    }
    col = ncol;
    v = nv;
#pragma unroll
    for (int k = 0; k < EPL; ++k) h[k] = hn[k];
  }
  store_row<EPL>(W + (long)cur * ldw + sl * EPL, w);
}

template <int R>
__global__ __launch_bounds__(256) void mf_sgd_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                     const float* __restrict__ vals, long n, int chunk,
                                                     float* __restrict__ W, int ldw, float* __restrict__ H, int ldh,
                                                     float lr, float lam) {
  const int sl = threadIdx.x & 15;
  const long sg = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const long i0 = sg * (long)chunk;
  long i1 = i0 + chunk;
  if (i1 > n) i1 = n;
  if (i0 >= i1) return;
  sgd_stream<R>(rows, cols, vals, i0, i1, sl, W, ldw, H, ldh, lr, lam);
}

constexpr int XCDS = 8;

// Sub-step `step` of the XCD-blocked schedule. off[c] .. off[c + 1] are the ratings of cell
// c = user_block * 8 + item_block (cell-major, user-sorted inside a cell). The blocks that
// share an XCD (same blockIdx.x % 8) stride over the streams of their cell.
template <int R>
__global__ __launch_bounds__(256) void mf_sgd_xcd_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                         const float* __restrict__ vals, const long* __restrict__ off,
                                                         int step, int chunk, float* __restrict__ W, int ldw,
                                                         float* __restrict__ H, int ldh, float lr, float lam) {
  const int x = blockIdx.x % XCDS;
  const long j = blockIdx.x / XCDS;
  const long per_xcd = gridDim.x / XCDS;
  const int cell = x * XCDS + (x + step) % XCDS;
  const long a = off[cell], e = off[cell + 1];
  const long nst = (e - a + chunk - 1) / chunk;
  const int sl = threadIdx.x & 15;
  const long sub = threadIdx.x >> 4;  // 16 streams per 256-thread block
  for (long st = j * 16 + sub; st < nst; st += per_xcd * 16) {
    const long i0 = a + st * chunk;
    const long i1 = i0 + chunk < e ? i0 + chunk : e;
    sgd_stream<R>(rows, cols, vals, i0, i1, sl, W, ldw, H, ldh, lr, lam);
  }
}

template <int R>
__global__ __launch_bounds__(256) void mf_rmse_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                      const float* __restrict__ vals, long n, const float* __restrict__ W,
                                                      int ldw, const float* __restrict__ H, int ldh,
                                                      double* __restrict__ partial) {
  constexpr int EPL = R / 16;
  const int sl = threadIdx.x & 15;
  const long nsub = ((long)gridDim.x * blockDim.x) >> 4;
  float acc = 0.f;
  for (long i = (((long)blockIdx.x * blockDim.x + threadIdx.x) >> 4); i < n; i += nsub) {
    float w[EPL], h[EPL];
    load_row<EPL>(W + (long)rows[i] * ldw + sl * EPL, w);
    load_row<EPL>(H + (long)cols[i] * ldh + sl * EPL, h);
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < EPL; ++k) dot = fmaf(w[k], h[k], dot);
    const float e = vals[i] - sub16_sum(dot);
    acc = fmaf(e, e, acc);
  }
  // one lane per subgroup holds the subgroup's sum (all 16 lanes hold equal values)
  double s = (sl == 0) ? (double)acc : 0.0;
  s = wave_sum_d(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

template <int R>
int launch_sgd(const int* rows, const int* cols, const float* vals, long n, int chunk, float* W, int ldw, float* H,
               int ldh, float lr, float lam, hipStream_t s) {
  const long streams = (n + chunk - 1) / chunk;
  const long threads = streams * 16;
  const long blocks = (threads + 255) / 256;
  mf_sgd_kernel<R><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(rows, cols, vals, n, chunk, W, ldw, H, ldh, lr, lam);
  return harp_launch_status();
}

template <int R>
int launch_sgd_xcd(const int* rows, const int* cols, const float* vals, const long* off, int steps, int chunk,
                   int blocks_per_xcd, float* W, int ldw, float* H, int ldh, float lr, float lam, hipStream_t s) {
  for (int step = 0; step < steps; ++step) {
    mf_sgd_xcd_kernel<R><<<dim3((unsigned)(blocks_per_xcd * XCDS)), dim3(256), 0, s>>>(
        rows, cols, vals, off, step, chunk, W, ldw, H, ldh, lr, lam);
    const int st = harp_launch_status();
    if (st != HARP_OK) return st;
  }
  return HARP_OK;
}

template <int R>
int launch_rmse(const int* rows, const int* cols, const float* vals, long n, const float* W, int ldw, const float* H,
                int ldh, double* partial, int nblocks, hipStream_t s) {
  mf_rmse_kernel<R><<<dim3(nblocks), dim3(256), 0, s>>>(rows, cols, vals, n, W, ldw, H, ldh, partial);
  return harp_launch_status();
}

}  // namespace

#define MF_DISPATCH(R, CALL)          \
  switch (R) {                        \
    case 16: return CALL(16);         \
    case 32: return CALL(32);         \
    case 48: return CALL(48);         \
    case 64: return CALL(64);         \
    case 128: return CALL(128);       \
    case 256: return CALL(256);       \
    default: return HARP_EUNSUPPORTED; \
  }

HARP_EXPORT int harp_mf_sgd(const int* rows, const int* cols, const float* vals, long n, int r, int chunk, float* W,
                            int ldw, float* H, int ldh, float lr, float lam, hipStream_t s) {
  if (n <= 0) return HARP_OK;
  if (chunk <= 0 || ldw < r || ldh < r) return HARP_EBADARG;
#define SGD_CALL(RR) launch_sgd<RR>(rows, cols, vals, n, chunk, W, ldw, H, ldh, lr, lam, s)
  MF_DISPATCH(r, SGD_CALL)
#undef SGD_CALL
}

HARP_EXPORT int harp_mf_xcds() { return XCDS; }

// All `steps` (= 8) sub-steps of the XCD-blocked schedule over one resident slice: `off`
// is a DEVICE array of 65 int64 cell offsets into rows/cols/vals.
HARP_EXPORT int harp_mf_sgd_xcd(const int* rows, const int* cols, const float* vals, const long* off, int r,
                                int steps, int chunk, int blocks_per_xcd, float* W, int ldw, float* H, int ldh,
                                float lr, float lam, hipStream_t s) {
  if (chunk <= 0 || blocks_per_xcd <= 0 || steps <= 0 || steps > XCDS || ldw < r || ldh < r) return HARP_EBADARG;
#define SGDX_CALL(RR) \
  launch_sgd_xcd<RR>(rows, cols, vals, off, steps, chunk, blocks_per_xcd, W, ldw, H, ldh, lr, lam, s)
  MF_DISPATCH(r, SGDX_CALL)
#undef SGDX_CALL
}

HARP_EXPORT int harp_mf_rmse_blocks() { return 1024; }

HARP_EXPORT int harp_mf_rmse(const int* rows, const int* cols, const float* vals, long n, int r, const float* W, int ldw,
                             const float* H, int ldh, double* partial, hipStream_t s) {
  if (n <= 0) return HARP_OK;
#define RMSE_CALL(RR) launch_rmse<RR>(rows, cols, vals, n, W, ldw, H, ldh, partial, 1024, s)
  MF_DISPATCH(r, RMSE_CALL)
#undef RMSE_CALL
}
