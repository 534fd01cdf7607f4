// ALS normal equations per row on gfx950 (explicit and implicit feedback).
//
// Reference: ml/daal/.../als/ (DAAL implicit ALS: per user u,
//   (Y^T Y + Y^T (C_u - I) Y + lambda I) x_u = Y^T C_u p(u))
// and ml/java/.../als/ (explicit: (F_u^T F_u + lambda n_u I) x_u = F_u^T r_u).
// The torch path materialises one f x f outer product per rating (nnz x f^2 values)
// before an index_add. Here one workgroup owns one row: the row's rated factor rows are
// staged through LDS 32 at a time with their weights, and each thread accumulates its
// 16 (i, k) entries of the f x f system in registers, so nothing per-rating reaches
// HBM. G (= F^T F for implicit), the lambda diagonal and the right-hand side are
// applied in the same pass. The batched Cholesky solve stays on rocSOLVER.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 32;   // rated rows staged per LDS trip
constexpr int kMaxF = 64;    // f x f entries = 4096 = 16 per thread

// A[r] = sum_j aw_j F[c_j] F[c_j]^T + G + lam_r I ;  rhs[r] = sum_j bw_j F[c_j]
// explicit:  aw = 1,          bw = v,                lam_r = lam * max(n_r, 1)
// implicit:  aw = alpha v,    bw = (1 + alpha v) [v > 0], lam_r = lam (* max(n_r,1) if wl)
template <typename T>
__global__ __launch_bounds__(kThreads) void als_normal_kernel(const long* __restrict__ crow,
                                                              const long* __restrict__ cols,
                                                              const T* __restrict__ vals,
                                                              const T* __restrict__ F, int f,
                                                              const T* __restrict__ G, int implicit, T alpha,
                                                              T lam, int scale_lam, T* __restrict__ A,
                                                              T* __restrict__ rhs, long row0) {
  __shared__ T sF[kChunk][kMaxF];
  __shared__ T sa[kChunk], sb[kChunk];
  const long r = blockIdx.x;
  const long s = crow[row0 + r], e = crow[row0 + r + 1];
  const int tid = threadIdx.x;
  const int ff = f * f;
  T acc[kMaxF * kMaxF / kThreads];
#pragma unroll
  for (int q = 0; q < kMaxF * kMaxF / kThreads; ++q) acc[q] = T(0);
  T racc = T(0);
  for (long j0 = s; j0 < e; j0 += kChunk) {
    const int m = (int)((e - j0) < kChunk ? (e - j0) : kChunk);
    for (int t = tid; t < m * f; t += kThreads) {
      const int jj = t / f, c = t - jj * f;
      sF[jj][c] = F[cols[j0 + jj] * (long)f + c];
    }
    if (tid < m) {
      const T v = vals[j0 + tid];
      if (implicit) {
        sa[tid] = alpha * v;
        sb[tid] = v > T(0) ? T(1) + alpha * v : T(0);
      } else {
        sa[tid] = T(1);
        sb[tid] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kMaxF * kMaxF / kThreads; ++q) {
      const int idx = tid + q * kThreads;
      if (idx < ff) {
        const int i = idx / f, k = idx - i * f;
        T a = acc[q];
        for (int jj = 0; jj < m; ++jj) a += sa[jj] * sF[jj][i] * sF[jj][k];
        acc[q] = a;
      }
    }
    if (tid < f)
      for (int jj = 0; jj < m; ++jj) racc += sb[jj] * sF[jj][tid];
    __syncthreads();
  }
  const long n_r = e - s;
  const T lr = scale_lam ? lam * (T)(n_r > 0 ? n_r : 1) : lam;
  T* Ar = A + r * (long)ff;
#pragma unroll
  for (int q = 0; q < kMaxF * kMaxF / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    if (idx < ff) {
      const int i = idx / f, k = idx - i * f;
      T a = acc[q] + (G ? G[idx] : T(0));
      if (i == k) a += lr;
      Ar[idx] = a;
    }
  }
  if (tid < f) rhs[r * (long)f + tid] = racc;
}

template <typename T>
int launch(const long* crow, const long* cols, const T* vals, const T* F, int f, const T* G, int implicit, T alpha,
           T lam, int scale_lam, T* A, T* rhs, long row0, long nrows, hipStream_t s) {
  if (nrows <= 0) return HARP_OK;
  if (f <= 0 || f > kMaxF || nrows > 0x7fffffffL) return HARP_EBADARG;
  als_normal_kernel<T><<<dim3((unsigned)nrows), dim3(kThreads), 0, s>>>(crow, cols, vals, F, f, G, implicit, alpha,
                                                                       lam, scale_lam, A, rhs, row0);
  return harp_launch_status();
}

}  // namespace

// rows [row0, row0 + nrows) of a CSR (crow over all rows, cols int64 into F [*, f]);
// A [nrows, f, f], rhs [nrows, f]; G may be null; f <= 64
HARP_EXPORT int harp_als_normal_f32(const long* crow, const long* cols, const float* vals, const float* F, int f,
                                    const float* G, int implicit, float alpha, float lam, int scale_lam, float* A,
                                    float* rhs, long row0, long nrows, hipStream_t s) {
  return launch<float>(crow, cols, vals, F, f, G, implicit, alpha, lam, scale_lam, A, rhs, row0, nrows, s);
}

HARP_EXPORT int harp_als_normal_f64(const long* crow, const long* cols, const double* vals, const double* F, int f,
                                    const double* G, int implicit, double alpha, double lam, int scale_lam, double* A,
                                    double* rhs, long row0, long nrows, hipStream_t s) {
  return launch<double>(crow, cols, vals, F, f, G, implicit, alpha, lam, scale_lam, A, rhs, row0, nrows, s);
}
