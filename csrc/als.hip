// ALS normal equations per row on gfx950 (explicit and implicit feedback).
//
// Reference: ml/daal/.../als/ (DAAL implicit ALS: per user u,
//   (Y^T Y + Y^T (C_u - I) Y + lambda I) x_u = Y^T C_u p(u))
// and ml/java/.../als/ (explicit: (F_u^T F_u + lambda n_u I) x_u = F_u^T r_u).
// The torch path materialises one f x f outer product per rating (nnz x f^2 values)
// before an index_add. Here one workgroup owns one row: the row's rated factor rows are
// staged through LDS 32 at a time with their weights, and each thread accumulates its
// 4 x 4 register tile of the (zero-padded 64 x 64) f x f system, so nothing per-rating reaches
// HBM. G (= F^T F for implicit), the lambda diagonal and the right-hand side are
// applied in the same pass. By default the system is then solved in the same
// workgroup (Cholesky in LDS); the A / rhs mode feeds rocSOLVER's batched solver.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 32;   // rated rows staged per LDS trip
constexpr int kMaxF = 64;    // f x f entries = 4096 = 16 per thread
int ALS_BUILD_DMA = 1;       // host switch for A/B (harp_als_set_build_dma)


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
                                                              T* __restrict__ rhs, long row0,
                                                              T* __restrict__ X, int* __restrict__ info) {
  __shared__ T sF[kChunk][kMaxF];
  __shared__ T sA[kMaxF][kMaxF + 1];
  __shared__ T sx[kMaxF];
  __shared__ int sbad;
  __shared__ T sa[kChunk], sb[kChunk];
  const long r = blockIdx.x;
  const long s = crow[row0 + r], e = crow[row0 + r + 1];
  const int tid = threadIdx.x;
  // thread owns the 4 x 4 tile rows [ti, ti + 4) x cols [tk, tk + 4) of the 64 x 64
  // (zero-padded) system: 8 LDS reads per 16 FMAs per rating
  const int ti = (tid >> 4) * 4, tk = (tid & 15) * 4;
  T acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = T(0);
  T racc = T(0);
  for (long j0 = s; j0 < e; j0 += kChunk) {
    const int m = (int)((e - j0) < kChunk ? (e - j0) : kChunk);
    for (int t = tid; t < m * kMaxF; t += kThreads) {
      const int jj = t / kMaxF, c = t - jj * kMaxF;
      sF[jj][c] = c < f ? F[cols[j0 + jj] * (long)f + c] : T(0);
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
    for (int jj = 0; jj < m; ++jj) {
      const T w = sa[jj];
      T a[4], b[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        a[x] = w * sF[jj][ti + x];
        b[x] = sF[jj][tk + x];
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] += a[x] * b[y];
    }
    if (tid < f)
      for (int jj = 0; jj < m; ++jj) racc += sb[jj] * sF[jj][tid];
    __syncthreads();
  }
  const long n_r = e - s;
  const T lr = scale_lam ? lam * (T)(n_r > 0 ? n_r : 1) : lam;
  if (X) {
    // fused solve: Cholesky of the system in LDS (right-looking, lower triangle in
    // place), then L y = rhs and L^T x = y; a non-positive pivot flags the row in info.
    // (A one-wave register-resident variant with lane broadcasts measured no faster:
    // 8.1 vs 7.8 ms per 131k-row block at f=64, 2x slower at f=32 from the padding.)
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int i = ti + x, k = tk + y;
        if (i < f && k < f) sA[i][k] = acc[x][y] + (G ? G[i * f + k] : T(0)) + (i == k ? lr : T(0));
      }
    if (tid < f) sx[tid] = racc;
    if (tid == 0) sbad = 0;
    __syncthreads();
    for (int j = 0; j < f; ++j) {
      if (tid == 0) {
        T d = sA[j][j];
        if (!(d > T(0))) {
          sbad = 1;
          d = T(1);
        }
        sA[j][j] = sqrt(d);
      }
      __syncthreads();
      const T piv = sA[j][j];
      for (int i = j + 1 + tid; i < f; i += kThreads) sA[i][j] /= piv;
      __syncthreads();
      const int w = f - j - 1;
      for (int t = tid; t < w * w; t += kThreads) {
        const int i = j + 1 + t / w, k = j + 1 + t % w;
        if (k <= i) sA[i][k] -= sA[i][j] * sA[k][j];
      }
      __syncthreads();
    }
    for (int j = 0; j < f; ++j) {  // L y = b
      if (tid == 0) sx[j] /= sA[j][j];
      __syncthreads();
      for (int i = j + 1 + tid; i < f; i += kThreads) sx[i] -= sA[i][j] * sx[j];
      __syncthreads();
    }
    for (int j = f - 1; j >= 0; --j) {  // L^T x = y
      if (tid == 0) sx[j] /= sA[j][j];
      __syncthreads();
      for (int i = tid; i < j; i += kThreads) sx[i] -= sA[j][i] * sx[j];
      __syncthreads();
    }
    if (tid < f) X[r * (long)f + tid] = sx[tid];
    if (tid == 0) info[r] = sbad;
    return;
  }
  T* Ar = A + r * (long)f * f;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int i = ti + x, k = tk + y;
      if (i < f && k < f) {
        T a = acc[x][y] + (G ? G[i * f + k] : T(0));
        if (i == k) a += lr;
        Ar[i * f + k] = a;
      }
    }
  if (tid < f) rhs[r * (long)f + tid] = racc;
}

// Build-only fp32 variant (f % 4 == 0): the rated factor rows of chunk c+1 stream into the
// other half of a double-buffered LDS slab by LDS-DMA (global_load_lds, 16 B per lane,
// 4 rows of 256 B per wave-instruction) while chunk c is accumulated, so the gather latency
// no longer sits between the chunk barriers. Columns past f read a zero source.
__device__ __attribute__((aligned(16))) float g_als_zero[4] = {0.f, 0.f, 0.f, 0.f};

__global__ __launch_bounds__(kThreads) void als_build_dma_kernel(const long* __restrict__ crow,
                                                                 const long* __restrict__ cols,
                                                                 const float* __restrict__ vals,
                                                                 const float* __restrict__ F, int f,
                                                                 const float* __restrict__ G, int implicit,
                                                                 float alpha, float lam, int scale_lam,
                                                                 float* __restrict__ A, float* __restrict__ rhs,
                                                                 long row0) {
  __shared__ __attribute__((aligned(16))) float sF[2][kChunk][kMaxF];
  __shared__ float sa[2][kChunk], sb[2][kChunk];
  const long r = blockIdx.x;
  const long s = crow[row0 + r], e = crow[row0 + r + 1];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int ti = (tid >> 4) * 4, tk = (tid & 15) * 4;
  float acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = 0.f;
  float racc = 0.f;
  auto stage = [&](int buf, long j0) {
    const int m = (int)((e - j0) < kChunk ? (e - j0) : kChunk);
    // kChunk rows x 256 B = 8 one-KiB DMA pieces; wave wv issues pieces wv and wv + 4
#pragma unroll
    for (int q = wv; q < kChunk / 4; q += kThreads / 64) {
      const int jj = q * 4 + (lane >> 4), c4 = (lane & 15) * 4;
      const float* src = (jj < m && c4 < f) ? F + cols[j0 + jj] * (long)f + c4 : g_als_zero;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)&sF[buf][q * 4][0], 16, 0, 0);
    }
    if (tid < m) {
      const float v = vals[j0 + tid];
      sa[buf][tid] = implicit ? alpha * v : 1.f;
      sb[buf][tid] = implicit ? (v > 0.f ? 1.f + alpha * v : 0.f) : v;
    }
  };
  int buf = 0;
  if (s < e) stage(0, s);
  for (long j0 = s; j0 < e; j0 += kChunk, buf ^= 1) {
    const int m = (int)((e - j0) < kChunk ? (e - j0) : kChunk);
    // this wave's DMA pieces of chunk j0 landed; the barrier makes every wave's visible and
    // ends every wave's reads of the other buffer (the next prefetch target)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (j0 + kChunk < e) stage(buf ^ 1, j0 + kChunk);
    for (int jj = 0; jj < m; ++jj) {
      const float w = sa[buf][jj];
      float a[4], b[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        a[x] = w * sF[buf][jj][ti + x];
        b[x] = sF[buf][jj][tk + x];
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] += a[x] * b[y];
    }
    if (tid < f)
      for (int jj = 0; jj < m; ++jj) racc += sb[buf][jj] * sF[buf][jj][tid];
  }
  const long n_r = e - s;
  const float lr = scale_lam ? lam * (float)(n_r > 0 ? n_r : 1) : lam;
  float* Ar = A + r * (long)f * f;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int i = ti + x, k = tk + y;
      if (i < f && k < f) {
        float a = acc[x][y] + (G ? G[i * f + k] : 0.f);
        if (i == k) a += lr;
        Ar[i * f + k] = a;
      }
    }
  if (tid < f) rhs[r * (long)f + tid] = racc;
}

// Batched SPD solve A x = rhs (fp32, f <= 64), ONE WAVE PER SYSTEM and no barriers: lane i
// holds row i of A (zero-padded to 64, identity rows past f) in 64 VGPRs. Right-looking
// Cholesky over the unrolled columns j: the pivot and the column entries L[k][j] are wave
// broadcasts (v_readlane), each lane updates its own row; L y = b broadcasts y_j; L^T x = y
// takes x_j = (y_j - sum_{k>j} L[k][j] x_k) / L[j][j] as a wave reduction per column. The
// fused kernel's in-LDS Cholesky spent 3 workgroup barriers per column (about 70 % of a
// 131k-row block, profiles/r2_als); this one is VALU-issue bound.
// LDS_BCAST = 1: column j of L goes through a per-wave LDS row (one ds_write, then
// same-address broadcast reads the compiler merges into ds_read_b128) instead of 63 - j
// v_readlane + SGPR-operand FMA pairs (measured in profiles/r2_als).
template <int LDS_BCAST>
__global__ __launch_bounds__(256) void als_chol_solve_kernel(const float* __restrict__ A, const float* __restrict__ rhs,
                                                            int f, long m, float* __restrict__ X,
                                                            int* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) float scol[4][kMaxF];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long r = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= m) return;  // wave-uniform
  float a[kMaxF];
  const float* Ar = A + r * (long)f * f + (long)lane * f;
  if ((f & 3) == 0) {
#pragma unroll
    for (int k = 0; k < kMaxF; k += 4) {
      if (lane < f && k < f) {
        const float4 v = *(const float4*)(Ar + k);
        a[k] = v.x; a[k + 1] = v.y; a[k + 2] = v.z; a[k + 3] = v.w;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[k + q] = k + q == lane ? 1.f : 0.f;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kMaxF; ++k) a[k] = lane < f ? (k < f ? Ar[k] : 0.f) : (k == lane ? 1.f : 0.f);
  }
  float b = lane < f ? rhs[r * (long)f + lane] : 0.f;
  int bad = 0;
  float* col = scol[wv];
#pragma unroll
  for (int j = 0; j < kMaxF; ++j) {
    float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a[j]), j));
    if (!(d > 0.f)) {
      bad = 1;
      d = 1.f;
    }
    const float sq = sqrtf(d), inv = 1.f / sq;
    a[j] = lane == j ? sq : a[j] * inv;  // column j of L (rows > j); the diagonal
    if constexpr (LDS_BCAST) {
      col[lane] = a[j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = j + 1; k < kMaxF; ++k) a[k] = fmaf(-a[j], col[k], a[k]);  // row `lane`, column k
      __builtin_amdgcn_wave_barrier();  // every lane read col before the next column overwrites it
    } else {
#pragma unroll
      for (int k = j + 1; k < kMaxF; ++k) {
        const float lk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a[j]), k));
        a[k] = fmaf(-a[j], lk, a[k]);  // row `lane`, column k (only k <= lane is ever read)
      }
    }
  }
  // L y = b
#pragma unroll
  for (int j = 0; j < kMaxF; ++j) {
    const float ljj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a[j]), j));
    const float yj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b), j)) / ljj;
    if (lane == j) b = yj;
    else if (lane > j) b = fmaf(-a[j], yj, b);
  }
  // L^T x = y
  float x = 0.f;
#pragma unroll
  for (int j = kMaxF - 1; j >= 0; --j) {
    float t = lane > j ? a[j] * x : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    const float ljj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a[j]), j));
    const float yj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b), j));
    if (lane == j) x = (yj - t) / ljj;
  }
  if (lane < f) X[r * (long)f + lane] = x;
  if (lane == 0) info[r] = bad;
}

template <typename T>
int launch(const long* crow, const long* cols, const T* vals, const T* F, int f, const T* G, int implicit, T alpha,
           T lam, int scale_lam, T* A, T* rhs, long row0, long nrows, T* X, int* info, hipStream_t s) {
  if (nrows <= 0) return HARP_OK;
  if (f <= 0 || f > kMaxF || nrows * (long)kThreads > 0xffffffffL || (X && !info) || (!X && (!A || !rhs))) return HARP_EBADARG;
  als_normal_kernel<T><<<dim3((unsigned)nrows), dim3(kThreads), 0, s>>>(crow, cols, vals, F, f, G, implicit, alpha,
                                                                       lam, scale_lam, A, rhs, row0, X, info);
  return harp_launch_status();
}

}  // namespace

// rows [row0, row0 + nrows) of a CSR (crow over all rows, cols int64 into F [*, f]);
// A [nrows, f, f], rhs [nrows, f]; G may be null; f <= 64. With X (and info) non-null
// the systems are solved in the kernel instead: X [nrows, f], info [nrows] (1 = not SPD)
HARP_EXPORT int harp_als_normal_f32(const long* crow, const long* cols, const float* vals, const float* F, int f,
                                    const float* G, int implicit, float alpha, float lam, int scale_lam, float* A,
                                    float* rhs, long row0, long nrows, float* X, int* info, hipStream_t s) {
  if (!X && f % 4 == 0 && ALS_BUILD_DMA) {
    if (nrows <= 0) return HARP_OK;
    if (f <= 0 || f > kMaxF || !A || !rhs || nrows * (long)kThreads > 0xffffffffL) return HARP_EBADARG;
    als_build_dma_kernel<<<dim3((unsigned)nrows), dim3(kThreads), 0, s>>>(crow, cols, vals, F, f, G, implicit, alpha,
                                                                        lam, scale_lam, A, rhs, row0);
    return harp_launch_status();
  }
  return launch<float>(crow, cols, vals, F, f, G, implicit, alpha, lam, scale_lam, A, rhs, row0, nrows, X, info, s);
}

HARP_EXPORT int harp_als_normal_f64(const long* crow, const long* cols, const double* vals, const double* F, int f,
                                    const double* G, int implicit, double alpha, double lam, int scale_lam, double* A,
                                    double* rhs, long row0, long nrows, double* X, int* info, hipStream_t s) {
  return launch<double>(crow, cols, vals, F, f, G, implicit, alpha, lam, scale_lam, A, rhs, row0, nrows, X, info,
                        s);
}

// X [m, f] = A [m, f, f]^-1 rhs [m, f] for SPD A (fp32, f <= 64; one wave per system);
// info[r] = 1 marks a non-positive pivot (that row's X is not a solution)
// variant 0: LDS column broadcast (default), 1: v_readlane broadcast
HARP_EXPORT int harp_als_chol_solve_f32(const float* A, const float* rhs, int f, long m, float* X, int* info,
                                        int variant, hipStream_t s) {
  if (m <= 0) return HARP_OK;
  if (f <= 0 || f > kMaxF || !A || !rhs || !X || !info || m > 0x7fffffffL / 4 || variant < 0 || variant > 1)
    return HARP_EBADARG;
  const dim3 g((unsigned)((m + 3) / 4)), bl(256);
  if (variant == 0) als_chol_solve_kernel<1><<<g, bl, 0, s>>>(A, rhs, f, m, X, info);
  else als_chol_solve_kernel<0><<<g, bl, 0, s>>>(A, rhs, f, m, X, info);
  return harp_launch_status();
}

// A/B switch for the LDS-DMA build variant (1 = on, the default)
HARP_EXPORT int harp_als_set_build_dma(int on) {
  ALS_BUILD_DMA = on ? 1 : 0;
  return HARP_OK;
}
