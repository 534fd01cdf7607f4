// Label-bucketed row sums: sums[k] = sum of rows X[i] with label[i] == k.
//
// Replaces float-atomic scatter accumulation for workloads whose per-item contribution is a
// whole feature row (K-means partial sums, Naive-Bayes class sums, per-cluster statistics;
// the reference's CenCalcTask accumulate + CenMergeTask merge, ml/java/.../kmeans/
// regroupallgather/CenCalcTask.java:67-100, CenMergeTask.java:36-54).
//
// Why not atomics: on gfx950 float atomics run at ~1.3 TB/s of added bytes chip-wide
// (memory-side), so 1e8 rows x 101 fp32 = 40 GB costs ~25-30 ms. Bucketing the labels
// (counting sort) and gathering each bucket's rows reads the bf16 rows once at gather
// bandwidth (~4-5 TB/s) and sums them in registers in a fixed order.
//
// Pipeline (all int32, K = number of buckets <= 16384):
//   1. hist:    per chunk of CH labels an LDS histogram -> H[chunk][K]
//   2. colscan: per-bucket exclusive scan over chunks (two levels: 64-chunk segments)
//   3. segscan: exclusive scan of bucket totals -> seg_start[K+1]
//   4. bucket:  per chunk, LDS cursors = global base; perm[pos] = i
//   5. rowsum:  each 16-lane slot sums a fixed run of the sorted permutation (balanced for any
//               bucket skew) in fp32 registers, flushing at bucket boundaries
#include "common.h"

namespace {

constexpr int SEG = 64;  // chunks per column-scan segment

__global__ __launch_bounds__(256) void label_hist_kernel(const int* __restrict__ lab, long n, int K, long chunk,
                                                         int* __restrict__ H) {
  extern __shared__ __attribute__((aligned(16))) int hist[];
  for (int k = threadIdx.x; k < K; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  const long a = (long)blockIdx.x * chunk;
  long b = a + chunk;
  if (b > n) b = n;
  for (long i = a + threadIdx.x; i < b; i += blockDim.x) atomicAdd(&hist[lab[i]], 1);
  __syncthreads();
  int* row = H + (long)blockIdx.x * K;
  for (int k = threadIdx.x; k < K; k += blockDim.x) row[k] = hist[k];
}

// level 1: inside each segment of SEG chunks, exclusive scan per bucket; T[seg][k] = total
__global__ void colscan1_kernel(int* __restrict__ H, int nchunks, int K, int* __restrict__ T) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (k >= K) return;
  const int c0 = s * SEG;
  int c1 = c0 + SEG;
  if (c1 > nchunks) c1 = nchunks;
  int run = 0;
  for (int c = c0; c < c1; ++c) {
    const int v = H[(long)c * K + k];
    H[(long)c * K + k] = run;
    run += v;
  }
  T[(long)s * K + k] = run;
}

// level 2: exclusive scan over segments per bucket; counts[k] = total rows of bucket k
__global__ void colscan2_kernel(int* __restrict__ T, int nseg, int K, int* __restrict__ counts) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  int run = 0;
  for (int s = 0; s < nseg; ++s) {
    const int v = T[(long)s * K + k];
    T[(long)s * K + k] = run;
    run += v;
  }
  counts[k] = run;
}

// exclusive scan of counts -> start[K+1] (one workgroup of 1024 threads)
__global__ __launch_bounds__(1024) void segscan_kernel(const int* __restrict__ counts, int K, int* __restrict__ start) {
  __shared__ int part[1024];
  const int per = (K + 1023) / 1024;
  const int a = threadIdx.x * per;
  int s = 0;
  for (int j = 0; j < per; ++j)
    if (a + j < K) s += counts[a + j];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int j = 0; j < per; ++j)
    if (a + j < K) {
      start[a + j] = run;
      run += counts[a + j];
    }
  if (threadIdx.x == 1023) start[K] = part[1023];
}

// XCD-contiguous chunk order: workgroup b runs on XCD b % 8, and the chunks of one XCD are a
// contiguous range, so the per-bucket runs that consecutive chunks write into perm meet in
// the SAME L2 and leave it as whole lines (round-robin chunks split every bucket's
// ~6-entry run boundary across two XCDs' L2s, i.e. partial-line writes to HBM).
__device__ __forceinline__ int xcd_contiguous(unsigned b, unsigned nb) {
  const unsigned q = nb / 8, r = nb % 8, x = b % 8;
  return (int)((x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8);
}

__global__ __launch_bounds__(256) void bucket_kernel(const int* __restrict__ lab, long n, int K, long chunk,
                                                     const int* __restrict__ H, const int* __restrict__ T,
                                                     const int* __restrict__ start, int* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) int cur[];
  const int c = xcd_contiguous(blockIdx.x, gridDim.x), s = c / SEG;
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    cur[k] = start[k] + T[(long)s * K + k] + H[(long)c * K + k];
  __syncthreads();
  const long a = (long)c * chunk;
  long b = a + chunk;
  if (b > n) b = n;
  // 8 labels per thread in flight: their loads are independent, so the loop is not one
  // dependent global-load -> LDS-atomic -> store chain per label
  constexpr int U = 8;
  for (long i0 = a + threadIdx.x; i0 < b; i0 += (long)U * blockDim.x) {
    int l[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + (long)u * blockDim.x;
      l[u] = i < b ? lab[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (l[u] >= 0) perm[atomicAdd(&cur[l[u]], 1)] = (int)(i0 + (long)u * blockDim.x);
  }
}

// Skew-proof gather-sum: every LPR-lane slot owns RUN consecutive entries of the
// bucket-sorted permutation (so work is balanced whatever the bucket sizes), keeps the
// running row sum in registers, and flushes it with one contiguous fp32 atomic row segment
// whenever it crosses a bucket boundary (~1 flush per slot for buckets >> RUN).
template <int LPR, int RUN, int ROWS = 4>
__global__ __launch_bounds__(256) void rowsum_bf16_kernel(const __bf16* __restrict__ X, int dp, long ldx,
                                                          const int* __restrict__ perm,
                                                          const int* __restrict__ start, int K, long n,
                                                          float* __restrict__ sums, int ld) {
  constexpr int SPW = 64 / LPR;  // slots per wave
  const int lane = threadIdx.x & 63;
  const int sl = lane % LPR;
  const long slot = ((long)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const long j0 = slot * RUN;
  if (j0 >= n) return;
  long j1 = j0 + RUN;
  if (j1 > n) j1 = n;
  const bool active = sl * 8 < dp;
  // bucket containing j0: last k with start[k] <= j0
  int lo = 0, hi = K;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (start[mid] <= j0) lo = mid; else hi = mid;
  }
  int k = lo;
  long kend = start[k + 1];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto flush = [&](int kk) {
    if (active) {
      float* o = sums + (long)kk * ld + sl * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (acc[e] != 0.f) atomicAdd(o + e, acc[e]);
        acc[e] = 0.f;
      }
    }
  };
  long j = j0;
  while (j < j1) {
    while (j >= kend) {  // crossed into the next non-empty bucket
      flush(k);
      ++k;
      kend = start[k + 1];
    }
    long stop = kend < j1 ? kend : j1;
    // ROWS rows in flight per slot inside one bucket
    for (; j + ROWS <= stop; j += ROWS) {
      bf16x8 v[ROWS];
      int pj[ROWS];
#pragma unroll
      for (int q = 0; q < ROWS; ++q) pj[q] = perm[j + q];
#pragma unroll
      for (int q = 0; q < ROWS; ++q) v[q] = active ? *(const bf16x8*)(X + (long)pj[q] * ldx + sl * 8) : bf16x8{};
#pragma unroll
      for (int q = 0; q < ROWS; q += 4)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          acc[e] += ((float)v[q][e] + (float)v[q + 1][e]) + ((float)v[q + 2][e] + (float)v[q + 3][e]);
    }
    for (; j < stop; ++j) {
      if (active) {
        const bf16x8 v = *(const bf16x8*)(X + (long)perm[j] * ldx + sl * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
      }
    }
  }
  flush(k);
  (void)SPW;
}

// Rows wider than 256 columns (the wide-row K-means, d up to 1024 per call): one wave per
// slot, each lane VEC 16-B chunks of the row (chunk c of lane l at column 8 * (64 c + l), so
// each chunk index is one contiguous 1 KB read per wave), ROWS rows in flight; one pass over
// the permutation instead of one per 256-column slice.
template <int VEC, int RUN, int ROWS = 4>
__global__ __launch_bounds__(256) void rowsum_wide_bf16_kernel(const __bf16* __restrict__ X, int dp, long ldx,
                                                               const int* __restrict__ perm,
                                                               const int* __restrict__ start, int K, long n,
                                                               float* __restrict__ sums, int ld) {
  const int lane = threadIdx.x & 63;
  const long slot = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long j0 = slot * RUN;
  if (j0 >= n) return;
  long j1 = j0 + RUN;
  if (j1 > n) j1 = n;
  bool active[VEC];
#pragma unroll
  for (int c = 0; c < VEC; ++c) active[c] = (64 * c + lane) * 8 < dp;
  int lo = 0, hi = K;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (start[mid] <= j0) lo = mid; else hi = mid;
  }
  int k = lo;
  long kend = start[k + 1];
  float acc[VEC][8];
#pragma unroll
  for (int c = 0; c < VEC; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[c][e] = 0.f;
  auto flush = [&](int kk) {
#pragma unroll
    for (int c = 0; c < VEC; ++c) {
      if (active[c]) {
        float* o = sums + (long)kk * ld + (64 * c + lane) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (acc[c][e] != 0.f) atomicAdd(o + e, acc[c][e]);
          acc[c][e] = 0.f;
        }
      }
    }
  };
  long j = j0;
  while (j < j1) {
    while (j >= kend) {
      flush(k);
      ++k;
      kend = start[k + 1];
    }
    const long stop = kend < j1 ? kend : j1;
    for (; j + ROWS <= stop; j += ROWS) {
      int pj[ROWS];
#pragma unroll
      for (int q = 0; q < ROWS; ++q) pj[q] = perm[j + q];
      bf16x8 v[ROWS][VEC];
#pragma unroll
      for (int q = 0; q < ROWS; ++q)
#pragma unroll
        for (int c = 0; c < VEC; ++c)
          v[q][c] = active[c] ? *(const bf16x8*)(X + (long)pj[q] * ldx + (64 * c + lane) * 8) : bf16x8{};
#pragma unroll
      for (int c = 0; c < VEC; ++c)
#pragma unroll
        for (int q = 0; q < ROWS; q += 4)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            acc[c][e] += ((float)v[q][c][e] + (float)v[q + 1][c][e]) + ((float)v[q + 2][c][e] + (float)v[q + 3][c][e]);
    }
    for (; j < stop; ++j) {
      const long r = perm[j];
#pragma unroll
      for (int c = 0; c < VEC; ++c) {
        if (active[c]) {
          const bf16x8 v = *(const bf16x8*)(X + r * ldx + (64 * c + lane) * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[c][e] += (float)v[e];
        }
      }
    }
  }
  flush(k);
}

}  // namespace

// Labels per histogram chunk: 65536 for large n; smaller for small n so the histogram and
// scatter passes still launch >= ~1500 workgroups (6 rounds over 256 CUs); >= 4096 keeps
// the per-chunk K-cursor load (K ints) amortised.
HARP_EXPORT long harp_bucket_chunk(long n) {
  long c = 65536;
  while (c > 4096 && (n + c - 1) / c < 1536) c >>= 1;
  return c;
}

HARP_EXPORT long harp_bucket_workspace_ints(long n, int K) {
  const long chunk = harp_bucket_chunk(n);
  const long nch = (n + chunk - 1) / chunk;
  const long nseg = (nch + SEG - 1) / SEG;
  // H[nch][K] + T[nseg][K] + counts[K] + start[K+1] + perm[n]
  return nch * K + nseg * K + K + (K + 1) + n;
}

// Bucket labels: fills perm[n] (indices grouped by label) and start[K+1] (bucket offsets)
// inside the workspace; returns offsets (in ints) of start and perm through out params.
HARP_EXPORT int harp_bucket_labels(const int* lab, long n, int K, int* ws, long* start_off, long* perm_off,
                                   hipStream_t s) {
  if (n <= 0 || K <= 0 || K > 16384) return HARP_EBADARG;
  const long chunk = harp_bucket_chunk(n);
  const int nch = (int)((n + chunk - 1) / chunk);
  const int nseg = (nch + SEG - 1) / SEG;
  int* H = ws;
  int* T = H + (long)nch * K;
  int* counts = T + (long)nseg * K;
  int* start = counts + K;
  int* perm = start + K + 1;
  *start_off = start - ws;
  *perm_off = perm - ws;
  const size_t lds = (size_t)K * sizeof(int);
  label_hist_kernel<<<dim3(nch), dim3(256), lds, s>>>(lab, n, K, chunk, H);
  colscan1_kernel<<<dim3((K + 255) / 256, nseg), dim3(256), 0, s>>>(H, nch, K, T);
  colscan2_kernel<<<dim3((K + 255) / 256), dim3(256), 0, s>>>(T, nseg, K, counts);
  segscan_kernel<<<dim3(1), dim3(1024), 0, s>>>(counts, K, start);
  bucket_kernel<<<dim3(nch), dim3(256), lds, s>>>(lab, n, K, chunk, H, T, start, perm);
  return harp_launch_status();
}

// sums[k][0..dp) += sum of bf16 rows X[perm[j]] for j in [start[k], start[k+1]) (sums must be
// zeroed by the caller: partial rows are added with fp32 atomics at bucket boundaries)
// X rows of dp elements at a row stride of ldx >= dp (ldx % 8 == 0).
HARP_EXPORT int harp_bucket_rowsum_bf16(const void* X, int dp, long ldx, const int* perm, const int* start, int K,
                                        long n, float* sums, int ld, hipStream_t s) {
  if (dp % 8 || dp > 1024 || ld < dp || ldx < dp || ldx % 8 || n <= 0) return n == 0 ? HARP_OK : HARP_EBADARG;
  const int lpr_min = dp / 8;
  const __bf16* Xb = (const __bf16*)X;
  constexpr int RUN = 256;
  auto grid = [&](int lpr) { return dim3((unsigned)(((n + RUN - 1) / RUN * lpr + 255) / 256)); };
  if (lpr_min <= 8) rowsum_bf16_kernel<8, RUN><<<grid(8), dim3(256), 0, s>>>(Xb, dp, ldx, perm, start, K, n, sums, ld);
  // 8 rows in flight at 16 lanes per row (dp 72..128, the K-means headline's 112): 5.13 ->
  // 5.00 ms at N = 1e8, K = 1e4 (profiles/r4_endstate/rowsum_rows.log)
  else if (lpr_min <= 16) rowsum_bf16_kernel<16, RUN, 8><<<grid(16), dim3(256), 0, s>>>(Xb, dp, ldx, perm, start, K, n, sums, ld);
  else if (lpr_min <= 32) rowsum_bf16_kernel<32, RUN><<<grid(32), dim3(256), 0, s>>>(Xb, dp, ldx, perm, start, K, n, sums, ld);
  else if (dp <= 512) rowsum_wide_bf16_kernel<1, RUN><<<grid(64), dim3(256), 0, s>>>(Xb, dp, ldx, perm, start, K, n, sums, ld);
  else rowsum_wide_bf16_kernel<2, RUN><<<grid(64), dim3(256), 0, s>>>(Xb, dp, ldx, perm, start, K, n, sums, ld);
  return harp_launch_status();
}
