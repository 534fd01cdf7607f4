// Subgraph counting by color coding (FASCIA / SAHAD) on gfx950: the two per-level
// operations of the dynamic program, in fp64 (colorful-embedding counts of big graphs
// pass 2^53 only in their totals; the reference keeps doubles too).
//
// Reference: ml/java/.../subgraph/colorcount_HJ.java (count table per sub-template,
// neighbour sums over the adjacency, color-set splits) and sahad/rotation*/ (the passive
// child's table travels the ring). Here a level is:
//   N[v, :] = sum_{u in adj(v)} M[u, :]          (csr_spmm_kernel)
//   T[v, C] = sum_{(C1, C2) split of C} A[v, C1] * N[v, C2]   (colorset_combine_kernel)
// The first replaces an index_add_ over the edge list: fp64 atomics on every (edge,
// color set) and a gathered copy of M per edge. It becomes one CSR pass with no atomics.
// Each vertex gets one wave. The lanes are (neighbour slot, color set) pairs, so one
// wave-wide load reads 64 / Cp neighbour rows of M, each row contiguous. Slot partials
// are folded with xor-shuffles.
#include "common.h"

namespace {

template <int CP>  // color sets rounded up to a power of two (<= 64)
__global__ __launch_bounds__(256) void csr_spmm_kernel(const long* __restrict__ rowptr, const int* __restrict__ col,
                                                       const double* __restrict__ M, int C, double* __restrict__ out,
                                                       long n) {
  constexpr int SLOTS = 64 / CP;
  const int lane = threadIdx.x & 63;
  const int c = lane % CP, slot = lane / CP;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long v = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < n; v += nw) {
    const long a = rowptr[v], b = rowptr[v + 1];
    double acc = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    if (c < C) {
      // four neighbour rows in flight per lane: the index -> row load chain is latency
      // bound, not bandwidth bound, at one row per wave per trip
      long j = a + slot;
      for (; j + 3 * SLOTS < b; j += 4 * SLOTS) {
        const int u0 = col[j], u1 = col[j + SLOTS], u2 = col[j + 2 * SLOTS], u3 = col[j + 3 * SLOTS];
        acc += M[(long)u0 * C + c];
        acc1 += M[(long)u1 * C + c];
        acc2 += M[(long)u2 * C + c];
        acc3 += M[(long)u3 * C + c];
      }
      for (; j < b; j += SLOTS) acc += M[(long)col[j] * C + c];
      acc += (acc1 + acc2) + acc3;
    }
#pragma unroll
    for (int o = CP; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (slot == 0 && c < C) out[v * C + c] = acc;
  }
}

// T[v, ci] = sum over the splits t in [toff[ci], toff[ci+1]) of A[v, t1[t]] * N[v, t2[t]]
// (one thread per (vertex, output color set); the split tables live in LDS)
__global__ __launch_bounds__(256) void colorset_combine_kernel(const double* __restrict__ A, int ca,
                                                               const double* __restrict__ Nn, int cn,
                                                               const int* __restrict__ toff,
                                                               const int* __restrict__ t1, const int* __restrict__ t2,
                                                               int co, int nt, double* __restrict__ out, long n) {
  extern __shared__ int sh[];
  int* s_off = sh;
  int* s_t1 = sh + co + 1;
  int* s_t2 = s_t1 + nt;
  for (int k = threadIdx.x; k <= co; k += blockDim.x) s_off[k] = toff[k];
  for (int k = threadIdx.x; k < nt; k += blockDim.x) {
    s_t1[k] = t1[k];
    s_t2[k] = t2[k];
  }
  __syncthreads();
  const long total = n * co;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long v = e / co;
    const int ci = (int)(e - v * co);
    const double* a = A + v * ca;
    const double* nn = Nn + v * cn;
    double acc = 0.0;
    for (int t = s_off[ci]; t < s_off[ci + 1]; ++t) acc = fma(a[s_t1[t]], nn[s_t2[t]], acc);
    out[e] = acc;
  }
}


// PageRank pull step (contrib simplepagerank: PageRankMapper.java accumulates
// pr(u) / outdeg(u) into every out-neighbour; here the edges are grouped by target once,
// so an iteration is a CSR gather with no atomics):
//   out[v] = alpha * sum_{u in in(v)} x[u] + b0 + b1 * (*dm)
//   xnext[v] = out[v] * invdeg[v]   (v < nx; optional: fuses the next iteration's x)
// G lanes per row (G = in-degree rounded to a power of two, 4..64), 64 / G rows per
// wave, so short web-graph rows do not leave most of a wave idle.
template <int G>
__global__ __launch_bounds__(256) void pagerank_pull_kernel(const long* __restrict__ rowptr,
                                                            const int* __restrict__ col,
                                                            const double* __restrict__ x, double alpha, double b0,
                                                            double b1, const double* __restrict__ dm,
                                                            double* __restrict__ out,
                                                            const double* __restrict__ invdeg,
                                                            double* __restrict__ xnext, long nx, long n) {
  const int sub = threadIdx.x & (G - 1);
  const double beta = b0 + (dm ? b1 * dm[0] : 0.0);
  const long ng = ((long)gridDim.x * blockDim.x) / G;
  for (long v = ((long)blockIdx.x * blockDim.x + threadIdx.x) / G; v < n; v += ng) {
    const long a = rowptr[v], b = rowptr[v + 1];
    double acc = 0.0, acc1 = 0.0;
    long j = a + sub;
    for (; j + G < b; j += 2 * G) {
      const int u0 = col[j], u1 = col[j + G];
      acc += x[u0];
      acc1 += x[u1];
    }
    if (j < b) acc += x[col[j]];
    acc += acc1;
#pragma unroll
    for (int o = 1; o < G; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (sub == 0) {
      const double r = alpha * acc + beta;
      out[v] = r;
      if (xnext && v < nx) xnext[v] = r * invdeg[v];
    }
  }
}

}  // namespace

// out[v, :] = sum of M[col[j], :] over j in [rowptr[v], rowptr[v+1]); M and out are
// row-major [*, C] fp64, C <= 64
HARP_EXPORT int harp_csr_spmm_f64(const long* rowptr, const int* col, const double* M, int C, double* out, long n,
                                  hipStream_t s) {
  if (n <= 0) return HARP_OK;
  if (C <= 0 || C > 64) return HARP_EBADARG;
  long blocks = (n + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  const dim3 g((unsigned)blocks), b(256);
  if (C <= 1) csr_spmm_kernel<1><<<g, b, 0, s>>>(rowptr, col, M, C, out, n);
  else if (C <= 2) csr_spmm_kernel<2><<<g, b, 0, s>>>(rowptr, col, M, C, out, n);
  else if (C <= 4) csr_spmm_kernel<4><<<g, b, 0, s>>>(rowptr, col, M, C, out, n);
  else if (C <= 8) csr_spmm_kernel<8><<<g, b, 0, s>>>(rowptr, col, M, C, out, n);
  else if (C <= 16) csr_spmm_kernel<16><<<g, b, 0, s>>>(rowptr, col, M, C, out, n);
  else if (C <= 32) csr_spmm_kernel<32><<<g, b, 0, s>>>(rowptr, col, M, C, out, n);
  else csr_spmm_kernel<64><<<g, b, 0, s>>>(rowptr, col, M, C, out, n);
  return harp_launch_status();
}

// out[v, ci] = sum_{t in [toff[ci], toff[ci+1])} A[v, t1[t]] * N[v, t2[t]]; all tables fp64
// row-major ([n, ca], [n, cn], [n, co]); the split tables (co + 1 + 2 nt ints) must fit in LDS
HARP_EXPORT int harp_colorset_combine_f64(const double* A, int ca, const double* Nn, int cn, const int* toff,
                                          const int* t1, const int* t2, int co, int nt, double* out, long n,
                                          hipStream_t s) {
  if (n <= 0) return HARP_OK;
  const size_t lds = sizeof(int) * ((size_t)co + 1 + 2 * (size_t)nt);
  if (co <= 0 || nt <= 0 || ca <= 0 || cn <= 0 || lds > 65536) return HARP_EBADARG;
  long blocks = (n * co + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  colorset_combine_kernel<<<dim3((unsigned)blocks), dim3(256), lds, s>>>(A, ca, Nn, cn, toff, t1, t2, co, nt, out, n);
  return harp_launch_status();
}

// one PageRank pull step over a by-target CSR (see pagerank_pull_kernel); dm, invdeg and
// xnext may be null
HARP_EXPORT int harp_pagerank_pull_f64(const long* rowptr, const int* col, const double* x, double alpha, double b0,
                                       double b1, const double* dm, double* out, const double* invdeg, double* xnext,
                                       long nx, long n, long nnz, hipStream_t s) {
  if (n <= 0) return HARP_OK;
  if (xnext && !invdeg) return HARP_EBADARG;
  const long avg = nnz / n;
  const dim3 b(256);
  auto grid = [&](int G) {
    long blocks = (n * G + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    return dim3((unsigned)blocks);
  };
  if (avg <= 4) pagerank_pull_kernel<4><<<grid(4), b, 0, s>>>(rowptr, col, x, alpha, b0, b1, dm, out, invdeg, xnext, nx, n);
  else if (avg <= 8) pagerank_pull_kernel<8><<<grid(8), b, 0, s>>>(rowptr, col, x, alpha, b0, b1, dm, out, invdeg, xnext, nx, n);
  else if (avg <= 16) pagerank_pull_kernel<16><<<grid(16), b, 0, s>>>(rowptr, col, x, alpha, b0, b1, dm, out, invdeg, xnext, nx, n);
  else if (avg <= 32) pagerank_pull_kernel<32><<<grid(32), b, 0, s>>>(rowptr, col, x, alpha, b0, b1, dm, out, invdeg, xnext, nx, n);
  else pagerank_pull_kernel<64><<<grid(64), b, 0, s>>>(rowptr, col, x, alpha, b0, b1, dm, out, invdeg, xnext, nx, n);
  return harp_launch_status();
}
