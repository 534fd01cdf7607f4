// LDA collapsed Gibbs sampling for gfx950 (MI355X / CDNA4).
//
// Replaces the reference's SparseLDA sampler (ml/java/.../lda/LDAMPTask.java:85-330:
// per token remove it from the doc-topic / word-topic / topic-sum counts, draw a new topic
// from p(k) ~ (n_dk + alpha)(n_wk + beta) / (n_k + V beta), add it back) and the
// topic-count bookkeeping. Used under model rotation: the word-topic rows of the resident
// word slice are local to this worker for the duration of a step (LDAMPCollectiveMapper).
//
// Design (MI355X-first):
//  * tokens of the resident slice are sorted by word and cut into chunks of one word;
//    ONE wave owns a chunk, holding that word's topic row n_w[*] in VGPRs (16 topics per
//    lane for K <= 1024): no atomics on the word row inside the chunk, one atomic delta
//    flush at the end (long words are split over several chunks).
//  * per token the wave reads the doc-topic row (16 ints per lane, dwordx4 loads),
//    forms the 1024 unnormalised probabilities in registers (1/(n_k + V beta) comes from
//    LDS, refreshed per launch — the reference's stale-topic-sum approximation), samples by
//    a wave-level inclusive scan + ballot, and updates n_dk with two global atomics.
//  * the token's own count is removed in registers (no read-after-atomic hazard).
//  * counter-based RNG (splitmix64 of seed, token index): reproducible, no state.
#include "common.h"

namespace {

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float wave_incl_scan(float v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

template <int TPL>  // topics per lane; K_pad = 64 * TPL
__global__ __launch_bounds__(256) void lda_cgs_kernel(
    const int* __restrict__ tdoc, const int* __restrict__ tword, int* __restrict__ tz,
    const long* __restrict__ chunk_start, long nchunks, int* __restrict__ ndk, int ldd, int* __restrict__ nwk, int ldw,
    const float* __restrict__ inv_nk, int* __restrict__ nk_delta, int K, float alpha, float beta,
    unsigned long long seed) {
  constexpr int KP = 64 * TPL;
  __shared__ float s_inv[KP];
  __shared__ int s_delta[KP];
  for (int k = threadIdx.x; k < KP; k += blockDim.x) {
    s_inv[k] = k < K ? inv_nk[k] : 0.f;
    s_delta[k] = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long wave_g = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  const int k0 = lane * TPL;
  for (long c = wave_g; c < nchunks; c += nwaves) {
    const long a = chunk_start[c], b = chunk_start[c + 1];
    const int w = tword[a];
    int* wrow = nwk + (long)w * ldw + k0;
    int nw0[TPL], nw[TPL];
#pragma unroll
    for (int t = 0; t < TPL; t += 4) {
      const int4 v = *(const int4*)(wrow + t);
      nw0[t] = v.x; nw0[t + 1] = v.y; nw0[t + 2] = v.z; nw0[t + 3] = v.w;
    }
#pragma unroll
    for (int t = 0; t < TPL; ++t) nw[t] = nw0[t];
    for (long i = a; i < b; ++i) {
      const int d = tdoc[i];
      const int z = tz[i];
      int* drow = ndk + (long)d * ldd;
      int nd[TPL];
#pragma unroll
      for (int t = 0; t < TPL; t += 4) {
        const int4 v = *(const int4*)(drow + k0 + t);
        nd[t] = v.x; nd[t + 1] = v.y; nd[t + 2] = v.z; nd[t + 3] = v.w;
      }
      // remove the token (registers; the global doc count is decremented below)
      const int zl = z / TPL, zt = z % TPL;
      float p[TPL];
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < TPL; ++t) {
        const int own = (lane == zl && t == zt) ? 1 : 0;
        nw[t] -= own;
        const float pt = ((float)(nd[t] - own) + alpha) * ((float)nw[t] + beta) * s_inv[k0 + t];
        p[t] = (k0 + t < K) ? pt : 0.f;
        s += p[t];
      }
      const float incl = wave_incl_scan(s, lane);
      const float total = __shfl(incl, 63, 64);
      const unsigned long long rbits = mix64(seed ^ ((unsigned long long)i * 0xD6E8FEB86659FD93ull));
      const float u = (float)((rbits >> 40) * (1.0 / 16777216.0)) * total;
      const unsigned long long hit = __ballot(incl > u);
      int src = hit ? (int)__builtin_ctzll(hit) : 63;
      // walk the chosen lane's topics: first t with excl + prefix(t) > u
      float acc = incl - s;
      int found = -1;
#pragma unroll
      for (int t = 0; t < TPL; ++t) {
        acc += p[t];
        if (found < 0 && acc > u) found = t;
      }
      const int sel = found < 0 ? TPL - 1 : found;
      int nz = __shfl(k0 + sel, src, 64);
      if (nz >= K) nz = K - 1;
      // add the token back with its new topic
      const int nzl = nz / TPL, nzt = nz % TPL;
#pragma unroll
      for (int t = 0; t < TPL; ++t) nw[t] += (lane == nzl && t == nzt) ? 1 : 0;
      if (lane == 0) {
        tz[i] = nz;
        if (nz != z) {
          atomicSub(drow + z, 1);
          atomicAdd(drow + nz, 1);
          atomicSub(&s_delta[z], 1);
          atomicAdd(&s_delta[nz], 1);
        }
      }
    }
    // flush this chunk's word-row delta
#pragma unroll
    for (int t = 0; t < TPL; ++t) {
      const int dlt = nw[t] - nw0[t];
      if (dlt) atomicAdd(wrow + t, dlt);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    if (s_delta[k]) atomicAdd(nk_delta + k, s_delta[k]);
}

// count tables from assignments: ndk[d][z]++, nwk[w][z]++, nk[z]++
__global__ void lda_count_kernel(const int* __restrict__ tdoc, const int* __restrict__ tword, const int* __restrict__ tz,
                                 long n, int* __restrict__ ndk, int ldd, int* __restrict__ nwk, int ldw,
                                 int* __restrict__ nk) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int z = tz[i];
    if (ndk) atomicAdd(ndk + (long)tdoc[i] * ldd + z, 1);
    if (nwk) atomicAdd(nwk + (long)tword[i] * ldw + z, 1);
    if (nk) atomicAdd(nk + z, 1);
  }
}

}  // namespace

HARP_EXPORT int harp_lda_cgs(const int* tdoc, const int* tword, int* tz, const long* chunk_start, long nchunks, int* ndk,
                             int ldd, int* nwk, int ldw, const float* inv_nk, int* nk_delta, int K, float alpha,
                             float beta, unsigned long long seed, hipStream_t s) {
  if (nchunks <= 0) return HARP_OK;
  if (K <= 0 || K > 1024 || ldd % 4 || ldw % 4) return HARP_EBADARG;
  long blocks = (nchunks + 3) / 4;  // 4 waves per block
  if (blocks > 8192) blocks = 8192;
  const dim3 g((unsigned)blocks), bl(256);
  if (K <= 256) {
    if (ldd < 256 || ldw < 256) return HARP_EBADARG;
    lda_cgs_kernel<4><<<g, bl, 0, s>>>(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, nwk, ldw, inv_nk, nk_delta, K,
                                       alpha, beta, seed);
  } else if (K <= 512) {
    if (ldd < 512 || ldw < 512) return HARP_EBADARG;
    lda_cgs_kernel<8><<<g, bl, 0, s>>>(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, nwk, ldw, inv_nk, nk_delta, K,
                                       alpha, beta, seed);
  } else {
    if (ldd < 1024 || ldw < 1024) return HARP_EBADARG;
    lda_cgs_kernel<16><<<g, bl, 0, s>>>(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, nwk, ldw, inv_nk, nk_delta, K,
                                        alpha, beta, seed);
  }
  return harp_launch_status();
}

HARP_EXPORT int harp_lda_count(const int* tdoc, const int* tword, const int* tz, long n, int* ndk, int ldd, int* nwk,
                               int ldw, int* nk, hipStream_t s) {
  if (n <= 0) return HARP_OK;
  long blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  lda_count_kernel<<<dim3((unsigned)blocks), dim3(256), 0, s>>>(tdoc, tword, tz, n, ndk, ldd, nwk, ldw, nk);
  return harp_launch_status();
}
