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

#ifdef HARP_LDA_STAMPS
// diagnostic build only (scripts/lda_stamps.py): per-phase shader-clock totals of the dense
// sampler's chunk loop: [0] prologue, [1] token loop, [2] flush, [3] chunks, [4] tokens,
// [5] whole wave
__device__ unsigned long long g_lda_stamps[8];
#endif

namespace {

// wave-uniform copies (SGPRs) of values every lane of the wave holds equally
__device__ __forceinline__ long uni64(long v) {
  return ((long)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
         (unsigned)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ float uni_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// murmur3 finalizer
__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// wave64 inclusive prefix sum on the DPP network (no LDS round trips): Hillis-Steele
// within each 16-lane row (row_shr 1, 2, 4, 8), then row_bcast:15 into rows 1 and 3
// and row_bcast:31 into rows 2 and 3. Lanes without a source add 0 (old = 0).
__device__ __forceinline__ float dpp_add(float v, int ctrl_sel) {
  int t;
  switch (ctrl_sel) {
    case 0: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false); break;
    case 1: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xf, 0xf, false); break;
    case 2: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xf, 0xf, false); break;
    case 3: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xf, 0xf, false); break;
    case 4: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false); break;
    default: t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false); break;
  }
  return v + __int_as_float(t);
}

__device__ __forceinline__ float wave_incl_scan(float v, int) {
  v = dpp_add(v, 0);
  v = dpp_add(v, 1);
  v = dpp_add(v, 2);
  v = dpp_add(v, 3);
  v = dpp_add(v, 4);
  v = dpp_add(v, 5);
  return v;
}

// a relaxed device-scope atomic add by ONE lane at a uniform row base + a byte offset that is
// laundered into a VGPR: a uniform address would be rewritten into a wave reduction (mbcnt,
// popcount and two branches around the atomic) although only one lane is active, and a
// laundered 64-bit address costs a scalar 64-bit add chain; base (SGPRs) + 32-bit VGPR
// offset is the instruction's own addressing mode
__device__ __forceinline__ void lane_atomic_add(const void* base, unsigned off, unsigned v) {
  typedef __attribute__((address_space(1))) unsigned gu32;
  typedef __attribute__((address_space(1))) char gchar;
  asm volatile("" : "+v"(off));
  __hip_atomic_fetch_add((gu32*)((gchar*)(unsigned long)base + off), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a 32-bit load / store at a uniform base + a byte offset in a VGPR (the instruction's base
// + offset addressing: no per-access 64-bit address arithmetic); ld_at takes an offset the
// caller has laundered into a VGPR once for several loads
__device__ __forceinline__ unsigned in_vgpr(unsigned v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ int ld_at(const int* base, unsigned voff) {
  typedef __attribute__((address_space(1))) const int gi32;
  typedef __attribute__((address_space(1))) const char gchar;
  return *(gi32*)((gchar*)(unsigned long)base + voff);
}
__device__ __forceinline__ void st_at(int* base, unsigned off, int v) {
  typedef __attribute__((address_space(1))) int gi32;
  typedef __attribute__((address_space(1))) char gchar;
  asm volatile("" : "+v"(off));
  *(gi32*)((gchar*)(unsigned long)base + off) = v;
}

// doc-topic row element: int (32-bit counts) or unsigned short (16-bit counts, half the
// bytes of the per-token row read that bounds this kernel; updated with 32-bit atomics
// on the containing dword: counts stay in [0, 65535], so a +-1 on one half never
// carries or borrows into the other)
template <class DT>
struct DocRow;
template <>
struct DocRow<int> {
  template <int TPL>
  __device__ static __forceinline__ void load(const int* drow, int k0, int (&nd)[TPL]) {
#pragma unroll
    for (int t = 0; t < TPL; t += 4) {
      const int4 v = *(const int4*)(drow + k0 + t);
      nd[t] = v.x; nd[t + 1] = v.y; nd[t + 2] = v.z; nd[t + 3] = v.w;
    }
  }
  __device__ static __forceinline__ void add(int* drow, int k, int v) { atomicAdd(drow + k, v); }
  __device__ static __forceinline__ void add1(int* drow, int k, int v) { lane_atomic_add(drow, 4u * k, (unsigned)v); }
};
template <>
struct DocRow<unsigned short> {
  template <int TPL>
  __device__ static __forceinline__ void load(const unsigned short* drow, int k0, int (&nd)[TPL]) {
    static_assert(TPL % 4 == 0, "TPL must be a multiple of 4");
    if constexpr (TPL % 8 != 0) {
#pragma unroll
      for (int t = 0; t < TPL; t += 4) {
        const uint2 v = *(const uint2*)(drow + k0 + t);
        nd[t] = (int)(v.x & 0xFFFFu);
        nd[t + 1] = (int)(v.x >> 16);
        nd[t + 2] = (int)(v.y & 0xFFFFu);
        nd[t + 3] = (int)(v.y >> 16);
      }
      return;
    }
#pragma unroll
    for (int t = 0; t < (TPL % 8 == 0 ? TPL : 0); t += 8) {
      const uint4 v = *(const uint4*)(drow + k0 + t);
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        nd[t + 2 * q] = (int)(w[q] & 0xFFFFu);
        nd[t + 2 * q + 1] = (int)(w[q] >> 16);
      }
    }
  }
  __device__ static __forceinline__ void add(unsigned short* drow, int k, int v) {
    unsigned* word = (unsigned*)(drow + (k & ~1));
    const unsigned sh = (k & 1) ? 16u : 0u;
    if (v > 0) atomicAdd(word, (unsigned)v << sh);
    else atomicSub(word, (unsigned)(-v) << sh);
  }
  // v = +-1 from one lane (two's complement: a -1 on a nonzero count borrows only inside
  // its own field)
  __device__ static __forceinline__ void add1(unsigned short* drow, int k, int v) {
    lane_atomic_add(drow, 2u * (k & ~1), (unsigned)v << ((k & 1) ? 16u : 0u));
  }
};

// packed uint8 counts (every doc shorter than 256 tokens, so no byte carries or borrows):
// a token's doc-row read halves again (1 KB at K_pad = 1024)
template <>
struct DocRow<unsigned char> {
  template <int TPL>
  __device__ static __forceinline__ void load(const unsigned char* drow, int k0, int (&nd)[TPL]) {
    static_assert(TPL % 4 == 0, "TPL must be a multiple of 4");
    if constexpr (TPL % 16 == 0) {
#pragma unroll
      for (int t = 0; t < TPL; t += 16) {
        const uint4 v = *(const uint4*)(drow + k0 + t);
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int b = 0; b < 4; ++b) nd[t + 4 * q + b] = (int)((w[q] >> (8 * b)) & 0xFFu);
      }
    } else if constexpr (TPL % 8 == 0) {
#pragma unroll
      for (int t = 0; t < TPL; t += 8) {
        const uint2 v = *(const uint2*)(drow + k0 + t);
        const unsigned w[2] = {v.x, v.y};
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int b = 0; b < 4; ++b) nd[t + 4 * q + b] = (int)((w[q] >> (8 * b)) & 0xFFu);
      }
    } else {
#pragma unroll
      for (int t = 0; t < TPL; t += 4) {
        const unsigned w = *(const unsigned*)(drow + k0 + t);
#pragma unroll
        for (int b = 0; b < 4; ++b) nd[t + b] = (int)((w >> (8 * b)) & 0xFFu);
      }
    }
  }
  __device__ static __forceinline__ void add(unsigned char* drow, int k, int v) {
    unsigned* word = (unsigned*)(drow + (k & ~3));
    const unsigned sh = (unsigned)(k & 3) * 8u;
    if (v > 0) atomicAdd(word, (unsigned)v << sh);
    else atomicSub(word, (unsigned)(-v) << sh);
  }
  __device__ static __forceinline__ void add1(unsigned char* drow, int k, int v) {
    lane_atomic_add(drow, (unsigned)(k & ~3), (unsigned)v << ((unsigned)(k & 3) * 8u));
  }
};

// Fused parameter-server rows (push-pull with sparse rows, models/lda.py): the word rows
// are read straight from the PULL payload (slot of local row w at pull_off[w], capacity
// pull_cap[w]; parallel/sparse_ps.py layout, csrc/rowcodec.hip slot format) into the wave's
// LDS row, and a chunk's word-row delta is written straight into the PUSH payload slot
// (dense slot: atomic adds; sparse slot: one reservation per wave on the slot's nnz word,
// entries of several chunks of one word may repeat a topic -- the owner's decode_add sums
// them). No dense local table is materialised, decoded or re-encoded.
struct PsRows {
  const unsigned char* pbuf;
  const long* poff;
  const int* pcap;
  unsigned char* qbuf;
  const long* qoff;
  const int* qcap;
  int* overflow;
};

// Dense sampler: one wave per word chunk, the word's factors qw in registers (TPL topics per
// lane), the token's doc row read per token. XW: waves per SIMD over six (variant 3: seven,
// the default). The round-1 doc-row prefetch for float rows measured slower (its VGPRs cost a
// wave per SIMD, profiles/r1_lda/ldapf); the round-5 packed uint8 path (PK below) keeps a
// row in 4 VGPRs, so it prefetches the next token's row.
template <int TPL, class DT, int XW = 0>  // topics per lane; K_pad = 64 * TPL
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6 + XW < 8 ? 6 + XW : 8, 8))) void lda_cgs_kernel(
    const int* __restrict__ tdoc, const int* __restrict__ tword, int* __restrict__ tz,
    const long* __restrict__ chunk_start, long nchunks, DT* __restrict__ ndk, int ldd, int* __restrict__ nwk, int ldw,
    const float* __restrict__ inv_nk, int* __restrict__ nk_delta, int K, float alpha, float beta,
    unsigned long long seed, int det, PsRows ps, const long* __restrict__ lpt) {
  constexpr int KP = 64 * TPL;
  constexpr int WAVES = 4;
  constexpr bool PK = sizeof(DT) == 1 && TPL == 16;  // packed-row token loop (below)
  __shared__ int s_delta[KP];
  __shared__ int s_nw0[WAVES][KP];  // per wave: the pulled word row, then the chunk's moves
  __shared__ float4 s_x[WAVES][TPL / 2];  // the drawn lane's doc counts + qw (topic walk)
  // per wave: the chunk's first kMoves moves (z | nz << 16): a chunk with few moves flushes
  // only the topics it touched. The LDS row s_nw0[wv] is all zero between chunks (the flush
  // takes each touched entry by an exchange with 0, or re-zeroes the whole row)
  constexpr int kMoves = 32;
  __shared__ unsigned s_mv[WAVES][kMoves];
  for (int k = threadIdx.x; k < KP; k += blockDim.x) {
    s_delta[k] = 0;
  }
  for (int k = threadIdx.x; k < WAVES * KP; k += blockDim.x) (&s_nw0[0][0])[k] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  // det: ONE wave samples every chunk in order (no races on doc rows: bit-reproducible,
  // independent of the word-row numbering; a test mode, launched as one workgroup)
  // wave-uniform (SGPR): the chunk bounds, the token index and its RNG are scalar work
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const long wave_g = det ? (wvu == 0 ? 0 : nchunks) : (long)blockIdx.x * (blockDim.x >> 6) + wvu;
  const long nwaves = det ? 1 : ((long)gridDim.x * blockDim.x) >> 6;
  const int k0 = lane * TPL;
  int* nw0s = &s_nw0[wv][k0];
#ifdef HARP_LDA_STAMPS
  unsigned long long st_pro = 0, st_tok = 0, st_fl = 0, st_n = 0, st_t = 0, st_t1 = 0, st_t2 = 0;
  const unsigned long long st_w0 = clock64();
#endif
  // lpt (not in det mode): chunk descriptors longest first, dealt to the resident waves in
  // snake order (round r: wave w takes rank r W + w, or r W + W-1-w on odd rounds), so every
  // wave gets about the same number of tokens (the static stride over word order left the
  // waves that drew the longest word chunks running long after the rest). A descriptor is 4
  // int64: start, length | sole << 31 | word << 32 (sole: the word's only chunk), the word's
  // pull-slot and push-slot offsets (fused rows; else 0) -- one scalar load instead of the
  // chain bounds -> word -> slot offsets.
  // det == 2: the one wave walks the descriptors in their (longest-first) order -- the
  // production schedule, sequentially (the exact-distribution test)
  const bool lptm = lpt != nullptr && det != 1;
  const unsigned seed32 = hash32((unsigned)seed ^ hash32((unsigned)(seed >> 32) ^ 0x85EBCA6Bu));
  for (long r = 0;; ++r) {
#ifdef HARP_LDA_STAMPS
    const unsigned long long st_t0 = clock64();
#endif
    long a, b, poff_c = 0, qoff_c = 0;
    int w;
    bool sole = false;  // the only chunk of its word: its push slot has no other writer
    if (lptm) {
      const long k = r * nwaves + ((r & 1) ? nwaves - 1 - wave_g : wave_g);
      if (k >= nchunks) break;
      const long* dk = lpt + 4 * k;
      a = dk[0];
      const long lw = dk[1];
      b = a + (lw & 0x7FFFFFFFL);
      sole = ((lw >> 31) & 1) != 0;
      w = (int)(lw >> 32);
      poff_c = dk[2];
      qoff_c = dk[3];
    } else {
      const long c = wave_g + r * nwaves;
      if (c >= nchunks) break;
      a = chunk_start[c];
      b = chunk_start[c + 1];
      w = tword[a];
      if (ps.pbuf) {
        poff_c = ps.poff[w];
        qoff_c = ps.qoff[w];
      }
    }
    int* wrow = nwk + (long)w * ldw + k0;
    // chunk start: every load that depends only on the descriptor is issued before any wait
    // (the first token's ids, the pull slot's capacity and entry count), then the first doc
    // row (PK) and the slot's entries: two memory round trips before the token loop instead
    // of six (vmcnt is in order: a wait for one load waits for every load issued before it)
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const int* tdoc_c = tdoc + a;
    int* tz_c = tz + a;
    const int n = (int)(b - a);
    const unsigned char* slot = ps.pbuf + poff_c;
    const int* capp = ps.pbuf ? ps.pcap + w : tdoc_c;  // (any valid address without a PS)
    const int* nnzp = ps.pbuf ? (const int*)slot : tdoc_c;
    int d_first = tdoc_c[0], z_first = tz_c[0], cap_l = *capp, nnz_l = *nnzp;
    // (one wait for all four here: the compiler would otherwise sink each load to its use)
    asm volatile("" : "+v"(d_first), "+v"(z_first), "+v"(cap_l), "+v"(nnz_l));
    int dcur = 0, zcur = 0;
    v4u rw_nx = {0u, 0u, 0u, 0u};
    if constexpr (PK) {
      dcur = __builtin_amdgcn_readfirstlane(d_first);
      zcur = __builtin_amdgcn_readfirstlane(z_first);
      rw_nx = __builtin_nontemporal_load((const v4u*)(ndk + (long)dcur * ldd + k0));
    }
    // the per-word factor qw_t = (n_wt + beta) / (n_t + V beta) in registers; a token then
    // costs ONE multiply-add per topic, p_t = (n_dt + alpha) * qw_t, and only the two topics
    // a token moves have their qw changed
    float qw[TPL];
    if (ps.pbuf) {
      // the word row from its pull slot into this wave's LDS row, scattered
      // (the row is all zero here: the previous flush left it so)
      int* lrow = &s_nw0[wv][0];
      const int cap = __builtin_amdgcn_readfirstlane(cap_l);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (cap < 0) {
        const int4* s4 = (const int4*)slot;
        // a dense slot holds the whole padded row (the PS is built with K_pad = KP ints,
        // models/lda.py): copy all of it, so topics K - K % 4 .. K - 1 are not left at 0
        for (int q = lane; q < KP / 4; q += 64) ((int4*)lrow)[q] = s4[q];
      } else {
        int nnz = __builtin_amdgcn_readfirstlane(nnz_l);
        nnz = nnz < 0 ? 0 : (nnz > cap ? cap : nnz);
        const int* cnt = (const int*)(slot + 4);
        const unsigned short* top = (const unsigned short*)(slot + 4 + 4 * (long)cap);
        for (int e = lane; e < nnz; e += 64) {
          int t = top[e], c = cnt[e];
          asm volatile("" : "+v"(t), "+v"(c));  // (both loads in flight together: e < nnz <= cap)
          if (t < K) lrow[t] = c;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int t = 0; t < TPL; t += 4) {
        const int4 v = *(const int4*)(nw0s + t);
        qw[t] = (float)v.x; qw[t + 1] = (float)v.y; qw[t + 2] = (float)v.z; qw[t + 3] = (float)v.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < TPL; t += 4) {
        const int4 v = *(const int4*)(wrow + t);
        qw[t] = (float)v.x; qw[t + 1] = (float)v.y; qw[t + 2] = (float)v.z; qw[t + 3] = (float)v.w;
      }
    }
    // qw is linear in the word count (a move changes qw_t by exactly +-1/(n_t + V beta)),
    // so no count row is kept in registers: the chunk's word-row moves are counted in this
    // wave's LDS row (zeroed here, flushed at the chunk end)
    float qs = 0.f;  // sum of this lane's qw: the token's mass is alpha * qs + sum n_dt qw_t
#pragma unroll
    for (int t = 0; t < TPL; ++t) {
      qw[t] = (qw[t] + beta) * inv_nk[k0 + t];  // (inv_nk holds K_pad entries, 0 past K)
      qs += qw[t];
    }
    if (ps.pbuf) {  // the landing row back to zero
#pragma unroll
      for (int t = 0; t < TPL; t += 4) *(int4*)(nw0s + t) = int4{0, 0, 0, 0};
    }
    int* wdel = &s_nw0[wv][0];
    int mv = 0;  // the chunk's moves (wave-uniform)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef HARP_LDA_STAMPS
    st_t1 = clock64();
    st_pro += st_t1 - st_t0;
    st_n += 1;
    st_t += b - a;
#endif
    if constexpr (PK) {
      // packed uint8 rows, 16 topics per lane: the lane's counts stay the 4 loaded dwords
      // (unpacked by one v_cvt_f32_ubyteN per use: 4 VGPRs, not 16 floats), and the NEXT
      // token's row is loaded while this token samples. The previous token's writes are
      // issued at the start of this token, before that row load: every wait then falls on
      // memory operations issued a whole token earlier (vmcnt counts stores and atomics
      // too, and the compiler's count is conservative over lane 0's branches). The row
      // loaded for this token missed only the previous token's move: applied in registers
      // when it is of the same document.
      // a chunk-relative 32-bit token index (tdoc_c, tz_c, n above): ids are loaded and
      // stored at the chunk's base pointers + a VGPR byte offset, and bounds are 32-bit
      // scalar compares
      // the draw's random key: a per-chunk hash of the start token, xored with the index
      const unsigned ckey = hash32((unsigned)a ^ seed32 ^ ((unsigned)(a >> 32) * 0x9E3779B9u));
      int d_nx, z_nx;  // ids of the token after the current one (vector loads, one token ahead)
      {
        const unsigned ix = in_vgpr(1 < n ? 4u : 0u);
        d_nx = ld_at(tdoc_c, ix);
        z_nx = ld_at(tz_c, ix);
      }
      int pd = -1, pz = 0, pnz = 0;
      float inv_cur = inv_nk[zcur];  // inv_nk of the token's topic: a scalar load one token ahead
      for (int j = 0; j < n; ++j) {
        const int d = dcur, z = zcur;
        unsigned r[4] = {rw_nx.x, rw_nx.y, rw_nx.z, rw_nx.w};
        const int dn = __builtin_amdgcn_readfirstlane(d_nx), zn = __builtin_amdgcn_readfirstlane(z_nx);
        const float inv_z = inv_cur;
        inv_cur = *(const float*)((const char*)inv_nk + 4u * (unsigned)zn);
        if (j > 0 && lane == 0) {
          st_at(tz_c, 4u * (unsigned)(j - 1), pnz);
          if (pnz != pz) {  // (the row address only when the token moved)
            DT* prow = ndk + (long)pd * ldd;
            DocRow<DT>::add1(prow, pz, -1);
            DocRow<DT>::add1(prow, pnz, 1);
          }
        }
        if (j + 1 < n) rw_nx = __builtin_nontemporal_load((const v4u*)(ndk + (long)dn * ldd + k0));
        {
          const unsigned ix = in_vgpr(4u * (unsigned)(j + 2 < n ? j + 2 : j));
          d_nx = ld_at(tdoc_c, ix);
          z_nx = ld_at(tz_c, ix);
        }
        if (d == pd && pnz != pz) {  // this row was loaded before the previous token's move
          const unsigned m1 = lane == (int)((unsigned)pz / TPL) ? 1u << (8 * (pz & 3)) : 0u;
          r[((unsigned)pz % TPL) >> 2] -= m1;  // (topics are >= 0: unsigned index arithmetic)
          const unsigned m2 = lane == (int)((unsigned)pnz / TPL) ? 1u << (8 * (pnz & 3)) : 0u;
          r[((unsigned)pnz % TPL) >> 2] += m2;
        }
        // the token's own count is left in the packed row: its removal is the product
        // correction -qw_z (after qw_z's own update) on lane z / TPL, and the walk below
        // takes 1 off topic z when it reads that lane's row
        const int zl = (unsigned)z / TPL, zt = (unsigned)z % TPL;
        const bool mez = lane == zl;
        float s;
        {  // (the lane-selected change is 0 elsewhere: x - 0 == x, no select on the write)
          const float dz = mez ? inv_z : 0.f;
          const float qn = qw[zt] - dz;
          qw[zt] = qn;
          qs -= dz;
          s = alpha * qs - (mez ? qn : 0.f);
        }
#pragma unroll
        for (int t = 0; t < TPL; ++t) s = fmaf((float)((r[t >> 2] >> (8 * (t & 3))) & 0xFFu), qw[t], s);
        const float incl = wave_incl_scan(s, lane);
        const float total = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
        // 32-bit hash of (chunk key, index): a few scalar instructions (the loop issues about
        // as many SALU as VALU instructions, both pipes ~70 % busy)
        // u = (f - 1) * total for f = 1.m in [1, 2) with the hash's top 23 bits as m: the
        // float is built by scalar bit operations, one fma (no int -> float conversion)
        const unsigned rb = hash32(ckey ^ (unsigned)j);
        const float u = fmaf(__uint_as_float(0x3F800000u | (rb >> 9)), total, -total);
        const unsigned long long hit = __builtin_amdgcn_ballot_w64(incl > u);
        const int src = hit ? (int)__builtin_ctzll(hit) : 63;
        int found;
        {  // the drawn lane's topics walked by lanes 0..15 (as below, packed counts)
          const float ex = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl - s), src));
          if (lane == src) {
#pragma unroll
            for (int t = 0; t < TPL; t += 4) s_x[wv][t / 4] = float4{qw[t], qw[t + 1], qw[t + 2], qw[t + 3]};
            ((uint4*)s_x[wv])[TPL / 4] = uint4{r[0], r[1], r[2], r[3]};
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const float* xr = (const float*)s_x[wv];
          const unsigned char* xb = (const unsigned char*)(xr + TPL);
          const float own = src == zl && lane == zt ? 1.f : 0.f;
          const float pv = lane < TPL ? ((float)xb[lane] - own + alpha) * xr[lane] : 0.f;
          float c = dpp_add(pv, 0);
          c = dpp_add(c, 1);
          c = dpp_add(c, 2);
          c = dpp_add(c, 3);
          const unsigned long long h = __builtin_amdgcn_ballot_w64(c + ex > u) & ((1ull << TPL) - 1);
          const unsigned long long nzp = __builtin_amdgcn_ballot_w64(pv > 0.f) & ((1ull << TPL) - 1);
          found = h ? (int)__builtin_ctzll(h) : (nzp ? 63 - (int)__builtin_clzll(nzp) : TPL - 1);
        }
        int nz = src * TPL + found;
        if (nz >= K) nz = K - 1;
        const int nzl = (unsigned)nz / TPL, nzt = (unsigned)nz % TPL;
        const float inv_nz = *(const float*)((const char*)inv_nk + 4u * (unsigned)nz);
        {
          const float dn = lane == nzl ? inv_nz : 0.f;
          qw[nzt] += dn;
          qs += dn;
        }
        if (lane == 0 && nz != z) {
          // byte offsets laundered into VGPRs once (per-lane LDS addresses: no wave-reduction
          // rewrite) for both rows; returnless LDS adds, no read-modify-write waits
          const unsigned zo = in_vgpr(4u * (unsigned)z), no = in_vgpr(4u * (unsigned)nz);
          atomicAdd((int*)((char*)s_delta + zo), -1);
          atomicAdd((int*)((char*)s_delta + no), 1);
          atomicAdd((int*)((char*)wdel + zo), -1);
          atomicAdd((int*)((char*)wdel + no), 1);
          if (mv < kMoves) s_mv[wv][mv] = (unsigned)z | ((unsigned)nz << 16);
        }
        mv += nz != z ? 1 : 0;
        pz = z;
        pnz = nz;
        pd = d;
        dcur = dn;
        zcur = zn;
      }
      if (lane == 0) {  // the chunk's last token
        st_at(tz_c, 4u * (unsigned)(n - 1), pnz);
        if (pnz != pz) {
          DT* prow = ndk + (long)pd * ldd;
          DocRow<DT>::add1(prow, pz, -1);
          DocRow<DT>::add1(prow, pnz, 1);
        }
      }
    } else {
      int d_next = tdoc[a], z_next = tz[a];  // token ids one ahead: the doc-row fetch then
                                             // waits on ONE memory round trip, not two
      for (long i = a; i < b; ++i) {
        const int d = d_next;
        // wave-uniform (every lane loaded the same id): the topic slot index below is then a
        // scalar, and the one-lane row updates are dynamic register indexing (s_set_gpr_idx),
        // not a select over all TPL registers
        const int z = __builtin_amdgcn_readfirstlane(z_next);
        DT* drow = ndk + (long)d * ldd;
        float nd[TPL];
        if (i + 1 < b) {
          long ix = i + 1;
          asm volatile("" : "+v"(ix));  // vector loads (a scalar load's lgkmcnt wait also covers LDS)
          d_next = tdoc[ix];
          z_next = tz[ix];
        }
        {
          int ndi[TPL];
          DocRow<DT>::template load<TPL>(drow, k0, ndi);
  #pragma unroll
          for (int t = 0; t < TPL; ++t) nd[t] = (float)ndi[t];
        }
        // remove the token: only lane z / TPL changes, at the uniform slot z % TPL. The slot is
        // read and written by dynamic register indexing with the scalar index (a loop of
        // "if (t == zt)" was if-converted into selects over all TPL registers: ~5 VALU per
        // topic per update, most of the token's VALU work)
        const int zl = z / TPL, zt = z % TPL;
        const float inv_z = inv_nk[z];
        {
          const bool me = lane == zl;
          const float dv = nd[zt], qv = qw[zt];
          nd[zt] = me ? dv - 1.f : dv;
          qw[zt] = me ? qv - inv_z : qv;
          qs -= me ? inv_z : 0.f;
        }
        float s = alpha * qs;
  #pragma unroll
        for (int t = 0; t < TPL; ++t) s = fmaf(nd[t], qw[t], s);
        const float incl = wave_incl_scan(s, lane);
        const float total = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
        const unsigned long long rbits = mix64(seed ^ ((unsigned long long)i * 0xD6E8FEB86659FD93ull));
        const float u = ((float)(unsigned)(rbits >> 40) * (1.f / 16777216.f)) * total;
        const unsigned long long hit = __ballot(incl > u);
        const int src = hit ? (int)__builtin_ctzll(hit) : 63;
        // walk the chosen lane's topics: the lane hands its TPL counts and factors to lanes
        // 0 .. TPL-1 through LDS (one topic per lane, a 16-lane DPP row scan, one ballot)
        // instead of every lane walking its own TPL topics (~3 VALU per topic, a third of the
        // token's VALU work)
        int found;
        {
          const float ex = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl - s), src));
          if (lane == src) {
  #pragma unroll
            for (int t = 0; t < TPL; t += 4) {
              s_x[wv][t / 4] = float4{nd[t], nd[t + 1], nd[t + 2], nd[t + 3]};
              s_x[wv][TPL / 4 + t / 4] = float4{qw[t], qw[t + 1], qw[t + 2], qw[t + 3]};
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const float* xr = (const float*)s_x[wv];
          const float pv = lane < TPL ? (xr[lane] + alpha) * xr[TPL + lane] : 0.f;
          float c = dpp_add(pv, 0);
          c = dpp_add(c, 1);
          c = dpp_add(c, 2);
          c = dpp_add(c, 3);  // inclusive prefix over lanes 0..15 (one DPP row)
          const unsigned long long h = __ballot(lane < TPL && c + ex > u) & ((1ull << TPL) - 1);
          const unsigned long long nzp = __ballot(pv > 0.f) & ((1ull << TPL) - 1);
          found = h ? (int)__builtin_ctzll(h) : (nzp ? 63 - (int)__builtin_clzll(nzp) : TPL - 1);
        }
        int nz = src * TPL + found;
        if (nz >= K) nz = K - 1;
        // add the token back with its new topic (uniform slot: dynamic register indexing)
        const int nzl = nz / TPL, nzt = nz % TPL;
        const float inv_nz = inv_nk[nz];
        {
          const bool me = lane == nzl;
          const float qv = qw[nzt];
          qw[nzt] = me ? qv + inv_nz : qv;
          qs += me ? inv_nz : 0.f;
        }
        if (lane == 0) {
          tz[i] = nz;
          if (nz != z) {
            DocRow<DT>::add1(drow, z, -1);
            DocRow<DT>::add1(drow, nz, 1);
            atomicSub(&s_delta[z], 1);
            atomicAdd(&s_delta[nz], 1);
            wdel[z] -= 1;
            wdel[nz] += 1;
            if (mv < kMoves) s_mv[wv][mv] = (unsigned)z | ((unsigned)nz << 16);
          }
        }
        mv = __builtin_amdgcn_readfirstlane(mv + (nz != z ? 1 : 0));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // lane 0's row moves -> every lane
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef HARP_LDA_STAMPS
    st_t2 = clock64();
    st_tok += st_t2 - st_t1;
#endif
    // flush this chunk's word-row delta. Up to kMoves moves: lanes 0 .. 2 mv - 1 take one
    // touched topic each from the move list and its delta by an LDS exchange with 0 (a topic
    // touched twice is taken by one lane, the other reads 0); more: every lane its TPL topics
    // of the row, then zeroes them
    const bool lst = mv <= kMoves;
    int lt = 0, ldl = 0;
    if (lst && lane < 2 * mv) {
      const unsigned e = s_mv[wv][lane >> 1];
      lt = (lane & 1) ? (int)(e >> 16) : (int)(e & 0xFFFFu);
      ldl = atomicExch(&wdel[lt], 0);
    }
    if (ps.qbuf) {
      unsigned char* slot = ps.qbuf + qoff_c;
      const int cap = ps.qcap[w];
      if (cap < 0) {
        if (lst) {
          if (ldl) atomicAdd((int*)slot + lt, ldl);
        } else {
#pragma unroll
          for (int t = 0; t < TPL; ++t) {
            const int dlt = nw0s[t];
            if (dlt) atomicAdd((int*)slot + k0 + t, dlt);
          }
        }
      } else {
        int mine = 0;
        if (lst) {
          mine = ldl != 0 ? 1 : 0;
        } else {
#pragma unroll
          for (int t = 0; t < TPL; ++t) mine += nw0s[t] != 0 ? 1 : 0;
        }
        const float incl = wave_incl_scan((float)mine, lane);
        const int tot = (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
        int base = 0;
        if (tot) {
          // the sole chunk of its word writes the slot's count (zeroed push payload, no other
          // writer this sweep): no returning atomic, whose round trip ended every chunk
          if (sole) {
            if (lane == 0) *(int*)slot = tot;
          } else {
            if (lane == 0) base = atomicAdd((int*)slot, tot);
            base = __builtin_amdgcn_readfirstlane(base);
          }
        }
        int pos = base + (int)incl - mine;
        int* cnt = (int*)(slot + 4);
        unsigned short* top = (unsigned short*)(slot + 4 + 4 * (long)cap);
        bool over = false;
        if (lst) {
          if (ldl) {
            if (pos < cap) {
              cnt[pos] = ldl;
              top[pos] = (unsigned short)lt;
            } else {
              over = true;
            }
          }
        } else {
#pragma unroll
          for (int t = 0; t < TPL; ++t) {
            const int dlt = nw0s[t];
            if (dlt) {
              if (pos < cap) {
                cnt[pos] = dlt;
                top[pos] = (unsigned short)(k0 + t);
              } else {
                over = true;
              }
              ++pos;
            }
          }
        }
        if (__ballot(over) && lane == 0) ps.overflow[0] = 1;
      }
    } else if (lst) {
      if (ldl) atomicAdd(nwk + (long)w * ldw + lt, ldl);
    } else {
#pragma unroll
      for (int t = 0; t < TPL; ++t) {
        const int dlt = nw0s[t];
        if (dlt) atomicAdd(wrow + t, dlt);
      }
    }
    if (!lst) {
#pragma unroll
      for (int t = 0; t < TPL; t += 4) *(int4*)(nw0s + t) = int4{0, 0, 0, 0};
    }
#ifdef HARP_LDA_STAMPS
    st_fl += clock64() - st_t2;
#endif
  }
#ifdef HARP_LDA_STAMPS
  if (lane == 0) {
    atomicAdd(&g_lda_stamps[0], st_pro);
    atomicAdd(&g_lda_stamps[1], st_tok);
    atomicAdd(&g_lda_stamps[2], st_fl);
    atomicAdd(&g_lda_stamps[3], st_n);
    atomicAdd(&g_lda_stamps[4], st_t);
    atomicAdd(&g_lda_stamps[5], clock64() - st_w0);
  }
#endif
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    if (s_delta[k]) atomicAdd(nk_delta + k, s_delta[k]);
}

// count tables from assignments: ndk[d][z]++, nwk[w][z]++, nk[z]++
template <class DT>
__global__ void lda_count_kernel(const int* __restrict__ tdoc, const int* __restrict__ tword, const int* __restrict__ tz,
                                 long n, DT* __restrict__ ndk, int ldd, int* __restrict__ nwk, int ldw,
                                 int* __restrict__ nk) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int z = tz[i];
    if (ndk) DocRow<DT>::add(ndk + (long)tdoc[i] * ldd, z, 1);
    if (nwk) atomicAdd(nwk + (long)tword[i] * ldw + z, 1);
    if (nk) atomicAdd(nk + z, 1);
  }
}


// ---------------------------------------------------------------------------------------
// Sparse-doc sampler (any K <= 32768; the only path for K > 1024 — BASELINE #5 runs
// K = 10,000). The reference's SparseLDA (LDAMPTask.java:85-330) splits
//   p(t) ~ (n_dt + alpha) * qw_t,   qw_t = (n_wt + beta) / (n_t + V beta)
// into a doc bucket sum_t n_dt qw_t and a smoothing bucket alpha * sum_t qw_t. Here the
// doc bucket is formed WITHOUT doc-topic counts: sum_t n_dt qw_t == sum over the doc's
// other tokens j of qw[z_j], so a token reads its document's topic list (zdoc, doc
// order, 2 B per token: a few hundred bytes, not a K-wide row) and gathers qw from LDS.
//  * ONE workgroup per word chunk; the word's qw[Kp] row lives in LDS (4 B x Kp: 40 KB at
//    K = 10,000, four 8-wave workgroups per CU; 128 KB at the K = 32768 limit, one per CU) and the workgroup's waves sample the
//    chunk's tokens round-robin. qw is linear in the count (a move changes qw_t by exactly
//    +-1/(n_t + V beta)), so moves are LDS float atomics on qw itself and no count row is
//    kept (an 8 B/topic {count, qw} layout fitted only two workgroups per CU: 0.85e9 vs
//    1.14e9 tokens/s at K = 10,000).
//  * the smoothing bucket is a two-level draw: per-64-topic block sums of qw (LDS, moved
//    by exactly +-1/(n_t + V beta) per token move, rebuilt per chunk) pick the block with
//    one wave scan, a second scan over the block's 64 topics picks the topic — ~60
//    instructions instead of a K-wide scan (which bounded the first version at
//    3.5e8 tokens/s for K = 10,000);
//  * doc-bucket draws scan the doc list; the lane holding the draw walks its elements;
//  * chunks are handed out by an atomic work counter in ``order`` (longest first): the
//    grid is only the resident workgroups, and a static chunk stride left the CUs
//    waiting on the few longest words;
//  * the next token's ids are fetched one token ahead (the doc range read is otherwise
//    a chain of three dependent memory round trips);
//  * zdoc and the word row are read with non-temporal loads (past the CU L1, which other
//    CUs' writes do not invalidate);
//  * word-row moves go straight to the global n_wk row (two atomics) so chunks of one
//    word on different workgroups stay exact; doc-topic counts (when kept) and topic-sum
//    deltas are updated with atomics as in the dense kernel.
// SPAN: tspan[i] = doc_off[doc of token i] | (doc length << 40), precomputed per token, so the
// next token's doc range needs no dependent doc_off load (no doc-topic table, no doc ids)
template <int WAVES, class DT, bool SPAN = false>
// (16-wave workgroups forced to 64 VGPRs for eight waves per SIMD measured slower at K = 10,000:
// 57.2 vs 54.6 ms rotation, with a worse likelihood from more concurrent chunk tokens;
// profiles/r6_sparse/waves_*.log)
__global__ __launch_bounds__(64 * WAVES) void lda_cgs_sparse_kernel(
    const int* __restrict__ tdoc, const long* __restrict__ tspan, const int* __restrict__ tword, int* __restrict__ tz,
    const long* __restrict__ chunk_start, long nchunks, const int* __restrict__ order, int* __restrict__ work,
    const long* __restrict__ tpos, const long* __restrict__ doc_off, unsigned short* __restrict__ zdoc,
    DT* __restrict__ ndk, int ldd,
    int* __restrict__ nwk, int ldw, const float* __restrict__ inv_nk, int* __restrict__ nk_delta, int K, int Kp,
    float alpha, float beta, unsigned long long seed, int ldelta, int wdelta, PsRows ps) {
  extern __shared__ float smem[];
  // fused parameter-server rows (ps.pbuf != null, the dense kernel's PsRows contract): a
  // chunk's qw row is built from its word's PULL slot and the chunk's word-row moves go to
  // the word's PUSH slot (no dense local table, no decode / delta re-encode around the sweep);
  // chunks of one word see the sweep-start counts plus their own moves
  const bool fused = ps.pbuf != nullptr;
  float* s_qw = smem;
  // ldelta: this workgroup's topic-sum deltas accumulate in LDS (after s_qw) and are
  // flushed once when it exits, instead of two global atomics per moved token on only K
  // addresses shared by every workgroup of the GPU
  int* s_nkd = ldelta ? (int*)(smem + Kp) : nullptr;
  // wdelta: each wave gathers its word-row moves in a private LDS row (plain adds by lane 0)
  // and adds them to the global word row every WFLUSH of its tokens and at the chunk end,
  // so other workgroups starting a chunk of the same word see the moves at most WFLUSH
  // tokens late (a once-per-chunk flush cost 0.36 % likelihood after 5 sweeps)
  constexpr int WFLUSH = 16;
  // wdelta == 2 (Kp > 1024, no room for per-wave rows): one workgroup row right after s_qw,
  // LDS atomics, flushed at the chunk end
  int* s_wd = wdelta == 1 ? (int*)(smem + 2 * Kp) + (long)(threadIdx.x >> 6) * Kp
                          : wdelta == 2 ? (int*)(smem + (ldelta ? 2 : 1) * Kp) : nullptr;
  __shared__ float s_bs[512];  // per-64-topic block sums of qw (Kp <= 32768)
  __shared__ float s_q;
  // no LDS delta row (wdelta == 0, K > 4096): each wave keeps its moves in a list and writes
  // them out together -- into a sparse push slot as (-1, z), (+1, nz) entries with ONE slot
  // reservation per kMvList moves (one returning atomic per move had stalled the wave for a
  // global round trip twice per moved token: K = 10,000 push-pull 68.7 -> 55.7 ms), into a
  // dense slot / the global word row and the topic-sum deltas as 64-lane atomics (every
  // kMvFlush moves when other workgroups read the global row: at most that many moves late)
  constexpr int kMvList = 64, kMvFlush = 16;
  // wdelta == 0: the move lists [WAVES][kMvList] in the dynamic LDS after s_qw
  unsigned* s_mvl_base = (unsigned*)(smem + Kp);
  auto s_mvl_at = [&](int w, int i) -> unsigned& { return s_mvl_base[w * kMvList + i]; };
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int nb = Kp >> 6;
  __shared__ int s_c;
  if (ldelta)
    for (int t = threadIdx.x; t < Kp; t += 64 * WAVES) s_nkd[t] = 0;
  if (wdelta == 1)
    for (int t = threadIdx.x & 63; t < Kp; t += 64) s_wd[t] = 0;
  for (;;) {
    __syncthreads();  // the previous chunk's samplers are done with the LDS rows (and s_c)
    if (threadIdx.x == 0) s_c = atomicAdd(work, 1);
    __syncthreads();
    if (s_c >= nchunks) break;
    const long c = order ? order[s_c] : s_c;
    const long a = chunk_start[c], b = chunk_start[c + 1];
    const int wl = tword[a];
    int* wrow = fused ? nullptr : nwk + (long)wl * ldw;
    unsigned char* qslot = fused ? ps.qbuf + ps.qoff[wl] : nullptr;
    const int qcap = fused ? ps.qcap[wl] : 0;
    // one word-row move of v (+-1 or a flushed sum) for topic t: the global row, or the
    // push slot (dense: add at t; sparse: one reserved (count, topic) entry -- entries of
    // several flushes may repeat a topic, the owner's decode_add sums them)
    auto put_move = [&](int t, int v) {
      if (!fused) {
        atomicAdd(wrow + t, v);
      } else if (qcap < 0) {
        atomicAdd((int*)qslot + t, v);
      } else {
        const int pos = atomicAdd((int*)qslot, 1);
        if (pos < qcap) {
          ((int*)(qslot + 4))[pos] = v;
          ((unsigned short*)(qslot + 4 + 4 * (long)qcap))[pos] = (unsigned short)t;
        } else {
          ps.overflow[0] = 1;
        }
      }
    };
    // a delta row (this wave's topics t0, t0 + stride, ...) -> global row / push slot, all 64
    // lanes; into a sparse push slot with ONE reservation per wave (a scan of the lanes'
    // nonzero counts), not one atomic on the slot's nnz word per entry
    auto flush_row = [&](int* row, int t0, int stride) {
      if (!fused || qcap < 0) {
        for (int t = t0; t < K; t += stride) {
          const int v = row[t];
          if (v) {
            put_move(t, v);
            row[t] = 0;
          }
        }
        return;
      }
      int mine = 0;
      for (int t = t0; t < K; t += stride) mine += row[t] != 0 ? 1 : 0;
      const float incl = wave_incl_scan((float)mine, lane);
      const int tot = (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
      if (tot == 0) return;
      int base = 0;
      if (lane == 0) base = atomicAdd((int*)qslot, tot);
      base = __builtin_amdgcn_readfirstlane(base);
      int pos = base + (int)incl - mine;
      int* cnt = (int*)(qslot + 4);
      unsigned short* top = (unsigned short*)(qslot + 4 + 4 * (long)qcap);
      bool over = false;
      for (int t = t0; t < K; t += stride) {
        const int v = row[t];
        if (v) {
          if (pos < qcap) {
            cnt[pos] = v;
            top[pos] = (unsigned short)t;
          } else {
            over = true;
          }
          ++pos;
          row[t] = 0;
        }
      }
      if (__ballot(over) && lane == 0) ps.overflow[0] = 1;
    };
    auto flush_wd = [&]() { flush_row(s_wd, lane, 64); };  // this wave's word-row moves
    const bool mvlist = wdelta == 0;
    const int mv_cap = fused ? kMvList : kMvFlush;
    int nmv = 0;  // moves in this wave's list (wave-uniform)
    auto flush_mv = [&]() {
      if (nmv == 0) return;
      const bool sparse_slot = fused && qcap >= 0;
      int base = 0;
      if (sparse_slot) {
        if (lane == 0) base = atomicAdd((int*)qslot, 2 * nmv);
        base = __builtin_amdgcn_readfirstlane(base);
      }
      if (lane < nmv) {
        const unsigned m = s_mvl_at(wv, lane);
        const int zo = (int)(m & 0xFFFFu), zn = (int)(m >> 16);
        if (sparse_slot) {
          int* cnt = (int*)(qslot + 4);
          unsigned short* top = (unsigned short*)(qslot + 4 + 4 * (long)qcap);
          const int pos = base + 2 * lane;
          if (pos + 1 < qcap) {
            cnt[pos] = -1;
            top[pos] = (unsigned short)zo;
            cnt[pos + 1] = 1;
            top[pos + 1] = (unsigned short)zn;
          } else {
            ps.overflow[0] = 1;
          }
        } else {
          int* row = fused ? (int*)qslot : wrow;
          atomicSub(row + zo, 1);
          atomicAdd(row + zn, 1);
        }
        if (!ldelta) {
          atomicSub(nk_delta + zo, 1);
          atomicAdd(nk_delta + zn, 1);
        }
      }
      nmv = 0;
    };
    int ntok = 0;
    if (!fused) {
      for (int t = threadIdx.x; t < Kp; t += 64 * WAVES) {
        s_qw[t] = t < K ? ((float)__builtin_nontemporal_load(wrow + t) + beta) * inv_nk[t] : 0.f;
        if (wdelta == 2) s_wd[t] = 0;
      }
    } else {
      const unsigned char* pslot = ps.pbuf + ps.poff[wl];
      const int pcap = ps.pcap[wl];
      if (pcap < 0) {  // dense slot: the whole padded row
        for (int t = threadIdx.x; t < Kp; t += 64 * WAVES) {
          s_qw[t] = t < K ? ((float)((const int*)pslot)[t] + beta) * inv_nk[t] : 0.f;
          if (wdelta == 2) s_wd[t] = 0;
        }
      } else {  // sparse slot: the smoothing value everywhere, then the row's nonzeros
        for (int t = threadIdx.x; t < Kp; t += 64 * WAVES) {
          s_qw[t] = t < K ? beta * inv_nk[t] : 0.f;
          if (wdelta == 2) s_wd[t] = 0;
        }
        __syncthreads();
        int nnz = *(const int*)pslot;
        nnz = nnz < 0 ? 0 : (nnz > pcap ? pcap : nnz);
        const int* cnt = (const int*)(pslot + 4);
        const unsigned short* top = (const unsigned short*)(pslot + 4 + 4 * (long)pcap);
        for (int e = threadIdx.x; e < nnz; e += 64 * WAVES) {  // a row's topics are distinct
          const int t = top[e];
          if (t < K) s_qw[t] = ((float)cnt[e] + beta) * inv_nk[t];
        }
      }
    }
    __syncthreads();
    for (int k = wv; k < nb; k += WAVES) {
      const float v = wave_incl_scan(s_qw[64 * k + lane], lane);
      if (lane == 63) s_bs[k] = v;
    }
    __syncthreads();
    if (wv == 0) {
      float v = 0.f;
      for (int k = lane; k < nb; k += 64) v += s_bs[k];
      v = wave_incl_scan(v, lane);
      if (lane == 63) s_q = v;
    }
    __syncthreads();
    // every per-token value below is wave-uniform (the wave samples ONE token at a time):
    // they are read into SGPRs (readfirstlane), so the doc-list bounds, positions and the
    // RNG are scalar work and each lane's list entry is a 32-bit offset from a scalar base
    // (the 64-bit per-lane index arithmetic of the first form was a third of the loop's VALU
    // instructions; PMC of the round-5 kernel: 190 VALU per token, VALU-bound at 81 %)
    const long a_u = uni64(a), b_u = uni64(b);
    long i = a_u + wvu;
    int d = 0, z = 0;
    long p = 0, lo = 0;
    int len = 0;
    float inv_z = 0.f;
    // the first 128 entries of the token's doc list sit in registers (zv0: lo + lane, zv1:
    // lo + 64 + lane), loaded one token ahead; the (rare) rest is read in the loop
    int zv0 = 0, zv1 = 0;
    if (i < b_u) {
      z = __builtin_amdgcn_readfirstlane(tz[i]);
      p = uni64(tpos[i]);
      if constexpr (SPAN) {
        const long sp = uni64(tspan[i]);
        lo = sp & ((1L << 40) - 1);
        len = (int)(sp >> 40);
      } else {
        d = __builtin_amdgcn_readfirstlane(tdoc[i]);
        lo = uni64(doc_off[d]);
        len = (int)(uni64(doc_off[d + 1]) - lo);
      }
      inv_z = uni_f(inv_nk[z]);
      const unsigned short* zb = zdoc + lo;
      if (lane < len) zv0 = __builtin_nontemporal_load(zb + lane);
      if (64 + lane < len) zv1 = __builtin_nontemporal_load(zb + 64 + lane);
    }
    // the ids (span or doc, topic, list position) are loaded TWO tokens ahead into VGPRs
    // through a VGPR index (vector loads, after the doc-list sum, so that sum waits only on
    // its own list): a scalar load of them, or a readfirstlane next to the load, put a full
    // memory round trip in every token (s_waitcnt lgkmcnt also covers the LDS reads)
    auto load_ids = [&](long t, long& sp, int& dd, int& zz, long& pp) {
      long ix = t < b_u ? t : b_u - 1;  // clamped: no branch around the loads
      asm volatile("" : "+v"(ix));
      if constexpr (SPAN) sp = tspan[ix];
      else dd = tdoc[ix];
      zz = tz[ix];
      pp = tpos[ix];
    };
    long sp1 = 0, pp1 = 0;
    int dd1 = 0, zz1 = 0;
    load_ids(i + WAVES, sp1, dd1, zz1, pp1);
    for (; i < b_u; i += WAVES) {
      const long inx = i + WAVES;
      const unsigned short* zb = zdoc + lo;
      const int pl = (int)(p - lo);  // this token's own entry in its doc list
      const float qz = s_qw[z] - inv_z;  // z's factor without this token
      float sb = 0.f;
      if (lane < len && lane != pl) sb += zv0 == z ? qz : s_qw[zv0];
      if (64 + lane < len && 64 + lane != pl) sb += zv1 == z ? qz : s_qw[zv1];
      // the rest of a long document's list (clueweb1 averages 392 tokens per doc): four
      // entries per lane per round with their loads issued together (one memory round trip
      // per 256 entries, not per 64), added in list order as before
      // (a predicated form that also batches the last < 256 entries took 81 VGPRs and ran
      // 1.99 vs 1.54 s per clueweb1 half-share sweep)
      int j = 128 + lane;
      for (; j + 192 < len; j += 256) {
        int zq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) zq[q] = __builtin_nontemporal_load(zb + j + 64 * q);
#pragma unroll
        for (int q = 0; q < 4; ++q) sb += j + 64 * q == pl ? 0.f : (zq[q] == z ? qz : s_qw[zq[q]]);
      }
      for (; j < len; j += 64) {
        const int zj = __builtin_nontemporal_load(zb + j);
        sb += j == pl ? 0.f : (zj == z ? qz : s_qw[zj]);
      }
      long sp2 = 0, pp2 = 0;
      int dd2 = 0, zz2 = 0;
      load_ids(i + 2 * WAVES, sp2, dd2, zz2, pp2);
      const float inclb = wave_incl_scan(sb, lane);
      const float B = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inclb), 63));
      const float corr = inv_z;
      const float A = alpha * fmaxf(uni_f(s_q) - corr, 0.f);
      const unsigned long long rbits = mix64(seed ^ ((unsigned long long)i * 0xD6E8FEB86659FD93ull));
      const float u = ((float)(unsigned)(rbits >> 40) * (1.f / 16777216.f)) * (A + B);
      // next token's doc range and topic factor: its ids have arrived by now
      long lon = 0;
      int lenn = 0;
      float invn = 0.f;
      int zn0 = 0, zn1 = 0;
      const int zn = __builtin_amdgcn_readfirstlane(zz1);
      const long pn = uni64(pp1);
      const int dn = SPAN ? 0 : __builtin_amdgcn_readfirstlane(dd1);
      if (inx < b_u) {
        if constexpr (SPAN) {
          const long spn = uni64(sp1);
          lon = spn & ((1L << 40) - 1);
          lenn = (int)(spn >> 40);
        } else {
          lon = uni64(doc_off[dn]);
          lenn = (int)(uni64(doc_off[dn + 1]) - lon);
        }
        invn = uni_f(inv_nk[zn]);
        // the next token's doc list, in flight while this token samples
        const unsigned short* zbn = zdoc + lon;
        if (lane < lenn) zn0 = __builtin_nontemporal_load(zbn + lane);
        if (64 + lane < lenn) zn1 = __builtin_nontemporal_load(zbn + 64 + lane);
      }
      int nz;
      if (u < B) {  // doc bucket: the topic of one of the doc's other tokens
        const unsigned long long hit = __ballot(inclb > u);
        const int src = hit ? (int)__builtin_ctzll(hit) : 63;
        int f = z;
        if (lane == src) {
          float pre = inclb - sb;
          bool done = false;
          for (int q = 0; q < 2 && !done; ++q) {  // the two entries held in registers
            const int jq = lane + 64 * q;
            if (jq >= len) break;
            if (jq == pl) continue;
            const int zj = q == 0 ? zv0 : zv1;
            f = zj;
            pre += zj == z ? qz : s_qw[zj];
            done = pre > u;
          }
          int jw = lane + 128;
          for (; !done && jw + 192 < len; jw += 256) {  // then four loads per round trip
            int zq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) zq[q] = __builtin_nontemporal_load(zb + jw + 64 * q);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (!done && jw + 64 * q != pl) {
                f = zq[q];
                pre += zq[q] == z ? qz : s_qw[zq[q]];
                done = pre > u;
              }
            }
          }
          for (; !done && jw < len; jw += 64) {
            if (jw == pl) continue;
            const int zj = __builtin_nontemporal_load(zb + jw);
            f = zj;
            pre += zj == z ? qz : s_qw[zj];
            done = pre > u;
          }
        }
        nz = __builtin_amdgcn_readlane(f, src);
      } else {  // smoothing bucket: block by block sums, then topic within the block
        const float u2 = (u - B) / alpha;
        const int zb6 = z >> 6;
        float sd = 0.f;
        for (int k = lane; k < nb; k += 64) sd += s_bs[k] - (k == zb6 ? corr : 0.f);
        const float incld = wave_incl_scan(sd, lane);
        const unsigned long long hit = __ballot(incld > u2);
        const int src = hit ? (int)__builtin_ctzll(hit) : 63;
        int fb = nb - 1;
        float base = 0.f;
        if (lane == src) {
          float pre = incld - sd;
          for (int k = lane; k < nb; k += 64) {
            const float v = s_bs[k] - (k == zb6 ? corr : 0.f);
            fb = k;
            base = pre;
            if (pre + v > u2) break;
            pre += v;
          }
        }
        fb = __builtin_amdgcn_readlane(fb, src);
        base = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(base), src));
        const int t = 64 * fb + lane;
        const float q = t < K ? (t == z ? qz : s_qw[t]) : 0.f;
        const float inclt = wave_incl_scan(q, lane) + base;
        const unsigned long long h2 = __ballot(inclt > u2);
        const unsigned long long pos = __ballot(q > 0.f);
        const int s2 = h2 ? (int)__builtin_ctzll(h2) : (pos ? 63 - (int)__builtin_clzll(pos) : 0);
        nz = 64 * fb + s2;
      }
      if (nz < 0 || nz >= K) nz = z;
      if (lane == 0) {
        tz[i] = nz;
        if (nz != z) {
          zdoc[p] = (unsigned short)nz;
          if (!SPAN && ndk) {
            DocRow<DT>::add(ndk + (long)d * ldd, z, -1);
            DocRow<DT>::add(ndk + (long)d * ldd, nz, 1);
          }
          const float inv_nz = inv_nk[nz];
          atomicAdd(&s_qw[z], -inv_z);
          atomicAdd(&s_qw[nz], inv_nz);
          atomicAdd(&s_bs[z >> 6], -inv_z);
          atomicAdd(&s_bs[nz >> 6], inv_nz);
          atomicAdd(&s_q, inv_nz - inv_z);
          if (wdelta == 1) {
            s_wd[z] -= 1;
            s_wd[nz] += 1;
          } else if (wdelta == 2) {
            atomicSub(&s_wd[z], 1);
            atomicAdd(&s_wd[nz], 1);
          } else if (mvlist) {
            s_mvl_at(wv, nmv) = (unsigned)z | ((unsigned)nz << 16);
          } else {
            put_move(z, -1);
            put_move(nz, 1);
          }
          if (ldelta) {
            atomicSub(&s_nkd[z], 1);
            atomicAdd(&s_nkd[nz], 1);
          } else if (!mvlist) {  // (with the move list: flushed with it)
            atomicSub(nk_delta + z, 1);
            atomicAdd(nk_delta + nz, 1);
          }
        }
      }
      // the next token's LDS reads (all lanes) must follow lane 0's row update: lanes of
      // one wave are separate threads to the compiler, so order them explicitly
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (mvlist && nz != z && ++nmv == mv_cap) {
        flush_mv();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // lane 0's next list writes follow the reads
      }
      if (wdelta == 1 && !fused && ++ntok % WFLUSH == 0) {
        flush_wd();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // lane 0's next adds follow the reset
      }
      // the next token of the same document: its prefetched list missed this token's move
      if ((SPAN ? lon == lo : dn == d) && nz != z && inx < b_u) {
        if (lane == pl) zn0 = nz;
        if (64 + lane == pl) zn1 = nz;
      }
      d = dn;
      z = zn;
      p = pn;
      lo = lon;
      len = lenn;
      inv_z = invn;
      zv0 = zn0;
      zv1 = zn1;
      sp1 = sp2;
      dd1 = dd2;
      zz1 = zz2;
      pp1 = pp2;
    }
    if (mvlist) {
      flush_mv();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    if (wdelta == 1) {
      flush_wd();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    } else if (wdelta == 2) {
      __syncthreads();  // every wave's moves of this chunk are in the row
      flush_row(s_wd, threadIdx.x, 64 * WAVES);  // zeroes it too (re-zeroed per chunk anyway)
    }
  }
  if (ldelta) {  // every wave left the chunk loop together (the break follows a barrier)
    for (int t = threadIdx.x; t < K; t += 64 * WAVES)
      if (s_nkd[t]) atomicAdd(nk_delta + t, s_nkd[t]);
  }
}

}  // namespace

namespace {
// workgroups of the dense sampler resident at once on this device (occupancy x CUs)
template <class DT, int XW>
long resident_blocks(int K) {
  static long cached[3] = {0, 0, 0};
  const int slot = K <= 256 ? 0 : K <= 512 ? 1 : 2;
  if (cached[slot]) return cached[slot];
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  hipError_t e = slot == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lda_cgs_kernel<4, DT, XW>, 256, 0)
                 : slot == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lda_cgs_kernel<8, DT, XW>, 256, 0)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lda_cgs_kernel<16, DT, XW>, 256, 0);
  if (e != hipSuccess || per <= 0) return 0;
  cached[slot] = (long)per * cus;
  return cached[slot];
}

template <class DT, int XW = 0>
int launch_cgs(const int* tdoc, const int* tword, int* tz, const long* chunk_start, long nchunks, DT* ndk, int ldd,
               int* nwk, int ldw, const float* inv_nk, int* nk_delta, int K, float alpha, float beta,
               unsigned long long seed, int det, PsRows ps, const long* lpt, hipStream_t s) {
  long blocks = (nchunks + 3) / 4;  // 4 waves per block
  if (blocks > 8192) blocks = 8192;
  if (lpt && !det) {  // the snake deal assumes every wave is resident: one wave per slot
    const long res = resident_blocks<DT, XW>(K);
    if (res > 0 && blocks > res) blocks = res;
  }
  if (det) blocks = 1;
  const dim3 g((unsigned)blocks), bl(256);
  if (K <= 256) {
    if (ldd < 256 || ldw < 256) return HARP_EBADARG;
    lda_cgs_kernel<4, DT, XW><<<g, bl, 0, s>>>(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, nwk, ldw, inv_nk,
                                           nk_delta, K, alpha, beta, seed, det, ps, lpt);
  } else if (K <= 512) {
    if (ldd < 512 || ldw < 512) return HARP_EBADARG;
    lda_cgs_kernel<8, DT, XW><<<g, bl, 0, s>>>(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, nwk, ldw, inv_nk,
                                           nk_delta, K, alpha, beta, seed, det, ps, lpt);
  } else {
    if (ldd < 1024 || ldw < 1024) return HARP_EBADARG;
    lda_cgs_kernel<16, DT, XW><<<g, bl, 0, s>>>(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, nwk, ldw, inv_nk,
                                            nk_delta, K, alpha, beta, seed, det, ps, lpt);
  }
  return harp_launch_status();
}
}  // namespace

// ndk_bits: 32 -> int32 doc-topic counts; 16 -> packed uint16 (ldd multiple of 8); 8 -> packed
// uint8 (every doc < 256 tokens; ldd multiple of 16)
// variant: 0 = compiler occupancy, 3 = two more waves per SIMD (fewer VGPRs, some spilled)
static int lda_cgs_impl(const int* tdoc, const int* tword, int* tz, const long* chunk_start, long nchunks, void* ndk,
                        int ldd, int ndk_bits, int* nwk, int ldw, const float* inv_nk, int* nk_delta, int K, float alpha,
                        float beta, unsigned long long seed, int variant, PsRows ps, const long* lpt, hipStream_t s);

HARP_EXPORT int harp_lda_cgs(const int* tdoc, const int* tword, int* tz, const long* chunk_start, long nchunks,
                             void* ndk, int ldd, int ndk_bits, int* nwk, int ldw, const float* inv_nk, int* nk_delta,
                             int K, float alpha, float beta, unsigned long long seed, int variant, const long* lpt,
                             hipStream_t s) {
  const PsRows none{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  return lda_cgs_impl(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, ndk_bits, nwk, ldw, inv_nk, nk_delta, K, alpha,
                      beta, seed, variant, none, lpt, s);
}

// The dense sampler on fused parameter-server rows (PsRows above): pull payload slots in,
// push payload slots out (zeroed by the caller); nwk / ldw are unused.
HARP_EXPORT int harp_lda_cgs_ps(const int* tdoc, const int* tword, int* tz, const long* chunk_start, long nchunks,
                                void* ndk, int ldd, int ndk_bits, const float* inv_nk, int* nk_delta, int K,
                                float alpha, float beta, unsigned long long seed, int variant,
                                const unsigned char* pbuf, const long* poff, const int* pcap, unsigned char* qbuf,
                                const long* qoff, const int* qcap, int* overflow, const long* lpt, hipStream_t s) {
  if (!pbuf || !poff || !pcap || !qbuf || !qoff || !qcap || !overflow) return HARP_EBADARG;
  const PsRows ps{pbuf, poff, pcap, qbuf, qoff, qcap, overflow};
  int kp = K <= 256 ? 256 : K <= 512 ? 512 : 1024;
  return lda_cgs_impl(tdoc, tword, tz, chunk_start, nchunks, ndk, ldd, ndk_bits, nullptr, kp, inv_nk, nk_delta, K,
                      alpha, beta, seed, variant, ps, lpt, s);
}

static int lda_cgs_impl(const int* tdoc, const int* tword, int* tz, const long* chunk_start, long nchunks, void* ndk,
                        int ldd, int ndk_bits, int* nwk, int ldw, const float* inv_nk, int* nk_delta, int K, float alpha,
                        float beta, unsigned long long seed, int variant, PsRows ps, const long* lpt, hipStream_t s) {
  if (nchunks <= 0) return HARP_OK;
  // variant 0: six waves per SIMD; 3: seven (the default). Round 1's variants (1: a
  // float-row prefetch; 2, 4, 5: other forced occupancies) measured slower
  // (profiles/r1_lda/occupancy) and are no longer built.
  // variant | 0x100: deterministic one-wave sampling in chunk order (tests); | 0x200: one
  // wave in the chunk-descriptor order of lpt (tests of the production schedule)
  const int det = (variant & 0x200) ? 2 : (variant & 0x100) ? 1 : 0;
  variant &= 0xff;
  if (K <= 0 || K > 1024 || ldw % 4 || (variant != 0 && variant != 3)) return HARP_EBADARG;
#define CGS_ARGS tdoc, tword, tz, chunk_start, nchunks
#define CGS_TAIL nwk, ldw, inv_nk, nk_delta, K, alpha, beta, seed, det, ps, lpt, s
  if (ndk_bits == 32) {
    if (ldd % 4) return HARP_EBADARG;
    return variant == 3 ? launch_cgs<int, 1>(CGS_ARGS, (int*)ndk, ldd, CGS_TAIL)
                        : launch_cgs<int, 0>(CGS_ARGS, (int*)ndk, ldd, CGS_TAIL);
  }
  if (ndk_bits == 16) {
    if (ldd % 8) return HARP_EBADARG;
    return variant == 3 ? launch_cgs<unsigned short, 1>(CGS_ARGS, (unsigned short*)ndk, ldd, CGS_TAIL)
                        : launch_cgs<unsigned short, 0>(CGS_ARGS, (unsigned short*)ndk, ldd, CGS_TAIL);
  }
  if (ndk_bits == 8) {
    if (ldd % 16) return HARP_EBADARG;
    return variant == 3 ? launch_cgs<unsigned char, 1>(CGS_ARGS, (unsigned char*)ndk, ldd, CGS_TAIL)
                        : launch_cgs<unsigned char, 0>(CGS_ARGS, (unsigned char*)ndk, ldd, CGS_TAIL);
  }
#undef CGS_ARGS
#undef CGS_TAIL
  return HARP_EBADARG;
}

namespace {
// LDS modes of the sparse sampler by padded topic count: K_pad <= 1024: workgroup topic
// deltas + per-wave word rows; <= 4096: workgroup topic deltas + one workgroup word row
// (chunk-end flush); larger: qw only (both deltas as global atomics -- a second 40 KB row
// would halve the resident workgroups at K = 10,000).
// K limit of the sparse sampler: the word's qw row (4 B per topic) lives in LDS, so 32768
// topics take 128 KB of the CU's 160 KB (one workgroup per CU); larger K runs the exact
// host sampler (ops/lda.py cgs_sample)
constexpr int kSparseMaxK = 32768;
int sparse_wdelta(int Kp) { return Kp <= 1024 ? 1 : Kp <= 4096 ? 2 : 0; }
size_t sparse_lds_bytes(int Kp, int waves) {
  const int wd = sparse_wdelta(Kp);
  // wd == 0: s_qw and the move lists (64 per wave)
  return (Kp <= 4096 ? 8 : 4) * (size_t)Kp +
         (wd == 1 ? 4 * (size_t)Kp * waves : wd == 2 ? 4 * (size_t)Kp : 4 * 64 * (size_t)waves);
}

template <int WAVES, class DT, bool SPAN = false>
int launch_sparse(const int* tdoc, const long* tspan, const int* tword, int* tz, const long* chunk_start, long nchunks,
                  const int* order,
                  int* work, const long* tpos,
                  const long* doc_off, unsigned short* zdoc, DT* ndk, int ldd, int* nwk, int ldw, const float* inv_nk,
                  int* nk_delta, int K, float alpha, float beta, unsigned long long seed, int det, hipStream_t s,
                  PsRows ps = PsRows{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr}) {
  const int Kp = (K + 63) / 64 * 64;
  const int ldelta = Kp <= 4096;  // LDS topic-sum deltas while they cost at most 16 KB
  const int wdelta = sparse_wdelta(Kp);
  const size_t lds = sparse_lds_bytes(Kp, WAVES);
  // raise the dynamic-LDS cap past 64 KB (per launch: no process-wide cache that a second
  // device or a concurrent caller could skip past)
  if (lds > 65536 && hipFuncSetAttribute((const void*)lda_cgs_sparse_kernel<WAVES, DT, SPAN>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return HARP_ELAUNCH;
  // grid = resident workgroups (LDS- or wave-slot-bound), striding over the chunks
  long per_cu = 163840 / (long)(lds + 1100);
  if (per_cu > 32 / WAVES) per_cu = 32 / WAVES;
  if (per_cu < 1) per_cu = 1;
  long blocks = nchunks;
  if (blocks > 256 * per_cu) blocks = 256 * per_cu;
  if (det) blocks = 1;
  lda_cgs_sparse_kernel<WAVES, DT, SPAN><<<dim3((unsigned)blocks), dim3(64 * WAVES), lds, s>>>(
      tdoc, tspan, tword, tz, chunk_start, nchunks, order, work, tpos, doc_off, zdoc, ndk, ldd, nwk, ldw, inv_nk, nk_delta, K, Kp, alpha,
      beta, seed, ldelta, wdelta, ps);
  return harp_launch_status();
}
}  // namespace

// Sparse-doc sampler (see lda_cgs_sparse_kernel): tpos[i] = doc-order position of token i
// in zdoc (uint16 topics, doc_off[d] .. doc_off[d + 1] = doc d); ndk may be null (no
// doc-topic counts kept); waves: workgroup size in waves (1, 2, 4, 8 or 16; 0 = by K); order: chunk
// processing order (null = 0..nchunks-1); work: ONE int, zero on entry (chunk counter).
HARP_EXPORT int harp_lda_cgs_sparse(const int* tdoc, const int* tword, int* tz, const long* chunk_start, long nchunks,
                                    const int* order, int* work, const long* tpos, const long* doc_off, unsigned short* zdoc, void* ndk, int ldd,
                                    int ndk_bits, int* nwk, int ldw, const float* inv_nk, int* nk_delta, int K,
                                    float alpha, float beta, unsigned long long seed, int waves, hipStream_t s) {
  if (nchunks <= 0) return HARP_OK;
  if (K <= 0 || K > kSparseMaxK || ldw < K || (ndk && ldd < K) || !tpos || !doc_off || !zdoc || !work) return HARP_EBADARG;
  const int det = waves < 0 ? 1 : 0;  // waves < 0: one one-wave workgroup, bit-reproducible (tests)
  if (det) waves = 1;
  if (waves == 0) {  // auto: the smallest workgroup that still puts >= 24 waves on a CU
    const int Kp = (K + 63) / 64 * 64;
    waves = 16;
    for (int w = 4; w <= 8; w *= 2) {
      const long per_cu = 163840 / ((long)sparse_lds_bytes(Kp, w) + 1100);  // LDS-resident workgroups
      if (per_cu * w >= 24) {
        waves = w;
        break;
      }
    }
  }
#define SP_ARGS tdoc, nullptr, tword, tz, chunk_start, nchunks, order, work, tpos, doc_off, zdoc
#define SP_TAIL nwk, ldw, inv_nk, nk_delta, K, alpha, beta, seed, det, s
  if (ndk_bits == 16) {
    if (ldd % 2) return HARP_EBADARG;
    unsigned short* n16 = (unsigned short*)ndk;
    return waves == 1    ? launch_sparse<1>(SP_ARGS, n16, ldd, SP_TAIL)
           : waves == 2  ? launch_sparse<2>(SP_ARGS, n16, ldd, SP_TAIL)
           : waves == 4  ? launch_sparse<4>(SP_ARGS, n16, ldd, SP_TAIL)
           : waves == 16 ? launch_sparse<16>(SP_ARGS, n16, ldd, SP_TAIL)
                         : launch_sparse<8>(SP_ARGS, n16, ldd, SP_TAIL);
  }
  if (ndk_bits == 8) {
    if (ldd % 4) return HARP_EBADARG;
    unsigned char* n8 = (unsigned char*)ndk;
    return waves == 1    ? launch_sparse<1>(SP_ARGS, n8, ldd, SP_TAIL)
           : waves == 2  ? launch_sparse<2>(SP_ARGS, n8, ldd, SP_TAIL)
           : waves == 4  ? launch_sparse<4>(SP_ARGS, n8, ldd, SP_TAIL)
           : waves == 16 ? launch_sparse<16>(SP_ARGS, n8, ldd, SP_TAIL)
                         : launch_sparse<8>(SP_ARGS, n8, ldd, SP_TAIL);
  }
  if (ndk_bits != 32) return HARP_EBADARG;
  int* n32 = (int*)ndk;
  return waves == 1    ? launch_sparse<1>(SP_ARGS, n32, ldd, SP_TAIL)
         : waves == 2  ? launch_sparse<2>(SP_ARGS, n32, ldd, SP_TAIL)
         : waves == 4  ? launch_sparse<4>(SP_ARGS, n32, ldd, SP_TAIL)
         : waves == 16 ? launch_sparse<16>(SP_ARGS, n32, ldd, SP_TAIL)
                       : launch_sparse<8>(SP_ARGS, n32, ldd, SP_TAIL);
#undef SP_ARGS
#undef SP_TAIL
}

// The same sampler with per-token doc spans (tspan[i] = doc_off[d_i] | (len_i << 40)) in place
// of doc ids, and no doc-topic table: the next token's doc range is one independent load.
HARP_EXPORT int harp_lda_cgs_sparse_span(const long* tspan, const int* tword, int* tz, const long* chunk_start,
                                         long nchunks, const int* order, int* work, const long* tpos,
                                         unsigned short* zdoc, int* nwk, int ldw, const float* inv_nk, int* nk_delta,
                                         int K, float alpha, float beta, unsigned long long seed, int waves,
                                         hipStream_t s) {
  if (nchunks <= 0) return HARP_OK;
  if (K <= 0 || K > kSparseMaxK || ldw < K || !tspan || !tpos || !zdoc || !work) return HARP_EBADARG;
  const int det = waves < 0 ? 1 : 0;
  if (det) waves = 1;
  if (waves == 0) {
    const int Kp = (K + 63) / 64 * 64;
    waves = 16;
    for (int w = 4; w <= 8; w *= 2) {
      const long per_cu = 163840 / ((long)sparse_lds_bytes(Kp, w) + 1100);
      if (per_cu * w >= 24) {
        waves = w;
        break;
      }
    }
  }
#define SS_ARGS nullptr, tspan, tword, tz, chunk_start, nchunks, order, work, tpos, nullptr, zdoc, (int*)nullptr, 0
#define SS_TAIL nwk, ldw, inv_nk, nk_delta, K, alpha, beta, seed, det, s
  return waves == 1    ? launch_sparse<1, int, true>(SS_ARGS, SS_TAIL)
         : waves == 2  ? launch_sparse<2, int, true>(SS_ARGS, SS_TAIL)
         : waves == 4  ? launch_sparse<4, int, true>(SS_ARGS, SS_TAIL)
         : waves == 16 ? launch_sparse<16, int, true>(SS_ARGS, SS_TAIL)
                       : launch_sparse<8, int, true>(SS_ARGS, SS_TAIL);
#undef SS_ARGS
#undef SS_TAIL
}

// harp_lda_cgs_sparse_span with fused parameter-server rows: word rows come from the pull
// payload slots (pbuf / poff / pcap, one per local row) and the sweep's word-row moves are
// written into the zeroed push payload (qbuf / qoff / qcap); no dense word table. Slot
// formats: parallel/sparse_ps.py, csrc/rowcodec.hip (K_pad ints per dense slot).
HARP_EXPORT int harp_lda_cgs_sparse_span_ps(const long* tspan, const int* tword, int* tz, const long* chunk_start,
                                            long nchunks, const int* order, int* work, const long* tpos,
                                            unsigned short* zdoc, const float* inv_nk, int* nk_delta, int K,
                                            float alpha, float beta, unsigned long long seed, int waves,
                                            const unsigned char* pbuf, const long* poff, const int* pcap,
                                            unsigned char* qbuf, const long* qoff, const int* qcap, int* overflow,
                                            hipStream_t s) {
  if (nchunks <= 0) return HARP_OK;
  if (K <= 0 || K > kSparseMaxK || !tspan || !tpos || !zdoc || !work) return HARP_EBADARG;
  if (!pbuf || !poff || !pcap || !qbuf || !qoff || !qcap || !overflow) return HARP_EBADARG;
  const PsRows ps{pbuf, poff, pcap, qbuf, qoff, qcap, overflow};
  const int det = waves < 0 ? 1 : 0;
  if (det) waves = 1;
  if (waves == 0) {
    const int Kp = (K + 63) / 64 * 64;
    waves = 16;
    for (int w = 4; w <= 8; w *= 2) {
      const long per_cu = 163840 / ((long)sparse_lds_bytes(Kp, w) + 1100);
      if (per_cu * w >= 24) {
        waves = w;
        break;
      }
    }
  }
#define SS_ARGS nullptr, tspan, tword, tz, chunk_start, nchunks, order, work, tpos, nullptr, zdoc, (int*)nullptr, 0
#define SS_TAIL nullptr, 0, inv_nk, nk_delta, K, alpha, beta, seed, det, s, ps
  return waves == 1    ? launch_sparse<1, int, true>(SS_ARGS, SS_TAIL)
         : waves == 2  ? launch_sparse<2, int, true>(SS_ARGS, SS_TAIL)
         : waves == 4  ? launch_sparse<4, int, true>(SS_ARGS, SS_TAIL)
         : waves == 16 ? launch_sparse<16, int, true>(SS_ARGS, SS_TAIL)
                       : launch_sparse<8, int, true>(SS_ARGS, SS_TAIL);
#undef SS_ARGS
#undef SS_TAIL
}

HARP_EXPORT int harp_lda_count(const int* tdoc, const int* tword, const int* tz, long n, void* ndk, int ldd,
                               int ndk_bits, int* nwk, int ldw, int* nk, hipStream_t s) {
  if (n <= 0) return HARP_OK;
  long blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (ndk_bits == 16) {
    if (ldd % 2) return HARP_EBADARG;
    lda_count_kernel<unsigned short><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(tdoc, tword, tz, n,
                                                                                  (unsigned short*)ndk, ldd, nwk, ldw,
                                                                                  nk);
  } else if (ndk_bits == 8) {
    if (ldd % 4) return HARP_EBADARG;
    lda_count_kernel<unsigned char><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(tdoc, tword, tz, n,
                                                                                 (unsigned char*)ndk, ldd, nwk, ldw, nk);
  } else {
    lda_count_kernel<int><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(tdoc, tword, tz, n, (int*)ndk, ldd, nwk, ldw,
                                                                       nk);
  }
  return harp_launch_status();
}

#ifdef HARP_LDA_STAMPS
HARP_EXPORT int harp_lda_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lda_stamps), sizeof(unsigned long long) * 8) != hipSuccess) return HARP_EBADARG;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lda_stamps), z, sizeof(z)) != hipSuccess) return HARP_EBADARG;
  }
  return HARP_OK;
}
#endif
