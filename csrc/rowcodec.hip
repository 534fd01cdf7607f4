// Sparse row codec for parameter-server push / pull of count tables (gfx950).
//
// The LDA word-topic model lives in a distributed global table (owner = word block mod P);
// every iteration a worker pulls the rows of the words its tokens touch and pushes the
// rows' count deltas back (reference: contrib/.../lda/LDAMapperDyn.java push :380 / pull
// :429 with sparse TopicCountList rows, ml/java/.../lda/LDAUtil.java:159-213). Word-topic
// rows are mostly zero, so over point-to-point xGMI the dense rows are link-bound.
//
// Payload of one peer = a sequence of per-row SLOTS at static byte offsets. A slot's
// capacity comes from token totals that never change during sampling (pull: min(K, global
// tokens of the word); push delta: min(K, 2 x local tokens)), so both ends derive the same
// layout once and every call is a fixed-size all-to-all with no size exchange and no host
// sync. A slot is
//   sparse (cap >= 0): [int32 nnz][int32 counts cap][uint16 topics cap]   (4 + 6 cap bytes, 4-aligned)
//   dense  (cap <  0): [int32 row K]                      (16-aligned; when 4 + 6 cap >= 4 K)
//
// One wave per row (up to 4 per workgroup, fewer for K > 4096 so the LDS rows stay
// within 64 KB; K <= 16384), the row staged once in LDS (4 KB at K = 1024):
//   encode        : global row -> lanes (16 consecutive topics each) -> one wave scan
//                   places the nonzeros into the slot in column order              (1 read)
//   encode_delta  : LDS = row - "before" (the row's slot of the PULL payload it was
//                   decoded from: the pull payload doubles as the snapshot)         (1 read)
//   decode_replace: LDS = 0, scatter slot entries, LDS -> row                      (1 write)
//   decode_add    : atomic adds of the slot entries into the row (several peers may
//                   push into one owner row within one launch)
// Received payloads are bounds-checked (nnz clamped to the slot, topics < K).
#include "common.h"

namespace {

constexpr int kMaxWaves = 4;               // rows per workgroup (at most)
constexpr int kLdsBudget = 64 * 1024;      // default dynamic-LDS limit per workgroup

__device__ __forceinline__ const int* slot_counts(const unsigned char* slot) { return (const int*)(slot + 4); }
__device__ __forceinline__ const unsigned short* slot_topics(const unsigned char* slot, int cap) {
  return (const unsigned short*)(slot + 4 + 4 * (long)cap);
}

// stage one row (K ints, 16-B aligned rows: K % 4 == 0, ld % 4 == 0) into this wave's LDS row
__device__ __forceinline__ void load_row(int* lrow, const int* __restrict__ g, int K, int lane) {
  const int4* g4 = (const int4*)g;
  int4* l4 = (int4*)lrow;
  for (int c = lane; c < K / 4; c += 64) l4[c] = g4[c];
}

// subtract a slot (dense or sparse) from the LDS row
__device__ __forceinline__ void sub_slot(int* lrow, const unsigned char* slot, int cap, int K, int lane) {
  if (cap < 0) {
    const int4* s4 = (const int4*)slot;
    int4* l4 = (int4*)lrow;
    for (int c = lane; c < K / 4; c += 64) {
      int4 a = l4[c];
      const int4 b = s4[c];
      a.x -= b.x; a.y -= b.y; a.z -= b.z; a.w -= b.w;
      l4[c] = a;
    }
    return;
  }
  int nnz = *(const int*)slot;
  nnz = nnz < 0 ? 0 : (nnz > cap ? cap : nnz);
  const int* cnt = slot_counts(slot);
  const unsigned short* top = slot_topics(slot, cap);
  for (int e = lane; e < nnz; e += 64) {  // topics are distinct within a slot: no LDS races
    const int t = top[e];
    if (t < K) lrow[t] -= cnt[e];
  }
}

// LDS row -> slot (dense copy, or ballot compaction in column order)
__device__ __forceinline__ void store_slot(const int* lrow, unsigned char* slot, int cap, int K, int lane,
                                           int* overflow) {
  if (cap < 0) {
    const int4* l4 = (const int4*)lrow;
    int4* s4 = (int4*)slot;
    for (int c = lane; c < K / 4; c += 64) s4[c] = l4[c];
    return;
  }
  int* cnt = (int*)(slot + 4);
  unsigned short* top = (unsigned short*)(slot + 4 + 4 * (long)cap);
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  int base = 0;
  bool over = false;
  for (int j0 = 0; j0 < K; j0 += 64) {
    const int j = j0 + lane;
    const int v = j < K ? lrow[j] : 0;
    const unsigned long long m = __ballot(v != 0);
    if (v != 0) {
      const int pos = base + __popcll(m & below);
      if (pos < cap) {
        cnt[pos] = v;
        top[pos] = (unsigned short)j;
      } else {
        over = true;
      }
    }
    base += __popcll(m);
  }
  if (lane == 0) *(int*)slot = base < cap ? base : cap;
  if (__ballot(over) && lane == 0) overflow[0] = 1;
}

// 16 consecutive counts of a row (t0 % 16 == 0; zero past K, K % 4 == 0)
__device__ __forceinline__ void load16(const int* __restrict__ g, int t0, int K, int (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int t = t0 + 4 * q;
    const int4 x = t < K ? *(const int4*)(g + t) : make_int4(0, 0, 0, 0);
    v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
  }
}
__device__ __forceinline__ void load16(const unsigned short* __restrict__ g, int t0, int K, int (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {  // K % 8 == 0 for narrow rows
    const int t = t0 + 8 * q;
    const uint4 x = t < K ? *(const uint4*)(g + t) : make_uint4(0u, 0u, 0u, 0u);
    const unsigned w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[8 * q + 2 * k] = (int)(w4[k] & 0xFFFFu);
      v[8 * q + 2 * k + 1] = (int)(w4[k] >> 16);
    }
  }
}

// Plain encode (no delta) without LDS staging: lane L takes topics [16 L, 16 L + 16) of each
// 1024-topic stretch straight from the row, one wave scan of the lanes' nonzero counts
// places them, so the slot is written in column order as before (the staged form made 16
// ballot passes over an LDS copy of the row: the pull encode of the LDA push-pull).
template <class ST>
__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_encode_direct_kernel(
    const ST* __restrict__ src, long ld, int K, const int* __restrict__ rows, int n,
    const long* __restrict__ slot_off, const int* __restrict__ cap, unsigned char* __restrict__ out,
    int* __restrict__ overflow) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * (blockDim.x >> 6) + w;
  if (j >= n) return;  // the whole wave
  const ST* g = src + (long)rows[j] * ld;
  unsigned char* slot = out + slot_off[j];
  const int c = cap[j];
  if (c < 0) {  // dense slot: the row as int32
    int4* s4 = (int4*)slot;
    for (int t0 = 16 * lane; t0 < K; t0 += 1024) {
      int v[16];
      load16(g, t0, K, v);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (t0 + 4 * q < K) s4[(t0 >> 2) + q] = make_int4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
    return;
  }
  int* cnt = (int*)(slot + 4);
  unsigned short* top = (unsigned short*)(slot + 4 + 4 * (long)c);
  int base = 0;
  bool over = false;
  for (int s0 = 0; s0 < K; s0 += 1024) {
    const int t0 = s0 + 16 * lane;
    int v[16];
    load16(g, t0, K, v);
    int mine = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) mine += v[e] != 0 ? 1 : 0;
    const float incl = wave_scan_incl((float)mine);  // <= 1024: exact
    int pos = base + (int)incl - mine;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (v[e] != 0) {
        if (pos < c) {
          cnt[pos] = v[e];
          top[pos] = (unsigned short)(t0 + e);
        } else {
          over = true;
        }
        ++pos;
      }
    }
    base += (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
  }
  if (lane == 0) *(int*)slot = base < c ? base : c;
  if (__ballot(over) && lane == 0) overflow[0] = 1;
}

template <bool kDelta>
__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_encode_kernel(
    const int* __restrict__ src, long ld, int K, const int* __restrict__ rows, int n,
    const long* __restrict__ slot_off, const int* __restrict__ cap, unsigned char* __restrict__ out,
    const unsigned char* __restrict__ before, const long* __restrict__ b_off, const int* __restrict__ b_cap,
    int* __restrict__ overflow) {
  extern __shared__ int lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * (blockDim.x >> 6) + w;
  int* lrow = lds + w * K;
  const bool live = j < n;
  if (live) load_row(lrow, src + (long)rows[j] * ld, K, lane);
  __syncthreads();
  if (kDelta) {
    if (live) sub_slot(lrow, before + b_off[j], b_cap[j], K, lane);
    __syncthreads();
  }
  if (live) store_slot(lrow, out + slot_off[j], cap[j], K, lane, overflow);
}

__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_decode_replace_kernel(
    int* __restrict__ dst, long ld, int K, const int* __restrict__ rows, int n, const long* __restrict__ slot_off,
    const int* __restrict__ cap, const unsigned char* __restrict__ in) {
  extern __shared__ int lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * (blockDim.x >> 6) + w;
  int* lrow = lds + w * K;
  const bool live = j < n;
  const int c = live ? cap[j] : -1;
  const unsigned char* slot = live ? in + slot_off[j] : nullptr;
  if (live && c >= 0) {
    int4* l4 = (int4*)lrow;
    for (int q = lane; q < K / 4; q += 64) l4[q] = make_int4(0, 0, 0, 0);
  }
  __syncthreads();
  if (live && c >= 0) {
    int nnz = *(const int*)slot;
    nnz = nnz < 0 ? 0 : (nnz > c ? c : nnz);
    const int* cnt = slot_counts(slot);
    const unsigned short* top = slot_topics(slot, c);
    for (int e = lane; e < nnz; e += 64) {
      const int t = top[e];
      if (t < K) lrow[t] = cnt[e];
    }
  }
  __syncthreads();
  if (!live) return;
  const int4* s4 = c < 0 ? (const int4*)slot : (const int4*)lrow;
  int4* d4 = (int4*)(dst + (long)rows[j] * ld);
  for (int q = lane; q < K / 4; q += 64) d4[q] = s4[q];
}

__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_decode_add_kernel(
    int* __restrict__ dst, long ld, int K, const int* __restrict__ rows, int n, const long* __restrict__ slot_off,
    const int* __restrict__ cap, const unsigned char* __restrict__ in) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * (blockDim.x >> 6) + w;
  if (j >= n) return;
  int* d = dst + (long)rows[j] * ld;
  const int c = cap[j];
  const unsigned char* slot = in + slot_off[j];
  if (c < 0) {
    const int* s = (const int*)slot;
    for (int t = lane; t < K; t += 64) {
      const int v = s[t];
      if (v) atomicAdd(d + t, v);
    }
    return;
  }
  int nnz = *(const int*)slot;
  nnz = nnz < 0 ? 0 : (nnz > c ? c : nnz);
  const int* cnt = slot_counts(slot);
  const unsigned short* top = slot_topics(slot, c);
  for (int e = lane; e < nnz; e += 64) {
    const int t = top[e];
    if (t < K) atomicAdd(d + t, cnt[e]);
  }
}

// add a slot into a narrow (uint16) row: one 32-bit atomic on the dword holding the count,
// +v or -(-v) in its half. Counts stay in [0, 65535] (every count is at most its word's
// token total, < 65536 for a narrow table, and a requester's decrements never exceed its
// own tokens counted in the row), so neither half ever carries or borrows into the other.
__device__ __forceinline__ void add16(unsigned short* row, int t, int v) {
  unsigned* word = (unsigned*)(row + (t & ~1));
  const unsigned sh = (t & 1) ? 16u : 0u;
  if (v > 0) atomicAdd(word, (unsigned)v << sh);
  else atomicSub(word, (unsigned)(-v) << sh);
}

__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_decode_add16_kernel(
    unsigned short* __restrict__ dst, long ld, int K, const int* __restrict__ rows, int n,
    const long* __restrict__ slot_off, const int* __restrict__ cap, const unsigned char* __restrict__ in) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * (blockDim.x >> 6) + w;
  if (j >= n) return;
  unsigned short* d = dst + (long)rows[j] * ld;
  const int c = cap[j];
  const unsigned char* slot = in + slot_off[j];
  if (c < 0) {
    const int* s = (const int*)slot;
    for (int t = lane; t < K; t += 64) {
      const int v = s[t];
      if (v) add16(d, t, v);
    }
    return;
  }
  int nnz = *(const int*)slot;
  nnz = nnz < 0 ? 0 : (nnz > c ? c : nnz);
  const int* cnt = slot_counts(slot);
  const unsigned short* top = slot_topics(slot, c);
  for (int e = lane; e < nnz; e += 64) {
    const int t = top[e], v = cnt[e];
    if (v && t < K) add16(d, t, v);
  }
}

// slot j of `out` := slot src_off[j] of `in` (same capacity): the owner's pull sends every
// requester of a row the same slot, so the row is encoded once and its slot copied -- only
// the header and the used entries of a sparse slot
__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_copy_slots_kernel(
    const unsigned char* __restrict__ in, const long* __restrict__ src_off, unsigned char* __restrict__ out,
    const long* __restrict__ dst_off, const int* __restrict__ cap, int n, int K) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blockIdx.x * (blockDim.x >> 6) + w;
  if (j >= n) return;
  const unsigned char* a = in + src_off[j];
  unsigned char* d = out + dst_off[j];
  const int c = cap[j];
  if (c < 0) {
    const int4* a4 = (const int4*)a;
    int4* d4 = (int4*)d;
    for (int q = lane; q < K / 4; q += 64) d4[q] = a4[q];
    return;
  }
  int nnz = *(const int*)a;
  nnz = nnz < 0 ? 0 : (nnz > c ? c : nnz);
  if (lane == 0) *(int*)d = nnz;
  const int* ac = slot_counts(a);
  int* dc = (int*)(d + 4);
  const unsigned short* at = slot_topics(a, c);
  unsigned short* dt = (unsigned short*)(d + 4 + 4 * (long)c);
  for (int e = lane; e < nnz; e += 64) {
    dc[e] = ac[e];
    dt[e] = at[e];
  }
}

inline bool bad_shape(long ld, int K) { return K <= 0 || (K & 3) || ld < K || (ld & 3) || 4L * K > kLdsBudget; }
// waves (rows) per workgroup so that the LDS rows fit the default dynamic-LDS limit
inline int waves_for(int K) {
  const int w = kLdsBudget / (4 * K);
  return w < 1 ? 1 : (w > kMaxWaves ? kMaxWaves : w);
}
inline bool misaligned(const void* p) { return ((uintptr_t)p) & 15; }

}  // namespace

// src rows[j] (K ints at stride ld) -> slot j of `out`; with `before` (the pull payload the
// rows were decoded from, slots b_off / b_cap) the slot holds row - before (a count delta)
HARP_EXPORT int harp_rowcodec_encode(const int* src, long ld, int K, const int* rows, int n, const long* slot_off,
                                     const int* cap, void* out, const void* before, const long* b_off,
                                     const int* b_cap, int* overflow, hipStream_t s) {
  if (n < 0 || bad_shape(ld, K) || misaligned(src) || misaligned(out) || (before && misaligned(before)) || !overflow)
    return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  const int wv = waves_for(K);
  const size_t lds = sizeof(int) * (size_t)K * wv;
  const dim3 grid((n + wv - 1) / wv), block(wv * 64);
  if (before) {
    rowcodec_encode_kernel<true><<<grid, block, lds, s>>>(src, ld, K, rows, n, slot_off, cap,
                                                                  (unsigned char*)out, (const unsigned char*)before,
                                                                  b_off, b_cap, overflow);
  } else {
    rowcodec_encode_direct_kernel<int><<<dim3((n + kMaxWaves - 1) / kMaxWaves), dim3(kMaxWaves * 64), 0, s>>>(
        src, ld, K, rows, n, slot_off, cap, (unsigned char*)out, overflow);
  }
  return harp_launch_status();
}

// slot j of `in` -> dst rows[j]: mode 0 replaces the row, mode 1 adds into it (atomics)
HARP_EXPORT int harp_rowcodec_decode(int* dst, long ld, int K, const int* rows, int n, const long* slot_off,
                                     const int* cap, const void* in, int mode, hipStream_t s) {
  if (n < 0 || bad_shape(ld, K) || misaligned(dst) || misaligned(in) || (mode != 0 && mode != 1)) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  const int wv = waves_for(K);
  const dim3 grid((n + wv - 1) / wv), block(wv * 64);
  if (mode == 0) {
    rowcodec_decode_replace_kernel<<<grid, block, sizeof(int) * (size_t)K * wv, s>>>(dst, ld, K, rows, n, slot_off, cap,
                                                                     (const unsigned char*)in);
  } else {
    rowcodec_decode_add_kernel<<<grid, block, 0, s>>>(dst, ld, K, rows, n, slot_off, cap, (const unsigned char*)in);
  }
  return harp_launch_status();
}

// narrow (uint16) global tables: encode from, and add slots into, rows of K uint16 counts
// at stride ld (K % 8 == 0, ld % 8 == 0)
HARP_EXPORT int harp_rowcodec_encode16(const unsigned short* src, long ld, int K, const int* rows, int n,
                                       const long* slot_off, const int* cap, void* out, int* overflow, hipStream_t s) {
  if (n < 0 || bad_shape(ld, K) || (K & 7) || (ld & 7) || misaligned(src) || misaligned(out) || !overflow)
    return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  rowcodec_encode_direct_kernel<unsigned short><<<dim3((n + kMaxWaves - 1) / kMaxWaves), dim3(kMaxWaves * 64), 0, s>>>(
      src, ld, K, rows, n, slot_off, cap, (unsigned char*)out, overflow);
  return harp_launch_status();
}

HARP_EXPORT int harp_rowcodec_decode_add16(unsigned short* dst, long ld, int K, const int* rows, int n,
                                           const long* slot_off, const int* cap, const void* in, hipStream_t s) {
  if (n < 0 || bad_shape(ld, K) || (K & 7) || (ld & 7) || misaligned(dst) || misaligned(in)) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  const int wv = waves_for(K);
  const dim3 grid((n + wv - 1) / wv), block(wv * 64);
  rowcodec_decode_add16_kernel<<<grid, block, 0, s>>>(dst, ld, K, rows, n, slot_off, cap, (const unsigned char*)in);
  return harp_launch_status();
}

HARP_EXPORT int harp_rowcodec_copy_slots(const void* in, const long* src_off, void* out, const long* dst_off,
                                         const int* cap, int n, int K, hipStream_t s) {
  if (n < 0 || K <= 0 || (K & 3) || misaligned(in) || misaligned(out)) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  rowcodec_copy_slots_kernel<<<dim3((n + kMaxWaves - 1) / kMaxWaves), dim3(kMaxWaves * 64), 0, s>>>(
      (const unsigned char*)in, src_off, (unsigned char*)out, dst_off, cap, n, K);
  return harp_launch_status();
}
