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
//   merge         : owner table held as slots itself: canonical slot += pushed delta slots,
//                   re-encoded in place (no dense table, no encode pass for the pull)
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

// Owner-side merge for a table held in slot form (sparse owner table): canonical slot u :=
// slot u + every delta slot pushed for its row (src_idx[src_ptr[u] .. src_ptr[u + 1])),
// written back in place without zero counts (the form the samplers and copy_slots read;
// topic order within a slot is free). One wave per row, grid-stride over a row list. Rows
// come in two classes the host fixes once from the slot capacities (static bounds):
//  * rows with at most 64 / 256 / 512 entries (old + pushed; a word's handful of tokens is the
//    common case at an 8-rank share): 16 / 32 / 64 lanes and a 128 / 512 / 1024-entry
//    open-addressing LDS hash per row, four / two / one rows per wave, so a wave overlaps
//    several rows' chains of dependent slot loads;
//  * big rows: a K-int LDS accumulator plus a K-bit bitmap of the touched topics, re-zeroed
//    only where touched (ascending output).
// Dense canonical rows (cap < 0) take the deltas as atomic adds. overflow |= 1: a row
// exceeded its capacity; |= 2: a count went negative.
// row classes by entry bound: (G lanes, S hash entries) per row
constexpr int kTinyBound = 64, kSmallBound = 256, kHashBound = 512;  // (16, 128), (32, 512), (64, 1024)

// every (topic, value) of the canonical slot (sparse) and of the row's delta slots
template <class F>
__device__ __forceinline__ void merge_entries(const unsigned char* slot, int c, int q0, int q1,
                                              const int* __restrict__ src_idx, const unsigned char* __restrict__ in,
                                              const long* __restrict__ in_off, const int* __restrict__ in_cap, int K,
                                              int lane, F&& f, int stride = 64) {
  if (c >= 0) {
    int nnz = *(const int*)slot;
    nnz = nnz < 0 ? 0 : (nnz > c ? c : nnz);
    const int* ocn = slot_counts(slot);
    const unsigned short* otp = slot_topics(slot, c);
    for (int e = lane; e < nnz; e += stride) {
      const int t = otp[e];
      if (t < K) f(t, ocn[e]);
    }
  }
  for (int q = q0; q < q1; ++q) {
    const int si = src_idx[q];
    const unsigned char* ds = in + in_off[si];
    const int dc = in_cap[si];
    if (dc < 0) {
      for (int t = lane; t < K; t += stride) {
        const int v = ((const int*)ds)[t];
        if (v) f(t, v);
      }
    } else {
      int nz = *(const int*)ds;
      nz = nz < 0 ? 0 : (nz > dc ? dc : nz);
      const int* dcn = slot_counts(ds);
      const unsigned short* dtp = slot_topics(ds, dc);
      for (int e = lane; e < nz; e += stride) {
        const int t = dtp[e], v = dcn[e];
        if (v && t < K) f(t, v);
      }
    }
  }
}

__device__ __forceinline__ void hash_add(int* hk, int* hv, int slots, int t, int v, bool& over) {
  unsigned h = ((unsigned)t * 2654435761u) >> 16;
  for (int probe = 0;; ++probe) {
    h &= (unsigned)(slots - 1);
    if (probe == slots) {  // table full: the host's row bound was wrong (never loops)
      over = true;
      return;
    }
    const int k = atomicCAS(&hk[h], -1, t);
    if (k == -1 || k == t) {
      atomicAdd(&hv[h], v);
      return;
    }
    ++h;
  }
}

// G lanes per row (256 / G rows per workgroup), an S-entry LDS hash per row (S >= 2 x the
// class bound); the G-lane groups of one wave run different rows, so the wave overlaps
// their dependent slot loads
// Per-row merge metadata, built once on the host from the static layouts (32 B per row):
// canonical slot offset, first delta slot offset, capacities, and the row's range of delta
// slots (the first one is inlined; more, at P > 1, come from qoff / qcap in CSR order). A row's
// loads are then independent of each other, so the next row's are issued under this one.
struct MergeMeta {
  long off, doff;
  int cap, dcap, q0, q1;
};

// G lanes per row (256 / G rows per workgroup), an S-entry LDS hash per row (S >= 2 x the
// class bound); the G-lane groups of one wave run different rows, so the wave overlaps
// their slot loads, and each group loads the next row's metadata under the current row
template <int G, int S>
__global__ __launch_bounds__(256) void rowcodec_merge_group_kernel(
    unsigned char* __restrict__ canon, const MergeMeta* __restrict__ meta, int nrows,
    const long* __restrict__ qoff, const int* __restrict__ qcap, const unsigned char* __restrict__ in, int K,
    int* __restrict__ overflow) {
  constexpr int R = 256 / G;
  __shared__ int keys[R][S];
  __shared__ int vals[R][S];
  const int grp = threadIdx.x / G, gl = threadIdx.x % G, gshift = (threadIdx.x & 63) / G * G;
  int* hk = keys[grp];
  int* hv = vals[grp];
  for (int i = gl; i < S; i += G) {
    hk[i] = -1;
    hv[i] = 0;
  }
  bool over = false, neg = false;
  const unsigned long long gmask = G == 64 ? ~0ull : ((1ull << G) - 1ull);
  auto add = [&](int t, int v) { hash_add(hk, hv, S, t, v, over); };
  // one delta slot's entries (sparse or dense)
  auto delta = [&](const unsigned char* ds, int dc) {
    if (dc < 0) {
      for (int t = gl; t < K; t += G) {
        const int v = ((const int*)ds)[t];
        if (v) add(t, v);
      }
    } else {
      int nz = *(const int*)ds;
      nz = nz < 0 ? 0 : (nz > dc ? dc : nz);
      const int* dcn = slot_counts(ds);
      const unsigned short* dtp = slot_topics(ds, dc);
      for (int e = gl; e < nz; e += G) {
        const int t = dtp[e], v = dcn[e];
        if (v && t < K) add(t, v);
      }
    }
  };
  const int stride = gridDim.x * R;
  int j = blockIdx.x * R + grp;
  MergeMeta m{0, 0, 0, 0, 0, 0};
  if (j < nrows) m = meta[j];
  for (; j < nrows; j += stride) {
    MergeMeta mn{0, 0, 0, 0, 0, 0};
    if (j + stride < nrows) mn = meta[j + stride];  // in flight during this row
    unsigned char* slot = canon + m.off;
    const int c = m.cap;  // >= 0: these classes are sparse rows
    int nnz = *(const int*)slot;
    nnz = nnz < 0 ? 0 : (nnz > c ? c : nnz);
    int* ocn = (int*)(slot + 4);
    unsigned short* otp = (unsigned short*)(slot + 4 + 4 * (long)c);
    for (int e = gl; e < nnz; e += G) {
      const int t = otp[e];
      if (t < K) add(t, ocn[e]);
    }
    if (m.q1 > m.q0) delta(in + m.doff, m.dcap);
    for (int q = m.q0 + 1; q < m.q1; ++q) delta(in + qoff[q], qcap[q]);
    const unsigned long long below = (1ull << gl) - 1ull;
    int base = 0;
    for (int i0 = 0; i0 < S; i0 += G) {
      const int i = i0 + gl;
      const int t = hk[i], v = hv[i];
      const bool keep = t >= 0 && v != 0;
      neg |= v < 0;
      const unsigned long long mk = (__ballot(keep) >> gshift) & gmask;  // this row's G lanes
      if (keep) {
        const int pos = base + __popcll(mk & below);
        if (pos < c) {
          ocn[pos] = v;
          otp[pos] = (unsigned short)t;
        } else {
          over = true;
        }
      }
      base += __popcll(mk);
      hk[i] = -1;
      hv[i] = 0;
    }
    if (gl == 0) *(int*)slot = base < c ? base : c;
    m = mn;
  }
  if (over) atomicOr(overflow, 1);
  if (neg) atomicOr(overflow, 2);
}

__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_merge_kernel(
    unsigned char* __restrict__ canon, const long* __restrict__ c_off, const int* __restrict__ c_cap,
    const int* __restrict__ rows, int nrows, const int* __restrict__ src_ptr, const int* __restrict__ src_idx,
    const unsigned char* __restrict__ in, const long* __restrict__ in_off, const int* __restrict__ in_cap, int K,
    int per_wave, int* __restrict__ overflow) {
  extern __shared__ int lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, W = blockDim.x >> 6;
  int* acc = lds + w * per_wave;
  const int nbw = (K + 31) >> 5;
  unsigned* bits = (unsigned*)(acc + K);
  for (int i = lane; i < K + nbw; i += 64) acc[i] = 0;
  bool over = false, neg = false;
  for (int j = blockIdx.x * W + w; j < nrows; j += gridDim.x * W) {
    const int u = rows[j];
    unsigned char* slot = canon + c_off[u];
    const int c = c_cap[u];
    const int q0 = src_ptr[u], q1 = src_ptr[u + 1];
    if (c < 0) {  // dense canonical row
      int* row = (int*)slot;
      merge_entries(slot, c, q0, q1, src_idx, in, in_off, in_cap, K, lane, [&](int t, int v) { atomicAdd(row + t, v); });
      continue;
    }
    merge_entries(slot, c, q0, q1, src_idx, in, in_off, in_cap, K, lane, [&](int t, int v) {
      atomicAdd(&acc[t], v);
      atomicOr(&bits[t >> 5], 1u << (t & 31));
    });
    int* ocn = (int*)(slot + 4);
    unsigned short* otp = (unsigned short*)(slot + 4 + 4 * (long)c);
    // compaction in topic order: lane L scans bitmap word wb + L (32 topics)
    int base = 0;
    for (int wb = 0; wb < nbw; wb += 64) {
      const int wi = wb + lane;
      const unsigned m = wi < nbw ? bits[wi] : 0u;
      int mine = 0;
      for (unsigned mm = m; mm; mm &= mm - 1) {
        const int v = acc[(wi << 5) + __builtin_ctz(mm)];
        mine += v != 0;
        neg |= v < 0;
      }
      const float incl = wave_scan_incl((float)mine);  // <= 64 x 32: exact
      int pos = base + (int)incl - mine;
      for (unsigned mm = m; mm; mm &= mm - 1) {
        const int t = (wi << 5) + __builtin_ctz(mm);
        const int v = acc[t];
        if (v != 0) {
          if (pos < c) {
            ocn[pos] = v;
            otp[pos] = (unsigned short)t;
          } else {
            over = true;
          }
          ++pos;
        }
        acc[t] = 0;
      }
      if (wi < nbw) bits[wi] = 0u;
      base += (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
    }
    if (lane == 0) *(int*)slot = base < c ? base : c;
  }
  if (__ballot(over) && lane == 0) atomicOr(overflow, 1);
  if (__ballot(neg) && lane == 0) atomicOr(overflow, 2);
}

// empty every slot for a kernel to fill: the nnz word of a sparse slot, the whole row of a
// dense one (the entries past nnz are never read), instead of clearing the whole payload
__global__ __launch_bounds__(kMaxWaves * 64) void rowcodec_reset_kernel(unsigned char* __restrict__ buf,
                                                                       const long* __restrict__ off,
                                                                       const int* __restrict__ cap, int n, int K) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, W = blockDim.x >> 6;
  for (int j = blockIdx.x * W + w; j < n; j += gridDim.x * W) {
    unsigned char* slot = buf + off[j];
    if (cap[j] < 0) {
      int4* s4 = (int4*)slot;
      for (int q = lane; q < K / 4; q += 64) s4[q] = make_int4(0, 0, 0, 0);
    } else if (lane == 0) {
      *(int*)slot = 0;
    }
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

// canonical slots u (canon + c_off[u], cap c_cap[u]) += the delta slots src_idx[src_ptr[u] ..
// src_ptr[u + 1]) of `in` (in_off / in_cap), re-encoded in place: the rows listed in
// tiny / small / hash rows (entry bounds: harp_rowcodec_merge_bounds) by the lane-group LDS
// hash kernels, the rows in big_rows by the dense-accumulator kernel
// class bounds, smallest first: rows with at most bound[i] entries go to list i
HARP_EXPORT int harp_rowcodec_merge_bounds(int* out3) {
  out3[0] = kTinyBound;
  out3[1] = kSmallBound;
  out3[2] = kHashBound;
  return HARP_OK;
}

HARP_EXPORT int harp_rowcodec_merge_meta_bytes() { return (int)sizeof(MergeMeta); }

// meta_tiny / meta_small / meta_hash: MergeMeta rows of each lane-group class (qoff / qcap:
// every delta slot's offset / capacity in CSR order, for rows with more than one); big_rows:
// the rest, by the dense-accumulator kernel (c_off, c_cap, src_ptr, src_idx, in_off, in_cap)
HARP_EXPORT int harp_rowcodec_merge(void* canon, const void* in, const void* meta_tiny, int n_tiny,
                                    const void* meta_small, int n_small, const void* meta_hash, int n_hash,
                                    const long* qoff, const int* qcap, const int* big_rows, int n_big,
                                    const long* c_off, const int* c_cap, const int* src_ptr, const int* src_idx,
                                    const long* in_off, const int* in_cap, int K, int* overflow, hipStream_t s) {
  if (n_tiny < 0 || n_small < 0 || n_hash < 0 || n_big < 0 || K <= 0 || (K & 3) || K > 16384 ||
      misaligned(canon) || misaligned(in) || !overflow)
    return HARP_EBADARG;
  auto group = [&](auto kern, const void* meta, int nr, int per_wg) {
    int grid = (nr + per_wg - 1) / per_wg;
    if (grid > 16384) grid = 16384;
    kern<<<dim3((unsigned)grid), dim3(256), 0, s>>>((unsigned char*)canon, (const MergeMeta*)meta, nr, qoff, qcap,
                                                   (const unsigned char*)in, K, overflow);
  };
  if (n_tiny > 0) group(rowcodec_merge_group_kernel<16, 128>, meta_tiny, n_tiny, 16);
  if (n_small > 0) group(rowcodec_merge_group_kernel<32, 512>, meta_small, n_small, 8);
  if (n_hash > 0) group(rowcodec_merge_group_kernel<64, 1024>, meta_hash, n_hash, 4);
  if (n_big > 0) {
    const int per_wave = (K + (K + 31) / 32 + 3) & ~3;  // ints: accumulator + bitmap
    int wv = kLdsBudget / (4 * per_wave);
    wv = wv < 1 ? 1 : (wv > kMaxWaves ? kMaxWaves : wv);
    int grid = (n_big + wv - 1) / wv;
    if (grid > 4096) grid = 4096;
    const size_t lds = sizeof(int) * (size_t)per_wave * wv;
    if (lds > 65536 && hipFuncSetAttribute((const void*)rowcodec_merge_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return HARP_ELAUNCH;
    rowcodec_merge_kernel<<<dim3((unsigned)grid), dim3(wv * 64), lds, s>>>(
        (unsigned char*)canon, c_off, c_cap, big_rows, n_big, src_ptr, src_idx, (const unsigned char*)in, in_off,
        in_cap, K, per_wave, overflow);
  }
  return harp_launch_status();
}

HARP_EXPORT int harp_rowcodec_reset(void* buf, const long* off, const int* cap, int n, int K, hipStream_t s) {
  if (n < 0 || K <= 0 || (K & 3) || misaligned(buf)) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  int grid = (n + kMaxWaves - 1) / kMaxWaves;
  if (grid > 8192) grid = 8192;
  rowcodec_reset_kernel<<<dim3((unsigned)grid), dim3(kMaxWaves * 64), 0, s>>>((unsigned char*)buf, off, cap, n, K);
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
