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
//    product is r/16 packed FMAs per lane + a 4-step DPP row reduction; a wave runs four
//    independent streams.
//  * each stream owns a contiguous run of the slice's ratings sorted by USER: the user's
//    w row stays in registers while its ratings stream past and is written back once per
//    run; H rows are read (from L2, bypassing the CU's L1) and written per rating,
//    lock-free across streams (Hogwild, as DAAL-SGD).
//  * XCD blocking (mf_sgd_xcd_kernel, the production path): the 8 XCDs have private,
//    mutually non-coherent L2s. A flat Hogwild launch lets every XCD cache its own copy of
//    hot H rows, so concurrent updates of one item from different XCDs overwrite each other
//    at write-back, and H is served from the Infinity Fabric / MALL. The blocked layout
//    cuts the resident slice into 8 x 8 equal-work (user block, item block) cells; in
//    sub-step s the blocks of one XCD (blocks sharing blockIdx.x % 8 share an XCD) train
//    cell (x, (x + s) mod 8). The 8 cells of a sub-step share no user and no item, so each
//    H block (~1/8 of the slice, inside one XCD's 4 MB L2) is updated by one XCD only, and
//    the kernel boundary between sub-steps publishes it — the Harp rotation schedule
//    (dymoro), applied one level down, across the XCDs of a GPU. Index triples are staged
//    through LDS and H rows prefetched two ratings ahead (sgd_stream_lds).
//  * the flat kernel (mf_sgd_kernel) keeps the original one-stream-per-chunk launch for
//    comparison and for unblocked rating sets.
#include "common.h"

#include <climits>

namespace {

// Factor-row layout inside a 16-lane stream: lane sl holds the float4 chunks at
// row + 64*q + 4*sl (q < EPL/4), or for EPL % 4 != 0 the floats at row + 16*k + sl. Every
// wave instruction then reads / writes whole contiguous 256-B (64-B) row segments — full
// 128-B L2 lines. (The first layout, lane-contiguous chunks of EPL floats, made each
// dwordx4 instruction touch every other 16 B: half-filled sectors, twice the L2 write
// requests, and the texture addresser 86 % busy — profiles/r1_sgd_xcd/sgdpmc.) Any
// layout works as long as W and H use the same one: the update is elementwise and the
// dot product sums over all factors.
template <int EPL>
__device__ __forceinline__ unsigned lane_off(int sl) {
  return EPL % 4 == 0 ? 4u * (unsigned)sl : (unsigned)sl;
}

template <int EPL>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&x)[EPL]) {
  if constexpr (EPL % 4 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) {
      const floatx4 v = *(const floatx4*)(p + 16 * k);
      x[k] = v[0]; x[k + 1] = v[1]; x[k + 2] = v[2]; x[k + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = p[16 * k];
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
      const floatx4 v = __builtin_nontemporal_load((const floatx4*)(p + 16 * k));
      x[k] = v[0]; x[k + 1] = v[1]; x[k + 2] = v[2]; x[k + 3] = v[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) x[k] = __builtin_nontemporal_load(p + 16 * k);
  }
}

template <int EPL>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&x)[EPL]) {
  if constexpr (EPL % 4 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4) *(floatx4*)(p + 16 * k) = floatx4{x[k], x[k + 1], x[k + 2], x[k + 3]};
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k) p[16 * k] = x[k];
  }
}

// Delta write-back for conflicting concurrent streams (ATOM kernels): x is ADDED to the row
// with L2 float atomics (no return) instead of overwriting it, so two streams that update
// one row at the same time both keep their contribution (a plain store keeps only the last
// writer's). Workgroup scope: all global atomics execute in the XCD's L2, which every CU of
// the XCD shares -- the only agents that touch a cell's rows inside a launch.
template <int EPL>
__device__ __forceinline__ void add_row(float* __restrict__ p, const float (&x)[EPL]) {
  if constexpr (EPL % 4 == 0) {
#pragma unroll
    for (int k = 0; k < EPL; k += 4)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __hip_atomic_fetch_add(p + 16 * k + j, x[k + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
#pragma unroll
    for (int k = 0; k < EPL; ++k)
      __hip_atomic_fetch_add(p + 16 * k, x[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// W rows: L1-cached loads, or (persistent flow kernel, where rows written earlier in the
// same launch by other CUs of the XCD must be seen) loads from L2 like the H rows
template <int EPL, bool L2>
__device__ __forceinline__ void load_w(const float* __restrict__ p, float (&x)[EPL]) {
  if constexpr (L2)
    load_row_l2<EPL>(p, x);
  else
    load_row<EPL>(p, x);
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

// Sum over the 16 lanes of a DPP row (= one update stream), result in every lane: row
// rotations by 8 and 4, then the two quad permutations. Four dependent VALU ops with DPP
// operands instead of four ds_bpermute round trips through the LDS crossbar.
__device__ __forceinline__ float sub16_sum(float v) {
  v += dpp<0x128>(v);  // row_ror:8
  v += dpp<0x124>(v);  // row_ror:4
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  return v;
}

__device__ __forceinline__ int shfl16(int v, int src) { return __shfl(v, src, 16); }
__device__ __forceinline__ float shfl16(float v, int src) { return __shfl(v, src, 16); }

// 16 consecutive ratings, one per lane of the subgroup (coalesced; masked past u1)
__device__ __forceinline__ void load16(const int* __restrict__ rows, const int* __restrict__ cols,
                                       const float* __restrict__ vals, unsigned base, unsigned u1, int sl, int& r,
                                       int& c, float& v) {
  const unsigned k = base + (unsigned)sl;
  if (k < u1) {
    r = rows[k];
    c = cols[k];
    v = vals[k];
  }
}

// One update stream: ratings [u0, u1) of rows/cols/vals in order, run by the 16-lane
// subgroup holding lane `sl`.
//  * indices: the (row, col, value) triples arrive 16 at a time (one per lane, the next batch
//    in flight) and are broadcast inside the subgroup, so an H-row prefetch never waits on
//    an index load;
//  * H rows are prefetched TWO ratings ahead into ping-pong buffers, and each prefetch is
//    issued after the previous rating's H store. CDNA's vmcnt retires loads and stores in
//    issue order, so with a distance of one every wait for the next row also waited for the
//    store just issued (measured: dropping the stores alone ran 1.7x faster); at distance two
//    the wait only covers the load issued a full update earlier. A row is forwarded in
//    registers when the next rating hits the same item; a row loaded after the store of the
//    same item (same wave, program order) already sees it;
//  * update w' = (1 - lr*lam) w - lr*err*h (and h' alike): 2 packed fp32 ops per factor pair.
// All offsets are 32-bit (uniform 64-bit bases stay in SGPRs).
template <int R>
__device__ __forceinline__ void sgd_stream(const int* __restrict__ rows, const int* __restrict__ cols,
                                           const float* __restrict__ vals, unsigned u0, unsigned u1, int sl,
                                           float* __restrict__ W, unsigned ldw, float* __restrict__ H, unsigned ldh,
                                           float lr, float lam) {
  constexpr int EPL = R / 16;
  constexpr int PAIRS = EPL / 2;
  const float decay = 1.0f - lr * lam;
  const unsigned lo = lane_off<EPL>(sl);
  float w[EPL], h[EPL], hA[EPL], hB[EPL];
  unsigned base = u0;
  int bR = 0, bC = 0, nR = 0, nC = 0;
  float bV = 0.f, nV = 0.f;
  load16(rows, cols, vals, base, u1, sl, bR, bC, bV);
  load16(rows, cols, vals, base + 16, u1, sl, nR, nC, nV);
  // rating i = u0 (current) and i + 1 (in flight)
  unsigned cur = (unsigned)shfl16(bR, 0), col0 = (unsigned)shfl16(bC, 0);
  float v0 = shfl16(bV, 0);
  unsigned row1 = (unsigned)shfl16(bR, 1), col1 = (unsigned)shfl16(bC, 1);
  float v1 = shfl16(bV, 1);
  load_row<EPL>(W + (cur * ldw + lo), w);
  load_row_l2<EPL>(H + (col0 * ldh + lo), h);
  if (u0 + 1 < u1) load_row_l2<EPL>(H + (col1 * ldh + lo), hB);
  unsigned i = u0;

  // one rating; `hl` receives the prefetch of rating i + 2, `hx` holds rating i + 1's row
  auto step = [&](float(&hl)[EPL], float(&hx)[EPL]) -> bool {
    floatx2 d2 = {0.f, 0.f};
#pragma unroll
    for (int p = 0; p < PAIRS; ++p)
      d2 = __builtin_elementwise_fma(floatx2{w[2 * p], w[2 * p + 1]}, floatx2{h[2 * p], h[2 * p + 1]}, d2);
    float dot = d2[0] + d2[1];
    if constexpr (EPL % 2) dot = fmaf(w[EPL - 1], h[EPL - 1], dot);
    const float ge = -lr * (sub16_sum(dot) - v0);
    const floatx2 g = {ge, ge}, dc = {decay, decay};
#pragma unroll
    for (int p = 0; p < PAIRS; ++p) {
      const floatx2 wk = {w[2 * p], w[2 * p + 1]}, hk = {h[2 * p], h[2 * p + 1]};
      const floatx2 wn = __builtin_elementwise_fma(g, hk, dc * wk);
      const floatx2 hn = __builtin_elementwise_fma(g, wk, dc * hk);
      w[2 * p] = wn[0];
      w[2 * p + 1] = wn[1];
      h[2 * p] = hn[0];
      h[2 * p + 1] = hn[1];
    }
    if constexpr (EPL % 2) {
      const float wk = w[EPL - 1], hk = h[EPL - 1];
      w[EPL - 1] = fmaf(ge, hk, decay * wk);
      h[EPL - 1] = fmaf(ge, wk, decay * hk);
    }
    store_row<EPL>(H + (col0 * ldh + lo), h);
    // indices + prefetch of rating i + 2 (issued after the store above)
    const unsigned t2 = i + 2 - base;
    if (t2 == 16) {
      base += 16;
      bR = nR;
      bC = nC;
      bV = nV;
      load16(rows, cols, vals, base + 16, u1, sl, nR, nC, nV);
    }
    unsigned row2 = row1, col2 = col1;
    float v2 = 0.f;
    if (i + 2 < u1) {
      const int tt = (int)(t2 & 15u);
      row2 = (unsigned)shfl16(bR, tt);
      col2 = (unsigned)shfl16(bC, tt);
      v2 = shfl16(bV, tt);
      load_row_l2<EPL>(H + (col2 * ldh + lo), hl);
    }
    if (i + 1 >= u1) return false;
    if (row1 != cur) {
      store_row<EPL>(W + (cur * ldw + lo), w);
      cur = row1;
      load_row<EPL>(W + (cur * ldw + lo), w);
    }
    if (col1 != col0) {  // else: same item again, keep the row just updated
#pragma unroll
      for (int k = 0; k < EPL; ++k) h[k] = hx[k];
    }
    col0 = col1;
    v0 = v1;
    row1 = row2;
    col1 = col2;
    v1 = v2;
    ++i;
    return true;
  };
  while (step(hA, hB) && step(hB, hA)) {
  }
  store_row<EPL>(W + (cur * ldw + lo), w);
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
  sgd_stream<R>(rows + i0, cols + i0, vals + i0, 0u, (unsigned)(i1 - i0), sl, W, (unsigned)ldw, H, (unsigned)ldh,
                lr, lam);
}

constexpr int XCDS = 8;

// One update stream whose (row, col, value) triples sit in LDS (sR/sC/sV[0..n)), staged by
// the workgroup. CDNA retires vmcnt in issue order and counts stores too, so the loop is
// ordered never to wait on anything younger than what it consumes (no vmcnt(0) in the loop):
//  * index reads are LDS traffic (lgkmcnt), not vector memory;
//  * per rating: update -> W switch (rare; store old row, load new) -> prefetch the H row of
//    rating i+2 into a ping-pong buffer -> store this rating's H row;
//  * a prefetch is issued before the stores of the two ratings preceding its use, so a row
//    is forwarded in registers when rating i+1 repeats the item of rating i or i-1 (the
//    updated rows of the last two ratings are kept: h, hp).
// Loads are unconditional (clamped indices), so the wait counts stay exact. Measured on
// MI355X (profiles/r1_sgd_xcd): per-stream latency is NOT the limit — removing the index /
// store waits changed nothing, while ablating the H stores (+66 %) or the H loads (+32 %)
// and uniform instead of skewed item popularity (+30 %) did: the kernel is bound by L2
// traffic on hot H rows.
//
// ATOM: conflict-preserving write-back. Concurrent streams of an XCD share hot H rows and
// the rows of users whose ratings straddle two streams; a plain store keeps one writer's
// update (measured on the reference's ML-10M gate: 0.855 test RMSE after 200 epochs on the
// GPU vs 0.834 sequential). Bit 0: a W row is written back as the atomic add of the
// stream's total change to it (w - w at load; one add per factor per user run). Bit 1:
// the H write of every rating is an L2 atomic add of that rating's change (measured 60x
// slower on the skewed Netflix-shape bench: hot rows serialise in the L2 atomic units).
// With both no update is lost -- concurrent updates are merely stale. Bit 2 (hot H): only
// the items flagged hot by the host (bit 31 of the column index: the few items that carry
// most of a cell's sum of squared shares, where concurrent streams collide) take the atomic
// add; every other H row keeps the plain store, so a skewed set pays atomics only on the
// rows whose updates would otherwise be lost (ops/mf.py hot_flags).
template <int R, bool WL2 = false, int ATOM = 0>
__device__ __forceinline__ void sgd_stream_lds(const int* sR, const int* sC, const float* sV, int n, int sl,
                                               float* __restrict__ W, unsigned ldw, float* __restrict__ H,
                                               unsigned ldh, float lr, float lam) {
  constexpr int EPL = R / 16;
  constexpr int PAIRS = EPL / 2;
  constexpr bool AW = (ATOM & 1) != 0, AH = (ATOM & 2) != 0, HH = (ATOM & 4) != 0 && !AH;
  constexpr int W0 = AW ? EPL : 1;
  // hot-H mode: the column index carries the hot flag in bit 31 (addresses drop it; the
  // flag is a property of the item, so equal indices still mean equal rows)
  auto hrow = [&](unsigned c) -> unsigned { return HH ? (c & 0x7fffffffu) : c; };
  const float decay = 1.0f - lr * lam;
  const unsigned lo = lane_off<EPL>(sl);
  float w[EPL], h[EPL], hp[EPL], hA[EPL], hB[EPL];
  float w0[W0];  // ATOM: the W row as loaded (its write-back is w - w0)
  auto keep_w0 = [&]() {
    if constexpr (AW) {
#pragma unroll
      for (int k = 0; k < EPL; ++k) w0[k] = w[k];
    }
  };
  auto put_w = [&](float* p) {
    if constexpr (AW) {
      float dw[EPL];
#pragma unroll
      for (int k = 0; k < EPL; ++k) dw[k] = w[k] - w0[k];
      add_row<EPL>(p, dw);
    } else {
      store_row<EPL>(p, w);
    }
  };
  unsigned cur = (unsigned)sR[0], col0 = (unsigned)sC[0], colp = 0xffffffffu;
  float v0 = sV[0];
  const int i1c = n > 1 ? 1 : 0;
  unsigned row1 = (unsigned)sR[i1c], col1 = (unsigned)sC[i1c];
  float v1 = sV[i1c];
  load_w<EPL, WL2>(W + (cur * ldw + lo), w);
  keep_w0();
  load_row_l2<EPL>(H + (hrow(col0) * ldh + lo), h);
  load_row_l2<EPL>(H + (hrow(col1) * ldh + lo), hB);
#pragma unroll
  for (int k = 0; k < EPL; ++k) hp[k] = 0.f;
  int i = 0;
  float dh[AH || HH ? EPL : 1];  // AH / HH: this rating's change of its H row
  const float dm1 = -lr * lam;
  auto step = [&](float(&hl)[EPL], float(&hx)[EPL]) -> bool {
    floatx2 d2 = {0.f, 0.f};
#pragma unroll
    for (int p = 0; p < PAIRS; ++p)
      d2 = __builtin_elementwise_fma(floatx2{w[2 * p], w[2 * p + 1]}, floatx2{h[2 * p], h[2 * p + 1]}, d2);
    float dot = d2[0] + d2[1];
    if constexpr (EPL % 2) dot = fmaf(w[EPL - 1], h[EPL - 1], dot);
    const float ge = -lr * (sub16_sum(dot) - v0);
    const floatx2 g = {ge, ge}, dc = {decay, decay};
#pragma unroll
    for (int p = 0; p < PAIRS; ++p) {
      const floatx2 wk = {w[2 * p], w[2 * p + 1]}, hk = {h[2 * p], h[2 * p + 1]};
      const floatx2 wn = __builtin_elementwise_fma(g, hk, dc * wk);
      if constexpr (AH || HH) {
        const floatx2 d = __builtin_elementwise_fma(g, wk, floatx2{dm1, dm1} * hk);
        dh[2 * p] = d[0];
        dh[2 * p + 1] = d[1];
        h[2 * p] += d[0];
        h[2 * p + 1] += d[1];
      } else {
        const floatx2 hn = __builtin_elementwise_fma(g, wk, dc * hk);
        h[2 * p] = hn[0];
        h[2 * p + 1] = hn[1];
      }
      w[2 * p] = wn[0];
      w[2 * p + 1] = wn[1];
    }
    if constexpr (EPL % 2) {
      const float wk = w[EPL - 1], hk = h[EPL - 1];
      w[EPL - 1] = fmaf(ge, hk, decay * wk);
      if constexpr (AH || HH) {
        dh[EPL - 1] = fmaf(ge, wk, dm1 * hk);
        h[EPL - 1] = hk + dh[EPL - 1];
      } else {
        h[EPL - 1] = fmaf(ge, wk, decay * hk);
      }
    }
    const bool last = i + 1 >= n;
    if (!last && row1 != cur) {
      put_w(W + (cur * ldw + lo));
      cur = row1;
      load_w<EPL, WL2>(W + (cur * ldw + lo), w);
      keep_w0();
    }
    const int i2 = i + 2 < n ? i + 2 : n - 1;  // clamped: the last prefetch is a harmless re-read
    const unsigned row2 = (unsigned)sR[i2], col2 = (unsigned)sC[i2];
    const float v2 = sV[i2];
    load_row_l2<EPL>(H + (hrow(col2) * ldh + lo), hl);
    if constexpr (AH) {
      add_row<EPL>(H + (col0 * ldh + lo), dh);
    } else if constexpr (HH) {
      if (col0 >> 31)
        add_row<EPL>(H + (hrow(col0) * ldh + lo), dh);
      else
        store_row<EPL>(H + (col0 * ldh + lo), h);
    } else {
      store_row<EPL>(H + (col0 * ldh + lo), h);
    }
    if (last) return false;
    // row of rating i+1: just updated (same item as i), updated one rating ago (same item as
    // i-1, its store was issued after the prefetch), or the prefetched copy
    const bool s0 = col1 == col0, s1 = col1 == colp;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
      const float nx = s0 ? h[k] : (s1 ? hp[k] : hx[k]);
      hp[k] = h[k];
      h[k] = nx;
    }
    colp = col0;
    col0 = col1;
    v0 = v1;
    row1 = row2;
    col1 = col2;
    v1 = v2;
    ++i;
    return true;
  };
  while (step(hA, hB) && step(hB, hA)) {
  }
  put_w(W + (cur * ldw + lo));
}

// Sub-step `step` of the XCD-blocked schedule. off[c] .. off[c + 1] are the ratings of cell
// c = user_block * 8 + item_block (cell-major, user-sorted inside a cell). The blocks that
// share an XCD (same blockIdx.x % 8) take rounds of 16 consecutive streams of CH ratings:
// the round's 16*CH index triples are one contiguous, coalesced copy into LDS, then each
// 16-lane subgroup runs one stream. `win` (optional, 2 x 64 int64): cell c trains only the
// window of win[64 + c] ratings starting at win[c], wrapping around the cell — the
// fixed-fraction mode standing in for the reference's timer-bounded rotation steps.
//
// Placement check (chk != NULL): the schedule is only coherent if every block of residue x
// runs on ONE XCD (its W and H blocks then live in one L2; residues sharing an XCD touch
// disjoint blocks, and launches are ordered by the stream). Thread 0 of each block reads
// HW_REG_XCC_ID at the block's end and tags, for launch number `gen` (host counter, > 0),
// residue -> XCC in a 64-bit word ((gen << 8) | id + 1; the first block of a launch to see an
// older generation installs its own, so no reset launch is needed). A block whose XCC
// disagrees with the installed one raises chk[kChkErr] (sticky; the host reads it once per
// epoch, ops.mf.check_placement, and switches to the placed kernel below).
constexpr int kChkWords = 32;  // [0, 8) residue map | [24] error
constexpr int kChkErr = 24;

__device__ __forceinline__ unsigned tag_once(unsigned long long* p, unsigned long long gen, unsigned val) {
  unsigned long long cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long mine = (gen << 8) | val;
  while ((cur >> 8) != gen) {
    if (__hip_atomic_compare_exchange_strong(p, &cur, mine, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return val;
  }
  return (unsigned)(cur & 0xff);
}

__device__ __forceinline__ int hw_xcc_id() {
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;  // HW_REG_XCC_ID
}

// Called by thread 0 at the END of a block (at the start, every block's first barrier waited
// on these device-scope atomics, which all blocks of a residue aim at one word: 2.5 % of an
// epoch). Only residue -> XCC is checked: it is what coherence needs (all of a residue's
// blocks in one L2); two residues sharing an XCD touch disjoint W / H blocks.
__device__ __forceinline__ void placement_check(unsigned long long* chk, unsigned long long gen, int x) {
  if (chk == nullptr || threadIdx.x != 0) return;
  const int hw = hw_xcc_id();
  if (tag_once(chk + x, gen, (unsigned)hw + 1) != (unsigned)hw + 1)
    __hip_atomic_store(chk + kChkErr, 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int R, int CH, int ATOM>
__global__ __launch_bounds__(256) void mf_sgd_xcd_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                         const float* __restrict__ vals, const long* __restrict__ off,
                                                         const long* __restrict__ win, int step,
                                                         float* __restrict__ W, int ldw, float* __restrict__ H, int ldh,
                                                         float lr, float lam, unsigned long long* chk,
                                                         unsigned long long gen) {
  __shared__ int sR[16 * CH], sC[16 * CH];
  __shared__ float sV[16 * CH];
  const int x = blockIdx.x % XCDS;
  const long j = blockIdx.x / XCDS;
  const long per_xcd = gridDim.x / XCDS;
  const int cell = x * XCDS + (x + step) % XCDS;
  const long a = off[cell];
  const long ncell = off[cell + 1] - a;
  const long w0 = win ? win[cell] : 0;
  const long n = win ? win[XCDS * XCDS + cell] : ncell;
  const long nst = (n + CH - 1) / CH;
  const int sl = threadIdx.x & 15;
  const int sub = threadIdx.x >> 4;  // 16 streams per 256-thread block
  for (long st0 = j * 16; st0 < nst; st0 += per_xcd * 16) {
    const long r0 = st0 * CH;
    __syncthreads();  // the previous round is done with the LDS triples
    for (int k = threadIdx.x; k < 16 * CH; k += 256) {
      if (r0 + k < n) {
        long q = w0 + r0 + k;
        if (q >= ncell) q -= ncell;
        sR[k] = rows[a + q];
        sC[k] = cols[a + q];
        sV[k] = vals[a + q];
      }
    }
    __syncthreads();
    const long mine = n - (r0 + (long)sub * CH);
    if (mine > 0)
      sgd_stream_lds<R, false, ATOM>(sR + sub * CH, sC + sub * CH, sV + sub * CH, mine < CH ? (int)mine : CH, sl, W,
                             (unsigned)ldw, H, (unsigned)ldh, lr, lam);
  }
  placement_check(chk, gen, x);
}

// Placement-independent sub-step (the fallback when placement_check fires): a block trains
// the cell of the XCD it RUNS on (row x = HW_REG_XCC_ID), not the one its blockIdx.x
// names, so one XCD per cell holds by construction whatever the dispatcher does. Blocks
// of an XCD claim rounds of the cell from a counter (ws[x]); a cell whose XCD received no
// block at all (every block of the grid landed elsewhere) is left fully unclaimed -- its
// rows were touched by nobody in this launch -- and the LAST block to leave trains it
// alone (ws[9] counts such drains), then zeroes the counters for the next launch on this
// stream. Every round of every cell is trained exactly once.
// ws layout (int32): claim[8] | exit | drained
constexpr int kPlacedWs = 10;

template <int R, int CH, int ATOM>
__device__ __forceinline__ void xcd_round(const int* __restrict__ rows, const int* __restrict__ cols,
                                          const float* __restrict__ vals, long a, long w0, long ncell, long n, long rd,
                                          int* sR, int* sC, float* sV, float* __restrict__ W, int ldw,
                                          float* __restrict__ H, int ldh, float lr, float lam) {
  const int sl = threadIdx.x & 15;
  const int sub = threadIdx.x >> 4;
  const long r0 = rd * 16 * CH;
  __syncthreads();  // the previous round is done with the LDS triples
  for (int k = threadIdx.x; k < 16 * CH; k += 256) {
    if (r0 + k < n) {
      long q = w0 + r0 + k;
      if (q >= ncell) q -= ncell;
      sR[k] = rows[a + q];
      sC[k] = cols[a + q];
      sV[k] = vals[a + q];
    }
  }
  __syncthreads();
  const long left = n - (r0 + (long)sub * CH);
  if (left > 0)
    sgd_stream_lds<R, false, ATOM>(sR + sub * CH, sC + sub * CH, sV + sub * CH, left < CH ? (int)left : CH, sl, W,
                                   (unsigned)ldw, H,
                      (unsigned)ldh, lr, lam);
}

template <int R, int CH, int ATOM>
__global__ __launch_bounds__(256) void mf_sgd_xcd_placed_kernel(const int* __restrict__ rows,
                                                                const int* __restrict__ cols,
                                                                const float* __restrict__ vals,
                                                                const long* __restrict__ off,
                                                                const long* __restrict__ win, int step,
                                                                float* __restrict__ W, int ldw, float* __restrict__ H,
                                                                int ldh, float lr, float lam, int* __restrict__ ws) {
  __shared__ int sR[16 * CH], sC[16 * CH];
  __shared__ float sV[16 * CH];
  __shared__ int s_round, s_last;
  const int x = hw_xcc_id() & (XCDS - 1);
  auto cell_of = [&](int xx, long& a, long& w0, long& ncell, long& n) {
    const int cell = xx * XCDS + (xx + step) % XCDS;
    a = off[cell];
    ncell = off[cell + 1] - a;
    w0 = win ? win[cell] : 0;
    n = win ? win[XCDS * XCDS + cell] : ncell;
  };
  long a, w0, ncell, n;
  cell_of(x, a, w0, ncell, n);
  const long rounds = (n + 16 * CH - 1) / (16 * CH);
  for (;;) {
    if (threadIdx.x == 0)
      s_round = __hip_atomic_fetch_add(ws + x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const long rd = s_round;
    __syncthreads();  // everyone read s_round before it is rewritten
    if (rd >= rounds) break;
    xcd_round<R, CH, ATOM>(rows, cols, vals, a, w0, ncell, n, rd, sR, sC, sV, W, ldw, H, ldh, lr, lam);
  }
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(ws + 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  for (int xx = 0; xx < XCDS; ++xx) {
    if (__hip_atomic_load(ws + xx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) continue;
    cell_of(xx, a, w0, ncell, n);
    const long rr = (n + 16 * CH - 1) / (16 * CH);
    for (long rd = 0; rd < rr; ++rd)
      xcd_round<R, CH, ATOM>(rows, cols, vals, a, w0, ncell, n, rd, sR, sC, sV, W, ldw, H, ldh, lr, lam);
    if (threadIdx.x == 0 && rr > 0) __hip_atomic_fetch_add(ws + 9, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 0; k < 9; ++k) __hip_atomic_store(ws + k, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Persistent XCD-blocked pass: all `steps` sub-steps of one slice in ONE launch, ordered by
// point-to-point completion flags instead of kernel boundaries (the reference's dymoro
// Scheduler hands a block to a thread as soon as its row and column are free,
// ml/java/.../dymoro/Scheduler.java:95-237; here the unit is an XCD cell).
//
// In sub-step s XCD x trains cell (x, (x + s) mod 8): its user block x is private to the
// XCD in every sub-step, and its item block (x + s) mod 8 was trained in sub-step s - 1 by
// XCD x + 1 (and in s + 1 by XCD x - 1). So XCD x may start sub-step s as soon as XCD
// x + 1 has FINISHED sub-step s - 1 -- a dependency on one neighbour, no grid barrier.
//  * work: rounds of 16 streams x CH ratings are claimed from a per-(XCD, sub-step)
//    counter by any block of the XCD, so no block ever waits on a specific other block;
//    a block waits for the neighbour only after it has claimed a round (blocks left
//    without work move on, so few blocks poll); the first 8 blocks dispatched cover the
//    8 XCDs, so every XCD always has a running block and every wait terminates (the chain
//    of waits ends at sub-step 0);
//  * completion: a block that finds no more rounds of (x, s) waits for its own stores
//    (once) and adds the rounds it trained; the block whose add completes the count writes
//    the XCD's L2 back (agent release) and raises fin[x][s];
//  * visibility: XCD x reads item block b only after its producer's write-back, and its
//    own L2 holds no line of b in this launch (b was not touched by x since the launch
//    started, and a launch starts with invalidated caches), so no invalidation is needed;
//    W rows (written by other CUs of the same XCD in earlier sub-steps) are read from L2;
//  * the last block to leave zeroes the counters for the next launch on this stream;
//  * a wait gives up after ~1 s and raises the error word (1; a launch-geometry bug must
//    never hang the GPU); a block that runs on another XCD than blockIdx.x mod 8 raises it
//    too (2); the host checks it once per epoch.
// ws layout (int32): claim[64] | done[64] | fin[64] | xcc map[9] | exit | error
constexpr int kFlowWs = 3 * 64 + 9 + 2;

// compare-and-swap 0 -> v; returns the previous value (0 when this call stored v)
__device__ __forceinline__ int cas_zero(int* p, int v) {
  int expected = 0;
  __hip_atomic_compare_exchange_strong(p, &expected, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return expected;
}

// raise a completion flag after writing this XCD's L2 back (agent-scope release), with an
// explicit wait so the flag cannot overtake the write-back
__device__ __forceinline__ void publish(int* flag) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_s_waitcnt(0);
  __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int R, int CH>
__global__ __launch_bounds__(256) void mf_sgd_xcd_flow_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                              const float* __restrict__ vals,
                                                              const long* __restrict__ off,
                                                              const long* __restrict__ win, int steps,
                                                              float* __restrict__ W, int ldw, float* __restrict__ H,
                                                              int ldh, float lr, float lam, int* __restrict__ ws) {
  __shared__ int sR[16 * CH], sC[16 * CH];
  __shared__ float sV[16 * CH];
  __shared__ int s_round;
  int* claim = ws;
  int* done = ws + 64;
  int* fin = ws + 128;
  int* xccmap = ws + 192;  // [8] XCC id + 1 per residue, [8] bit set of claimed XCCs
  int* exit_ctr = ws + 201;
  int* err = ws + 202;
  const int x = blockIdx.x % XCDS;
  const int nxt = (x + 1) % XCDS;
  const int sl = threadIdx.x & 15;
  const int sub = threadIdx.x >> 4;
  // the visibility argument above needs all blocks of one residue b mod 8 to RUN on one
  // XCD, and the 8 residues on 8 different XCDs (the round-robin dispatch of a single-
  // partition device; which physical XCD serves a residue does not matter -- measured: the
  // logical order is not the HW_REG_XCC_ID order on MI355X). The first block of residue x
  // records its XCC id; a block of x on another XCC, or two residues on one XCC, raise the
  // error word (2) and the host refuses the pass (ops.mf.check_flow_errors)
  if (threadIdx.x == 0) {
    const int hw = (__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf) + 1;  // HW_REG_XCC_ID
    const int prev = cas_zero(xccmap + x, hw);
    if (prev != 0 && prev != hw) __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int bit = 1 << (hw - 1);
    const int seen = __hip_atomic_fetch_or(xccmap + XCDS, prev == 0 ? bit : 0, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    if (prev == 0 && (seen & bit)) __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int step = 0; step < steps; ++step) {
    const int cell = x * XCDS + (x + step) % XCDS;
    const long a = off[cell];
    const long ncell = off[cell + 1] - a;
    const long w0 = win ? win[cell] : 0;
    const long n = win ? win[XCDS * XCDS + cell] : ncell;
    const long nst = (n + CH - 1) / CH;
    const int rounds = (int)((nst + 15) / 16);
    if (rounds == 0) {  // empty cell: complete at once (idempotent)
      if (threadIdx.x == 0) publish(fin + x * XCDS + step);
      continue;
    }
    int mine = 0;  // rounds of (x, step) this block trained
    for (;;) {
      if (threadIdx.x == 0)
        s_round = __hip_atomic_fetch_add(claim + x * XCDS + step, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int rd = s_round;
      __syncthreads();  // everyone read s_round before it is rewritten
      if (rd >= rounds) break;
      if (mine == 0 && step > 0) {
        // claimed work in (x, step): item block (x + step) mod 8 must be released by XCD
        // x + 1 (its sub-step step - 1). Blocks without work never wait, so only the
        // blocks that train poll the flag.
        if (threadIdx.x == 0) {
          long spins = 0;
          while (__hip_atomic_load(fin + nxt * XCDS + (step - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1L << 24)) {
              __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
          }
        }
        __syncthreads();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
      }
      const long r0 = (long)rd * 16 * CH;
      for (int k = threadIdx.x; k < 16 * CH; k += 256) {
        if (r0 + k < n) {
          long q = w0 + r0 + k;
          if (q >= ncell) q -= ncell;
          sR[k] = rows[a + q];
          sC[k] = cols[a + q];
          sV[k] = vals[a + q];
        }
      }
      __syncthreads();
      const long left = n - (r0 + (long)sub * CH);
      if (left > 0)
        sgd_stream_lds<R, true>(sR + sub * CH, sC + sub * CH, sV + sub * CH, left < CH ? (int)left : CH, sl, W,
                                (unsigned)ldw, H, (unsigned)ldh, lr, lam);
      __syncthreads();  // the LDS triples are free
      ++mine;
    }
    if (mine) {
      // every wave's H / W stores of this block's rounds are acknowledged by the XCD's L2
      // before they count (once per block and sub-step, not per round)
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (threadIdx.x == 0) {
        const int prev = __hip_atomic_fetch_add(done + x * XCDS + step, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + mine == rounds) publish(fin + x * XCDS + step);  // the last rounds of (x, step)
      }
    }
  }
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(exit_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (int)gridDim.x - 1) {  // every block has left: reset for the next launch
      for (int k = 0; k < 202; ++k) __hip_atomic_store(ws + k, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int R, int CH>
int launch_sgd_xcd_flow(const int* rows, const int* cols, const float* vals, const long* off, const long* win,
                        int steps, int blocks_per_xcd, float* W, int ldw, float* H, int ldh, float lr, float lam,
                        int* ws, hipStream_t s) {
  mf_sgd_xcd_flow_kernel<R, CH><<<dim3((unsigned)(blocks_per_xcd * XCDS)), dim3(256), 0, s>>>(
      rows, cols, vals, off, win, steps, W, ldw, H, ldh, lr, lam, ws);
  return harp_launch_status();
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
    load_row<EPL>(W + (long)rows[i] * ldw + lane_off<EPL>(sl), w);
    load_row<EPL>(H + (long)cols[i] * ldh + lane_off<EPL>(sl), h);
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

constexpr int kAtomBits = 28;  // variant bits 2..4: ATOM write-back mode (sgd_stream_lds: 4 = W, 8 = H, 16 = hot H)

// variant 0: blockIdx-placed sub-steps (+ placement check when chk != NULL; `gen` is the
// first launch's generation, one per sub-step); 2: mf_sgd_xcd_placed_kernel (pws)
template <int R, int CH>
int launch_sgd_xcd(const int* rows, const int* cols, const float* vals, const long* off, const long* win, int steps,
                   int blocks_per_xcd, float* W, int ldw, float* H, int ldh, float lr, float lam, int variant,
                   unsigned long long* chk, unsigned long long gen, int* pws, hipStream_t s) {
  const dim3 grid((unsigned)(blocks_per_xcd * XCDS));
  const int atom = (variant >> 2) & 7;
  const bool placed = (variant & 3) == 2;
  for (int step = 0; step < steps; ++step) {
    const unsigned long long g = gen + (unsigned long long)step;
#define XCD_LAUNCH(A)                                                                                        \
  do {                                                                                                       \
    if (placed)                                                                                              \
      mf_sgd_xcd_placed_kernel<R, CH, A><<<grid, dim3(256), 0, s>>>(rows, cols, vals, off, win, step, W, ldw, H, \
                                                                    ldh, lr, lam, pws);                        \
    else                                                                                                     \
      mf_sgd_xcd_kernel<R, CH, A><<<grid, dim3(256), 0, s>>>(rows, cols, vals, off, win, step, W, ldw, H, ldh,   \
                                                             lr, lam, chk, g);                                \
  } while (0)
    switch (atom) {
      case 1: XCD_LAUNCH(1); break;
      case 2: XCD_LAUNCH(2); break;
      case 3: XCD_LAUNCH(3); break;
      case 4: XCD_LAUNCH(4); break;
      case 5: XCD_LAUNCH(5); break;
      default: XCD_LAUNCH(0); break;
    }
#undef XCD_LAUNCH
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

// ---- wide ranks (256 < R <= 4096, R % 4 == 0; BASELINE #1 runs rank 2000) -------------
// ONE wave per update stream: lane l holds the float4 chunks at row + 4*l + 256*q (q < Q),
// so each wave instruction covers one contiguous 1 KB row segment; chunks at or past R are
// masked (no padding of the caller's rows needed). The row is too long for the 16-lane
// streams of the narrow kernels (R / 16 floats per lane); the dot product is a full-wave
// reduction. The next rating's H row is prefetched before this rating's H store (vmcnt
// retires in order: the wait for the prefetch never covers the store).
__device__ __forceinline__ float wave_sum_f(float v) {
  v = sub16_sum(v);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

template <int Q, bool NT>
__device__ __forceinline__ void load_wide(const float* __restrict__ p, int lane, int R, floatx4 (&x)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = 4 * lane + 256 * q;
    if (c < R) x[q] = NT ? __builtin_nontemporal_load((const floatx4*)(p + c)) : *(const floatx4*)(p + c);
    else x[q] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int Q>
__device__ __forceinline__ void store_wide(float* __restrict__ p, int lane, int R, const floatx4 (&x)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int c = 4 * lane + 256 * q;
    if (c < R) *(floatx4*)(p + c) = x[q];
  }
}

// ratings i0 .. i1 - 1 of the stream; rating i sits at index a + ((w0 + i) mod ncell)
// (the window wrap of the blocked schedule; a flat stream passes w0 = 0, ncell = huge)
template <int Q>
__device__ __forceinline__ void sgd_stream_wide(const int* __restrict__ rows, const int* __restrict__ cols,
                                                const float* __restrict__ vals, long a, long w0, long ncell, long i0,
                                                long i1, int lane, int R, float* __restrict__ W, long ldw,
                                                float* __restrict__ H, long ldh, float lr, float lam) {
  const float decay = 1.0f - lr * lam;
  auto at = [&](long i) {
    long q = w0 + i;
    if (q >= ncell) q -= ncell;
    return a + q;
  };
  floatx4 w[Q], h[Q], hn[Q];
  long k = at(i0);
  int cur = rows[k], col = cols[k];
  load_wide<Q, false>(W + cur * ldw, lane, R, w);
  load_wide<Q, true>(H + col * ldh, lane, R, h);
  for (long i = i0; i < i1; ++i) {
    const float v = vals[k];
    const bool more = i + 1 < i1;
    int nrow = cur, ncol = col;
    if (more) {
      k = at(i + 1);
      nrow = rows[k];
      ncol = cols[k];
      if (ncol != col) load_wide<Q, true>(H + ncol * ldh, lane, R, hn);
    }
    float d = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      d = fmaf(w[q][0], h[q][0], d);
      d = fmaf(w[q][1], h[q][1], d);
      d = fmaf(w[q][2], h[q][2], d);
      d = fmaf(w[q][3], h[q][3], d);
    }
    const float ge = -lr * (wave_sum_f(d) - v);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const floatx4 wk = w[q], hk = h[q];
      w[q] = ge * hk + decay * wk;
      h[q] = ge * wk + decay * hk;
    }
    store_wide<Q>(H + col * ldh, lane, R, h);
    if (!more) break;
    if (nrow != cur) {
      store_wide<Q>(W + cur * ldw, lane, R, w);
      cur = nrow;
      load_wide<Q, false>(W + cur * ldw, lane, R, w);
    }
    if (ncol != col) {
#pragma unroll
      for (int q = 0; q < Q; ++q) h[q] = hn[q];
      col = ncol;
    }
  }
  store_wide<Q>(W + cur * ldw, lane, R, w);
}

// flat: wave g runs ratings [g*chunk, (g+1)*chunk)
template <int Q>
__global__ __launch_bounds__(256) void mf_sgd_wide_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                          const float* __restrict__ vals, long n, int chunk, int R,
                                                          float* __restrict__ W, int ldw, float* __restrict__ H,
                                                          int ldh, float lr, float lam) {
  const long g = __builtin_amdgcn_readfirstlane(((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const long i0 = g * (long)chunk;
  long i1 = i0 + chunk;
  if (i1 > n) i1 = n;
  if (i0 >= i1) return;
  sgd_stream_wide<Q>(rows, cols, vals, 0, 0, LONG_MAX, i0, i1, threadIdx.x & 63, R, W, ldw, H, ldh, lr, lam);
}

// XCD-blocked sub-step (same cell schedule and windows as mf_sgd_xcd_kernel): the 4 waves
// of a block take consecutive streams of CH ratings of the XCD's cell
template <int Q, int CH>
__global__ __launch_bounds__(256) void mf_sgd_xcd_wide_kernel(const int* __restrict__ rows,
                                                              const int* __restrict__ cols,
                                                              const float* __restrict__ vals,
                                                              const long* __restrict__ off,
                                                              const long* __restrict__ win, int step, int R,
                                                              float* __restrict__ W, int ldw, float* __restrict__ H,
                                                              int ldh, float lr, float lam,
                                                              unsigned long long* chk, unsigned long long gen) {
  const int x = blockIdx.x % XCDS;
  const long j = blockIdx.x / XCDS;
  const long per_xcd = gridDim.x / XCDS;
  const int cell = x * XCDS + (x + step) % XCDS;
  const long a = off[cell];
  const long ncell = off[cell + 1] - a;
  const long w0 = win ? win[cell] : 0;
  const long n = win ? win[XCDS * XCDS + cell] : ncell;
  const long nst = (n + CH - 1) / CH;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (long st = j * 4 + wv; st < nst; st += per_xcd * 4) {
    const long i0 = st * CH;
    const long i1 = i0 + CH < n ? i0 + CH : n;
    sgd_stream_wide<Q>(rows, cols, vals, a, w0, ncell, i0, i1, threadIdx.x & 63, R, W, ldw, H, ldh, lr, lam);
  }
  placement_check(chk, gen, x);
}

template <int Q>
__global__ __launch_bounds__(256) void mf_rmse_wide_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                           const float* __restrict__ vals, long n, int R,
                                                           const float* __restrict__ W, int ldw,
                                                           const float* __restrict__ H, int ldh,
                                                           double* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  double acc = 0.0;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nw) {
    floatx4 w[Q], h[Q];
    load_wide<Q, false>(W + (long)rows[i] * ldw, lane, R, w);
    load_wide<Q, false>(H + (long)cols[i] * ldh, lane, R, h);
    float d = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q)
      d += w[q][0] * h[q][0] + w[q][1] * h[q][1] + w[q][2] * h[q][2] + w[q][3] * h[q][3];
    const float e = vals[i] - wave_sum_f(d);
    acc += (double)e * e;
  }
  double s = lane == 0 ? acc : 0.0;
  s = wave_sum_d(s);
  __shared__ double red[4];
  if (lane == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

int wide_q(int r) { return r <= 512 ? 2 : r <= 1024 ? 4 : r <= 2048 ? 8 : 16; }
bool wide_ok(int r) { return r > 256 && r <= 4096 && r % 4 == 0; }

#define WIDE_DISPATCH(R, CALL)                                                          \
  switch (wide_q(R)) {                                                                  \
    case 2: return CALL(2);                                                             \
    case 4: return CALL(4);                                                             \
    case 8: return CALL(8);                                                             \
    default: return CALL(16);                                                           \
  }

template <int Q>
int launch_sgd_wide(const int* rows, const int* cols, const float* vals, long n, int chunk, int r, float* W, int ldw,
                    float* H, int ldh, float lr, float lam, hipStream_t s) {
  const long streams = (n + chunk - 1) / chunk;
  const long blocks = (streams + 3) / 4;
  mf_sgd_wide_kernel<Q><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(rows, cols, vals, n, chunk, r, W, ldw, H, ldh,
                                                                      lr, lam);
  return harp_launch_status();
}

template <int Q>
int launch_sgd_xcd_wide(const int* rows, const int* cols, const float* vals, const long* off, const long* win,
                        int steps, int chunk, int blocks_per_xcd, int r, float* W, int ldw, float* H, int ldh,
                        float lr, float lam, unsigned long long* chk, unsigned long long gen0, hipStream_t s) {
  for (int step = 0; step < steps; ++step) {
    const unsigned long long gen = gen0 + (unsigned long long)step;
    if (chunk == 32)
      mf_sgd_xcd_wide_kernel<Q, 32><<<dim3((unsigned)(blocks_per_xcd * XCDS)), dim3(256), 0, s>>>(
          rows, cols, vals, off, win, step, r, W, ldw, H, ldh, lr, lam, chk, gen);
    else if (chunk == 128)
      mf_sgd_xcd_wide_kernel<Q, 128><<<dim3((unsigned)(blocks_per_xcd * XCDS)), dim3(256), 0, s>>>(
          rows, cols, vals, off, win, step, r, W, ldw, H, ldh, lr, lam, chk, gen);
    else
      mf_sgd_xcd_wide_kernel<Q, 64><<<dim3((unsigned)(blocks_per_xcd * XCDS)), dim3(256), 0, s>>>(
          rows, cols, vals, off, win, step, r, W, ldw, H, ldh, lr, lam, chk, gen);
    const int st = harp_launch_status();
    if (st != HARP_OK) return st;
  }
  return HARP_OK;
}

template <int Q>
int launch_rmse_wide(const int* rows, const int* cols, const float* vals, long n, int r, const float* W, int ldw,
                     const float* H, int ldh, double* partial, int nblocks, hipStream_t s) {
  mf_rmse_wide_kernel<Q><<<dim3(nblocks), dim3(256), 0, s>>>(rows, cols, vals, n, r, W, ldw, H, ldh, partial);
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
  if (wide_ok(r)) {
#define SGDW_CALL(QQ) launch_sgd_wide<QQ>(rows, cols, vals, n, chunk, r, W, ldw, H, ldh, lr, lam, s)
    WIDE_DISPATCH(r, SGDW_CALL)
#undef SGDW_CALL
  }
#define SGD_CALL(RR) launch_sgd<RR>(rows, cols, vals, n, chunk, W, ldw, H, ldh, lr, lam, s)
  MF_DISPATCH(r, SGD_CALL)
#undef SGD_CALL
}

HARP_EXPORT int harp_mf_xcds() { return XCDS; }

// All `steps` (= 8) sub-steps of the XCD-blocked schedule over one resident slice: `off`
// is a DEVICE array of 65 int64 cell offsets into rows/cols/vals (every cell < 2^31 ratings).
// `chunk` (ratings per stream and round) is 8, 16, 32, 64 or 128 (32..128 for wide ranks);
// `variant`: 0 = blockIdx-placed sub-steps, checked when `chk` (harp_mf_chk_words() zeroed
// uint64 per stream) is given: launch generations gen .. gen + steps - 1 (> 0, never reused
// on that chk); 2 = the placement-independent kernel (`pws`: harp_mf_placed_ws_ints()
// zeroed int32, left zeroed; ranks <= 256); + 4 / + 8 (kAtomBits, ranks <= 256): the ATOM
// write-back of W / of H (changes added with L2 atomics, no lost updates). Non-temporal H stores (23 % slower) and forced
// 6 / 7 / 8 waves per SIMD were measured in round 1 and are no longer built.
// `win`: optional DEVICE array [2 x 64] of per-cell window starts and lengths (NULL = all).
HARP_EXPORT int harp_mf_chk_words() { return kChkWords; }
HARP_EXPORT int harp_mf_placed_ws_ints() { return kPlacedWs; }

HARP_EXPORT int harp_mf_sgd_xcd(const int* rows, const int* cols, const float* vals, const long* off, const long* win,
                                int r, int steps, int chunk, int blocks_per_xcd, int variant, float* W, int ldw,
                                float* H, int ldh, float lr, float lam, unsigned long long* chk,
                                unsigned long long gen, int* pws, hipStream_t s) {
  const int base_variant = variant & ~kAtomBits;
  if (blocks_per_xcd <= 0 || steps <= 0 || steps > XCDS || ldw < r || ldh < r || (base_variant != 0 && base_variant != 2))
    return HARP_EBADARG;
  if ((chk && gen == 0) || (base_variant == 2 && (!pws || wide_ok(r))) || ((variant & kAtomBits) && wide_ok(r)))
    return HARP_EBADARG;
  if (wide_ok(r)) {  // wide ranks: one wave per stream
    if (chunk != 32 && chunk != 64 && chunk != 128) return HARP_EBADARG;
#define SGDXW_CALL(QQ) \
  launch_sgd_xcd_wide<QQ>(rows, cols, vals, off, win, steps, chunk, blocks_per_xcd, r, W, ldw, H, ldh, lr, lam, chk, \
                          gen, s)
    WIDE_DISPATCH(r, SGDXW_CALL)
#undef SGDXW_CALL
  }
#define SGDX_ARGS rows, cols, vals, off, win, steps, blocks_per_xcd, W, ldw, H, ldh, lr, lam, variant, chk, gen, pws, s
#define SGDX_CALL(RR)                                                             \
  (chunk == 8 ? launch_sgd_xcd<RR, 8>(SGDX_ARGS)                                    \
   : chunk == 16 ? launch_sgd_xcd<RR, 16>(SGDX_ARGS)                                \
   : chunk == 32 ? launch_sgd_xcd<RR, 32>(SGDX_ARGS)                                \
   : chunk == 64 ? launch_sgd_xcd<RR, 64>(SGDX_ARGS)                                \
   : chunk == 128 ? launch_sgd_xcd<RR, 128>(SGDX_ARGS)                              \
                  : HARP_EBADARG)
  MF_DISPATCH(r, SGDX_CALL)
#undef SGDX_CALL
#undef SGDX_ARGS
}

// One launch for all `steps` sub-steps (mf_sgd_xcd_flow_kernel); same arguments as
// harp_mf_sgd_xcd plus `ws`, a zeroed device int32 workspace of harp_mf_flow_ws_ints()
// entries private to the stream (left zeroed again by the launch; ws[193] != 0 afterwards
// means a wait timed out). Ranks <= 256 only.
HARP_EXPORT int harp_mf_flow_ws_ints() { return kFlowWs; }

HARP_EXPORT int harp_mf_sgd_xcd_flow(const int* rows, const int* cols, const float* vals, const long* off,
                                     const long* win, int r, int steps, int chunk, int blocks_per_xcd, float* W,
                                     int ldw, float* H, int ldh, float lr, float lam, int* ws, hipStream_t s) {
  if (blocks_per_xcd <= 0 || steps <= 0 || steps > XCDS || ldw < r || ldh < r || wide_ok(r) || !ws)
    return HARP_EBADARG;
#define SGDF_ARGS rows, cols, vals, off, win, steps, blocks_per_xcd, W, ldw, H, ldh, lr, lam, ws, s
#define SGDF_CALL(RR)                                                                  \
  (chunk == 8 ? launch_sgd_xcd_flow<RR, 8>(SGDF_ARGS)                                   \
   : chunk == 16 ? launch_sgd_xcd_flow<RR, 16>(SGDF_ARGS)                               \
   : chunk == 32 ? launch_sgd_xcd_flow<RR, 32>(SGDF_ARGS)                               \
   : chunk == 64 ? launch_sgd_xcd_flow<RR, 64>(SGDF_ARGS)                               \
   : chunk == 128 ? launch_sgd_xcd_flow<RR, 128>(SGDF_ARGS)                             \
                  : HARP_EBADARG)
  MF_DISPATCH(r, SGDF_CALL)
#undef SGDF_CALL
#undef SGDF_ARGS
}

HARP_EXPORT int harp_mf_rmse_blocks() { return 1024; }

HARP_EXPORT int harp_mf_rmse(const int* rows, const int* cols, const float* vals, long n, int r, const float* W, int ldw,
                             const float* H, int ldh, double* partial, hipStream_t s) {
  if (n <= 0) return HARP_OK;
  if (wide_ok(r)) {
#define RMSEW_CALL(QQ) launch_rmse_wide<QQ>(rows, cols, vals, n, r, W, ldw, H, ldh, partial, 1024, s)
    WIDE_DISPATCH(r, RMSEW_CALL)
#undef RMSEW_CALL
  }
#define RMSE_CALL(RR) launch_rmse<RR>(rows, cols, vals, n, W, ldw, H, ldh, partial, 1024, s)
  MF_DISPATCH(r, RMSE_CALL)
#undef RMSE_CALL
}
