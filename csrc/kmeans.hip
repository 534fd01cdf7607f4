// K-means kernels for gfx950 (MI355X / CDNA4).
//
// Replaces the reference's K-means E-step + accumulate hot loop
// (ml/java/.../kmeans/regroupallgather/CenCalcTask.java:67-100: per point, argmin
// over all centroids of the squared L2 distance, then local[c] += (1, x)) and the
// thread merge (CenMergeTask.java:36-54) and the owner-side average
// (KMeansCollectiveMapper.java:170-183).
//
// Design (MI355X-first, not a translation):
//  * distances are a GEMM: X[N,dp] (bf16) x (-2C)[Kp,dp]^T on v_mfma_f32_32x32x16_bf16.
//    ||c||^2 is folded INTO the GEMM: X carries 1.0 in columns d..d+3 and -2C carries
//    0, hi, mid, lo there (||c||^2 = hi + mid + lo in three bf16 terms, ~24-bit exact), so
//    the zero-initialised accumulator IS the distance minus ||x||^2 and the epilogue is a
//    pure argmin (no row-constant registers, no norm reads from LDS). d=100 pads to 112,
//    the same K as without the fold.
//  * centroids sit on the MFMA row axis, points on the lane (column) axis: each lane
//    owns one point and 16 candidate centroids per 32x32 tile, so the argmin is
//    register-local (16 keyed fminf -> v_min3) plus one lane<->lane+32 exchange.
//    The within-tile register index is packed into the 4 low mantissa bits of the
//    distance (relative perturbation 2^-19, far below the bf16 operand rounding).
//  * X fragments stay in VGPRs for the whole centroid sweep; centroid tiles stream
//    through double-buffered LDS filled by global_load_lds (LDS-DMA, no staging VGPRs)
//    with a per-row chunk rotation applied to the DMA source so ds_read_b128 stays
//    conflict-free; A fragments are register double-buffered across 32-row groups; one
//    barrier per stage.
//  * column d of X (1.0) meets column d of -2C (0): the accumulation adds (x, 1) =
//    (partial sum, count) in one row: the Harp centroid row layout (sum + count) falls out
//    of the data layout.
//  * accumulation: per assigned point, one 256-B contiguous f32 atomic row segment
//    per wave-instruction (the full-rate atomic shape on gfx950).
#include "common.h"

#include <type_traits>

namespace {

constexpr float KM_BIG = 1.0e38f;
constexpr int KM_ONES = 4;  // X columns d..d+3 hold 1.0: count + the 3 folded ||c||^2 terms

__device__ __forceinline__ float keyed(float v, unsigned idx) {
  return __uint_as_float((__float_as_uint(v) & ~0xFu) | idx);
}

template <int KS, int G, int WAVES_, int RG>
struct KMCfg {
  static constexpr int DP = KS * 16;                 // padded feature dim (elements)
  static constexpr int CPR = KS * 2;                 // 16-byte chunks per row
  static constexpr int TILE = RG * 32;               // centroids per stage
  static constexpr int WAVES = WAVES_;
  static constexpr int THREADS = WAVES_ * 64;
  static constexpr int TILE_BYTES = TILE * DP * 2;
  static constexpr int DMA_INSTR = TILE * CPR / 64;  // 1-KiB LDS-DMA wave-instructions per tile
  static constexpr int PTS = WAVES_ * G * 32;        // points per workgroup
  static_assert((TILE * CPR) % 64 == 0, "tile must be whole 1-KiB DMA pieces");
};

// LDS image of a centroid tile: row-major [TILE][CPR] 16-B chunks, chunk c of row r stored at
// position (c + s(r)) mod CPR with s(r) = (r >> 3) & 1. Rows r and r+8 then sit on different
// 16-B bank slots, so every ds_read_b128 lane group (16 distinct rows) is conflict-free, while
// the image stays lane-linear for global_load_lds (the swizzle is applied to the SOURCE).
template <class C>
__device__ __forceinline__ void stage_dma(const __bf16* __restrict__ cm2, int tile, char* lds, int wave, int lane) {
#pragma unroll
  for (int j0 = 0; j0 < C::DMA_INSTR; j0 += C::WAVES) {
    const int j = j0 + wave;
    if (C::DMA_INSTR % C::WAVES == 0 || j < C::DMA_INSTR) {
      const int q = j * 64 + lane;
      const int row = q / C::CPR;
      int c = q - row * C::CPR - ((row >> 3) & 1);
      if (c < 0) c += C::CPR;
      const __bf16* src = cm2 + ((size_t)tile * C::TILE + row) * C::DP + c * 8;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)(lds + j * 1024), 16, 0, 0);
    }
  }
}

template <int KS, int G, int WAVES, int RG, int PIPE, int PRIO = 0>
__global__ __launch_bounds__(WAVES * 64) void kmeans_assign_kernel(
    const __bf16* __restrict__ X, long ldx, const __bf16* __restrict__ Cm2, long N, int ntiles, int tail_rg,
    int dcount, int* __restrict__ labels, float* __restrict__ sums, int ld_sums, float* __restrict__ obj_partial,
    float* __restrict__ mind) {
  using C = KMCfg<KS, G, WAVES, RG>;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::TILE_BYTES + WAVES * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int srot = (r >> 3) & 1;
  const long pbase = ((long)blockIdx.x * WAVES + wave) * (G * 32);

  // PRIO (variant 15): static VALU-arbitration priority for the younger half of the
  // workgroup, set once (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if constexpr (PRIO)
    if (__builtin_amdgcn_readfirstlane(tid) >= WAVES * 32) __builtin_amdgcn_s_setprio(1);
  // kick off the first centroid tile before loading this wave's points
  stage_dma<C>(Cm2, 0, smem, wave, lane);

  // ---- this wave's points: B-operand fragments, resident for the whole sweep
  bf16x8 xf[G][KS];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    long p = pbase + g * 32 + r;
    if (p > N - 1) p = N - 1;
    const bf16x8* row = (const bf16x8*)(X + p * ldx);
#pragma unroll
    for (int s = 0; s < KS; ++s) xf[g][s] = row[2 * s + h];
  }

  float best[G];
  int bestt[G];
#pragma unroll
  for (int g = 0; g < G; ++g) { best[g] = KM_BIG; bestt[g] = 0; }
  // argmin of one 32x32 tile into (best, bestt)[g]: the 16 candidates' register index rides
  // in the low mantissa bits (one v_and_or per candidate). A plain v_min3 with the index
  // searched only on improvement measured 5 % slower (it spills; profiles/r2_ktail).
  auto tile_argmin = [&](const floatx16& ac, int g, int tg) {
    float m = keyed(ac[0], 0u);
#pragma unroll
    for (int q = 1; q < 16; ++q) m = fminf(m, keyed(ac[q], (unsigned)q));
    if (m < best[g]) { best[g] = m; bestt[g] = tg; }
  };

  // per-lane byte offsets of its A-fragment chunks inside a 32-row group
  int aoff[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    int cp = 2 * s + h + srot;
    if (cp >= C::CPR) cp -= C::CPR;
    aoff[s] = (r * C::CPR + cp) * 16;
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // full tiles; a last tile of only tail_rg (< RG) row groups runs after the loop
  const int nfull = tail_rg ? ntiles - 1 : ntiles;
  for (int t = 0; t < nfull; ++t) {
    if (t + 1 < ntiles) stage_dma<C>(Cm2, t + 1, smem + ((t + 1) & 1) * C::TILE_BYTES, wave, lane);
    const char* buf = smem + (t & 1) * C::TILE_BYTES;
    bf16x8 af[2][KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) af[0][s] = *(const bf16x8*)(buf + aoff[s]);
    if constexpr (PIPE > 0) {
      // software pipeline over the stage's RG*G (row group, point group) items: the MFMA
      // chain of item i+1 is issued before the argmin epilogue of item i, so the epilogue's
      // VALU work fills the MFMA gaps instead of waiting on the chain's tail latency
      constexpr int NI = RG * G;
      floatx16 acc[2];
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[0][q] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][s], xf[0][s], acc[0], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int rg = i / G, g = i % G;
        if (g == 0 && rg + 1 < RG) {
          const char* nb = buf + (rg + 1) * 32 * C::CPR * 16;
#pragma unroll
          for (int s = 0; s < KS; ++s) af[(rg + 1) & 1][s] = *(const bf16x8*)(nb + aoff[s]);
        }
        if (i + 1 < NI) {
          const int rg1 = (i + 1) / G, g1 = (i + 1) % G;
          floatx16& an = acc[(i + 1) & 1];
#pragma unroll
          for (int q = 0; q < 16; ++q) an[q] = 0.f;
#pragma unroll
          for (int s = 0; s < KS; ++s) an = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[rg1 & 1][s], xf[g1][s], an, 0, 0, 0);
        }
        tile_argmin(acc[i & 1], g, t * RG + rg);
        if constexpr (PIPE == 2) {
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // then up to 4 VALU
          }
        }
      }
    } else
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
      if (rg + 1 < RG) {
        const char* nb = buf + (rg + 1) * 32 * C::CPR * 16;
#pragma unroll
        for (int s = 0; s < KS; ++s) af[(rg + 1) & 1][s] = *(const bf16x8*)(nb + aoff[s]);
      }
      const int tg = t * RG + rg;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        floatx16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[rg & 1][s], xf[g][s], acc, 0, 0, 0);
        tile_argmin(acc, g, tg);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (tail_rg) {
    // K not a multiple of the stage: only the live 32-row groups of the last tile (its DMA
    // landed with the previous stage's wait + barrier; the rows past them are never read)
    const int t = ntiles - 1;
    const char* buf = smem + (t & 1) * C::TILE_BYTES;
    for (int rg = 0; rg < tail_rg; ++rg) {
      const char* nb = buf + rg * 32 * C::CPR * 16;
      bf16x8 af[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) af[s] = *(const bf16x8*)(nb + aoff[s]);
      const int tg = t * RG + rg;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        floatx16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], xf[g][s], acc, 0, 0, 0);
        tile_argmin(acc, g, tg);
      }
    }
  }

  // ---- resolve argmin across the two lane halves, write labels / objective partials
  int lab[G];
  float local_obj = 0.f;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float xs = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = (float)xf[g][s][j];
        xs = fmaf(v, v, xs);
      }
    xs += __shfl_xor(xs, 32, 64);
    xs -= (float)KM_ONES;  // the 1.0 columns of X
    const float ob = __shfl_xor(best[g], 32, 64);
    const int obt = __shfl_xor(bestt[g], 32, 64);
    const bool take = h ? (ob <= best[g]) : (ob < best[g]);
    const float bv = take ? ob : best[g];
    const int bt = take ? obt : bestt[g];
    const int hw = take ? (1 - h) : h;
    const unsigned reg = __float_as_uint(bv) & 0xFu;
    const int idx = bt * 32 + (int)(reg & 3u) + 8 * (int)(reg >> 2) + 4 * hw;
    lab[g] = idx;
    const long p = pbase + g * 32 + r;
    if (h == 0 && p < N) {
      labels[p] = idx;
      local_obj += fmaxf(bv + xs, 0.f);
      if (mind) mind[p] = bv + xs;  // squared distance to the chosen centroid (rotation merge)
    }
  }
  if (obj_partial) {
    local_obj = wave_sum(local_obj);
    float* red = (float*)(smem + 2 * C::TILE_BYTES);
    if (lane == 0) red[wave] = local_obj;
    __syncthreads();
    if (tid == 0) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) acc += red[w];
      obj_partial[blockIdx.x] = acc;
    }
  }

  // ---- accumulate (x, 1) rows into the per-centroid partial sums
  if (sums) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      for (int i = 0; i < 32; ++i) {
        const long p = pbase + g * 32 + i;
        if (p >= N) break;
        const int l = __shfl(lab[g], i, 64);
        const __bf16* xr = X + p * ldx;
        float* sr = sums + (long)l * ld_sums;
        for (int c = lane; c <= dcount; c += 64) atomicAdd(sr + c, (float)xr[c]);
      }
    }
  }
}

// sums[Kr][ld] (column d = count) -> c[Kr][d]; empty clusters keep their old centroid.
__global__ void kmeans_normalize_kernel(const float* __restrict__ sums, int ld, float* __restrict__ c,
                                        int Kr, int d, float* __restrict__ counts) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= Kr) return;
  const float cnt = sums[(long)row * ld + d];
  if (counts && lane == 0) counts[row] = cnt;
  if (cnt > 0.f) {
    const float inv = 1.0f / cnt;
    for (int j = lane; j < d; j += 64) c[(long)row * d + j] = sums[(long)row * ld + j] * inv;
  }
}

// c[K][d] fp32 -> Cm2[Kp][dp]: cols [0,d) = -2*bf16(c), col d = 0 (count column of X),
// cols d+1..d+3 = ||bf16(c)||^2 split into three bf16 terms (hi + mid + lo ~ 24-bit exact),
// rest 0; cn[Kp] = ||bf16(c)||^2 in fp32. Padding rows: distance +BIG.
__global__ void kmeans_prepare_kernel(const float* __restrict__ c, int K, int d, int Kp, int dp,
                                      __bf16* __restrict__ Cm2, float* __restrict__ cn) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= Kp) return;
  float s = 0.f;
  for (int j = lane; j < d; j += 64) {
    float v = row < K ? c[(long)row * d + j] : 0.f;
    const float bf = (float)(__bf16)v;
    s = fmaf(bf, bf, s);
    Cm2[(long)row * dp + j] = (__bf16)(-2.0f * bf);
  }
  s = wave_sum(s);
  if (row >= K) s = KM_BIG;
  const __bf16 hi = (__bf16)s;
  const float r1 = s - (float)hi;
  const __bf16 mid = (__bf16)r1;
  const __bf16 lo = (__bf16)(r1 - (float)mid);
  for (int j = d + lane; j < dp; j += 64) {
    __bf16 v = (__bf16)0.f;
    if (j == d + 1) v = hi;
    else if (j == d + 2) v = mid;
    else if (j == d + 3) v = lo;
    Cm2[(long)row * dp + j] = v;
  }
  if (lane == 0) cn[row] = s;
}

// Counter-based uniform generator (splitmix64 of the element index): device-side
// synthetic points like the reference's DataGenRunnable (U[lo,hi)), no host copy.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void uniform_rows_bf16_kernel(__bf16* __restrict__ X, long N, int d, int dp, float lo,
                                         float hi, unsigned long long seed, long row0, int one_col) {
  const long total = N * (long)dp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long row = i / dp;
    const int col = (int)(i - row * dp);
    float v = 0.f;
    if (col < d) {
      const unsigned long long z = splitmix64(seed ^ ((unsigned long long)(row0 + row) * 0x100000001B3ull + col));
      v = lo + (hi - lo) * (float)((z >> 40) * (1.0 / 16777216.0));
    } else if (one_col && col < d + KM_ONES) {
      v = 1.0f;
    }
    X[i] = (__bf16)v;
  }
}

// ---------------------------------------------------------------------------------------
// Wide rows (dp > 256, any d up to the operand's padding): X fragments no longer fit the
// register file for a whole centroid sweep, so the reduction over features is staged:
//  * a workgroup (4 waves, 64 points per wave = 2 MFMA point groups) owns 256 points and ONE
//    block of 256 centroids (8 row groups of 32); its 16 accumulators (256 fp32 per lane)
//    stay live across the feature stages;
//  * feature stage f covers dp columns [64 f, 64 f + 64): the centroid block's 256 x 64 bf16
//    slice streams through double-buffered LDS by LDS-DMA (the swizzled image of the
//    narrow kernel), the points' 64-column slices are register double-buffered straight
//    from global (next stage's loads in flight under this stage's 64 MFMAs per wave);
//  * the epilogue is the narrow kernel's keyed argmin over the block's 256 candidates, the
//    workgroup's result (squared distance, index) is merged across centroid blocks with ONE
//    64-bit atomic min per point (distance bits above the index: non-negative floats order
//    as integers, ties go to the lower index);
//  * grid: consecutive ids of one XCD (id mod 8) take the centroid blocks of one point block
//    one after another, so that block's rows come from HBM once and from L2 after.
constexpr int KW_CB = 256, KW_RG = KW_CB / 32;  // centroids per workgroup (8 row groups of 32)

// G point groups of 32 per wave (4 waves), DC features per stage, OCC waves per SIMD
template <int G, int DC>
struct KWCfg {
  static constexpr int KS = DC / 16;                  // MFMA k-steps per stage
  static constexpr int CPR = DC / 8;                  // 16-B chunks per centroid row per stage
  static constexpr int TILE_BYTES = KW_CB * DC * 2;
  static constexpr int DMA = KW_CB * CPR / 64;        // 1-KiB DMA pieces per stage
  static constexpr int PTS = 4 * G * 32;              // points per workgroup
};

// LDS chunk rotation of centroid row `row` for the wide tiles: ds_read_b128 serves 16 lanes
// (rows r..r+15 of one 16-B chunk column) per LDS cycle, so their 16 addresses must fall on
// 16 distinct 16-B slots of a 256-B bank row. With 128-B rows (CPR 8) rows r and r + 2
// alias, so the rotation walks r >> 1; with 256-B rows (CPR 16) every row aliases, so it
// walks r.
template <int CPR>
__device__ __forceinline__ int wide_rot(int row) {
  return CPR == 4 ? (row >> 2) & 3 : CPR == 8 ? (row >> 1) & 7 : CPR == 16 ? row & 15 : (row >> 3) & 1;
}

template <class C>
__device__ __forceinline__ void stage_dma_wide(const __bf16* __restrict__ cm2, int dp, int row0, int kp, int f,
                                               char* lds, int wave, int lane) {
#pragma unroll
  for (int j0 = 0; j0 < C::DMA; j0 += 4) {
    const int j = j0 + wave;
    const int q = j * 64 + lane;
    const int row = q / C::CPR;
    int c = q - row * C::CPR - wide_rot<C::CPR>(row);
    if (c < 0) c += C::CPR;
    int gr = row0 + row;
    if (gr > kp - 1) gr = kp - 1;  // past the padded rows: a valid address, never read
    const __bf16* src = cm2 + (size_t)gr * dp + f * (C::CPR * 8) + c * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)(lds + j * 1024), 16, 0, 0);
  }
}

template <int G, int DC, int OCC>
__global__ __launch_bounds__(256, OCC) void kmeans_assign_wide_kernel(
    const __bf16* __restrict__ X, long ldx, const __bf16* __restrict__ Cm2, long N, int dp, int kswept, int kp,
    int nkb, unsigned long long* __restrict__ keys) {
  using C = KWCfg<G, DC>;
  constexpr int KS = C::KS;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::TILE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int srot = (r >> 3) & 1;
  // XCD-aware id -> (point block, centroid block): ids x, x + 8, x + 16, ... (one XCD) walk
  // the nkb centroid blocks of one point block before the next
  const long id = blockIdx.x;
  const long xcd = id & 7, round = id >> 3;
  const long pb = (round / nkb) * 8 + xcd;
  const int kb = (int)(round % nkb);
  const long npb = (N + C::PTS - 1) / C::PTS;
  if (pb >= npb) return;
  const int row0 = kb * KW_CB;
  const int live_rg = (kswept - row0) >= KW_CB ? KW_RG : (kswept - row0 + 31) / 32;
  const long pbase = pb * C::PTS + wave * (G * 32);
  const int nst = dp / DC;

  stage_dma_wide<C>(Cm2, dp, row0, kp, 0, smem, wave, lane);
  const bf16x8* xrow[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    long p = pbase + g * 32 + r;
    if (p > N - 1) p = N - 1;
    xrow[g] = (const bf16x8*)(X + p * ldx);
  }
  bf16x8 xf[2][G][KS];  // [buffer][point group][k-step]
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int k = 0; k < KS; ++k) xf[0][g][k] = xrow[g][2 * k + h];
  floatx16 acc[KW_RG][G];
#pragma unroll
  for (int a = 0; a < KW_RG; ++a)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][g][q] = 0.f;
  int aoff[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int cp = (2 * k + h + wide_rot<C::CPR>(r)) % C::CPR;
    aoff[k] = (r * C::CPR + cp) * 16;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // one feature stage; the register buffer index is a template constant (a runtime index
  // into xf would put the fragments in scratch)
  auto stage = [&](int f, auto curtag) {
    constexpr int cur = decltype(curtag)::value;
    if (f + 1 < nst) {
      stage_dma_wide<C>(Cm2, dp, row0, kp, f + 1, smem + (cur ^ 1) * C::TILE_BYTES, wave, lane);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int k = 0; k < KS; ++k) xf[cur ^ 1][g][k] = xrow[g][(f + 1) * C::CPR + 2 * k + h];
    }
    const char* buf = smem + cur * C::TILE_BYTES;
    bf16x8 af[2][KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) af[0][k] = *(const bf16x8*)(buf + aoff[k]);
#pragma unroll
    for (int rg = 0; rg < KW_RG; ++rg) {
      if (rg + 1 < KW_RG) {
        const char* nb = buf + (rg + 1) * 32 * C::CPR * 16;
#pragma unroll
        for (int k = 0; k < KS; ++k) af[(rg + 1) & 1][k] = *(const bf16x8*)(nb + aoff[k]);
      }
      if (rg < live_rg) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
          for (int k = 0; k < KS; ++k)
            acc[rg][g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[rg & 1][k], xf[cur][g][k], acc[rg][g], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int f = 0; f < nst; f += 2) {
    stage(f, std::integral_constant<int, 0>{});
    if (f + 1 < nst) stage(f + 1, std::integral_constant<int, 1>{});
  }
  // |x|^2 per point group, from global once after the sweep (L2-warm rows)
  float xsg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float t = 0.f;
    for (int c = h; c < dp / 8; c += 2) {
      const bf16x8 v = xrow[g][c];
#pragma unroll
      for (int j = 0; j < 8; ++j) t = fmaf((float)v[j], (float)v[j], t);
    }
    t += __shfl_xor(t, 32, 64);
    xsg[g] = t - (float)KM_ONES;
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float best = KM_BIG;
    int bestt = 0;
#pragma unroll
    for (int rg = 0; rg < KW_RG; ++rg) {
      if (rg >= live_rg) break;
      float m = keyed(acc[rg][g][0], 0u);
#pragma unroll
      for (int q = 1; q < 16; ++q) m = fminf(m, keyed(acc[rg][g][q], (unsigned)q));
      if (m < best) {
        best = m;
        bestt = rg;
      }
    }
    const float ob = __shfl_xor(best, 32, 64);
    const int obt = __shfl_xor(bestt, 32, 64);
    const bool take = h ? (ob <= best) : (ob < best);
    const float bv = take ? ob : best;
    const int bt = take ? obt : bestt;
    const int hw = take ? (1 - h) : h;
    const unsigned reg = __float_as_uint(bv) & 0xFu;
    const int idx = row0 + bt * 32 + (int)(reg & 3u) + 8 * (int)(reg >> 2) + 4 * hw;
    const long p = pbase + g * 32 + r;
    if (h == 0 && p < N) {
      const float dist = fmaxf(bv + xsg[g], 0.f);
      const unsigned long long key = ((unsigned long long)__float_as_uint(dist) << 32) | (unsigned)idx;
      __hip_atomic_fetch_min(keys + p, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int G, int DC, int NBUF>
__global__ __launch_bounds__(256, 1) void kmeans_assign_wide_lds_kernel(
    const __bf16* __restrict__ X, long ldx, const __bf16* __restrict__ Cm2, long N, int dp, int kswept, int kp,
    int nkb, unsigned long long* __restrict__ keys) {
  using C = KWCfg<G, DC>;
  constexpr int KS = C::KS, CPR = C::CPR;
  constexpr int XROWS = 4 * G * 32;                  // points per workgroup
  constexpr int XBYTES = XROWS * DC * 2;             // point slice per stage
  constexpr int SBYTES = C::TILE_BYTES + XBYTES;     // one ring slot
  constexpr int XDMA = XROWS * CPR / 64;             // 1-KiB pieces of the point slice
  constexpr int OPS = C::DMA / 4 + XDMA / 4;         // DMA instructions per wave per stage
  static_assert(C::DMA % 4 == 0 && XDMA % 4 == 0, "whole pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const long id = blockIdx.x;
  const long xcd = id & 7, round = id >> 3;
  const long pb = (round / nkb) * 8 + xcd;
  const int kb = (int)(round % nkb);
  const long npb = (N + XROWS - 1) / XROWS;
  if (pb >= npb) return;
  const int row0 = kb * KW_CB;
  const int live_rg = (kswept - row0) >= KW_CB ? KW_RG : (kswept - row0 + 31) / 32;
  const long p0 = pb * XROWS;  // first point of the workgroup
  const long pbase = p0 + wave * (G * 32);
  const int nst = dp / DC;
  auto issue = [&](int f, int slot) {
    char* buf = smem + slot * SBYTES;
    stage_dma_wide<C>(Cm2, dp, row0, kp, f, buf, wave, lane);
    char* xb = buf + C::TILE_BYTES;
#pragma unroll
    for (int j0 = 0; j0 < XDMA; j0 += 4) {
      const int j = j0 + wave;
      const int q = j * 64 + lane;
      const int row = q / CPR;
      int c = q - row * CPR - wide_rot<CPR>(row);
      if (c < 0) c += CPR;
      long pr = p0 + row;
      if (pr > N - 1) pr = N - 1;
      const __bf16* src = X + pr * ldx + f * DC + c * 8;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)(xb + j * 1024), 16, 0, 0);
    }
  };
  floatx16 acc[KW_RG][G];
#pragma unroll
  for (int a = 0; a < KW_RG; ++a)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][g][q] = 0.f;
  int aoff[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) aoff[k] = (r * CPR + (2 * k + h + wide_rot<CPR>(r)) % CPR) * 16;
#pragma unroll
  for (int q = 0; q < NBUF - 1; ++q)
    if (q < nst) issue(q, q);
  float xs[G];
#pragma unroll
  for (int g = 0; g < G; ++g) xs[g] = 0.f;
  for (int f = 0; f < nst; ++f) {
    // stage f landed when at most the younger stages' pieces are outstanding
    const int younger = (nst - 1 - f) < (NBUF - 2) ? (nst - 1 - f) : (NBUF - 2);
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * OPS) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (f + NBUF - 1 < nst) issue(f + NBUF - 1, (f + NBUF - 1) % NBUF);
    const char* buf = smem + (f % NBUF) * SBYTES;
    const char* xb = buf + C::TILE_BYTES + wave * (G * 32) * CPR * 16;
    bf16x8 xf[G][KS];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int k = 0; k < KS; ++k) xf[g][k] = *(const bf16x8*)(xb + g * 32 * CPR * 16 + aoff[k]);
    // |x|^2 from the staged fragments (VALU work under the stage's MFMAs)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) xs[g] = fmaf((float)xf[g][k][j], (float)xf[g][k][j], xs[g]);
    bf16x8 af[2][KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) af[0][k] = *(const bf16x8*)(buf + aoff[k]);
#pragma unroll
    for (int rg = 0; rg < KW_RG; ++rg) {
      if (rg + 1 < KW_RG) {
        const char* nb = buf + (rg + 1) * 32 * CPR * 16;
#pragma unroll
        for (int k = 0; k < KS; ++k) af[(rg + 1) & 1][k] = *(const bf16x8*)(nb + aoff[k]);
      }
      if (rg < live_rg) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
          for (int k = 0; k < KS; ++k)
            acc[rg][g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[rg & 1][k], xf[g][k], acc[rg][g], 0, 0, 0);
      }
    }
  }
  float xsg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) xsg[g] = xs[g] + __shfl_xor(xs[g], 32, 64) - (float)KM_ONES;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float best = KM_BIG;
    int bestt = 0;
#pragma unroll
    for (int rg = 0; rg < KW_RG; ++rg) {
      if (rg >= live_rg) break;
      float m = keyed(acc[rg][g][0], 0u);
#pragma unroll
      for (int q = 1; q < 16; ++q) m = fminf(m, keyed(acc[rg][g][q], (unsigned)q));
      if (m < best) {
        best = m;
        bestt = rg;
      }
    }
    const float ob = __shfl_xor(best, 32, 64);
    const int obt = __shfl_xor(bestt, 32, 64);
    const bool take = h ? (ob <= best) : (ob < best);
    const float bv = take ? ob : best;
    const int bt = take ? obt : bestt;
    const int hw = take ? (1 - h) : h;
    const unsigned reg = __float_as_uint(bv) & 0xFu;
    const int idx = row0 + bt * 32 + (int)(reg & 3u) + 8 * (int)(reg >> 2) + 4 * hw;
    const long p = pbase + g * 32 + r;
    if (h == 0 && p < N) {
      const float dist = fmaxf(bv + xsg[g], 0.f);
      const unsigned long long key = ((unsigned long long)__float_as_uint(dist) << 32) | (unsigned)idx;
      __hip_atomic_fetch_min(keys + p, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// 8 waves (2 per SIMD) on the same 256 x 256 tile: wave w takes centroid half w & 1 and
// point quarter w >> 1 (4 x 2 accumulators), so each SIMD has a second wave to issue while
// one waits (the 4-wave form parks 44 % of its cycles on instruction dependencies)
template <int C_DMA8, class C>
__device__ __forceinline__ void stage_dma_wide8(const __bf16* __restrict__ cm2, int dp, int row0, int kp, int f,
                                                char* lds, int wave, int lane) {
#pragma unroll
  for (int j0 = 0; j0 < C::DMA; j0 += 8) {
    const int j = j0 + wave;
    const int q = j * 64 + lane;
    const int row = q / C::CPR;
    int c = q - row * C::CPR - wide_rot<C::CPR>(row);
    if (c < 0) c += C::CPR;
    int gr = row0 + row;
    if (gr > kp - 1) gr = kp - 1;
    const __bf16* src = cm2 + (size_t)gr * dp + f * (C::CPR * 8) + c * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)(lds + j * 1024), 16, 0, 0);
  }
}

template <int G, int DC, int NBUF>
__global__ __launch_bounds__(512, 1) void kmeans_assign_wide8_kernel(
    const __bf16* __restrict__ X, long ldx, const __bf16* __restrict__ Cm2, long N, int dp, int kswept, int kp,
    int nkb, unsigned long long* __restrict__ keys) {
  using C = KWCfg<G, DC>;
  constexpr int KS = C::KS, CPR = C::CPR;
  constexpr int XROWS = 4 * G * 32;                  // points per workgroup (256 at G = 2)
  constexpr int RGW = KW_RG / 2, GW = G;             // per wave: 4 centroid groups x G point groups
  constexpr int XBYTES = XROWS * DC * 2;             // point slice per stage
  constexpr int SBYTES = C::TILE_BYTES + XBYTES;     // one ring slot
  constexpr int XDMA = XROWS * CPR / 64;             // 1-KiB pieces of the point slice
  constexpr int OPS = C::DMA / 8 + XDMA / 8;         // DMA instructions per wave per stage
  static_assert(C::DMA % 8 == 0 && XDMA % 8 == 0, "whole pieces per wave");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int rgo = (wave & 1) * RGW;                  // first centroid group of this wave
  const int pwo = (wave >> 1) * (GW * 32);           // first point of this wave in the block
  const long id = blockIdx.x;
  const long xcd = id & 7, round = id >> 3;
  const long pb = (round / nkb) * 8 + xcd;
  const int kb = (int)(round % nkb);
  const long npb = (N + XROWS - 1) / XROWS;
  if (pb >= npb) return;
  const int row0 = kb * KW_CB;
  const int live_blk = (kswept - row0) >= KW_CB ? KW_RG : (kswept - row0 + 31) / 32;
  const int live_rg = live_blk - rgo < 0 ? 0 : (live_blk - rgo > RGW ? RGW : live_blk - rgo);
  const long p0 = pb * XROWS;  // first point of the workgroup
  const long pbase = p0 + pwo;
  const int nst = dp / DC;
  auto issue = [&](int f, int slot) {
    char* buf = smem + slot * SBYTES;
    stage_dma_wide8<0, C>(Cm2, dp, row0, kp, f, buf, wave, lane);
    char* xb = buf + C::TILE_BYTES;
#pragma unroll
    for (int j0 = 0; j0 < XDMA; j0 += 8) {
      const int j = j0 + wave;
      const int q = j * 64 + lane;
      const int row = q / CPR;
      int c = q - row * CPR - wide_rot<CPR>(row);
      if (c < 0) c += CPR;
      long pr = p0 + row;
      if (pr > N - 1) pr = N - 1;
      const __bf16* src = X + pr * ldx + f * DC + c * 8;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)(xb + j * 1024), 16, 0, 0);
    }
  };
  floatx16 acc[RGW][G];
#pragma unroll
  for (int a = 0; a < RGW; ++a)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][g][q] = 0.f;
  int aoff[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) aoff[k] = (r * CPR + (2 * k + h + wide_rot<CPR>(r)) % CPR) * 16;
#pragma unroll
  for (int q = 0; q < NBUF - 1; ++q)
    if (q < nst) issue(q, q);
  float xs[G];
#pragma unroll
  for (int g = 0; g < G; ++g) xs[g] = 0.f;
  for (int f = 0; f < nst; ++f) {
    // stage f landed when at most the younger stages' pieces are outstanding
    const int younger = (nst - 1 - f) < (NBUF - 2) ? (nst - 1 - f) : (NBUF - 2);
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * OPS) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (f + NBUF - 1 < nst) issue(f + NBUF - 1, (f + NBUF - 1) % NBUF);
    const char* buf = smem + (f % NBUF) * SBYTES;
    const char* xb = buf + C::TILE_BYTES + pwo * CPR * 16;
    const char* cb = buf + rgo * 32 * CPR * 16;
    bf16x8 xf[G][KS];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int k = 0; k < KS; ++k) xf[g][k] = *(const bf16x8*)(xb + g * 32 * CPR * 16 + aoff[k]);
    // |x|^2 from the staged fragments (VALU work under the stage's MFMAs)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) xs[g] = fmaf((float)xf[g][k][j], (float)xf[g][k][j], xs[g]);
    bf16x8 af[2][KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) af[0][k] = *(const bf16x8*)(cb + aoff[k]);
#pragma unroll
    for (int rg = 0; rg < RGW; ++rg) {
      if (rg + 1 < RGW) {
        const char* nb = cb + (rg + 1) * 32 * CPR * 16;
#pragma unroll
        for (int k = 0; k < KS; ++k) af[(rg + 1) & 1][k] = *(const bf16x8*)(nb + aoff[k]);
      }
      if (rg < live_rg) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
          for (int k = 0; k < KS; ++k)
            acc[rg][g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[rg & 1][k], xf[g][k], acc[rg][g], 0, 0, 0);
      }
    }
  }
  float xsg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) xsg[g] = xs[g] + __shfl_xor(xs[g], 32, 64) - (float)KM_ONES;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float best = KM_BIG;
    int bestt = 0;
#pragma unroll
    for (int rg = 0; rg < RGW; ++rg) {
      if (rg >= live_rg) break;
      float m = keyed(acc[rg][g][0], 0u);
#pragma unroll
      for (int q = 1; q < 16; ++q) m = fminf(m, keyed(acc[rg][g][q], (unsigned)q));
      if (m < best) {
        best = m;
        bestt = rg;
      }
    }
    const float ob = __shfl_xor(best, 32, 64);
    const int obt = __shfl_xor(bestt, 32, 64);
    const bool take = h ? (ob <= best) : (ob < best);
    const float bv = take ? ob : best;
    const int bt = take ? obt : bestt;
    const int hw = take ? (1 - h) : h;
    const unsigned reg = __float_as_uint(bv) & 0xFu;
    const int idx = row0 + (rgo + bt) * 32 + (int)(reg & 3u) + 8 * (int)(reg >> 2) + 4 * hw;
    const long p = pbase + g * 32 + r;
    if (h == 0 && p < N && live_rg > 0) {
      const float dist = fmaxf(bv + xsg[g], 0.f);
      const unsigned long long key = ((unsigned long long)__float_as_uint(dist) << 32) | (unsigned)idx;
      __hip_atomic_fetch_min(keys + p, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int G, int DC, int NBUF>
int launch_wide8(const void* X, long ldx, const void* Cm2, long N, int dp, int kswept, int kp,
                 unsigned long long* keys, hipStream_t s) {
  constexpr int XROWS = 4 * G * 32;
  if (dp % DC || (ldx * 2) % 16) return HARP_EBADARG;
  const long npb = (N + XROWS - 1) / XROWS;
  const int nkb = (kswept + KW_CB - 1) / KW_CB;
  const long rounds = (npb + 7) / 8 * nkb;
  kmeans_assign_wide8_kernel<G, DC, NBUF><<<dim3((unsigned)(rounds * 8)), dim3(512), 0, s>>>(
      (const __bf16*)X, ldx, (const __bf16*)Cm2, N, dp, kswept, kp, nkb, keys);
  return harp_launch_status();
}

template <int G, int DC, int NBUF>
int launch_wide_lds(const void* X, long ldx, const void* Cm2, long N, int dp, int kswept, int kp,
                    unsigned long long* keys, hipStream_t s) {
  constexpr int XROWS = 4 * G * 32;
  constexpr int SBYTES = KW_CB * DC * 2 + XROWS * DC * 2;
  if (dp % DC || (ldx * 2) % 16) return HARP_EBADARG;
  const long npb = (N + XROWS - 1) / XROWS;
  const int nkb = (kswept + KW_CB - 1) / KW_CB;
  const long rounds = (npb + 7) / 8 * nkb;
  (void)SBYTES;
  kmeans_assign_wide_lds_kernel<G, DC, NBUF><<<dim3((unsigned)(rounds * 8)), dim3(256), 0, s>>>(
      (const __bf16*)X, ldx, (const __bf16*)Cm2, N, dp, kswept, kp, nkb, keys);
  return harp_launch_status();
}

template <int G, int DC, int OCC>
int launch_wide(const void* X, long ldx, const void* Cm2, long N, int dp, int kswept, int kp,
                unsigned long long* keys, hipStream_t s) {
  using C = KWCfg<G, DC>;
  if (dp % DC) return HARP_EBADARG;
  const long npb = (N + C::PTS - 1) / C::PTS;
  const int nkb = (kswept + KW_CB - 1) / KW_CB;
  const long rounds = (npb + 7) / 8 * nkb;
  kmeans_assign_wide_kernel<G, DC, OCC><<<dim3((unsigned)(rounds * 8)), dim3(256), 0, s>>>(
      (const __bf16*)X, ldx, (const __bf16*)Cm2, N, dp, kswept, kp, nkb, keys);
  return harp_launch_status();
}

// keys -> labels, squared distances, per-block objective partials (256 points per block)
__global__ __launch_bounds__(256) void kmeans_wide_finish_kernel(const unsigned long long* __restrict__ keys, long N,
                                                                 int* __restrict__ labels, float* __restrict__ obj_partial,
                                                                 float* __restrict__ mind) {
  __shared__ float red[4];
  const long p = blockIdx.x * 256L + threadIdx.x;
  float v = 0.f;
  if (p < N) {
    const unsigned long long k = keys[p];
    labels[p] = (int)(k & 0xffffffffull);
    v = __uint_as_float((unsigned)(k >> 32));
    if (mind) mind[p] = v;
  }
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0 && obj_partial) obj_partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

template <int KS, int G, int WAVES, int RG, int PIPE = 0, int PRIO = 0>
int launch_assign(const void* X, long ldx, const void* Cm2, long N, int Kp, int d, int* labels, float* sums,
                  int ld_sums, float* obj_partial, float* mind, hipStream_t stream) {
  using C = KMCfg<KS, G, WAVES, RG>;
  if (Kp % 32) return HARP_EBADARG;
  const long nblk = (N + C::PTS - 1) / C::PTS;
  const int ntiles = (Kp + C::TILE - 1) / C::TILE, tail_rg = (Kp % C::TILE) / 32;
  kmeans_assign_kernel<KS, G, WAVES, RG, PIPE, PRIO><<<dim3((unsigned)nblk), dim3(C::THREADS), 0, stream>>>(
      (const __bf16*)X, ldx, (const __bf16*)Cm2, N, ntiles, tail_rg, d, labels, sums, ld_sums, obj_partial, mind);
  return harp_launch_status();
}

// variant -> (G, WAVES, RG, PIPE). Kp (the rows swept) must be a multiple of 32; Cm2 must
// hold round_up(Kp, 128) rows (the last stage's DMA reads the whole tile).
// Only the measured frontier ships (profiles/r1_kmeans_*): 15 (= 14 + static priority for the
// younger half, profiles/r3_setprio) is the default for d <= 124, 13 the RG=2 neighbour of 14,
// 4 the one-group shape wide rows (9..16 k-steps) use.
#define KM_VARIANTS(KS)                                                                       \
  switch (variant) {                                                                        \
    case 4: return launch_assign<KS, 1, 16, 2>(X, ldx, Cm2, N, Kp, d, labels, sums, ld, op, md, s);  \
    case 13: return launch_assign<KS, 4, 8, 2, 2>(X, ldx, Cm2, N, Kp, d, labels, sums, ld, op, md, s); \
    case 14: return launch_assign<KS, 4, 8, 4, 2>(X, ldx, Cm2, N, Kp, d, labels, sums, ld, op, md, s); \
    case 15: return launch_assign<KS, 4, 8, 4, 2, 1>(X, ldx, Cm2, N, Kp, d, labels, sums, ld, op, md, s); \
    default: return HARP_EBADARG;                                                           \
  }

}  // namespace

HARP_EXPORT int harp_kmeans_points_per_block(int variant) {
  switch (variant) {
    case 4: return 16 * 1 * 32;
    case 13: case 14: case 15: return 8 * 4 * 32;
    default: return -1;
  }
}

// X rows of dp (MFMA k) elements at a row stride of ldx >= dp elements (ldx % 8 == 0: 16-B
// aligned rows; a 256-B multiple makes every row whole 128-B lines for the gather-sum).
HARP_EXPORT int harp_kmeans_assign(const void* X, long ldx, const void* Cm2, long N, int dp, int Kp, int d,
                                   int* labels, float* sums, int ld, float* op, float* md, int variant,
                                   hipStream_t s) {
  if (N <= 0 || d + KM_ONES > dp || dp % 16 || Kp <= 0 || Kp % 32 || ldx < dp || ldx % 8) return HARP_EBADARG;
  switch (dp / 16) {
    case 1: KM_VARIANTS(1)
    case 2: KM_VARIANTS(2)
    case 3: KM_VARIANTS(3)
    case 4: KM_VARIANTS(4)
    case 5: KM_VARIANTS(5)
    case 6: KM_VARIANTS(6)
    case 7: KM_VARIANTS(7)
    case 8: KM_VARIANTS(8)
    // wide rows: one 32-point group per wave keeps the X fragments within budget
#define KM_WIDE(KSV) case KSV: return launch_assign<KSV, 1, 16, 2>(X, ldx, Cm2, N, Kp, d, labels, sums, ld, op, md, s);
    KM_WIDE(9) KM_WIDE(10) KM_WIDE(11) KM_WIDE(12) KM_WIDE(13) KM_WIDE(14) KM_WIDE(15) KM_WIDE(16)
#undef KM_WIDE
    default: return HARP_EUNSUPPORTED;
  }
}

// Wide rows (dp > 256, dp % 64 == 0): keys (N uint64, filled with ~0 by the caller) take the
// per-point (distance, index) minimum over all centroid blocks; harp_kmeans_wide_finish then
// writes labels / distances / objective partials (one per 256 points). variant: 0 = 6 (both
// operands through LDS-DMA into a 256 x 256 tile, 8 waves = 2 per SIMD, each 128 centroids x
// 64 points); 5 = the same tile with 4 waves (256 centroids x 64 points each); 1 / 3 =
// point fragments loaded straight into registers (2 groups at 1 wave / SIMD, 1 group at 2).
// Measured at N = 1e7, K = 1e3 (profiles/r4_kwide): d = 1000 6 and 5 both 0.98 PF useful,
// d = 512 6 at 0.86 vs 5 at 0.81 PF; 1 / 3 at 0.56 / 0.61 (waves parked 52-66 % of their
// cycles on 32-row-per-instruction point loads); 128-feature stages, a 3-deep register
// pipeline, 32-feature stages with 3- and 4-deep LDS rings, one group per wave with a 3-deep
// ring, a persistent stage stream across tiles and square 128 x 128 per-wave tiles all
// measured 0.44-0.93 PF and were removed.
HARP_EXPORT int harp_kmeans_assign_wide(const void* X, long ldx, const void* Cm2, long N, int dp, int kswept, int kp,
                                        int d, unsigned long long* keys, int variant, hipStream_t s) {
  if (N <= 0 || d + KM_ONES > dp || dp % 64 || dp <= 0 || kswept <= 0 || kswept % 32 || kp < kswept ||
      ldx < dp || ldx % 8 || !keys)
    return HARP_EBADARG;
  if (variant == 0) variant = 6;
  switch (variant) {
    case 1: return launch_wide<2, 64, 1>(X, ldx, Cm2, N, dp, kswept, kp, keys, s);
    case 3: return launch_wide<1, 64, 2>(X, ldx, Cm2, N, dp, kswept, kp, keys, s);
    case 5: return launch_wide_lds<2, 64, 2>(X, ldx, Cm2, N, dp, kswept, kp, keys, s);
    case 6: return launch_wide8<2, 64, 2>(X, ldx, Cm2, N, dp, kswept, kp, keys, s);
    default: return HARP_EBADARG;
  }
}

HARP_EXPORT int harp_kmeans_wide_finish(const unsigned long long* keys, long N, int* labels, float* obj_partial,
                                        float* mind, hipStream_t s) {
  if (N <= 0) return HARP_OK;
  kmeans_wide_finish_kernel<<<dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s>>>(keys, N, labels, obj_partial, mind);
  return harp_launch_status();
}

HARP_EXPORT int harp_kmeans_normalize(const float* sums, int ld, float* c, int Kr, int d, float* counts,
                                      hipStream_t s) {
  if (Kr <= 0) return HARP_OK;
  const int wpb = 4;
  kmeans_normalize_kernel<<<dim3((Kr + wpb - 1) / wpb), dim3(64 * wpb), 0, s>>>(sums, ld, c, Kr, d, counts);
  return harp_launch_status();
}

HARP_EXPORT int harp_kmeans_prepare(const float* c, int K, int d, int Kp, int dp, void* Cm2, float* cn,
                                    hipStream_t s) {
  if (Kp < K || dp < d) return HARP_EBADARG;
  const int wpb = 4;
  kmeans_prepare_kernel<<<dim3((Kp + wpb - 1) / wpb), dim3(64 * wpb), 0, s>>>(c, K, d, Kp, dp, (__bf16*)Cm2, cn);
  return harp_launch_status();
}

HARP_EXPORT int harp_uniform_rows_bf16(void* X, long N, int d, int dp, float lo, float hi,
                                       unsigned long long seed, long row0, int one_col, hipStream_t s) {
  if (N <= 0) return HARP_OK;
  long blocks = (N * (long)dp + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  uniform_rows_bf16_kernel<<<dim3((unsigned)blocks), dim3(256), 0, s>>>((__bf16*)X, N, d, dp, lo, hi, seed, row0,
                                                                       one_col);
  return harp_launch_status();
}
