// SYRK partial G += X^T X on MFMA (bf16 in, fp32 accumulate/out) for gfx950.
//
// The step-1 partial of covariance / low-order moments / correlation PCA / normal-equation
// regression (DAAL DistributedStep1Local: ml/daal/.../daal_cov/densedistri/
// COVDaalCollectiveMapper.java:146-175, daal_pca/cordensedistr/PCADaalCollectiveMapper.java:
// 121-147, daal_linreg/normaleq). N = 1e8 x d = 1000 is ~1e14 MFMA FLOP per pass.
//
// Design (MI355X-first):
//  * data is stored FEATURE-MAJOR in 48-sample blocks, XT[ld/48][d_pad][48]: for
//    G = XT XT^T both MFMA operands want 8 consecutive samples of one feature per lane,
//    which is then a plain 16-B read — no transposes anywhere — and one stage's MT x 48
//    operand panel is ONE contiguous MT*96-B run. (A flat [d_pad][ld] layout puts the
//    panel's rows ld*2 = 200 MB apart at N = 1e8: every stage then touches 256-512
//    distinct pages and the loads are address-translation bound, not L2 bound.) A row of
//    ones in XT makes G's last column the column sums and G[ones][ones] = n, so moments
//    come out of the same pass.
//  * only upper-triangular MT x MT output tiles are computed (diagonal tiles in pairs, see
//    syrk_kernel); the sample dimension is split over workgroups (split-K), each workgroup
//    adds its fp32 tile into G with contiguous 128-B atomic row segments.
//  * per 48-sample stage both operand panels stream through a 3-deep LDS ring by
//    global_load_lds (LDS-DMA) -- 2 x 3 x 24 KB = 144 KB of the 160 KB for 256-feature
//    panels -- so a stage's loads are issued two stages ahead, with counted vmcnt waits and
//    raw s_barriers (a __syncthreads() would drain the ring). A 64-sample stage fits only
//    two buffers, one stage of look-ahead, and measured 0.106 s vs the MFMA-only 0.069 s
//    (profiles/r2_syrk2). The 96-B LDS rows (6 chunks of 16 B) are rotated by one chunk for
//    rows 16-31 of every 32-row block: conflict-free for ds_read_b128's lane groups
//    (exhaustive search over the 6-chunk rotations; the rotation is applied on the DMA
//    source side, the LDS image stays lane-linear). 8 waves, each a 64x128 sub-tile =
//    2x4 accumulators of v_mfma_f32_32x32x16_bf16.
#include "common.h"

namespace {

constexpr int KT = 48;        // samples per stage (= the layout's sample block)
constexpr int CPR = KT / 8;   // 16-B chunks per LDS row (6)
constexpr int NBUF = 3;       // LDS ring depth

// LDS position of logical 16-B chunk c of panel row `row`, and its inverse
__device__ __forceinline__ int swz_pos(int row, int c) { return (c + ((row >> 4) & 1)) % CPR; }
__device__ __forceinline__ int swz_src(int row, int cp) { return (cp + (CPR - ((row >> 4) & 1))) % CPR; }

// Workgroup geometry: MT x MT output tile; each wave owns (32*BA) x (32*BB).
template <int MT_, int BA_, int BB_>
struct SyrkCfg {
  static constexpr int MT = MT_, BA = BA_, BB = BB_;
  static constexpr int WR = MT / (32 * BA), WC = MT / (32 * BB);
  static constexpr int WAVES = WR * WC;
  static constexpr int PANEL_BYTES = MT * KT * 2;
  static constexpr int DMA = PANEL_BYTES / 1024;
};

// one MT x 48 panel of XT (features r0.., sample block k0/48 of d_pad x 48) -> LDS via LDS-DMA
template <class C>
__device__ __forceinline__ void stage_panel(const __bf16* __restrict__ XT, long d_pad, int r0, long k0, char* lds,
                                            int wave, int lane) {
  const __bf16* blk = XT + k0 * d_pad + (long)r0 * KT;  // k0 % KT == 0: the block's panel is contiguous
#pragma unroll
  for (int j = wave; j < C::DMA; j += C::WAVES) {
    const int q = j * 64 + lane;          // chunk position in the LDS image
    const int row = q / CPR, cp = q % CPR;
    const int c = swz_src(row, cp);       // source chunk for this position
    const __bf16* src = blk + row * KT + c * 8;
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)(lds + j * 1024), 16, 0, 0);
  }
}

// MFMA fragment of 32-row block `blk` of a staged panel: lane (r, h) reads row blk*32 + r,
// 16-B chunk kc = 2*kstep + h. swz_pos(blk*32 + r, kc) does not depend on blk, so `lo` =
// r*96 + (swz_pos(r, kc) << 4) is per lane and k-step, and the block is an immediate offset.
__device__ __forceinline__ int frag_off(int r, int kc) { return r * (CPR * 16) + (swz_pos(r, kc) << 4); }
__device__ __forceinline__ bf16x8 frag(const char* P, int blk, int lo) {
  return *(const bf16x8*)(P + blk * (32 * CPR * 16) + lo);
}

// DIAG (timing diagnostics only, results are garbage): 1 = no global loads after the first
// stage (MFMA + LDS + barriers), 2 = no MFMA (loads + LDS reads + a VALU use of the
// fragments), 3 = loads + barriers only, 4 = every stage loads the first stage's (L2-hot)
// samples (same instruction stream, no L2 misses), 5 = off-diagonal tiles only (pairs exit),
// 6 = diagonal pairs only
template <int DIAG>
__device__ __forceinline__ void mma(const bf16x8& a, const bf16x8& b, floatx16& c) {
  if constexpr (DIAG == 2) c[0] += (float)a[0] * (float)b[7];
  else c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Upper triangle of one diagonal MT x MT panel product, shared by NB/2 waves: wave W owns
// 32-block rows W and NB-1-W (NB+1 blocks each: equal work), and since G = XT XT^T a block
// row's A fragment IS that block's B fragment, so it reads only the NB-W fragments of
// blocks W..NB-1 per k-step. acc[j]: j < NB-W -> (W, W+j), else (NB-1-W, NB-1-W+j-(NB-W)).
template <int NB, int W, int DIAG>
__device__ __forceinline__ void tri_step(const char* P, int lo, floatx16* acc) {
  bf16x8 f[NB - W];
#pragma unroll
  for (int c = W; c < NB; ++c) f[c - W] = frag(P, c, lo);
#pragma unroll
  for (int c = W; c < NB; ++c) mma<DIAG>(f[0], f[c - W], acc[c - W]);
#pragma unroll
  for (int c = NB - 1 - W; c < NB; ++c) mma<DIAG>(f[NB - 1 - 2 * W], f[c - W], acc[NB - W + c - (NB - 1 - W)]);
}

struct SyrkJob {
  const __bf16* XT;
  long dpad, kbeg, kend, split;
  int ti, tj, ntiles, ldg, sync_every;
  bool one, second;
  float* G;
  int* sync;
};

// The k-loop + epilogue of one work item. MODE < 0: an off-diagonal tile or a lone diagonal
// tile (B == A), every wave a (32BA) x (32BB) block; MODE = W >= 0: a diagonal pair, the
// wave's row pair W (tri_step) of panel ti (waves < NB/2) or tj. One body per mode, so the
// register allocator sees one accumulator assignment per loop (two alternative MFMA paths
// in one loop body made it copy the accumulators between them and spill).
template <class C, int MODE, int DIAG>
__device__ __forceinline__ void syrk_body(const SyrkJob& J, char* smem, int tid) {
  constexpr int MT = C::MT, BA = C::BA, BB = C::BB, PANEL = C::PANEL_BYTES, NB = MT / 32;
  constexpr int NACC = MODE < 0 ? BA * BB : NB + 1;
  const int lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int wr = wave / C::WC, wc = wave % C::WC;
  floatx16 acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[j][v] = 0.f;

  // ring: stage i in A = smem + (i%3)*PANEL, B = smem + (3 + i%3)*PANEL
  static_assert(C::DMA == 3 * C::WAVES, "3 LDS-DMA pieces per wave per panel (the vmcnt counts below)");
  const int nst = (int)((J.kend - J.kbeg) / KT);
  auto issue = [&](int st) {
    const long k = DIAG == 4 ? J.kbeg : J.kbeg + (long)st * KT;  // DIAG 4: re-read the first (L2-hot)
    const int bf = st % NBUF;
    stage_panel<C>(J.XT, J.dpad, J.ti * MT, k, smem + bf * PANEL, wave, lane);
    if (!J.one) stage_panel<C>(J.XT, J.dpad, J.tj * MT, k, smem + (NBUF + bf) * PANEL, wave, lane);
  };
  issue(0);
  if (DIAG != 1 && nst > 1) issue(1);
  for (int i = 0; i < nst; ++i) {
    // this wave's DMA of stage i landed (stage i+1's, issued later, may stay in flight) ...
    if (DIAG != 1 && i + 1 < nst) {
      if (J.one) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // ... then every wave's, and every wave is done reading stage i-1 (whose buffer stage
    // i+2 reuses): raw barrier, no vmcnt drain
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (J.sync && i > 0 && i % J.sync_every == 0) {
      // soft lock-step of the split's tiles (they share feature panels through this XCD's
      // L2 only while they stream the same samples): every sync_every stages, arrive on the
      // split's counter and wait -- boundedly, so progress never depends on it -- until
      // every tile of the split has arrived. Correctness does not depend on the wait.
      if (tid == 0) {
        int* c = J.sync + J.split;
        atomicAdd(c, 1);
        const int target = J.ntiles * (i / J.sync_every);
        for (int it = 0; it < 2000; ++it) {
          if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
          __builtin_amdgcn_s_sleep(4);
        }
      }
      __syncthreads();
    }
    if (DIAG != 1 && i + 2 < nst) issue(i + 2);
    const int bf = i % NBUF;
    const char* A = smem + bf * PANEL;
    const char* B = J.one ? A : smem + (NBUF + bf) * PANEL;
    if constexpr (DIAG != 3 && MODE >= 0) {
      const char* P = J.second ? B : A;
#pragma unroll
      for (int s = 0; s < KT / 16; ++s) tri_step<NB, (MODE >= 0 ? MODE : 0), DIAG>(P, frag_off(r, 2 * s + h), acc);
    } else if constexpr (DIAG != 3) {
#pragma unroll
      for (int s = 0; s < KT / 16; ++s) {
        bf16x8 af[BA], bfr[BB];
#pragma unroll
        for (int a = 0; a < BA; ++a) af[a] = frag(A, wr * BA + a, frag_off(r, 2 * s + h));
#pragma unroll
        for (int bb = 0; bb < BB; ++bb) bfr[bb] = frag(B, wc * BB + bb, frag_off(r, 2 * s + h));
#pragma unroll
        for (int a = 0; a < BA; ++a)
#pragma unroll
          for (int bb = 0; bb < BB; ++bb) mma<DIAG>(af[a], bfr[bb], acc[a * BB + bb]);
      }
    }
  }
  // D[i][j]: lane holds col = lane&31, rows (v&3) + 8*(v>>2) + 4h of each 32x32 block
  if constexpr (MODE >= 0) {
    constexpr int W = MODE, LO = NB - W;  // LO blocks in row W, then W+1 in row NB-1-W
    const int base = (J.second ? J.tj : J.ti) * MT;
#pragma unroll
    for (int j = 0; j < NB + 1; ++j) {
      const int rb = j < LO ? W : NB - 1 - W;
      const int cb = j < LO ? W + j : NB - 1 - W + (j - LO);
      const int i0 = base + rb * 32, j0 = base + cb * 32;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = (v & 3) + 8 * (v >> 2) + 4 * h;
        atomicAdd(J.G + (long)(i0 + row) * J.ldg + j0 + r, acc[j][v]);
      }
    }
  } else {
#pragma unroll
    for (int a = 0; a < BA; ++a)
#pragma unroll
      for (int bb = 0; bb < BB; ++bb) {
        const int i0 = J.ti * MT + wr * (32 * BA) + a * 32;
        const int j0 = J.tj * MT + wc * (32 * BB) + bb * 32;
        if (J.one && i0 > j0 + 31) continue;  // strictly-lower block of a diagonal tile: unused
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int row = (v & 3) + 8 * (v >> 2) + 4 * h;
          atomicAdd(J.G + (long)(i0 + row) * J.ldg + j0 + r, acc[a * BB + bb][v]);
        }
      }
  }
}

// Work items per sample split: every off-diagonal MT-tile (two panels, full product) and
// the diagonal tiles in PAIRS (two panels, two upper triangles: NB+1 of NB*NB blocks per
// wave, so a pair costs a full tile's loads and ~1.1x its MFMAs); an odd last diagonal
// tile runs alone (one panel, full product). d_pad = 1024, MT = 256: 6 + 2 = 8 workgroups
// per split (was 10 with lone diagonal tiles at half load), 32 splits fill all 256 CUs.
template <int MT_, int BA_, int BB_, int DIAG = 0>
__global__ __launch_bounds__((MT_ / (32 * BA_)) * (MT_ / (32 * BB_)) * 64) void syrk_kernel(
    const __bf16* __restrict__ XT, long n, int nt, long chunk, float* __restrict__ G, int ldg,
    int* __restrict__ sync, int sync_every) {
  using C = SyrkCfg<MT_, BA_, BB_>;
  constexpr int MT = C::MT, PANEL = C::PANEL_BYTES, NB = MT / 32;
  static_assert(C::WAVES == NB && (NB == 4 || NB == 8), "diagonal pairs: NB/2 waves per panel");
  __shared__ __attribute__((aligned(16))) char smem[2 * NBUF * PANEL];
  const int tid = threadIdx.x, wave = tid >> 6;
  // XCD-aware remap (bijective): consecutive logical ids share an XCD (blocks b, b+8, ...
  // are co-located), so the tiles of one sample split hit the same L2
  const unsigned nb = gridDim.x, b = blockIdx.x;
  const unsigned q8 = nb / 8, r8 = nb % 8, xcd = b % 8;
  const unsigned L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
  SyrkJob J;
  const int noff = nt * (nt - 1) / 2;
  J.ntiles = noff + (nt + 1) / 2;
  const int tile = L % J.ntiles;
  J.split = L / J.ntiles;
  if (tile < noff) {
    int rem = tile, ti = 0;
    while (rem >= nt - 1 - ti) { rem -= nt - 1 - ti; ++ti; }
    J.ti = ti;
    J.tj = ti + 1 + rem;
  } else {
    J.ti = 2 * (tile - noff);
    J.tj = J.ti + 1 < nt ? J.ti + 1 : J.ti;
  }
  const bool pair = tile >= noff && J.tj != J.ti;  // two diagonal panels, triangles only
  J.one = J.ti == J.tj;                            // a lone diagonal tile: one panel, full product
  J.kbeg = J.split * chunk;
  J.kend = J.kbeg + chunk < n ? J.kbeg + chunk : n;
  if (J.kbeg >= J.kend) return;
  J.XT = XT;
  J.dpad = (long)nt * MT;
  J.G = G;
  J.ldg = ldg;
  J.sync = sync;
  J.sync_every = sync_every;
  J.second = wave >= NB / 2;
  if constexpr (DIAG == 6) {  // diagnostics: diagonal pairs only
    if (!pair) return;
  }
  if (!pair) return syrk_body<C, -1, DIAG>(J, smem, tid);
  if constexpr (DIAG == 5) return;  // diagnostics: off-diagonal tiles only
  switch (wave % (NB / 2)) {  // wave-uniform
    case 0: return syrk_body<C, 0, DIAG>(J, smem, tid);
    case 1: return syrk_body<C, 1, DIAG>(J, smem, tid);
    case 2: if constexpr (NB == 8) return syrk_body<C, 2, DIAG>(J, smem, tid); return;
    default: if constexpr (NB == 8) return syrk_body<C, 3, DIAG>(J, smem, tid); return;
  }
}

// row-major X[n][d] (bf16/any) -> blocked feature-major XT[ld/48][d_pad][48] bf16 with a
// ones row at index d (tiled transpose through LDS).
__global__ void to_feature_major_kernel(const __bf16* __restrict__ X, long n, int d, long ldx,
                                        __bf16* __restrict__ XT, long ld, int d_pad, int ones_row) {
  __shared__ __bf16 tile[32][33];
  const long k0 = (long)blockIdx.x * 32;
  const int f0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int yy = ty; yy < 32; yy += 8) {
    const long k = k0 + yy;
    const int f = f0 + tx;
    __bf16 v = (__bf16)0.f;
    if (k < n) {
      if (f < d) v = X[k * ldx + f];
      else if (f == ones_row) v = (__bf16)1.f;
    }
    tile[yy][tx] = v;
  }
  __syncthreads();
  for (int yy = ty; yy < 32; yy += 8) {
    const int f = f0 + yy;
    const long k = k0 + tx;
    if (k < ld) XT[(k - k % KT) * d_pad + (long)f * KT + k % KT] = tile[tx][yy];
  }
}

}  // namespace

template <int MT, int BA, int BB, int DIAG = 0>
static int launch_syrk(const void* XT, long ld, long n, int d_pad, float* G, int ldg, int num_splits, int target_wg,
                       hipStream_t s, int* sync_ws = nullptr, int sync_every = 0) {
  using C = SyrkCfg<MT, BA, BB>;
  const int nt = d_pad / MT;
  const int ntiles = nt * (nt - 1) / 2 + (nt + 1) / 2;  // off-diagonal tiles + diagonal pairs
  if (num_splits <= 0) {
    // co-resident grid: every XCD runs whole splits (all ntiles tiles of one sample range at
    // once, so the 2-4 tiles reading a feature panel share it in that XCD's L2) and every
    // workgroup starts in the first wave -- no split straddles dispatch waves. 256 x 256
    // tiles, d_pad = 1024: 32 splits x (6 off-diagonal tiles + 2 diagonal pairs) = 256
    // workgroups, one per CU. (Lone diagonal tiles: 24 x 10 = 240 workgroups, 0.143 s vs
    // 0.150 s for the ~1030-workgroup split-K grid, 0.122 s with the split lock-step hint:
    // L2 hit 49 % -> 71 %, the 75 % ceiling of 4 tiles per panel; profiles/r2_syrk.)
    const int per_xcd = 32 * (MT >= 256 ? 1 : 2);  // one 256-tile (144 KB) / two 128-tile (72 KB) WGs per CU
    if (ntiles <= per_xcd) {
      num_splits = 8 * (per_xcd / ntiles);
    } else {
      // about target_wg workgroups, rounded so the grid fills whole rounds of the 256 CUs
      const int s0 = (target_wg + ntiles - 1) / ntiles;
      num_splits = s0;
      double best = 0.0;
      for (int sp = s0; sp <= 2 * s0; ++sp) {
        const long B = (long)ntiles * sp;
        const double eff = (double)B / (double)(((B + 255) / 256) * 256);
        if (eff > best + 1e-9) { best = eff; num_splits = sp; }
        if (eff > 0.999) break;
      }
    }
    const long min_chunk = 64L * KT;  // keep >= 64 stages per workgroup on small inputs
    while (num_splits > 1 && (n + num_splits - 1) / num_splits < min_chunk) num_splits /= 2;
  }
  long chunk = (n + num_splits - 1) / num_splits;
  chunk = (chunk + KT - 1) / KT * KT;
  const long splits = (n + chunk - 1) / chunk;
  {
    // the lock-step hint only pays when every tile of a split is resident at once
    int* sw = (sync_ws && sync_every > 0 && ntiles * splits <= 256 && splits <= 1024) ? sync_ws : nullptr;
    if (sw && hipMemsetAsync(sw, 0, sizeof(int) * splits, s) != hipSuccess) return HARP_ELAUNCH;
    syrk_kernel<MT, BA, BB, DIAG><<<dim3((unsigned)(ntiles * splits)), dim3(C::WAVES * 64), 0, s>>>(
        (const __bf16*)XT, n, nt, chunk, G, ldg, sw, sync_every);
  }
  return harp_launch_status();
}

// G[d_pad][ldg] (+)= XT XT^T over the upper tiles; XT [ld/48][d_pad][48] bf16 (blocked
// feature-major), d_pad % 128 == 0, n % 48 == 0 (zero-padded samples), ld >= n, ld % 48 == 0.
// 256x256 tiles (8 waves) when d_pad % 256 == 0 and d_pad >= 512 (half the operand re-reads),
// else 128x128 (4 waves).
// variant 0 (the only one): 48-sample stages, 3-deep LDS-DMA ring. sync_ws (>= 1024 ints, may be null) + sync_every (stages, 0 = off):
// the split lock-step hint of the 256-tile kernel (see syrk_kernel).
HARP_EXPORT int harp_syrk_t_bf16(const void* XT, long ld, long n, int d_pad, float* G, int ldg, int num_splits,
                                 int variant, int* sync_ws, int sync_every, hipStream_t s) {
  if (d_pad % 128 || n % KT || ld < n || ld % KT || ldg < d_pad) return HARP_EBADARG;
  if (n == 0) return HARP_OK;
  const bool big = d_pad >= 512 && d_pad % 256 == 0;
  if (variant != 0) return HARP_EBADARG;
  if (big) return launch_syrk<256, 2, 4>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s, sync_ws, sync_every);
  return launch_syrk<128, 2, 2>(XT, ld, n, d_pad, G, ldg, num_splits, 2048, s);
}

HARP_EXPORT int harp_to_feature_major_bf16(const void* X, long n, int d, long ldx, void* XT, long ld, int d_pad,
                                           int ones_row, hipStream_t s) {
  if (ld < n || ld % KT || d_pad < d || d_pad % 32) return HARP_EBADARG;
  dim3 grid((unsigned)((ld + 31) / 32), (unsigned)(d_pad / 32));
  to_feature_major_kernel<<<grid, dim3(256), 0, s>>>((const __bf16*)X, n, d, ldx, (__bf16*)XT, ld, d_pad, ones_row);
  return harp_launch_status();
}

// Timing diagnostics of the default kernel (see DIAG above; G receives garbage).
HARP_EXPORT int harp_syrk_diag(const void* XT, long ld, long n, int d_pad, float* G, int ldg, int num_splits, int mode,
                               hipStream_t s) {
  if (d_pad % 256 || d_pad < 512 || n % KT || ld < n || ld % KT || ldg < d_pad) return HARP_EBADARG;
  switch (mode) {
    case 0: return launch_syrk<256, 2, 4, 0>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s);
    case 1: return launch_syrk<256, 2, 4, 1>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s);
    case 2: return launch_syrk<256, 2, 4, 2>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s);
    case 3: return launch_syrk<256, 2, 4, 3>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s);
    case 4: return launch_syrk<256, 2, 4, 4>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s);
    case 5: return launch_syrk<256, 2, 4, 5>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s);
    case 6: return launch_syrk<256, 2, 4, 6>(XT, ld, n, d_pad, G, ldg, num_splits, 1024, s);
    default: return HARP_EBADARG;
  }
}
