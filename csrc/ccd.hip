// MF-CCD coordinate phases for gfx950 (MI355X / CDNA4).
//
// Replaces the reference's CCDMPTask.doRowCCD / doColCCD (ml/java/.../ccd/CCDMPTask.java:67-125)
// and the residual recompute of ResTask: for every owned row r and every latent dimension t,
//   z* = sum_j (res_j + w_rt h_jt) h_jt / (lambda |row| + sum_j h_jt^2),
//   res_j -= (z* - w_rt) h_jt,  w_rt = z*,
// with the other factor fixed.
//
// Design: ONE wave per row (grid-stride). Rows of up to 64*RR nonzeros keep their column
// ids and residuals in VGPRs for the whole t-loop; per t the wave gathers h_jt (the other
// factor is row-major [n][k], so a lane walks one 128-B line per 32 dimensions -> L1/L2
// hits after the first t), forms both sums with DPP wave reductions (no LDS), and one
// lane writes w_rt. Longer rows take the same loop over global residuals. All of a
// phase is one launch (the torch formulation needed ~8 kernels per dimension).
#include "common.h"

namespace {

constexpr int RR = 4;  // register-resident nonzeros per lane

__global__ __launch_bounds__(256) void ccd_phase_kernel(const long* __restrict__ row_ptr, const int* __restrict__ col,
                                                        float* __restrict__ res, int n_rows, float* __restrict__ Fo,
                                                        const float* __restrict__ Fx, int k, float lam,
                                                        int skip_long) {
  const int lane = threadIdx.x & 63;
  const long wave_g = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wave_g; r < n_rows; r += nwaves) {
    const long a = row_ptr[r], b = row_ptr[r + 1];
    const long n = b - a;
    if (n == 0 || (skip_long && n > 64 * RR)) continue;
    float* w = Fo + r * (long)k;
    const float down0 = lam * (float)n;
    if (n <= 64 * RR) {
      int cj[RR];
      float rj[RR];
#pragma unroll
      for (int q = 0; q < RR; ++q) {
        const long j = a + lane + 64 * q;
        cj[q] = j < b ? col[j] : -1;
        rj[q] = j < b ? res[j] : 0.f;
      }
      // dimensions in groups of 4: one 16-B load brings h_{j,t..t+3} (4x fewer gather
      // requests — the phase is bound by them), then 4 sequential coordinate updates
      int t = 0;
      if ((k & 3) == 0) {
        for (; t < k; t += 4) {
          float4 h4[RR];
#pragma unroll
          for (int q = 0; q < RR; ++q)
            h4[q] = cj[q] >= 0 ? *(const float4*)(Fx + (long)cj[q] * k + t) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 w4 = *(const float4*)(w + t);
          float wn[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            float up = 0.f, dn = 0.f;
#pragma unroll
            for (int q = 0; q < RR; ++q) {
              const float h = tt == 0 ? h4[q].x : tt == 1 ? h4[q].y : tt == 2 ? h4[q].z : h4[q].w;
              up = fmaf(fmaf(wn[tt], h, rj[q]), h, up);
              dn = fmaf(h, h, dn);
            }
            up = wave_total(up);
            dn = wave_total(dn) + down0;
            const float z = dn > 0.f ? up / dn : wn[tt];
            const float delta = z - wn[tt];
#pragma unroll
            for (int q = 0; q < RR; ++q) {
              const float h = tt == 0 ? h4[q].x : tt == 1 ? h4[q].y : tt == 2 ? h4[q].z : h4[q].w;
              rj[q] = fmaf(-delta, h, rj[q]);
            }
            wn[tt] = z;
          }
          if (lane == 0) *(float4*)(w + t) = make_float4(wn[0], wn[1], wn[2], wn[3]);
        }
      }
      for (; t < k; ++t) {
        const float wt = w[t];
        float hv[RR];
        float up = 0.f, dn = 0.f;
#pragma unroll
        for (int q = 0; q < RR; ++q) {
          hv[q] = cj[q] >= 0 ? Fx[(long)cj[q] * k + t] : 0.f;
          up = fmaf(fmaf(wt, hv[q], rj[q]), hv[q], up);
          dn = fmaf(hv[q], hv[q], dn);
        }
        up = wave_total(up);
        dn = wave_total(dn) + down0;
        const float z = dn > 0.f ? up / dn : wt;
        const float delta = z - wt;
#pragma unroll
        for (int q = 0; q < RR; ++q) rj[q] = fmaf(-delta, hv[q], rj[q]);
        if (lane == 0) w[t] = z;
      }
#pragma unroll
      for (int q = 0; q < RR; ++q) {
        const long j = a + lane + 64 * q;
        if (j < b) res[j] = rj[q];
      }
    } else {
      for (int t = 0; t < k; ++t) {
        const float wt = w[t];
        float up = 0.f, dn = 0.f;
        for (long j = a + lane; j < b; j += 64) {
          const float h = Fx[(long)col[j] * k + t];
          up = fmaf(fmaf(wt, h, res[j]), h, up);
          dn = fmaf(h, h, dn);
        }
        up = wave_total(up);
        dn = wave_total(dn) + down0;
        const float z = dn > 0.f ? up / dn : wt;
        const float delta = z - wt;
        for (long j = a + lane; j < b; j += 64) res[j] = fmaf(-delta, Fx[(long)col[j] * k + t], res[j]);
        if (lane == 0) w[t] = z;
      }
    }
  }
}

// Medium rows (64*RR < n <= BT*RB nonzeros: most items in the column phase) get ONE
// 1024-thread workgroup per row, column ids and residuals register-resident for the whole
// t-loop, exactly the per-row update order of ccd_phase_kernel: per group of 4 dimensions
// each thread gathers its RB float4 pieces of the other factor, and every coordinate
// update reduces (up, down) over the workgroup (DPP per wave, then 16 wave partials in
// double-buffered LDS: one barrier per dimension). One pass over the row's nonzeros per
// phase instead of the lockstep path's k+2 streaming passes.
// RB = 8: column ids and residuals in registers (rows <= 8192; 10+ spill). RB = 12 (rows
// <= 12288): the column ids move to LDS (48 KB; read once per 4 dimensions), residuals and
// the gathered float4 pieces stay in registers (14+ spill).
constexpr int BT = 1024, BW = BT / 64;  // threads / waves per medium-row workgroup

template <int RB>
__global__ __launch_bounds__(BT) void ccd_block_kernel(const int* __restrict__ rows, int n_list,
                                                       const long* __restrict__ row_ptr, const int* __restrict__ col,
                                                       float* __restrict__ res, float* __restrict__ Fo,
                                                       const float* __restrict__ Fx, int k, float lam) {
  constexpr bool CJ_LDS = RB > 8;
  __shared__ float s_red[2][BW][2];
  __shared__ int s_cj[CJ_LDS ? BT * RB : 1];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int par = 0;
  // one WG-wide (up, down) total; the parity buffer written here is not rewritten before
  // every thread has passed the NEXT barrier, i.e. finished these reads
  auto wg_total = [&](float up, float dn, float& U, float& D) {
    up = wave_total(up);
    dn = wave_total(dn);
    if (lane == 0) { s_red[par][wv][0] = up; s_red[par][wv][1] = dn; }
    __syncthreads();
    U = 0.f;
    D = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < BW; ++w2) { U += s_red[par][w2][0]; D += s_red[par][w2][1]; }
    par ^= 1;
  };
  for (int li = blockIdx.x; li < n_list; li += gridDim.x) {
    const int r = rows[li];
    const long a = row_ptr[r], b = row_ptr[r + 1];
    const float down0 = lam * (float)(b - a);
    float* w = Fo + (long)r * k;
    int cjr[CJ_LDS ? 1 : RB];
    float rj[RB];
    if (CJ_LDS) __syncthreads();  // the previous row's readers of s_cj are done
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const long j = a + tid + (long)BT * q;
      const int c = j < b ? col[j] : -1;
      if constexpr (CJ_LDS) s_cj[q * BT + tid] = c;  // own slots only: no barrier needed
      else cjr[q] = c;
      rj[q] = j < b ? res[j] : 0.f;
    }
    auto cj = [&](int q) -> int {
      if constexpr (CJ_LDS) return s_cj[q * BT + tid];
      else return cjr[q];
    };
    int t = 0;
    if ((k & 3) == 0) {
      for (; t < k; t += 4) {
        float4 h4[RB];
#pragma unroll
        for (int q = 0; q < RB; ++q) {
          const int c = cj(q);
          h4[q] = c >= 0 ? *(const float4*)(Fx + (long)c * k + t) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        const float4 w4 = *(const float4*)(w + t);
        float wn[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          float up = 0.f, dn = 0.f;
#pragma unroll
          for (int q = 0; q < RB; ++q) {
            const float h = tt == 0 ? h4[q].x : tt == 1 ? h4[q].y : tt == 2 ? h4[q].z : h4[q].w;
            up = fmaf(fmaf(wn[tt], h, rj[q]), h, up);
            dn = fmaf(h, h, dn);
          }
          float U, D;
          wg_total(up, dn, U, D);
          D += down0;
          const float z = D > 0.f ? U / D : wn[tt];
          const float delta = z - wn[tt];
#pragma unroll
          for (int q = 0; q < RB; ++q) {
            const float h = tt == 0 ? h4[q].x : tt == 1 ? h4[q].y : tt == 2 ? h4[q].z : h4[q].w;
            rj[q] = fmaf(-delta, h, rj[q]);
          }
          wn[tt] = z;
        }
        if (tid == 0) *(float4*)(w + t) = make_float4(wn[0], wn[1], wn[2], wn[3]);
      }
    }
    for (; t < k; ++t) {
      const float wt = w[t];
      float hv[RB];
      float up = 0.f, dn = 0.f;
#pragma unroll
      for (int q = 0; q < RB; ++q) {
        const int c = cj(q);
        hv[q] = c >= 0 ? Fx[(long)c * k + t] : 0.f;
        up = fmaf(fmaf(wt, hv[q], rj[q]), hv[q], up);
        dn = fmaf(hv[q], hv[q], dn);
      }
      float U, D;
      wg_total(up, dn, U, D);
      D += down0;
      const float z = D > 0.f ? U / D : wt;
      const float delta = z - wt;
#pragma unroll
      for (int q = 0; q < RB; ++q) rj[q] = fmaf(-delta, hv[q], rj[q]);
      __syncthreads();  // every thread read w[t] before it changes
      if (tid == 0) w[t] = z;
    }
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const long j = a + tid + (long)BT * q;
      if (j < b) res[j] = rj[q];
    }
  }
}

// Rows with more than BT*RB nonzeros (the most popular items in the column phase) run in
// LOCKSTEP over the dimensions: they are cut into chunks spread over many workgroups and
// launch t (t = 0..k+1) does, per chunk,
//   (a) t-1 < k, t >= 1: res_j -= (z_{t-1} - w_{t-1}) h_{j,t-1}, z from the complete sums
//       of launch t-1 (acc[(t-1) % 3]);
//   (b) t < k: partial sums of dimension t (DPP + LDS, one atomic pair per chunk) into
//       acc[t % 3];
//   (c) the chunk that starts its row publishes w_{t-2} = z_{t-2} (nobody reads it in
//       this launch) and clears acc[(t-2) % 3] for launch t+1.
// The other factor is read FEATURE-MAJOR (FxT[t][col]): a launch touches two of its
// columns (2 x n_other x 4 B: L2-resident) instead of k-strided rows from HBM.
// chunks[c] = (row, begin, end, slot); acc[slot][3][2]
__global__ __launch_bounds__(256) void ccd_lockstep_kernel(const long4* __restrict__ chunks, int n_chunks,
                                                           const long* __restrict__ row_ptr,
                                                           const int* __restrict__ col, float* __restrict__ res,
                                                           float* __restrict__ Fo, const float* __restrict__ FxT,
                                                           long ld_t, int k, int t, float lam,
                                                           float* __restrict__ acc, float* __restrict__ hbuf) {
  __shared__ float s_u[4], s_d[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool upd = t >= 1 && t - 1 < k;
  const bool sum = t < k;
  for (int c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const long4 ch = chunks[c];
    float* a = acc + 6 * ch.w;
    const float nrow = (float)(row_ptr[ch.x + 1] - row_ptr[ch.x]);
    float delta = 0.f;
    if (upd) {
      const float U = a[2 * ((t - 1) % 3)], D = a[2 * ((t - 1) % 3) + 1] + lam * nrow;
      const float wprev = Fo[ch.x * k + (t - 1)];
      delta = (D > 0.f ? U / D : wprev) - wprev;
    }
    const float wt = sum ? Fo[ch.x * k + t] : 0.f;
    const float* hc = FxT + (long)t * ld_t;
    float up = 0.f, dn = 0.f;
    // h_{j,t-1} comes back from hbuf (streamed, written by launch t-1) instead of a
    // second random gather; this launch leaves h_{j,t} there for launch t+1
    for (long j = ch.y + tid; j < ch.z; j += 256) {
      float r = res[j];
      if (upd) {
        r = fmaf(-delta, hbuf[j], r);
        if (!sum) res[j] = r;
      }
      if (sum) {
        const float h = hc[col[j]];
        up = fmaf(fmaf(wt, h, r), h, up);
        dn = fmaf(h, h, dn);
        hbuf[j] = h;
        if (upd) res[j] = r;
      }
    }
    if (sum) {
      up = wave_total(up);
      dn = wave_total(dn);
      if (lane == 0) { s_u[wv] = up; s_d[wv] = dn; }
      __syncthreads();
      if (tid == 0) {
        atomicAdd(a + 2 * (t % 3), s_u[0] + s_u[1] + s_u[2] + s_u[3]);
        atomicAdd(a + 2 * (t % 3) + 1, s_d[0] + s_d[1] + s_d[2] + s_d[3]);
      }
      __syncthreads();
    }
    if (t >= 2 && tid == 0 && ch.y == row_ptr[ch.x]) {
      const int p = (t - 2) % 3;
      const float U = a[2 * p], D = a[2 * p + 1] + lam * nrow;
      const float w2 = Fo[ch.x * k + (t - 2)];
      Fo[ch.x * k + (t - 2)] = D > 0.f ? U / D : w2;
      a[2 * p] = 0.f;
      a[2 * p + 1] = 0.f;
    }
  }
}

// res_j = val_j - <Fr[row_j], Fc[col_j]> (ResTask); one wave per 64 nonzeros, k-loop in
// registers (rows of both factors are contiguous k-vectors)
__global__ __launch_bounds__(256) void ccd_residual_kernel(const int* __restrict__ rows, const int* __restrict__ cols,
                                                           const float* __restrict__ val, long nnz,
                                                           const float* __restrict__ Fr, const float* __restrict__ Fc,
                                                           int k, float* __restrict__ res) {
  for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < nnz; j += (long)gridDim.x * blockDim.x) {
    const float* a = Fr + (long)rows[j] * k;
    const float* b = Fc + (long)cols[j] * k;
    float s = 0.f;
    int t = 0;
    if ((k & 3) == 0) {
      for (; t < k; t += 4) {
        const float4 x = *(const float4*)(a + t), y = *(const float4*)(b + t);
        s = fmaf(x.x, y.x, fmaf(x.y, y.y, fmaf(x.z, y.z, fmaf(x.w, y.w, s))));
      }
    }
    for (; t < k; ++t) s = fmaf(a[t], b[t], s);
    res[j] = val[j] - s;
  }
}

}  // namespace

// skip_long: rows with more than 64*RR nonzeros are left to the lockstep path
HARP_EXPORT int harp_ccd_phase(const long* row_ptr, const int* col, float* res, int n_rows, float* F_own,
                               const float* F_other, int k, float lam, int skip_long, hipStream_t s) {
  if (n_rows <= 0) return HARP_OK;
  if (k <= 0) return HARP_EBADARG;
  long blocks = ((long)n_rows + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  ccd_phase_kernel<<<dim3((unsigned)blocks), dim3(256), 0, s>>>(row_ptr, col, res, n_rows, F_own, F_other, k, lam,
                                                                skip_long);
  return harp_launch_status();
}

// medium rows (rows[] lists them): wide = 0 takes rows of <= harp_ccd_block_max(0) nonzeros,
// wide = 1 rows of <= harp_ccd_block_max(1)
HARP_EXPORT int harp_ccd_block_max(int wide) { return BT * (wide ? 12 : 8); }

HARP_EXPORT int harp_ccd_block(const int* rows, int n_list, const long* row_ptr, const int* col, float* res,
                               float* F_own, const float* F_other, int k, float lam, int wide, hipStream_t s) {
  if (n_list <= 0) return HARP_OK;
  if (k <= 0) return HARP_EBADARG;
  const int blocks = n_list < 8192 ? n_list : 8192;
  if (wide)
    ccd_block_kernel<12><<<dim3(blocks), dim3(BT), 0, s>>>(rows, n_list, row_ptr, col, res, F_own, F_other, k, lam);
  else
    ccd_block_kernel<8><<<dim3(blocks), dim3(BT), 0, s>>>(rows, n_list, row_ptr, col, res, F_own, F_other, k, lam);
  return harp_launch_status();
}

// one lockstep launch (t = 0..k+1); acc (6 floats per slot) zero before t = 0
HARP_EXPORT int harp_ccd_lockstep(const void* chunks, int n_chunks, const long* row_ptr, const int* col, float* res,
                                  float* F_own, const float* F_other_t, long ld_t, int k, int t, float lam, float* acc,
                                  float* hbuf, hipStream_t s) {
  if (n_chunks <= 0) return HARP_OK;
  const int blocks = n_chunks < 65536 ? n_chunks : 65536;
  ccd_lockstep_kernel<<<dim3(blocks), dim3(256), 0, s>>>((const long4*)chunks, n_chunks, row_ptr, col, res, F_own,
                                                         F_other_t, ld_t, k, t, lam, acc, hbuf);
  return harp_launch_status();
}

HARP_EXPORT int harp_ccd_residual(const int* rows, const int* cols, const float* val, long nnz, const float* F_rows,
                                  const float* F_cols, int k, float* res, hipStream_t s) {
  if (nnz <= 0) return HARP_OK;
  long blocks = (nnz + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  ccd_residual_kernel<<<dim3((unsigned)blocks), dim3(256), 0, s>>>(rows, cols, val, nnz, F_rows, F_cols, k, res);
  return harp_launch_status();
}

