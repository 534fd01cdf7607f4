// WDA-MDS (weighted deterministic-annealing SMACOF) row-block kernels for gfx950, fp64.
//
// Reference: ml/java/.../wdamds/BCCalcTask.java:97-170 (B(Z) X) and
// StressCalcTask.java:72-96 (weighted stress); SURVEY §2.10 "mds_bofz_gemm". For the
// worker's row block [n_r, n] of the distance matrix delta and the weights w:
//   b_ij = -w_ij (delta_ij - diff) / d_ij(Z)   if w_ij != 0, d_ij >= 1e-10, delta_ij > diff
//   b_ii = -sum_{j != i} b_ij,   BC_i = sum_j b_ij x_j
//   stress_i = sum_j w_ij (delta_ij - diff - d_ij)^2 over w_ij != 0, delta_ij >= diff
// with diff = sqrt(2 dim) T. The torch version builds the Gram GEMM, the distance matrix,
// the masks and B as separate [n_r, n] fp64 tensors (about ten passes over n_r x n) and
// then a skinny GEMM with dim = 2..4 columns. The embedding dimension is tiny, so here a
// wave per row streams its delta and w rows once, computes d_ij directly from the
// coordinates (more accurate than the Gram expression near zero; X is L2-resident) and
// accumulates BC_i (or stress_i) in registers: one pass over the two fp64 row blocks.
#include "common.h"

namespace {

template <int DIM, bool STRESS>
__global__ __launch_bounds__(256) void mds_row_kernel(const double* __restrict__ delta, const double* __restrict__ w,
                                                      long ld, int n_r, int n, int row0,
                                                      const double* __restrict__ X, double diff,
                                                      double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n_r; i += nw) {
    const long gi = row0 + i;
    double xi[DIM];
#pragma unroll
    for (int k = 0; k < DIM; ++k) xi[k] = X[gi * DIM + k];
    const double* drow = delta + i * ld;
    const double* wrow = w + i * ld;
    double acc[DIM], bsum = 0.0, st = 0.0;
#pragma unroll
    for (int k = 0; k < DIM; ++k) acc[k] = 0.0;
    for (int j = lane; j < n; j += 64) {
      const double wij = wrow[j], dij = drow[j];
      double xj[DIM], dz2 = 0.0;
#pragma unroll
      for (int k = 0; k < DIM; ++k) {
        xj[k] = X[(long)j * DIM + k];
        const double t = xi[k] - xj[k];
        dz2 = fma(t, t, dz2);
      }
      const double dz = sqrt(dz2);
      if (STRESS) {
        if (wij != 0.0 && dij >= diff) {
          const double e = dij - diff - dz;
          st = fma(wij * e, e, st);
        }
      } else if (j != gi && wij != 0.0 && dz >= 1e-10 && dij > diff) {
        const double b = -wij * (dij - diff) / dz;
        bsum += b;
#pragma unroll
        for (int k = 0; k < DIM; ++k) acc[k] = fma(b, xj[k], acc[k]);
      }
    }
    if (STRESS) {
      st = wave_sum_d(st);
      if (lane == 0) out[i] = st;
    } else {
      bsum = wave_sum_d(bsum);
#pragma unroll
      for (int k = 0; k < DIM; ++k) acc[k] = wave_sum_d(acc[k]);
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < DIM; ++k) out[i * DIM + k] = fma(-bsum, xi[k], acc[k]);
      }
    }
  }
}

template <int DIM>
int launch(const double* delta, const double* w, long ld, int n_r, int n, int row0, const double* X, double diff,
           int stress, double* out, hipStream_t s) {
  long blocks = ((long)n_r + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  const dim3 g((unsigned)blocks), b(256);
  if (stress) mds_row_kernel<DIM, true><<<g, b, 0, s>>>(delta, w, ld, n_r, n, row0, X, diff, out);
  else mds_row_kernel<DIM, false><<<g, b, 0, s>>>(delta, w, ld, n_r, n, row0, X, diff, out);
  return harp_launch_status();
}

}  // namespace

// delta, w: the row block [n_r][ld] (fp64) of global rows row0 .. row0+n_r-1; X [n][dim]
// fp64 (dim 1..4). stress = 0: out [n_r][dim] = (B(Z) X) rows; stress = 1: out [n_r] =
// per-row weighted stress sums.
HARP_EXPORT int harp_mds_rows(const double* delta, const double* w, long ld, int n_r, int n, int row0,
                              const double* X, int dim, double diff, int stress, double* out, hipStream_t s) {
  if (n_r <= 0) return HARP_OK;
  if (n <= 0 || ld < n || row0 < 0 || row0 + n_r > n) return HARP_EBADARG;
  switch (dim) {
    case 1: return launch<1>(delta, w, ld, n_r, n, row0, X, diff, stress, out, s);
    case 2: return launch<2>(delta, w, ld, n_r, n, row0, X, diff, stress, out, s);
    case 3: return launch<3>(delta, w, ld, n_r, n, row0, X, diff, stress, out, s);
    case 4: return launch<4>(delta, w, ld, n_r, n, row0, X, diff, stress, out, s);
    default: return HARP_EUNSUPPORTED;
  }
}
