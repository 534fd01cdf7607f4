// One-vs-rest logistic regression SGD pass for gfx950 (contrib MLR).
//
// Reference: contrib/src/main/java/edu/iu/mlr/GDtask.java:30-72 — for every instance of
// the local shard, for every topic model resident on this worker:
//   W[t] += alpha * (label_t - sigmoid(W[t] . x)) * x      (bias in W[t][0], x_0 = 1)
// SURVEY §2.10 "sparse_logreg_sgd". harp_amd/models/mlr.py runs it in mini-batches (the
// gradient of a batch uses the weights before the batch; batch 1 = the reference order).
//
// The torch formulation issues ~10 small kernels per mini-batch, so a pass over a shard is
// launch bound. Here the whole pass is ONE launch: the topics are independent chains
// (one-vs-rest), so each workgroup owns one topic row of W and walks the batches in order.
//   phase 1: each wave takes rows of the batch; lanes stride the row's nonzeros, a DPP/xor
//            wave sum gives W[t] . x; the residual alpha (y - sigmoid) goes to LDS.
//   phase 2: lanes scatter R_i * v into W[t] with fp64 atomics (rows of a batch share
//            columns), wave 0 adds the summed residuals to the bias.
//   an agent-scope fence + barrier publishes the batch's updates (L2) and invalidates the
//   CU's L1 before the next batch reads W[t] again.
#include "common.h"

namespace {

constexpr int MAXB = 1024;  // residuals of one batch held in LDS

__global__ __launch_bounds__(1024) void mlr_sgd_pass_kernel(const long* __restrict__ crow,
                                                           const int* __restrict__ col,
                                                           const double* __restrict__ val, int n,
                                                           const float* __restrict__ Y, long ldy, double* W, long ldw,
                                                           double alpha, int batch) {
  __shared__ double R[MAXB];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  double* w = W + (long)t * ldw;
  for (int a = 0; a < n; a += batch) {
    const int b = a + batch < n ? a + batch : n;
    for (int i = a + wave; i < b; i += nwave) {
      const long s = crow[i], e = crow[i + 1];
      double acc = 0.0;
      for (long p = s + lane; p < e; p += 64) acc = fma(w[1 + col[p]], val[p], acc);
      acc = wave_sum_d(acc) + w[0];
      if (lane == 0) R[i - a] = alpha * ((double)Y[(long)i * ldy + t] - 1.0 / (1.0 + exp(-acc)));
    }
    __syncthreads();
    for (int i = a + wave; i < b; i += nwave) {
      const long s = crow[i], e = crow[i + 1];
      const double r = R[i - a];
      for (long p = s + lane; p < e; p += 64) unsafeAtomicAdd(&w[1 + col[p]], r * val[p]);
    }
    if (wave == 0) {
      double rs = 0.0;
      for (int i = lane; i < b - a; i += 64) rs += R[i];
      rs = wave_sum_d(rs);
      if (lane == 0) unsafeAtomicAdd(&w[0], rs);
    }
    __threadfence();
    __syncthreads();
  }
}

}  // namespace

// crow int64 [n+1], col int32, val fp64 (CSR rows of the local shard); Y fp32 labels with
// row stride ldy, column t = topic t; W fp64 [T][ldw] (bias in column 0), updated in place.
// threads = workgroup size (waves share a batch's rows; one workgroup per topic chain).
HARP_EXPORT int harp_mlr_sgd_pass(const long* crow, const int* col, const double* val, int n, const float* Y,
                                  long ldy, double* W, int T, long ldw, double alpha, int batch, int threads,
                                  hipStream_t s) {
  if (n <= 0 || T <= 0) return HARP_OK;
  if (batch <= 0 || batch > MAXB || threads < 64 || threads > 1024 || (threads & 63)) return HARP_EBADARG;
  mlr_sgd_pass_kernel<<<dim3((unsigned)T), dim3(threads), 0, s>>>(crow, col, val, n, Y, ldy, W, ldw, alpha, batch);
  return harp_launch_status();
}
