// Fused MLP epilogues for gfx950 (fp32): the non-GEMM half of a fully-connected layer.
//
// Reference: DAAL neural_networks fully-connected + softmax-cross-entropy layers trained
// by the distributed SGD solver (ml/daal/.../daal_nn/NNDaalCollectiveMapper.java) and the
// contrib jblas sigmoid MLP (contrib/.../NN/HarpNeuralNetwork.java). The GEMMs stay on
// hipBLASLt (plain library GEMMs); everything between two GEMMs is ONE pass here:
//  * bias_act_fwd:      a = act(z + b)                       (z written by the GEMM)
//  * softmax_xent:      p = softmax(z), loss += -log p[y], delta = (p - onehot(y)) * scale,
//                       db += column sums of delta            (one wave per row)
//  * dact_bgrad:        delta *= act'(a), db += column sums of the result
// The column sums are reduced in LDS per workgroup (4 rows -> one partial) before one
// atomic per column, so the bias gradients need no extra pass over delta.
#include "common.h"

namespace {

enum Act { kSigmoid = 0, kTanh = 1, kRelu = 2, kNone = 3 };

__device__ __forceinline__ float act_f(float z, int act) {
  switch (act) {
    case kSigmoid: return 1.f / (1.f + __expf(-z));
    case kTanh: return tanhf(z);
    case kRelu: return z > 0.f ? z : 0.f;
    default: return z;
  }
}

// derivative expressed through the activation value a = act(z)
__device__ __forceinline__ float dact(float a, int act) {
  switch (act) {
    case kSigmoid: return a * (1.f - a);
    case kTanh: return 1.f - a * a;
    case kRelu: return a > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

__global__ void bias_act_kernel(float* __restrict__ z, const float* __restrict__ b, long total, int N, int act) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % N);
    z[i] = act_f(z[i] + (b ? b[c] : 0.f), act);
  }
}

// one wave per row; 4 rows per workgroup; C columns strided over the lanes
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ z, int B, int C,
                                                           const int* __restrict__ labels, float scale,
                                                           float* __restrict__ delta, float* __restrict__ loss,
                                                           float* __restrict__ dbias) {
  extern __shared__ float colsum[];  // [C]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int c = threadIdx.x; c < C; c += blockDim.x) colsum[c] = 0.f;
  __syncthreads();
  const int row = blockIdx.x * 4 + w;
  float lrow = 0.f;
  if (row < B) {
    const float* zr = z + (long)row * C;
    float m = -3.4e38f;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, zr[c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += __expf(zr[c] - m);
    s = wave_sum(s);
    const float inv = 1.f / s;
    const int y = labels[row];
    float* dr = delta + (long)row * C;
    for (int c = lane; c < C; c += 64) {
      const float p = __expf(zr[c] - m) * inv;
      const float g = (p - (c == y ? 1.f : 0.f)) * scale;
      dr[c] = g;
      atomicAdd(&colsum[c], g);  // LDS: 4 rows per column slot
    }
    // an out-of-range label contributes no target (and is never used as an index)
    if (lane == 0 && y >= 0 && y < C) lrow = -(zr[y] - m - __logf(s));
  }
  __shared__ float wl[4];
  if (lane == 0) wl[w] = row < B ? lrow : 0.f;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss, wl[0] + wl[1] + wl[2] + wl[3]);  // one per workgroup
  if (dbias)
    for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&dbias[c], colsum[c]);
}

// delta[B][N] *= act'(a); dbias[N] += column sums (rows tiled 32 per workgroup)
__global__ __launch_bounds__(256) void dact_bgrad_kernel(float* __restrict__ delta, const float* __restrict__ a, int B,
                                                         int N, int act, float* __restrict__ dbias) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r0 = blockIdx.y * 32;
  if (c >= N) return;
  float s = 0.f;
  const int r1 = r0 + 32 < B ? r0 + 32 : B;
  for (int r = r0; r < r1; ++r) {
    const long i = (long)r * N + c;
    const float g = delta[i] * dact(a[i], act);
    delta[i] = g;
    s += g;
  }
  if (dbias) atomicAdd(&dbias[c], s);
}

}  // namespace

HARP_EXPORT int harp_nn_bias_act(float* z, const float* b, long rows, int N, int act, hipStream_t s) {
  if (rows <= 0 || N <= 0) return HARP_OK;
  if (act < 0 || act > 3) return HARP_EBADARG;
  const long total = rows * (long)N;
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  bias_act_kernel<<<dim3((unsigned)blocks), dim3(256), 0, s>>>(z, b, total, N, act);
  return harp_launch_status();
}

// labels int32 [B] in [0, C); loss (one float, accumulated), dbias [C] accumulated (may be null)
HARP_EXPORT int harp_nn_softmax_xent(const float* z, int B, int C, const int* labels, float scale, float* delta,
                                     float* loss, float* dbias, hipStream_t s) {
  if (B <= 0) return HARP_OK;
  if (C <= 0 || C > 16384) return HARP_EBADARG;
  softmax_xent_kernel<<<dim3((B + 3) / 4), dim3(256), (size_t)C * sizeof(float), s>>>(z, B, C, labels, scale, delta,
                                                                                    loss, dbias);
  return harp_launch_status();
}

HARP_EXPORT int harp_nn_dact_bgrad(float* delta, const float* a, int B, int N, int act, float* dbias, hipStream_t s) {
  if (B <= 0 || N <= 0) return HARP_OK;
  if (act < 0 || act > 3) return HARP_EBADARG;
  dact_bgrad_kernel<<<dim3((N + 255) / 256, (B + 31) / 32), dim3(256), 0, s>>>(delta, a, B, N, act, dbias);
  return harp_launch_status();
}
