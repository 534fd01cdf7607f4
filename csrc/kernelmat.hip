// Kernel-matrix epilogue for SVM / kernel functions (gfx950): one in-place pass over the
// Gram block G = X Y^T that hipBLASLt produced, turning it into the RBF kernel
//   K_ij = exp(-max(|x_i|^2 + |y_j|^2 - 2 G_ij, 0) * inv2s2),   inv2s2 = 1 / (2 sigma^2).
// Reference: the DAAL kernel_function (rbf) that the SVM mappers build their Gram matrix
// with (ml/daal/src/main/java/edu/iu/daal_svm/MultiClassDenseBatch/SVMDaalCollectiveMapper.java:179
// via the svm training algorithm's kernel parameter). The torch expression took five
// elementwise passes over the n x m matrix (3.2 GB at n = m = 20k fp64); this is one read
// and one write, rows of the block streamed with coalesced accesses.
#include "common.h"

namespace {

template <class T>
__global__ __launch_bounds__(256) void rbf_from_gram_kernel(T* __restrict__ G, long ldg, int n, int m,
                                                            const T* __restrict__ nx, const T* __restrict__ ny,
                                                            T inv2s2) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= m) return;
  const T yc = ny[c];
  for (int r = blockIdx.y; r < n; r += gridDim.y) {
    T* p = G + (long)r * ldg + c;
    T d2 = nx[r] + yc - T(2) * *p;
    d2 = d2 > T(0) ? d2 : T(0);
    *p = exp(-d2 * inv2s2);
  }
}

template <class T>
int launch_rbf(T* G, long ldg, int n, int m, const T* nx, const T* ny, T inv2s2, hipStream_t s) {
  const unsigned gx = (unsigned)((m + 255) / 256);
  unsigned gy = (unsigned)(n < 2048 ? n : 2048);  // rows per column block strided over gy
  while ((long)gx * gy < 4096 && gy < (unsigned)n) gy *= 2;
  if (gy > (unsigned)n) gy = (unsigned)n;
  rbf_from_gram_kernel<T><<<dim3(gx, gy), dim3(256), 0, s>>>(G, ldg, n, m, nx, ny, inv2s2);
  return harp_launch_status();
}

}  // namespace

// G [n x m] (row stride ldg) holds X Y^T on entry and the RBF kernel on return; nx [n],
// ny [m]: squared row norms. dtype: 0 = fp32, 1 = fp64.
HARP_EXPORT int harp_rbf_from_gram(void* G, long ldg, int n, int m, const void* nx, const void* ny, double inv2s2,
                                   int dtype, hipStream_t s) {
  if (n < 0 || m < 0 || ldg < m || !(inv2s2 > 0)) return HARP_EBADARG;
  if (n == 0 || m == 0) return HARP_OK;
  if (dtype == 1)
    return launch_rbf<double>((double*)G, ldg, n, m, (const double*)nx, (const double*)ny, inv2s2, s);
  if (dtype == 0)
    return launch_rbf<float>((float*)G, ldg, n, m, (const float*)nx, (const float*)ny, (float)inv2s2, s);
  return HARP_EBADARG;
}
