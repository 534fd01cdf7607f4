// Sequential CPU reference of the MF-SGD update and RMSE (ml/java/.../sgd/SGDMPTask.java:
// 46-77, RMSETask.java:91-103). Used on CPU-only workers (gloo tests) and as the numerics
// oracle for the HIP kernel. Updates W and H from the OLD values, error = w.h - v.
#include <math.h>

#include "harp_runtime.h"

HARP_HOST_EXPORT void harp_mf_sgd_cpu(const int32_t* rows, const int32_t* cols, const float* vals, int64_t n, int r,
                                      float* W, int ldw, float* H, int ldh, float lr, float lam) {
  for (int64_t i = 0; i < n; ++i) {
    float* w = W + (int64_t)rows[i] * ldw;
    float* h = H + (int64_t)cols[i] * ldh;
    float dot = 0.f;
    for (int k = 0; k < r; ++k) dot = fmaf(w[k], h[k], dot);
    const float ge = -lr * (dot - vals[i]);
    const float decay = 1.0f - lr * lam;
    // w' = w - lr*(err*h + lam*w) = (1 - lr*lam) w - lr*err*h  (and h' alike)
    for (int k = 0; k < r; ++k) {
      const float wk = w[k], hk = h[k];
      w[k] = fmaf(ge, hk, decay * wk);
      h[k] = fmaf(ge, wk, decay * hk);
    }
  }
}

HARP_HOST_EXPORT double harp_mf_sse_cpu(const int32_t* rows, const int32_t* cols, const float* vals, int64_t n, int r,
                                        const float* W, int ldw, const float* H, int ldh) {
  double sse = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const float* w = W + (int64_t)rows[i] * ldw;
    const float* h = H + (int64_t)cols[i] * ldh;
    float dot = 0.f;
    for (int k = 0; k < r; ++k) dot = fmaf(w[k], h[k], dot);
    const double e = (double)vals[i] - dot;
    sse += e * e;
  }
  return sse;
}
