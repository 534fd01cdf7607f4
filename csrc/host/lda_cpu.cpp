// Sequential collapsed Gibbs sampler (CPU reference of csrc/lda.hip; the reference's
// LDAMPTask.java:85-330 computes the same conditional with SparseLDA buckets). Counts are
// updated exactly (no staleness): the oracle for the GPU sampler's log-likelihood.
#include <math.h>
#include <stdint.h>
#include <vector>

#include "harp_runtime.h"

static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

HARP_HOST_EXPORT void harp_lda_cgs_cpu(const int32_t* tdoc, const int32_t* tword, int32_t* tz, int64_t n,
                                       int32_t* ndk, int ldd, int32_t* nwk, int ldw, int32_t* nk, int K, float alpha,
                                       float beta, float vbeta, uint64_t seed) {
  std::vector<double> p(K);
  for (int64_t i = 0; i < n; ++i) {
    const int d = tdoc[i], w = tword[i], z = tz[i];
    int32_t* nd = ndk + (int64_t)d * ldd;
    int32_t* nw = nwk + (int64_t)w * ldw;
    nd[z]--; nw[z]--; nk[z]--;
    double tot = 0;
    for (int k = 0; k < K; ++k) {
      tot += (nd[k] + alpha) * (nw[k] + beta) / (nk[k] + vbeta);
      p[k] = tot;
    }
    const double u = (double)(mix64(seed ^ ((uint64_t)i * 0xD6E8FEB86659FD93ull)) >> 40) * (1.0 / 16777216.0) * tot;
    int nz = K - 1;
    for (int k = 0; k < K; ++k)
      if (p[k] > u) { nz = k; break; }
    nd[nz]++; nw[nz]++; nk[nz]++;
    tz[i] = nz;
  }
}
