/* A C caller of include/eigenface.h with no Python in the process: the integration a
 * C/C++ host (or a cgo / JNI / N-API binding) does.  Fits eigenfaces on
 * synthetic uint8 faces, checks the fit against plain double-precision arithmetic in this
 * file (orthonormal rows, covariance residual ||C v - lambda v||), projects a gallery,
 * recognises perturbed copies of gallery faces with both metrics, and checks every
 * identity against a brute-force double scan of the same float features.
 * Test-side only: tests/test_gpu_native_c.py builds it with gcc and runs it on the GPU box.
 * Exit 0 and "C_PIPELINE_OK" on success. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "eigenface.h"

#define CHECK(call)                                                                     \
  do {                                                                                  \
    int rc_ = (call);                                                                   \
    if (rc_ != EF_OK) {                                                                 \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, ctx ? ef_last_error(ctx) : ""); \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

static uint64_t lcg_state = 88172645463325252ull;
static double urand(void) { /* xorshift64*, uniform in [0, 1) */
  lcg_state ^= lcg_state >> 12;
  lcg_state ^= lcg_state << 25;
  lcg_state ^= lcg_state >> 27;
  return (double)((lcg_state * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
}

int main(void) {
  ef_ctx* ctx = NULL;
  if (ef_api_version() != EF_API_VERSION) {
    fprintf(stderr, "API version %d, header %d\n", ef_api_version(), EF_API_VERSION);
    return 1;
  }
  CHECK(ef_create(0, &ctx));
  const int64_t n = 700, d = 1024, r = 24;
  const int32_t k = 16;
  /* faces: 128 + sum_j z_ij s_j b_j + noise, clipped to uint8 */
  double* B = malloc(sizeof(double) * r * d);
  for (int64_t i = 0; i < r * d; ++i) B[i] = urand() * 2.0 - 1.0;
  uint8_t* X = malloc(n * d);
  for (int64_t i = 0; i < n; ++i) {
    double z[24];
    for (int j = 0; j < r; ++j) z[j] = (urand() * 2.0 - 1.0) * 60.0 / (1.0 + j);
    for (int64_t c = 0; c < d; ++c) {
      double v = 128.0 + 4.0 * (urand() - 0.5);
      for (int j = 0; j < r; ++j) v += z[j] * B[j * d + c];
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      X[i * d + c] = (uint8_t)lrint(v);
    }
  }
  double* mean = malloc(sizeof(double) * d);
  double* comp = malloc(sizeof(double) * k * d);
  double* lam = malloc(sizeof(double) * k);
  int32_t kout = 0, iters = 0;
  CHECK(ef_fit(ctx, X, n, d, k, 0, mean, NULL, NULL, comp, lam, NULL, NULL, &kout, &iters));
  if (kout != k) {
    fprintf(stderr, "k_out %d\n", kout);
    return 1;
  }
  /* orthonormal rows */
  double orth = 0.0;
  for (int a = 0; a < k; ++a)
    for (int b = 0; b < k; ++b) {
      double s = 0.0;
      for (int64_t c = 0; c < d; ++c) s += comp[a * d + c] * comp[b * d + c];
      orth = fmax(orth, fabs(s - (a == b ? 1.0 : 0.0)));
    }
  /* residual of C v = lambda v with C = (X - mu)^T (X - mu) / (n - 1), applied through X */
  double resid = 0.0;
  double* cv = malloc(sizeof(double) * d);
  for (int a = 0; a < k; ++a) {
    memset(cv, 0, sizeof(double) * d);
    for (int64_t i = 0; i < n; ++i) {
      double t = 0.0;
      for (int64_t c = 0; c < d; ++c) t += (X[i * d + c] - mean[c]) * comp[a * d + c];
      for (int64_t c = 0; c < d; ++c) cv[c] += (X[i * d + c] - mean[c]) * t;
    }
    double e = 0.0;
    for (int64_t c = 0; c < d; ++c) {
      const double u = cv[c] / (double)(n - 1) - lam[a] * comp[a * d + c];
      e += u * u;
    }
    resid = fmax(resid, sqrt(e) / lam[0]);
    if (a > 0 && lam[a] > lam[a - 1]) {
      fprintf(stderr, "eigenvalues not descending at %d\n", a);
      return 1;
    }
  }
  printf("fit: k=%d iters=%d lambda1=%.6g max|VV'-I|=%.3e max||Cv-lv||/l1=%.3e\n", kout, iters, lam[0], orth, resid);
  if (!(orth < 1e-12) || !(resid < 1e-10)) return 1;

  /* recognition model and gallery = projected training faces */
  float* meanf = malloc(sizeof(float) * d);
  float* W = malloc(sizeof(float) * d * k);
  for (int64_t c = 0; c < d; ++c) {
    meanf[c] = (float)mean[c];
    for (int a = 0; a < k; ++a) W[c * k + a] = (float)comp[a * d + c];
  }
  CHECK(ef_model_set(ctx, meanf, W, d, k, 0));
  float* G = malloc(sizeof(float) * n * k);
  CHECK(ef_project(ctx, X, EF_U8, n, G, 0));
  CHECK(ef_gallery_set(ctx, G, n, k, 0, 0));
  /* probes: gallery faces with pixel noise */
  const int64_t b = 300;
  uint8_t* P = malloc(b * d);
  int64_t* truth = malloc(sizeof(int64_t) * b);
  for (int64_t q = 0; q < b; ++q) {
    truth[q] = (int64_t)(urand() * n);
    for (int64_t c = 0; c < d; ++c) {
      int v = X[truth[q] * d + c] + (int)lrint(6.0 * (urand() - 0.5));
      P[q * d + c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
  }
  int64_t* keys = malloc(sizeof(int64_t) * b);
  float* F = malloc(sizeof(float) * b * k);
  float* best = malloc(sizeof(float) * b);
  int64_t* idx = malloc(sizeof(int64_t) * b);
  for (int metric = 0; metric < 2; ++metric) {
    CHECK(ef_recognize(ctx, P, EF_U8, b, metric, keys, F, 0));
    ef_keys_decode(keys, b, metric, best, idx);
    int64_t agree = 0, planted = 0;
    for (int64_t q = 0; q < b; ++q) {
      /* brute force in double over the same float features: first best index wins */
      int64_t arg = -1;
      double bv = 0.0, qn = 0.0;
      for (int a = 0; a < k; ++a) qn += (double)F[q * k + a] * F[q * k + a];
      for (int64_t g = 0; g < n; ++g) {
        double s = 0.0, gn = 0.0;
        for (int a = 0; a < k; ++a) {
          const double x = F[q * k + a], y = G[g * k + a];
          s += metric == EF_METRIC_L2 ? (x - y) * (x - y) : x * y;
          gn += y * y;
        }
        if (metric == EF_METRIC_COSINE) s = s / (sqrt(qn) * sqrt(gn));
        if (arg < 0 || (metric == EF_METRIC_L2 ? s < bv : s > bv)) arg = g, bv = s;
      }
      agree += arg == idx[q];
      planted += truth[q] == idx[q];
    }
    printf("%s: %lld/%lld identities equal the double brute force, %lld/%lld planted\n",
           metric == EF_METRIC_L2 ? "l2" : "cosine", (long long)agree, (long long)b, (long long)planted,
           (long long)b);
    if (agree != b) return 1;
  }
  ef_destroy(ctx);
  printf("C_PIPELINE_OK\n");
  return 0;
}
