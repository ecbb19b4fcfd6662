// Microbenchmark of the fit's tall GEMMs (csrc/ef_dgemm.hip) at the C3 subspace shape:
// Y (16384 x 256) = C (16384 x 16384, symmetric) . Q, fp64 and fp32, A walked by rows
// (a_trans) or by columns, against the MFMA peak; checks a few entries on the host.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I face-detection-recognization-pca_amd/csrc \
//          tools/micro/tall_gemm_bench.cpp face-detection-recognization-pca_amd/csrc/ef_dgemm.hip -o /tmp/tgb
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ef_linalg.hpp"

template <class T>
static void run(const char* name, int64_t dim, int m, bool at, double peak_tf) {
  std::vector<T> hC((size_t)dim * dim), hQt((size_t)m * dim);
  unsigned long long st = 1;
  auto rnd = [&]() { st = st * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(st >> 11) / 9007199254740992.0 - 0.5; };
  for (int64_t i = 0; i < dim; ++i)
    for (int64_t j = 0; j <= i; ++j) hC[i * dim + j] = hC[j * dim + i] = (T)rnd();
  for (auto& v : hQt) v = (T)rnd();
  T *C, *Qt, *Y, *work;
  (void)hipMalloc(&C, hC.size() * sizeof(T));
  (void)hipMalloc(&Qt, hQt.size() * sizeof(T));
  (void)hipMalloc(&Y, (size_t)dim * m * sizeof(T));
  (void)hipMalloc(&work, (size_t)1 << 27);
  (void)hipMemcpy(C, hC.data(), hC.size() * sizeof(T), hipMemcpyHostToDevice);
  (void)hipMemcpy(Qt, hQt.data(), hQt.size() * sizeof(T), hipMemcpyHostToDevice);
  auto go = [&]() {
    if constexpr (sizeof(T) == 8)
      (void)ef::tall_gemm_f64(0, C, dim, at, Qt, dim, Y, m, dim, m, dim, 1.0, work, ((size_t)1 << 27) / 8);
    else
      (void)ef::tall_gemm_f32(0, C, dim, at, Qt, dim, Y, m, dim, m, dim, 1.f, work, ((size_t)1 << 27) / 4);
  };
  go();
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int reps = 10;
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) go();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  std::vector<T> hY((size_t)dim * m);
  (void)hipMemcpy(hY.data(), Y, hY.size() * sizeof(T), hipMemcpyDeviceToHost);
  double err = 0;
  for (int t = 0; t < 64; ++t) {
    const int64_t i = (t * 2654435761u) % dim, n = (t * 40503u) % m;
    double ref = 0, mag = 0;
    for (int64_t k = 0; k < dim; ++k) ref += (double)hC[i * dim + k] * hQt[n * dim + k], mag += std::fabs((double)hC[i * dim + k] * hQt[n * dim + k]);
    err = std::fmax(err, std::fabs(hY[i * m + n] - ref) / mag);
  }
  const double tf = 2.0 * dim * dim * m / (ms * 1e-3) / 1e12;
  printf("%-6s dim=%lld m=%d a_trans=%d  %.3f ms  %.1f TF/s  %.1f %% of %.1f  max rel err %.2e\n", name, (long long)dim, m,
         (int)at, ms, tf, 100 * tf / peak_tf, peak_tf, err);
  (void)hipFree(C);
  (void)hipFree(Qt);
  (void)hipFree(Y);
  (void)hipFree(work);
}

int main(int argc, char** argv) {
  const int64_t dim = argc > 1 ? atoll(argv[1]) : 16384;
  const int m = argc > 2 ? atoi(argv[2]) : 256;
  run<double>("fp64", dim, m, true, 78.6);
  run<double>("fp64", dim, m, false, 78.6);
  run<float>("fp32", dim, m, true, 157.3);
  run<float>("fp32", dim, m, false, 157.3);
  return 0;
}
