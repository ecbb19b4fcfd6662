// Microbenchmark of chol_inv_kernel (csrc/ef_linalg.hip, the fit's CholQR factor) at the
// C3 subspace order m = 256: average launch time over back-to-back launches and the
// host check max |L^-1 G L^-T - I|.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I face-detection-recognization-pca_amd/csrc \
//          tools/micro/chol_inv_bench.cpp face-detection-recognization-pca_amd/csrc/ef_linalg.hip -o /tmp/cib
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ef_linalg.hpp"

namespace ef {  // ef_api.hip's helper, for the other launchers in ef_linalg.hip
hipError_t allow_dynamic_lds(const void* fn, int bytes) {
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
}  // namespace ef

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 256, reps = argc > 2 ? atoi(argv[2]) : 200;
  // G = B^T B / m + I/4 with B uniform: well conditioned, like the Gram of a nearly
  // orthonormal block
  std::vector<double> B((size_t)m * m), G((size_t)m * m, 0.0);
  unsigned long long st = 7;
  auto rnd = [&]() { st = st * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(st >> 11) / 9007199254740992.0 - 0.5; };
  for (auto& v : B) v = rnd();
  for (int i = 0; i < m; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      for (int k = 0; k < m; ++k) s += B[(size_t)k * m + i] * B[(size_t)k * m + j];
      G[(size_t)i * m + j] = G[(size_t)j * m + i] = s / m + (i == j ? 0.25 : 0.0);
    }
  double *dG, *dLi;
  int* dinfo;
  (void)hipMalloc(&dG, G.size() * sizeof(double));
  (void)hipMalloc(&dLi, G.size() * sizeof(double));
  (void)hipMalloc(&dinfo, sizeof(int));
  (void)hipMemcpy(dG, G.data(), G.size() * sizeof(double), hipMemcpyHostToDevice);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int i = 0; i < 10; ++i)
    if (ef::launch_chol_inv(s, dG, m, m, 1e-13, dLi, dinfo) != hipSuccess) return 2;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i) (void)ef::launch_chol_inv(s, dG, m, m, 1e-13, dLi, dinfo);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<double> Li(G.size());
  int info = 1;
  (void)hipMemcpy(Li.data(), dLi, Li.size() * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipMemcpy(&info, dinfo, sizeof(int), hipMemcpyDeviceToHost);
  // R = Li G Li^T
  std::vector<double> T((size_t)m * m);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) {
      double acc = 0.0;
      for (int k = 0; k <= i; ++k) acc += Li[(size_t)i * m + k] * G[(size_t)k * m + j];
      T[(size_t)i * m + j] = acc;
    }
  double err = 0.0;
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) {
      double acc = 0.0;
      for (int k = 0; k <= j; ++k) acc += T[(size_t)i * m + k] * Li[(size_t)j * m + k];
      err = fmax(err, fabs(acc - (i == j ? 1.0 : 0.0)));
    }
  printf("{\"m\": %d, \"reps\": %d, \"us_per_launch\": %.2f, \"info\": %d, \"max_err\": %.3e}\n", m, reps,
         1000.0 * ms / reps, info, err);
  return info == 0 && err < 1e-10 ? 0 : 1;
}
