// Microbenchmark of the fit's CholQR factor at the subspace orders the fit uses: the
// blocked kernels (csrc/ef_chol_blk.hip, launch_chol_inv) against round 4's
// register-resident kernel (csrc/ef_linalg.hip, launch_chol_inv_reg): average launch time
// over back-to-back launches, the host check max |L^-1 G L^-T - I| for each, the largest
// difference between the two inverses (relative to max |Li|), and a rank-deficient G,
// which must report the failing column and leave Li untouched.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I face-detection-recognization-pca_amd/csrc \
//          tools/micro/chol_inv_bench.cpp face-detection-recognization-pca_amd/csrc/ef_linalg.hip \
//          face-detection-recognization-pca_amd/csrc/ef_chol_blk.hip -o /tmp/cib
// usage: cib [m ...]   (default 256 128 88 200)
// -fgpu-rdc -DEF_CB_STAMP (both sources too): also print per-block-column phase stamps
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ef_linalg.hpp"
#ifdef EF_CB_STAMP
namespace ef {
extern __device__ unsigned long long g_cb_stamp[2][16][8];
}
#endif

namespace ef {  // ef_api.hip's helper, for the other launchers in ef_linalg.hip
hipError_t allow_dynamic_lds(const void* fn, int bytes) {
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
}  // namespace ef

static double orth_err(const std::vector<double>& G, const std::vector<double>& Li, int m) {
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
  for (int i = 0; i < m; ++i)  // zeros above the diagonal
    for (int j = i + 1; j < m; ++j)
      if (Li[(size_t)i * m + j] != 0.0) err = INFINITY;
  return err;
}

int main(int argc, char** argv) {
  std::vector<int> ms;
  for (int a = 1; a < argc; ++a) ms.push_back(atoi(argv[a]));
  if (ms.empty()) ms = {256, 128, 88, 200};
  const int reps = 200;
  int rc = 0;
  for (int m : ms) {
    // G = B^T B / m + I/4 with B uniform: well conditioned, like the Gram of a nearly
    // orthonormal block; then scaled columns to spread the pivots over 1e-6 .. 1
    std::vector<double> B((size_t)m * m), G((size_t)m * m, 0.0), sc(m);
    unsigned long long st = 7 + m;
    auto rnd = [&]() { st = st * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(st >> 11) / 9007199254740992.0 - 0.5; };
    for (auto& v : B) v = rnd();
    for (int i = 0; i < m; ++i) sc[i] = pow(10.0, -3.0 * i / m);
    for (int i = 0; i < m; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = 0.0;
        for (int k = 0; k < m; ++k) s += B[(size_t)k * m + i] * B[(size_t)k * m + j];
        G[(size_t)i * m + j] = G[(size_t)j * m + i] = (s / m + (i == j ? 0.25 : 0.0)) * sc[i] * sc[j];
      }
    double *dG, *dLi, *dLr, *dW;
    int* dinfo;
    (void)hipMalloc(&dG, G.size() * sizeof(double));
    (void)hipMalloc(&dLi, G.size() * sizeof(double));
    (void)hipMalloc(&dLr, G.size() * sizeof(double));
    (void)hipMalloc(&dW, ef::chol_inv_work_elems(m) * sizeof(double));
    (void)hipMalloc(&dinfo, sizeof(int));
    (void)hipMemcpy(dG, G.data(), G.size() * sizeof(double), hipMemcpyHostToDevice);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto timeit = [&](bool blocked, double* out) -> double {
      for (int i = 0; i < 5; ++i) {
        const hipError_t e = blocked ? ef::launch_chol_inv(s, dG, m, m, 1e-13, out, dinfo, dW)
                                     : ef::launch_chol_inv_reg(s, dG, m, m, 1e-13, out, dinfo);
        if (e != hipSuccess) return -1.0;
      }
      (void)hipEventRecord(e0, s);
      for (int i = 0; i < reps; ++i)
        (void)(blocked ? ef::launch_chol_inv(s, dG, m, m, 1e-13, out, dinfo, dW)
                       : ef::launch_chol_inv_reg(s, dG, m, m, 1e-13, out, dinfo));
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      return 1000.0 * ms / reps;
    };
    const double t_blk = timeit(true, dLi);
    int info_blk = 1;
    (void)hipMemcpy(&info_blk, dinfo, sizeof(int), hipMemcpyDeviceToHost);
    const bool reg_ok = ef::chol_inv_reg_supported(m);
    const double t_reg = reg_ok ? timeit(false, dLr) : -1.0;
    std::vector<double> Li(G.size()), Lr(G.size());
    (void)hipMemcpy(Li.data(), dLi, Li.size() * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipMemcpy(Lr.data(), dLr, Lr.size() * sizeof(double), hipMemcpyDeviceToHost);
    const double err_blk = orth_err(G, Li, m);
    const double err_reg = reg_ok ? orth_err(G, Lr, m) : -1.0;
    double dmax = 0.0, lmax = 0.0;
    if (reg_ok)
      for (size_t i = 0; i < Li.size(); ++i) {
        dmax = fmax(dmax, fabs(Li[i] - Lr[i]));
        lmax = fmax(lmax, fabs(Lr[i]));
      }
    // rank-deficient G: column 37 (or m/2) a copy of column 5 -> pivot ~0 there
    const int dup = m > 40 ? 37 : m / 2;
    std::vector<double> Gs = G;
    for (int i = 0; i < m; ++i) {
      Gs[(size_t)i * m + dup] = G[(size_t)i * m + 5];
      Gs[(size_t)dup * m + i] = G[(size_t)5 * m + i];
    }
    Gs[(size_t)dup * m + dup] = G[(size_t)5 * m + 5];
    (void)hipMemcpy(dG, Gs.data(), Gs.size() * sizeof(double), hipMemcpyHostToDevice);
    (void)hipMemset(dLi, 0x7f, G.size() * sizeof(double));
    int info_bad = 0;
    (void)ef::launch_chol_inv(s, dG, m, m, 1e-13, dLi, dinfo, dW);
    (void)hipMemcpy(&info_bad, dinfo, sizeof(int), hipMemcpyDeviceToHost);
    std::vector<unsigned char> raw(G.size() * sizeof(double));
    (void)hipMemcpy(raw.data(), dLi, raw.size(), hipMemcpyDeviceToHost);
    bool untouched = true;
    for (unsigned char b : raw) untouched = untouched && b == 0x7f;
#ifdef EF_CB_STAMP
    {  // phase stamps (s_memtime) of one blocked launch on the well-conditioned G
      (void)hipMemcpy(dG, G.data(), G.size() * sizeof(double), hipMemcpyHostToDevice);
      (void)ef::launch_chol_inv(s, dG, m, m, 1e-13, dLi, dinfo, dW);
      (void)hipStreamSynchronize(s);
      unsigned long long st[2][16][8];
      (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(ef::g_cb_stamp), sizeof(st));
      const int nb = (m + 15) / 16;
      const unsigned long long t0 = st[0][0][0] < st[1][0][0] ? st[0][0][0] : st[1][0][0];
      for (int J = 0; J < nb; ++J) {
        printf("J=%2d worker:", J);
        for (int k = 0; k < 7; ++k) printf(" %7llu", st[0][J][k] - t0);
        printf("   diag:");
        for (int k = 0; k < 7; ++k) printf(" %7llu", st[1][J][k] - t0);
        printf("\n");
      }
    }
#endif
    printf("{\"m\": %d, \"reps\": %d, \"us_blocked\": %.2f, \"us_reg\": %.2f, \"info\": %d, \"err_blocked\": %.3e, "
           "\"err_reg\": %.3e, \"max_diff_rel\": %.3e, \"singular_info\": %d, \"singular_li_untouched\": %s}\n",
           m, reps, t_blk, t_reg, info_blk, err_blk, err_reg, lmax > 0 ? dmax / lmax : 0.0, info_bad,
           untouched ? "true" : "false");
    const bool ok = info_blk == 0 && err_blk < 1e-9 && info_bad == -(dup + 1) && untouched;
    if (!ok) rc = 1;
    (void)hipFree(dG);
    (void)hipFree(dLi);
    (void)hipFree(dLr);
    (void)hipFree(dW);
    (void)hipFree(dinfo);
    (void)hipStreamDestroy(s);
  }
  return rc;
}
