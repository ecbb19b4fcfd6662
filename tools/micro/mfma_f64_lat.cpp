// Latency vs throughput of v_mfma_f64_16x16x4_f64 on one wave (s_memtime cycles):
// a chain of dependent MFMAs on one accumulator, and the same count over 4 independent
// accumulators.  build: hipcc -O3 --offload-arch=gfx950 tools/micro/mfma_f64_lat.cpp -o tools/micro/bin/mfma_f64_lat
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* in, double* out, unsigned long long* t) {
  const int lane = threadIdx.x;
  double a = in[lane], b = in[lane + 64], b1 = in[lane + 1], b2 = in[lane + 2], b3 = in[lane + 3];
  f64x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; ++i) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  out[lane] = c0[0] + c0[1] + c0[2] + c0[3];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b1, c1, 0, 0, 0);  // distinct operands: no CSE
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b2, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b3, c3, 0, 0, 0);
  }
  out[lane + 64] = c0[0] + c1[1] + c2[2] + c3[3];
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { t[0] = t1 - t0; t[1] = t2 - t1; }
}
int main() {
  double *in, *out; unsigned long long* t;
  hipMalloc(&in, 1024); hipMalloc(&out, 1024); hipMalloc(&t, 16);
  hipMemset(in, 0, 1024);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, in, out, t);
  unsigned long long h[2];
  hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
  printf("{\"chained_64_cycles\": %llu, \"per_dependent_mfma\": %.1f, \"independent4x16_cycles\": %llu, \"per_mfma\": %.1f}\n",
         h[0], h[0] / 64.0, h[1], h[1] / 64.0);
  return 0;
}
