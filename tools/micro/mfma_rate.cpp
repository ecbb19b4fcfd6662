// MFMA issue-rate probe: one workgroup of 4 waves per CU (one wave per SIMD), NACC
// independent accumulators, operands in registers (no memory in the loop).  Gives the
// ceiling of the tall-GEMM kernels' instruction shape (csrc/ef_dgemm.hip).
// build: hipcc -O3 --offload-arch=gfx950 tools/micro/mfma_rate.cpp -o /tmp/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void f64_rate(const double* in, double* out, int iters) {
  const int lane = threadIdx.x & 63;
  double a[4], b[4];
  for (int i = 0; i < 4; ++i) a[i] = in[(lane + i) & 255], b[i] = in[(lane + 7 * i) & 255];
  f64x4 acc[NACC];
  for (int c = 0; c < NACC; ++c) acc[c] = f64x4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < NACC; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[(c + s) & 3], b[s], acc[c], 0, 0, 0);
  double r = 0;
  for (int c = 0; c < NACC; ++c) r += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int NACC>
__global__ __launch_bounds__(256) void f32_rate(const float* in, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  float a[4], b[4];
  for (int i = 0; i < 4; ++i) a[i] = in[(lane + i) & 255], b[i] = in[(lane + 7 * i) & 255];
  f32x16 acc[NACC];
  for (int c = 0; c < NACC; ++c)
    for (int q = 0; q < 16; ++q) acc[c][q] = 0.f;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < NACC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[(c + s) & 3], b[s], acc[c], 0, 0, 0);
  float r = 0;
  for (int c = 0; c < NACC; ++c)
    for (int q = 0; q < 16; ++q) r += acc[c][q];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <class T, class K>
static void time_it(K k, const T* in, T* out, int iters, double flop_per_iter_wave, const char* name, int wgs = 256) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k, dim3(wgs), dim3(256), 0, 0, in, out, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL(k, dim3(wgs), dim3(256), 0, 0, in, out, iters);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double tf = flop_per_iter_wave * iters * 4.0 * wgs / (ms * 1e-3) / 1e12;
  printf("%-24s %.3f ms  %.1f TF/s\n", name, ms, tf);
}

int main(int argc, char** argv) {
  double* in;
  double* out;
  (void)hipMalloc(&in, 4096 * 8);
  (void)hipMalloc(&out, 1 << 22);
  (void)hipMemset(in, 0, 4096 * 8);
  const int it = 20000;
  if (argc > 1) {  // "rand": fp64 shapes on random operands in [-1, 1) (the power-limited rate)
    double h[4096];
    unsigned long long st = 1;
    for (double& v : h) {
      st = st * 6364136223846793005ULL + 1442695040888963407ULL;
      v = (double)(st >> 11) / 4503599627370496.0 - 1.0;
    }
    (void)hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
      time_it(f64_rate<16>, in, out, it, 4.0 * 16 * 2048, "rand f64 16x16x4, 16 acc");
      time_it(f64_rate<8>, in, out, it, 4.0 * 8 * 2048, "rand f64 16x16x4, 8 acc, 2 w/SIMD", 512);
    }
    return 0;
  }
  time_it(f64_rate<16>, in, out, it, 4.0 * 16 * 2048, "f64 16x16x4, 16 acc");
  time_it(f64_rate<4>, in, out, it, 4.0 * 4 * 2048, "f64 16x16x4, 4 acc");
  time_it(f64_rate<8>, in, out, it, 4.0 * 8 * 2048, "f64 16x16x4, 8 acc, 2 w/SIMD", 512);
  time_it(f64_rate<8>, in, out, it, 4.0 * 8 * 2048, "f64 16x16x4, 8 acc, 4 w/SIMD", 1024);
  time_it(f32_rate<4>, (const float*)in, (float*)out, it, 4.0 * 4 * 4096, "f32 32x32x2, 4 acc");
  time_it(f32_rate<8>, (const float*)in, (float*)out, it, 4.0 * 8 * 4096, "f32 32x32x2, 8 acc");
  return 0;
}
