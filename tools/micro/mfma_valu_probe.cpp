// Microbenchmark: how many independent VALU instructions can issue between
// v_mfma_f32_32x32x2_f32 instructions (64-cycle issue) before the MFMA rate drops —
// i.e. what the search kernel's arg-best epilogue costs when interleaved with its chains.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_valu_probe.cpp -o mfma_valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NV, int WAVES>
__global__ __launch_bounds__(64 * 4 * WAVES) void probe(const float* in, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  float a = in[lane], b = in[lane + 64];
  f32x16 acc0 = {}, acc1 = {};
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = in[lane + 128 + j];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc1, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV; ++j) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(v[j & 7]) : "v"(a), "v"(b));
    }
  }
  float r = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) r += acc0[j] + acc1[j];
#pragma unroll
  for (int j = 0; j < 8; ++j) r += v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int NV, int WAVES>
void run(const float* in, float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256;  // one workgroup per CU
  hipLaunchKernelGGL((probe<NV, WAVES>), dim3(blocks), dim3(256 * WAVES), 0, 0, in, out, 2);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<NV, WAVES>), dim3(blocks), dim3(256 * WAVES), 0, 0, in, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 2 * 64.0 * iters * 4.0 * WAVES * blocks;  // 64 MFMA per iter per wave
  printf("waves/SIMD=%d VALU per 2 MFMA=%2d  %.3f ms  %.1f TFLOP/s (%.1f%% of 157.3)\n", WAVES, NV, ms,
         flops / ms / 1e9, flops / ms / 1e9 / 157.3 * 100);
}

int main() {
  float *in, *out;
  hipMalloc(&in, 4096 * 4);
  hipMalloc(&out, 1 << 24);
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int iters = 2000;
  run<0, 1>(in, out, iters);
  run<1, 1>(in, out, iters);
  run<2, 1>(in, out, iters);
  run<4, 1>(in, out, iters);
  run<8, 1>(in, out, iters);
  run<16, 1>(in, out, iters);
  run<0, 2>(in, out, iters);
  run<2, 2>(in, out, iters);
  run<4, 2>(in, out, iters);
  run<8, 2>(in, out, iters);
  return 0;
}
