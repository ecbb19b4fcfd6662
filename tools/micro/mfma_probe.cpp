// Microbenchmark: sustained v_mfma_f32_32x32x2_f32 throughput for the search kernel's
// instruction pattern (probe B operands in VGPRs, A fragments from LDS via ds_read_b128),
// by number of independent accumulator chains and with/without the LDS reads.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_probe.cpp -o mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS, bool LDS>
__global__ __launch_bounds__(256, 2) void probe(const float* in, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float s[64 * 132];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 64 * 132; i += 256) s[i] = in[i & 1023];
  float qb[CHAINS][64];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int j = 0; j < 64; ++j) qb[c][j] = in[(c * 64 + j + lane) & 1023];
  __syncthreads();
  f32x16 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x16{};
  const float* arow = s + (lane & 31) * 132 + (lane >> 5) * 64;
  float4 areg = make_float4(in[lane], in[lane + 1], in[lane + 2], in[lane + 3]);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 64; k += 4) {
      const float4 a = LDS ? *reinterpret_cast<const float4*>(arow + k) : areg;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float av = e == 0 ? a.x : e == 1 ? a.y : e == 2 ? a.z : a.w;
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, qb[c][k + e], acc[c], 0, 0, 0);
      }
    }
  }
  float r = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int j = 0; j < 16; ++j) r += acc[c][j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int C, bool L>
void run(const float* in, float* out, int blocks, int iters, const char* name) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((probe<C, L>), dim3(blocks), dim3(256), 0, 0, in, out, 2);
  hipEventRecord(a);
  hipLaunchKernelGGL((probe<C, L>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double flops = 2.0 * 32 * 32 * 2 * 64 * (double)C * iters * 4.0 * blocks;  // per wave: C chains x 64 MFMA
  printf("%-28s blocks=%5d  %.3f ms  %.1f TFLOP/s  (%.1f%% of 157.3)\n", name, blocks, ms, flops / ms / 1e9,
         flops / ms / 1e9 / 157.3 * 100);
}

int main() {
  float *in, *out;
  hipMalloc(&in, 4096 * 4);
  hipMalloc(&out, 1 << 24);
  hipMemset(in, 0, 4096 * 4);
  // random-ish data (zero data raises the clock: bench on non-zero)
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int iters = 400;
  for (int blocks : {512, 2048}) {
    run<2, true>(in, out, blocks, iters, "2 chains, A from LDS");
    run<2, false>(in, out, blocks, iters, "2 chains, A in regs");
    run<1, true>(in, out, blocks, iters, "1 chain, A from LDS");
  }
  return 0;
}
