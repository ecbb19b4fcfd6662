// Clock ceiling of bf16 MFMA loads on the whole chip: bare
// v_mfma_f32_32x32x16_bf16 and v_mfma_f32_16x16x32_bf16 loops on random operands, every
// CU busy, at the occupancy of search_wide3_kernel (8 waves per CU = 2 per SIMD, one
// 512-thread workgroup per CU) and at 1 wave per SIMD; optionally with every A/B operand
// re-read from LDS by ds_read_b128 (the scan's operand path).  After >= 2 s of
// back-to-back launches the last launch is timed with hipEvents and stamped in-kernel
// (s_memtime / s_memrealtime around the loop, MI355X_MICROARCH.md "DVFS give-back" item 6)
// -> TFLOP/s, fraction of the 2.5 PF dense bf16 peak, and the clock the chip held.  The
// scan kernels' fractions are then also stated against this power-limited rate.
// build: hipcc -O3 --offload-arch=gfx950 tools/micro/bf16_clock.cpp -o tools/micro/bf16_clock
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef long i64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ i64x2 as_i64x2(const bf16x8& v) {
  i64x2 r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}

// SHAPE 0: 32x32x16 (32 cyc), 1: 16x16x32 (16 cyc); 2: i8 32x32x32, 3: i8 16x16x64 (the
// covariance SYRK's instruction and its 16x16 form; int32 accumulators).  NACC accumulators of 512 (32x32) or
// 4x 16x16 = the same 1024 outputs per accumulator group.  LDS: operands re-read from LDS.
template <int SHAPE, bool LDS>
__global__ __launch_bounds__(512) void bf16_loop(const unsigned* __restrict__ in, float* __restrict__ out,
                                                 unsigned long long* __restrict__ stamps, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned lds[8192];  // 32 KiB of random bf16 pairs
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 8192; i += blockDim.x) lds[i] = in[(blockIdx.x * 977 + i) & 65535];
  __syncthreads();
  bf16x8 a[4], b[4];
  for (int i = 0; i < 4; ++i) {
    const uint4 va = *reinterpret_cast<const uint4*>(lds + ((lane * 4 + i * 256) & 8191));
    const uint4 vb = *reinterpret_cast<const uint4*>(lds + ((lane * 4 + i * 256 + 4096) & 8191));
    __builtin_memcpy(&a[i], &va, 16);
    __builtin_memcpy(&b[i], &vb, 16);
  }
  f32x16 acc[8];
  f32x4 acc4[32];
  i32x16 iacc[8];
  i32x4 iacc4[16];
  for (int c = 0; c < 8; ++c) acc[c] = f32x16{};
  for (int c = 0; c < 32; ++c) acc4[c] = f32x4{};
  for (int c = 0; c < 8; ++c) iacc[c] = i32x16{};
  for (int c = 0; c < 16; ++c) iacc4[c] = i32x4{};
  unsigned long long t0 = 0, r0 = 0;
  if (tid == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  const int wave = tid >> 6;
  for (int it = 0; it < iters; ++it) {
    if constexpr (LDS) {  // fresh operands from LDS each step (2 + 2 ds_read_b128 per 4 MFMA groups)
      const int base = ((it * 8 + wave) * 256 + lane * 4) & 8191;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint4 va = *reinterpret_cast<const uint4*>(lds + ((base + i * 1024) & 8191));
        const uint4 vb = *reinterpret_cast<const uint4*>(lds + ((base + i * 1024 + 512) & 8191));
        __builtin_memcpy(&a[i], &va, 16);
        __builtin_memcpy(&b[i], &vb, 16);
      }
    }
    if constexpr (SHAPE == 0) {
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[c & 3], b[(c >> 1) & 3], acc[c], 0, 0, 0);
    } else if constexpr (SHAPE == 1) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        acc4[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c & 3], b[(c >> 2) & 3], acc4[c], 0, 0, 0);
    } else if constexpr (SHAPE == 2) {
#pragma unroll
      for (int c = 0; c < 8; ++c)
        iacc[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i64x2(a[c & 3]), as_i64x2(b[(c >> 1) & 3]), iacc[c], 0, 0, 0);
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        iacc4[c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(as_i64x2(a[c & 3]), as_i64x2(b[(c >> 2) & 3]), iacc4[c], 0, 0, 0);
    }
  }
  float r = 0.f;
  for (int c = 0; c < 8; ++c)
    for (int q = 0; q < 16; ++q) r += acc[c][q];
  for (int c = 0; c < 32; ++c)
    for (int q = 0; q < 4; ++q) r += acc4[c][q];
  for (int c = 0; c < 8; ++c)
    for (int q = 0; q < 16; ++q) r += (float)iacc[c][q];
  for (int c = 0; c < 16; ++c)
    for (int q = 0; q < 4; ++q) r += (float)iacc4[c][q];
  if (tid == 0) {
    stamps[blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - t0;
    stamps[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  out[blockIdx.x * blockDim.x + tid] = r;
}

template <int SHAPE, bool LDS>
static void run(const char* name, int threads, const unsigned* in, float* out, unsigned long long* stamps, int cus) {
  // flops per loop iteration per wave: 8 x 32x32x16 = 8 x 32768, or 16 x 16x16x32 = 16 x 16384
  const double flop_it_wave = SHAPE == 0 ? 8.0 * 32768 : SHAPE == 1 ? 16.0 * 16384 : SHAPE == 2 ? 8.0 * 65536 : 16.0 * 32768;
  const int iters = 20000;
  const int waves = threads / 64;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto launch = [&]() {
    hipLaunchKernelGGL((bf16_loop<SHAPE, LDS>), dim3(cus), dim3(threads), 0, 0, in, out, stamps, iters);
  };
  const auto start = std::chrono::steady_clock::now();
  int n = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count() < 2.5) {
    launch();
    if (++n % 8 == 0) (void)hipDeviceSynchronize();
  }
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(2 * cus);
  (void)hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> ghz;
  for (int i = 0; i < cus; ++i)
    if (st[2 * i + 1]) ghz.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 0.1);  // memrealtime: 100 MHz
  std::sort(ghz.begin(), ghz.end());
  const double tf = flop_it_wave * iters * waves * cus / (ms * 1e-3) / 1e12;
  const double cyc = (SHAPE % 2) == 0 ? 32.0 : 16.0;  // cycles per MFMA per SIMD at full issue
  const double mfma_per_simd = ((SHAPE % 2) == 0 ? 8.0 : 16.0) * iters * waves / 4.0;
  const double busy = mfma_per_simd * cyc / (ghz.empty() ? 1.0 : ghz[ghz.size() / 2] * 1e9) / (ms * 1e-3);
  printf("{\"loop\": \"%s\", \"threads_per_cu\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"frac_of_2500\": %.4f, "
         "\"clock_ghz_median\": %.3f, \"clock_ghz_min\": %.3f, \"clock_ghz_max\": %.3f, \"mfma_busy_at_clock\": %.3f, "
         "\"launches_before\": %d}\n",
         name, threads, ms, tf, tf / (SHAPE >= 2 ? 5000.0 : 2500.0), ghz.empty() ? 0.0 : ghz[ghz.size() / 2], ghz.empty() ? 0.0 : ghz[0],
         ghz.empty() ? 0.0 : ghz.back(), busy, n);
  fflush(stdout);
}

int main(int argc, char** argv) {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<unsigned> h(65536);
  unsigned s = 12345u;
  for (auto& v : h) {  // random bf16 pairs in about [-1, 1], exponent varied
    s = s * 1664525u + 1013904223u;
    const unsigned lo = 0x3c00u + ((s >> 8) & 0x3ffu) | ((s >> 20) & 1u) << 15;
    s = s * 1664525u + 1013904223u;
    const unsigned hi = 0x3c00u + ((s >> 8) & 0x3ffu) | ((s >> 20) & 1u) << 15;
    v = lo | hi << 16;
  }
  unsigned* in;
  float* out;
  unsigned long long* stamps;
  (void)hipMalloc(&in, h.size() * 4);
  (void)hipMalloc(&out, (size_t)cus * 512 * 4);
  (void)hipMalloc(&stamps, (size_t)cus * 16);
  (void)hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  const bool lds_only = argc > 1 && argv[1][0] == 'l';
  const bool i8_only = argc > 1 && argv[1][0] == 'i';
  if (i8_only || argc == 1) {  // int8 (the covariance SYRK): TOPS, fraction of the 5 POPS dense peak
    run<2, false>("i8 32x32x32 regs", 512, in, out, stamps, cus);
    run<3, false>("i8 16x16x64 regs", 512, in, out, stamps, cus);
    run<2, true>("i8 32x32x32 lds", 512, in, out, stamps, cus);
    run<3, true>("i8 16x16x64 lds", 512, in, out, stamps, cus);
    if (i8_only) return 0;
  }
  if (!lds_only) {
    run<0, false>("32x32x16 regs", 512, in, out, stamps, cus);
    run<1, false>("16x16x32 regs", 512, in, out, stamps, cus);
    run<0, false>("32x32x16 regs", 256, in, out, stamps, cus);
    run<1, false>("16x16x32 regs", 256, in, out, stamps, cus);
  }
  run<0, true>("32x32x16 lds", 512, in, out, stamps, cus);
  run<1, true>("16x16x32 lds", 512, in, out, stamps, cus);
  return 0;
}
