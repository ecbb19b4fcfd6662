// bf16 probe projection (BASELINE.json config 5: 256x256 faces, k = 512, "bf16 projection
// (CDNA4 bf16 MFMA) with fp32 distance accumulate").
//
// f = (p - mean).W is evaluated as  (p - round(mean)).W16  -  (mean - round(mean)).W
//   * p - round(mean) is an integer in [-255, 255] for uint8 pixels, exact in bf16, so the
//     only rounding of the GEMM inputs is W -> W16 (bf16, round-to-nearest-even);
//   * the correction row (mean - round(mean)).W is computed once per model in fp64;
//   * accumulation is fp32 on v_mfma_f32_32x32x16_bf16; the features and everything
//     after them (gallery search, arg-best) stay fp32 / fp64-resolved.
// Error vs the fp32 projection: |f16 - f| <= 2^-8 * sum_px |p - round(mean)| |W| (stated
// and tested in tests/test_gpu_project.py).
//
// GEMM M = probes, N = components (128-column tiles over gridDim.z), K = pixels, split-K
// over gridDim.y into fp32 slabs reduced by project_reduce_kernel (ef_project.hip), the
// same slab contract as the fp32 kernel.  Workgroup tile 128 probes x 128 components,
// 4 waves of 64 x 64, BK = 32 pixels per stage (two 16-deep MFMA steps), LDS rows padded
// to 80 B so the ds_read_b128 fragment reads are conflict-free.
#include "ef_internal.hpp"

namespace ef {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int HM = 128;      // probes per workgroup
constexpr int HN = 128;      // components per workgroup
constexpr int HK = 32;       // pixels per stage
constexpr int HS = HK + 8;   // LDS row stride in bf16 elements (80 B)

__device__ __forceinline__ unsigned bf16_bits(float x) {  // round to nearest even (finite x)
  const unsigned u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ unsigned pack2(float lo, float hi) { return bf16_bits(lo) | (bf16_bits(hi) << 16); }

template <int PDT, bool VEC>
__global__ __launch_bounds__(256, 2) void project_bf16_kernel(const void* __restrict__ Pv, int64_t b, int64_t d,
                                                              const float* __restrict__ mean_r,
                                                              const unsigned short* __restrict__ Wt16, int ldw,
                                                              float* __restrict__ part, int64_t bpad,
                                                              int64_t pix_per_split) {
  __shared__ __attribute__((aligned(16))) unsigned short sA[2][HM * HS];
  __shared__ __attribute__((aligned(16))) unsigned short sB[2][HN * HS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * HM;
  const int col0 = blockIdx.z * HN;
  const int64_t k_beg = (int64_t)blockIdx.y * pix_per_split;
  const int64_t k_end = k_beg + pix_per_split < d ? k_beg + pix_per_split : d;
  const int nsteps = (int)((k_end - k_beg + HK - 1) / HK);

  // staging: thread -> (row | column, 16-pixel half)
  const int sr = tid >> 1, sh = (tid & 1) * 16;
  uint4 av[2], bv[2];

  auto load_stage = [&](int step) {
    const int64_t px0 = k_beg + (int64_t)step * HK + sh;
    const int64_t row = m0 + sr;
    float v[16];
    if constexpr (PDT == EF_U8) {
      const uint8_t* P = reinterpret_cast<const uint8_t*>(Pv);
      if (VEC && row < b && px0 + 16 <= k_end) {
        const uint4 raw = *reinterpret_cast<const uint4*>(P + row * d + px0);
        const unsigned w4[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = (float)((w4[j >> 2] >> (8 * (j & 3))) & 0xffu);
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = (row < b && px0 + j < k_end) ? (float)P[row * d + px0 + j] : 0.f;
      }
    } else {
      const float* P = reinterpret_cast<const float*>(Pv);
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = (row < b && px0 + j < k_end) ? P[row * d + px0 + j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (row < b && px0 + j < k_end) v[j] -= mean_r[px0 + j];
    av[0] = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
    av[1] = make_uint4(pack2(v[8], v[9]), pack2(v[10], v[11]), pack2(v[12], v[13]), pack2(v[14], v[15]));
    // W16 is [ldw][d] (pixels contiguous per component): 32 B per thread
    const unsigned short* wrow = Wt16 + (int64_t)(col0 + sr) * d;
    if (VEC && px0 + 16 <= k_end) {
      bv[0] = *reinterpret_cast<const uint4*>(wrow + px0);
      bv[1] = *reinterpret_cast<const uint4*>(wrow + px0 + 8);
    } else {
      unsigned w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned lo = px0 + 2 * j < k_end ? wrow[px0 + 2 * j] : 0u;
        const unsigned hi = px0 + 2 * j + 1 < k_end ? wrow[px0 + 2 * j + 1] : 0u;
        w[j] = lo | (hi << 16);
      }
      bv[0] = make_uint4(w[0], w[1], w[2], w[3]);
      bv[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
  };
  auto store_stage = [&](int buf) {
    *reinterpret_cast<uint4*>(&sA[buf][sr * HS + sh]) = av[0];
    *reinterpret_cast<uint4*>(&sA[buf][sr * HS + sh + 8]) = av[1];
    *reinterpret_cast<uint4*>(&sB[buf][sr * HS + sh]) = bv[0];
    *reinterpret_cast<uint4*>(&sB[buf][sr * HS + sh + 8]) = bv[1];
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  if (nsteps > 0) {
    load_stage(0);
    store_stage(0);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const bool more = st + 1 < nsteps;
    if (more) load_stage(st + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // lane (r, h) holds A[r][16s + 8h + j], B[16s + 8h + j][r]
      bf16x8 a[2], w[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&sA[buf][(wm * 64 + i * 32 + c32) * HS + 16 * s + 8 * h]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        w[j] = *reinterpret_cast<const bf16x8*>(&sB[buf][(wn * 64 + j * 32 + c32) * HS + 16 * s + 8 * h]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], w[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_stage(buf ^ 1);
    __syncthreads();
  }

  float* out = part + (int64_t)blockIdx.y * bpad * ldw + col0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[row * ldw + wn * 64 + j * 32 + c32] = acc[i][j][r];
      }
}

// Wt16[c][px] = bf16(W[px][c]) (32 x 32 tiles through LDS), mean_r = round(mean).
__global__ void bf16_model_kernel(const float* __restrict__ W, const float* __restrict__ mean, int64_t d, int ldw,
                                  unsigned short* __restrict__ Wt16, float* __restrict__ mean_r) {
  __shared__ float t[32][33];
  const int64_t p0 = (int64_t)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int64_t px = p0 + r;
    t[r][tx] = px < d ? W[px * ldw + c0 + tx] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t px = p0 + tx;
    if (px < d) Wt16[(int64_t)(c0 + r) * d + px] = (unsigned short)bf16_bits(t[tx][r]);
  }
  if (blockIdx.y == 0 && threadIdx.x < 32 && p0 + threadIdx.x < d) mean_r[p0 + threadIdx.x] = rintf(mean[p0 + threadIdx.x]);
}

// corr_part[chunk][c] = sum over the chunk's pixels of (mean - round(mean)) W[px][c] (fp64).
__global__ void bf16_corr_kernel(const float* __restrict__ W, const float* __restrict__ mean, int64_t d, int ldw,
                                 int64_t chunk, double* __restrict__ corr_part) {
  const int c = threadIdx.x + blockIdx.y * blockDim.x;
  if (c >= ldw) return;
  const int64_t a = (int64_t)blockIdx.x * chunk;
  const int64_t e = a + chunk < d ? a + chunk : d;
  double s = 0.0;
  for (int64_t px = a; px < e; ++px) s += ((double)mean[px] - (double)rintf(mean[px])) * (double)W[px * ldw + c];
  corr_part[(int64_t)blockIdx.x * ldw + c] = s;
}

__global__ void bf16_corr_sum_kernel(const double* __restrict__ corr_part, int nchunk, int ldw, float* __restrict__ corr) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ldw) return;
  double s = 0.0;
  for (int z = 0; z < nchunk; ++z) s += corr_part[(int64_t)z * ldw + c];
  corr[c] = (float)s;
}

hipError_t launch_bf16_model(hipStream_t s, const float* W, const float* mean, int64_t d, int ldw,
                             unsigned short* Wt16, float* mean_r, float* corr, double* corr_part, int nchunk) {
  hipLaunchKernelGGL(bf16_model_kernel, dim3((unsigned)((d + 31) / 32), (unsigned)(ldw / 32)), dim3(256), 0, s, W,
                     mean, d, ldw, Wt16, mean_r);
  const int64_t chunk = (d + nchunk - 1) / nchunk;
  hipLaunchKernelGGL(bf16_corr_kernel, dim3((unsigned)nchunk, (unsigned)((ldw + 127) / 128)), dim3(128), 0, s, W,
                     mean, d, ldw, chunk, corr_part);
  hipLaunchKernelGGL(bf16_corr_sum_kernel, dim3((unsigned)((ldw + 127) / 128)), dim3(128), 0, s, corr_part, nchunk,
                     ldw, corr);
  return hipGetLastError();
}

int project_bf16_nsplit(int64_t bpad, int64_t d, int ldw, int64_t* pix_per_split) {
  const int64_t tiles = bpad / HM * ((ldw + HN - 1) / HN);
  int64_t ns = (512 + tiles - 1) / tiles;  // ~2 workgroups per CU
  const int64_t steps = (d + HK - 1) / HK;
  if (ns > steps) ns = steps;
  if (ns < 1) ns = 1;
  if (ns > 64) ns = 64;
  const int64_t steps_per = (steps + ns - 1) / ns;
  *pix_per_split = steps_per * HK;
  return (int)((d + *pix_per_split - 1) / *pix_per_split);
}

hipError_t launch_project_bf16(hipStream_t s, int p_dtype, const void* P, int64_t b, int64_t bpad, int64_t d,
                               const float* mean_r, const unsigned short* Wt16, int ldw, float* part, int nsplit,
                               int64_t pps) {
  if (ldw % HN != 0) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(bpad / HM), (unsigned)nsplit, (unsigned)(ldw / HN));
  const bool vec = (d % 16 == 0) && (pps % 16 == 0) && ((reinterpret_cast<uintptr_t>(P) & 15) == 0);
  if (p_dtype == EF_U8) {
    if (vec)
      hipLaunchKernelGGL((project_bf16_kernel<EF_U8, true>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw, part,
                         bpad, pps);
    else
      hipLaunchKernelGGL((project_bf16_kernel<EF_U8, false>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw,
                         part, bpad, pps);
  } else {
    if (vec)
      hipLaunchKernelGGL((project_bf16_kernel<EF_F32, true>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw,
                         part, bpad, pps);
    else
      hipLaunchKernelGGL((project_bf16_kernel<EF_F32, false>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw,
                         part, bpad, pps);
  }
  return hipGetLastError();
}

}  // namespace ef
