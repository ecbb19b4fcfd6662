// Split-bf16 tall GEMM for the fit's coarse phase (ef_fit.hip subspace_wide): Y = C.Q with
// C the dim x dim covariance and Q the dim x 256 block, while the Ritz values still move by
// more than ~1e-6 (the fp64 products that follow correct whatever this phase leaves).
// Each fp32 operand x is carried as hi + lo (hi = bf16(x), lo = bf16(x - hi); |x - hi - lo|
// <= 2^-18 |x|) and x.y ~ hi.hi' + hi.lo' + lo.hi' on v_mfma_f32_16x16x32_bf16 with fp32
// accumulation: a relative error of ~2^-17 per product, at 16/3 x the fp32 MFMA rate.
// Split layout (ef_search.hip split_rows_kernel): per 8 consecutive elements, 16 B of hi
// then 16 B of lo — 4 B per element, the fp32 matrix's byte layout.
//
// Workgroup = 8 waves, output tile 256 rows x 256 columns (the whole block), K split over
// gridDim into `splits` ranges whose fp32 partial tiles are summed in a fixed order by
// gemm_s3_reduce_kernel (deterministic), which also forms Y - sigma Q in fp64.  Operand
// staging, swizzle and fragment layout are those of search_wide16_kernel
// (ef_search_wide.hip): 32-k slices of both operands by LDS-DMA, double-buffered (128 KiB),
// s(row) = (row >> 1) & 5 chunk swizzle, wave w = rows 128 (w >> 2) ..+128 x columns
// 64 (w & 3) ..+64, 96 MFMAs per 24 ds_read_b128 per slice.
#include "ef_dma.hpp"
#include "ef_linalg.hpp"

#include <algorithm>

namespace ef {

namespace {

typedef short bf16x8g __attribute__((ext_vector_type(8)));
typedef float f32x4g __attribute__((ext_vector_type(4)));

constexpr int GR = 256;   // rows per tile
constexpr int GN = 256;   // columns (the block width)
constexpr int GBK = 32;   // k per slice
constexpr int GSL = GR * GBK;  // floats per operand slice (32 KiB)

__device__ __forceinline__ bf16x8g as_bf16x8g(const float4& v) {
  bf16x8g r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}

// part[split][M][GN] = A3[rows, K range] . Bt3[:, K range]^T
__global__ __launch_bounds__(512, 1) void gemm_s3_kernel(const float* __restrict__ A3, int64_t lda,
                                                         const float* __restrict__ Bt3, int64_t ldb, int64_t M,
                                                         int64_t K, int splits, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float smem[4 * GSL];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qd = lane >> 4, r16 = lane & 15;
  const int pg = wave & 3, rh = wave >> 2;
  // XCD-aware: the workgroups of one K range share an XCD (its slice of Bt3 stays in L2)
  const int total = gridDim.x;  // host guarantees total % 8 == 0
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  const int mtiles = total / splits;
  const int split = lin / mtiles, mt = lin - split * mtiles;
  const int64_t kslices = K / GBK;
  const int64_t s0 = kslices * split / splits, s1 = kslices * (split + 1) / splits;
  const int64_t row0 = (int64_t)mt * GR;
  const int nrem = (int)(M - row0 < GR ? M - row0 : GR);

  const int prow = lane >> 3;
  unsigned goff[4], qoff[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int r = (wave * 4 + jj) * 8 + prow;
    const unsigned lch16 = (unsigned)(((lane & 7) ^ ((4 * jj + (lane >> 4)) & 5)) * 16);
    const int ra = r < nrem ? r : nrem - 1;  // tail tile: re-read the last row (not stored)
    goff[jj] = (unsigned)ra * (unsigned)(lda * 4) + lch16;
    qoff[jj] = (unsigned)r * (unsigned)(ldb * 4) + lch16;
  }
  const unsigned lds_base = lds_addr(smem);
  auto issue = [&](int64_t sl, int buf) {
    const unsigned long long ab = (unsigned long long)(size_t)(A3 + row0 * lda + sl * GBK);
    const unsigned long long bb = (unsigned long long)(size_t)(Bt3 + sl * GBK);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = wave * 4 + jj;
      glds16s(goff[jj], ab, lds_base + (unsigned)((buf * 2 * GSL + j * 256) * 4));
      glds16s(qoff[jj], bb, lds_base + (unsigned)((buf * 2 * GSL + GSL + j * 256) * 4));
    }
  };

  f32x4g acc[8][4];
#pragma unroll
  for (int rb = 0; rb < 8; ++rb)
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) acc[rb][pb] = f32x4g{0.f, 0.f, 0.f, 0.f};

  if (s0 < s1) issue(s0, 0);
  dma_wait_all();
  __syncthreads();
  const int sw = (r16 >> 1) & 5;
  const int ph = ((2 * qd) ^ sw) * 4, pl = ((2 * qd + 1) ^ sw) * 4;
  for (int64_t sl = s0; sl < s1; ++sl) {
    const int buf = (int)((sl - s0) & 1);
    const bool more = sl + 1 < s1;
    if (more && wave < 4) issue(sl + 1, buf ^ 1);  // staggered as in search_wide16_kernel
    const float* sa = smem + buf * 2 * GSL + (128 * rh + r16) * GBK;
    const float* sb = smem + buf * 2 * GSL + GSL + (64 * pg + r16) * GBK;
    bf16x8g bh[4], bl[4];
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      bh[pb] = as_bf16x8g(*reinterpret_cast<const float4*>(sb + 16 * pb * GBK + ph));
      bl[pb] = as_bf16x8g(*reinterpret_cast<const float4*>(sb + 16 * pb * GBK + pl));
    }
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const bf16x8g ah = as_bf16x8g(*reinterpret_cast<const float4*>(sa + 16 * rb * GBK + ph));
      const bf16x8g al = as_bf16x8g(*reinterpret_cast<const float4*>(sa + 16 * rb * GBK + pl));
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[pb], acc[rb][pb], 0, 0, 0);
        acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[pb], acc[rb][pb], 0, 0, 0);
        acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[pb], acc[rb][pb], 0, 0, 0);
      }
      if (rb == 1 && more && wave >= 4) issue(sl + 1, buf ^ 1);
    }
    dma_wait_all();
    __syncthreads();
  }
  // acc[rb][pb][r] = row 128 rh + 16 rb + 4 qd + r, column 64 pg + 16 pb + r16
  float* out = part + (int64_t)split * M * GN;
#pragma unroll
  for (int rb = 0; rb < 8; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 128 * rh + 16 * rb + 4 * qd + r;
      if (row < nrem) {
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) out[(row0 + row) * GN + 64 * pg + 16 * pb + r16] = acc[rb][pb][r];
      }
    }
}

// Y (fp64, M x GN) = sum over splits of part (fixed order) - sigma Q
__global__ void gemm_s3_reduce_kernel(const float* __restrict__ part, int splits, int64_t n, const double* __restrict__ Q,
                                      double sigma, double* __restrict__ Y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < splits; ++p) s += part[(int64_t)p * n + i];
    Y[i] = fma(-sigma, Q[i], (double)s);
  }
}

// fp64 -> split-bf16 (hi, lo) of the fp32 value, 8 elements per thread, the split layout
__global__ void split_f64_kernel(const double* __restrict__ x, int64_t groups, uint4* __restrict__ out) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += (int64_t)gridDim.x * blockDim.x) {
    unsigned hi[8], lo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)x[g * 8 + j];
      const unsigned u = __float_as_uint(v);
      const unsigned h = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
      const float r = v - __uint_as_float(h << 16);
      const unsigned ur = __float_as_uint(r);
      hi[j] = h;
      lo[j] = (ur + 0x7fffu + ((ur >> 16) & 1u)) >> 16;
    }
    out[2 * g] = make_uint4(hi[0] | hi[1] << 16, hi[2] | hi[3] << 16, hi[4] | hi[5] << 16, hi[6] | hi[7] << 16);
    out[2 * g + 1] = make_uint4(lo[0] | lo[1] << 16, lo[2] | lo[3] << 16, lo[4] | lo[5] << 16, lo[6] | lo[7] << 16);
  }
}

// Q (dim x GN, fp64 row-major) -> Bt3 = split(Q^T) (GN x dim): 64 x 64 tiles through LDS
__global__ void transpose_split_kernel(const double* __restrict__ Q, int64_t dim, uint4* __restrict__ Bt3) {
  __shared__ float t[64][65];
  const int64_t r0 = (int64_t)blockIdx.x * 64;  // rows of Q (k)
  const int c0 = blockIdx.y * 64;                // columns of Q (output rows)
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) {
    const int rr = e >> 6, cc = e & 63;
    t[cc][rr] = r0 + rr < dim ? (float)Q[(r0 + rr) * GN + c0 + cc] : 0.f;
  }
  __syncthreads();
  // 64 output rows x 8 groups of 8 k
  for (int e = threadIdx.x; e < 64 * 8; e += blockDim.x) {
    const int orow = e >> 3, grp = e & 7;
    if (r0 + grp * 8 >= dim) continue;
    unsigned hi[8], lo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = t[orow][grp * 8 + j];
      const unsigned u = __float_as_uint(v);
      const unsigned h = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
      const float rsd = v - __uint_as_float(h << 16);
      const unsigned ur = __float_as_uint(rsd);
      hi[j] = h;
      lo[j] = (ur + 0x7fffu + ((ur >> 16) & 1u)) >> 16;
    }
    const int64_t g = ((int64_t)(c0 + orow) * dim + r0) / 8 + grp;
    Bt3[2 * g] = make_uint4(hi[0] | hi[1] << 16, hi[2] | hi[3] << 16, hi[4] | hi[5] << 16, hi[6] | hi[7] << 16);
    Bt3[2 * g + 1] = make_uint4(lo[0] | lo[1] << 16, lo[2] | lo[3] << 16, lo[4] | lo[5] << 16, lo[6] | lo[7] << 16);
  }
}

}  // namespace

bool gemm_s3_supported(int64_t M, int64_t K, int64_t N) {
  // 32-bit per-lane DMA offsets: 256 rows of a K-float row (A3 and Bt3 rows are K long)
  return N == GN && M >= GR && K % GBK == 0 && K >= GBK && (int64_t)GR * K * 4 < (1ll << 32);
}

int gemm_s3_splits(int64_t M) {
  const int64_t mt = (M + GR - 1) / GR;
  int s = (int)std::max<int64_t>(1, (256 + mt - 1) / mt);  // ~256 workgroups: one per CU
  while ((mt * s) % 8) ++s;
  return s;
}

size_t gemm_s3_part_elems(int64_t M) { return (size_t)gemm_s3_splits(M) * ((M + GR - 1) / GR) * GR * GN; }

hipError_t launch_split_f64(hipStream_t s, const double* x, int64_t n, void* out) {
  const int64_t groups = n / 8;
  hipLaunchKernelGGL(split_f64_kernel, dim3((unsigned)std::min<int64_t>((groups + 255) / 256, 16384)), dim3(256), 0,
                     s, x, groups, static_cast<uint4*>(out));
  return hipGetLastError();
}

hipError_t launch_transpose_split(hipStream_t s, const double* Q, int64_t dim, void* Bt3) {
  hipLaunchKernelGGL(transpose_split_kernel, dim3((unsigned)((dim + 63) / 64), GN / 64), dim3(256), 0, s, Q, dim,
                     static_cast<uint4*>(Bt3));
  return hipGetLastError();
}

hipError_t gemm_s3(hipStream_t s, const float* A3, int64_t lda, const float* Bt3, int64_t ldb, int64_t M, int64_t K,
                   float* part, const double* Q, double sigma, double* Y) {
  const int splits = gemm_s3_splits(M);
  const int64_t mt = (M + GR - 1) / GR;
  hipLaunchKernelGGL(gemm_s3_kernel, dim3((unsigned)(mt * splits)), dim3(512), 0, s, A3, lda, Bt3, ldb, M, K, splits,
                     part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t n = M * GN;
  hipLaunchKernelGGL(gemm_s3_reduce_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 16384)), dim3(256), 0,
                     s, part, splits, n, Q, sigma, Y);
  return hipGetLastError();
}

}  // namespace ef
