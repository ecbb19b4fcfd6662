// Exact covariance / Gram of uint8 faces on the int8 matrix cores (fit K3).
//
// The fit's dominant GEMM (useless/train.py:82-85 Gram A.A^T when n < d; the np.cov
// branch :97-99 / sklearn's SVD of the centred matrix otherwise) has integer inputs.
// Shifting pixels by -128 maps them exactly onto int8, and the shift cancels in the
// centred product:
//   covariance (n >= d):  (n-1) n C_ij = n S'_ij - c_i c_j,           S' = X'^T X'
//   Gram       (n <  d):  (n-1) n^2 C_ij = n^2 S'_ij - n (R_i + R_j) + Q,   S' = X' X'^T
// with X' = X - 128, c = column sums of X', R_i = X'_i . c, Q = c . c — all exact
// integers.  S' runs on v_mfma_i32_32x32x32_i8 with int32 accumulators flushed into an
// int64 tile every 65536 samples (|x'| <= 128: 65536 * 128^2 = 2^30 fits), so the only
// rounding of the whole covariance is the final int128 -> fp64 conversion and division
// (<= 1 ulp), tighter than the fp64 GEMM the reference runs.  StandardScaler scaling
// (train-v4.py:131) is applied afterwards as C_ij / (scale_i scale_j).
//
// SYRK kernel: 256 x 256 output tile per workgroup (upper triangle of tiles only), 8 waves
// of 128 x 64, K-slices of 64 samples staged by global_load_lds into a 4-stage LDS ring
// (4 x 32 KiB, three stages in flight), 64-B rows XOR-swizzled by ((row >> 2) & 3) so the
// ds_read_b128 fragment reads are conflict-free.  Operands come from a K-contiguous int8 copy At (dim x Kpad):
// X' itself for the Gram path, its transpose for the covariance path.
#include <vector>

#include "ef_dma.hpp"
#include "ef_linalg.hpp"

namespace ef {

typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int YT = 256;                 // output tile (rows and columns)
constexpr int YK = 64;                  // samples per stage
constexpr int YSL = YT * YK;            // bytes per operand stage
constexpr int YNB = 4;                  // LDS stages in the ring (prefetch distance YNB - 1)
constexpr int64_t kFlushK = 65536;      // int32-safe accumulation length

// At[r][k] = X[r][k] - 128 (Gram path: rows = samples), zero for k >= d.
__global__ void shift_copy_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d, int64_t ldk,
                                  uint8_t* __restrict__ At) {
  const int64_t r = blockIdx.y;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < ldk; k += (int64_t)gridDim.x * blockDim.x)
    At[r * ldk + k] = k < d ? (uint8_t)(X[r * d + k] ^ 0x80u) : (uint8_t)0;
}

// At[c][k] = X[k][c] - 128 (covariance path: rows = pixels), zero for k >= n; 64x64 tiles.
__global__ void shift_transpose_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d, int64_t ldk,
                                       uint8_t* __restrict__ At) {
  __shared__ uint8_t t[64][65];
  const int64_t k0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: 4 rows per pass
  for (int r = ty; r < 64; r += 4) {
    const int64_t k = k0 + r, c = c0 + tx;
    t[r][tx] = (k < n && c < d) ? (uint8_t)(X[k * d + c] ^ 0x80u) : (uint8_t)0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int64_t c = c0 + r, k = k0 + tx;
    if (c < d && k < ldk) At[c * ldk + k] = t[tx][r];
  }
}

// S64[i][j] = sum_k At[i][k] At[j][k] for the upper triangle of 256-tiles (i-tile <= j-tile).
__global__ __launch_bounds__(512, 1) void syrk_i8_kernel(const uint8_t* __restrict__ At, int64_t dim, int64_t ldk,
                                                         int64_t kpad, int ntiles, const int2* __restrict__ order,
                                                         long long* __restrict__ S64) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[YNB * 2 * YSL];  // [stage][A | B], 128 KiB
  const int total = gridDim.x;  // multiple of 8; trailing blocks are idle padding
  // consecutive list entries run on one XCD (blocks b and b+8 share an XCD), and the
  // host orders the list in 4 x 8 blocks of tiles, so the ~32 workgroups an XCD runs at
  // once read 4 row panels and 8 column panels: most panel bytes hit its L2
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  if (lin >= ntiles) return;
  const int2 tt = order[lin];
  const int ti = tt.x, tj = tt.y;
  const int64_t i0 = (int64_t)ti * YT, j0 = (int64_t)tj * YT;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 2, wn = wave & 3;  // 2 x 4 waves of 128 x 64

  // DMA: a stage = 16 pieces of 1 KiB (16 rows x 64 B) per operand; wave w issues
  // pieces 2w, 2w+1 of A and of B.  Lane l -> row 16j + (l >> 2), physical chunk l & 3
  // holding logical chunk (l & 3) ^ ((l >> 4) & 3).
  const unsigned lds_base = lds_addr(smem);
  const int lrow = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lane >> 4) & 3);
  auto issue = [&](int64_t k0, int buf) {
    int lr = lrow, lc = lchunk;
    asm volatile("" : "+v"(lr), "+v"(lc));
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wave * 2 + jj;
      int64_t ra = i0 + j * 16 + lr, rb = j0 + j * 16 + lr;
      ra = ra < dim ? ra : dim - 1;
      rb = rb < dim ? rb : dim - 1;
      glds16(At + ra * ldk + k0 + lc * 16, lds_base + (unsigned)(buf * 2 * YSL + j * 1024));
      glds16(At + rb * ldk + k0 + lc * 16, lds_base + (unsigned)(buf * 2 * YSL + YSL + j * 1024));
    }
  };

  i32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = i32x16{};

  auto flush = [&]() {  // WG-owned tile: plain read-modify-write of the int64 output
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t col = j0 + wn * 64 + j * 32 + c32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = i0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row < dim && col < dim) S64[row * dim + col] += (long long)acc[i][j][r];
          acc[i][j][r] = 0;
        }
      }
  };

  const int sw = (c32 >> 2) & 3;  // swizzle key of every row this lane reads
  const int64_t nst = kpad / YK;
  // ring of YNB stages, YNB - 1 in flight ahead of the one being consumed (an HBM miss is
  // several stages of MFMA time); each stage is 4 DMA instructions per wave, so "stage st
  // landed" is vmcnt <= 4 x (stages issued after it).  Tail stages past nst are issued as
  // harmless re-reads of stage 0 so the count stays uniform.
  for (int j = 0; j < YNB - 1; ++j) issue((j < nst ? j : 0) * YK, j);
  for (int64_t st = 0; st < nst; ++st) {
    const int buf = (int)(st % YNB);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // stage st landed (2 newer stages pending)
    __syncthreads();                                   // ... for every wave; stage st-1 consumed
    {
      const int64_t nx = st + YNB - 1;
      issue((nx < nst ? nx : 0) * YK, (int)(nx % YNB));
    }
    const uint8_t* sa = smem + buf * 2 * YSL;
    const uint8_t* sb = sa + YSL;
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // lane (r, h) holds A[r][32s + 16h + j], B[32s + 16h + j][r]
      const int pch = ((2 * s + h) ^ sw) * 16;
      i32x4 a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const i32x4*>(sa + (wm * 128 + i * 32 + c32) * YK + pch);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const i32x4*>(sb + (wn * 64 + j * 32 + c32) * YK + pch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (((st + 1) * YK) % kFlushK == 0 && st + 1 < nst) flush();
  }
  dma_wait_all();
  flush();
}

// R[r] = sum_k At[r][k] * c[k]   (Gram path; exact in int64)
__global__ void rowdot_kernel(const uint8_t* __restrict__ At, int64_t rows, int64_t ldk, int64_t d,
                              const long long* __restrict__ c, long long* __restrict__ R) {
  const int64_t r = blockIdx.x;
  long long s = 0;
  for (int64_t k = threadIdx.x; k < d; k += blockDim.x) s += (long long)(int8_t)At[r * ldk + k] * c[k];
  __shared__ long long red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) R[r] = red[0];
}

// c'[j] = S1[j] - 128 n, and Q = sum_j c'[j]^2 (Gram path) in int128 halves.
__global__ void shifted_sums_kernel(const unsigned long long* __restrict__ S1, int64_t n, int64_t d,
                                    long long* __restrict__ c) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < d) c[j] = (long long)S1[j] - 128LL * n;
}

__global__ void sumsq128_kernel(const long long* __restrict__ c, int64_t d, unsigned long long* __restrict__ out) {
  __shared__ unsigned __int128 red[256];
  unsigned __int128 s = 0;
  for (int64_t j = threadIdx.x; j < d; j += blockDim.x) {
    const __int128 v = c[j];
    s += (unsigned __int128)(v * v);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = (unsigned long long)red[0];
    out[1] = (unsigned long long)(red[0] >> 64);
  }
}

// C[i][j] from the exact integer pieces (one rounding); w = 1/scale or null.
__global__ void cov_finalize_kernel(const long long* __restrict__ S64, int64_t dim, int64_t n, int gram,
                                    const long long* __restrict__ cvec, const long long* __restrict__ R,
                                    const unsigned long long* __restrict__ Q2, const double* __restrict__ w,
                                    double* __restrict__ C) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= dim * dim) return;
  const int64_t i = e / dim, j = e - (e / dim) * dim;
  const bool upper = (i / YT) <= (j / YT);
  const __int128 s = upper ? S64[i * dim + j] : S64[j * dim + i];
  const __int128 nn = n;
  double v;
  if (gram) {
    const __int128 q = (__int128)(((unsigned __int128)Q2[1] << 64) | Q2[0]);
    const __int128 num = nn * nn * s - nn * ((__int128)R[i] + R[j]) + q;
    v = (double)num / ((double)n * (double)n * (double)(n - 1));
  } else {
    const __int128 num = nn * s - (__int128)cvec[i] * cvec[j];
    v = (double)num / ((double)n * (double)(n - 1));
  }
  if (w) v *= w[i] * w[j];
  C[e] = v;
}

int64_t cov_i8_kpad(int64_t K) { return (K + YK - 1) / YK * YK; }

int64_t cov_i8_order_bytes(int64_t dim) {
  const int64_t t = (dim + YT - 1) / YT;
  return t * (t + 1) / 2 * (int64_t)sizeof(int2) + 64;
}

hipError_t launch_cov_i8(hipStream_t s, const uint8_t* X, int64_t n, int64_t d, bool gram,
                         const unsigned long long* S1, const double* w, uint8_t* At, long long* S64,
                         long long* cvec, long long* R, unsigned long long* Q2, void* order_dev, double* C) {
  const int64_t dim = gram ? n : d;
  const int64_t K = gram ? d : n;
  const int64_t kpad = cov_i8_kpad(K);
  if (gram) {
    hipLaunchKernelGGL(shift_copy_kernel, dim3((unsigned)((kpad + 255) / 256 < 64 ? (kpad + 255) / 256 : 64),
                                               (unsigned)n),
                       dim3(256), 0, s, X, n, d, kpad, At);
  } else {
    hipLaunchKernelGGL(shift_transpose_kernel, dim3((unsigned)(kpad / 64), (unsigned)((d + 63) / 64)), dim3(256), 0,
                       s, X, n, d, kpad, At);
  }
  hipError_t e = hipMemsetAsync(S64, 0, (size_t)dim * dim * sizeof(long long), s);
  if (e != hipSuccess) return e;
  const int ntile = (int)((dim + YT - 1) / YT);
  // upper-triangle tiles in 4 x 8 blocks (L2 reuse within an XCD), one H2D of the list
  std::vector<int2> order;
  for (int bi = 0; bi < ntile; bi += 4)
    for (int bj = bi / 8 * 8; bj < ntile; bj += 8)
      for (int ti = bi; ti < bi + 4 && ti < ntile; ++ti)
        for (int tj = bj; tj < bj + 8 && tj < ntile; ++tj)
          if (ti <= tj) order.push_back(make_int2(ti, tj));
  const int ntiles = (int)order.size();
  const int grid = (ntiles + 7) / 8 * 8;
  e = hipMemcpyAsync(order_dev, order.data(), order.size() * sizeof(int2), hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(syrk_i8_kernel, dim3((unsigned)grid), dim3(512), 0, s, At, dim, kpad, kpad, ntiles,
                     static_cast<const int2*>(order_dev), S64);
  e = hipStreamSynchronize(s);  // the host list must outlive the copy
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(shifted_sums_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, S1, n, d, cvec);
  if (gram) {
    hipLaunchKernelGGL(rowdot_kernel, dim3((unsigned)n), dim3(256), 0, s, At, n, kpad, d, cvec, R);
    hipLaunchKernelGGL(sumsq128_kernel, dim3(1), dim3(256), 0, s, cvec, d, Q2);
  }
  const int64_t tot = dim * dim;
  hipLaunchKernelGGL(cov_finalize_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, S64, dim, n,
                     gram ? 1 : 0, cvec, R, Q2, w, C);
  return hipGetLastError();
}

}  // namespace ef
