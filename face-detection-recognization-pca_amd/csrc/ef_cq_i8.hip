// The fit's fine-phase products Y = C.Q - sigma Q (fp64 accuracy) on the int8 matrix cores,
// by exact digit splitting (Ozaki-style).  fp64 MFMA peaks at 1/64 of the int8 rate, and the
// fp64 product already ran at 95 % of its issue ceiling (ef_dgemm.hip), so:
//   * each row i of the symmetric C (dim x dim) is scaled by 2^t_i so that its largest entry
//     lies in [2^45, 2^46), each column c of Q (dim x 256) by 2^u_c likewise; both are
//     rounded to integers and cut into 6 signed base-256 digits (a, b = 0 least significant);
//   * every digit pair whose weight 256^(a+b) is within 2^-40 of the top (a + b >= 5: 21 of
//     36) is an exact int32 product (|.| <= dim 2^14) on the covariance SYRK's
//     v_mfma_i32_16x16x64_i8 kernel (ef_cov_i8.hip syrk16_i8_kernel, OZ items of 256 x 256);
//   * oz_combine_kernel adds the pair products by level in exact int64, one fp64 Horner step
//     per level, and applies 2^-(t_i + u_c) and the shift -sigma Q.
// Error: the two roundings (2^-46 of the row / column maximum) and the dropped levels,
// the order of an fp64 GEMM's own dim x 2^-53 (useless/train.py:88 computes eigh in fp64).
// The medium form (15 pairs: a, b >= 1, a + b >= 6; ~2^-40 of the product) serves the
// products whose errors later products damp: ef_fit uses it for every fine product that is
// neither read by a Rayleigh-Ritz step nor the one before it.
//
// Operand layout: one K-blocked int8 array [dim / 64][R][64] (the SYRK's At layout),
// R = 6 dim + 6 x 256 rows: C's digit plane a at rows a dim + i, Q's digit b at rows
// 6 dim + 256 b + c.  C's planes are written once per fit (C does not change), Q's digits
// every product.
#include <cmath>

#include "ef_linalg.hpp"

namespace ef {

namespace {

constexpr int kOzDigits = 6;
constexpr int kOzTop = 46;  // largest scaled entry in [2^45, 2^46): 6 signed base-256 digits
constexpr int kOzQ = 256;   // Q's columns (the block width of the subspace iteration)
constexpr int kZK = 64;     // K bytes per block of the layout

__host__ __device__ inline int64_t oz_rows(int64_t dim) { return kOzDigits * dim + kOzDigits * kOzQ; }

// V = rint(2^t x) -> 6 signed base-256 digits, byte j of the packed words = digit of
// element j (low digit first; the top digit absorbs the sign)
__device__ __forceinline__ void oz_digits(double x, int t, unsigned (&w)[kOzDigits], int shift) {
  long long v = (long long)rint(ldexp(x, t));
#pragma unroll
  for (int a = 0; a < kOzDigits; ++a) {
    const long long lo = ((v + 128) & 255) - 128;
    w[a] |= (unsigned)(lo & 255) << shift;
    v = (v - lo) / 256;
  }
}

// C's row digit planes: one block per row i; the row maximum gives t_i; 8 columns per
// thread and step written as one 8-byte piece of each plane's K block.
__global__ __launch_bounds__(256) void oz_rows_kernel(const double* __restrict__ C, int64_t dim,
                                                      int8_t* __restrict__ Z, int* __restrict__ tr) {
  const int64_t i = blockIdx.x;
  const double* row = C + i * dim;
  double mx = 0.0;
  for (int64_t k = threadIdx.x; k < dim; k += 256) mx = fmax(mx, fabs(row[k]));
  __shared__ double red[256];
  __shared__ int tsh;
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int e = 0;
    if (red[0] > 0.0) (void)frexp(red[0], &e);
    tsh = red[0] > 0.0 ? kOzTop - e : 0;
    tr[i] = tsh;
  }
  __syncthreads();
  const int t = tsh;
  const int64_t R = oz_rows(dim);
  for (int64_t k0 = (int64_t)threadIdx.x * 8; k0 < dim; k0 += 256 * 8) {
    unsigned lo[kOzDigits], hi[kOzDigits];
#pragma unroll
    for (int a = 0; a < kOzDigits; ++a) lo[a] = hi[a] = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) oz_digits(row[k0 + q], t, lo, 8 * q);
#pragma unroll
    for (int q = 0; q < 4; ++q) oz_digits(row[k0 + 4 + q], t, hi, 8 * q);
    int8_t* base = Z + ((k0 / kZK) * R + i) * kZK + (k0 % kZK);
#pragma unroll
    for (int a = 0; a < kOzDigits; ++a) *reinterpret_cast<uint2*>(base + a * dim * kZK) = make_uint2(lo[a], hi[a]);
  }
}

// Column maxima of Q (dim x 256): block b folds 16 rows, merged by atomicMax on the bits
// (non-negative doubles order as their bit patterns); cmax zeroed before.
__global__ __launch_bounds__(256) void oz_colmax_kernel(const double* __restrict__ Q, int64_t dim,
                                                        unsigned long long* __restrict__ cmax) {
  const int c = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  double mx = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) mx = fmax(mx, fabs(Q[(r0 + q) * kOzQ + c]));
  atomicMax(cmax + c, (unsigned long long)__double_as_longlong(mx));
}

// Q's column digits: thread c of block b takes rows 16 b .. 16 b + 15 of column c (loads
// coalesced along c) and writes each digit's 16 bytes as one piece of its K block.
__global__ __launch_bounds__(256) void oz_qdigits_kernel(const double* __restrict__ Q, int64_t dim,
                                                         const unsigned long long* __restrict__ cmax,
                                                         int8_t* __restrict__ Z, int* __restrict__ tc) {
  const int c = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  const double mx = __longlong_as_double((long long)cmax[c]);
  int e = 0;
  if (mx > 0.0) (void)frexp(mx, &e);
  const int t = mx > 0.0 ? kOzTop - e : 0;
  if (blockIdx.x == 0) tc[c] = t;
  unsigned w[4][kOzDigits];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int j = 0; j < kOzDigits; ++j) w[g][j] = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) oz_digits(Q[(r0 + 4 * g + q) * kOzQ + c], t, w[g], 8 * q);
  }
  const int64_t R = oz_rows(dim);
  int8_t* base = Z + ((r0 / kZK) * R + kOzDigits * dim + c) * kZK + (r0 % kZK);
#pragma unroll
  for (int j = 0; j < kOzDigits; ++j)
    *reinterpret_cast<uint4*>(base + (int64_t)j * kOzQ * kZK) = make_uint4(w[0][j], w[1][j], w[2][j], w[3][j]);
}

// Y[i][c] = 2^(8 lev - t_i - u_c) sum_L 256^L S_L - sigma Q[i][c]: S_L the exact int64 sum
// of the pair products of level a + b = L + lev (lev = 5 full, 6 medium), in the block
// order of syrk16_i8_kernel's OZ items (oz_pair, then the K-parts of the last pair); fp64
// Horner from the top level.
template <bool MED>
__global__ __launch_bounds__(256) void oz_combine_kernel(const int* __restrict__ I, int64_t dim,
                                                         const int* __restrict__ tr, const int* __restrict__ tc,
                                                         const double* __restrict__ Q, double sigma,
                                                         double* __restrict__ Y) {
  constexpr int lev = MED ? 6 : 5, nlev = 11 - lev, np = oz_pairs(MED);
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = dim * kOzQ;
  if (e >= total) return;
  const int64_t i = e / kOzQ;
  const int c = (int)(e - i * kOzQ);
  long long S[nlev];
#pragma unroll
  for (int L = 0; L < nlev; ++L) S[L] = 0;
#pragma unroll
  for (int p = 0; p < np - 1; ++p) {
    int a = 0, b = 0;
    oz_pair(p, MED, a, b);
    S[a + b - lev] += I[(int64_t)p * total + e];
  }
#pragma unroll
  for (int q = 0; q < kOzSplitParts; ++q) S[0] += I[(int64_t)(np - 1 + q) * total + e];  // the lowest level
  double v = (double)S[nlev - 1];
#pragma unroll
  for (int L = nlev - 2; L >= 0; --L) v = fma(v, 256.0, (double)S[L]);
  Y[e] = fma(-sigma, Q[e], ldexp(v, 8 * lev - tr[i] - tc[c]));
}

size_t oz_layout_bytes(int64_t dim) { return (size_t)oz_rows(dim) * dim; }
size_t oz_off_t(int64_t dim) { return (size_t)kOzBlocks * dim * kOzQ * sizeof(int); }

}  // namespace

// (dim: whole 256-row blocks, a multiple of 8 of them — the per-XCD item order)
bool cq_i8_supported(int64_t dim, int m) { return m == kOzQ && dim % 2048 == 0 && dim <= 32768; }
size_t cq_i8_plane_bytes(int64_t dim) { return oz_layout_bytes(dim) + (size_t)dim * sizeof(int); }
size_t cq_i8_work_bytes(int64_t dim, int m) { return oz_off_t(dim) + (size_t)m * (sizeof(int) + 8); }

hipError_t launch_cq_i8_planes(hipStream_t s, const double* C, int64_t dim, void* planes) {
  int8_t* Z = static_cast<int8_t*>(planes);
  int* tr = reinterpret_cast<int*>(Z + oz_layout_bytes(dim));
  hipLaunchKernelGGL(oz_rows_kernel, dim3((unsigned)dim), dim3(256), 0, s, C, dim, Z, tr);
  return hipGetLastError();
}

hipError_t launch_cq_i8(hipStream_t s, void* planes, int64_t dim, const double* Q, int m, double sigma, void* work,
                        double* Y, bool medium) {
  if (!cq_i8_supported(dim, m)) return hipErrorInvalidValue;
  int8_t* Z = static_cast<int8_t*>(planes);
  const int* tr = reinterpret_cast<const int*>(Z + oz_layout_bytes(dim));
  uint8_t* base = static_cast<uint8_t*>(work);
  int* I = reinterpret_cast<int*>(base);
  int* tc = reinterpret_cast<int*>(base + oz_off_t(dim));
  unsigned long long* cmax = reinterpret_cast<unsigned long long*>(base + oz_off_t(dim) + (size_t)m * sizeof(int));
  hipError_t e = hipMemsetAsync(cmax, 0, (size_t)m * 8, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(oz_colmax_kernel, dim3((unsigned)(dim / 16)), dim3(256), 0, s, Q, dim, cmax);
  hipLaunchKernelGGL(oz_qdigits_kernel, dim3((unsigned)(dim / 16)), dim3(256), 0, s, Q, dim, cmax, Z, tc);
  e = launch_oz_syrk16(s, reinterpret_cast<const uint8_t*>(Z), dim, oz_rows(dim), I, medium);
  if (e != hipSuccess) return e;
  if (medium)
    hipLaunchKernelGGL(oz_combine_kernel<true>, dim3((unsigned)(dim * kOzQ / 256)), dim3(256), 0, s, I, dim, tr, tc, Q,
                       sigma, Y);
  else
    hipLaunchKernelGGL(oz_combine_kernel<false>, dim3((unsigned)(dim * kOzQ / 256)), dim3(256), 0, s, I, dim, tr, tc,
                       Q, sigma, Y);
  return hipGetLastError();
}

}  // namespace ef
