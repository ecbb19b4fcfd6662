// Tall dense GEMMs of the fit's subspace iteration on the matrix cores, replacing the
// vendor BLAS calls of round 1 (the eigensolve of useless/train.py:88 /
// the covariance branch :97-99, realised as block subspace iteration):
//   Y = C.Q      C: dim x dim covariance (fp64, or its fp32 copy in the coarse phase),
//                Q: dim x m block (m <= 512)                       -> dim x m
//   Y.V, Q.V     dim x m times m x m                                -> dim x m
//   Q = Y.L^-T   CholQR: the explicit inverse of the m x m Cholesky factor, then a GEMM
// Row-major operands, C[M x N] = alpha . A[M x K] . B[K x N].
//
// Layout of the work (fp64, v_mfma_f64_16x16x4_f64): a workgroup of 4 waves owns a
// 64*RW x 64*CW output tile (RW * CW = 4); each wave a 64 x 64 tile = 4 x 4 MFMA blocks
// (16 accumulators of 4 doubles).  No LDS: inside each 32-deep K chunk the K order is
// permuted so that lane group g = lane >> 4 takes k = k0 + 8g + s for MFMA step s, which
// makes every lane's A fragments EIGHT CONSECUTIVE doubles of one row (two 32-byte loads;
// 16 rows x 256 contiguous bytes per wave), and B's 16 columns of one k row one 128-byte
// run.  The product is unchanged by a permutation of K applied to both operands.  The
// next chunk's fragments are loaded into a second register set while the current
// chunk's 128 MFMAs run (~8k cycles at the fp64 rate), so one wave per SIMD keeps the
// matrix pipe fed through L2/HBM latency.  K is split over gridDim.z into fixed slabs summed in order
// by a second kernel when the tile grid alone cannot fill the chip (deterministic).
//
// A may be given transposed (a_trans: element (i, k) at A[k * lda + i]); the symmetric
// C.Q product uses that form: a workgroup then walks DOWN the rows of C (32 rows x 512
// contiguous bytes per chunk) instead of across 64 rows 128 KB apart, so at any moment
// the whole grid touches a few MB of C (every WG at the same k) rather than 16384 rows
// — kind to the TLB and the DRAM pages.
//
// fp32 (coarse phase, v_mfma_f32_32x32x2_f32): the same plan with 32 x 32 blocks, 2 x 2
// per wave, lane group g = lane >> 5 taking k = k0 + 16g + s (four float4 loads per row).
#include <algorithm>

#include "ef_linalg.hpp"

namespace ef {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// MFMA traits: fp64 16x16x4 (4 lane groups of 16, 4 consecutive k per lane per 16-deep
// chunk), fp32 32x32x2 (2 lane groups of 32, 16 consecutive k per lane per 32-deep chunk).
template <class T>
struct Mfma;
template <>
struct Mfma<double> {
  static constexpr int BLK = 16, KPL = 4;  // 16-deep chunks: two register sets fit beside the accumulators
  typedef f64x4 acc_t;
  static constexpr int NACC = 4;
  __device__ static acc_t mma(double a, double b, acc_t c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
  // C/D: col = lane & 15, row = (lane >> 4) + 4 * reg
  __device__ static int row_of(int lane, int q) { return (lane >> 4) + 4 * q; }
};
template <>
struct Mfma<float> {
  static constexpr int BLK = 32, KPL = 16;  // 32-deep chunks
  typedef f32x16 acc_t;
  static constexpr int NACC = 16;
  __device__ static acc_t mma(float a, float b, acc_t c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }
  // C/D: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
  __device__ static int row_of(int lane, int q) { return (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5); }
};

// KPL consecutive elements from 16-byte aligned memory
template <class T>
__device__ __forceinline__ void load_run(const T* __restrict__ p, T (&v)[Mfma<T>::KPL]) {
  constexpr int PER = 16 / sizeof(T);
#pragma unroll
  for (int u = 0; u < Mfma<T>::KPL / PER; ++u) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(p + u * PER);
    const T* t = reinterpret_cast<const T*>(&x);
#pragma unroll
    for (int e = 0; e < PER; ++e) v[u * PER + e] = t[e];
  }
}

// C[M x N] = alpha A . B with B given TRANSPOSED (Bt: N x K row-major) and A row-major
// (AT = false) or transposed (AT = true, K x M: a symmetric A walked down its rows).
// Chunks of CK k: lane group g = lane / BLK takes k = k0 + g*KPL + s (s < KPL), so a
// lane's B fragments are KPL consecutive elements of one Bt row (vector loads), and so
// are its A fragments when AT = false.
template <class T, int CW, bool AT>
__global__ __launch_bounds__(256) void gemm_tall_kernel(const T* __restrict__ A, int64_t lda,
                                                        const T* __restrict__ Bt, int64_t ldbt,
                                                        T* __restrict__ C, int64_t ldc, int64_t M, int64_t N,
                                                        int64_t K, int64_t kps, T alpha, T* __restrict__ part) {
  using MF = Mfma<T>;
  constexpr int BLK = MF::BLK, KPL = MF::KPL, NB = 64 / BLK, RW = 4 / CW, CK = (64 / BLK) * KPL;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / CW, wc = wave - (wave / CW) * CW;
  const int64_t m0 = ((int64_t)blockIdx.x * RW + wr) * 64;
  const int64_t n0 = ((int64_t)blockIdx.y * CW + wc) * 64;
  const int64_t kb = (int64_t)blockIdx.z * kps;
  const int64_t ke = kb + kps < K ? kb + kps : K;
  const int r = lane % BLK, g = lane / BLK;

  const T* ap[NB];
  const T* bp[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    int64_t row = m0 + i * BLK + r;
    row = row < M ? row : M - 1;
    ap[i] = AT ? A + row + (int64_t)(g * KPL) * lda : A + row * lda + g * KPL;
    int64_t col = n0 + i * BLK + r;
    col = col < N ? col : N - 1;
    bp[i] = Bt + col * ldbt + g * KPL;
  }
  typename MF::acc_t acc[NB][NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int q = 0; q < MF::NACC; ++q) acc[i][j][q] = 0;

  // full CK-deep chunk at k0 (no masks)
  auto load = [&](int64_t k0, T (&a)[NB][KPL], T (&b)[NB][KPL]) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (AT) {
        const T* p = ap[i] + k0 * lda;
#pragma unroll
        for (int s = 0; s < KPL; ++s) a[i][s] = p[s * lda];
      } else {
        load_run<T>(ap[i] + k0, a[i]);
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) load_run<T>(bp[j] + k0, b[j]);
  };
  auto mma = [&](const T (&a)[NB][KPL], const T (&b)[NB][KPL]) {
#pragma unroll
    for (int s = 0; s < KPL; ++s)
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = MF::mma(a[i][s], b[j][s], acc[i][j]);
  };
  T a0[NB][KPL], a1[NB][KPL], b0[NB][KPL], b1[NB][KPL];
  const int64_t nfull = (ke - kb) / CK;
  if (nfull > 0) {
    // double-buffered main loop; the chunk after the last is clamped to the last (a
    // redundant, never-used load) so the loop body has no branches
    load(kb, a0, b0);
    int64_t t = 0;
    // sched_barrier pins the order (the scheduler would otherwise pull the MFMAs of a
    // buffer next to the loads that fill it, serialising each chunk's loads)
    for (; t + 2 <= nfull; t += 2) {
      load(kb + CK * (t + 1), a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      load(kb + CK * (t + 2 < nfull ? t + 2 : nfull - 1), a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t < nfull) mma(a0, b0);
  }
  // masked tail (K not a multiple of CK within this split)
  const int64_t kt = kb + CK * nfull;
  if (kt < ke) {
#pragma unroll
    for (int s = 0; s < KPL; ++s) {
      const int64_t k = kt + g * KPL + s;
      const bool ok = k < ke;
#pragma unroll
      for (int i = 0; i < NB; ++i) a0[i][s] = ok ? ap[i][AT ? (kt + s) * lda : kt + s] : T(0);
#pragma unroll
      for (int j = 0; j < NB; ++j) b0[j][s] = ok ? bp[j][kt + s] : T(0);
    }
    mma(a0, b0);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int q = 0; q < MF::NACC; ++q) {
        const int64_t row = m0 + i * BLK + MF::row_of(lane, q), col = n0 + j * BLK + r;
        if (row < M && col < N) {
          if (part)
            part[((int64_t)blockIdx.z * M + row) * N + col] = acc[i][j][q];
          else
            C[row * ldc + col] = alpha * acc[i][j][q];
        }
      }
}

// out[c][r] = in[r][c] (rows x cols -> cols x rows), T2 = T or float (fp64 -> fp32 copy)
template <class T, class T2>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ in, int64_t ldin, int64_t rows,
                                                        int64_t cols, T2* __restrict__ out, int64_t ldout) {
  __shared__ T tile[32][33];
  const int64_t r0 = (int64_t)blockIdx.x * 32, c0 = (int64_t)blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  for (int y = ty; y < 32; y += 8) {
    const int64_t r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < rows && c < cols) ? in[r * ldin + c] : T(0);
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int64_t c = c0 + y, r = r0 + tx;
    if (c < cols && r < rows) out[c * ldout + r] = (T2)tile[tx][y];
  }
}

template <class T>
__global__ void splitk_sum_kernel(const T* __restrict__ part, int nsplit, int64_t M, int64_t N, T alpha,
                                  T* __restrict__ C, int64_t ldc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  T s = 0;
  for (int z = 0; z < nsplit; ++z) s += part[(int64_t)z * M * N + i];
  const int64_t r = i / N, c = i - r * N;
  C[r * ldc + c] = alpha * s;
}

// L^-1 of a lower-triangular m x m L (row-major, m <= 512): one wave per column j,
// solving L x = e_j by forward substitution (x_i = 0 for i < j) with each row's dot
// product L[i][j:i] . x[j:i] spread over the 64 lanes; x lives in LDS.  L^-1 row-major is
// the transposed B operand of Q = Y . L^-T.
__global__ __launch_bounds__(256) void tri_inv_kernel(const double* __restrict__ L, int m,
                                                      double* __restrict__ Li) {
  __shared__ double xs[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 4 + w;
  if (j >= m) return;
  double* x = xs[w];
  for (int i = lane; i < m; i += 64) x[i] = 0.0;
  __builtin_amdgcn_s_waitcnt(0);
  for (int i = j; i < m; ++i) {
    const double* li = L + (int64_t)i * m;
    double v = 0.0;
    for (int l = j + lane; l < i; l += 64) v = fma(li[l], x[l], v);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const double xi = ((i == j ? 1.0 : 0.0) - v) / li[i];
    if (lane == 0) x[i] = xi;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  for (int i = lane; i < m; i += 64) Li[(int64_t)i * m + j] = x[i];
}

// target: resident workgroups wanted, one (4 waves) per CU (measured at C3: a second
// fp32 workgroup per CU through split-K is slower, 1.18 -> 1.91 ms)
int64_t plan_split(int64_t tiles, int64_t K, int64_t M, int64_t N, size_t work_elems, int64_t target, int64_t* kps) {
  const int64_t chunks = (K + 31) / 32;
  int64_t ns = 1;
  if (tiles < target && work_elems > 0) {
    ns = (target + tiles - 1) / tiles;
    ns = std::min<int64_t>(ns, std::max<int64_t>(chunks / 4, 1));  // >= 128 deep per split
    while (ns > 1 && (size_t)(ns * M * N) > work_elems) --ns;
  }
  *kps = ((chunks + ns - 1) / ns) * 32;
  return (K + *kps - 1) / *kps;
}

template <class T, bool AT>
hipError_t launch_tall(hipStream_t s, const T* A, int64_t lda, const T* Bt, int64_t ldbt, T* C, int64_t ldc, int64_t M,
                       int64_t N, int64_t K, T alpha, T* work, size_t work_elems) {
  if (M <= 0 || N <= 0) return hipSuccess;
  // waves along N: 4 for N > 128 (a 64-row x 256-column workgroup), 2 up to 128, 1 up to 64
  const int cw = N > 128 ? 4 : (N > 64 ? 2 : 1);
  const int rw = 4 / cw;
  const int64_t gx = (M + 64 * rw - 1) / (64 * rw), gy = (N + 64 * cw - 1) / (64 * cw);
  int64_t kps = 0;
  const int64_t ns = plan_split(gx * gy, K, M, N, work_elems, 256, &kps);
  auto k = cw == 4 ? gemm_tall_kernel<T, 4, AT> : (cw == 2 ? gemm_tall_kernel<T, 2, AT> : gemm_tall_kernel<T, 1, AT>);
  hipLaunchKernelGGL(k, dim3((unsigned)gx, (unsigned)gy, (unsigned)ns), dim3(256), 0, s, A, lda, Bt, ldbt, C, ldc, M,
                     N, K, kps, alpha, ns > 1 ? work : nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ns == 1) return e;
  const int64_t tot = M * N;
  hipLaunchKernelGGL(splitk_sum_kernel<T>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, work, (int)ns, M, N,
                     alpha, C, ldc);
  return hipGetLastError();
}

}  // namespace

bool tall_gemm_supported(int64_t ld, const void* p, int elem_bytes) {
  return (ld * elem_bytes) % 16 == 0 && (reinterpret_cast<uintptr_t>(p) % 16) == 0;
}

hipError_t tall_gemm_f64(hipStream_t s, const double* A, int64_t lda, bool a_trans, const double* Bt, int64_t ldbt,
                         double* C, int64_t ldc, int64_t M, int64_t N, int64_t K, double alpha, double* work,
                         size_t work_elems) {
  return a_trans ? launch_tall<double, true>(s, A, lda, Bt, ldbt, C, ldc, M, N, K, alpha, work, work_elems)
                 : launch_tall<double, false>(s, A, lda, Bt, ldbt, C, ldc, M, N, K, alpha, work, work_elems);
}

hipError_t tall_gemm_f32(hipStream_t s, const float* A, int64_t lda, bool a_trans, const float* Bt, int64_t ldbt,
                         float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha, float* work,
                         size_t work_elems) {
  return a_trans ? launch_tall<float, true>(s, A, lda, Bt, ldbt, C, ldc, M, N, K, alpha, work, work_elems)
                 : launch_tall<float, false>(s, A, lda, Bt, ldbt, C, ldc, M, N, K, alpha, work, work_elems);
}

hipError_t launch_transpose_f64(hipStream_t s, const double* in, int64_t ldin, int64_t rows, int64_t cols, double* out,
                                int64_t ldout) {
  hipLaunchKernelGGL((transpose_kernel<double, double>), dim3((unsigned)((rows + 31) / 32), (unsigned)((cols + 31) / 32)),
                     dim3(256), 0, s, in, ldin, rows, cols, out, ldout);
  return hipGetLastError();
}

hipError_t launch_transpose_f64_to_f32(hipStream_t s, const double* in, int64_t ldin, int64_t rows, int64_t cols,
                                       float* out, int64_t ldout) {
  hipLaunchKernelGGL((transpose_kernel<double, float>), dim3((unsigned)((rows + 31) / 32), (unsigned)((cols + 31) / 32)),
                     dim3(256), 0, s, in, ldin, rows, cols, out, ldout);
  return hipGetLastError();
}

hipError_t launch_tri_inv(hipStream_t s, const double* L, int m, double* Li) {
  if (m > 512) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tri_inv_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, s, L, m, Li);
  return hipGetLastError();
}

}  // namespace ef
