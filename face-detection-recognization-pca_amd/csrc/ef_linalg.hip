// Fit-path kernels (SURVEY.md K1 column statistics, K3 Gram/covariance, K4 eigensolver,
// K5 back-projection helpers).  Everything here is float64: the survey measured that
// fp32 eigenvectors cannot meet 1e-4 on the trailing real-face components
// (SURVEY.md §7 "fp32 conditioning"), and the reference itself is fp64 LAPACK
// (useless/train.py:84-95).
#include "ef_dma.hpp"
#include "ef_linalg.hpp"

#include <climits>
#include <cmath>
#include <type_traits>

namespace ef {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- K1: column stats
// Exact integer sums: S1[c] = sum_i x_ic, S2[c] = sum_i x_ic^2 (uint64 atomics are exact,
// so the result does not depend on arrival order).
__global__ void colstats_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d, int64_t rows_per,
                                unsigned long long* __restrict__ S1,
                                unsigned long long* __restrict__ S2) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  int64_t r1 = r0 + rows_per;
  if (r1 > n) r1 = n;
  unsigned long long s1 = 0, s2 = 0;
  for (int64_t r = r0; r < r1; ++r) {
    const unsigned v = X[r * d + c];
    s1 += v;
    s2 += v * v;
  }
  atomicAdd(&S1[c], s1);
  atomicAdd(&S2[c], s2);
}

// mean, population variance, StandardScaler scale_ (sklearn _data.py:1040-1051:
// near-constant features -> scale 1), and the centring weight w (1/scale or 1).
__global__ void stats_finalize_kernel(const unsigned long long* __restrict__ S1,
                                      const unsigned long long* __restrict__ S2, int64_t n, int64_t d,
                                      int standardize, double* __restrict__ mean,
                                      double* __restrict__ var, double* __restrict__ scale,
                                      double* __restrict__ w) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  const long long s1 = (long long)S1[c], s2 = (long long)S2[c];
  const double dn = (double)n;
  const double mu = (double)s1 / dn;
  const long long num = (long long)n * s2 - s1 * s1;  // exact: n*sum(x^2) - (sum x)^2
  const double v = (double)num / (dn * dn);
  const double eps = 2.220446049250313e-16;
  const double bound = dn * eps * v + (dn * mu * eps) * (dn * mu * eps);
  const double sc = (v <= bound) ? 1.0 : sqrt(v);
  mean[c] = mu;
  var[c] = v;
  scale[c] = sc;
  w[c] = standardize ? 1.0 / sc : 1.0;
}

// Float input (ManualStandardScaler output, float64 faces): fp64 column statistics in two
// passes, partial sums per row block (part[blk][d]) summed in a fixed order.
// Pass 1: part[blk][c] = sum x.  Pass 2: part[blk][c] = sum (x - mean), part2 = sum (x - mean)^2.
template <class T>
__global__ void colsum_float_kernel(const T* __restrict__ X, int64_t n, int64_t d, int64_t rows_per,
                                    const double* __restrict__ mean, double* __restrict__ part,
                                    double* __restrict__ part2) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = r0 + rows_per < n ? r0 + rows_per : n;
  double s1 = 0.0, s2 = 0.0;
  if (!mean) {
    for (int64_t r = r0; r < r1; ++r) s1 += (double)X[r * d + c];
  } else {
    const double m = mean[c];
    for (int64_t r = r0; r < r1; ++r) {
      const double t = (double)X[r * d + c] - m;
      s1 += t;
      s2 = fma(t, t, s2);
    }
    part2[(int64_t)blockIdx.y * d + c] = s2;
  }
  part[(int64_t)blockIdx.y * d + c] = s1;
}

__global__ void colmean_float_kernel(const double* __restrict__ part, int nblk, int64_t n, int64_t d,
                                     double* __restrict__ mean) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * d + c];
  mean[c] = s / (double)n;
}

__global__ void colvar_float_kernel(const double* __restrict__ part, const double* __restrict__ part2, int nblk,
                                    int64_t n, int64_t d, int standardize, const double* __restrict__ mean,
                                    double* __restrict__ var, double* __restrict__ scale, double* __restrict__ w) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  double s1 = 0.0, s2 = 0.0;
  for (int b = 0; b < nblk; ++b) {
    s1 += part[(int64_t)b * d + c];
    s2 += part2[(int64_t)b * d + c];
  }
  const double dn = (double)n;
  double v = (s2 - s1 * s1 / dn) / dn;
  if (v < 0.0) v = 0.0;
  const double mu = mean[c];
  const double eps = 2.220446049250313e-16;
  const double bound = dn * eps * v + (dn * mu * eps) * (dn * mu * eps);  // sklearn _is_constant_feature
  const double sc = (v <= bound) ? 1.0 : sqrt(v);
  var[c] = v;
  scale[c] = sc;
  w[c] = standardize ? 1.0 / sc : 1.0;
}

// ------------------------------------------------------------ generic f64 MFMA GEMM
// C[M][N] = alpha * sum_k A(m,k) * B(k,n) on v_mfma_f64_16x16x4_f64.  A/B are read
// through loaders so the centred/scaled pixel matrix ((x - mu) * w) is formed in the
// operand load and never materialised (K2).  Split-K over gridDim.z writes fp64 slabs
// that reduce_splitk sums in a fixed order.
constexpr int GT = 64;          // tile M and N
constexpr int GK = 16;          // tile K
constexpr int GS = GT + 16;     // LDS row stride (doubles): conflict-free ds_read_b64

template <class LA, class LB>
__global__ __launch_bounds__(256) void gemm64_kernel(LA A, LB B, int64_t M, int64_t N, int64_t K,
                                                     int64_t k_per_split, double alpha,
                                                     double* __restrict__ C, int64_t ldc,
                                                     double* __restrict__ part) {
  __shared__ double sA[GK * GS];
  __shared__ double sB[GK * GS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.y * GT, n0 = (int64_t)blockIdx.x * GT;
  const int64_t kb = (int64_t)blockIdx.z * k_per_split;
  int64_t ke = kb + k_per_split;
  if (ke > K) ke = K;

  f64x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f64x4{0, 0, 0, 0};

  for (int64_t k0 = kb; k0 < ke; k0 += GK) {
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      const int e = tid + 256 * e4;
      int mm, kk;
      if (A.kfast) { kk = e % GK; mm = e / GK; } else { mm = e % GT; kk = e / GT; }
      const int64_t gm = m0 + mm, gk = k0 + kk;
      sA[kk * GS + mm] = (gm < M && gk < ke) ? A(gm, gk) : 0.0;
      int nn;
      if (B.kfast) { kk = e % GK; nn = e / GK; } else { nn = e % GT; kk = e / GT; }
      const int64_t gn = n0 + nn, gk2 = k0 + kk;
      sB[kk * GS + nn] = (gn < N && gk2 < ke) ? B(gk2, gn) : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < GK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sA[kr * GS + wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = sB[kr * GS + wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // f64 16x16x4 C/D map: col = lane&15, row = (lane>>4) + 4*r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 32 + i * 16 + (lane >> 4) + 4 * r;
        const int64_t col = n0 + wn * 32 + j * 16 + (lane & 15);
        if (row < M && col < N) {
          if (part)
            part[((int64_t)blockIdx.z * M + row) * N + col] = acc[i][j][r];
          else
            C[row * ldc + col] = alpha * acc[i][j][r];
        }
      }
}

__global__ void reduce_splitk_kernel(const double* __restrict__ part, int nsplit, int64_t M, int64_t N,
                                     double alpha, double* __restrict__ C, int64_t ldc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  double s = 0.0;
  for (int z = 0; z < nsplit; ++z) s += part[(int64_t)z * M * N + i];
  const int64_t r = i / N, c = i - r * N;
  C[r * ldc + c] = alpha * s;
}

template <class LA, class LB>
static hipError_t gemm_t(hipStream_t s, const LA& A, const LB& B, int64_t M, int64_t N, int64_t K,
                         double alpha, double* C, int64_t ldc, double* work, size_t work_elems) {
  const int64_t mt = (M + GT - 1) / GT, nt = (N + GT - 1) / GT;
  const int64_t ksteps = (K + GK - 1) / GK;
  int64_t ns = 1;
  const int64_t tiles = mt * nt;
  if (tiles < 512 && work) {
    ns = (1024 + tiles - 1) / tiles;
    if (ns > ksteps) ns = ksteps;
    if (ns > 256) ns = 256;
    while (ns > 1 && (size_t)(ns * M * N) > work_elems) --ns;
  }
  const int64_t kps = ((ksteps + ns - 1) / ns) * GK;
  ns = (K + kps - 1) / kps;
  if (ns < 1) ns = 1;
  const dim3 grid((unsigned)nt, (unsigned)mt, (unsigned)ns);
  hipLaunchKernelGGL((gemm64_kernel<LA, LB>), grid, dim3(256), 0, s, A, B, M, N, K, kps, alpha, C, ldc,
                     ns > 1 ? work : nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ns == 1) return e;
  const int64_t tot = M * N;
  hipLaunchKernelGGL(reduce_splitk_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, work,
                     (int)ns, M, N, alpha, C, ldc);
  return hipGetLastError();
}

// Calls fn(loader) with the operand's loader; kfast: the contiguous tile index is k.
template <class Fn>
static hipError_t with_loader(const Operand& o, bool kfast, Fn&& fn) {
  if (!o.u8) return fn(DenseLd{o.p, o.ld, o.trans, kfast});
  switch (o.elem) {
    case EF_U8:
      return fn(PixLd<uint8_t>{static_cast<const uint8_t*>(o.x), o.ld, o.trans, o.mu, o.w, kfast});
    case EF_F32:
      return fn(PixLd<float>{static_cast<const float*>(o.x), o.ld, o.trans, o.mu, o.w, kfast});
    case EF_F64:
      return fn(PixLd<double>{static_cast<const double*>(o.x), o.ld, o.trans, o.mu, o.w, kfast});
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t gemm64(hipStream_t s, const Operand& A, const Operand& B, int64_t M, int64_t N, int64_t K,
                  double alpha, double* C, int64_t ldc, double* work, size_t work_elems) {
  // the two pixel operands of a product are always the same matrix (same element type)
  if (A.u8 && B.u8 && A.elem != B.elem) return hipErrorInvalidValue;
  return with_loader(A, A.trans == 0, [&](const auto& a) {
    return with_loader(B, B.trans != 0, [&](const auto& b) {
      if constexpr (!std::is_same_v<std::decay_t<decltype(a)>, std::decay_t<decltype(b)>> &&
                    !std::is_same_v<std::decay_t<decltype(a)>, DenseLd> &&
                    !std::is_same_v<std::decay_t<decltype(b)>, DenseLd>) {
        return hipErrorInvalidValue;  // mixed pixel types: never instantiated as a kernel
      } else {
        return gemm_t(s, a, b, M, N, K, alpha, C, ldc, work, work_elems);
      }
    });
  });
}

// ------------------------------------------------------------- K4: Jacobi in LDS
// Cyclic two-sided Jacobi for a symmetric m x m (m <= kJacobiMax) matrix, fully in LDS
// (T and the accumulated rotations V, both fp64).  Each round applies m/2 disjoint
// rotations (round-robin "circle" ordering) in parallel: rows, barrier, columns.
// Output: eigenvalues descending, eigenvectors as columns of evecs (row-major m x m).
__global__ __launch_bounds__(1024) void jacobi_kernel(const double* __restrict__ A, int m, int64_t lda,
                                                      double* __restrict__ evals, double* __restrict__ evecs,
                                                      int64_t ldv, int max_sweeps, int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double jsm[];
  const int mp = m + (m & 1);
  const int S = mp + 1;
  const int np = mp / 2;
  double* T = jsm;
  double* V = T + mp * S;
  double* cs = V + mp * S;
  double* sn = cs + np;
  int* pp = reinterpret_cast<int*>(sn + np);
  int* qq = pp + np;
  int* flag = qq + np;
  int* rcnt = flag + 1;
  const int tid = threadIdx.x, nth = blockDim.x;

  for (int e = tid; e < mp * mp; e += nth) {
    const int i = e / mp, j = e - (e / mp) * mp;
    double v = 0.0;
    if (i < m && j < m) v = 0.5 * (A[(int64_t)i * lda + j] + A[(int64_t)j * lda + i]);
    T[i * S + j] = v;
    V[i * S + j] = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();

  int sweep = 0;
  bool converged = false;
  if (tid < 2) rcnt[tid] = 0;
  __syncthreads();
  for (; sweep < max_sweeps; ++sweep) {
    if (tid == 0) *flag = 0;
    __syncthreads();
    for (int r = 0; r < mp - 1; ++r) {
      int* cnt = &rcnt[r & 1];
      if (tid < np) {
        auto pos = [&](int j) { return j == 0 ? 0 : 1 + ((j - 1 + r) % (mp - 1)); };
        int p = pos(tid), q = pos(mp - 1 - tid);
        if (p > q) { const int t = p; p = q; q = t; }
        const double apq = T[p * S + q];
        const double app = T[p * S + p], aqq = T[q * S + q];
        const double g = 100.0 * fabs(apq);
        if (apq == 0.0 || (fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq))) {
          pp[tid] = -1;
        } else {
          const double theta = (aqq - app) / (2.0 * apq);
          double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
          if (fabs(theta) > 1e150) t = 0.5 / fabs(theta);
          if (theta < 0.0) t = -t;
          const double c = 1.0 / sqrt(t * t + 1.0);
          cs[tid] = c;
          sn[tid] = t * c;
          pp[tid] = p;
          qq[tid] = q;
          atomicAdd(cnt, 1);
        }
      }
      __syncthreads();
      if (tid == 0) rcnt[(r + 1) & 1] = 0;  // next round's counter (read >= 1 barrier ago)
      if (*cnt == 0) continue;              // uniform: nothing to rotate this round
      if (tid == 0) *flag = 1;
      for (int e = tid; e < np * mp; e += nth) {  // rows p, q  <- J^T T
        const int i = e / mp, j = e - (e / mp) * mp;
        const int p = pp[i];
        if (p < 0) continue;
        const int q = qq[i];
        const double c = cs[i], s = sn[i];
        const double tp = T[p * S + j], tq = T[q * S + j];
        T[p * S + j] = c * tp - s * tq;
        T[q * S + j] = s * tp + c * tq;
      }
      __syncthreads();
      for (int e = tid; e < np * mp; e += nth) {  // columns p, q <- T J ; V <- V J
        const int i = e / mp, rr = e - (e / mp) * mp;
        const int p = pp[i];
        if (p < 0) continue;
        const int q = qq[i];
        const double c = cs[i], s = sn[i];
        const double tp = T[rr * S + p], tq = T[rr * S + q];
        double np_ = c * tp - s * tq, nq_ = s * tp + c * tq;
        if (rr == p) nq_ = 0.0;
        if (rr == q) np_ = 0.0;
        T[rr * S + p] = np_;
        T[rr * S + q] = nq_;
        const double vp = V[rr * S + p], vq = V[rr * S + q];
        V[rr * S + p] = c * vp - s * vq;
        V[rr * S + q] = s * vp + c * vq;
      }
      __syncthreads();
    }
    __syncthreads();
    const int f = *flag;
    __syncthreads();
    if (f == 0) { converged = true; break; }
  }

  // descending sort by rank (ties -> lower index first); the padding index goes last
  if (tid < mp) {
    const int i = tid;
    const bool dummy = (i >= m);
    const double li = T[i * S + i];
    int rank = mp - 1;
    if (!dummy) {
      rank = 0;
      for (int j = 0; j < m; ++j) {
        const double lj = T[j * S + j];
        rank += (lj > li) || (lj == li && j < i);
      }
      evals[rank] = li;
      for (int rr = 0; rr < m; ++rr) evecs[(int64_t)rr * ldv + rank] = V[rr * S + i];
    }
  }
  if (tid == 0) *info = converged ? sweep + 1 : -1;
}

size_t jacobi_lds_bytes(int m) {
  const int mp = m + (m & 1);
  return (size_t)2 * mp * (mp + 1) * sizeof(double) + (size_t)mp * sizeof(double) +
         (size_t)(mp + 4) * sizeof(int) + 16;
}

hipError_t launch_jacobi(hipStream_t s, const double* A, int m, int64_t lda, double* evals, double* evecs,
                         int64_t ldv, int max_sweeps, int* info) {
  if (m < 1 || m > kJacobiMax) return hipErrorInvalidValue;
  const size_t lds = jacobi_lds_bytes(m);
  {
    const hipError_t e = allow_dynamic_lds(reinterpret_cast<const void*>(jacobi_kernel), (int)jacobi_lds_bytes(kJacobiMax));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(jacobi_kernel, dim3(1), dim3(1024), lds, s, A, m, lda, evals, evecs, ldv, max_sweeps,
                     info);
  return hipGetLastError();
}

// ------------------------------------------------------------ Cholesky (one workgroup)
// In-place lower Cholesky of the symmetric positive definite m x m matrix A (row-major,
// lda): A[i][j] (j <= i) <- L, upper triangle zeroed.  A pivot <= tol_rel * max diagonal
// stops with *info = -(j+1) (numerically rank-deficient block: the caller falls back to
// the Jacobi orthonormalisation); *info = 0 on success.  Used by the CholQR
// orthonormalisation of the subspace iteration (m <= 1024, L2-resident).
// Right-looking, 32-column panels: the panel (rows jb.., 32 columns) is factored in LDS
// with LDS-only barriers, then the trailing lower triangle takes one rank-32 update.
constexpr int kCholNB = 32;
constexpr int kCholPS = kCholNB + 1;  // LDS panel row stride (odd: rows spread over banks)
constexpr int kCholMaxM = 512;        // panel rows held in LDS: 512 x 33 doubles = 132 KiB

__global__ __launch_bounds__(1024) void chol_kernel(double* __restrict__ A, int m, int64_t lda, double tol_rel,
                                                    int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double P[];  // [m - jb][kCholPS]
  __shared__ double red[1024];
  __shared__ double piv_s[kCholNB];
  const int tid = threadIdx.x, nth = blockDim.x;
  double mx = 0.0;
  for (int i = tid; i < m; i += nth) mx = fmax(mx, A[(int64_t)i * lda + i]);
  red[tid] = mx;
  __syncthreads();
  for (int o = nth / 2; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
    __syncthreads();
  }
  const double tol = tol_rel * red[0];
  for (int jb = 0; jb < m; jb += kCholNB) {
    const int nb = m - jb < kCholNB ? m - jb : kCholNB;
    const int rows = m - jb;
    for (int e = tid; e < rows * kCholNB; e += nth) {  // load the panel
      const int i = e / kCholNB, t = e % kCholNB;
      P[i * kCholPS + t] = t < nb ? A[(int64_t)(jb + i) * lda + jb + t] : 0.0;
    }
    __syncthreads();
    // unblocked factorisation of the panel on UNSCALED columns (A[i][l] -= a_it a_lt / d_t,
    // the chol_small_kernel form): every thread reads the pivot itself, so a column step
    // is one barrier instead of three; the columns are scaled by 1/sqrt(d_t) afterwards
    for (int t = 0; t < nb; ++t) {
      const double d = P[t * kCholPS + t];
      if (!(d > tol)) {  // uniform: every thread read the same pivot
        if (tid == 0) *info = -(jb + t + 1);
        return;
      }
      const double inv = 1.0 / d;
      // update the panel's remaining columns: 32 lanes per row (column l = lane), 32 rows
      // per pass — no per-element index division
      const int l = tid & 31;
      if (l > t && l < nb) {
        const double plt = P[l * kCholPS + t] * inv;
        for (int i = t + 1 + (tid >> 5); i < rows; i += nth >> 5)
          if (l <= i) P[i * kCholPS + l] -= P[i * kCholPS + t] * plt;
      }
      __syncthreads();
    }
    if (tid < nb) piv_s[tid] = sqrt(P[tid * kCholPS + tid]);
    __syncthreads();
    for (int e = tid; e < rows * nb; e += nth) {
      const int i = e / nb, t = e % nb;
      if (i >= t) P[i * kCholPS + t] /= piv_s[t];
    }
    __syncthreads();
    for (int e = tid; e < rows * kCholNB; e += nth) {  // store the panel
      const int i = e / kCholNB, t = e % kCholNB;
      if (t < nb && t <= i) A[(int64_t)(jb + i) * lda + jb + t] = P[i * kCholPS + t];
    }
    // trailing lower triangle: A[i][l] -= P[i] . P[l]  (jb + nb <= l <= i), 4 x 4 output
    // blocks per thread (8 LDS reads per t for 16 dot products; each dot product still
    // accumulates t = 0..31 in order, so the result is unchanged)
    const int w = rows - nb;
    const int nbw = (w + 3) >> 2;
    for (int e = tid; e < nbw * nbw; e += nth) {
      const int bi = e / nbw, bj = e - bi * nbw;
      if (bj > bi) continue;
      double acc[4][4] = {};
      const double* pi = P + (nb + 4 * bi) * kCholPS;
      const double* pl = P + (nb + 4 * bj) * kCholPS;
      const int ri = min(4, w - 4 * bi), rl = min(4, w - 4 * bj);
#pragma unroll 4
      for (int t = 0; t < kCholNB; ++t) {
        double a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u] = u < ri ? pi[u * kCholPS + t] : 0.0;
          b[u] = u < rl ? pl[u * kCholPS + t] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[u][v] = fma(a[u], b[v], acc[u][v]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int i = 4 * bi + u, l = 4 * bj + v;
          if (u < ri && v < rl && l <= i) A[(int64_t)(jb + nb + i) * lda + jb + nb + l] -= acc[u][v];
        }
    }
    __syncthreads();
  }
  for (int e = tid; e < m * m; e += nth) {
    const int i = e / m, l = e % m;
    if (l > i) A[(int64_t)i * lda + l] = 0.0;
  }
  if (tid == 0) *info = 0;
}

// Small orders (m <= 128): the whole factorisation in one workgroup with the matrix in
// registers — thread (bi, bj) of a 32 x 32 grid owns the 4 x 4 block of rows 4bi.., columns
// 4bj..  Step t: the owners of column t publish it (already final) to LDS, one barrier,
// then every thread applies the rank-1 update  A[i][l] -= A[i][t] A[l][t] / A[t][t]  to its
// entries with l > t (unscaled column; the diagonal's square root and the column scaling
// are applied at the end).  One barrier per column, no global traffic inside the loop.
constexpr int kCholSmall = 128;
__global__ __launch_bounds__(1024) void chol_small_kernel(double* __restrict__ A, int m, int64_t lda, double tol_rel,
                                                          int* __restrict__ info) {
  __shared__ double col[2][kCholSmall];
  __shared__ double red[32];
  __shared__ int bad;
  const int tid = threadIdx.x;
  const int bi = tid >> 5, bj = tid & 31;
  double a[4][4];
  double dmax = 0.0;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * bi + u, l = 4 * bj + v;
      a[u][v] = (i < m && l < m) ? A[(int64_t)i * lda + l] : 0.0;
      if (i == l && i < m) dmax = fmax(dmax, a[u][v]);
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dmax = fmax(dmax, __shfl_xor(dmax, off));
  if ((tid & 63) == 0) red[tid >> 6] = dmax;
  if (tid == 0) bad = 0;
  __syncthreads();
  double mx = 0.0;
  for (int w = 0; w < 16; ++w) mx = fmax(mx, red[w]);
  const double tol = tol_rel * mx;
  for (int t = 0; t < m; ++t) {
    const int buf = t & 1;
    if (bj == (t >> 2)) {  // publish column t (rows 4bi..4bi+3)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (v == (t & 3)) col[buf][4 * bi + u] = a[u][v];
    }
    __syncthreads();
    const double d = col[buf][t];
    if (!(d > tol)) {
      if (tid == 0) *info = -(t + 1);
      return;  // uniform: every thread read the same d
    }
    const double inv = 1.0 / d;
    if (4 * bj + 3 > t && 4 * bi + 3 > t) {
      double ci[4], cl[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ci[u] = col[buf][4 * bi + u];
        cl[u] = col[buf][4 * bj + u] * inv;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int i = 4 * bi + u, l = 4 * bj + v;
          if (l > t && i >= l) a[u][v] = fma(-ci[u], cl[v], a[u][v]);
        }
    }
  }
  // L[i][l] = a[i][l] / sqrt(a[l][l]) for l <= i (the diagonal becomes its square root);
  // the diagonal is published once more through LDS
  __syncthreads();
  if (bi == bj) {
#pragma unroll
    for (int u = 0; u < 4; ++u) col[0][4 * bi + u] = a[u][u];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * bi + u, l = 4 * bj + v;
      if (i < m && l < m) A[(int64_t)i * lda + l] = l <= i ? a[u][v] / sqrt(col[0][l]) : 0.0;
    }
  if (tid == 0) *info = 0;
  (void)bad;
}

hipError_t launch_cholesky(hipStream_t s, double* A, int m, int64_t lda, double tol_rel, int* info) {
  if (m < 1 || m > kCholMaxM) return hipErrorInvalidValue;
  if (m <= kCholSmall) {
    hipLaunchKernelGGL(chol_small_kernel, dim3(1), dim3(1024), 0, s, A, m, lda, tol_rel, info);
    return hipGetLastError();
  }
  {
    const hipError_t e = allow_dynamic_lds(reinterpret_cast<const void*>(chol_kernel),
                                           (int)((size_t)kCholMaxM * kCholPS * sizeof(double)));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(chol_kernel, dim3(1), dim3(1024), (size_t)m * kCholPS * sizeof(double), s, A, m, lda, tol_rel,
                     info);
  return hipGetLastError();
}

// CholQR factor for the subspace block (m <= 256): Li = L^-1 with G = L L^T, in ONE
// workgroup with the matrices in registers.  1024 threads as a 32 x 32 grid (p, q); thread
// (p, q) owns the lower-triangle entries (i, l) = (p + 32x, q + 32y), x, y in 0..7: x > y,
// or x == y when p >= q — at most 36 fp64 values, packed in slots s(x, y) = x(x+1)/2 + y.
// (Row/column blocks of 8 would need 528 threads x 128 VGPRs: over the 3-wave budget.)
// Orders below 256 are padded with a diagonal equal to the largest pivot candidate.
//  Phase 1 (right-looking Cholesky on unscaled columns, the chol_small_kernel form): step t
//  publishes column t through LDS, one barrier, then A[i][l] -= A[i][t] A[l][t] / A[t][t]
//  for l > t; the square roots and the scaling come at the end.  L^T goes to Li.
//  Phase 2 (forward substitution L X = I, right-looking): step t finalises row t of X,
//  X[t][:] = R[t][:] / L[t][t], publishes it, one barrier, then R[i][l] -= L[i][t] X[t][l]
//  for i > t; the columns of L stream back from Li into LDS eight at a time by LDS-DMA,
//  one chunk ahead.  X then overwrites Li (zeros above the diagonal).
// t = 32 Y + tq with the block index Y unrolled, so every register slot is addressed by a
// compile-time constant (a run-time index would move the array to scratch).  Replaces
// the global-memory pair chol_kernel (0.34 ms at m = 256) + tri_inv_kernel (0.19 ms),
// which were bound by per-step L2 round trips.  A pivot <= tol_rel * max diagonal:
// *info = -(t+1), Li untouched.
constexpr int kCholInvMax = 256;

__device__ __forceinline__ constexpr int cslot(int x, int y) { return x * (x + 1) / 2 + y; }

__global__ __launch_bounds__(1024) void chol_inv_kernel(const double* __restrict__ G, int m, int64_t lda,
                                                        double tol_rel, double* __restrict__ Li,
                                                        int* __restrict__ info) {
  __shared__ double col[2][kCholInvMax];  // phase 1: column t; phase 2: row t of X
  __shared__ double sq[kCholInvMax];      // diag(L) = sqrt of the pivots
  __shared__ double isq[kCholInvMax];     // and their reciprocals
  __shared__ __attribute__((aligned(16))) double lch[2][8][kCholInvMax];  // phase 2: 8 columns of L
  __shared__ double red[16];
  const int tid = threadIdx.x, p = tid >> 5, q = tid & 31;
  const bool pq = p >= q;
  if (tid < 2 * kCholInvMax) col[tid >> 8][tid & 255] = 0.0;

  // max diagonal (pivot tolerance and padding value)
  double dm = 0.0;
  if (p == q)
    for (int x = 0; x < 8; ++x)
      if (p + 32 * x < m) dm = fmax(dm, G[(int64_t)(p + 32 * x) * lda + p + 32 * x]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dm = fmax(dm, __shfl_xor(dm, off));
  if ((tid & 63) == 0) red[tid >> 6] = dm;
  __syncthreads();
  double mx = 0.0;
#pragma unroll
  for (int w = 0; w < 16; ++w) mx = fmax(mx, red[w]);
  const double tol = tol_rel * mx;
  const double pad = mx > 0.0 ? mx : 1.0;

  double a[36];
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int y = 0; y <= x; ++y) {
      const int i = p + 32 * x, l = q + 32 * y;
      double v = 0.0;
      if (x > y || pq) v = (i < m && l < m) ? G[(int64_t)i * lda + l] : (i == l ? pad : 0.0);
      a[cslot(x, y)] = v;
    }

  // ---- phase 1: unscaled right-looking Cholesky
#pragma unroll
  for (int Y = 0; Y < 8; ++Y) {
    for (int tq = 0; tq < 32; ++tq) {
      const int t = 32 * Y + tq, buf = t & 1;
      if (q == tq) {  // publish column t: rows p + 32x, x >= Y
#pragma unroll
        for (int x = Y; x < 8; ++x)
          if (x > Y || pq) col[buf][p + 32 * x] = a[cslot(x, Y)];
      }
      __syncthreads();
      // every LDS read of the step issued together, then one wait (the pivot's division
      // overlaps the reads)
      const double d = col[buf][t];
      double cl[8], ci[8];
#pragma unroll
      for (int y = Y; y < 8; ++y) cl[y] = col[buf][q + 32 * y];
#pragma unroll
      for (int x = Y; x < 8; ++x) ci[x] = col[buf][p + 32 * x];
      if (!(d > tol)) {  // uniform: every thread read the same pivot
        if (tid == 0) *info = -(t + 1);
        return;
      }
      // branch-free update: operands of entries that must not change are selected to 0
      // (columns l <= t are final; slots outside the triangle are never read); col holds
      // only finite values (zeroed at entry), so 0 * col stays 0
      const double inv = rcp_nr(d);  // (the step's critical path: pivot read -> scale)
#pragma unroll
      for (int y = Y; y < 8; ++y) cl[y] = (y > Y || q > tq) ? cl[y] * inv : 0.0;
#pragma unroll
      for (int x = Y; x < 8; ++x)
#pragma unroll
        for (int y = Y; y <= x; ++y) a[cslot(x, y)] = fma(-ci[x], cl[y], a[cslot(x, y)]);
    }
  }
  if (pq && p == q) {
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      sq[p + 32 * x] = sqrt(a[cslot(x, x)]);
      isq[p + 32 * x] = 1.0 / sq[p + 32 * x];  // phase 2's row scale, off its serial path
    }
  }
  __syncthreads();
  // L^T into Li: row l holds column l of L (L[i][l] = a / sqrt(d_l), sqrt(d_l) on the diagonal)
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int y = 0; y <= x; ++y) {
      const int i = p + 32 * x, l = q + 32 * y;
      if ((x > y || pq) && i < m && l < m) Li[(int64_t)l * m + i] = i == l ? sq[l] : a[cslot(x, y)] / sq[l];
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- phase 2: X = L^-1, rows finalised in order (R starts as the identity)
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int y = 0; y <= x; ++y) a[cslot(x, y)] = (x == y && p == q) ? 1.0 : 0.0;
  const int lane = tid & 63, wave = tid >> 6;
  const int nch = (m + 7) >> 3;
  const int segs = (m * 8 + 1023) / 1024;  // 1-KiB DMA pieces per row of L^T
  auto issue_chunk = [&](int ch) {          // rows 8ch..8ch+7 of L^T -> lch[ch & 1]
    const int row = 8 * ch + wave;
    if (wave < 8 && row < m) {
      for (int sg = 0; sg < segs; ++sg) {
        const int off = sg * 1024 + lane * 16;
        if (off < m * 8)
          glds16(reinterpret_cast<const char*>(Li + (int64_t)row * m) + off,
                 lds_addr(&lch[ch & 1][wave][0]) + (unsigned)(sg * 1024));
      }
    }
  };
  issue_chunk(0);
#pragma unroll
  for (int X = 0; X < 8; ++X) {
    for (int tp = 0; tp < 32; ++tp) {
      const int t = 32 * X + tp, buf = t & 1;
      if (t >= m) break;  // uniform
      if ((t & 7) == 0) {
        dma_wait_all();
        __syncthreads();  // chunk t/8 landed; the previous chunk's buffer is free
        if ((t >> 3) + 1 < nch) issue_chunk((t >> 3) + 1);
      }
      if (p == tp) {  // row t of X: R[t][:] / L[t][t] (entries l <= t), published
        const double f = isq[t];
#pragma unroll
        for (int y = 0; y <= X; ++y)
          if (y < X || pq) {
            a[cslot(X, y)] *= f;
            col[buf][q + 32 * y] = a[cslot(X, y)];
          }
      }
      __syncthreads();
      // branch-free: rows i <= t are final (L entry selected to 0; the staged row may hold
      // stale bytes there), X[t][l] = 0 for l > t
      const double* lc = lch[(t >> 3) & 1][t & 7];
      double xr[8], li[8];
#pragma unroll
      for (int y = 0; y <= X; ++y) xr[y] = col[buf][q + 32 * y];
#pragma unroll
      for (int x = X; x < 8; ++x) li[x] = lc[p + 32 * x];
#pragma unroll
      for (int y = 0; y <= X; ++y) xr[y] = (y < X || q <= tp) ? xr[y] : 0.0;
#pragma unroll
      for (int x = X; x < 8; ++x) li[x] = (x > X || p > tp) ? li[x] : 0.0;
#pragma unroll
      for (int x = X; x < 8; ++x)
#pragma unroll
        for (int y = 0; y <= X && y <= x; ++y) a[cslot(x, y)] = fma(-li[x], xr[y], a[cslot(x, y)]);
    }
  }
  __syncthreads();  // every DMA read of L^T is done (awaited at its chunk boundary)
#pragma unroll
  for (int x = 0; x < 8; ++x)
#pragma unroll
    for (int y = 0; y < 8; ++y) {
      const int i = p + 32 * x, l = q + 32 * y;
      if (i < m && l < m) Li[(int64_t)i * m + l] = (y < x || (y == x && pq)) ? a[cslot(x, y < x ? y : x)] : 0.0;
    }
  if (tid == 0) *info = 0;
}

bool chol_inv_reg_supported(int m) { return m >= 1 && m <= kCholInvMax && m % 2 == 0; }

hipError_t launch_chol_inv_reg(hipStream_t s, const double* G, int m, int64_t lda, double tol_rel, double* Li,
                               int* info) {
  if (!chol_inv_reg_supported(m)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(chol_inv_kernel, dim3(1), dim3(1024), 0, s, G, m, lda, tol_rel, Li, info);
  return hipGetLastError();
}

// ------------------------------------------------------------------ small helpers
__global__ void trace_kernel(const double* __restrict__ C, int64_t m, int64_t ldc, double* out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < m; i += 256) s += C[i * ldc + i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void rand_init_kernel(double* __restrict__ Q, int64_t count, unsigned long long seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const unsigned long long r = splitmix64(seed ^ (unsigned long long)i * 0xD1B54A32D192ED03ull);
  Q[i] = ((double)(r >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
}

// W'[i][j] = W[i][j] / sqrt(max(lam[j], floor))  (Q <- Y W Lambda^{-1/2})
__global__ void scale_cols_rsqrt_kernel(const double* __restrict__ W, int64_t rows, int cols,
                                        const double* __restrict__ lam, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const int j = (int)(i % cols);
  double floor_ = lam[0] * 1e-28;
  if (!(floor_ > 0.0)) floor_ = 1e-300;
  const double l = lam[j] > floor_ ? lam[j] : floor_;
  out[i] = W[i] / sqrt(l);
}

// Per column j of E (rows x cols, row-major, ld): unit-normalise (useless/train.py:94-95)
// and apply sklearn's svd_flip row rule (largest-|.| entry positive, first on ties;
// extmath.py:946-952).  Writes comps[j][r] (k x rows) and En[r][j] (rows x k).
__global__ __launch_bounds__(256) void normalize_sign_kernel(const double* __restrict__ E, int64_t rows,
                                                             int cols, int64_t ld,
                                                             double* __restrict__ comps,
                                                             double* __restrict__ En) {
  __shared__ double rs[256];
  __shared__ double rm[256];
  __shared__ long long ri[256];
  const int j = blockIdx.x;
  double ss = 0.0, mx = -1.0;
  long long mi = LLONG_MAX;
  for (int64_t r = threadIdx.x; r < rows; r += 256) {
    const double v = E[r * ld + j];
    ss += v * v;
    const double a = fabs(v);
    if (a > mx) { mx = a; mi = r; }
  }
  rs[threadIdx.x] = ss;
  rm[threadIdx.x] = mx;
  ri[threadIdx.x] = mi;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      rs[threadIdx.x] += rs[threadIdx.x + w];
      const double om = rm[threadIdx.x + w];
      const long long oi = ri[threadIdx.x + w];
      if (om > rm[threadIdx.x] || (om == rm[threadIdx.x] && oi < ri[threadIdx.x])) {
        rm[threadIdx.x] = om;
        ri[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  const double nrm = sqrt(rs[0]);
  const double piv = ri[0] == LLONG_MAX ? 1.0 : E[ri[0] * ld + j];
  const double f = (piv < 0.0 ? -1.0 : 1.0) / (nrm > 0.0 ? nrm : 1.0);
  for (int64_t r = threadIdx.x; r < rows; r += 256) {
    const double v = E[r * ld + j] * f;
    comps[(int64_t)j * rows + r] = v;
    if (En) En[r * cols + j] = v;
  }
}

hipError_t launch_colstats(hipStream_t s, const uint8_t* X, int64_t n, int64_t d,
                           unsigned long long* S1, unsigned long long* S2) {
  const int64_t cgroups = (d + 255) / 256;
  int64_t ny = (262144 + d - 1) / d;  // ~256K threads in flight
  if (ny > n) ny = n;
  if (ny < 1) ny = 1;
  if (ny > 65535) ny = 65535;
  const int64_t rows_per = (n + ny - 1) / ny;
  ny = (n + rows_per - 1) / rows_per;
  hipLaunchKernelGGL(colstats_kernel, dim3((unsigned)cgroups, (unsigned)ny), dim3(256), 0, s, X, n, d,
                     rows_per, S1, S2);
  return hipGetLastError();
}

static int64_t colstats_float_blocks(int64_t n, int64_t d) {
  int64_t ny = (262144 + d - 1) / d;
  if (ny > n) ny = n;
  if (ny < 1) ny = 1;
  if (ny > 1024) ny = 1024;
  return ny;
}

size_t colstats_float_work_elems(int64_t n, int64_t d) { return (size_t)2 * colstats_float_blocks(n, d) * d; }

hipError_t launch_colstats_float(hipStream_t s, const void* X, int elem, int64_t n, int64_t d, int standardize,
                                 double* part, double* mean, double* var, double* scale, double* w) {
  int64_t ny = colstats_float_blocks(n, d);
  const int64_t rows_per = (n + ny - 1) / ny;
  ny = (n + rows_per - 1) / rows_per;
  const dim3 grid((unsigned)((d + 255) / 256), (unsigned)ny);
  const unsigned cb = (unsigned)((d + 255) / 256);
  double* part2 = part + ny * d;
  for (int pass = 0; pass < 2; ++pass) {
    const double* m = pass ? mean : nullptr;
    if (elem == EF_F32)
      hipLaunchKernelGGL(colsum_float_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(X), n, d,
                         rows_per, m, part, part2);
    else if (elem == EF_F64)
      hipLaunchKernelGGL(colsum_float_kernel<double>, grid, dim3(256), 0, s, static_cast<const double*>(X), n, d,
                         rows_per, m, part, part2);
    else
      return hipErrorInvalidValue;
    if (pass == 0)
      hipLaunchKernelGGL(colmean_float_kernel, dim3(cb), dim3(256), 0, s, part, (int)ny, n, d, mean);
  }
  hipLaunchKernelGGL(colvar_float_kernel, dim3(cb), dim3(256), 0, s, part, part2, (int)ny, n, d, standardize, mean,
                     var, scale, w);
  return hipGetLastError();
}

hipError_t launch_stats_finalize(hipStream_t s, const unsigned long long* S1, const unsigned long long* S2,
                                 int64_t n, int64_t d, int standardize, double* mean, double* var,
                                 double* scale, double* w) {
  hipLaunchKernelGGL(stats_finalize_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, S1, S2,
                     n, d, standardize, mean, var, scale, w);
  return hipGetLastError();
}

hipError_t launch_trace(hipStream_t s, const double* C, int64_t m, int64_t ldc, double* out) {
  hipLaunchKernelGGL(trace_kernel, dim3(1), dim3(256), 0, s, C, m, ldc, out);
  return hipGetLastError();
}

hipError_t launch_rand_init(hipStream_t s, double* Q, int64_t count, unsigned long long seed) {
  hipLaunchKernelGGL(rand_init_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, Q, count,
                     seed);
  return hipGetLastError();
}

hipError_t launch_scale_cols_rsqrt(hipStream_t s, const double* W, int64_t rows, int cols,
                                   const double* lam, double* out) {
  const int64_t tot = rows * cols;
  hipLaunchKernelGGL(scale_cols_rsqrt_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, W,
                     rows, cols, lam, out);
  return hipGetLastError();
}

hipError_t launch_normalize_sign(hipStream_t s, const double* E, int64_t rows, int cols, int64_t ld,
                                 double* comps, double* En) {
  hipLaunchKernelGGL(normalize_sign_kernel, dim3((unsigned)cols), dim3(256), 0, s, E, rows, cols, ld,
                     comps, En);
  return hipGetLastError();
}

}  // namespace ef
