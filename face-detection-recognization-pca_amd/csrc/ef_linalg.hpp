// Fit-path (float64) kernel interfaces.
#pragma once

#include "ef_internal.hpp"

namespace ef {

// 1/x and 1/sqrt(x) (x > 0) from v_rcp_f64 / v_rsq_f64 refined by two Newton steps (~1 ulp;
// a few dependent instructions instead of the IEEE division / square-root sequences) for
// the serial chains of the small eigen- and Cholesky solvers
__device__ __forceinline__ double rcp_nr(double x) {
  double y = __builtin_amdgcn_rcp(x);
  y = fma(y, fma(-x, y, 1.0), y);
  return fma(y, fma(-x, y, 1.0), y);
}
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = fma(0.5 * y, fma(-x * y, y, 1.0), y);
  return fma(0.5 * y, fma(-x * y, y, 1.0), y);
}

// LDS-only workgroup barrier: waits for this wave's LDS operations (and scalar loads), not
// for its global stores and atomics, which __syncthreads also waits to complete.  For
// kernels whose global writes are read only by later launches or the host.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Loader semantics: L(r, c) = trans ? M[c][r] : M[r][c] for the stored row-major M.
// A operands are read as A(m, k), B operands as B(k, n).  kfast tells the staging loop
// which tile index is contiguous in memory so global reads coalesce.
struct DenseLd {
  const double* p;
  int64_t ld;
  int trans;
  bool kfast;
  __device__ __forceinline__ double operator()(int64_t r, int64_t c) const {
    return trans ? p[c * ld + r] : p[r * ld + c];
  }
};

// Stored M = X[sample][pixel] of element type T (uint8 pixels, or float / double for
// already-scaled data such as ManualStandardScaler's output); value = (x - mu[pixel]) *
// w[pixel] (w may be null).
template <class T>
struct PixLd {
  const T* x;
  int64_t ld;
  int trans;
  const double* mu;
  const double* w;
  bool kfast;
  __device__ __forceinline__ double operator()(int64_t r, int64_t c) const {
    const int64_t smp = trans ? c : r;
    const int64_t px = trans ? r : c;
    const double v = (double)x[smp * ld + px] - mu[px];
    return w ? v * w[px] : v;
  }
};
using U8Ld = PixLd<uint8_t>;

// Host-side operand description for gemm64.  elem: EF_U8 / EF_F32 / EF_F64 for a pixel
// operand (x), -1 for a dense fp64 matrix (p).
struct Operand {
  bool u8 = false;  // pixel operand (any element type): read through PixLd
  int elem = -1;
  const double* p = nullptr;
  const void* x = nullptr;
  int64_t ld = 0;
  int trans = 0;
  bool sym = false;  // symmetric: either orientation may be read (tall GEMM walks its rows)
  const double* mu = nullptr;
  const double* w = nullptr;
  static Operand symmetric(const double* p, int64_t ld) {
    Operand o = dense(p, ld, false);
    o.sym = true;
    return o;
  }
  static Operand dense(const double* p, int64_t ld, bool trans) {
    Operand o;
    o.p = p;
    o.ld = ld;
    o.trans = trans;
    return o;
  }
  static Operand pixels(const void* x, int elem, int64_t ld, bool trans, const double* mu, const double* w) {
    Operand o;
    o.u8 = true;
    o.elem = elem;
    o.x = x;
    o.ld = ld;
    o.trans = trans;
    o.mu = mu;
    o.w = w;
    return o;
  }
  static Operand pixels(const uint8_t* x, int64_t ld, bool trans, const double* mu, const double* w) {
    return pixels(x, EF_U8, ld, trans, mu, w);
  }
};

// C[M][N] = alpha * A . B (split-K slabs in `work` when it helps; work may be null).
hipError_t gemm64(hipStream_t s, const Operand& A, const Operand& B, int64_t M, int64_t N, int64_t K,
                  double alpha, double* C, int64_t ldc, double* work, size_t work_elems);

size_t jacobi_lds_bytes(int m);

// Tall dense GEMMs on the matrix cores (ef_dgemm.hip): C[M x N] = alpha A[M x K] B[K x N]
// with B given TRANSPOSED (Bt: N x K, row-major, ldbt) and A row-major or, with a_trans,
// stored transposed (element (i, k) at A[k * lda + i]; a symmetric A either way); N <= 512
// intended; work: split-K slabs (M*N*splits elements, may be null).  Rows of A (a_trans:
// of A^T) and of Bt must be 16-byte aligned (tall_gemm_supported).
bool tall_gemm_supported(int64_t ld, const void* p, int elem_bytes);
hipError_t tall_gemm_f64(hipStream_t s, const double* A, int64_t lda, bool a_trans, const double* Bt, int64_t ldbt,
                         double* C, int64_t ldc, int64_t M, int64_t N, int64_t K, double alpha, double* work,
                         size_t work_elems);
hipError_t tall_gemm_f32(hipStream_t s, const float* A, int64_t lda, bool a_trans, const float* Bt, int64_t ldbt,
                         float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha, float* work,
                         size_t work_elems);
// Split-bf16 tall GEMM of the fit's coarse phase (ef_gemm_s3.hip): Y (M x 256, fp64) =
// A3 . Bt3^T - sigma Q with A3 (M x K, lda) and Bt3 (256 x K, ldb) in the split layout
// (launch_split_f64 / launch_transpose_split); part: gemm_s3_part_elems(M) floats.
bool gemm_s3_supported(int64_t M, int64_t K, int64_t N);
size_t gemm_s3_part_elems(int64_t M);
hipError_t launch_split_f64(hipStream_t s, const double* x, int64_t n, void* out);
hipError_t launch_transpose_split(hipStream_t s, const double* Q, int64_t dim, void* Bt3);
hipError_t gemm_s3(hipStream_t s, const float* A3, int64_t lda, const float* Bt3, int64_t ldb, int64_t M, int64_t K,
                   float* part, const double* Q, double sigma, double* Y);
// out (cols x rows, ldout) = in (rows x cols, ldin)^T; the second also converts to fp32
hipError_t launch_transpose_f64(hipStream_t s, const double* in, int64_t ldin, int64_t rows, int64_t cols, double* out,
                                int64_t ldout);
hipError_t launch_transpose_f64_to_f32(hipStream_t s, const double* in, int64_t ldin, int64_t rows, int64_t cols,
                                       float* out, int64_t ldout);
// Li = L^-1 for a lower-triangular m x m L (m <= 512), row-major
hipError_t launch_tri_inv(hipStream_t s, const double* L, int m, double* Li);
hipError_t launch_jacobi(hipStream_t s, const double* A, int m, int64_t lda, double* evals, double* evecs,
                         int64_t ldv, int max_sweeps, int* info);
// Grid-parallel Jacobi for any order (ef_jacobi_big.hip): one hipGraph per sweep, built
// once per (order, workspace).  work: jacobi_big_work_elems(m) doubles.  solve returns 0
// converged, 1 not converged, -1 HIP error (*err).
size_t jacobi_big_work_elems(int m);
struct JacobiBig {
  int m = 0, mp = 0;
  bool block = false;  // block-Jacobi rounds (orders >= 128)
  bool fused = true;   // block path: a round's solve and the previous round's apply in one launch
  int rounds() const { return block ? mp / 16 - 1 : mp - 1; }
  double* work = nullptr;
  int* flag = nullptr;
  void* exec[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  // block path: the sweep's largest off-diagonal ratio (double bits, atomicMax), the slot
  // after the tolerance scalar in work
  unsigned long long* pmax_slot() const {
    return reinterpret_cast<unsigned long long*>(work + 4 * (int64_t)mp * mp + 4 * 16 * (int64_t)mp + 1);
  }
  hipError_t init(int m, double* work, int* flag, hipStream_t capture);
  // tol: a sweep in which no off-diagonal entry exceeds tol of its diagonal scale ends the
  // solve (block path; the scalar rounds always use 1e-12)
  int solve(hipStream_t s, const double* A, int64_t lda, double* evals, double* evecs, int64_t ldv, int max_sweeps,
            int* sweeps_out, hipError_t* err, double tol = 1e-12);
  void destroy();
  ~JacobiBig() { destroy(); }
};
// Exact integer covariance / Gram on int8 MFMA (ef_cov_i8.hip).  At: dim x cov_i8_kpad(K)
// bytes in the K-blocked layout [kpad/64][dim][64]; slabs: plan.slab_elems int32; S64:
// dim*dim int64 (only when plan.passes > 1); cvec: d int64, R: n int64 (Gram), Q2: 2 uint64.
struct CovPlan {
  int64_t nst = 0;              // 64-sample K stages
  int64_t stages_per_pass = 0;  // K stages per syrk launch
  int64_t kps = 0;              // K stages per work item (<= 2047: int32-exact)
  int64_t slab_elems = 0;       // splits * dim * dim
  int ntiles = 0, splits = 1, passes = 1;
  int tj = 256;                 // SYRK tile columns (tiles are 256 x tj)
  int njb = 0;                  // > 0: the 16x16x64 kernel (syrk16_i8_kernel, tj = 64 njb)
};
int64_t cov_i8_kpad(int64_t K);
constexpr int64_t kSyrkPadBytes = 384 * 64;  // readable slack the At allocation carries past its end
int64_t cov_i8_order_bytes(int64_t dim);  // device scratch for the tile order list
CovPlan cov_i8_plan(int64_t dim, int64_t K, int64_t slab_budget);
bool cov_i8_fused_stats(const uint8_t* X, int64_t d);  // covariance-path prep can produce S1/S2
// Gram path: At = X' (K = d).  Covariance path: At = X'^T (K = n); with S1/S2 non-null
// (requires cov_i8_fused_stats) also S1 += sum x, S2 += sum x^2 per pixel.
hipError_t launch_cov_i8_prep(hipStream_t s, const uint8_t* X, int64_t n, int64_t d, bool gram, uint8_t* At,
                              unsigned long long* S1, unsigned long long* S2);
hipError_t launch_cov_i8(hipStream_t s, const CovPlan& p, int64_t n, int64_t d, bool gram,
                         const unsigned long long* S1, const double* w, const uint8_t* At, int* slabs,
                         long long* S64, long long* cvec, long long* R, unsigned long long* Q2, void* order_dev,
                         double* C, hipEvent_t syrk_begin = nullptr, hipEvent_t syrk_end = nullptr);
// Sample-sharded covariance (ef_fit_shard_stats / ef_fit_from_stats): S64 (int64, d x d;
// the upper 64-blocks exact) = X'^T X' of the rows in At (covariance-path layout, K = n),
// every pass's int32 slabs accumulated; then C from globally summed pieces (S64, S1, n) with
// the finalize arithmetic of launch_cov_i8 — the same integer gives the same double.
hipError_t launch_cov_i8_cross(hipStream_t s, const CovPlan& p, int64_t d, const uint8_t* At, int* slabs,
                               long long* S64, void* order_dev);
hipError_t launch_cov_from_cross(hipStream_t s, const long long* S64, const unsigned long long* S1, int64_t n,
                                 int64_t d, const double* w, long long* cvec, double* C);
hipError_t launch_cholesky(hipStream_t s, double* A, int m, int64_t lda, double tol_rel, int* info);
// Li = L^-1 (row-major, zeros above the diagonal) for G = L L^T, m <= 256
// (chol_inv_supported); G is not modified; *info as launch_cholesky.  launch_chol_inv: the
// blocked one-workgroup Cholesky + block-column-parallel inverse (ef_chol_blk.hip; work:
// chol_inv_work_elems(m) doubles); launch_chol_inv_reg: round 4's register-resident
// single-workgroup kernel (m even), kept for A/B and the microbenchmark.
bool chol_inv_supported(int m);
size_t chol_inv_work_elems(int m);
hipError_t launch_chol_inv(hipStream_t s, const double* G, int m, int64_t lda, double tol_rel, double* Li, int* info,
                           double* work);
bool chol_inv_reg_supported(int m);
hipError_t launch_chol_inv_reg(hipStream_t s, const double* G, int m, int64_t lda, double tol_rel, double* Li,
                               int* info);
// Training projection F (n x kk, fp64) = ((X - mu) * w) . E on int8 MFMA with E split into
// base-256 digits (ef_proj_i8.hip); w may be null.  work: proj_i8_work_bytes bytes.
bool proj_i8_supported(const uint8_t* X, int64_t n, int64_t d, int kk);
size_t proj_i8_work_bytes(int64_t n, int64_t d, int kk);
hipError_t launch_proj_i8(hipStream_t s, const uint8_t* X, int64_t n, int64_t d, const double* mu, const double* w,
                          const double* E, int kk, void* work, double* F);
// The fit's fine-phase product Y = C.Q - sigma Q (C symmetric dim x dim, Q dim x m) on the
// int8 matrix cores with C and Q cut into base-256 digits (ef_cq_i8.hip, launch_cq_i8):
// planes (cq_i8_plane_bytes: C's digit planes + room for Q's) from launch_cq_i8_planes once
// per C; work: cq_i8_work_bytes.
bool cq_i8_supported(int64_t dim, int m);
size_t cq_i8_plane_bytes(int64_t dim);
size_t cq_i8_work_bytes(int64_t dim, int m);
hipError_t launch_cq_i8_planes(hipStream_t s, const double* C, int64_t dim, void* planes);
hipError_t launch_cq_i8(hipStream_t s, void* planes, int64_t dim, const double* Q, int m, double sigma, void* work,
                        double* Y, bool medium = false);
// Its digit-pair products (ef_cov_i8.hip, syrk16_i8_kernel's OZ items).  Full form
// (med = false): every pair a + b >= 5 of the 6 + 6 digits, 21; medium form (med = true,
// the products no Rayleigh-Ritz step reads directly): a, b >= 1 and a + b >= 6, 15 pairs,
// ~2^-40 of the full product (its lowest level and both lowest digits dropped).  Pair p
// enumerates a descending, b ascending; the last pair — (0, 5) full, (1, 5) medium — runs
// in kOzSplitParts K-parts (so 64 row blocks fill 256 CUs in whole-round steps); output
// block p, then the parts, each dim x 256 int32.  Z: the K-blocked [dim/64][R][64] digits.
constexpr int kOzSplitParts = 4;
__host__ __device__ constexpr int oz_pairs(bool med) { return med ? 15 : 21; }
__host__ __device__ constexpr int oz_blocks(bool med) { return oz_pairs(med) - 1 + kOzSplitParts; }
constexpr int kOzBlocks = oz_blocks(false);  // the larger
__host__ __device__ inline void oz_pair(int p, bool med, int& a, int& b) {
  const int lo = med ? 1 : 0, lev = med ? 6 : 5;  // smallest digit, smallest level a + b
  a = 5;
  int base = 0;
  for (;;) {
    const int b0 = lev - a > lo ? lev - a : lo, cnt = 6 - b0;
    if (p < base + cnt) {
      b = b0 + (p - base);
      return;
    }
    base += cnt;
    --a;
  }
}
hipError_t launch_oz_syrk16(hipStream_t s, const uint8_t* Z, int64_t dim, int64_t R, int* I, bool med);
hipError_t launch_colstats(hipStream_t s, const uint8_t* X, int64_t n, int64_t d,
                           unsigned long long* S1, unsigned long long* S2);
// Float input (EF_F32 / EF_F64): column mean and population variance in fp64 by two
// passes with the one-batch form of sklearn's _incremental_mean_and_var (extmath.py:
// mean = sum/n; var = (sum t^2 - (sum t)^2/n)/n with t = x - mean), partial sums per row
// block added in a fixed order (deterministic); then the StandardScaler rule as
// launch_stats_finalize.  part: colstats_float_work_elems(n, d) doubles.
size_t colstats_float_work_elems(int64_t n, int64_t d);
hipError_t launch_colstats_float(hipStream_t s, const void* X, int elem, int64_t n, int64_t d, int standardize,
                                 double* part, double* mean, double* var, double* scale, double* w);
hipError_t launch_stats_finalize(hipStream_t s, const unsigned long long* S1, const unsigned long long* S2,
                                 int64_t n, int64_t d, int standardize, double* mean, double* var,
                                 double* scale, double* w);
hipError_t launch_trace(hipStream_t s, const double* C, int64_t m, int64_t ldc, double* out);
hipError_t launch_rand_init(hipStream_t s, double* Q, int64_t count, unsigned long long seed);
hipError_t launch_scale_cols_rsqrt(hipStream_t s, const double* W, int64_t rows, int cols,
                                   const double* lam, double* out);
hipError_t launch_normalize_sign(hipStream_t s, const double* E, int64_t rows, int cols, int64_t ld,
                                 double* comps, double* En);

}  // namespace ef
