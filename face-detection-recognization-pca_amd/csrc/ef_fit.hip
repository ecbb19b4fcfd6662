// ef_fit: the eigenfaces fit on the GPU (mean -> centre -> covariance -> eigensolve ->
// back-project -> unit eigenfaces -> training projection), float64 throughout.
//
// Restates manual_pca (useless/train.py:56-128) and, with EF_FIT_STANDARDIZE, the
// StandardScaler + PCA(svd_solver='full') fit of train-v4.py:126-146:
//   * covariance: Gram A.A^T/(n-1) when n < d (useless/train.py:82-85), else the d x d
//     A^T.A/(n-1) (np.cov branch, :97-99).  Exact integer products on the int8 matrix
//     cores (ef_cov_i8.hip) whenever the StandardScaler weights commute with them
//     (covariance path, and the Gram path without scaling); the standardised Gram runs
//     the f64 MFMA GEMM with centring and 1/scale applied in the operand loads;
//   * eigensolve: orders <= kJacobiMax go straight to the LDS Jacobi kernel, k > 80 on
//     orders <= 1024 to the grid-parallel Jacobi (ef_jacobi_big.hip); larger problems
//     run block subspace iteration (Y = C.Q; G = Y^T.Y; G = W.L.W^T by Jacobi;
//     Q = Y.W.L^-1/2) to convergence, then a Rayleigh-Ritz step (T = Q^T.C.Q, Jacobi)
//     — the top-k pairs are all manual_pca keeps (:114-116) and all sklearn reports
//     (explained_variance_ratio_ uses trace(C) as the total, _pca.py:644-646);
//   * eigenfaces: E = A^T.U (:91), unit columns (:94-95), sklearn svd_flip sign rule.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ef_linalg.hpp"

namespace {

using namespace ef;

// Workspaces of one fit: slots of the context's pool (ef_ctx::fit_pool), grown on demand
// and kept for the next fit — a C3 fit otherwise spends tens of ms in hipMalloc/hipFree of
// its ~30 GB of operand copies and blocks.  ef_trim releases the pool.
struct Bufs {
  size_t next = 0;
  template <class T>
  void drop(hipStream_t, T*) {}  // pooled: the slot stays allocated for the next fit
  template <class T>
  int get(ef_ctx* c, size_t count, T** out) {
    if (c->fit_pool.size() <= next) c->fit_pool.resize(next + 1);
    DevBuf& b = c->fit_pool[next++];
    const int rc = ensure(c, b, count * sizeof(T) + 16);
    *out = static_cast<T*>(b.p);
    return rc;
  }
};

#define EF_TRY(expr)              \
  do {                            \
    int _rc = (expr);             \
    if (_rc != EF_OK) return _rc; \
  } while (0)
#define EF_HIP(ctx, expr, what)                          \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return hip_err(ctx, _e, what); \
  } while (0)

// Plain dense fp64 products of the subspace iteration with a large output (C.Q, Y.V, Q.V)
// run on the tall matrix-core GEMM (ef_dgemm.hip), which takes B transposed: B^T is
// written into bt_scratch (>= K x N doubles) first — at most dim x m, 32 MiB at C3, a few
// microseconds.  Products with a small output over a long K (Y^T.Y, Q^T.Y) and the
// pixel-operand products keep gemm64's split-K.
hipError_t dense_gemm(ef_ctx* c, hipStream_t s, const Operand& A, const Operand& B, int64_t M, int64_t N, int64_t K,
                      double alpha, double* C, int64_t ldc, double* work, size_t work_elems,
                      double* bt_scratch = nullptr) {
  (void)c;
  const bool small_out = M * N <= (int64_t)512 * 512 && K >= 4096;
  // Y^T.Y, Q^T.Y (small output, long K, A given transposed): B transposed once into
  // bt_scratch, then the register-direct tall kernel walking down A's rows with split-K —
  // the LDS-staged split-K gemm64 is latency-bound here (C3: 79 + 18 us per product)
  bool tn_tall = true;
#ifdef EF_DIAGNOSTICS
  if (const char* e = getenv("EF_FIT_TN_TALL")) tn_tall = atoi(e) != 0;
#endif
  if (tn_tall && bt_scratch && small_out && A.trans && !B.trans && !A.u8 && !B.u8 && tall_gemm_supported(A.ld, A.p, 8) &&
      tall_gemm_supported(K, bt_scratch, 8)) {
    hipError_t e = launch_transpose_f64(s, B.p, B.ld, K, N, bt_scratch, K);
    if (e != hipSuccess) return e;
    return tall_gemm_f64(s, A.p, A.ld, true, bt_scratch, K, C, ldc, M, N, K, alpha, work, work_elems);
  }
  if (bt_scratch && !A.u8 && !B.u8 && !A.trans && !B.trans && !small_out && tall_gemm_supported(A.ld, A.p, 8) &&
      tall_gemm_supported(K, bt_scratch, 8)) {
    hipError_t e = launch_transpose_f64(s, B.p, B.ld, K, N, bt_scratch, K);
    if (e != hipSuccess) return e;
    return tall_gemm_f64(s, A.p, A.ld, false, bt_scratch, K, C, ldc, M, N, K, alpha, work, work_elems);
  }
  return gemm64(s, A, B, M, N, K, alpha, C, ldc, work, work_elems);
}

constexpr int kMaxSweeps = 60;
constexpr int kDirectMax = 1024;                 // direct grid-Jacobi up to this order
constexpr size_t kWorkElems = size_t(1) << 24;  // split-K slab budget (128 MiB)

// Small symmetric eigenproblem G (m x m) -> descending eigenvalues + eigenvectors:
// the LDS Jacobi up to kJacobiMax, the grid-parallel Jacobi beyond.
struct SmallEig {
  int m = 0;
  int* info = nullptr;
  double* jwork = nullptr;
  JacobiBig big;
  long sweeps = 0, calls = 0;  // grid-Jacobi statistics (EF_FIT_DEBUG)
  int init(ef_ctx* c, Bufs& B, int m_) {
    m = m_;
    EF_TRY(B.get(c, 4, &info));
    if (m > kJacobiMax) {
      EF_TRY(B.get(c, jacobi_big_work_elems(m), &jwork));
      EF_HIP(c, big.init(m, jwork, info, c->own_stream), "jacobi graph");
    }
    return EF_OK;
  }
  // tol: the block-Jacobi stopping tolerance (relative off-diagonal size); 1e-12 except
  // for Rayleigh-Ritz solves whose Ritz values cannot decide convergence (see below)
  int solve(ef_ctx* c, const double* G, int64_t ldg, double* lam, double* V, int64_t ldv, const char* what,
            double tol = 1e-12) {
    hipStream_t s = c->stream;
    if (m <= kJacobiMax) {
      EF_HIP(c, launch_jacobi(s, G, m, ldg, lam, V, ldv, kMaxSweeps, info), what);
      int hinfo = 0;
      EF_HIP(c, hipMemcpyAsync(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost, s), "D2H info");
      EF_HIP(c, hipStreamSynchronize(s), "sync");
      if (hinfo < 0) return set_err(c, EF_E_NUMERIC, std::string(what) + ": Jacobi did not converge");
      return EF_OK;
    }
    hipError_t e = hipSuccess;
    int sw = 0;
    const int rc = big.solve(s, G, ldg, lam, V, ldv, kMaxSweeps, &sw, &e, tol);
    sweeps += sw;
    ++calls;
    if (rc < 0) return hip_err(c, e, what);
    if (rc > 0) return set_err(c, EF_E_NUMERIC, std::string(what) + ": Jacobi did not converge");
    return EF_OK;
  }
};

// Wide-block subspace iteration (m > kJacobiMax): orthonormalise by CholQR every
// iteration (G = Y^T.Y = L.L^T, Q = Y.L^-T — one small Cholesky instead of an m x m
// eigensolve), Rayleigh-Ritz (H = Q^T.C.Q, block Jacobi) at iterations (1, 2, 4,) 8 and every
// rr_period(dim) after: its Ritz values give the convergence test, its vectors re-order the
// block (Y <- Y.V), and the converged RR is the final one.  A numerically rank-deficient
// block (Cholesky pivot <= 1e-13 of the largest) falls back to the eigen-orthonormalisation
// Q = Y.W.L^-1/2 for that iteration.
// Rayleigh-Ritz period: a grid-Jacobi RR costs ~ a few iterations at dim ~ 16k, ~10 at dim ~ 2k
inline int rr_period(int64_t dim) { return dim >= 12288 ? 8 : 16; }
inline double rr_loose_tol() {
#ifdef EF_DIAGNOSTICS  // EF_FIT_RR_LOOSE: the coarse-phase Rayleigh-Ritz tolerance (A/B; 1e-12 = off)
  if (const char* e = getenv("EF_FIT_RR_LOOSE")) return atof(e);
#endif
  return 1e-4;
}
// The first Rayleigh-Ritz step's tolerance: its Ritz values only set the first shift and
// Chebyshev rate (there is no previous step to compare with), and its basis is re-mixed
// by the products and CholQR factors that follow.  1e-2 takes 2 of the C3 fit's 20 Jacobi
// sweeps off, ~1.9 ms, same 23 iterations, eigenvalues equal to 3e-15
// (profiles/r05/rr_first_ab.txt).
inline double rr_first_tol() {
#ifdef EF_DIAGNOSTICS  // EF_FIT_RR_FIRST (A/B)
  if (const char* e = getenv("EF_FIT_RR_FIRST")) return atof(e);
#endif
  return 1e-2;
}
// Ritz-residual acceptance: a Rayleigh-Ritz step after an fp64 product also ends the
// iteration when every kept pair has |C u_i - theta_i u_i| <= 1e-9 theta_1.  Then each
// theta_i is within |r|^2 / gap of an eigenvalue and u_i within |r| / gap of its vector.
// The value-change test needs a second fp64 step to compare with.  The residual test
// decides from one step, so the C3 fit stops after 22 products instead of 23.  Its
// eigenvalues move by 1.6e-13 and its components by 1.7e-8 against the 23-product fit,
// 4.7 ms per fit (profiles/r05/resid_ab.txt).  The residuals come from Y.V, the
// continuation product, and U = Q.V, the result's.
inline double fit_resid_tol() {
#ifdef EF_DIAGNOSTICS  // EF_FIT_RESID_TOL (A/B; 0 = off)
  if (const char* e = getenv("EF_FIT_RESID_TOL")) return atof(e);
#endif
  return 1e-9;
}
// Gap-aware acceptance (round 6): the residual bounds the eigenvector error only through
// |r_i| / gap_i (Davis-Kahan), so EVERY acceptance — residual or value-change — also needs
// |r_i| <= 1e-5 gap_i for each kept pair, gap_i the distance from theta_i to the nearest
// other Ritz value of the block (theta_{k+1} included).  On the reference's Dark spectrum
// (min gap 2.4e-6 lambda_1, models/Joseph_Lai_dark_model_info.json) the absolute test alone
// guaranteed only 4.2e-4.  Gaps below the fp64 residual floor (1e-12 theta_1 / 1e-5: an
// exactly or numerically degenerate pair, whose vectors are not unique) are held to that
// floor instead, and a value-converged step whose residuals stopped shrinking is accepted
// (the floor of the arithmetic), so a degenerate spectrum still terminates.
inline double fit_gap_tol() {
#ifdef EF_DIAGNOSTICS  // EF_FIT_GAP_TOL (A/B; 0 = off)
  if (const char* e = getenv("EF_FIT_GAP_TOL")) return atof(e);
#endif
  return 1e-5;
}
constexpr double kResidFloor = 1e-12;  // |r_i| / theta_1 always accepted by the gap rule
constexpr int kCholeskyMax = 512;  // launch_cholesky's LDS panel limit (wider: eigen-orthonormalise)

__global__ void f64_to_f32_kernel(const double* __restrict__ a, int64_t n, float* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    b[i] = (float)a[i];
}
// Y (-)= sigma Q: the shifted product (C - sigma I) Q of the subspace iteration; the fp32
// coarse phase converts its product and shifts in one pass
__global__ void shift_kernel(double* __restrict__ y, const double* __restrict__ q, int64_t n, double sigma) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = fma(-sigma, q[i], y[i]);
}
__global__ void f32_to_f64_shift_kernel(const float* __restrict__ a, const double* __restrict__ q, int64_t n,
                                        double sigma, double* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    b[i] = fma(-sigma, q[i], (double)a[i]);
}
// Deferred CholQR check: the fit's sticky failure flag |= this factor's info
__global__ void sticky_info_kernel(const int* __restrict__ info, int* __restrict__ sticky) {
  if (*info != 0) *sticky = 1;
}
// subspace_wide's "a deferred Cholesky failed: run again with a host check per iteration"
constexpr int kRetryChecked = 1000;

// Chebyshev step of the subspace iteration: y = s * y - w (w null: y = s * y)
__global__ void cheb_combine_kernel(double* __restrict__ y, const double* __restrict__ w, int64_t n, double sc) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = w ? fma(sc, y[i], -w[i]) : sc * y[i];
}
// Ritz residuals of a Rayleigh-Ritz step: partial sums of |YV_i - lam_i U_i|^2 over row
// chunk blockIdx.y for columns 64 blockIdx.x + (tid & 63) (rows strided by the four
// 64-thread groups), YV = (C - sigma I) Q V and U = Q V; summed in chunk order on the host
// (deterministic).  part: [gridDim.y][kk].
constexpr int kResidChunks = 16;
__global__ __launch_bounds__(256) void ritz_resid_kernel(const double* __restrict__ YV, int64_t ldy,
                                                         const double* __restrict__ U, int64_t ldu,
                                                         const double* __restrict__ lam, int64_t dim, int kk,
                                                         double* __restrict__ part) {
  __shared__ double red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const int64_t r0 = dim * blockIdx.y / gridDim.y, r1 = dim * (blockIdx.y + 1) / gridDim.y;
  double acc = 0.0;
  if (col < kk) {
    const double l = lam[col];
    for (int64_t r = r0 + g; r < r1; r += 4) {
      const double d = fma(-l, U[r * ldu + col], YV[r * ldy + col]);
      acc = fma(d, d, acc);
    }
  }
  red[g][threadIdx.x & 63] = acc;
  __syncthreads();
  if (g == 0 && col < kk)
    part[(int64_t)blockIdx.y * kk + col] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                                           red[3][threadIdx.x];
}

static void cvt64to32(hipStream_t s, const double* a, int64_t n, float* b) {
  hipLaunchKernelGGL(f64_to_f32_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0, s, a, n,
                     b);
}

// deferred: the per-iteration Cholesky success check is made at the next Rayleigh-Ritz
// step instead of by a host round trip every iteration; a failure found there returns
// kRetryChecked (the caller runs the checked form, which takes the rank-deficient fallback
// in the iteration that needs it).
int subspace_wide(ef_ctx* c, Bufs& B, const double* C, int64_t dim, int kk, int m, double* work, double* U_out,
                  double* lam_out, int* iters, bool deferred) {
  hipStream_t s = c->stream;
  SmallEig se;
  EF_TRY(se.init(c, B, m));
  double *Q, *Y, *Y2, *G, *V, *W2, *Li, *Bt, *lam;
  int* cinfo;
  EF_TRY(B.get(c, (size_t)m * m, &Li));
  EF_TRY(B.get(c, (size_t)dim * m, &Bt));
  EF_TRY(B.get(c, (size_t)dim * m, &Q));
  EF_TRY(B.get(c, (size_t)dim * m, &Y));
  EF_TRY(B.get(c, (size_t)dim * m, &Y2));
  EF_TRY(B.get(c, (size_t)m * m, &G));
  EF_TRY(B.get(c, (size_t)m * m, &V));
  EF_TRY(B.get(c, (size_t)m * m, &W2));
  EF_TRY(B.get(c, (size_t)m, &lam));
  EF_TRY(B.get(c, 4, &cinfo));
  double* CW;  // blocked Cholesky + inverse scratch
  EF_TRY(B.get(c, chol_inv_work_elems(m), &CW));
  double* RP;  // Ritz residual partial sums [kResidChunks][kk]
  EF_TRY(B.get(c, (size_t)kResidChunks * kk, &RP));
  std::vector<double> rp((size_t)kResidChunks * kk);
  // Chebyshev recurrence state (EF_OPT_FIT_CHEBYSHEV): Qold = the block before the last
  // orthonormalisation, Wc = the previous filter iterate in the current block's frame
  double *Qold, *Wc;
  EF_TRY(B.get(c, (size_t)dim * m, &Qold));
  EF_TRY(B.get(c, (size_t)dim * m, &Wc));
  bool carried = false;
  int* sticky;  // deferred Cholesky failures since the fit began
  EF_TRY(B.get(c, 4, &sticky));
  const bool defer = deferred && chol_inv_supported(m);
  if (defer) EF_HIP(c, hipMemsetAsync(sticky, 0, sizeof(int), s), "sticky");
  EF_HIP(c, launch_rand_init(s, Y, dim * m, 0x5eedULL), "rand init");

  // Q <- orthonormal basis of span(Y) (Y is overwritten).  carry: also map the block
  // being replaced into the new frame, Wc = Qold . L^-T (the same right factor), which is
  // what the three-term recurrence needs (sets `carried`; the rank-deficient fallback
  // does not carry, and the recurrence restarts).
  auto orthonormalise = [&](bool carry) -> int {
    carried = false;
    if (carry) std::swap(Q, Qold);
    EF_HIP(c, dense_gemm(c, s, Operand::dense(Y, m, true), Operand::dense(Y, m, false), m, m, dim, 1.0, G, m, work,
                         kWorkElems, Bt),
           "G = Y^T.Y");
    int hinfo = -1;
    const bool fused = chol_inv_supported(m);  // blocked Cholesky + L^-1 (ef_chol_blk.hip)
    if (fused) {
#ifdef EF_CHOL_REG  // A/B build (tools/r05_chol.sh): round 4's register-resident kernel
      if (chol_inv_reg_supported(m))
        EF_HIP(c, launch_chol_inv_reg(s, G, m, m, 1e-13, Li, cinfo), "cholesky + L^-1");
      else
#endif
      EF_HIP(c, launch_chol_inv(s, G, m, m, 1e-13, Li, cinfo, CW), "cholesky + L^-1");
    } else if (m <= kCholeskyMax) {
      EF_HIP(c, launch_cholesky(s, G, m, m, 1e-13, cinfo), "cholesky");
    }
    if (defer) {  // checked at the next Rayleigh-Ritz step (a failed factor leaves Li as it was)
      hipLaunchKernelGGL(sticky_info_kernel, dim3(1), dim3(1), 0, s, cinfo, sticky);
      hinfo = 0;
    } else if (fused || m <= kCholeskyMax) {
      EF_HIP(c, hipMemcpyAsync(&hinfo, cinfo, sizeof(int), hipMemcpyDeviceToHost, s), "D2H info");
      EF_HIP(c, hipStreamSynchronize(s), "sync");
    }
    if (hinfo == 0) {  // Q = Y . L^-T: explicit inverse of the m x m factor (it IS (L^-T)^T), one GEMM
      if (!fused) EF_HIP(c, launch_tri_inv(s, G, m, Li), "L^-1");
      if (tall_gemm_supported(m, Y, 8)) {
        EF_HIP(c, tall_gemm_f64(s, Y, m, false, Li, m, Q, m, dim, m, m, 1.0, work, kWorkElems), "Q = Y.L^-T");
        if (carry)
          EF_HIP(c, tall_gemm_f64(s, Qold, m, false, Li, m, Wc, m, dim, m, m, 1.0, work, kWorkElems), "W = Q'.L^-T");
      } else {  // odd row pitch: generic GEMM on L^-T written out
        EF_HIP(c, launch_transpose_f64(s, Li, m, m, m, Bt, m), "L^-T");
        EF_HIP(c, gemm64(s, Operand::dense(Y, m, false), Operand::dense(Bt, m, false), dim, m, m, 1.0, Q, m, work,
                         kWorkElems),
               "Q = Y.L^-T");
        if (carry)
          EF_HIP(c, gemm64(s, Operand::dense(Qold, m, false), Operand::dense(Bt, m, false), dim, m, m, 1.0, Wc, m,
                           work, kWorkElems),
                 "W = Q'.L^-T");
      }
      carried = carry;
      return EF_OK;
    }
    // rank-deficient block: eigen-orthonormalisation with a floored spectrum
    EF_HIP(c, dense_gemm(c, s, Operand::dense(Y, m, true), Operand::dense(Y, m, false), m, m, dim, 1.0, G, m, work,
                         kWorkElems, Bt),
           "G = Y^T.Y");
    EF_TRY(se.solve(c, G, m, lam, V, m, "jacobi(G)"));
    EF_HIP(c, launch_scale_cols_rsqrt(s, V, m, m, lam, W2), "W.L^-1/2");
    EF_HIP(c, dense_gemm(c, s, Operand::dense(Y, m, false), Operand::dense(W2, m, false), dim, m, m, 1.0, Q, m, work,
                         kWorkElems, Bt),
           "Q = Y.W");
    return EF_OK;
  };
  EF_TRY(orthonormalise(false));

  // Coarse phase in fp32: while the Ritz values still move by > 1e-4 between Rayleigh-Ritz
  // steps, Y = C.Q runs as an fp32 sgemm on an fp32 copy of C (twice the fp64 matrix
  // rate); the iteration is self-correcting, and convergence is only declared between two
  // Rayleigh-Ritz steps that both follow fp64 products, so the result is the fp64 one.
  // Its products run on the split-bf16 matrix cores (ef_gemm_s3.hip: hi.hi' + hi.lo' +
  // lo.hi', ~2^-17 relative per product, 16/3 x the fp32 rate) when the block is 256 wide
  // (option value 1, the default), else — or with option value 2 — as fp32 MFMA GEMMs.
  float *C32 = nullptr, *Q32 = nullptr, *Y32 = nullptr;
  bool coarse = dim >= 4096 && c->opt_fit_fp32_coarse != 0 && tall_gemm_supported(dim, C, 8);
  const bool coarse_s3 = coarse && c->opt_fit_fp32_coarse == 1 && gemm_s3_supported(dim, dim, m);
  if (coarse) {
    EF_TRY(B.get(c, (size_t)dim * dim, &C32));  // fp32 C, or its split-bf16 copy (same bytes)
    EF_TRY(B.get(c, (size_t)dim * m, &Q32));    // Q^T in fp32 / split-bf16 (the GEMM's transposed B)
    EF_TRY(B.get(c, coarse_s3 ? gemm_s3_part_elems(dim) : (size_t)dim * m, &Y32));
    if (coarse_s3)
      EF_HIP(c, launch_split_f64(s, C, dim * dim, C32), "C (split-bf16)");
    else
      cvt64to32(s, C, dim * dim, C32);
  }
  // fp64-accuracy products on the int8 matrix cores (launch_cq_i8, ef_cq_i8.hip: C and Q in
  // base-256 digits, 21 exact digit-pair products); C's digit planes are built once.
  bool cq_i8 = cq_i8_supported(dim, m) && tall_gemm_supported(dim, C, 8);
#ifdef EF_DIAGNOSTICS  // EF_FIT_CQ_I8=0: the fp64 MFMA product (A/B)
  if (const char* e = getenv("EF_FIT_CQ_I8")) cq_i8 = cq_i8 && atoi(e) != 0;
#endif
  uint8_t *cq_planes = nullptr, *cq_work = nullptr;
  bool cq_ready = false;
  // C's digit planes are built on the fit's side stream while the coarse phase runs (its
  // Jacobi rounds and small GEMMs leave most CUs idle); the first fine product waits for
  // them.  The guard orders the main stream after the side work on every exit, so no
  // later work (or a pool reallocation on the next fit) can overtake it.
  struct SideJoin {
    ef_ctx* c;
    bool armed = false;
    ~SideJoin() {
      if (armed) (void)hipStreamWaitEvent(c->stream, c->fit_side_ev[1], 0);
    }
  } side_join{c};
  bool side = true;
#ifdef EF_DIAGNOSTICS  // EF_FIT_SIDE=0: the planes on the main stream at the first fine product (A/B)
  if (const char* e = getenv("EF_FIT_SIDE")) side = atoi(e) != 0;
#endif
  if (cq_i8) {
    EF_TRY(B.get(c, cq_i8_plane_bytes(dim), &cq_planes));
    EF_TRY(B.get(c, cq_i8_work_bytes(dim, m), &cq_work));
  }
  if (cq_i8 && side) {
    if (!c->fit_side) EF_HIP(c, hipStreamCreateWithFlags(&c->fit_side, hipStreamNonBlocking), "fit side stream");
    for (int i = 0; i < 2; ++i)
      if (!c->fit_side_ev[i]) EF_HIP(c, hipEventCreateWithFlags(&c->fit_side_ev[i], hipEventDisableTiming), "fit event");
    EF_HIP(c, hipEventRecord(c->fit_side_ev[0], s), "C ready");
    EF_HIP(c, hipStreamWaitEvent(c->fit_side, c->fit_side_ev[0], 0), "side waits C");
    EF_HIP(c, launch_cq_i8_planes(c->fit_side, C, dim, cq_planes), "C (int8 digit planes)");
    EF_HIP(c, hipEventRecord(c->fit_side_ev[1], c->fit_side), "planes ready");
    side_join.armed = true;
  }
  std::vector<double> th(m), prev(m, 0.0);
  bool have_prev = false, prev_fine = false;
  // Spectral shift: the iteration multiplies by C - sigma I.  Convergence of eigenpair i
  // goes as max_{j > m} |lambda_j - sigma| / (lambda_i - sigma) per product instead of
  // lambda_{m+1} / lambda_i.  sigma = theta_m / 2 (theta_m, the block's smallest Ritz
  // value, never exceeds lambda_m) is safe for any PSD C: every unwanted |lambda_j - sigma|
  // is at most max(lambda_{m+1} - sigma, sigma) < lambda_k - sigma, so the wanted block
  // stays dominant.  Ritz values are reported and tested unshifted.
  // Chebyshev acceleration (EF_OPT_FIT_CHEBYSHEV, default on): with [0, theta_m] as the
  // interval of the unwanted spectrum (centre = half-width = sigma), the iterates follow
  // the three-term recurrence X_{j+1} = 2 A~ X_j - X_{j-1}, A~ = (C - sigma I) / sigma,
  // restarted (X_0 = the current block) at every Rayleigh-Ritz step, which refreshes
  // sigma.  Eigenpair i then converges per product as 1 / (x + sqrt(x^2 - 1)),
  // x = lambda_i / sigma - 1, instead of (lambda_{m+1} - sigma) / (lambda_i - sigma): the
  // C3 fit's 40 products drop to ~27 in a model of its spectrum.  Each iterate is
  // orthonormalised (Y = Q' L^T); the previous one is carried into the same frame
  // (W = Q_old L^-T, one extra tall GEMM), so the recurrence holds exactly for the block's
  // span while the columns stay orthonormal (no growth of the dominant components).
  double sigma = 0.0;
  bool shift_on = true;
#ifdef EF_DIAGNOSTICS
  if (const char* e = getenv("EF_FIT_SHIFT")) shift_on = atoi(e) != 0;
#endif
  const bool cheb_on = c->opt_fit_chebyshev != 0;
  int cheb_j = 0;  // recurrence steps since the last restart (Wc valid when > 0)
  const unsigned ew_blocks = (unsigned)std::min<int64_t>((dim * m + 255) / 256, 8192);
  // Ritz-residual acceptance (see the Rayleigh-Ritz step): a step after an fp64 product is
  // also converged when every kept pair's |C u - theta u| <= resid_tol * theta_1
  double resid_tol = fit_resid_tol();
  const double gap_tol = fit_gap_tol();
  std::vector<double> rnorm(kk);
  double prev_resid_max = 0.0;  // largest |r_i| / theta_1 at the previous fp64 step (0: none)
  bool fit_debug = false;
#ifdef EF_DIAGNOSTICS
  fit_debug = getenv("EF_FIT_DEBUG") != nullptr;
#endif
  int it = 0;
  const int max_iters = (int)std::max<int64_t>(1, std::min<int64_t>(c->opt_fit_max_iters, 1 << 20));
  bool converged = false;
  double last_worst = 1.0;
  int next_rr = 8;  // iteration of the next scheduled Rayleigh-Ritz step
  double rate_prev = 0.0;  // predicted per-product error factor of the products since the last step
  int last_rr_it = 0;
  for (it = 1; it <= max_iters; ++it) {
    const bool fine = !coarse;  // this iteration's product is fp64
    const double sig_it = sigma;  // the shift this iteration's product carries
    bool restarted = false;
    if (coarse && coarse_s3) {
      EF_HIP(c, launch_transpose_split(s, Q, dim, Q32), "Q^T (split-bf16)");
      EF_HIP(c, gemm_s3(s, C32, dim, Q32, dim, dim, dim, Y32, Q, sigma, Y), "Y = C.Q (split-bf16)");
    } else if (coarse) {
      EF_HIP(c, launch_transpose_f64_to_f32(s, Q, m, dim, m, Q32, dim), "Q^T (fp32)");
      EF_HIP(c, tall_gemm_f32(s, C32, dim, false, Q32, dim, Y32, m, dim, m, dim, 1.f, reinterpret_cast<float*>(work),
                              kWorkElems * 2),
             "Y = C.Q (fp32)");
      hipLaunchKernelGGL(f32_to_f64_shift_kernel, dim3(ew_blocks), dim3(256), 0, s, Y32, Q, dim * m, sigma, Y);
    } else if (cq_i8) {
      if (!cq_ready) {
        if (side) EF_HIP(c, hipStreamWaitEvent(s, c->fit_side_ev[1], 0), "planes ready");
        else EF_HIP(c, launch_cq_i8_planes(s, C, dim, cq_planes), "C (int8 digit planes)");
      }
      cq_ready = true;
      // the medium form (15 digit pairs, ~2^-40) unless a Rayleigh-Ritz step reads this
      // product or the next: the errors of earlier products are damped by the later ones
      // (residual floor 1e-12 theta_1), the accepted step's Ritz pairs come from full ones
      // (iterations <= 4 may hold the small orders' early Rayleigh-Ritz steps)
      bool medium = it >= 5 && it + 1 < next_rr && it + 1 < max_iters;
#ifdef EF_DIAGNOSTICS  // EF_FIT_CQ_MED=0: every fine product in the full form (A/B)
      static const bool med_on = [] { const char* e = getenv("EF_FIT_CQ_MED"); return !(e && atoi(e) == 0); }();
      medium = medium && med_on;
#endif
      EF_HIP(c, launch_cq_i8(s, cq_planes, dim, Q, m, sigma, cq_work, Y, medium), "Y = C.Q (int8 digits)");
    } else {
      EF_HIP(c, dense_gemm(c, s, Operand::symmetric(C, dim), Operand::dense(Q, m, false), dim, m, dim, 1.0, Y, m, work,
                           kWorkElems, Bt),
             "Y = C.Q");
      if (sigma != 0.0) hipLaunchKernelGGL(shift_kernel, dim3(ew_blocks), dim3(256), 0, s, Y, Q, dim * m, sigma);
    }
    // Rayleigh-Ritz at iterations 1, 2, 4 (small orders only: there they re-order the block
    // early enough to matter; at order >= 12288 they cost 26 of 62 Jacobi sweeps and change
    // no iteration count), 8, then every rr_period(dim)
#ifdef EF_DIAGNOSTICS
    static const int early_rule = [] { const char* e = getenv("EF_FIT_EARLY"); return e ? atoi(e) : 0; }();
    const bool early = early_rule == 0 ? dim < 12288 && (it <= 2 || it == 4)
                     : early_rule == 1 ? (it <= 2 || it == 4) : it == early_rule;
#else
    const bool early = dim < 12288 && (it <= 2 || it == 4);
#endif
    const bool rr = early || it == next_rr || it == max_iters;
    if (rr && defer) {  // the deferred Cholesky checks, before anything reads this block
      int hs = 0;
      EF_HIP(c, hipMemcpyAsync(&hs, sticky, sizeof(int), hipMemcpyDeviceToHost, s), "D2H sticky");
      EF_HIP(c, hipStreamSynchronize(s), "sync");
      if (hs != 0) return kRetryChecked;
    }
    if (rr) {
      EF_HIP(c, dense_gemm(c, s, Operand::dense(Q, m, true), Operand::dense(Y, m, false), m, m, dim, 1.0, G, m,
                           work, kWorkElems, Bt),
             "H = Q^T.C.Q");
      // A Rayleigh-Ritz step after reduced-precision products can never be the converged
      // one (that needs two steps after fp64 products), and its Ritz values only steer the
      // shift, the rate and the switch to fp64 (1e-4 / 1e-6 decisions): its Jacobi stops at
      // off-diagonals of 1e-4 of the diagonal scale (Ritz value error ~1e-8 / relative
      // gap) instead of 1e-12 — the last sweeps of those solves (C3: 1e-4 0.1461 s, 1e-6
      // 0.1467 s, 1e-3 one more iteration; profiles/r04/rr_loose_ab.txt).  The Ritz basis V stays
      // orthogonal to rounding either way (rotations), so the block's span is unchanged.
      EF_TRY(se.solve(c, G, m, lam, V, m, "jacobi(H)", fine ? 1e-12 : have_prev ? rr_loose_tol() : rr_first_tol()));
      // Ritz residuals |C u_i - theta_i u_i| of the kept pairs after an fp64 product: YV = Y.V
      // is the continuation product anyway, U = Q.V the result's
      const bool resid = fine && (resid_tol > 0.0 || gap_tol > 0.0 || fit_debug);
      if (resid) {
        EF_HIP(c, dense_gemm(c, s, Operand::dense(Y, m, false), Operand::dense(V, m, false), dim, m, m, 1.0, Y2, m,
                             work, kWorkElems, Bt),
               "Y.V");
        EF_HIP(c, dense_gemm(c, s, Operand::dense(Q, m, false), Operand::dense(V, m, false), dim, kk, m, 1.0, U_out,
                             kk, work, kWorkElems, Bt),
               "U = Q.V");
        hipLaunchKernelGGL(ritz_resid_kernel, dim3((unsigned)((kk + 63) / 64), kResidChunks), dim3(256), 0, s, Y2,
                           (int64_t)m, U_out, (int64_t)kk, lam, dim, kk, RP);
        EF_HIP(c, hipMemcpyAsync(rp.data(), RP, rp.size() * sizeof(double), hipMemcpyDeviceToHost, s), "D2H resid");
      }
      EF_HIP(c, hipMemcpyAsync(th.data(), lam, m * sizeof(double), hipMemcpyDeviceToHost, s), "D2H lam");
      EF_HIP(c, hipStreamSynchronize(s), "sync");
      double resid_max = 1.0;
      if (resid) {
        resid_max = 0.0;
        for (int i = 0; i < kk; ++i) {
          double a = 0.0;
          for (int q = 0; q < kResidChunks; ++q) a += rp[(size_t)q * kk + i];
          rnorm[i] = std::sqrt(a);
          resid_max = std::fmax(resid_max, rnorm[i]);
        }
      }
      if (!std::isfinite(th[0])) return set_err(c, EF_E_NUMERIC, "subspace iteration diverged");
      for (int i = 0; i < m; ++i) th[i] += sigma;  // Ritz values of C (H = Q^T (C - sigma I) Q)
      // converged when every kept Ritz value moved by <= 1e-13 relative (floor 1e-15 of
      // the largest) since the previous Rayleigh-Ritz step
      bool ok_vals = have_prev && prev_fine && fine;
      for (int i = 0; i < kk && ok_vals; ++i)
        ok_vals = std::fabs(th[i] - prev[i]) <= std::fmax(1e-13 * std::fabs(th[i]), 1e-15 * std::fabs(th[0]));
      const double th1 = std::fabs(th[0]);
      resid_max /= th1;
      bool ok = ok_vals || (resid && resid_tol > 0.0 && resid_max <= resid_tol);
      // gap-aware part (see fit_gap_tol): every kept pair's |r_i| <= 1e-5 gap_i
      bool ok_gap = true;
      double gap_worst = 0.0;  // max |r_i| / gap_i (diagnostics)
      double gap_need = 0.0;   // max |r_i| / its gap-rule bound (> 1: not yet)
      int gap_wi = -1;
      if (resid && gap_tol > 0.0) {
        for (int i = 0; i < kk; ++i) {
          double g = HUGE_VAL;
          for (int j = 0; j < m; ++j)
            if (j != i) g = std::fmin(g, std::fabs(th[i] - th[j]));
          const double q = rnorm[i] / std::fmax(g, 1e-300);
          if (q > gap_worst) gap_worst = q, gap_wi = i;
          const double need = rnorm[i] / std::fmax(gap_tol * g, kResidFloor * th1);
          gap_need = std::fmax(gap_need, need);
          if (need > 1.0) ok_gap = false;
        }
        // floor of the arithmetic: values converged and the residuals no longer shrinking
        const bool stalled = ok_vals && prev_resid_max > 0.0 && resid_max > 0.5 * prev_resid_max;
        ok = ok && (ok_gap || stalled);
      }
      if (resid) prev_resid_max = resid_max;
      double worst = have_prev ? 0.0 : 1.0;
      int wi = 0;
      for (int i = 0; i < kk && have_prev; ++i) {
        const double r = std::fabs(th[i] - prev[i]) / std::fmax(std::fabs(th[i]), 1e-300);
        if (r > worst) worst = r, wi = i;
      }
#ifdef EF_DIAGNOSTICS
      if (getenv("EF_FIT_DEBUG"))
        fprintf(stderr,
                "[ef_fit] rr it=%d %s sweeps_total=%ld worst_rel=%.3e at %d theta_k=%.6g theta_m=%.6g resid=%.3e "
                "r/gap=%.3e at %d ok=%d\n",
                it, fine ? "fp64" : "fp32", se.sweeps, worst, wi, th[kk - 1], th[m - 1], resid ? resid_max : -1.0,
                gap_worst, gap_wi, (int)ok);
#else
      (void)wi;
      (void)gap_wi;
#endif
      double coarse_tol = 1e-4, coarse_pred = 1e-6;
#ifdef EF_DIAGNOSTICS
      if (const char* e = getenv("EF_FIT_COARSE_TOL")) coarse_tol = atof(e);
      if (const char* e = getenv("EF_FIT_COARSE_PRED")) coarse_pred = atof(e);
#endif
      // Chebyshev rate: the k-th Ritz value's error shrinks per product by 1 / rho^2,
      // rho = x + sqrt(x^2 - 1), x = theta_k / sigma - 1 on the next interval [0, theta_m]
      const double sig_next = shift_on && th[m - 1] > 0.0 ? 0.5 * th[m - 1] : 0.0;
      double rate_next = 0.0;
      if (cheb_on && sig_next > 0.0) {
        const double x = th[kk - 1] / sig_next - 1.0;
        if (x > 1.0 + 1e-9) {
          const double rho = x + std::sqrt(x * x - 1.0);
          rate_next = 1.0 / (rho * rho);
        }
      }
      // error of this step's Ritz values: the change since the previous step bounds the
      // previous step's error, which the products since then shrank by rate_prev each
      const double e_now = have_prev && rate_prev > 0.0 ? worst * std::pow(rate_prev, it - last_rr_it) : worst;
      // fp64 products from the next iteration on once the fp32 phase has done its part
      if (coarse && (worst < coarse_tol || (rate_prev > 0.0 && e_now < coarse_pred))) coarse = false;
      // Schedule the next Rayleigh-Ritz step.  The test above passes once the PREVIOUS
      // step's Ritz values were already within 1e-13, so with the change per period
      // shrinking geometrically (worst now vs worst at the previous step) the current error
      // is predicted as worst * rate: when that is below the tolerance the next step comes
      // one iteration later (the test then passes instead of waiting out the period); a
      // wrong prediction only costs that one extra Rayleigh-Ritz step.  With the Chebyshev
      // rate known, the next step is placed where the predicted error reaches the
      // tolerance (from the fp32 floor ~3e-7 when the products so far were fp32).
      {
        const int period = rr_period(dim);
        next_rr = (it / period + 1) * period;
        if (it < 8) next_rr = 8;
        if (fine && prev_fine && have_prev && last_worst > 0.0 && worst < last_worst) {
          const double e_pred = worst * (worst / last_worst);
          if (e_pred <= 3e-14) next_rr = it + 1;
        }
        if (rate_next > 0.0 && have_prev && !coarse) {
          const double e_start = fine ? e_now : std::max(e_now, 3e-7);
          int p = (int)std::ceil(std::log(e_start / 3e-14) / std::log(1.0 / rate_next));
          if (p < 1) p = 1;
          next_rr = std::min(next_rr, it + p);
        }
        // Gap rule not met yet: no step can accept before it is, so the next one goes where
        // it should be met (an earlier step would also restart the recurrence and lose the
        // acceleration).  p Chebyshev products shrink the slowest kept vector's residual by
        // T_p(x) = cosh(p acosh x), x = theta_k / sigma - 1; a factor 2 of margin.  (C3: the
        // steps at 23 and 24 that the value rule placed are skipped, 22 -> 25.  The
        // asymptotic rate rho^p >= 1.5 need — diagnostic EF_FIT_GAP_MARGIN=1.5 — placed the
        // step at 24, where the residual had shrunk only 5.2x, not rho^2 = 11x, right after
        // the restart: 1.345e-5 of the gap, one more step, 0.1390 vs 0.1378 s;
        // profiles/r06/fit_gap_sched_ab.txt.)
        if (gap_need > 1.0 && rate_next > 0.0 && !coarse) {
          const double x = th[kk - 1] / sig_next - 1.0;
          double margin = 0.0;
#ifdef EF_DIAGNOSTICS  // EF_FIT_GAP_MARGIN (A/B; > 0: p = log(margin need) / log(rho))
          if (const char* e = getenv("EF_FIT_GAP_MARGIN")) margin = atof(e);
#endif
          int p = margin > 0.0 ? (int)std::ceil(std::log(margin * gap_need) / std::log(x + std::sqrt(x * x - 1.0)))
                               : (int)std::ceil(std::acosh(2.0 * gap_need) / std::acosh(x));
          next_rr = std::max(next_rr, it + std::max(p, 1));
        }
      }
      rate_prev = rate_next;
      last_rr_it = it;
      // the next products use the shift of this step's block (the continuation Y.V below
      // still carries the old one: any sequence of shifts is a valid polynomial filter)
      sigma = sig_next;
      prev = th;
      have_prev = true;
      prev_fine = fine;
      last_worst = worst;
      converged = ok;
      // the iteration cap ends the loop with EF_E_NUMERIC (useless/train.py has no cap:
      // LAPACK either converges or raises LinAlgError; train-v4.py:114-120 returns False)
      if (ok || it == max_iters) {
        if (!resid)  // (the residual check formed it already)
          EF_HIP(c, dense_gemm(c, s, Operand::dense(Q, m, false), Operand::dense(V, m, false), dim, kk, m, 1.0, U_out,
                               kk, work, kWorkElems, Bt),
                 "U = Q.V");
        EF_HIP(c, hipMemcpyAsync(lam_out, th.data(), kk * sizeof(double), hipMemcpyHostToDevice, s), "lam");
        EF_HIP(c, hipStreamSynchronize(s), "sync");
        break;
      }
      // continue from the Ritz basis: C.(Q.V) = Y.V (and restart the recurrence there)
      if (!resid)
        EF_HIP(c, dense_gemm(c, s, Operand::dense(Y, m, false), Operand::dense(V, m, false), dim, m, m, 1.0, Y2, m,
                             work, kWorkElems, Bt),
               "Y.V");
      std::swap(Y, Y2);
      restarted = true;
    }
    if (cheb_on && sig_it > 0.0 && !restarted) {
      // X_1 = A~ X_0, X_{j+1} = 2 A~ X_j - X_{j-1}; Y holds (C - sigma I) Q, Wc the carried X_{j-1}
      hipLaunchKernelGGL(cheb_combine_kernel, dim3(ew_blocks), dim3(256), 0, s, Y, cheb_j > 0 ? Wc : nullptr,
                         dim * m, (cheb_j > 0 ? 2.0 : 1.0) / sig_it);
      EF_TRY(orthonormalise(true));
      cheb_j = carried ? cheb_j + 1 : 0;
    } else {
      EF_TRY(orthonormalise(false));
      cheb_j = 0;
    }
  }
  if (it > max_iters) it = max_iters;
#ifdef EF_DIAGNOSTICS
  if (getenv("EF_FIT_DEBUG"))
    fprintf(stderr, "[ef_fit] wide dim=%lld k=%d m=%d iters=%d jacobi calls=%ld sweeps=%ld\n", (long long)dim, kk, m,
            it, se.calls, se.sweeps);
#endif
  *iters = it;
  if (!converged) {
    char msg[160];
    snprintf(msg, sizeof msg,
             "eigensolver did not converge: %d subspace iterations, Ritz values still moving by %.3e (relative)",
             it, last_worst);
    return set_err(c, EF_E_NUMERIC, msg);
  }
  return EF_OK;
}

// Top-kk eigenpairs of the symmetric dim x dim matrix C (device, ld = dim).
// U_out: dim x kk (row-major, ld kk), lam_out: kk (device).  iters: host.
int eig_topk(ef_ctx* c, Bufs& B, const double* C, int64_t dim, int kk, double* work, double* U_out,
             double* lam_out, int* iters) {
  hipStream_t s = c->stream;
  if (dim <= kJacobiMax || (kk > kJacobiMax - 8 && dim <= kDirectMax)) {  // direct
    SmallEig se;
    EF_TRY(se.init(c, B, (int)dim));
    double *ev, *V;
    EF_TRY(B.get(c, (size_t)dim, &ev));
    EF_TRY(B.get(c, (size_t)dim * dim, &V));
    EF_TRY(se.solve(c, C, dim, ev, V, dim, "eigensolve"));
    EF_HIP(c, hipMemcpy2DAsync(U_out, kk * sizeof(double), V, dim * sizeof(double), kk * sizeof(double), dim,
                               hipMemcpyDeviceToDevice, s),
           "copy U");
    EF_HIP(c, hipMemcpyAsync(lam_out, ev, kk * sizeof(double), hipMemcpyDeviceToDevice, s), "copy lam");
    EF_HIP(c, hipStreamSynchronize(s), "sync");
    *iters = 0;
    return EF_OK;
  }

  // Block width m = max(2k, 88) (Ritz values converge as (lambda_{m+1} / lambda_k)^2 per
  // iteration), even, <= dim: CholQR subspace iteration with periodic Rayleigh-Ritz.
  int64_t mm = std::max<int64_t>(2 * (int64_t)kk, kJacobiMax);
  mm = (mm + 7) / 8 * 8;
  if (mm > dim) mm = dim & ~int64_t(1);
  int m = (int)mm;
#ifdef EF_DIAGNOSTICS
  if (const char* em = getenv("EF_FIT_M")) {  // experiments only
    const int64_t e = atoi(em);
    if (e >= kk + 2 && e <= dim) m = (int)(e & ~int64_t(1));
  }
#endif
  const size_t mark = B.next;  // a checked rerun reuses the same pool slots
  bool defer = true;
#ifdef EF_DIAGNOSTICS  // EF_FIT_DEFER=0: the host check of every CholQR factor (A/B)
  if (const char* e = getenv("EF_FIT_DEFER")) defer = atoi(e) != 0;
#endif
  int rc = subspace_wide(c, B, C, dim, kk, m, work, U_out, lam_out, iters, defer);
  if (rc == kRetryChecked) {
    B.next = mark;
    rc = subspace_wide(c, B, C, dim, kk, m, work, U_out, lam_out, iters, false);
  }
  return rc;
}

// Numerically null components.  With k = n (train-v5.py:540-545 sets n_components to the
// face count) the centred data has rank n - 1 and the last eigenvalue is rounding noise:
// the Gram path's back-projection A^T.u of its eigenvector is itself rounding noise, and
// normalising it would give an arbitrary direction with large projections.  In exact
// arithmetic any unit vector orthogonal to the data span is a valid component (sklearn's
// full SVD returns LAPACK's choice); this takes a fixed one: a seeded vector, made
// orthogonal (two Gram-Schmidt passes) to every other component, unit length, svd_flip
// sign rule.  Rare and small (k x d), so on the host.
int complete_null_components(ef_ctx* c, int64_t n, int64_t d, int kk, const double* lam_dev, double* comps_dev,
                             double* En_dev) {
  hipStream_t s = c->stream;
  std::vector<double> lam(kk);
  EF_HIP(c, hipMemcpyAsync(lam.data(), lam_dev, kk * sizeof(double), hipMemcpyDeviceToHost, s), "D2H lam");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  const double tol = 1e-14 * (double)std::max(n, d) * std::fabs(lam[0]);
  std::vector<int> null_cols;
  for (int j = 0; j < kk; ++j)
    if (!(lam[j] > tol)) null_cols.push_back(j);
  if (null_cols.empty() || (int)null_cols.size() == kk) return EF_OK;
  std::vector<double> C((size_t)kk * d);
  EF_HIP(c, hipMemcpyAsync(C.data(), comps_dev, C.size() * sizeof(double), hipMemcpyDeviceToHost, s), "D2H comps");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  std::vector<char> done(kk, 0);
  for (int j = 0; j < kk; ++j) done[j] = lam[j] > tol;
  unsigned long long st = 0x9e3779b97f4a7c15ULL;
  for (int j : null_cols) {
    double* v = &C[(size_t)j * d];
    for (int64_t i = 0; i < d; ++i) {  // splitmix64 -> uniform(-1, 1)
      st += 0x9e3779b97f4a7c15ULL;
      unsigned long long z = st;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
      z ^= z >> 31;
      v[i] = (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
    }
    for (int pass = 0; pass < 2; ++pass)
      for (int q = 0; q < kk; ++q) {
        if (!done[q]) continue;
        const double* u = &C[(size_t)q * d];
        double dot = 0.0;
        for (int64_t i = 0; i < d; ++i) dot += u[i] * v[i];
        for (int64_t i = 0; i < d; ++i) v[i] -= dot * u[i];
      }
    double nrm = 0.0, mx = -1.0;
    int64_t mi = 0;
    for (int64_t i = 0; i < d; ++i) {
      nrm += v[i] * v[i];
      if (std::fabs(v[i]) > mx) mx = std::fabs(v[i]), mi = i;
    }
    const double f = (v[mi] < 0 ? -1.0 : 1.0) / std::sqrt(nrm);
    for (int64_t i = 0; i < d; ++i) v[i] *= f;
    done[j] = 1;
  }
  std::vector<double> T((size_t)d * kk);
  for (int j = 0; j < kk; ++j)
    for (int64_t i = 0; i < d; ++i) T[(size_t)i * kk + j] = C[(size_t)j * d + i];
  EF_HIP(c, hipMemcpyAsync(comps_dev, C.data(), C.size() * sizeof(double), hipMemcpyHostToDevice, s), "H2D comps");
  EF_HIP(c, hipMemcpyAsync(En_dev, T.data(), T.size() * sizeof(double), hipMemcpyHostToDevice, s), "H2D En");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  return EF_OK;
}

}  // namespace

extern "C" int ef_fit_ex(ef_ctx* c, const void* Xv, int32_t x_dtype, int64_t n, int64_t d, int32_t k,
                         uint32_t flags, double* mean_out, double* var_out, double* scale_out, double* comps_out,
                         double* eig_out, double* proj_out, double* tv_out, int32_t* k_out, int32_t* iters_out) {
  if (!c) return EF_E_INVALID;
  if (!Xv || n < 2 || d < 1 || k < 1 || !mean_out || !comps_out || !eig_out)
    return set_err(c, EF_E_INVALID, "ef_fit: bad arguments (need X, n >= 2, d >= 1, k >= 1, outputs)");
  if (x_dtype != EF_U8 && x_dtype != EF_F32 && x_dtype != EF_F64)
    return set_err(c, EF_E_INVALID, "ef_fit: x_dtype must be EF_U8, EF_F32 or EF_F64");
  const bool u8 = x_dtype == EF_U8;
  const size_t esize = u8 ? 1 : (x_dtype == EF_F32 ? 4 : 8);
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  const bool dev = flags & EF_MEM_DEVICE;
  const bool stdz = flags & EF_FIT_STANDARDIZE;
  const bool gram = n < d;
  const int64_t dim = gram ? n : d;
  const int kk = (int)(k < dim ? k : dim);

  Bufs B;
  const void* Xdv = Xv;
  if (!dev) {
    uint8_t* xb;
    EF_TRY(B.get(c, (size_t)n * d * esize, &xb));
    EF_HIP(c, hipMemcpyAsync(xb, Xv, (size_t)n * d * esize, hipMemcpyHostToDevice, s), "H2D X");
    Xdv = xb;
  }
  // uint8 pixels take the exact integer kernels; float input the fp64 loaders
  const uint8_t* Xd = u8 ? static_cast<const uint8_t*>(Xdv) : nullptr;
  auto pix = [&](bool trans, const double* mu, const double* wv) {
    return Operand::pixels(Xdv, x_dtype, d, trans, mu, wv);
  };
  unsigned long long *S1, *S2;
  double *mean, *var, *scale, *w, *C, *work, *U, *lam, *E = nullptr, *comps, *En, *proj = nullptr, *tv;
  EF_TRY(B.get(c, (size_t)d, &S1));
  EF_TRY(B.get(c, (size_t)d, &S2));
  EF_TRY(B.get(c, (size_t)d, &mean));
  EF_TRY(B.get(c, (size_t)d, &var));
  EF_TRY(B.get(c, (size_t)d, &scale));
  EF_TRY(B.get(c, (size_t)d, &w));
  EF_TRY(B.get(c, (size_t)dim * dim, &C));
  EF_TRY(B.get(c, kWorkElems, &work));
  EF_TRY(B.get(c, (size_t)dim * kk, &U));
  EF_TRY(B.get(c, (size_t)kk, &lam));
  EF_TRY(B.get(c, (size_t)kk * d, &comps));
  EF_TRY(B.get(c, (size_t)d * kk, &En));
  EF_TRY(B.get(c, 1, &tv));

  // K1: exact column statistics -> mean / var / scale / centring weights.  On the int8
  // covariance path the operand transpose produces the sums in the same pass over X.
  const double inv = 1.0 / (double)(n - 1);
  const bool int8_path = u8 && (!gram || !stdz);
  uint8_t* At = nullptr;
  if (u8) {
    EF_HIP(c, hipMemsetAsync(S1, 0, d * sizeof(unsigned long long), s), "memset");
    EF_HIP(c, hipMemsetAsync(S2, 0, d * sizeof(unsigned long long), s), "memset");
    const bool fused = int8_path && !gram && cov_i8_fused_stats(Xd, d);
    if (int8_path) {
      EF_TRY(B.get(c, (size_t)dim * cov_i8_kpad(gram ? d : n) + kSyrkPadBytes, &At));
      EF_HIP(c, launch_cov_i8_prep(s, Xd, n, d, gram, At, fused ? S1 : nullptr, fused ? S2 : nullptr), "cov prep");
    }
    if (!fused) EF_HIP(c, launch_colstats(s, Xd, n, d, S1, S2), "colstats");
    EF_HIP(c, launch_stats_finalize(s, S1, S2, n, d, stdz ? 1 : 0, mean, var, scale, w), "stats");
  } else {
    double* part;
    EF_TRY(B.get(c, colstats_float_work_elems(n, d), &part));
    EF_HIP(c, launch_colstats_float(s, Xdv, x_dtype, n, d, stdz ? 1 : 0, part, mean, var, scale, w), "colstats (float)");
  }
  const double* wp = stdz ? w : nullptr;

  // K2+K3: covariance.  Exact integer product on the int8 matrix cores whenever the
  // pixel scaling commutes with it (covariance path; Gram path without StandardScaler),
  // else the fp64 GEMM with the centring/scaling fused into the operand loads.
  if (int8_path) {
    const CovPlan plan = cov_i8_plan(dim, gram ? d : n, c->opt_cov_slab_bytes);
    int* slabs;
    long long *S64 = nullptr, *cvec, *R;
    unsigned long long* Q2;
    EF_TRY(B.get(c, (size_t)plan.slab_elems, &slabs));
    if (plan.passes > 1) EF_TRY(B.get(c, (size_t)dim * dim, &S64));
    EF_TRY(B.get(c, (size_t)d, &cvec));
    EF_TRY(B.get(c, (size_t)(gram ? n : 1), &R));
    EF_TRY(B.get(c, 2, &Q2));
    uint8_t* order;
    EF_TRY(B.get(c, (size_t)cov_i8_order_bytes(dim), &order));
    TimerEvt tev;
    timer_arm(c, EF_KERNEL_SYRK, &tev);
    const hipError_t ecov = launch_cov_i8(s, plan, n, d, gram, S1, stdz ? w : nullptr, At, slabs, S64, cvec, R, Q2,
                                          order, C, tev.kernel >= 0 ? tev.a : nullptr,
                                          tev.kernel >= 0 ? tev.b : nullptr);
    timer_commit(c, &tev);  // (the drain skips a pair whose end was never recorded)
    EF_HIP(c, ecov, "covariance (int8)");
    B.drop(s, At);
    B.drop(s, slabs);
    if (S64) B.drop(s, S64);
  } else if (gram)
    EF_HIP(c, gemm64(s, pix(false, mean, wp), pix(true, mean, wp), n, n, d,
                     inv, C, n, work, kWorkElems),
           "Gram");
  else
    EF_HIP(c, gemm64(s, pix(true, mean, wp), pix(false, mean, wp), d, d, n,
                     inv, C, d, work, kWorkElems),
           "covariance");
  EF_HIP(c, launch_trace(s, C, dim, dim, tv), "trace");

  // K4: top-kk eigenpairs
  int iters = 0;
  EF_TRY(eig_topk(c, B, C, dim, kk, work, U, lam, &iters));

  // K5: back-project (Gram path), unit columns + sign rule
  if (gram) {
    EF_TRY(B.get(c, (size_t)d * kk, &E));
    EF_HIP(c, gemm64(s, pix(true, mean, wp), Operand::dense(U, kk, false), d, kk, n, 1.0, E, kk,
                     work, kWorkElems),
           "E = A^T.U");
    EF_HIP(c, launch_normalize_sign(s, E, d, kk, kk, comps, En), "normalize");
  } else {
    EF_HIP(c, launch_normalize_sign(s, U, d, kk, kk, comps, En), "normalize");
  }
  EF_TRY(complete_null_components(c, n, d, kk, lam, comps, En));
  // training projection A.E (projected_data / fit_transform output)
  if (proj_out) {
    EF_TRY(B.get(c, (size_t)n * kk, &proj));
#ifdef EF_DIAGNOSTICS
    const bool f64proj = getenv("EF_FIT_PROJ_F64") != nullptr;
#else
    constexpr bool f64proj = false;
#endif
    if (u8 && proj_i8_supported(Xd, n, d, kk) && !f64proj) {  // exact int8 digits (ef_proj_i8.hip)
      uint8_t* pw;
      EF_TRY(B.get(c, proj_i8_work_bytes(n, d, kk), &pw));
      EF_HIP(c, launch_proj_i8(s, Xd, n, d, mean, wp, En, kk, pw, proj), "F = A.E (int8 digits)");
    } else {
      EF_HIP(c, gemm64(s, pix(false, mean, wp), Operand::dense(En, kk, false), n, kk, d, 1.0,
                       proj, kk, work, kWorkElems),
             "F = A.E");
    }
  }

  const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  EF_HIP(c, hipMemcpyAsync(mean_out, mean, d * sizeof(double), kind, s), "out mean");
  if (var_out) EF_HIP(c, hipMemcpyAsync(var_out, var, d * sizeof(double), kind, s), "out var");
  if (scale_out) EF_HIP(c, hipMemcpyAsync(scale_out, scale, d * sizeof(double), kind, s), "out scale");
  EF_HIP(c, hipMemcpyAsync(comps_out, comps, (size_t)kk * d * sizeof(double), kind, s), "out comps");
  EF_HIP(c, hipMemcpyAsync(eig_out, lam, kk * sizeof(double), kind, s), "out eig");
  if (proj_out) EF_HIP(c, hipMemcpyAsync(proj_out, proj, (size_t)n * kk * sizeof(double), kind, s), "out proj");
  if (tv_out) EF_HIP(c, hipMemcpyAsync(tv_out, tv, sizeof(double), kind, s), "out tv");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  if (k_out) *k_out = kk;
  if (iters_out) *iters_out = iters;
  return EF_OK;
}

extern "C" int ef_fit(ef_ctx* c, const uint8_t* X, int64_t n, int64_t d, int32_t k, uint32_t flags,
                      double* mean_out, double* var_out, double* scale_out, double* comps_out,
                      double* eig_out, double* proj_out, double* tv_out, int32_t* k_out, int32_t* iters_out) {
  return ef_fit_ex(c, X, EF_U8, n, d, k, flags, mean_out, var_out, scale_out, comps_out, eig_out, proj_out, tv_out,
                   k_out, iters_out);
}

// ---------------------------------------------------------------- sample-sharded fit
// SURVEY.md §8(e), the fit collective: rank r holds rows X_r; the exact integer pieces
// (column sums of x and x^2, X'_r^T X'_r) of every rank add up to the pieces of the whole
// set, so after a sum over ranks the covariance, and everything computed from it, equals
// ef_fit's on the concatenated rows bit for bit (covariance path: n_total >= d).
extern "C" int ef_fit_shard_stats(ef_ctx* c, const uint8_t* X, int64_t n, int64_t d, uint64_t* sum_out,
                                  uint64_t* sumsq_out, int64_t* cross_out, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if ((!X && n > 0) || n < 0 || d < 1 || !sum_out || !sumsq_out || !cross_out)
    return set_err(c, EF_E_INVALID, "ef_fit_shard_stats: bad arguments (need X, n >= 0, d >= 1, outputs)");
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  const bool dev = flags & EF_MEM_DEVICE;
  Bufs B;
  unsigned long long *S1, *S2;
  long long* S64;
  EF_TRY(B.get(c, (size_t)d, &S1));
  EF_TRY(B.get(c, (size_t)d, &S2));
  if (dev) {
    S64 = reinterpret_cast<long long*>(cross_out);
  } else {
    EF_TRY(B.get(c, (size_t)d * d, &S64));
  }
  EF_HIP(c, hipMemsetAsync(S1, 0, d * sizeof(unsigned long long), s), "memset");
  EF_HIP(c, hipMemsetAsync(S2, 0, d * sizeof(unsigned long long), s), "memset");
  if (n == 0) {  // an empty shard contributes nothing
    EF_HIP(c, hipMemsetAsync(S64, 0, (size_t)d * d * sizeof(long long), s), "memset");
  } else {
    const uint8_t* Xd = X;
    if (!dev) {
      uint8_t* xb;
      EF_TRY(B.get(c, (size_t)n * d, &xb));
      EF_HIP(c, hipMemcpyAsync(xb, X, (size_t)n * d, hipMemcpyHostToDevice, s), "H2D X");
      Xd = xb;
    }
    uint8_t* At;
    EF_TRY(B.get(c, (size_t)d * cov_i8_kpad(n) + kSyrkPadBytes, &At));
    const bool fused = cov_i8_fused_stats(Xd, d);
    EF_HIP(c, launch_cov_i8_prep(s, Xd, n, d, false, At, fused ? S1 : nullptr, fused ? S2 : nullptr), "cov prep");
    if (!fused) EF_HIP(c, launch_colstats(s, Xd, n, d, S1, S2), "colstats");
    const CovPlan plan = cov_i8_plan(d, n, c->opt_cov_slab_bytes);
    int* slabs;
    uint8_t* order;
    EF_TRY(B.get(c, (size_t)plan.slab_elems, &slabs));
    EF_TRY(B.get(c, (size_t)cov_i8_order_bytes(d), &order));
    EF_HIP(c, launch_cov_i8_cross(s, plan, d, At, slabs, S64, order), "X'^T X' (int8)");
  }
  const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  EF_HIP(c, hipMemcpyAsync(sum_out, S1, d * sizeof(uint64_t), kind, s), "out sum");
  EF_HIP(c, hipMemcpyAsync(sumsq_out, S2, d * sizeof(uint64_t), kind, s), "out sumsq");
  if (!dev) EF_HIP(c, hipMemcpyAsync(cross_out, S64, (size_t)d * d * sizeof(int64_t), kind, s), "out cross");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  return EF_OK;
}

extern "C" int ef_fit_from_stats(ef_ctx* c, const uint64_t* sum, const uint64_t* sumsq, const int64_t* cross,
                                 int64_t n_total, int64_t d, int32_t k, uint32_t flags, double* mean_out,
                                 double* var_out, double* scale_out, double* comps_out, double* eig_out, double* tv_out,
                                 int32_t* k_out, int32_t* iters_out) {
  if (!c) return EF_E_INVALID;
  if (!sum || !sumsq || !cross || d < 1 || k < 1 || !mean_out || !comps_out || !eig_out)
    return set_err(c, EF_E_INVALID, "ef_fit_from_stats: bad arguments (need the pieces, d >= 1, k >= 1, outputs)");
  if (n_total < 2 || n_total < d)
    return set_err(c, EF_E_INVALID, "ef_fit_from_stats: the sample-sharded fit is the covariance path (n_total >= d, "
                                    "n_total >= 2)");
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  const bool dev = flags & EF_MEM_DEVICE;
  const bool stdz = flags & EF_FIT_STANDARDIZE;
  const int kk = (int)(k < d ? k : d);
  Bufs B;
  const unsigned long long *S1 = reinterpret_cast<const unsigned long long*>(sum),
                           *S2 = reinterpret_cast<const unsigned long long*>(sumsq);
  const long long* S64 = reinterpret_cast<const long long*>(cross);
  if (!dev) {  // stage the host pieces
    unsigned long long *h1, *h2;
    long long* h3;
    EF_TRY(B.get(c, (size_t)d, &h1));
    EF_TRY(B.get(c, (size_t)d, &h2));
    EF_TRY(B.get(c, (size_t)d * d, &h3));
    EF_HIP(c, hipMemcpyAsync(h1, sum, d * sizeof(uint64_t), hipMemcpyHostToDevice, s), "H2D sum");
    EF_HIP(c, hipMemcpyAsync(h2, sumsq, d * sizeof(uint64_t), hipMemcpyHostToDevice, s), "H2D sumsq");
    EF_HIP(c, hipMemcpyAsync(h3, cross, (size_t)d * d * sizeof(int64_t), hipMemcpyHostToDevice, s), "H2D cross");
    S1 = h1, S2 = h2, S64 = h3;
  }
  double *mean, *var, *scale, *w, *C, *work, *U, *lam, *comps, *En, *tv;
  long long* cvec;
  EF_TRY(B.get(c, (size_t)d, &mean));
  EF_TRY(B.get(c, (size_t)d, &var));
  EF_TRY(B.get(c, (size_t)d, &scale));
  EF_TRY(B.get(c, (size_t)d, &w));
  EF_TRY(B.get(c, (size_t)d * d, &C));
  EF_TRY(B.get(c, kWorkElems, &work));
  EF_TRY(B.get(c, (size_t)d * kk, &U));
  EF_TRY(B.get(c, (size_t)kk, &lam));
  EF_TRY(B.get(c, (size_t)kk * d, &comps));
  EF_TRY(B.get(c, (size_t)d * kk, &En));
  EF_TRY(B.get(c, 1, &tv));
  EF_TRY(B.get(c, (size_t)d, &cvec));
  EF_HIP(c, launch_stats_finalize(s, S1, S2, n_total, d, stdz ? 1 : 0, mean, var, scale, w), "stats");
  EF_HIP(c, launch_cov_from_cross(s, S64, S1, n_total, d, stdz ? w : nullptr, cvec, C), "covariance (from pieces)");
  EF_HIP(c, launch_trace(s, C, d, d, tv), "trace");
  int iters = 0;
  EF_TRY(eig_topk(c, B, C, d, kk, work, U, lam, &iters));
  EF_HIP(c, launch_normalize_sign(s, U, d, kk, kk, comps, En), "normalize");
  EF_TRY(complete_null_components(c, n_total, d, kk, lam, comps, En));
  const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  EF_HIP(c, hipMemcpyAsync(mean_out, mean, d * sizeof(double), kind, s), "out mean");
  if (var_out) EF_HIP(c, hipMemcpyAsync(var_out, var, d * sizeof(double), kind, s), "out var");
  if (scale_out) EF_HIP(c, hipMemcpyAsync(scale_out, scale, d * sizeof(double), kind, s), "out scale");
  EF_HIP(c, hipMemcpyAsync(comps_out, comps, (size_t)kk * d * sizeof(double), kind, s), "out comps");
  EF_HIP(c, hipMemcpyAsync(eig_out, lam, kk * sizeof(double), kind, s), "out eig");
  if (tv_out) EF_HIP(c, hipMemcpyAsync(tv_out, tv, sizeof(double), kind, s), "out tv");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  if (k_out) *k_out = kk;
  if (iters_out) *iters_out = iters;
  return EF_OK;
}

namespace {
__global__ void recip_kernel(const double* __restrict__ a, int64_t n, double* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = 1.0 / a[i];  // the division stats_finalize_kernel makes for w
}
}  // namespace

extern "C" int ef_fit_transform(ef_ctx* c, const uint8_t* X, int64_t n, int64_t d, const double* mean,
                                const double* scale, const double* comps, int32_t k, uint32_t flags, double* proj_out) {
  if (!c) return EF_E_INVALID;
  if (!X || n < 1 || d < 1 || k < 1 || !mean || !comps || !proj_out)
    return set_err(c, EF_E_INVALID, "ef_fit_transform: bad arguments (need X, n >= 1, d >= 1, k >= 1, model, out)");
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  const bool dev = flags & EF_MEM_DEVICE;
  Bufs B;
  const uint8_t* Xd = X;
  const double *mu = mean, *sc = scale, *cp = comps;
  if (!dev) {
    uint8_t* xb;
    double *m1, *s1 = nullptr, *c1;
    EF_TRY(B.get(c, (size_t)n * d, &xb));
    EF_TRY(B.get(c, (size_t)d, &m1));
    EF_TRY(B.get(c, (size_t)k * d, &c1));
    EF_HIP(c, hipMemcpyAsync(xb, X, (size_t)n * d, hipMemcpyHostToDevice, s), "H2D X");
    EF_HIP(c, hipMemcpyAsync(m1, mean, d * sizeof(double), hipMemcpyHostToDevice, s), "H2D mean");
    EF_HIP(c, hipMemcpyAsync(c1, comps, (size_t)k * d * sizeof(double), hipMemcpyHostToDevice, s), "H2D comps");
    if (scale) {
      EF_TRY(B.get(c, (size_t)d, &s1));
      EF_HIP(c, hipMemcpyAsync(s1, scale, d * sizeof(double), hipMemcpyHostToDevice, s), "H2D scale");
    }
    Xd = xb, mu = m1, sc = s1, cp = c1;
  }
  double *w = nullptr, *En, *proj, *work;
  if (sc) {
    EF_TRY(B.get(c, (size_t)d, &w));
    hipLaunchKernelGGL(recip_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, sc, d, w);
  }
  EF_TRY(B.get(c, (size_t)d * k, &En));
  EF_TRY(B.get(c, (size_t)n * k, &proj));
  EF_TRY(B.get(c, kWorkElems, &work));
  EF_HIP(c, launch_transpose_f64(s, cp, d, k, d, En, k), "E = comps^T");
  if (proj_i8_supported(Xd, n, d, k)) {
    uint8_t* pw;
    EF_TRY(B.get(c, proj_i8_work_bytes(n, d, k), &pw));
    EF_HIP(c, launch_proj_i8(s, Xd, n, d, mu, w, En, k, pw, proj), "F = A.E (int8 digits)");
  } else {
    EF_HIP(c, gemm64(s, Operand::pixels(Xd, EF_U8, d, false, mu, w), Operand::dense(En, k, false), n, k, d, 1.0, proj,
                     k, work, kWorkElems),
           "F = A.E");
  }
  EF_HIP(c, hipMemcpyAsync(proj_out, proj, (size_t)n * k * sizeof(double),
                           dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s),
         "out proj");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  return EF_OK;
}

// Column statistics alone (ManualStandardScaler.fit, scripts/manual/train-v2.py:58-64, and
// StandardScaler.fit): exact integer sums for uint8, two-pass fp64 for float input.
extern "C" int ef_colstats(ef_ctx* c, const void* Xv, int32_t x_dtype, int64_t n, int64_t d, uint32_t flags,
                           double* mean_out, double* var_out) {
  if (!c) return EF_E_INVALID;
  if (!Xv || n < 1 || d < 1 || !mean_out)
    return set_err(c, EF_E_INVALID, "ef_colstats: bad arguments (need X, n >= 1, d >= 1, mean_out)");
  if (x_dtype != EF_U8 && x_dtype != EF_F32 && x_dtype != EF_F64)
    return set_err(c, EF_E_INVALID, "ef_colstats: x_dtype must be EF_U8, EF_F32 or EF_F64");
  (void)hipSetDevice(c->device);
  hipStream_t s = c->stream;
  const bool dev = flags & EF_MEM_DEVICE;
  const size_t esize = x_dtype == EF_U8 ? 1 : (x_dtype == EF_F32 ? 4 : 8);
  Bufs B;
  const void* Xdv = Xv;
  if (!dev) {
    uint8_t* xb;
    EF_TRY(B.get(c, (size_t)n * d * esize, &xb));
    EF_HIP(c, hipMemcpyAsync(xb, Xv, (size_t)n * d * esize, hipMemcpyHostToDevice, s), "H2D X");
    Xdv = xb;
  }
  double *mean, *var, *scale, *w;
  EF_TRY(B.get(c, (size_t)d, &mean));
  EF_TRY(B.get(c, (size_t)d, &var));
  EF_TRY(B.get(c, (size_t)d, &scale));
  EF_TRY(B.get(c, (size_t)d, &w));
  if (x_dtype == EF_U8) {
    unsigned long long *S1, *S2;
    EF_TRY(B.get(c, (size_t)d, &S1));
    EF_TRY(B.get(c, (size_t)d, &S2));
    EF_HIP(c, hipMemsetAsync(S1, 0, d * sizeof(unsigned long long), s), "memset");
    EF_HIP(c, hipMemsetAsync(S2, 0, d * sizeof(unsigned long long), s), "memset");
    EF_HIP(c, launch_colstats(s, static_cast<const uint8_t*>(Xdv), n, d, S1, S2), "colstats");
    EF_HIP(c, launch_stats_finalize(s, S1, S2, n, d, 0, mean, var, scale, w), "stats");
  } else {
    double* part;
    EF_TRY(B.get(c, colstats_float_work_elems(n, d), &part));
    EF_HIP(c, launch_colstats_float(s, Xdv, x_dtype, n, d, 0, part, mean, var, scale, w), "colstats (float)");
  }
  const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  EF_HIP(c, hipMemcpyAsync(mean_out, mean, d * sizeof(double), kind, s), "out mean");
  if (var_out) EF_HIP(c, hipMemcpyAsync(var_out, var, d * sizeof(double), kind, s), "out var");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  return EF_OK;
}

// The fit's CholQR factor on its own (API v7; ADVICE r5: a direct check of the blocked
// factor for padded and odd orders and of the failed-pivot contract): Li = L^-1 for
// G = L L^T (m <= 256, row-major, ldg >= m), host pointers.  A pivot <= tol_rel x max diag(G)
// sets *info = -(column + 1) and leaves Li as given (the subspace iteration then
// eigen-orthonormalises); *info = 0 on success.
extern "C" int ef_chol_inv(ef_ctx* c, const double* G, int32_t m, int64_t ldg, double tol_rel, double* Li,
                           int32_t* info) {
  using namespace ef;
  if (!c) return EF_E_INVALID;
  if (!G || !Li || !info || m < 1 || ldg < m || !chol_inv_supported(m))
    return set_err(c, EF_E_INVALID, "ef_chol_inv: bad arguments (1 <= m <= 256, ldg >= m)");
  EF_HIP(c, hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  DevBuf dG, dL, dW, dI;
  auto done = [&](int rc) {
    release(dG);
    release(dL);
    release(dW);
    release(dI);
    return rc;
  };
  int rc = ensure(c, dG, (size_t)m * ldg * sizeof(double));
  if (rc == EF_OK) rc = ensure(c, dL, (size_t)m * m * sizeof(double));
  if (rc == EF_OK) rc = ensure(c, dW, chol_inv_work_elems(m) * sizeof(double));
  if (rc == EF_OK) rc = ensure(c, dI, sizeof(int));
  if (rc != EF_OK) return done(rc);
  hipError_t e = hipMemcpyAsync(dG.p, G, (size_t)m * ldg * sizeof(double), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(dL.p, Li, (size_t)m * m * sizeof(double), hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = launch_chol_inv(s, static_cast<const double*>(dG.p), m, ldg, tol_rel, static_cast<double*>(dL.p),
                        static_cast<int*>(dI.p), static_cast<double*>(dW.p));
  int hinfo = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(Li, dL.p, (size_t)m * m * sizeof(double), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(&hinfo, dI.p, sizeof(int), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return done(hip_err(c, e, "ef_chol_inv"));
  *info = hinfo;
  return done(EF_OK);
}
