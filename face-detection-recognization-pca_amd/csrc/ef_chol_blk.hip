// Blocked CholQR factor of the fit's subspace iteration (m <= 256): G = L L^T and
// Li = L^-1, the right factor of Q = Y . L^-T (ef_fit.hip orthonormalise).
//
// Round 5 replaces the register-resident one-workgroup kernel (chol_inv_reg_kernel in
// ef_linalg.hip: 512 barrier-separated column steps, ~0.31 ms at m = 256) by two kernels:
//
//  chol_blk_kernel (ONE workgroup of 8 waves): right-looking Cholesky over 16 x 16 blocks.
//    Waves 0..6 own the lower blocks (I, K), round robin over b = I(I+1)/2 + K, held in
//    MFMA accumulators; wave 7 factors the diagonal blocks.  Per block column J:
//      D  (wave 7)    L_JJ = chol(A_JJ) and Inv_JJ = L_JJ^-1 by lane-parallel column
//                     sweeps (lane c holds column c; column t reaches every lane by
//                     v_readlane, so no LDS round trip sits on the serial chain)
//      P  (workers)   L_IJ = A_IJ . Inv_JJ^T for I > J  (v_mfma_f64_16x16x4_f64)
//      T1 (workers)   A_I,J+1 -= L_IJ . L_J+1,J^T: block column J+1 first, so that
//      D of J+1 (wave 7) runs beside
//      T2 (workers)   A_IK -= L_IJ . L_KJ^T for K > J + 1 (the rest of the trailing matrix).
//    Three barriers per block column; the serial part is 16 diagonal factorisations
//    instead of 512 workgroup-wide column steps.
//  tri_inv_blk_kernel (one workgroup per block column J, 4 waves): X = L^-1 by blocked
//    forward substitution, X_JJ = Inv_JJ, X_IJ = -Inv_II . sum_{K=J}^{I-1} L_IK X_KJ, the
//    K sum split over the 4 waves and added in a fixed order.
//
// Operand images.  For v_mfma_f64_16x16x4_f64 (A lane l = A[l&15][l>>4], B lane l =
// B[l>>4][l&15], D lane l reg r = D[(l>>4)+4r][l&15]) every operand and accumulator here is
// a 16 x 16 block stored as 256 doubles with MFMA step r reading element 64r + lane:
// a ROW-major block is the accumulator / B-operand image of M, a COLUMN-major block the
// A-operand image of M.  D = M . X then takes M column-major and X row-major and yields D
// row-major, so the workers keep F(-A_IK) = column-major (-A_IK) (= row-major (-A_IK)^T)
// in their accumulators:  (-A_IK)^T += L_KJ . L_IJ^T  is the trailing update and
// L_IJ^T = (-Inv_JJ) . (-A_IJ)^T the panel solve, whose row-major result is column-major
// L_IJ, the operand image the trailing updates read.  All LDS reads are lane-contiguous
// 8-byte runs (conflict-free).
//
// Pivots: the unscaled right-looking rule of the old kernel, fail when a pivot <= tol_rel *
// max diag(G) (*info = -(column + 1), Li untouched).  Orders below a multiple of 16 are
// padded with a diagonal equal to that maximum (zero coupling, so the leading m x m block
// of the padded factor and inverse are the true ones).
#include "ef_linalg.hpp"

#include <cmath>

namespace ef {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kCbMaxNb = 16;              // blocks per side (m <= 256)
constexpr int kCbWorkers = 7;             // waves owning lower blocks
constexpr int kCbSlots = 20;              // ceil(136 / 7)
constexpr int kCbThreads = 64 * (kCbWorkers + 1);

__device__ __forceinline__ int blk_index(int I, int K) { return I * (I + 1) / 2 + K; }

__device__ __forceinline__ double rdlane(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ f64x4 mma(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// acc += M . X for 16 x 16 blocks: M column-major (A image), X row-major (B image), in LDS
__device__ __forceinline__ f64x4 block_mma(const double* Mcol, const double* Xrow, f64x4 acc, int lane) {
  double a[4], b[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    a[r] = Mcol[64 * r + lane];
    b[r] = Xrow[64 * r + lane];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) acc = mma(a[r], b[r], acc);
  return acc;
}

}  // namespace

#ifdef EF_CB_STAMP  // phase timing (tools/micro/chol_inv_bench.cpp -DEF_CB_STAMP): s_memtime
                    // per block column, [0] = worker wave 0, [1] = the diagonal wave
__device__ unsigned long long g_cb_stamp[2][kCbMaxNb][8];
#define CB_STAMP(w, J, k) \
  do {                    \
    if (lane == 0) g_cb_stamp[w][J][k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define CB_STAMP(w, J, k) \
  do {                    \
  } while (0)
#endif

// LF: column-major L blocks at blk_index(I, K) * 256; invN: column-major -Inv_JJ at J * 256
// (after the blocks); invT: row-major Inv_JJ
size_t chol_inv_work_elems(int m) {
  const int nb = (m + 15) / 16;
  return (size_t)(nb * (nb + 1) / 2 + 2 * nb) * 256;
}

__global__ __launch_bounds__(kCbThreads) void chol_blk_kernel(const double* __restrict__ G, int m, int64_t lda,
                                                              double tol_rel, double* __restrict__ LF,
                                                              double* __restrict__ invN, double* __restrict__ invT,
                                                              int* __restrict__ info) {
  __shared__ double panel[kCbMaxNb][256];  // column-major L_IJ of the current block column
  __shared__ double dbuf[256];             // column-major -A_JJ (after all its updates)
  __shared__ double ibuf[256];             // column-major -Inv_JJ
  __shared__ double lbuf[256];             // column-major L_JJ (diagonal wave only)
  __shared__ double rsb[16];               // 1 / L_tt
  __shared__ double red[kCbWorkers + 1];
  __shared__ int fail;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: block ownership in SGPRs
  const int c = lane & 15, g = lane >> 4;
  const int nb = (m + 15) >> 4, nblk = nb * (nb + 1) / 2;
  const bool worker = wave < kCbWorkers;
  if (tid == 0) fail = 0;

  double dm = 0.0;
  for (int i = tid; i < m; i += kCbThreads) dm = fmax(dm, G[(int64_t)i * lda + i]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dm = fmax(dm, __shfl_xor(dm, off));
  if (lane == 0) red[wave] = dm;
  __syncthreads();
  double mx = 0.0;
#pragma unroll
  for (int w = 0; w <= kCbWorkers; ++w) mx = fmax(mx, red[w]);
  const double tol = tol_rel * mx;
  const double pad = mx > 0.0 ? mx : 1.0;

  // Waves take one of two paths with the same barrier sequence per block column (B1 after
  // D / T2, B2 after P, B3 after T1), so the diagonal wave's registers and the workers'
  // accumulators are allocated separately.
  if (worker) {
    // this wave's blocks: packed 32 I + K (wave-uniform, -1 past the end) and their
    // accumulators F(-A_IK)
    int sIK[kCbSlots];
    f64x4 acc[kCbSlots];
#pragma unroll
    for (int s = 0; s < kCbSlots; ++s) {
      const int b = wave + kCbWorkers * s;
      int I = -1, K = -1;
      if (b < nblk) {
        I = (int)((sqrtf(8.0f * (float)b + 1.0f) - 1.0f) * 0.5f);
        while (I * (I + 1) / 2 > b) --I;
        while ((I + 1) * (I + 2) / 2 <= b) ++I;
        K = b - I * (I + 1) / 2;
      }
      sIK[s] = I < 0 ? -1 : 32 * I + K;
      acc[s] = f64x4{0.0, 0.0, 0.0, 0.0};
      if (I >= 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // element (c, 4r + g); diagonal blocks from the lower triangle
          int i = 16 * I + c, l = 16 * K + 4 * r + g;
          if (i < l) {
            const int t = i;
            i = l;
            l = t;
          }
          const double v = (i < m && l < m) ? G[(int64_t)i * lda + l] : (i == l ? pad : 0.0);
          acc[s][r] = -v;
        }
        if (I == 0 && K == 0)
#pragma unroll
          for (int r = 0; r < 4; ++r) dbuf[64 * r + lane] = acc[s][r];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    for (int J = 0; J < nb; ++J) {
      // (laundered each iteration: what derives from them is recomputed, not hoisted into
      // registers the accumulators need)
      int lane_j = lane;
      asm volatile("" : "+v"(lane_j));
#pragma unroll
      for (int s = 0; s < kCbSlots; ++s) asm volatile("" : "+s"(sIK[s]));
      if (wave == 0) CB_STAMP(0, J, 0);
      // ---- T2 of block column J - 1: the blocks with K > J
      if (J > 0) {
#pragma unroll
        for (int s = 0; s < kCbSlots; ++s) {
          const int I = sIK[s] >> 5, K = sIK[s] & 31;
          if (sIK[s] >= 0 && K > J) acc[s] = block_mma(panel[K], panel[I], acc[s], lane_j);
          __builtin_amdgcn_sched_barrier(0);  // one slot's operands live at a time
        }
      }
      if (wave == 0) CB_STAMP(0, J, 1);
      __syncthreads();  // B1
      if (fail) return;
      if (wave == 0) CB_STAMP(0, J, 2);
      // ---- P: L_IJ (column-major) = row-major result of (-Inv_JJ) . (-A_IJ)^T
#pragma unroll
      for (int s = 0; s < kCbSlots; ++s) {
        const int I = sIK[s] >> 5, K = sIK[s] & 31;
        if (sIK[s] >= 0 && K == J && I > J) {
          double a[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) a[r] = ibuf[64 * r + lane_j];
          f64x4 L = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int r = 0; r < 4; ++r) L = mma(a[r], acc[s][r], L);
          double* lf = LF + (int64_t)blk_index(I, J) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            panel[I][64 * r + lane_j] = L[r];
            lf[64 * r + lane_j] = L[r];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (wave == 0) CB_STAMP(0, J, 3);
      __syncthreads();  // B2
      if (wave == 0) CB_STAMP(0, J, 4);
      // ---- T1: block column J + 1 (its diagonal block goes to dbuf for the next D)
#pragma unroll
      for (int s = 0; s < kCbSlots; ++s) {
        const int I = sIK[s] >> 5, K = sIK[s] & 31;
        if (sIK[s] >= 0 && K == J + 1) {
          acc[s] = block_mma(panel[K], panel[I], acc[s], lane_j);
          if (I == K)
#pragma unroll
            for (int r = 0; r < 4; ++r) dbuf[64 * r + lane_j] = acc[s][r];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (wave == 0) CB_STAMP(0, J, 5);
      __syncthreads();  // B3
      if (wave == 0) CB_STAMP(0, J, 6);
    }
  } else {
    __syncthreads();
    for (int J = 0; J < nb; ++J) {
      int c = lane & 15;
      asm volatile("" : "+v"(c));  // keeps the lane-dependent masks and constants out of
                                   // loop-invariant hoisting (they would pin ~80 registers)
      CB_STAMP(1, J, 0);
      // ---- D: factor and invert the diagonal block; lane c holds column c (lanes 16..63
      // repeat lanes 0..15).  The block is symmetrised from its lower triangle.
      double a[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = -((i >= c) ? dbuf[16 * c + i] : dbuf[16 * i + c]);
      int bad = 0;
      double dc = 0.0, rc = 0.0;  // this lane's pivot and 1 / sqrt of it
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const double d = rdlane(a[t], t);
        // uniform; the sweep runs on (its results unused) so every index stays static
        if (bad == 0 && !(d > tol)) bad = t + 1;
        const double inv = rcp_nr(d);
        const double own = a[t];  // A[t][c] = A[c][t]
        const bool act = c > t;
#pragma unroll
        for (int i = t + 1; i < 16; ++i) {
          const double ci = rdlane(a[i], t);  // A[i][t]
          // (A[i][t] A[c][t]) / d: the same product for (i, c) and (c, i), so the trailing
          // block stays exactly symmetric
          const double nv = fma(-(ci * own), inv, a[i]);
          a[i] = act ? nv : a[i];
        }
        dc = (c == t) ? d : dc;
      }
      CB_STAMP(1, J, 1);
      if (bad) {
        if (lane == 0) {
          *info = -(16 * J + bad);
          fail = 1;
        }
      } else {
        // column c of L: a[i] / sqrt(d_c) below the diagonal, sqrt(d_c) on it; staged in
        // LDS (column-major) with the reciprocal diagonal for the inverse's broadcasts
        rc = rsq_nr(dc);
        double* lf = LF + (int64_t)blk_index(J, J) * 256;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const double v = i > c ? a[i] * rc : (i == c ? dc * rc : 0.0);
          if (lane < 16) {
            lbuf[16 * c + i] = v;
            lf[16 * c + i] = v;
          }
        }
        if (lane < 16) rsb[c] = rc;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
        __builtin_amdgcn_wave_barrier();
        CB_STAMP(1, J, 2);
        // column c of X = L^-1: forward substitution on e_c (x_k = 0 for k < c); the L
        // entries are same-address LDS reads, independent of x
        double x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = (i == c) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          x[k] *= rsb[k];
#pragma unroll
          for (int i = k + 1; i < 16; ++i) x[i] = fma(-lbuf[16 * k + i], x[k], x[i]);
        }
        if (lane < 16) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            ibuf[16 * c + i] = -x[i];
            invN[J * 256 + 16 * c + i] = -x[i];
            invT[J * 256 + 16 * i + c] = x[i];
          }
        }
      }
      CB_STAMP(1, J, 3);
      __syncthreads();  // B1
      if (fail) return;
      CB_STAMP(1, J, 4);
      __syncthreads();  // B2
      CB_STAMP(1, J, 5);
      __syncthreads();  // B3
      CB_STAMP(1, J, 6);
    }
    if (lane == 0) *info = 0;
  }
}

__global__ __launch_bounds__(256) void tri_inv_blk_kernel(const double* __restrict__ LF, const double* __restrict__ invN,
                                                          const double* __restrict__ invT, int m,
                                                          double* __restrict__ Li, const int* __restrict__ info) {
  __shared__ double xb[kCbMaxNb][256];  // row-major X_KJ of this block column
  __shared__ double part[4][256];       // the waves' partial sums
  if (*info != 0) return;               // failed factorisation: Li untouched
  const int J = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int nb = (m + 15) >> 4;
  auto store = [&](int I, int r, double v) {  // element 64r + lane of row-major X_IJ
    const int row = 16 * I + 4 * r + g, col = 16 * J + c;
    if (row < m && col < m) Li[(int64_t)row * m + col] = v;
  };
  for (int e = tid; e < 256 * J; e += 256) {  // zeros above the diagonal: rows < 16 J
    const int row = e >> 4, col = 16 * J + (e & 15);
    if (row < m && col < m) Li[(int64_t)row * m + col] = 0.0;
  }
  if (w == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double v = invT[J * 256 + 64 * r + lane];
      xb[J][64 * r + lane] = v;
      store(J, r, v);
    }
  }
  __syncthreads();
  for (int I = J + 1; I < nb; ++I) {
    f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int K = J + w; K < I; K += 4) acc = block_mma(LF + (int64_t)blk_index(I, K) * 256, xb[K], acc, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) part[w][64 * r + lane] = acc[r];
    __syncthreads();
    if (w == 0) {
      double a[4];
      f64x4 T;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = invN[I * 256 + 64 * r + lane];
        const int e = 64 * r + lane;
        T[r] = ((part[0][e] + part[1][e]) + part[2][e]) + part[3][e];
      }
      f64x4 X = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) X = mma(a[r], T[r], X);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        xb[I][64 * r + lane] = X[r];
        store(I, r, X[r]);
      }
    }
    __syncthreads();
  }
}

bool chol_inv_supported(int m) { return m >= 1 && m <= 16 * kCbMaxNb; }

hipError_t launch_chol_inv(hipStream_t s, const double* G, int m, int64_t lda, double tol_rel, double* Li, int* info,
                           double* work) {
  if (!chol_inv_supported(m) || !work) return hipErrorInvalidValue;
  const int nb = (m + 15) / 16, nblk = nb * (nb + 1) / 2;
  double* LF = work;
  double* invN = LF + (size_t)nblk * 256;
  double* invT = invN + (size_t)nb * 256;
  hipLaunchKernelGGL(chol_blk_kernel, dim3(1), dim3(kCbThreads), 0, s, G, m, lda, tol_rel, LF, invN, invT, info);
  hipLaunchKernelGGL(tri_inv_blk_kernel, dim3(nb), dim3(256), 0, s, LF, invN, invT, m, Li, info);
  return hipGetLastError();
}

}  // namespace ef
