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
//  tri_inv_blk_kernel (one workgroup per block column J, 16 waves): X = L^-1 by blocked
//    forward substitution, X_JJ = Inv_JJ, X_IJ = -Inv_II . sum_{K=J}^{I-1} L_IK X_KJ, one
//    K term per wave, the terms added in a fixed order.
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
#include <utility>

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

// Block ownership: block (I, K) -> worker (I + 2K) mod 7, listed in column order.  The
// blocks of every block column fall on consecutive residues, so the panel solve and the
// column-(J+1) update of each block column spread over all workers (at most 3 blocks
// each; round robin over b put 5 on one wave), and so do every block row's, which keeps
// the trailing updates balanced too.  At most kCbSlots blocks per worker.
struct CbTab {
  short ik[kCbWorkers][kCbSlots];  // 32 I + K, -1 past the wave's last block
};
constexpr CbTab make_cb_tab() {
  CbTab t{};
  int cnt[kCbWorkers] = {};
  for (int w = 0; w < kCbWorkers; ++w)
    for (int s = 0; s < kCbSlots; ++s) t.ik[w][s] = -1;
  for (int K = 0; K < kCbMaxNb; ++K)
    for (int I = K; I < kCbMaxNb; ++I) {
      const int w = (I + 2 * K) % kCbWorkers;
      if (cnt[w] < kCbSlots) t.ik[w][cnt[w]] = (short)(32 * I + K);
      ++cnt[w];
    }
  return t;
}
constexpr bool cb_tab_fits() {
  int cnt[kCbWorkers] = {};
  for (int K = 0; K < kCbMaxNb; ++K)
    for (int I = K; I < kCbMaxNb; ++I) ++cnt[(I + 2 * K) % kCbWorkers];
  for (int w = 0; w < kCbWorkers; ++w)
    if (cnt[w] > kCbSlots) return false;
  return true;
}
static_assert(cb_tab_fits(), "a worker owns more blocks than it has slots");
__constant__ CbTab kCbTab = make_cb_tab();

// The diagonal wave's LDS images (dbuf, ibuf) are column-major with a 17-double column
// stride: its column reads (lane c: column c) and the lane-contiguous MFMA operand reads
// (flat index f = 64 r + lane -> column f >> 4, row f & 15) are then both conflict-free.
constexpr int kPs = 17;
__device__ __forceinline__ int pidx(int f) { return f + (f >> 4); }

// acc += src(lane T of this 16-lane row) * mul: one v_fmac_f64 with a DPP row_newbcast
// source (gfx950 allows 64-bit DPP with that control only); s_nop 1 covers the
// VALU-write -> DPP-read hazard the compiler cannot see through the asm
template <int T>
__device__ __forceinline__ void fmac_bcast(double& acc, double src, double mul) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(src), "v"(mul), "i"(T));
}

// Column T of the diagonal block's Cholesky (unscaled right-looking form): lane c > T
// updates a[i] -= A[i][T] A[T][c] / d for i > T, A[i][T] broadcast from lane T
template <int T>
__device__ __forceinline__ void chol_step(double (&a)[16], int c, double tol, int& bad, double& dc) {
  const double d = rdlane(a[T], T);  // the pivot (uniform)
  // uniform; the sweep runs on (its results unused) so every index stays static
  if (bad == 0 && !(d > tol)) bad = T + 1;
  const double nf = c > T ? -(a[T] * rcp_nr(d)) : 0.0;  // a[T] = A[T][c] = A[c][T]
#pragma unroll
  for (int i = T + 1; i < 16; ++i) fmac_bcast<T>(a[i], a[i], nf);
  dc = (c == T) ? d : dc;
}
template <int... Ts>
__device__ __forceinline__ void chol_sweep(double (&a)[16], int c, double tol, int& bad, double& dc,
                                           std::integer_sequence<int, Ts...>) {
  (chol_step<Ts>(a, c, tol, bad, dc), ...);
}
// Row K of the forward substitution L x = e_c: x_K = b_K / L_KK, then x_i -= L_iK x_K for
// i > K with L_iK broadcast from lane K (which holds column K of L in l)
template <int K>
__device__ __forceinline__ void inv_step(double (&x)[16], const double (&l)[16], double rc) {
  x[K] *= rdlane(rc, K);
  const double nx = -x[K];
#pragma unroll
  for (int i = K + 1; i < 16; ++i) fmac_bcast<K>(x[i], l[i], nx);
}
template <int... Ks>
__device__ __forceinline__ void inv_sweep(double (&x)[16], const double (&l)[16], double rc,
                                          std::integer_sequence<int, Ks...>) {
  (inv_step<Ks>(x, l, rc), ...);
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
  __shared__ double dbuf[16 * kPs];        // column-major -A_JJ (after all its updates)
  __shared__ double ibuf[16 * kPs];        // column-major -Inv_JJ
  __shared__ double red[kCbWorkers + 1];
  __shared__ int fail;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: block ownership in SGPRs
  const int c = lane & 15, g = lane >> 4;
  const int nb = (m + 15) >> 4;
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
      int ik = kCbTab.ik[wave][s];
      if (ik >= 0 && (ik >> 5) >= nb) ik = -1;  // (K <= I: the block is outside the order)
      const int I = ik < 0 ? -1 : ik >> 5, K = ik < 0 ? -1 : ik & 31;
      sIK[s] = ik;
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
          for (int r = 0; r < 4; ++r) dbuf[pidx(64 * r + lane)] = acc[s][r];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();
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
      lds_barrier();  // B1
      if (fail) return;
      if (wave == 0) CB_STAMP(0, J, 2);
      // ---- P: L_IJ (column-major) = row-major result of (-Inv_JJ) . (-A_IJ)^T
      double a[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = ibuf[pidx(64 * r + lane_j)];
#pragma unroll
      for (int s = 0; s < kCbSlots; ++s) {
        const int I = sIK[s] >> 5, K = sIK[s] & 31;
        if (sIK[s] >= 0 && K == J && I > J) {
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
      lds_barrier();  // B2
      if (wave == 0) CB_STAMP(0, J, 4);
      // ---- T1: block column J + 1 (its diagonal block goes to dbuf for the next D)
      if (J + 1 < nb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = panel[J + 1][64 * r + lane_j];  // L_{J+1,J}: every block's A
      }
#pragma unroll
      for (int s = 0; s < kCbSlots; ++s) {
        const int I = sIK[s] >> 5, K = sIK[s] & 31;
        if (sIK[s] >= 0 && K == J + 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[s] = mma(a[r], panel[I][64 * r + lane_j], acc[s]);
          if (I == K)
#pragma unroll
            for (int r = 0; r < 4; ++r) dbuf[pidx(64 * r + lane_j)] = acc[s][r];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (wave == 0) CB_STAMP(0, J, 5);
      lds_barrier();  // B3
      if (wave == 0) CB_STAMP(0, J, 6);
    }
  } else {
    lds_barrier();
    for (int J = 0; J < nb; ++J) {
      int c = lane & 15;
      asm volatile("" : "+v"(c));  // keeps the lane-dependent masks and constants out of
                                   // loop-invariant hoisting (they would pin ~80 registers)
      CB_STAMP(1, J, 0);
      // ---- D: factor and invert the diagonal block; lane c holds column c (lanes 16..63
      // repeat lanes 0..15, so every 16-lane row can broadcast from its own lane t).  The
      // block is symmetrised from its lower triangle.
      double a[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) a[i] = -((i >= c) ? dbuf[kPs * c + i] : dbuf[kPs * i + c]);
      int bad = 0;
      double dc = 0.0;  // this lane's pivot
      chol_sweep(a, c, tol, bad, dc, std::make_integer_sequence<int, 16>{});
      CB_STAMP(1, J, 1);
      if (bad) {
        if (lane == 0) {
          *info = -(16 * J + bad);
          fail = 1;
        }
      } else {
        // column c of L: a[i] / sqrt(d_c) below the diagonal, sqrt(d_c) on it
        const double rc = rsq_nr(dc);
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = i > c ? a[i] * rc : (i == c ? dc * rc : 0.0);
        CB_STAMP(1, J, 2);
        // column c of X = L^-1: forward substitution on e_c (x_k = 0 for k < c)
        double x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = (i == c) ? 1.0 : 0.0;
        inv_sweep(x, a, rc, std::make_integer_sequence<int, 16>{});
        if (lane < 16) {
#pragma unroll
          for (int i = 0; i < 16; ++i) ibuf[kPs * c + i] = -x[i];
        }
        // global images, four stores per array: row group q (the lane's replica) stores
        // rows i = 4j + q
        const int q = lane >> 4;
        double* lf = LF + (int64_t)blk_index(J, J) * 256;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          double xv = x[4 * j], lv = a[4 * j];
#pragma unroll
          for (int u = 1; u < 4; ++u) {
            xv = q == u ? x[4 * j + u] : xv;
            lv = q == u ? a[4 * j + u] : lv;
          }
          const int i = 4 * j + q;
          invN[J * 256 + 16 * c + i] = -xv;
          invT[J * 256 + 16 * i + c] = xv;
          lf[16 * c + i] = lv;
        }
      }
      CB_STAMP(1, J, 3);
      lds_barrier();  // B1
      if (fail) return;
      CB_STAMP(1, J, 4);
      lds_barrier();  // B2
      CB_STAMP(1, J, 5);
      lds_barrier();  // B3
      CB_STAMP(1, J, 6);
    }
    if (lane == 0) *info = 0;
  }
}

// Wave w of block column J's workgroup owns X_{J+w,J} in its accumulator registers (the
// B image its products read): at step I every wave w < I - J adds its partial
// L_{I,J+w} . X_{J+w,J} into LDS, one barrier, and wave I - J, the only later reader of
// X_IJ, sums the partials in wave order and forms X_IJ = (-Inv_II) . sum.  One barrier per
// block row; the L blocks of the next step and the wave's own -Inv are loaded a step ahead.
__global__ __launch_bounds__(64 * kCbMaxNb) void tri_inv_blk_kernel(const double* __restrict__ LF,
                                                                  const double* __restrict__ invN,
                                                                  const double* __restrict__ invT, int m,
                                                                  double* __restrict__ Li,
                                                                  const int* __restrict__ info) {
  __shared__ double part[2][kCbMaxNb][256];  // partial sums, double-buffered by step parity
  if (*info != 0) return;                    // failed factorisation: Li untouched
  const int J = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int nb = (m + 15) >> 4;
  const int own = J + w;  // the block row this wave finalises and then holds
  auto store = [&](int I, int r, double v) {  // element 64r + lane of row-major X_IJ
    const int row = 16 * I + 4 * r + g, col = 16 * J + c;
    if (row < m && col < m) Li[(int64_t)row * m + col] = v;
  };
  for (int e = tid; e < 256 * J; e += 64 * kCbMaxNb) {  // zeros above the diagonal: rows < 16 J
    const int row = e >> 4, col = 16 * J + (e & 15);
    if (row < m && col < m) Li[(int64_t)row * m + col] = 0.0;
  }
  f64x4 X = f64x4{0.0, 0.0, 0.0, 0.0};
  double ninv[4] = {0.0, 0.0, 0.0, 0.0}, lf[4] = {0.0, 0.0, 0.0, 0.0};
  if (own < nb) {
    if (w == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        X[r] = invT[J * 256 + 64 * r + lane];
        store(J, r, X[r]);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) ninv[r] = invN[own * 256 + 64 * r + lane];
    }
    if (own + 1 < nb)  // L_{J+w+1, J+w}: this wave's first partial (step I = own + 1)
#pragma unroll
      for (int r = 0; r < 4; ++r) lf[r] = LF[(int64_t)blk_index(own + 1, own) * 256 + 64 * r + lane];
  }
  for (int I = J + 1; I < nb; ++I) {
    const int buf = I & 1;
    if (own < I) {  // partial L_{I,own} . X_{own,J}
      f64x4 p = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) p = mma(lf[r], X[r], p);
      if (I + 1 < nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) lf[r] = LF[(int64_t)blk_index(I + 1, own) * 256 + 64 * r + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) part[buf][w][64 * r + lane] = p[r];
    }
    lds_barrier();
    if (own == I) {  // X_IJ = (-Inv_II) . sum of the partials of waves 0 .. I-J-1
      f64x4 T;
#pragma unroll
      for (int r = 0; r < 4; ++r) T[r] = part[buf][0][64 * r + lane];
      for (int v = 1; v < w; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[r] += part[buf][v][64 * r + lane];
      X = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) X = mma(ninv[r], T[r], X);
#pragma unroll
      for (int r = 0; r < 4; ++r) store(I, r, X[r]);
    }
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
  hipLaunchKernelGGL(tri_inv_blk_kernel, dim3(nb), dim3(64 * kCbMaxNb), 0, s, LF, invN, invT, m, Li, info);
  return hipGetLastError();
}

}  // namespace ef
