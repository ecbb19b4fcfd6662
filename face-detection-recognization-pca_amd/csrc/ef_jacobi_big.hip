// Symmetric eigensolver for orders beyond the LDS Jacobi (m > kJacobiMax): the same
// cyclic two-sided Jacobi method (circle ordering, m/2 disjoint rotations per round,
// rotation skip test and sweep-level convergence of jacobi_kernel in ef_linalg.hip),
// with the matrix and the eigenvector accumulator in HBM/L2 and every round spread over
// the whole GPU:
//   * one launch per round; thread (t, u) owns the 2 x 2 block rows {p_t, q_t} x columns
//     {p_u, q_u} and applies both rotations (G' = J^T G J) — no intra-round barrier;
//   * the rotation of each pair is recomputed by every thread that needs it from the
//     round's input matrix, which is therefore ping-ponged (in-place would race on the
//     pivots); V <- V J is in place (thread (i, u) owns V[i][p_u], V[i][q_u]);
//   * a sweep whose pivots are all below 1e-12 of their diagonal scale ends the solve
//     (one host read of a flag per sweep).
// Orders >= kBlockJacobiMin run the BLOCK variant instead: the matrix is cut into 16-wide
// blocks, a round pairs the blocks (circle ordering over blocks, 15 rounds per sweep at
// order 256 instead of 255), each pair's 32 x 32 subproblem is diagonalised in LDS by the
// scalar method (bj_solve_kernel: kInnerSweeps inner sweeps of 31 rounds, each round's
// 16 rotations computed once by one wave, rotations accumulated into Z), and one launch applies every pair's Z to
// the matrix (G'[P][Q] = Z_P^T G[P][Q] Z_Q, block-pair parallel) and to V (V <- V Z).
// Same fixed point and convergence flag (a sweep in which no off-diagonal entry exceeded
// 1e-12 of its diagonal scale), 17x fewer launches per sweep.
// Used for the Rayleigh-Ritz / orthonormalisation problems of the subspace iteration at
// k > 80 (BASELINE.json config 3: k = 128; config 5: k = 512) and for direct solves of
// moderate orders.  Quadratic convergence: a nearly diagonal input (warm subspace) needs
// 2-3 sweeps.
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "ef_linalg.hpp"

namespace ef {

__device__ __forceinline__ int circle_pos(int j, int r, int mp) { return j == 0 ? 0 : 1 + ((j - 1 + r) % (mp - 1)); }

struct Rot {
  int p, q;
  double c, s;
  bool on;
};

__device__ __forceinline__ Rot pair_rotation(const double* __restrict__ G, int mp, int r, int t) {
  Rot R;
  int p = circle_pos(t, r, mp), q = circle_pos(mp - 1 - t, r, mp);
  if (p > q) { const int x = p; p = q; q = x; }
  R.p = p;
  R.q = q;
  const double apq = G[(int64_t)p * mp + q];
  const double app = G[(int64_t)p * mp + p], aqq = G[(int64_t)q * mp + q];
  const double g = 100.0 * fabs(apq);
  if (apq == 0.0 || (fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq))) {
    R.on = false;
    R.c = 1.0;
    R.s = 0.0;
  } else {
    const double theta = (aqq - app) / (2.0 * apq);
    double tt = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
    if (fabs(theta) > 1e150) tt = 0.5 / fabs(theta);
    if (theta < 0.0) tt = -tt;
    R.c = 1.0 / sqrt(tt * tt + 1.0);
    R.s = tt * R.c;
    R.on = true;
  }
  return R;
}

__global__ void jbig_init_kernel(const double* __restrict__ A, int m, int64_t lda, int mp, double* __restrict__ G,
                                 double* __restrict__ V) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)mp * mp) return;
  const int i = (int)(e / mp), j = (int)(e - (e / mp) * mp);
  G[e] = (i < m && j < m) ? 0.5 * (A[(int64_t)i * lda + j] + A[(int64_t)j * lda + i]) : 0.0;
  V[e] = i == j ? 1.0 : 0.0;
}

__global__ __launch_bounds__(256) void jbig_round_kernel(const double* __restrict__ Gin, double* __restrict__ Gout,
                                                        double* __restrict__ V, int mp, int r, int* __restrict__ flag) {
  const int np = mp / 2;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nb = (int64_t)np * np;
  if (e < nb) {
    const int t = (int)(e / np), u = (int)(e - (e / np) * np);
    const Rot a = pair_rotation(Gin, mp, r, t);
    const Rot b = t == u ? a : pair_rotation(Gin, mp, r, u);
    const double x00 = Gin[(int64_t)a.p * mp + b.p], x01 = Gin[(int64_t)a.p * mp + b.q];
    const double x10 = Gin[(int64_t)a.q * mp + b.p], x11 = Gin[(int64_t)a.q * mp + b.q];
    // rows: p <- c p - s q, q <- s p + c q
    const double y00 = a.c * x00 - a.s * x10, y01 = a.c * x01 - a.s * x11;
    const double y10 = a.s * x00 + a.c * x10, y11 = a.s * x01 + a.c * x11;
    // columns, same convention
    double z00 = b.c * y00 - b.s * y01, z01 = b.s * y00 + b.c * y01;
    double z10 = b.c * y10 - b.s * y11, z11 = b.s * y10 + b.c * y11;
    if (t == u && a.on) {
      z01 = 0.0;
      z10 = 0.0;
      // a sweep whose rotated pivots were all below 1e-12 of their diagonal scale ends
      // the solve: the matrix is then diagonal to ~1e-12 relative (near-degenerate pairs
      // may still rotate by large angles without extending the sweep count)
      if (fabs(x01) > 1e-12 * sqrt(fabs(x00 * x11))) *flag = 1;
    }
    Gout[(int64_t)a.p * mp + b.p] = z00;
    Gout[(int64_t)a.p * mp + b.q] = z01;
    Gout[(int64_t)a.q * mp + b.p] = z10;
    Gout[(int64_t)a.q * mp + b.q] = z11;
    return;
  }
  const int64_t f = e - nb;
  if (f >= (int64_t)mp * np) return;
  const int i = (int)(f / np), u = (int)(f - (f / np) * np);
  const Rot b = pair_rotation(Gin, mp, r, u);
  if (!b.on) return;
  const double vp = V[(int64_t)i * mp + b.p], vq = V[(int64_t)i * mp + b.q];
  V[(int64_t)i * mp + b.p] = b.c * vp - b.s * vq;
  V[(int64_t)i * mp + b.q] = b.s * vp + b.c * vq;
}

// ------------------------------------------------------------------ block Jacobi
#ifndef EF_BJ_EARLY  // 0: no early convergence test (A/B builds)
#define EF_BJ_EARLY 1
#endif
constexpr int kBlockJacobiMin = 128;
constexpr int BJ = 16;           // block width; a pair problem is 2 * BJ = 32
constexpr int kInnerSweeps = 1;  // inner sweeps per pair problem (the outer sweeps revisit every pair)

__device__ __forceinline__ int bj_index(int I, int J, int a) { return a < BJ ? I * BJ + a : J * BJ + (a - BJ); }

__device__ __forceinline__ void bj_pair(int r, int t, int nb, int* I, int* J) {
  int p = circle_pos(t, r, nb), q = circle_pos(nb - 1 - t, r, nb);
  if (p > q) { const int x = p; p = q; q = x; }
  *I = p;
  *J = q;
}

// rotation of LDS pair (p, q) of a 32 x 32 matrix (row stride 33), the rule of pair_rotation
__device__ __forceinline__ Rot lds_rotation(const double (*S)[33], int r, int t) {
  Rot R;
  int p = circle_pos(t, r, 2 * BJ), q = circle_pos(2 * BJ - 1 - t, r, 2 * BJ);
  if (p > q) { const int x = p; p = q; q = x; }
  R.p = p;
  R.q = q;
  const double apq = S[p][q], app = S[p][p], aqq = S[q][q];
  const double g = 100.0 * fabs(apq);
  if (apq == 0.0 || (fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq))) {
    R.on = false;
    R.c = 1.0;
    R.s = 0.0;
  } else {
    // the rule's quotients and roots from the hardware reciprocal / reciprocal square
    // root, each refined by two Newton steps (~1 ulp): the 16 rotations of an inner round
    // are its serial latency (a chain of three IEEE divisions and two square roots before)
    const double theta = (aqq - app) * rcp_nr(2.0 * apq);
    const double at = fabs(theta);
    double tt;
    if (at > 1e150) {
      tt = 0.5 * rcp_nr(at);
    } else {
      const double u = fma(theta, theta, 1.0);
      tt = rcp_nr(at + u * rsq_nr(u));
    }
    if (theta < 0.0) tt = -tt;
    R.c = rsq_nr(fma(tt, tt, 1.0));
    R.s = tt * R.c;
    R.on = true;
  }
  return R;
}

constexpr int BS = 2 * BJ;  // order of a pair problem
typedef double Tile[BS][BS + 1];

// (Z^T A)[a][b] and (X Z)[a][b] of 32 x 32 LDS tiles, k ascending: the one summation order
// every product of a pair rotation uses (the solve's recomputed blocks equal the apply's)
__device__ __forceinline__ double zt_dot(const Tile& Z, int a, const Tile& A, int b) {
  double acc = 0.0;
#pragma unroll 8
  for (int k = 0; k < BS; ++k) acc = fma(Z[k][a], A[k][b], acc);
  return acc;
}
__device__ __forceinline__ double xz_dot(const Tile& X, int a, const Tile& Z, int b) {
  double acc = 0.0;
#pragma unroll 8
  for (int k = 0; k < BS; ++k) acc = fma(X[a][k], Z[k][b], acc);
  return acc;
}

// the pair of round r holding block blk, and its half (0: the lower block of the pair)
__device__ __forceinline__ void bj_locate(int r, int nb, int blk, int* pair, int* half) {
  for (int t = 0; t < nb / 2; ++t) {
    int a, b;
    bj_pair(r, t, nb, &a, &b);
    if (a == blk) *pair = t, *half = 0;
    if (b == blk) *pair = t, *half = 1;
  }
}

// Solve of round r, one workgroup per block pair: diagonalise S = G[P][P] (32 x 32) in LDS,
// Zcur[pair] = the accumulated rotations, the diagonalised block into Gnext.  256 threads:
// thread (t, u) owns the 2 x 2 block {p_t, q_t} x {p_u, q_u} of each inner round
// (ping-pong S, one barrier per round).  S's diagonal 16-blocks come from Gcur (written
// by the previous round's solve); with a pending apply (Zprev: the rotations of round rp,
// not yet applied to Gcur's off-diagonal blocks) the two off-diagonal 16-blocks are
// recomputed here from Gprev exactly as the apply computes them, so this round need not
// wait for that apply.
__device__ __forceinline__ void bj_solve_part(const double* __restrict__ Gprev, const double* Gcur,
                                              double* __restrict__ Gnext, int mp, int r, int rp,
                                              const double* __restrict__ Zprev, double* __restrict__ Zcur,
                                              int* __restrict__ flag, const double* __restrict__ tolp,
                                              unsigned long long* __restrict__ pmax, int pair, Tile* sm) {
  const int nb = mp / BJ;
  int I, J;
  bj_pair(r, pair, nb, &I, &J);
  Tile(&S)[2] = *reinterpret_cast<Tile(*)[2]>(sm);
  Tile& Z = sm[2];
  __shared__ int any;
  __shared__ Rot rot[BJ];
  const int tid = threadIdx.x;
  int PI = 0, hI = 0, PJ = 0, hJ = 0;
  if (Zprev) {
    bj_locate(rp, nb, I, &PI, &hI);
    bj_locate(rp, nb, J, &PJ, &hJ);
  }
  const bool own = !Zprev || PI == PJ;  // the off-diagonal blocks are final in Gcur
  if (tid == 0) any = 0;
  for (int e = tid; e < BS * BS; e += 256) {
    const int a = e >> 5, b = e & 31;
    if (own || (a < BJ) == (b < BJ)) S[0][a][b] = Gcur[(int64_t)bj_index(I, J, a) * mp + bj_index(I, J, b)];
    Z[a][b] = a == b ? 1.0 : 0.0;
  }
  if (!own) {
    Tile &A = sm[3], &ZP = sm[4], &ZQ = sm[5], &T = sm[6];
    for (int side = 0; side < 2; ++side) {  // rows I, columns J; then rows J, columns I
      const int Pr = side ? PJ : PI, hr = side ? hJ : hI, Pc = side ? PI : PJ, hc = side ? hI : hJ;
      int IP, JP, IQ, JQ;
      bj_pair(rp, Pr, nb, &IP, &JP);
      bj_pair(rp, Pc, nb, &IQ, &JQ);
      __syncthreads();  // the scratch tiles are free
      const double* zp = Zprev + (int64_t)Pr * BS * BS;
      const double* zq = Zprev + (int64_t)Pc * BS * BS;
      for (int e = tid; e < BS * BS; e += 256) {
        const int a = e >> 5, b = e & 31;
        A[a][b] = Gprev[(int64_t)bj_index(IP, JP, a) * mp + bj_index(IQ, JQ, b)];
        ZP[a][b] = zp[e];
        ZQ[a][b] = zq[e];
      }
      __syncthreads();
      for (int e = tid; e < BJ * BS; e += 256) {  // T = Z_P^T A, the rows of half hr
        const int a = BJ * hr + (e >> 5), b = e & 31;
        T[a][b] = zt_dot(ZP, a, A, b);
      }
      __syncthreads();
      const int a = BJ * hr + (tid >> 4), b = BJ * hc + (tid & 15);
      S[0][(side ? BJ : 0) + (tid >> 4)][(side ? 0 : BJ) + (tid & 15)] = xz_dot(T, a, ZQ, b);
    }
  }
  __syncthreads();
  // outer convergence: any off-diagonal entry above tol (1e-12, or the looser tolerance
  // of a coarse-phase Rayleigh-Ritz solve) of its diagonal scale
  const double tol = *tolp;
  double rmax = 0.0;  // the sweep's largest off-diagonal ratio (JacobiBig::solve's early check)
  for (int e = tid; e < BS * BS; e += 256) {
    const int a = e >> 5, b = e & 31;
    const double x = fabs(S[0][a][b]), sc = sqrt(fabs(S[0][a][a] * S[0][b][b]));
    if (a != b && x > tol * sc) any = 1;
    if (a != b && x > 0.0) rmax = fmax(rmax, sc > 0.0 ? x / sc : __builtin_huge_val());
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) rmax = fmax(rmax, __shfl_xor(rmax, off));
  if ((tid & 63) == 0 && rmax > 0.0) atomicMax(pmax, (unsigned long long)__double_as_longlong(rmax));
  __syncthreads();
  if (any && tid == 0) {
    *flag = 1;
    pmax[1] = 1ull;  // the sweep's flag beside its ratio: one host read per sweep
  }
  const int t = tid >> 4, u = tid & 15;
  int cur = 0;
  for (int sw = 0; sw < kInnerSweeps && any; ++sw) {
    __syncthreads();
    if (tid == 0) any = 0;
    for (int rr = 0; rr < BS - 1; ++rr) {
      // the round's 16 rotations, computed once (the fp64 sqrt/div chain is the round's latency)
      if (tid < BJ) {
        const Rot R = lds_rotation(S[cur], rr, tid);
        rot[tid] = R;
        if (R.on) any = 1;
      }
      __syncthreads();
      const Rot ra = rot[t], rb = rot[u];
      const double x00 = S[cur][ra.p][rb.p], x01 = S[cur][ra.p][rb.q];
      const double x10 = S[cur][ra.q][rb.p], x11 = S[cur][ra.q][rb.q];
      const double y00 = ra.c * x00 - ra.s * x10, y01 = ra.c * x01 - ra.s * x11;
      const double y10 = ra.s * x00 + ra.c * x10, y11 = ra.s * x01 + ra.c * x11;
      double z00 = rb.c * y00 - rb.s * y01, z01 = rb.s * y00 + rb.c * y01;
      double z10 = rb.c * y10 - rb.s * y11, z11 = rb.s * y10 + rb.c * y11;
      if (t == u && ra.on) {
        z01 = 0.0;
        z10 = 0.0;
      }
      S[cur ^ 1][ra.p][rb.p] = z00;
      S[cur ^ 1][ra.p][rb.q] = z01;
      S[cur ^ 1][ra.q][rb.p] = z10;
      S[cur ^ 1][ra.q][rb.q] = z11;
      // Z <- Z J_b: thread (t, u) updates rows 2t, 2t+1 of the pair u columns
      if (rb.on) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * t + h;
          const double zp = Z[i][rb.p], zq = Z[i][rb.q];
          Z[i][rb.p] = rb.c * zp - rb.s * zq;
          Z[i][rb.q] = rb.s * zp + rb.c * zq;
        }
      }
      cur ^= 1;
      __syncthreads();
    }
  }
  // the diagonalised pair block goes out as computed (rotated pivots exactly zero), so
  // rounding noise of a Z^T S Z product never re-triggers the convergence flag
  double* Zp = Zcur + (int64_t)pair * BS * BS;
  for (int e = tid; e < BS * BS; e += 256) {
    const int a = e >> 5, b = e & 31;
    Zp[e] = Z[a][b];
    Gnext[(int64_t)bj_index(I, J, a) * mp + bj_index(I, J, b)] = S[cur][a][b];
  }
}

// Apply of round rp: Gout[P][Q] = Z_P^T Gin[P][Q] Z_Q for pair q's columns and pair py's
// rows (py < npair; the pair's own block P = Q is the solve's), or V[R][Q] <- V[R][Q] Z_Q
// for the 32-row tile R = py - npair of V (in place: a tile is read completely before it
// is written).
__device__ __forceinline__ void bj_apply_part(const double* __restrict__ Gin, double* Gout, double* __restrict__ V,
                                              int mp, int rp, const double* __restrict__ Zall, int q, int py,
                                              Tile* sm) {
  const int nb = mp / BJ, npair = nb / 2;
  int IQ, JQ;
  bj_pair(rp, q, nb, &IQ, &JQ);
  Tile &A = sm[0], &T = sm[1], &ZP = sm[2], &ZQ = sm[3];
  const int tid = threadIdx.x;
  const bool isv = py >= npair;
  if (!isv && py == q) return;
  int IP = 0, JP = 0;
  if (!isv) bj_pair(rp, py, nb, &IP, &JP);
  const int64_t r0 = (int64_t)(py - npair) * BS;  // V row tile
  const double* zq = Zall + (int64_t)q * BS * BS;
  const double* zp = Zall + (int64_t)py * BS * BS;
  for (int e = tid; e < BS * BS; e += 256) {
    const int a = e >> 5, b = e & 31;
    const int64_t col = bj_index(IQ, JQ, b);
    A[a][b] = isv ? V[(r0 + a) * mp + col] : Gin[(int64_t)bj_index(IP, JP, a) * mp + col];
    ZQ[a][b] = zq[e];
    if (!isv) ZP[a][b] = zp[e];
  }
  __syncthreads();
  const int a0 = tid >> 5, b = tid & 31;  // thread: rows a0 + 8j, column b
  if (!isv) {  // T = Z_P^T A
#pragma unroll
    for (int j = 0; j < 4; ++j) T[a0 + 8 * j][b] = zt_dot(ZP, a0 + 8 * j, A, b);
    __syncthreads();
  }
  const Tile& X = isv ? A : T;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int a = a0 + 8 * j;
    const double v = xz_dot(X, a, ZQ, b);
    const int64_t col = bj_index(IQ, JQ, b);
    if (isv)
      V[(r0 + a) * mp + col] = v;
    else
      Gout[(int64_t)bj_index(IP, JP, a) * mp + col] = v;
  }
}

// One launch per round g of the block method: workgroups [0, nsolve) solve round r (the
// pairs of G^(g)), the others apply round rp's rotations (Zprev) to G^(g-1) -> the
// off-diagonal pair blocks of G^(g) in Gcur, and to V.  Neither half waits for the other:
// the solve recomputes the two off-diagonal blocks it needs (bj_solve_part), so a round
// costs one solve instead of a solve plus an apply, in one launch instead of two.  G^(g-1),
// G^(g), G^(g+1) rotate through three buffers (the apply still reads G^(g-1) while the
// solve writes G^(g+1)); Z ping-pongs.
__global__ __launch_bounds__(256) void bj_round_kernel(const double* __restrict__ Gprev, double* Gcur,
                                                       double* __restrict__ Gnext, double* __restrict__ V, int mp,
                                                       int r, int rp, int nsolve, const double* __restrict__ Zprev,
                                                       double* __restrict__ Zcur, int* __restrict__ flag,
                                                       const double* __restrict__ tolp,
                                                       unsigned long long* __restrict__ pmax) {
  __shared__ Tile sm[7];
  const int b = blockIdx.x;
  if (b < nsolve) {
    bj_solve_part(Gprev, Gcur, Gnext, mp, r, rp, Zprev, Zcur, flag, tolp, pmax, b, sm);
    return;
  }
  const int npair = mp / BS, a = b - nsolve;
  bj_apply_part(Gprev, Gcur, V, mp, rp, Zprev, a % npair, a / npair, sm);
}

__global__ void set_scalar_kernel(double* p, double v) { *p = v; }

// Early convergence test of the block method (JacobiBig::solve): *flag = 1 when any
// off-diagonal entry of the completed matrix G exceeds tol of its diagonal scale — the
// decision the next sweep's pair problems would take before rotating anything (they read
// these same entries), without running that sweep.  grid: one block per row.
__global__ void bj_check_kernel(const double* __restrict__ G, int m, int mp, const double* __restrict__ tolp,
                                unsigned long long* __restrict__ flag) {
  const int i = blockIdx.x;
  const double tol = *tolp, gii = G[(int64_t)i * mp + i];
  bool bad = false;
  for (int j = threadIdx.x; j < m; j += blockDim.x)
    if (j != i && fabs(G[(int64_t)i * mp + j]) > tol * sqrt(fabs(gii * G[(int64_t)j * mp + j]))) bad = true;
  if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1ull;
}

// G^(-1) = G^(0) = the symmetrised input in buffers 2 and 0, V = I, Z^(-1) = I: the first
// round's pending apply is an exact identity
__global__ void bj_init_kernel(const double* __restrict__ A, int m, int64_t lda, int mp, double* __restrict__ G0,
                               double* __restrict__ G2, double* __restrict__ V, double* __restrict__ Zid) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < (int64_t)(mp / BS) * BS * BS) {
    const int w = (int)(e % (BS * BS));
    Zid[e] = (w >> 5) == (w & 31) ? 1.0 : 0.0;
  }
  if (e >= (int64_t)mp * mp) return;
  const int i = (int)(e / mp), j = (int)(e - (e / mp) * mp);
  const double g = (i < m && j < m) ? 0.5 * (A[(int64_t)i * lda + j] + A[(int64_t)j * lda + i]) : 0.0;
  G0[e] = g;
  G2[e] = g;
  V[e] = i == j ? 1.0 : 0.0;
}

// descending order (ties -> lower index first); evecs[r][rank] = V[r][i]
__global__ void jbig_sort_kernel(const double* __restrict__ G, const double* __restrict__ V, int m, int mp,
                                 double* __restrict__ evals, double* __restrict__ evecs, int64_t ldv) {
  const int i = blockIdx.x;
  __shared__ int rank_s;
  const double li = G[(int64_t)i * mp + i];
  if (threadIdx.x == 0) rank_s = 0;
  __syncthreads();
  int cnt = 0;
  for (int j = threadIdx.x; j < m; j += blockDim.x) {
    const double lj = G[(int64_t)j * mp + j];
    cnt += (lj > li) || (lj == li && j < i);
  }
  atomicAdd(&rank_s, cnt);
  __syncthreads();
  const int rank = rank_s;
  if (threadIdx.x == 0) evals[rank] = li;
  for (int rr = threadIdx.x; rr < m; rr += blockDim.x) evecs[(int64_t)rr * ldv + rank] = V[(int64_t)rr * mp + i];
}

static int padded_order(int m) { return m >= kBlockJacobiMin ? (m + 2 * BJ - 1) / (2 * BJ) * (2 * BJ) : m + (m & 1); }

size_t jacobi_big_work_elems(int m) {
  const int64_t mp = padded_order(m);
  // scalar: G ping-pong + V; block: G^(g-1), G^(g), G^(g+1), V, two sets of pair rotations
  return (size_t)(4 * mp * mp + 4 * BJ * mp) + 64;  // + the tolerance scalar
}

static inline int mod_pos(int x, int n) { return ((x % n) + n) % n; }

void JacobiBig::destroy() {
  for (auto& g : exec) {
    if (g) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(g));
    g = nullptr;
  }
}

// Graphs: one sweep per graph.  Scalar path: two graphs for the two ping-pong parities.
// Block path: one graph per phase (first global round of the sweep) mod 6 — the three G
// buffers and the two Z buffers cycle with the global round count.
hipError_t JacobiBig::init(int m_, double* work_, int* flag_, hipStream_t capture) {
  destroy();
  m = m_;
  mp = padded_order(m);
  block = m >= kBlockJacobiMin;
  fused = true;
#ifdef EF_DIAGNOSTICS  // EF_BJ_FUSED=0: the solve and the apply of a round as two launches (A/B)
  if (const char* e = getenv("EF_BJ_FUSED")) fused = atoi(e) != 0;
#endif
  work = work_;
  flag = flag_;
  const int64_t mm = (int64_t)mp * mp;
  const int R = rounds();
  auto capture_graph = [&](int slot, auto&& body) -> hipError_t {
    hipError_t e = hipStreamBeginCapture(capture, hipStreamCaptureModeRelaxed);
    if (e != hipSuccess) return e;
    (void)hipMemsetAsync(flag, 0, sizeof(int), capture);
    if (block) (void)hipMemsetAsync(pmax_slot(), 0, 2 * sizeof(unsigned long long), capture);
    body();
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(capture, &g);
    if (e != hipSuccess) return e;
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return e;
    exec[slot] = x;
    return hipSuccess;
  };
  if (!block) {
    double* G[2] = {work, work + mm};
    double* V = work + 2 * mm;
    const int np = mp / 2;
    const int64_t threads = (int64_t)np * np + (int64_t)mp * np;
    const dim3 grid((unsigned)((threads + 255) / 256));
    for (int par = 0; par < 2; ++par) {
      hipError_t e = capture_graph(par, [&] {
        int cur = par;
        for (int r = 0; r < R; ++r) {
          hipLaunchKernelGGL(jbig_round_kernel, grid, dim3(256), 0, capture, G[cur], G[cur ^ 1], V, mp, r, flag);
          cur ^= 1;
        }
      });
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  double* G[3] = {work, work + mm, work + 2 * mm};
  double* V = work + 3 * mm;
  double* Z[2] = {work + 4 * mm, work + 4 * mm + (int64_t)BS * mp};
  double* tolv = work + 4 * mm + 2 * (int64_t)BS * mp;  // the solve's tolerance (set per solve)
  const int npair = mp / BS;
  const unsigned napply = (unsigned)(npair * (npair + mp / BS));
  if (!fused) {
    for (int par = 0; par < 2; ++par) {
      hipError_t e = capture_graph(par, [&] {
        int cur = par;
        for (int r = 0; r < R; ++r) {
          hipLaunchKernelGGL(bj_round_kernel, dim3((unsigned)npair), dim3(256), 0, capture, G[cur], G[cur],
                             G[cur ^ 1], V, mp, r, r, npair, nullptr, Z[0], flag, tolv, pmax_slot());
          hipLaunchKernelGGL(bj_round_kernel, dim3(napply), dim3(256), 0, capture, G[cur], G[cur ^ 1], G[cur ^ 1],
                             V, mp, r, r, 0, Z[0], Z[1], flag, tolv, pmax_slot());
          cur ^= 1;
        }
      });
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  for (int k = 0; k < 6; ++k) {
    const int ph = (k * R) % 6;
    if (exec[ph]) continue;
    hipError_t e = capture_graph(ph, [&] {
      for (int r = 0; r < R; ++r) {
        const int g = ph + r;
        hipLaunchKernelGGL(bj_round_kernel, dim3((unsigned)npair + napply), dim3(256), 0, capture,
                           G[mod_pos(g - 1, 3)], G[g % 3], G[(g + 1) % 3], V, mp, r, r == 0 ? R - 1 : r - 1, npair,
                           Z[mod_pos(g - 1, 2)], Z[g % 2], flag, tolv, pmax_slot());
      }
    });
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int JacobiBig::solve(hipStream_t s, const double* A, int64_t lda, double* evals, double* evecs, int64_t ldv,
                     int max_sweeps, int* sweeps_out, hipError_t* err, double tol) {
  const int64_t mm = (int64_t)mp * mp;
  const int R = rounds();
  double* G[3] = {work, work + mm, work + 2 * mm};
  double* V = work + (block ? 3 : 2) * mm;
  double* Z[2] = {work + 4 * mm, work + 4 * mm + (int64_t)BS * mp};
  double* tolv = work + 4 * mm + 2 * (int64_t)BS * mp;
  if (block) hipLaunchKernelGGL(set_scalar_kernel, dim3(1), dim3(1), 0, s, tolv, tol);
  if (block)
    hipLaunchKernelGGL(bj_init_kernel, dim3((unsigned)((mm + 255) / 256)), dim3(256), 0, s, A, m, lda, mp, G[0], G[2],
                       V, Z[1]);
  else
    hipLaunchKernelGGL(jbig_init_kernel, dim3((unsigned)((mm + 255) / 256)), dim3(256), 0, s, A, m, lda, mp, G[0], V);
  const bool three = block && fused;
  int cur = 0, sweep = 0;  // cur: the ping-pong parity, or (three buffers) the global round count
  bool converged = false;
  for (; sweep < max_sweeps; ++sweep) {
    *err = hipGraphLaunch(static_cast<hipGraphExec_t>(exec[three ? cur % 6 : cur]), s);
    if (*err != hipSuccess) return -1;
    cur = three ? cur + R : cur ^ (R & 1);  // an odd number of rounds swaps the ping-pong buffers
    int hflag = 0;
    unsigned long long hreg[2] = {0, 0};  // block path: {largest ratio (double bits), flag}
    if (block) {
      *err = hipMemcpyAsync(hreg, pmax_slot(), sizeof(hreg), hipMemcpyDeviceToHost, s);
    } else {
      *err = hipMemcpyAsync(&hflag, flag, sizeof(int), hipMemcpyDeviceToHost, s);
    }
    if (*err == hipSuccess) *err = hipStreamSynchronize(s);
    if (*err != hipSuccess) return -1;
    if (block) hflag = hreg[1] != 0;
    const unsigned long long hmax = hreg[0];
    if (hflag == 0) {
      converged = true;
      break;
    }
    // Early exit (round 5): Jacobi converges quadratically, so when the largest off-diagonal
    // ratio this sweep rotated away was below sqrt(tol) / 4, the next sweep is very likely
    // the confirming one that rotates nothing (~15 rounds of pair solves).  Complete G with
    // the pending apply of the last round (G tiles only: idempotent, the next round would
    // write the same values; V is left to the final apply), test every off-diagonal entry
    // as that sweep's pair problems would, and stop when none exceeds tol.  When the test
    // passes the result is bit-identical to running the confirming sweep (whose rotations
    // are all the identity); when it fails the next sweep runs as before.
    double dmax;
    memcpy(&dmax, &hmax, sizeof dmax);
    if (EF_BJ_EARLY && three && dmax > 0.0 && dmax < 0.25 * std::sqrt(tol)) {
      const int npair = mp / BS, gl = cur - 1;
      *err = hipMemsetAsync(pmax_slot() + 1, 0, sizeof(unsigned long long), s);
      if (*err != hipSuccess) return -1;
      hipLaunchKernelGGL(bj_round_kernel, dim3((unsigned)(npair * npair)), dim3(256), 0, s, G[gl % 3], G[cur % 3],
                         G[cur % 3], V, mp, 0, R - 1, 0, Z[gl % 2], Z[cur % 2], flag, tolv, pmax_slot());
      hipLaunchKernelGGL(bj_check_kernel, dim3((unsigned)m), dim3(256), 0, s, G[cur % 3], m, mp, tolv,
                         pmax_slot() + 1);
      *err = hipMemcpyAsync(hreg, pmax_slot(), sizeof(hreg), hipMemcpyDeviceToHost, s);
      if (*err == hipSuccess) *err = hipStreamSynchronize(s);
      if (*err != hipSuccess) return -1;
      if (hreg[1] == 0) {
        converged = true;
        ++sweep;  // the confirming sweep this test replaced
        break;
      }
    }
  }
  const double* Gfinal = G[cur];
  if (three) {
    // the last round's rotations still go to V (and to G's off-diagonal blocks)
    const int npair = mp / BS, gl = cur - 1;
    hipLaunchKernelGGL(bj_round_kernel, dim3((unsigned)(npair * (npair + mp / BS))), dim3(256), 0, s, G[gl % 3],
                       G[cur % 3], G[cur % 3], V, mp, 0, R - 1, 0, Z[gl % 2], Z[cur % 2], flag, tolv, pmax_slot());
    Gfinal = G[cur % 3];
  }
  hipLaunchKernelGGL(jbig_sort_kernel, dim3((unsigned)m), dim3(256), 0, s, Gfinal, V, m, mp, evals, evecs, ldv);
  *err = hipGetLastError();
  if (*err != hipSuccess) return -1;
  if (sweeps_out) *sweeps_out = sweep + 1;
  return converged ? 0 : 1;
}

}  // namespace ef
