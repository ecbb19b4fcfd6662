// Training projection F = ((X - mu) * w) . E on the int8 matrix cores (fit K5, the
// projected_data of useless/train.py:122 / face_features of train-v4.py:134, n x k).
//
// X is uint8, so X' = X - 128 is exact int8, and
//     F = X' . E'' + 1 . c^T,   E'' = diag(w) E,   c = (128 - mu)^T E''
// (c in fp64 by cc_kernel).  E'' is fp64; per output column it is scaled by 2^t_c so its
// largest entry is ~2^54 and rounded to an integer V (relative error <= 2^-54, i.e. fp64
// precision), which is written as P = 7 signed base-256 digits, V = sum_j 256^j D_j with
// D_j in [-128, 127].  Each X' . D_j is an exact int32 (|.| <= d * 2^14 <= 2^30 for
// d <= 65536), so the only roundings are the quantisation of E'' and the fp64 Horner
// combine 2^-t_c sum_j 256^j I_j (proj_combine_kernel) — the same order of error as the
// fp64 GEMM it replaces (reference: useless/train.py:122 in float64).
//
// proj_i8_kernel<TN>: C[n][N] (int32) = X' . D^T with D = [N = P * kk padded to TN][d] int8
// (K-contiguous).  Workgroup tile 256 rows x TN digit-columns, 8 waves (TN = 128: 4 x 2 of
// 64 x 64; TN = 256: 2 x 4 of 128 x 64), K stages of 64 bytes staged by LDS-DMA into a
// 4-stage ring (same 64-B row swizzle as the covariance kernel); A fragments are flipped to
// int8 (x ^ 0x80) in registers.  The N-tiles of one row block are consecutive on one XCD,
// so X is read from HBM about once.  A stage streams (256 + TN) x 64 B from L2 for
// 256 x TN x 64 MACs: 48 B per MFMA-clock of a CU at TN = 128, 32 at TN = 256 — the L2 -> LDS
// stream (~30 B/clk per CU, K3) is the limit, so 7 digits x kk = 128 run as 4 tiles of 256
// (14 % padding) rather than 7 of 128.
// Requires d % 64 == 0 (X rows are DMA'd 64 bytes at a time; otherwise the caller keeps
// the fp64 GEMM).
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "ef_dma.hpp"
#include "ef_linalg.hpp"

namespace ef {

namespace {

typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int PM = 256;           // rows per tile
constexpr int PK = 64;            // K bytes per stage
constexpr int PNB = 4;            // LDS ring stages
constexpr int kDigits = 7;        // base-256 digits of the scaled eigenvector entries
constexpr int kTopBit = 54;       // largest scaled entry ~ 2^54

// t_c: 2^t_c * max_r |w_r E[r][c]| lies in [2^(TOP-1), 2^TOP); zero columns get t_c = 0.
template <int TOP = kTopBit>
__global__ void digit_scale_kernel(const double* __restrict__ E, const double* __restrict__ w, int64_t d, int kk,
                                   int* __restrict__ tsh) {
  const int c = blockIdx.x;
  double m = 0.0;
  for (int64_t r = threadIdx.x; r < d; r += blockDim.x) m = fmax(m, fabs((w ? w[r] : 1.0) * E[r * kk + c]));
  __shared__ double red[256];
  red[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int e = 0;
    if (red[0] > 0.0) (void)frexp(red[0], &e);  // red[0] in [2^(e-1), 2^e)
    tsh[c] = red[0] > 0.0 ? TOP - e : 0;
  }
}

// D[(j * kk + c) * d + r] = digit j of rint(w_r E[r][c] 2^t_c); rows kk * P .. Npad are zero.
template <int ND = kDigits>
__global__ void digits_kernel(const double* __restrict__ E, const double* __restrict__ w, int64_t d, int kk,
                              const int* __restrict__ tsh, int8_t* __restrict__ D) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d * kk) return;
  const int64_t r = e / kk;
  const int c = (int)(e - r * kk);
  long long v = (long long)rint(ldexp((w ? w[r] : 1.0) * E[r * kk + c], tsh[c]));
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const long long lo = ((v + 128) & 255) - 128;  // signed low byte
    D[((int64_t)j * kk + c) * d + r] = (int8_t)lo;
    v = (v - lo) / 256;
  }
}

// c[col] = sum_r (128 - mu_r) w_r E[r][col]  (fp64, one block per column)
__global__ void cc_kernel(const double* __restrict__ E, const double* __restrict__ w, const double* __restrict__ mu,
                          int64_t d, int kk, double* __restrict__ cc) {
  const int c = blockIdx.x;
  double s = 0.0;
  for (int64_t r = threadIdx.x; r < d; r += blockDim.x) s += (128.0 - mu[r]) * (w ? w[r] : 1.0) * E[r * kk + c];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) cc[c] = red[0];
}

#ifndef EF_PROJ_LO  // DMA issue position (0 = after the barrier, n = after row block n - 1)
#define EF_PROJ_LO 1   // of waves 0-3 and 4-7 (the covariance SYRK's measured best)
#endif
#ifndef EF_PROJ_HI
#define EF_PROJ_HI 3
#endif
// Digit pairs of the fit's int8-digit product (launch_cq_i8): plane a of C's row digits
// against digit b of Q's column digits for every a + b >= kOzDigits - 1, a descending (the
// pairs of one plane consecutive, so they run together and share its rows in L2).
constexpr int kOzDigits = 6;   // base-256 digits per operand (largest scaled entry < 2^46)
constexpr int kOzTop = 46;
constexpr int kOzPairs = kOzDigits * (kOzDigits + 1) / 2;
// Work items per row block: the first kOzPairs - 1 pairs whole, the last pair (0, 5) in
// kOzSplit K-parts (its own output blocks), so a launch of 64 row blocks is 5.25 rounds of
// whole items on 256 CUs, not 6 (21 x 64 = 1344 = 5.25 x 256; the quarter items fill the
// last round); blocks: kOzPairs - 1 + kOzSplit.
constexpr int kOzSplit = 4;
constexpr int kOzItems = kOzPairs - 1 + kOzSplit;
constexpr int kOzBlocks = kOzItems;
__device__ __forceinline__ void oz_pair(int p, int& a, int& b) {
  a = kOzDigits - 1;
  int base = 0;
  while (p >= base + a + 1) {
    base += a + 1;
    --a;
  }
  b = kOzDigits - 1 - a + (p - base);
}

// OZ: the work item is (row block, digit pair p = (a, b)); X holds kOzDigits planes of
// n x d biased digits (digit + 128), D digit b's TN rows, C the pair's own n x ldc block.
template <int TN, bool OZ = false>
__global__ __launch_bounds__(512, 1) void proj_i8_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d,
                                                         const int8_t* __restrict__ D, int ntn, int nblocks,
                                                         int* __restrict__ C, int64_t ldc) {
  constexpr int WN = TN / 64, WM = 8 / WN;      // wave grid; a wave owns (PM / WM) x 64
  constexpr int IA = PM / WM / 32, JB = 2;      // 32 x 32 blocks per wave
  constexpr int BPW = TN / 128;                 // B pieces per wave per stage (A: 2)
  constexpr int PSTAGE = (PM + TN) * PK;        // bytes per stage: A panel, then B panel
  __shared__ __attribute__((aligned(16))) uint8_t smem[PNB * PSTAGE];
  const int total = gridDim.x;  // multiple of 8; trailing blocks are idle padding
  // blocks b and b+8 share an XCD: XCD x runs items [x*total/8, (x+1)*total/8), row-block
  // major, so the N-tiles of a row block run together and share its X rows in L2
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  if (lin >= nblocks) return;
  int mt, nt;
  int64_t c0 = 0;  // OZ: output columns are the pair block's own
  int64_t s0 = 0, nst = d / PK;  // K stages of the item
  if constexpr (OZ) {
    // per XCD (ntn = row blocks per XCD): its row blocks' whole pairs, then the split parts
    const int per = total >> 3, x = lin / per, r = lin - x * per;
    int p, blk;
    if (r < ntn * (kOzPairs - 1)) {
      mt = x * ntn + r / (kOzPairs - 1);
      p = r % (kOzPairs - 1);
      blk = p;
    } else {
      const int r2 = r - ntn * (kOzPairs - 1);
      mt = x * ntn + r2 / kOzSplit;
      const int part = r2 % kOzSplit;
      p = kOzPairs - 1;
      blk = p + part;
      const int64_t all = nst;
      s0 = all * part / kOzSplit;
      nst = all * (part + 1) / kOzSplit - s0;
    }
    int a, b;
    oz_pair(p, a, b);
    nt = b;
    X += (int64_t)a * n * d;
    C += (int64_t)blk * n * ldc;
    c0 = (int64_t)b * TN;
  } else {
    mt = lin / ntn;
    nt = lin - mt * ntn;
  }
  const int64_t m0 = (int64_t)mt * PM, n0 = (int64_t)nt * TN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, c32 = lane & 31;
  const int wm = wave / WN, wn = wave % WN;

  // DMA: a stage = 16 A pieces + TN / 16 B pieces of 1 KiB (16 rows x 64 B); wave w issues
  // A pieces 2w, 2w+1 and B pieces BPW w .. BPW w + BPW - 1.  Lane l -> row 16j + (l >> 2),
  // physical chunk l & 3 holding logical chunk (l & 3) ^ ((l >> 4) & 3).
  const unsigned lds_base = lds_addr(smem);
  const int lrow = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lane >> 4) & 3);
  // A rows are d bytes apart (X row-major): 64-bit per-lane row base, stage offset added
  const uint8_t* arow[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    int64_t ra = m0 + (wave * 2 + jj) * 16 + lrow;
    ra = ra < n ? ra : n - 1;
    arow[jj] = X + ra * d + s0 * PK + lchunk * 16;
  }
  // D is N x d (< 4 GiB)
  const unsigned voffB = (unsigned)((n0 + wave * BPW * 16 + lrow) * d + s0 * PK + lchunk * 16);
  auto issue = [&](int64_t st, int buf) {
    const unsigned sbuf = lds_base + (unsigned)(buf * PSTAGE);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) glds16(arow[jj] + st * PK, sbuf + (unsigned)((wave * 2 + jj) * 1024));
#pragma unroll
    for (int q = 0; q < BPW; ++q)
      glds16s(voffB + (unsigned)(q * 16 * d + st * PK), (unsigned long long)(size_t)D,
              sbuf + (unsigned)(PM * PK + (wave * BPW + q) * 1024));
  };

  i32x16 acc[IA][JB];
#pragma unroll
  for (int i = 0; i < IA; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[i][j] = i32x16{};

  const int sw = (c32 >> 2) & 3;
  const i32x4 flip = {(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
  // lane (r, h) holds A[r][32s + 16h + j], B[32s + 16h + j][r] for k-step s of a stage
  const unsigned offa[2] = {(unsigned)((wm * (PM / WM) + c32) * PK + ((h ^ sw) * 16)),
                            (unsigned)((wm * (PM / WM) + c32) * PK + (((2 + h) ^ sw) * 16))};
  const unsigned offb[2] = {(unsigned)(PM * PK + (wn * 64 + c32) * PK + ((h ^ sw) * 16)),
                            (unsigned)(PM * PK + (wn * 64 + c32) * PK + (((2 + h) ^ sw) * 16))};
  auto fa = [&](const uint8_t* sa, int ks, int i) {
    return *reinterpret_cast<const i32x4*>(sa + offa[ks] + i * 32 * PK) ^ flip;
  };
  auto fb = [&](const uint8_t* sa, int ks, i32x4 (&bb)[JB]) {
#pragma unroll
    for (int j = 0; j < JB; ++j) bb[j] = *reinterpret_cast<const i32x4*>(sa + offb[ks] + j * 32 * PK);
  };
  // one k-step's MFMAs, row block by row block; each A fragment is refilled with the next
  // k-step's as soon as its row block's MFMAs are issued
  auto mma = [&](i32x4 (&a)[IA], const i32x4 (&bb)[JB], const uint8_t* nsa, int ns, auto&& mid) {
#pragma unroll
    for (int i = 0; i < IA; ++i) {
#pragma unroll
      for (int j = 0; j < JB; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], bb[j], acc[i][j], 0, 0, 0);
      a[i] = fa(nsa, ns, i);
      mid(i + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto none = [](int) {};
  // Ring of PNB stages, 2 + BPW DMA instructions per wave per stage: "stage t landed" is
  // vmcnt <= (2 + BPW) x (stages issued after it); tail stages re-read stage 0 so the count
  // stays uniform.  As in the covariance SYRK (ef_cov_i8.hip), the one barrier per stage
  // sits between its two k-steps (stage st+1 published, stage st's slot retired), so the
  // next stage's first fragments are read, and the DMA into the retired slot issued, while
  // the second k-step's MFMAs still run.
  constexpr int Q = 2 + BPW;
  for (int j = 0; j < PNB; ++j) issue(j < nst ? j : 0, j);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Q * (PNB - 1)) : "memory");  // stage 0 landed
  __syncthreads();
  i32x4 a[IA], b0[JB], b1[JB];
#pragma unroll
  for (int i = 0; i < IA; ++i) a[i] = fa(smem, 0, i);
  fb(smem, 0, b0);
  for (int64_t st = 0; st < nst; ++st) {
    const uint8_t* cur = smem + (st % PNB) * PSTAGE;
    fb(cur, 1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a, b0, cur, 1, none);  // k-step 0; A refilled with k-step 1
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Q * (PNB - 2)) : "memory");  // stage st+1 landed
    __syncthreads();  // every wave done reading stage st; stage st+1 visible
    const int64_t nx = st + PNB;
    // the DMA into stage st's slot, at this wave's position of k-step 1 (the SYRK's stagger:
    // the two waves of a SIMD do not pay the pieces' issue cost at the same time)
    // (positions past the wave's last row block — IA is 2 for the TN = 128 tiles — clamp to it:
    // every wave must issue its Q pieces each stage, or the vmcnt accounting breaks)
    const int dpos = (wave < 4 ? EF_PROJ_LO : EF_PROJ_HI) < IA ? (wave < 4 ? EF_PROJ_LO : EF_PROJ_HI) : IA;
    auto at_pos = [&](int pos) {
      if (pos == dpos) issue(nx < nst ? nx : 0, (int)(nx % PNB));
    };
    at_pos(0);
    // (after the last stage these read a slot holding a re-read of the first stage:
    // harmless, unused, and branch-free)
    const uint8_t* nxt = smem + ((st + 1) % PNB) * PSTAGE;
    fb(nxt, 0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mma(a, b1, nxt, 0, at_pos);  // k-step 1; A refilled with the next stage's k-step 0
  }
  dma_wait_all();
#pragma unroll
  for (int i = 0; i < IA; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int64_t col = n0 - c0 + wn * 64 + j * 32 + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (PM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < n) C[row * ldc + col] = acc[i][j][r];
      }
    }
}

// F[i][c] = 2^-t_c sum_j 256^j I[i][j kk + c] + cc[c]   (fp64 Horner)
__global__ void proj_combine_kernel(const int* __restrict__ I, int64_t n, int kk, int64_t ldi,
                                    const int* __restrict__ tsh, const double* __restrict__ cc,
                                    double* __restrict__ F) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * kk) return;
  const int64_t i = e / kk;
  const int c = (int)(e - i * kk);
  const int* row = I + i * ldi + c;
  double v = (double)row[(int64_t)(kDigits - 1) * kk];
#pragma unroll
  for (int j = kDigits - 2; j >= 0; --j) v = fma(v, 256.0, (double)row[(int64_t)j * kk]);
  F[e] = ldexp(v, -tsh[c]) + cc[c];
}

// Row digits of the fit's covariance (launch_cq_i8_planes): one block per row i of the
// symmetric C, t_i such that 2^t_i max_k |C[i][k]| lies in [2^45, 2^46), and plane a
// (a = 0 least significant) of V = rint(2^t_i C[i][k]) written biased (digit + 128: the
// GEMM's A fragments flip it back to int8).  8 columns per thread and step.
__global__ __launch_bounds__(256) void oz_rows_kernel(const double* __restrict__ C, int64_t dim,
                                                      uint8_t* __restrict__ P, int* __restrict__ tr) {
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
  const int64_t plane = dim * dim;
  for (int64_t k0 = (int64_t)threadIdx.x * 8; k0 < dim; k0 += 256 * 8) {
    unsigned lo4[kOzDigits], hi4[kOzDigits];
#pragma unroll
    for (int a = 0; a < kOzDigits; ++a) lo4[a] = hi4[a] = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      long long v = (long long)rint(ldexp(row[k0 + q], t));
#pragma unroll
      for (int a = 0; a < kOzDigits; ++a) {
        const long long lo = ((v + 128) & 255) - 128;
        const unsigned byte = (unsigned)(lo + 128) << (8 * (q & 3));
        if (q < 4) lo4[a] |= byte;
        else hi4[a] |= byte;
        v = (v - lo) / 256;
      }
    }
#pragma unroll
    for (int a = 0; a < kOzDigits; ++a)
      *reinterpret_cast<uint2*>(P + a * plane + i * dim + k0) = make_uint2(lo4[a], hi4[a]);
  }
}

// Column maxima of Q (dim x m, m = 256 = blockDim): block b folds rows [b dim / G,
// (b + 1) dim / G) and merges by atomicMax on the bits (non-negative doubles order as
// their bit patterns); cmax zeroed before.
__global__ __launch_bounds__(256) void oz_colmax_kernel(const double* __restrict__ Q, int64_t dim, int m,
                                                        unsigned long long* __restrict__ cmax) {
  const int c = threadIdx.x;
  const int64_t r0 = dim * blockIdx.x / gridDim.x, r1 = dim * (blockIdx.x + 1) / gridDim.x;
  double mx = 0.0;
  for (int64_t r = r0; r < r1; ++r) mx = fmax(mx, fabs(Q[r * m + c]));
  atomicMax(cmax + c, (unsigned long long)__double_as_longlong(mx));
}
// Q's column digits, K-contiguous: D[(j m + c) dim + r] = digit j of rint(2^u_c Q[r][c]),
// u_c from the column maximum ([2^45, 2^46)).  Thread (c, 16-row group): reads Q[r][c]
// coalesced along c, writes 16 digits of each plane as one 16-byte store.
__global__ __launch_bounds__(256) void oz_qdigits_kernel(const double* __restrict__ Q, int64_t dim, int m,
                                                         const unsigned long long* __restrict__ cmax,
                                                         int8_t* __restrict__ D, int* __restrict__ tc) {
  const int c = threadIdx.x;  // m = 256
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  const double mx = __longlong_as_double((long long)cmax[c]);
  int e = 0;
  if (mx > 0.0) (void)frexp(mx, &e);
  const int t = mx > 0.0 ? kOzTop - e : 0;
  if (blockIdx.x == 0) tc[c] = t;
  unsigned w[kOzDigits][4];
#pragma unroll
  for (int j = 0; j < kOzDigits; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) w[j][q] = 0u;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    long long v = (long long)rint(ldexp(Q[(r0 + q) * m + c], t));
#pragma unroll
    for (int j = 0; j < kOzDigits; ++j) {
      const long long lo = ((v + 128) & 255) - 128;
      w[j][q >> 2] |= (unsigned)(lo & 255) << (8 * (q & 3));
      v = (v - lo) / 256;
    }
  }
#pragma unroll
  for (int j = 0; j < kOzDigits; ++j)
    *reinterpret_cast<uint4*>(D + ((int64_t)j * m + c) * dim + r0) = make_uint4(w[j][0], w[j][1], w[j][2], w[j][3]);
}

// Y[i][c] = 2^(40 - t_i - u_c) sum_{L=0..5} 256^L S_L - sigma Q[i][c], S_L the exact int64
// sum of the pair products of level a + b = L + 5 (fp64 Horner from the top level)
__global__ __launch_bounds__(256) void oz_combine_kernel(const int* __restrict__ I, int64_t dim, int m,
                                                         const int* __restrict__ tr, const int* __restrict__ tc,
                                                         const double* __restrict__ Q, double sigma,
                                                         double* __restrict__ Y) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = dim * m;
  if (e >= total) return;
  const int64_t i = e / m;
  const int c = (int)(e - i * m);
  long long S[kOzDigits];
#pragma unroll
  for (int L = 0; L < kOzDigits; ++L) S[L] = 0;
  int p = 0;
#pragma unroll
  for (int a = kOzDigits - 1; a >= 1; --a)
#pragma unroll
    for (int b = kOzDigits - 1 - a; b < kOzDigits; ++b, ++p) S[a + b - (kOzDigits - 1)] += I[(int64_t)p * total + e];
#pragma unroll
  for (int q = 0; q < kOzSplit; ++q) S[0] += I[(int64_t)(p + q) * total + e];  // pair (0, 5) by K-parts
  double v = (double)S[kOzDigits - 1];
#pragma unroll
  for (int L = kOzDigits - 2; L >= 0; --L) v = fma(v, 256.0, (double)S[L]);
  Y[e] = fma(-sigma, Q[e], ldexp(v, 8 * (kOzDigits - 1) - tr[i] - tc[c]));
}

}  // namespace

// ---- the fit's fp64 products C.Q on the int8 matrix cores (Ozaki-style digit splitting)
// C (symmetric, dim x dim) is scaled per row and Q (dim x 256) per column to integers
// below 2^46 and cut into 6 signed base-256 digits each; every pair of digit planes whose
// weight 256^(a+b) is within 2^-40 of the top (a + b >= 5: 21 of 36) is an exact int32
// product (|.| <= dim 2^14) on proj_i8_kernel's tiles, and the fp64 combine adds them by
// level.  Error: the two 2^-46 roundings plus the dropped levels (<= 15 x 2^-46 of
// rowmax x colmax x dim worst case), the order of an fp64 GEMM's dim x 2^-53.  The row
// planes are built once per fit (C does not change); Q's digits every product.
// (dim: whole 256-row blocks, a multiple of 8 of them — the per-XCD item order — and
// K-parts of whole 64-byte stages)
bool cq_i8_supported(int64_t dim, int m) { return m == 256 && dim % (8 * PM) == 0 && dim <= 32768; }
size_t cq_i8_plane_bytes(int64_t dim) { return (size_t)kOzDigits * dim * dim + (size_t)dim * sizeof(int); }
static size_t cq_off_d(int64_t dim, int m) { return (size_t)kOzBlocks * dim * m * sizeof(int); }
static size_t cq_off_t(int64_t dim, int m) { return cq_off_d(dim, m) + (size_t)kOzDigits * m * dim; }
size_t cq_i8_work_bytes(int64_t dim, int m) { return cq_off_t(dim, m) + (size_t)m * (sizeof(int) + 8); }
hipError_t launch_cq_i8_planes(hipStream_t s, const double* C, int64_t dim, void* planes) {
  uint8_t* P = static_cast<uint8_t*>(planes);
  int* tr = reinterpret_cast<int*>(P + (size_t)kOzDigits * dim * dim);
  hipLaunchKernelGGL(oz_rows_kernel, dim3((unsigned)dim), dim3(256), 0, s, C, dim, P, tr);
  return hipGetLastError();
}
hipError_t launch_cq_i8(hipStream_t s, const void* planes, int64_t dim, const double* Q, int m, double sigma,
                        void* work, double* Y) {
  if (!cq_i8_supported(dim, m)) return hipErrorInvalidValue;
  const uint8_t* P = static_cast<const uint8_t*>(planes);
  const int* tr = reinterpret_cast<const int*>(P + (size_t)kOzDigits * dim * dim);
  uint8_t* base = static_cast<uint8_t*>(work);
  int* I = reinterpret_cast<int*>(base);
  int8_t* D = reinterpret_cast<int8_t*>(base + cq_off_d(dim, m));
  int* tc = reinterpret_cast<int*>(base + cq_off_t(dim, m));
  unsigned long long* cmax = reinterpret_cast<unsigned long long*>(base + cq_off_t(dim, m) + (size_t)m * sizeof(int));
  hipError_t e = hipMemsetAsync(cmax, 0, (size_t)m * 8, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(oz_colmax_kernel, dim3((unsigned)(dim / 16)), dim3(256), 0, s, Q, dim, m, cmax);
  hipLaunchKernelGGL(oz_qdigits_kernel, dim3((unsigned)(dim / 16)), dim3(256), 0, s, Q, dim, m, cmax, D, tc);
  const int nrb = (int)(dim / PM);
  const int nblocks = nrb * kOzItems;  // a multiple of 8 (cq_i8_supported)
  hipLaunchKernelGGL((proj_i8_kernel<256, true>), dim3((unsigned)nblocks), dim3(512), 0, s,
                     reinterpret_cast<const uint8_t*>(P), dim, dim, D, nrb / 8, nblocks, I, (int64_t)m);
  hipLaunchKernelGGL(oz_combine_kernel, dim3((unsigned)((dim * m + 255) / 256)), dim3(256), 0, s, I, dim, m, tr, tc,
                     Q, sigma, Y);
  return hipGetLastError();
}

struct ProjLayout {
  int64_t np, off_i, off_t, off_c, bytes;
  int tn;  // digit-columns per tile (128 or 256)
};
static ProjLayout proj_layout(int64_t n, int64_t d, int kk) {
  auto a256 = [](int64_t v) { return (v + 255) / 256 * 256; };
  ProjLayout L;
  // 256-column tiles (two thirds of the L2 -> LDS bytes per MAC) unless they pad the digit
  // columns by > 15 % more than 128-column tiles do
  const int64_t p = (int64_t)kDigits * kk, n128 = (p + 127) / 128 * 128, n256 = (p + 255) / 256 * 256;
  L.tn = n256 * 100 <= n128 * 115 ? 256 : 128;
#ifdef EF_DIAGNOSTICS
  if (const char* e = getenv("EF_PROJ_TN")) L.tn = atoi(e) == 256 ? 256 : 128;
#endif
  L.np = L.tn == 256 ? n256 : n128;
  L.off_i = a256(L.np * d);
  L.off_t = L.off_i + a256(n * L.np * (int64_t)sizeof(int));
  L.off_c = L.off_t + a256((int64_t)kk * sizeof(int));
  L.bytes = L.off_c + (int64_t)kk * sizeof(double);
  return L;
}

bool proj_i8_supported(const uint8_t* X, int64_t n, int64_t d, int kk) {
  return ((size_t)X & 15) == 0 && n >= 1 && d >= PK && d % PK == 0 && d <= 65536 && kk >= 1 &&
         proj_layout(n, d, kk).np * d < ((int64_t)1 << 32);
}

size_t proj_i8_work_bytes(int64_t n, int64_t d, int kk) { return (size_t)proj_layout(n, d, kk).bytes; }

hipError_t launch_proj_i8(hipStream_t s, const uint8_t* X, int64_t n, int64_t d, const double* mu, const double* w,
                          const double* E, int kk, void* work, double* F) {
  const ProjLayout L = proj_layout(n, d, kk);
  const int64_t np = L.np;
  uint8_t* base = static_cast<uint8_t*>(work);
  int8_t* D = reinterpret_cast<int8_t*>(base);
  int* I = reinterpret_cast<int*>(base + L.off_i);
  int* tsh = reinterpret_cast<int*>(base + L.off_t);
  double* cc = reinterpret_cast<double*>(base + L.off_c);
  hipError_t e = hipMemsetAsync(D, 0, (size_t)(np * d), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(digit_scale_kernel<>, dim3((unsigned)kk), dim3(256), 0, s, E, w, d, kk, tsh);
  hipLaunchKernelGGL(digits_kernel<>, dim3((unsigned)((d * kk + 255) / 256)), dim3(256), 0, s, E, w, d, kk, tsh, D);
  hipLaunchKernelGGL(cc_kernel, dim3((unsigned)kk), dim3(256), 0, s, E, w, mu, d, kk, cc);
  const int ntn = (int)(np / L.tn);
  const int64_t nblocks = (n + PM - 1) / PM * ntn;
  if (nblocks > (int64_t)1 << 30) return hipErrorInvalidValue;
  const int grid = (int)((nblocks + 7) / 8 * 8);
  if (L.tn == 256)
    hipLaunchKernelGGL((proj_i8_kernel<256, false>), dim3((unsigned)grid), dim3(512), 0, s, X, n, d, D, ntn, (int)nblocks, I,
                       np);
  else
    hipLaunchKernelGGL((proj_i8_kernel<128, false>), dim3((unsigned)grid), dim3(512), 0, s, X, n, d, D, ntn, (int)nblocks, I,
                       np);
  hipLaunchKernelGGL(proj_combine_kernel, dim3((unsigned)((n * kk + 255) / 256)), dim3(256), 0, s, I, n, kk, np, tsh,
                     cc, F);
  return hipGetLastError();
}

}  // namespace ef
