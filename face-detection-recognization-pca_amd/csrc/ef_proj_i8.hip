// Training projection F = ((X - mu) * w) . E on the int8 matrix cores (fit K5, the
// projected_data of useless/train.py:122 / face_features of train-v4.py:134, n x k).
//
// X is uint8, so X' = X - 128 is exact int8, and
//     F = X' . E'' + 1 . c^T,   E'' = diag(w) E,   c = (128 - mu)^T E''
// (c in fp64 by cc_kernel).  E'' is fp64; per output column it is scaled by 2^t_c so its
// largest entry lies in [2^45, 2^46) and rounded to an integer V (error <= 2^-46 of the
// column's largest entry), which is written as P = 6 signed base-256 digits,
// V = sum_j 256^j D_j with D_j in [-128, 127].  Each X' . D_j is an exact int32
// (|.| <= d * 2^14 <= 2^30 for d <= 65536), so the only roundings are the quantisation of
// E'' and the fp64 Horner combine 2^-t_c sum_j 256^j I_j (proj_combine_kernel): an error
// of ~sqrt(d) 2^-47 of |x'| max|E''|, the order of the fp64 GEMM it replaces (its own
// sqrt(d) 2^-53 of |x'||E''| per output; reference: useless/train.py:122 in float64), and
// the same quantisation as the fit's C.Q digit products (ef_cq_i8.hip).  Round 6: 7 -> 6
// digits, so kk = 128 runs as exactly 3 tiles of 256 digit columns instead of 4.
//
// proj_i8_kernel<TN>: C[n][N] (int32) = X' . D^T with D = [N = P * kk padded to TN][d] int8
// (K-contiguous).  Workgroup tile 256 rows x TN digit-columns, 8 waves (TN = 128: 4 x 2 of
// 64 x 64; TN = 256: 2 x 4 of 128 x 64; TN = 384: 2 x 4 of 128 x 96, 192 accumulator
// registers, a 4 x 40 KiB ring), K stages of 64 bytes staged by LDS-DMA into a
// 4-stage ring (same 64-B row swizzle as the covariance kernel); A fragments are flipped to
// int8 (x ^ 0x80) in registers.  The N-tiles of one row block are consecutive on one XCD,
// so X is read from HBM about once.  A stage streams (256 + TN) x 64 B from L2 for
// 256 x TN x 64 MACs: 48 B per MFMA-clock of a CU at TN = 128, 32 at TN = 256 — the L2 -> LDS
// stream (~30 B/clk per CU, K3) is the limit, so 6 digits x kk = 128 run as 2 tiles of 384
// (26.7 B per MFMA-clock) rather than 3 of 256 or 6 of 128.
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
constexpr int kDigits = 6;        // base-256 digits of the scaled eigenvector entries
constexpr int kTopBit = 46;       // largest scaled entry in [2^45, 2^46)

// t_c: 2^t_c * max_r |w_r E[r][c]| lies in [2^45, 2^46); zero columns get t_c = 0.
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
    tsh[c] = red[0] > 0.0 ? kTopBit - e : 0;
  }
}

// D[(j * kk + c) * d + r] = digit j of rint(w_r E[r][c] 2^t_c); rows kk * P .. Npad are zero.
__global__ void digits_kernel(const double* __restrict__ E, const double* __restrict__ w, int64_t d, int kk,
                              const int* __restrict__ tsh, int8_t* __restrict__ D) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d * kk) return;
  const int64_t r = e / kk;
  const int c = (int)(e - r * kk);
  long long v = (long long)rint(ldexp((w ? w[r] : 1.0) * E[r * kk + c], tsh[c]));
#pragma unroll
  for (int j = 0; j < kDigits; ++j) {
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
template <int TN>
__global__ __launch_bounds__(512, 1) void proj_i8_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d,
                                                         const int8_t* __restrict__ D, int ntn, int nblocks,
                                                         int* __restrict__ C, int64_t ldc) {
  constexpr int WC = TN == 384 ? 96 : 64;       // columns per wave
  constexpr int WN = TN / WC, WM = 8 / WN;      // wave grid; a wave owns (PM / WM) x WC
  constexpr int IA = PM / WM / 32, JB = WC / 32;  // 32 x 32 blocks per wave
  constexpr int BPW = TN / 128;                 // B pieces per wave per stage (A: 2)
  constexpr int PSTAGE = (PM + TN) * PK;        // bytes per stage: A panel, then B panel
  __shared__ __attribute__((aligned(16))) uint8_t smem[PNB * PSTAGE];
  const int total = gridDim.x;  // multiple of 8; trailing blocks are idle padding
  // blocks b and b+8 share an XCD: XCD x runs items [x*total/8, (x+1)*total/8), row-block
  // major, so the N-tiles of a row block run together and share its X rows in L2
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  if (lin >= nblocks) return;
  const int mt = lin / ntn, nt = lin - (lin / ntn) * ntn;
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
    arow[jj] = X + ra * d + lchunk * 16;
  }
  const unsigned voffB = (unsigned)((n0 + wave * BPW * 16 + lrow) * d + lchunk * 16);  // D is N x d (< 4 GiB)
  const int64_t nst = d / PK;
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
  const unsigned offb[2] = {(unsigned)(PM * PK + (wn * WC + c32) * PK + ((h ^ sw) * 16)),
                            (unsigned)(PM * PK + (wn * WC + c32) * PK + (((2 + h) ^ sw) * 16))};
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
      const int64_t col = n0 + wn * WC + j * 32 + c32;
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

}  // namespace

struct ProjLayout {
  int64_t np, off_i, off_t, off_c, bytes;
  int tn;  // digit-columns per tile (128 or 256)
};
static ProjLayout proj_layout(int64_t n, int64_t d, int kk) {
  auto a256 = [](int64_t v) { return (v + 255) / 256 * 256; };
  ProjLayout L;
  // 384-column tiles (the covariance SYRK's 256 x 384 shape: 26.7 B of L2 -> LDS per
  // MFMA-clock) where they pad no more than 256-column tiles; 256-column tiles (32 B)
  // unless they pad the digit columns by > 15 % more than 128-column tiles (48 B) do
  const int64_t p = (int64_t)kDigits * kk, n128 = (p + 127) / 128 * 128, n256 = (p + 255) / 256 * 256,
                n384 = (p + 383) / 384 * 384;
  L.tn = n384 <= n256 ? 384 : n256 * 100 <= n128 * 115 ? 256 : 128;
#ifdef EF_DIAGNOSTICS
  if (const char* e = getenv("EF_PROJ_TN")) L.tn = atoi(e) == 384 ? 384 : atoi(e) == 256 ? 256 : 128;
#endif
  L.np = L.tn == 384 ? n384 : L.tn == 256 ? n256 : n128;
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
  hipLaunchKernelGGL(digit_scale_kernel, dim3((unsigned)kk), dim3(256), 0, s, E, w, d, kk, tsh);
  hipLaunchKernelGGL(digits_kernel, dim3((unsigned)((d * kk + 255) / 256)), dim3(256), 0, s, E, w, d, kk, tsh, D);
  hipLaunchKernelGGL(cc_kernel, dim3((unsigned)kk), dim3(256), 0, s, E, w, mu, d, kk, cc);
  const int ntn = (int)(np / L.tn);
  const int64_t nblocks = (n + PM - 1) / PM * ntn;
  if (nblocks > (int64_t)1 << 30) return hipErrorInvalidValue;
  const int grid = (int)((nblocks + 7) / 8 * 8);
  if (L.tn == 384)
    hipLaunchKernelGGL(proj_i8_kernel<384>, dim3((unsigned)grid), dim3(512), 0, s, X, n, d, D, ntn, (int)nblocks, I,
                       np);
  else if (L.tn == 256)
    hipLaunchKernelGGL(proj_i8_kernel<256>, dim3((unsigned)grid), dim3(512), 0, s, X, n, d, D, ntn, (int)nblocks, I,
                       np);
  else
    hipLaunchKernelGGL(proj_i8_kernel<128>, dim3((unsigned)grid), dim3(512), 0, s, X, n, d, D, ntn, (int)nblocks, I,
                       np);
  hipLaunchKernelGGL(proj_combine_kernel, dim3((unsigned)((n * kk + 255) / 256)), dim3(256), 0, s, I, n, kk, np, tsh,
                     cc, F);
  return hipGetLastError();
}

}  // namespace ef
