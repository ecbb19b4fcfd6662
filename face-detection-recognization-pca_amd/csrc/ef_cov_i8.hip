// Exact covariance / Gram of uint8 faces on the int8 matrix cores (fit K3).
//
// The fit's dominant GEMM (useless/train.py:82-85 Gram A.A^T when n < d; the np.cov
// branch :97-99 / sklearn's SVD of the centred matrix otherwise) has integer inputs.
// Shifting pixels by -128 maps them exactly onto int8, and the shift cancels in the
// centred product:
//   covariance (n >= d):  (n-1) n C_ij = n S'_ij - c_i c_j,           S' = X'^T X'
//   Gram       (n <  d):  (n-1) n^2 C_ij = n^2 S'_ij - n (R_i + R_j) + Q,   S' = X' X'^T
// with X' = X - 128, c = column sums of X', R_i = X'_i . c, Q = c . c — all exact
// integers.  S' runs on v_mfma_i32_32x32x32_i8 with int32 accumulators: a work item covers
// at most kMaxSplitK samples (|x'x'| <= 2^14, 131008 * 2^14 < 2^31), so it ends with one
// plain int32 store into its split's slab, and the finalize sums the slabs in int64/int128.
// The only rounding of the whole covariance is the final int128 -> fp64 conversion and
// division (<= 1 ulp), tighter than the fp64 GEMM the reference runs.  StandardScaler
// scaling (train-v4.py:131) is applied afterwards as C_ij / (scale_i scale_j).
//
// Operand layout in HBM: At = [kpad/64][dim][64] bytes ("K-blocked"): the 64 samples of one
// K-stage for all dim rows are one contiguous dim*64-byte block, so a stage's 256-row panel
// is a single 16-KiB run (a row-major [dim][kpad] copy puts every row of a panel on its own
// page, 1 MB apart at n = 1M).  The covariance path writes it with a fused transpose that
// also produces the exact column sums (sum x, sum x^2) the StandardScaler needs, so X is
// read once for both.
//
// SYRK kernel: 256 x 384 output tile per workgroup (the tiles that touch the upper
// triangle; 256 x 256 below order 2048), 8 waves of 128 x 96, K-slices of 64 samples staged
// by global_load_lds into a 4-stage LDS ring (4 x 40 KiB = all of LDS, three stages in
// flight behind the landed one, fragments of the next stage read ahead of the current
// stage's last MFMAs), 64-B rows XOR-swizzled by ((row >> 2) & 3) so the ds_read_b128
// fragment reads are conflict-free.  Work items = (tile, K-split): the split
// count is chosen so items fill whole rounds of the chip (no tail round), and the item list
// is split-major, so each XCD (blocks b = x mod 8) streams its own K range of every panel
// while its ~32 resident workgroups run one 8 x 4 block of tiles (12 panels shared in L2).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "ef_dma.hpp"
#include "ef_linalg.hpp"

namespace ef {

typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int YT = 256;                   // output tile rows (columns: 256 or 384, syrk_tile_cols)
constexpr int YK = 64;                    // samples per stage
constexpr int64_t kMaxSplitStages = 2047; // 2047 * 64 = 131008 samples: int32-safe
constexpr int FB = 64;                    // finalize block

// ---------------------------------------------------------------- operand preparation
// Gram path (rows = samples): At[kb][r][kk] = X[r][64 kb + kk] - 128, zero past d.
__global__ void shift_copy_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d, int64_t nkb,
                                  uint8_t* __restrict__ At) {
  const int64_t total = nkb * n * 4;  // 16-byte chunks
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t kb = q / (n * 4), rem = q - kb * n * 4;
    const int64_t r = rem >> 2;
    const int64_t k0 = kb * 64 + (rem & 3) * 16;
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unsigned v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t k = k0 + 4 * i + b;
        const unsigned x = k < d ? (unsigned)(X[r * d + k] ^ 0x80u) : 0u;
        v |= x << (8 * b);
      }
      w[i] = v;
    }
    *reinterpret_cast<uint4*>(At + q * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Covariance path (rows = pixels), byte-granular fallback for d % 4 != 0 or unaligned X:
// At[kb][c][kk] = X[64 kb + kk][c] - 128, zero past n.
__global__ void shift_transpose_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d, int64_t nkb,
                                       uint8_t* __restrict__ At) {
  __shared__ uint8_t t[64][65];
  const int64_t kb = blockIdx.x, c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: 4 rows per pass
  for (int r = ty; r < 64; r += 4) {
    const int64_t k = kb * 64 + r, c = c0 + tx;
    t[r][tx] = (k < n && c < d) ? (uint8_t)(X[k * d + c] ^ 0x80u) : (uint8_t)0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int64_t c = c0 + r;
    if (c < d) At[(kb * d + c) * 64 + tx] = t[tx][r];
  }
}

// Covariance path, d % 4 == 0: the fused transpose + exact column statistics.  Wave q of
// a workgroup owns rows 16q..16q+15 of every 64-sample block it visits, lane l the four
// pixels c0 + 4l..+3: 16 coalesced dword loads, a register 4x4 byte transpose, four 16-B
// stores (one per pixel row of At).  S1[c] += sum x, S2[c] += sum x^2 (uint32 partials per
// thread — at most 16 * 4096 rows — reduced over the 4 waves in LDS, one uint64 atomic
// per pixel and workgroup).
__global__ __launch_bounds__(256) void transpose_stats_kernel(const uint8_t* __restrict__ X, int64_t n, int64_t d,
                                                              int64_t nkb, uint8_t* __restrict__ At,
                                                              unsigned long long* __restrict__ S1,
                                                              unsigned long long* __restrict__ S2) {
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.y * 256 + 4 * lane;
  const bool cok = c < d;
  unsigned s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  for (int64_t kb = blockIdx.x; kb < nkb; kb += gridDim.x) {
    const int64_t kr = kb * 64 + 16 * q;
    unsigned v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      v[r] = (cok && kr + r < n) ? __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(X + (kr + r) * d + c))
                                 : 0x80808080u;  // pad rows: x = 128, x' = 0 (excluded from the sums below)
    if (cok) {
      const int valid = (int)(n - kr < 16 ? (n - kr < 0 ? 0 : n - kr) : 16);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r < valid) {
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const unsigned x = (v[r] >> (8 * m)) & 0xffu;
            s1[m] += x;
            s2[m] += x * x;
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        unsigned o[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          unsigned t = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) t |= ((v[4 * w + b] >> (8 * m)) & 0xffu) << (8 * b);
          o[w] = t ^ 0x80808080u;
        }
        *reinterpret_cast<uint4*>(At + (kb * d + c + m) * 64 + 16 * q) = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  }
  __shared__ unsigned red[2][4][256];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    red[0][q][4 * lane + m] = s1[m];
    red[1][q][4 * lane + m] = s2[m];
  }
  __syncthreads();
  const int cc = threadIdx.x;  // pixel c0 + cc
  const int64_t col = (int64_t)blockIdx.y * 256 + cc;
  if (col < d) {
    unsigned long long a = 0, b = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      a += red[0][w][cc];
      b += red[1][w][cc];
    }
    atomicAdd(&S1[col], a);
    atomicAdd(&S2[col], b);
  }
}

// The same pass with every HBM access a contiguous 1-KiB wave piece (d % 256 == 0):
// a step is 64 samples x 256 pixels (16 KiB in, 16 KiB out — At's block for those pixels
// is one contiguous run).  Thread t loads 16 B of sample row 16i + t/16 (dwordx4) into an
// LDS image [sample][256 px] whose 16-B column chunks are XORed by the row's quarter
// (r >> 4), then assembles At's 16-B piece t + 256i — pixel t/4 + 64i, samples
// 16(t%4) .. +15 — from 16 byte reads (the XOR puts a wave's four sample quarters on four
// distinct bank groups) and stores it at byte 16t + 4096i of the block.  The stats come
// from the assembled pieces (v_dot4_u32_u8: Σx against 1s, Σx² against itself), one pixel
// per thread slot; samples past n read as x = 0 for the sums and x' = 0 in At.
__global__ __launch_bounds__(256) void transpose_stats_lds_kernel(const uint8_t* __restrict__ X, int64_t n,
                                                                  int64_t d, int64_t nkb, uint8_t* __restrict__ At,
                                                                  unsigned long long* __restrict__ S1,
                                                                  unsigned long long* __restrict__ S2) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[64 * 256];
  const int t = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.y * 256;
  const int lc = t & 15, lr = t >> 4;  // load: 16-B column chunk, row within a 16-row group
  const int q = t & 3;                 // assemble: sample quarter
  unsigned s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  // the next step's four loads are issued before this step's assembly (registers v)
  u32x4 v[4];
  auto load = [&](int64_t kb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t smp = kb * 64 + 16 * i + lr;
      const int64_t sc = smp < n ? smp : n - 1;  // unconditional (all four in flight), zeroed below
      v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(X + sc * d + c0) + lc);
    }
  };
  if ((int64_t)blockIdx.x < nkb) load(blockIdx.x);
  for (int64_t kb = blockIdx.x; kb < nkb; kb += gridDim.x) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * i + lr;
      const u32x4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<u32x4*>(img + r * 256 + 16 * (lc ^ i)) = kb * 64 + r < n ? v[i] : z;
    }
    if (kb + gridDim.x < nkb) load(kb + gridDim.x);
    __syncthreads();
    const int64_t valid = n - (kb * 64 + 16 * q);  // samples of this quarter inside the data
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = (t >> 2) + 64 * i;
      const uint8_t* col = img + 16 * q * 256 + (p ^ (16 * q));
      unsigned w[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const unsigned b0 = col[(4 * g) * 256], b1 = col[(4 * g + 1) * 256], b2 = col[(4 * g + 2) * 256],
                       b3 = col[(4 * g + 3) * 256];
        w[g] = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
        s1[i] = __builtin_amdgcn_udot4(w[g], 0x01010101u, s1[i], false);
        s2[i] = __builtin_amdgcn_udot4(w[g], w[g], s2[i], false);
      }
      u32x4 o = {w[0] ^ 0x80808080u, w[1] ^ 0x80808080u, w[2] ^ 0x80808080u, w[3] ^ 0x80808080u};
      if (valid < 16) {  // the last block's pad samples: x' = 0
        unsigned m[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int64_t k = valid - 4 * g;  // valid bytes of dword g
          m[g] = k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : (0xffffffffu >> (8 * (4 - k))));
        }
        o.x &= m[0];
        o.y &= m[1];
        o.z &= m[2];
        o.w &= m[3];
      }
      __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(At + (kb * d + c0) * 64) + t + 256 * i);
    }
    __syncthreads();
  }
  // the four quarters of a pixel sit in lanes 4j .. 4j+3.  Each quarter's sums are exact in
  // 32 bits (<= 4096 blocks x 16 samples x 255^2 < 2^32 per workgroup, launch bound), but
  // four quarters of Σx² are not: widen before adding them.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned long long a = s1[i], b = s2[i];
    a += __shfl_xor(a, 1);
    a += __shfl_xor(a, 2);
    b += __shfl_xor(b, 1);
    b += __shfl_xor(b, 2);
    if (q == 0) {
      const int64_t col = c0 + (t >> 2) + 64 * i;
      atomicAdd(&S1[col], a);
      atomicAdd(&S2[col], b);
    }
  }
}

// ---------------------------------------------------------------- SYRK on int8 MFMA
// Slab[ks][i][j] = sum over split ks's samples of At[.][i][k] At[.][j][k] over the tiles
// (256 rows x TJ columns) that touch the upper triangle.  Item = (split, tile), split-major.
// Per CU the kernel is bound by the L2 -> LDS stream (an XCD-L2-resident gather runs at
// ~30 B/clk per CU): a stage moves (256 + TJ) x 64 B for 256 x TJ x 64 MACs, i.e. 32 B per
// MFMA-clock at TJ = 256 and 26.7 B at TJ = 384 (192 accumulator VGPRs per lane, the most
// two waves per SIMD can hold next to their fragments).
// When each wave issues the DMA pieces of the stage NB ahead, as positions in the second
// k-step of a stage (0 = right after the stage's barrier, n = after row block n - 1's
// MFMAs): pieces [0, EF_SYRK_SPLIT) at position A, the rest at position B, separately for
// waves 0..3 (LO) and 4..7 (HI) — the two waves sharing a SIMD.  Issuing every wave's
// burst right after the barrier (all positions 0) left both waves of a SIMD in their DMA
// issue at once; measured (C3 SYRK, profiles/r04/syrk_stagger_ab*.txt): all at 0 105.9 ms,
// HI at 1: 99.9, LO at 1 + HI at 3: 94.6.
#ifndef EF_SYRK_LO_A
#define EF_SYRK_LO_A 1
#endif
#ifndef EF_SYRK_LO_B
#define EF_SYRK_LO_B EF_SYRK_LO_A
#endif
#ifndef EF_SYRK_HI_A
#define EF_SYRK_HI_A 3
#endif
#ifndef EF_SYRK_HI_B
#define EF_SYRK_HI_B EF_SYRK_HI_A
#endif
#ifndef EF_SYRK_SPLIT
#define EF_SYRK_SPLIT 3
#endif
template <int TJ, int NB>
__global__ __launch_bounds__(512, 1) void syrk_i8_kernel(const uint8_t* __restrict__ At, int64_t dim,
                                                         int64_t st_begin, int64_t st_end, int64_t kps, int ntiles,
                                                         int nitems, const int2* __restrict__ order,
                                                         int* __restrict__ slabs) {
  constexpr int NJ = TJ / 128;              // 32-column blocks per wave (waves are 2 x 4 of 128 x TJ/4)
  constexpr int NPA = YT / 16, NP = (YT + TJ) / 16, PPW = NP / 8;  // 1-KiB DMA pieces: A, all, per wave
  constexpr int STG = (YT + TJ) * YK;       // bytes per stage (A panel, then B panel)
  static_assert(NP % 8 == 0, "pieces must split evenly over the 8 waves");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NB * STG];
  const int total = gridDim.x;  // multiple of 8; trailing blocks are idle padding
  // blocks b and b+8 share an XCD: XCD x runs list entries [x*total/8, (x+1)*total/8)
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  if (lin >= nitems) return;
  const int ks = lin / ntiles;
  const int2 tt = order[lin - ks * ntiles];
  // wave-uniform: keep the tile origin (and everything derived from it) in SGPRs
  const int64_t i0 = (int64_t)__builtin_amdgcn_readfirstlane(tt.x) * YT;
  const int64_t j0 = (int64_t)__builtin_amdgcn_readfirstlane(tt.y) * TJ;
  const int64_t sb = st_begin + ks * kps;
  const int64_t se = sb + kps < st_end ? sb + kps : st_end;
  const int64_t nst = se > sb ? se - sb : 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 2, wn = wave & 3;

  // DMA: a stage = NP pieces of 1 KiB (16 rows x 64 B), A's then B's, contiguous in LDS;
  // wave w issues pieces PPW*w .. PPW*w + PPW-1.  Lane l -> row 16j + (l >> 2), physical
  // chunk l & 3 holding logical chunk (l & 3) ^ ((l >> 4) & 3).  The per-lane byte offsets
  // inside a stage block are fixed for the item: the stage loop only moves the wave-uniform
  // SGPR base (no per-lane 64-bit address arithmetic per stage).
  const unsigned lds_base = lds_addr(smem);
  const int lrow = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lane >> 4) & 3);
  const int64_t blk = dim * YK;  // bytes per K-stage block of At
  // one per-lane offset for every piece; the piece's first row goes into the wave-uniform
  // SGPR base.  Rows past dim (the last tiles) read the next stage block, or the
  // kSyrkPadBytes the allocation carries past the last one: finite values whose products
  // land only in outputs the epilogue masks.
  const unsigned voff = (unsigned)(lrow * YK + lchunk * 16);
  auto issue = [&](int64_t st, int buf, int q0 = 0, int q1 = 1 << 30) {
    const uint8_t* base = At + st * blk;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      if (q < q0 || q >= q1) continue;
      const int p = wave * PPW + q;
      const int64_t r0 = p < NPA ? i0 + p * 16 : j0 + (p - NPA) * 16;
      glds16s(voff, (unsigned long long)(size_t)(base + r0 * YK), lds_base + (unsigned)(buf * STG + p * 1024));
    }
  };

  i32x16 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = i32x16{};

  const int sw = (c32 >> 2) & 3;  // swizzle key of every row this lane reads
  // lane (r, h) holds A[r][32s + 16h + j], B[32s + 16h + j][r] for k-step s of a stage
  // per-lane fragment offsets for the two k-steps; blocks i / j add i * 2048 / j * 2048
  // (immediate offsets of one ds_read_b128 base)
  const unsigned offa[2] = {(unsigned)((wm * 128 + c32) * YK + ((h ^ sw) * 16)),
                            (unsigned)((wm * 128 + c32) * YK + (((2 + h) ^ sw) * 16))};
  const unsigned offb[2] = {(unsigned)(YT * YK + (wn * (TJ / 4) + c32) * YK + ((h ^ sw) * 16)),
                            (unsigned)(YT * YK + (wn * (TJ / 4) + c32) * YK + (((2 + h) ^ sw) * 16))};
  auto fa = [&](const uint8_t* sa, int s, int i) {
    return *reinterpret_cast<const i32x4*>(sa + offa[s] + i * 32 * YK);
  };
  auto fb = [&](const uint8_t* sa, int s, i32x4 (&b)[NJ]) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const i32x4*>(sa + offb[s] + j * 32 * YK);
  };
  // One k-step's MFMAs, row block by row block; each A fragment is refilled with the
  // next k-step's as soon as its row block's MFMAs are issued (one A set + two B sets live:
  // 40 fragment VGPRs next to the 64 * NJ accumulators).
  auto mma = [&](i32x4 (&a)[4], const i32x4 (&b)[NJ], const uint8_t* nsa, int ns, auto&& mid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j], acc[i][j], 0, 0, 0);
      a[i] = fa(nsa, ns, i);
      mid(i + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto none = [](int) {};
  // Ring of NB stages.  Each stage is PPW DMA instructions per wave, so "stage t landed" is
  // vmcnt <= PPW x (stages issued after it); tail stages past nst are issued as harmless
  // re-reads of the first stage so the count stays uniform.  One barrier per stage, placed
  // between the stage's two k-steps: it publishes stage st+1 and retires stage st's slot,
  // so the next stage's first fragments are read, and the DMA into the retired slot issued,
  // while the second k-step's MFMAs are still to run — the MFMA pipe never waits for the
  // barrier plus an LDS round trip.  NB-1 stages stay in flight behind the landed one.
  if (nst > 0) {
    for (int j = 0; j < NB; ++j) issue(sb + (j < nst ? j : 0), j);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * (NB - 1)) : "memory");  // stage 0 landed
    __syncthreads();
    i32x4 a[4], b0[NJ], b1[NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = fa(smem, 0, i);
    fb(smem, 0, b0);
    for (int64_t st = 0; st < nst; ++st) {
      const uint8_t* cur = smem + (st % NB) * STG;
      fb(cur, 1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a, b0, cur, 1, none);  // k-step 0; A refilled with k-step 1
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * (NB - 2)) : "memory");  // stage st+1 landed
      __syncthreads();  // every wave done reading stage st; stage st+1 visible
      const int64_t nx = st + NB;
      auto issue_next = [&](int q0, int q1) { issue(sb + (nx < nst ? nx : 0), (int)(nx % NB), q0, q1); };  // into stage st's slot
      // this wave's pieces at positions (A, B) of k-step 1 (EF_SYRK_* above)
      static_assert(EF_SYRK_LO_A <= 4 && EF_SYRK_LO_B <= 4 && EF_SYRK_HI_A <= 4 && EF_SYRK_HI_B <= 4,
                    "issue positions must exist (4 row blocks): every wave issues its pieces each stage");
      const int pa = wave < 4 ? EF_SYRK_LO_A : EF_SYRK_HI_A, pb = wave < 4 ? EF_SYRK_LO_B : EF_SYRK_HI_B;
      auto at_pos = [&](int pos) {
        if (pos == pa) issue_next(0, EF_SYRK_SPLIT);
        if (pos == pb) issue_next(EF_SYRK_SPLIT, PPW);
      };
      at_pos(0);
      // (after the last stage these read a slot holding a re-read of the first stage:
      // harmless, unused, and branch-free)
      const uint8_t* nxt = smem + ((st + 1) % NB) * STG;
      fb(nxt, 0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a, b1, nxt, 0, at_pos);  // k-step 1; A refilled with the next stage's k-step 0
    }
    dma_wait_all();
  }
  int* out = slabs + (int64_t)ks * dim * dim;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t col = j0 + wn * (TJ / 4) + j * 32 + c32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = i0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < dim && col < dim) out[row * dim + col] = acc[i][j][r];
      }
    }
}

// The product SYRK for orders >= 2048 (256 x 384 tiles, NJB = 6; round 4).  The int8
// 16x16x64 MFMA holds a higher clock than 32x32x32 under load (tools/micro/bf16_clock i:
// 2.06 vs 1.78 GHz with LDS-fed operands, profiles/r03/i8_clock.json); in round 3 this
// kernel measured no faster in the C3 fit (NJB = 6: 0.165 vs 0.163-0.168 s) while every
// wave issued its stage's DMA right after the barrier.  With the issue staggered over the
// two waves of a SIMD (EF_S16_LO / EF_S16_HI below) it takes 91.8-92.7 ms against the
// staggered 32x32x32 kernel's 98.6-99.5 ms on the same box (C3, three alternations,
// identical eigenvalues; profiles/r04/syrk16_stagger_ab.txt).
// The same item on v_mfma_i32_16x16x64_i8 (one 64-sample k-step per stage): wave (wm, wn)
// owns 128 rows x 16 NJB columns as 8 x NJB 16 x 16 blocks (4 accumulator VGPRs each).
// Lane l supplies row l & 15 of a block and samples 16 (l >> 4) .. +15 (the K order inside a
// fragment is the same for A and B — both are At rows — so it cancels in the dot product).
// The stage's 64-B rows hold their 16-B chunks at chunk ^ f((row >> 2) & 3), f = {0, 2, 3, 1}:
// each ds_read_b128 lane group ({0-3,12-15,20-27}, … MI355X_MICROARCH §LDS) then covers all 16
// bank quads.  Order per stage: column block by column block over the 8 row blocks, the
// next column's B fragment read while a column's MFMAs run; the barrier (stage st+1
// visible, slot st retired) sits before the last column, during which the A fragments are
// refilled with stage st+1's.
__device__ __forceinline__ int syrk16_swz(int b) { return (0x78 >> (2 * b)) & 3; }
#ifndef EF_S16_LO  // measured (C3 SYRK): (LO, HI) = (0, 0) 109 ms, (1, 3) 92-93, (1, 2) 104,
#define EF_S16_LO 1  // (1, 4) 108, (1, 5) 104, (1, 6) 105, (2, 3) 106, (2, 4) 120, (0, 3) 115
#endif
#ifndef EF_S16_HI
#define EF_S16_HI 3
#endif

// OZ (the fit's int8 digit-pair products, ef_cq_i8.hip; NJB = 4: 256 x 256 items): At is
// the digits' K-blocked array of `dim` = R rows, kps the order of C (odim), ntiles the row
// blocks per XCD, [st_begin, st_end) all K stages; items per XCD: its row blocks' 20 whole
// pairs, then the 4 K-parts of pair (0, 5); each writes its pair block of slabs (odim x 256).
// PAIR (diagnostic EF_SYRK_PAIR=1): two stages per barrier — the ring's two older slots
// are consumed back to back, then retired together at one barrier while the two newer land.
template <int NJB, int NB, bool OZ = false, bool PAIR = false, bool OZMED = false>
__global__ __launch_bounds__(512, 1) void syrk16_i8_kernel(const uint8_t* __restrict__ At, int64_t dim,
                                                           int64_t st_begin, int64_t st_end, int64_t kps, int ntiles,
                                                           int nitems, const int2* __restrict__ order,
                                                           int* __restrict__ slabs) {
  constexpr int TJ = 64 * NJB;
  constexpr int NPA = YT / 16, NP = (YT + TJ) / 16;
  constexpr int PPW = (NP + 7) / 8;          // DMA pieces per wave (the last wave may pad)
  constexpr int STG = (YT + TJ) * YK;
  constexpr int DUMMY = NP % 8 ? 1024 : 0;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NB * STG + DUMMY];  // + a dummy DMA target
  const int total = gridDim.x;
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  if (lin >= nitems) return;
  int64_t i0, j0, sb, nst;
  int ks = 0;
  int64_t oz_row0 = 0;  // OZ: the item's first output row
  if constexpr (OZ) {
    const int64_t odim = kps;
    const int per = total >> 3, x = lin / per, r = lin - x * per;
    int p, mt;
    sb = st_begin;
    nst = st_end - st_begin;
    constexpr int whole = oz_pairs(OZMED) - 1;
    if (r < ntiles * whole) {
      mt = x * ntiles + r / whole;
      p = r % whole;
      ks = p;
    } else {
      const int r2 = r - ntiles * whole;
      mt = x * ntiles + r2 / kOzSplitParts;
      const int part = r2 % kOzSplitParts;
      p = whole;
      ks = p + part;
      sb = st_begin + nst * part / kOzSplitParts;
      nst = st_begin + nst * (part + 1) / kOzSplitParts - sb;
    }
    int a, b;
    oz_pair(p, OZMED, a, b);
    i0 = (int64_t)a * odim + (int64_t)mt * YT;
    j0 = 6 * odim + (int64_t)b * TJ;
    oz_row0 = (int64_t)mt * YT;
  } else {
    ks = lin / ntiles;
    const int2 tt = order[lin - ks * ntiles];
    i0 = (int64_t)__builtin_amdgcn_readfirstlane(tt.x) * YT;
    j0 = (int64_t)__builtin_amdgcn_readfirstlane(tt.y) * TJ;
    sb = st_begin + ks * kps;
    const int64_t se = sb + kps < st_end ? sb + kps : st_end;
    nst = se > sb ? se - sb : 0;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const unsigned lds_base = lds_addr(smem);
  const int lrow = lane >> 2;
  const int lchunk = (lane & 3) ^ syrk16_swz((lane >> 4) & 3);
  const int64_t blk = dim * YK;
  const unsigned voff = (unsigned)(lrow * YK + lchunk * 16);
  auto issue = [&](int64_t st, int buf, int q0 = 0, int q1 = 1 << 30) {
    const uint8_t* base = At + st * blk;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      if (q < q0 || q >= q1) continue;
      const int p = wave * PPW + q;
      if (p < NP) {
        const int64_t r0 = p < NPA ? i0 + p * 16 : j0 + (p - NPA) * 16;
        glds16s(voff, (unsigned long long)(size_t)(base + r0 * YK), lds_base + (unsigned)(buf * STG + p * 1024));
      } else {  // uniform DMA count per wave
        glds16s(voff, (unsigned long long)(size_t)base, lds_base + (unsigned)(NB * STG));
      }
    }
  };
  i32x4 acc[8][NJB];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJB; ++j) acc[i][j] = i32x4{};
  const int r16 = lane & 15;
  const unsigned foff = (unsigned)(r16 * YK + 16 * ((lane >> 4) ^ syrk16_swz(r16 >> 2)));
  const unsigned offa = (unsigned)(wm * 128 * YK) + foff;
  const unsigned offb = (unsigned)(YT * YK + wn * 16 * NJB * YK) + foff;
  auto fa = [&](const uint8_t* sa, int i) { return *reinterpret_cast<const i32x4*>(sa + offa + i * 16 * YK); };
  auto fb = [&](const uint8_t* sa, int j) { return *reinterpret_cast<const i32x4*>(sa + offb + j * 16 * YK); };
  if (nst > 0) {
    for (int j = 0; j < NB; ++j) issue(sb + (j < nst ? j : 0), j);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * (NB - 1)) : "memory");  // stage 0 landed
    __syncthreads();
    // registers: the stage's 8 A fragments, and a two-entry ring of B fragments (the column
    // being multiplied and the next one) — 40 VGPRs next to the 32 NJB accumulators
    i32x4 a[8], bq, bn;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = fa(smem, i);
    bq = fb(smem, 0);
    // DMA issue position of this wave (EF_S16_LO / EF_S16_HI for waves 0-3 / 4-7): 0 = right
    // after the barrier, 1 = after the last column's MFMAs, 2 + j = after column j of the
    // next stage (the pending stage index is carried across the iteration)
    static_assert(EF_S16_LO <= NJB && EF_S16_HI <= NJB, "issue positions must exist: 0 .. NJB");
    const int dpos = wave < 4 ? EF_S16_LO : EF_S16_HI;
    int64_t pend = -1;
    auto flush = [&](int pos) {
      if (pos == dpos && pend >= 0) {
        issue(sb + (pend < nst ? pend : 0), (int)(pend % NB));
        pend = -1;
      }
    };
    if constexpr (PAIR) {
      static_assert(NB == 4, "two consumed + two landing slots");
      int64_t pend2 = -1;  // the pair's second stage, issued one position after the first
      for (int64_t st = 0; st < nst; st += 2) {
        const bool two = st + 1 < nst;  // uniform
        const uint8_t* c0 = smem + (st % NB) * STG;
        const uint8_t* c1 = smem + ((st + 1) % NB) * STG;
        const uint8_t* nx = smem + ((st + 2) % NB) * STG;
        auto flush2 = [&](int pos) {
          if (pos == dpos && pend >= 0) {
            issue(sb + (pend < nst ? pend : 0), (int)(pend % NB));
            pend = -1;
          }
          if (pos == dpos + 1 && pend2 >= 0) {
            issue(sb + (pend2 < nst ? pend2 : 0), (int)(pend2 % NB));
            pend2 = -1;
          }
        };
#pragma unroll
        for (int j = 0; j < NJB - 1; ++j) {
          bn = fb(c0, j + 1);
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bq, acc[i][j], 0, 0, 0);
          bq = bn;
          flush2(2 + j);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (two) {  // stage st's last column (A refilled from st + 1, visible since the last barrier)
          bn = fb(c1, 0);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            acc[i][NJB - 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bq, acc[i][NJB - 1], 0, 0, 0);
            a[i] = fa(c1, i);
          }
          bq = bn;
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < NJB - 1; ++j) {
            bn = fb(c1, j + 1);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bq, acc[i][j], 0, 0, 0);
            bq = bn;
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if (pend >= 0) {
          issue(sb + (pend < nst ? pend : 0), (int)(pend % NB));
          pend = -1;
        }
        if (pend2 >= 0) {
          issue(sb + (pend2 < nst ? pend2 : 0), (int)(pend2 % NB));
          pend2 = -1;
        }
        // every read of stages st, st+1 is issued; st+2 and st+3 (issued a pair ago) landed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        pend = st + NB;  // into the slots of st and st + 1
        pend2 = st + NB + 1;
        flush2(0);
        bn = fb(nx, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // the pair's last column
          acc[i][NJB - 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bq, acc[i][NJB - 1], 0, 0, 0);
          a[i] = fa(nx, i);
        }
        bq = bn;
        flush2(1);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else
    for (int64_t st = 0; st < nst; ++st) {
      const uint8_t* cur = smem + (st % NB) * STG;
      const uint8_t* nxt = smem + ((st + 1) % NB) * STG;
#pragma unroll
      for (int j = 0; j < NJB - 1; ++j) {
        bn = fb(cur, j + 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bq, acc[i][j], 0, 0, 0);
        bq = bn;
        flush(2 + j);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (pend >= 0) {  // a position past this stage's columns: issue before the wait below
        issue(sb + (pend < nst ? pend : 0), (int)(pend % NB));
        pend = -1;
      }
      // every read of stage st is issued (the barrier waits for them); stage st+1 landed
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW * (NB - 2)) : "memory");
      __syncthreads();
      pend = st + NB;  // into stage st's slot
      flush(0);
      bn = fb(nxt, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i][NJB - 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], bq, acc[i][NJB - 1], 0, 0, 0);
        a[i] = fa(nxt, i);
      }
      bq = bn;
      flush(1);
      __builtin_amdgcn_sched_barrier(0);
    }
    dma_wait_all();
  }
  if constexpr (OZ) {
    int* out = slabs + (int64_t)ks * kps * TJ;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJB; ++j) {
        const int col = wn * 16 * NJB + j * 16 + r16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = oz_row0 + wm * 128 + i * 16 + 4 * (lane >> 4) + r;
          out[row * TJ + col] = acc[i][j][r];
        }
      }
    return;
  }
  int* out = slabs + (int64_t)ks * dim * dim;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJB; ++j) {
      const int64_t col = j0 + wn * 16 * NJB + j * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = i0 + wm * 128 + i * 16 + 4 * (lane >> 4) + r;
        if (row < dim && col < dim) out[row * dim + col] = acc[i][j][r];
      }
    }
}

// ---------------------------------------------------------------- exact finishing
// R[r] = sum_k At[.][r][k] * c[k]   (Gram path; exact in int64)
__global__ void rowdot_kernel(const uint8_t* __restrict__ At, int64_t rows, int64_t d,
                              const long long* __restrict__ c, long long* __restrict__ R) {
  const int64_t r = blockIdx.x;
  long long s = 0;
  for (int64_t k = threadIdx.x; k < d; k += blockDim.x)
    s += (long long)(int8_t)At[((k >> 6) * rows + r) * YK + (k & 63)] * c[k];
  __shared__ long long red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) R[r] = red[0];
}

// c'[j] = S1[j] - 128 n, and Q = sum_j c'[j]^2 (Gram path) in int128 halves.
__global__ void shifted_sums_kernel(const unsigned long long* __restrict__ S1, int64_t n, int64_t d,
                                    long long* __restrict__ c) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < d) c[j] = (long long)S1[j] - 128LL * n;
}

__global__ void sumsq128_kernel(const long long* __restrict__ c, int64_t d, unsigned long long* __restrict__ out) {
  __shared__ unsigned __int128 red[256];
  unsigned __int128 s = 0;
  for (int64_t j = threadIdx.x; j < d; j += blockDim.x) {
    const __int128 v = c[j];
    s += (unsigned __int128)(v * v);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = (unsigned long long)red[0];
    out[1] = (unsigned long long)(red[0] >> 64);
  }
}

// S64 (+)= sum of the slabs, over the upper 64-blocks (multi-pass accumulation).
__global__ void slab_accumulate_kernel(const int* __restrict__ slabs, int nslab, int64_t dim,
                                       long long* __restrict__ S64) {
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bi > bj) return;
  for (int e = threadIdx.x; e < FB * FB; e += blockDim.x) {
    const int64_t i = bi * FB + e / FB, j = bj * FB + (e & (FB - 1));
    if (i >= dim || j >= dim) continue;
    long long s = S64[i * dim + j];
    for (int q = 0; q < nslab; ++q) s += slabs[(int64_t)q * dim * dim + i * dim + j];
    S64[i * dim + j] = s;
  }
}

// C from the exact integer pieces (one rounding); w = 1/scale or null.  One workgroup per
// upper 64-block: the block and (off the diagonal) its mirror, the mirror through LDS so
// both writes are row-contiguous.
__global__ __launch_bounds__(256) void cov_finalize_kernel(const int* __restrict__ slabs, int nslab,
                                                           const long long* __restrict__ S64, int64_t dim, int64_t n,
                                                           int gram, const long long* __restrict__ cvec,
                                                           const long long* __restrict__ R,
                                                           const unsigned long long* __restrict__ Q2,
                                                           const double* __restrict__ w, double* __restrict__ C) {
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bi > bj) return;
  __shared__ double tr[FB][FB + 1];
  const __int128 nn = n;
  const __int128 q = gram ? (__int128)(((unsigned __int128)Q2[1] << 64) | Q2[0]) : 0;
  const double den = gram ? (double)n * (double)n * (double)(n - 1) : (double)n * (double)(n - 1);
  // covariance numerator in int64 when it provably fits: |s| <= 128^2 n, |cvec| <= 128 n,
  // so n s and cvec_i cvec_j are at most 2^14 n^2 <= 2^60 for n <= 2^23, and their
  // difference fits; (double) of the same integer rounds identically from either width
  // (the int128 form goes through a software conversion, the int64 one is one instruction)
  const bool narrow = !gram && n <= (int64_t(1) << 23);
  for (int e = threadIdx.x; e < FB * FB; e += blockDim.x) {
    const int li = e / FB, lj = e & (FB - 1);
    const int64_t i = bi * FB + li, j = bj * FB + lj;
    if (i >= dim || j >= dim) continue;
    long long s = S64 ? S64[i * dim + j] : 0;
    for (int t = 0; t < nslab; ++t) s += slabs[(int64_t)t * dim * dim + i * dim + j];
    double v;
    if (narrow) {
      v = (double)((long long)n * s - cvec[i] * cvec[j]) / den;
    } else {
      const __int128 num = gram ? nn * nn * (__int128)s - nn * ((__int128)R[i] + R[j]) + q
                                : nn * (__int128)s - (__int128)cvec[i] * cvec[j];
      v = (double)num / den;
    }
    if (w) v *= w[i] * w[j];
    C[i * dim + j] = v;
    tr[lj][li] = v;
  }
  if (bi == bj) return;
  __syncthreads();
  for (int e = threadIdx.x; e < FB * FB; e += blockDim.x) {
    const int lj = e / FB, li = e & (FB - 1);
    const int64_t i = bi * FB + li, j = bj * FB + lj;
    if (i < dim && j < dim) C[j * dim + i] = tr[lj][li];
  }
}

// cov_finalize_kernel for dim % 4 == 0: four columns per thread — 16-byte slab loads (four
// times the bytes in flight per load instruction: the one-int form ran at ~2 TB/s) and
// 32-byte row stores; the per-element arithmetic is the same expression as above.
__global__ __launch_bounds__(256) void cov_finalize4_kernel(const int* __restrict__ slabs, int nslab,
                                                            const long long* __restrict__ S64, int64_t dim, int64_t n,
                                                            int gram, const long long* __restrict__ cvec,
                                                            const long long* __restrict__ R,
                                                            const unsigned long long* __restrict__ Q2,
                                                            const double* __restrict__ w, double* __restrict__ C) {
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bi > bj) return;
  __shared__ double tr[FB][FB + 1];
  const __int128 nn = n;
  const __int128 q = gram ? (__int128)(((unsigned __int128)Q2[1] << 64) | Q2[0]) : 0;
  const double den = gram ? (double)n * (double)n * (double)(n - 1) : (double)n * (double)(n - 1);
  const bool narrow = !gram && n <= (int64_t(1) << 23);
  for (int e = threadIdx.x; e < FB * FB / 4; e += blockDim.x) {
    const int li = e >> 4, lj = (e & 15) * 4;
    const int64_t i = bi * FB + li, j = bj * FB + lj;
    if (i >= dim || j >= dim) continue;
    long long s[4] = {0, 0, 0, 0};
    if (S64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] = S64[i * dim + j + u];
    }
    for (int t = 0; t < nslab; ++t) {
      const int4 v = *reinterpret_cast<const int4*>(slabs + (int64_t)t * dim * dim + i * dim + j);
      s[0] += v.x;
      s[1] += v.y;
      s[2] += v.z;
      s[3] += v.w;
    }
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t jj = j + u;
      if (narrow) {
        v[u] = (double)((long long)n * s[u] - cvec[i] * cvec[jj]) / den;
      } else {
        const __int128 num = gram ? nn * nn * (__int128)s[u] - nn * ((__int128)R[i] + R[jj]) + q
                                  : nn * (__int128)s[u] - (__int128)cvec[i] * cvec[jj];
        v[u] = (double)num / den;
      }
      if (w) v[u] *= w[i] * w[jj];
      tr[lj + u][li] = v[u];
    }
    *reinterpret_cast<double2*>(C + i * dim + j) = make_double2(v[0], v[1]);
    *reinterpret_cast<double2*>(C + i * dim + j + 2) = make_double2(v[2], v[3]);
  }
  if (bi == bj) return;
  __syncthreads();
  for (int e = threadIdx.x; e < FB * FB; e += blockDim.x) {
    const int lj = e / FB, li = e & (FB - 1);
    const int64_t i = bi * FB + li, j = bj * FB + lj;
    if (i < dim && j < dim) C[j * dim + i] = tr[lj][li];
  }
}

// ---------------------------------------------------------------- host side
int64_t cov_i8_kpad(int64_t K) { return (K + YK - 1) / YK * YK; }

int64_t cov_i8_order_bytes(int64_t dim) {
  const int64_t t = (dim + YT - 1) / YT;  // the 256 x 256 tiling has the most tiles
  return t * (t + 1) / 2 * (int64_t)sizeof(int2) + 64;
}

// SYRK tile columns: 384 (fewer bytes per MAC) unless the matrix is too small for the
// wider tile to pay (its diagonal tiles compute more of the lower triangle).
static int syrk_tile_cols(int64_t dim) {
  int tj = dim >= 2048 ? 384 : 256;
#ifdef EF_DIAGNOSTICS
  if (const char* e = getenv("EF_SYRK_TJ")) tj = atoi(e) == 384 ? 384 : 256;
#endif
  return tj;
}

// Tiles (256 rows x tj columns) that hold an upper-triangle element, in blocks of 8 row
// tiles x bw column tiles: consecutive list entries run together on one XCD and share their
// panels in its L2.  bw = 3 on the 384-column tiles measured 1% faster than 5 or 4
// (profiles/r04/syrk_block_width_ab.txt).
static std::vector<int2> syrk_tiles(int64_t dim, int tj) {
  const int nti = (int)((dim + YT - 1) / YT), ntj = (int)((dim + tj - 1) / tj);
#ifndef EF_SYRK_BH  // block shape override (variant builds: experiments)
  const int bw = tj == 384 ? 3 : 2048 / tj, bh = 8;
#else
  const int bw = EF_SYRK_BW, bh = EF_SYRK_BH;
#endif
  std::vector<int2> order;
  for (int bi = 0; bi < nti; bi += bh)
    for (int bj = 0; bj < ntj; bj += bw)
      for (int ti = bi; ti < bi + bh && ti < nti; ++ti)
        for (int tj_ = bj; tj_ < bj + bw && tj_ < ntj; ++tj_)
          if (std::min<int64_t>((int64_t)tj_ * tj + tj - 1, dim - 1) >= (int64_t)ti * YT) order.push_back(make_int2(ti, tj_));
  return order;
}

CovPlan cov_i8_plan(int64_t dim, int64_t K, int64_t slab_budget) {
  CovPlan p;
  p.nst = cov_i8_kpad(K) / YK;
  p.tj = syrk_tile_cols(dim);
  if (p.tj == 384) p.njb = 6;  // the 16x16x64 kernel (syrk16_i8_kernel<6>) on the 384-column tiles
#ifdef EF_DIAGNOSTICS  // EF_SYRK16 = 0: the 32x32x32 kernel; 5 | 6: the 16x16x64 kernel with 16 n-column wave blocks
  if (const char* e = getenv("EF_SYRK16")) {
    const int v = atoi(e);
    if (v == 0) p.njb = 0;
    if ((v == 5 || v == 6) && dim >= 2048) p.njb = v, p.tj = 64 * v;
  }
#endif
  p.ntiles = (int)syrk_tiles(dim, p.tj).size();
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (ncu < 1) ncu = 256;
  // slab memory budget (EF_OPT_COV_SLAB_BYTES, default 8 GiB = 8 splits at d = 16384); the
  // tests lower it to force the multi-pass schedule on small inputs
  const int64_t slab = dim * dim * (int64_t)sizeof(int);
  const int64_t budget = std::max<int64_t>(slab_budget, 1);
  int64_t smax = budget / std::max<int64_t>(slab, 1);
  smax = std::min<int64_t>(std::max<int64_t>(smax, 1), 64);
  const int64_t smin_total = (p.nst + kMaxSplitStages - 1) / kMaxSplitStages;
  p.passes = (int)((smin_total + smax - 1) / smax);
  p.stages_per_pass = (p.nst + p.passes - 1) / p.passes;
  const int64_t smin = std::max<int64_t>(1, (p.stages_per_pass + kMaxSplitStages - 1) / kMaxSplitStages);
  int64_t best = -1, best_s = smin;
  for (int64_t s = smin; s <= smax && s <= std::max<int64_t>(smin, p.stages_per_pass); ++s) {
    // one workgroup per CU: time ~ rounds x stages per item
    const int64_t rounds = ((int64_t)p.ntiles * s + ncu - 1) / ncu;
    const int64_t cost = rounds * ((p.stages_per_pass + s - 1) / s);
    if (best < 0 || cost < best) best = cost, best_s = s;
  }
  p.splits = (int)best_s;
  p.kps = (p.stages_per_pass + p.splits - 1) / p.splits;
  p.slab_elems = (int64_t)p.splits * dim * dim;
  return p;
}

hipError_t launch_cov_i8_prep(hipStream_t s, const uint8_t* X, int64_t n, int64_t d, bool gram, uint8_t* At,
                              unsigned long long* S1, unsigned long long* S2) {
  if (gram) {
    const int64_t nkb = cov_i8_kpad(d) / YK;
    const int64_t chunks = nkb * n * 4;
    const int64_t blocks = std::min<int64_t>((chunks + 255) / 256, 16384);
    hipLaunchKernelGGL(shift_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X, n, d, nkb, At);
    return hipGetLastError();
  }
  const int64_t nkb = cov_i8_kpad(n) / YK;
  if (S1 && S2) {
    if (!cov_i8_fused_stats(X, d)) return hipErrorInvalidValue;
    // <= 4096 blocks of 64 rows per workgroup keeps each thread's uint32 partials exact (the
    // LDS kernel adds its four sample quarters in 64 bits)
    int64_t gx = std::min<int64_t>(nkb, 128);
    gx = std::max<int64_t>(gx, (nkb + 4095) / 4096);
    bool lds = d % 256 == 0;
#ifdef EF_DIAGNOSTICS
    if (const char* v = std::getenv("EF_TRANSPOSE_LDS")) lds = lds && std::atoi(v) != 0;
#endif
    if (lds)
      hipLaunchKernelGGL(transpose_stats_lds_kernel, dim3((unsigned)gx, (unsigned)(d / 256)), dim3(256), 0, s, X, n,
                         d, nkb, At, S1, S2);
    else
      hipLaunchKernelGGL(transpose_stats_kernel, dim3((unsigned)gx, (unsigned)((d + 255) / 256)), dim3(256), 0, s, X,
                         n, d, nkb, At, S1, S2);
  } else {
    hipLaunchKernelGGL(shift_transpose_kernel, dim3((unsigned)nkb, (unsigned)((d + 63) / 64)), dim3(256), 0, s, X,
                       n, d, nkb, At);
  }
  return hipGetLastError();
}

bool cov_i8_fused_stats(const uint8_t* X, int64_t d) { return d % 4 == 0 && ((size_t)X & 3) == 0; }

hipError_t launch_cov_i8(hipStream_t s, const CovPlan& p, int64_t n, int64_t d, bool gram,
                         const unsigned long long* S1, const double* w, const uint8_t* At, int* slabs,
                         long long* S64, long long* cvec, long long* R, unsigned long long* Q2, void* order_dev,
                         double* C, hipEvent_t syrk_begin, hipEvent_t syrk_end) {
  const int64_t dim = gram ? n : d;
  const std::vector<int2> order = syrk_tiles(dim, p.tj);  // one H2D of the list
  if ((int)order.size() != p.ntiles) return hipErrorInvalidValue;
  hipError_t e = hipMemcpyAsync(order_dev, order.data(), order.size() * sizeof(int2), hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  const int nitems = p.ntiles * p.splits;
  const int grid = (nitems + 7) / 8 * 8;
  const int nfb = (int)((dim + FB - 1) / FB);
  if (p.passes > 1) {
    if (!S64) return hipErrorInvalidValue;
    e = hipMemsetAsync(S64, 0, (size_t)dim * dim * sizeof(long long), s);
    if (e != hipSuccess) return e;
  }
  if (syrk_begin) (void)hipEventRecord(syrk_begin, s);  // EF_KERNEL_SYRK: every pass of the SYRK
  for (int pass = 0; pass < p.passes; ++pass) {
    const int64_t st0 = (int64_t)pass * p.stages_per_pass;
    const int64_t st1 = std::min<int64_t>(p.nst, st0 + p.stages_per_pass);
#ifdef EF_DIAGNOSTICS  // EF_SYRK_PAIR=1: two stages per barrier (A/B)
    static const bool syrk_pair = [] { const char* v = getenv("EF_SYRK_PAIR"); return v && atoi(v) != 0; }();
    if (syrk_pair && p.njb == 6)
      hipLaunchKernelGGL((syrk16_i8_kernel<6, 4, false, true>), dim3((unsigned)grid), dim3(512), 0, s, At, dim, st0, st1,
                         p.kps, p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
    else
#endif
    if (p.njb == 6)
      hipLaunchKernelGGL((syrk16_i8_kernel<6, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, dim, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
#ifdef EF_DIAGNOSTICS
    else if (p.njb == 5)
      hipLaunchKernelGGL((syrk16_i8_kernel<5, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, dim, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
#endif
    else if (p.tj == 384)
      hipLaunchKernelGGL((syrk_i8_kernel<384, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, dim, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
    else
      hipLaunchKernelGGL((syrk_i8_kernel<256, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, dim, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
    if (p.passes > 1)
      hipLaunchKernelGGL(slab_accumulate_kernel, dim3((unsigned)nfb, (unsigned)nfb), dim3(256), 0, s, slabs,
                         p.splits, dim, S64);
  }
  if (syrk_end) (void)hipEventRecord(syrk_end, s);
  e = hipStreamSynchronize(s);  // the host list must outlive the copy
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(shifted_sums_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, S1, n, d, cvec);
  if (gram) {
    hipLaunchKernelGGL(rowdot_kernel, dim3((unsigned)n), dim3(256), 0, s, At, n, d, cvec, R);
    hipLaunchKernelGGL(sumsq128_kernel, dim3(1), dim3(256), 0, s, cvec, d, Q2);
  }
  bool vec4 = dim % 4 == 0;
#ifdef EF_DIAGNOSTICS
  if (const char* v = std::getenv("EF_FINALIZE4")) vec4 = vec4 && std::atoi(v) != 0;
#endif
  hipLaunchKernelGGL(vec4 ? cov_finalize4_kernel : cov_finalize_kernel, dim3((unsigned)nfb, (unsigned)nfb), dim3(256),
                     0, s, p.passes > 1 ? nullptr : slabs, p.passes > 1 ? 0 : p.splits, p.passes > 1 ? S64 : nullptr,
                     dim, n, gram ? 1 : 0, cvec, R, Q2, w, C);
  return hipGetLastError();
}

hipError_t launch_cov_i8_cross(hipStream_t s, const CovPlan& p, int64_t d, const uint8_t* At, int* slabs,
                               long long* S64, void* order_dev) {
  const std::vector<int2> order = syrk_tiles(d, p.tj);
  if ((int)order.size() != p.ntiles) return hipErrorInvalidValue;
  hipError_t e = hipMemcpyAsync(order_dev, order.data(), order.size() * sizeof(int2), hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(S64, 0, (size_t)d * d * sizeof(long long), s);
  if (e != hipSuccess) return e;
  const int nitems = p.ntiles * p.splits;
  const int grid = (nitems + 7) / 8 * 8;
  const int nfb = (int)((d + FB - 1) / FB);
  for (int pass = 0; pass < p.passes; ++pass) {
    const int64_t st0 = (int64_t)pass * p.stages_per_pass;
    const int64_t st1 = std::min<int64_t>(p.nst, st0 + p.stages_per_pass);
    if (p.njb == 6)
      hipLaunchKernelGGL((syrk16_i8_kernel<6, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, d, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
#ifdef EF_DIAGNOSTICS
    else if (p.njb == 5)
      hipLaunchKernelGGL((syrk16_i8_kernel<5, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, d, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
#endif
    else if (p.tj == 384)
      hipLaunchKernelGGL((syrk_i8_kernel<384, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, d, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
    else
      hipLaunchKernelGGL((syrk_i8_kernel<256, 4>), dim3((unsigned)grid), dim3(512), 0, s, At, d, st0, st1, p.kps,
                         p.ntiles, nitems, static_cast<const int2*>(order_dev), slabs);
    hipLaunchKernelGGL(slab_accumulate_kernel, dim3((unsigned)nfb, (unsigned)nfb), dim3(256), 0, s, slabs, p.splits,
                       d, S64);
  }
  return hipStreamSynchronize(s);  // the host list must outlive the copy
}

hipError_t launch_cov_from_cross(hipStream_t s, const long long* S64, const unsigned long long* S1, int64_t n,
                                 int64_t d, const double* w, long long* cvec, double* C) {
  const int nfb = (int)((d + FB - 1) / FB);
  hipLaunchKernelGGL(shifted_sums_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, S1, n, d, cvec);
  hipLaunchKernelGGL(d % 4 == 0 ? cov_finalize4_kernel : cov_finalize_kernel, dim3((unsigned)nfb, (unsigned)nfb),
                     dim3(256), 0, s, nullptr, 0, S64, d, n, 0, cvec, nullptr, nullptr, w, C);
  return hipGetLastError();
}

// The fit's digit-pair products (ef_cq_i8.hip): 64 row blocks of 256 x 24 items at C3
hipError_t launch_oz_syrk16(hipStream_t s, const uint8_t* Z, int64_t dim, int64_t R, int* I, bool med) {
  if (dim % 2048 != 0) return hipErrorInvalidValue;
  const int nrb = (int)(dim / YT);
  const int nitems = nrb * oz_blocks(med);  // a multiple of 8
  if (med)
    hipLaunchKernelGGL((syrk16_i8_kernel<4, 4, true, false, true>), dim3((unsigned)nitems), dim3(512), 0, s, Z, R,
                       (int64_t)0, dim / YK, dim, nrb / 8, nitems, nullptr, I);
  else
    hipLaunchKernelGGL((syrk16_i8_kernel<4, 4, true>), dim3((unsigned)nitems), dim3(512), 0, s, Z, R, (int64_t)0,
                       dim / YK, dim, nrb / 8, nitems, nullptr, I);
  return hipGetLastError();
}

}  // namespace ef
