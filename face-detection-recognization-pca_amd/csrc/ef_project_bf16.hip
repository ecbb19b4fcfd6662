// bf16 probe projection (BASELINE.json config 5: 256x256 faces, k = 512, "bf16 projection
// (CDNA4 bf16 MFMA) with fp32 distance accumulate").
//
// f = (p - mean).W is evaluated as  (p - round(mean)).W16  -  (mean - round(mean)).W
//   * p - round(mean) is an integer in [-255, 255] for uint8 pixels, exact in bf16, so the
//     only rounding of the GEMM inputs is W -> W16 (bf16, round-to-nearest-even);
//   * the correction row (mean - round(mean)).W is computed once per model in fp64;
//   * accumulation is fp32 on v_mfma_f32_32x32x16_bf16; the features and everything
//     after them (gallery search, arg-best) stay fp32 / fp64-resolved.
// Error vs the fp32 projection: |f16 - f| <= 2^-8 * sum_px |p - round(mean)| |W| (stated
// and tested in tests/test_gpu_project.py).
//
// GEMM M = probes, N = components (128-column tiles over gridDim.z), K = pixels, split-K
// over gridDim.y into fp32 slabs reduced by project_reduce_kernel (ef_project.hip), the
// same slab contract as the fp32 kernel.  Workgroup tile 128 probes x 128 components,
// 4 waves of 64 x 64, BK = 32 pixels per stage (two 16-deep MFMA steps), LDS rows padded
// to 80 B so the ds_read_b128 fragment reads are conflict-free.
#include "ef_internal.hpp"

namespace ef {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int HM = 128;      // probes per workgroup
constexpr int HN = 128;      // components per workgroup
constexpr int HK = 32;       // pixels per stage
constexpr int HS = HK + 8;   // LDS row stride in bf16 elements (80 B)

__device__ __forceinline__ unsigned bf16_bits(float x) {  // round to nearest even (finite x)
  const unsigned u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ unsigned pack2(float lo, float hi) { return bf16_bits(lo) | (bf16_bits(hi) << 16); }

template <int PDT, bool VEC>
__global__ __launch_bounds__(256, 2) void project_bf16_kernel(const void* __restrict__ Pv, int64_t b, int64_t d,
                                                              const float* __restrict__ mean_r,
                                                              const unsigned short* __restrict__ Wt16, int ldw,
                                                              float* __restrict__ part, int64_t bpad,
                                                              int64_t pix_per_split) {
  __shared__ __attribute__((aligned(16))) unsigned short sA[2][HM * HS];
  __shared__ __attribute__((aligned(16))) unsigned short sB[2][HN * HS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * HM;
  const int col0 = blockIdx.z * HN;
  const int64_t k_beg = (int64_t)blockIdx.y * pix_per_split;
  const int64_t k_end = k_beg + pix_per_split < d ? k_beg + pix_per_split : d;
  const int nsteps = (int)((k_end - k_beg + HK - 1) / HK);

  // staging: thread -> (row | column, 16-pixel half)
  const int sr = tid >> 1, sh = (tid & 1) * 16;
  uint4 av[2], bv[2];

  auto load_stage = [&](int step) {
    const int64_t px0 = k_beg + (int64_t)step * HK + sh;
    const int64_t row = m0 + sr;
    float v[16];
    if constexpr (PDT == EF_U8) {
      const uint8_t* P = reinterpret_cast<const uint8_t*>(Pv);
      if (VEC && row < b && px0 + 16 <= k_end) {
        const uint4 raw = *reinterpret_cast<const uint4*>(P + row * d + px0);
        const unsigned w4[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = (float)((w4[j >> 2] >> (8 * (j & 3))) & 0xffu);
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = (row < b && px0 + j < k_end) ? (float)P[row * d + px0 + j] : 0.f;
      }
    } else {
      const float* P = reinterpret_cast<const float*>(Pv);
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = (row < b && px0 + j < k_end) ? P[row * d + px0 + j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (row < b && px0 + j < k_end) v[j] -= mean_r[px0 + j];
    av[0] = make_uint4(pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7]));
    av[1] = make_uint4(pack2(v[8], v[9]), pack2(v[10], v[11]), pack2(v[12], v[13]), pack2(v[14], v[15]));
    // W16 is [ldw][d] (pixels contiguous per component): 32 B per thread
    const unsigned short* wrow = Wt16 + (int64_t)(col0 + sr) * d;
    if (VEC && px0 + 16 <= k_end) {
      bv[0] = *reinterpret_cast<const uint4*>(wrow + px0);
      bv[1] = *reinterpret_cast<const uint4*>(wrow + px0 + 8);
    } else {
      unsigned w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned lo = px0 + 2 * j < k_end ? wrow[px0 + 2 * j] : 0u;
        const unsigned hi = px0 + 2 * j + 1 < k_end ? wrow[px0 + 2 * j + 1] : 0u;
        w[j] = lo | (hi << 16);
      }
      bv[0] = make_uint4(w[0], w[1], w[2], w[3]);
      bv[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
  };
  auto store_stage = [&](int buf) {
    *reinterpret_cast<uint4*>(&sA[buf][sr * HS + sh]) = av[0];
    *reinterpret_cast<uint4*>(&sA[buf][sr * HS + sh + 8]) = av[1];
    *reinterpret_cast<uint4*>(&sB[buf][sr * HS + sh]) = bv[0];
    *reinterpret_cast<uint4*>(&sB[buf][sr * HS + sh + 8]) = bv[1];
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  if (nsteps > 0) {
    load_stage(0);
    store_stage(0);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const bool more = st + 1 < nsteps;
    if (more) load_stage(st + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // lane (r, h) holds A[r][16s + 8h + j], B[16s + 8h + j][r]
      bf16x8 a[2], w[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&sA[buf][(wm * 64 + i * 32 + c32) * HS + 16 * s + 8 * h]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        w[j] = *reinterpret_cast<const bf16x8*>(&sB[buf][(wn * 64 + j * 32 + c32) * HS + 16 * s + 8 * h]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], w[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_stage(buf ^ 1);
    __syncthreads();
  }

  float* out = part + (int64_t)blockIdx.y * bpad * ldw + col0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[row * ldw + wn * 64 + j * 32 + c32] = acc[i][j][r];
      }
}

// ---------------------------------------------------------------------------------
// Wide form for uint8 probes (the config-5 shape: 4096 probes x 65536 pixels x k = 512).
// The 128 x 128 kernel above converts every pixel once per 128-column tile with ~6 VALU
// instructions per pixel and re-reads W for every 128 probes: it runs VALU-bound at ~9 %
// of the bf16 peak.  Here a workgroup of 8 waves owns 256 probes x NT components (NT =
// 256: each wave 64 x 128, eight 32x32 accumulators = 128 AGPRs), so each (probe, pixel)
// is converted at most ldw / 256 times and each W element is read once per 256 probes:
//   per 32-pixel stage: 8 KiB of uint8 pixels + NT x 64 B of W16 from L2 for 2 x 8
//   MFMAs per wave (512 cycles per SIMD at 2 waves/SIMD) = 24 B/clk/CU at NT = 256;
//   conversion p - round(mean) -> bf16 is exact for uint8 (|p - mr| <= 255) and costs
//   ~2 VALU instructions per pixel: v_cvt_f32_ubyte, a packed subtract, a v_perm of the
//   two high halves (bf16 truncation of an exactly representable value).
// K splits over gridDim.y (fp32 slabs, the project_reduce_kernel contract); the grid is
// XCD-aware: the workgroups of one K split are dealt to one XCD so that split's W and
// probe slices stream through that XCD's L2 once.
constexpr int WM = 256;  // probes per workgroup (wide form)
constexpr int WKS = 64;  // pixels per stage (wide form)

template <int NT, int WK>
__global__ __launch_bounds__(512, 1) void project_bf16_wide_kernel(const uint8_t* __restrict__ P, int64_t b, int64_t d,
                                                                   const uint8_t* __restrict__ mean_u8,
                                                                   const unsigned short* __restrict__ Wt16, int ldw,
                                                                   float* __restrict__ part, int64_t bpad,
                                                                   int64_t pps, int mt, int nt, int ns) {
  constexpr int WN = NT / 2;       // components per wave (4 x 2 waves)
  constexpr int JB = WN / 32;      // 32-column blocks per wave
  constexpr int WS = WK + 8;       // LDS row stride (bf16): 16-B pad keeps ds_read_b128 conflict-free
  constexpr int PT = WK / 2;       // pixels per thread per stage (two threads per row)
  constexpr int NV = PT / 16;      // uint4 of raw pixels per thread per stage
  __shared__ __attribute__((aligned(16))) unsigned short sA[2][WM * WS];
  __shared__ __attribute__((aligned(16))) unsigned short sB[2][NT * WS];

  // XCD-aware deal: consecutive block ids go round-robin over the 8 XCDs; give XCD x the
  // contiguous run [x * per, (x + 1) * per) of (split, m-tile, n-tile) items, split-major
  // (the grid is total rounded up to a multiple of 8; the few padding workgroups exit)
  const int total = mt * nt * ns;
  const int per = (total + 7) / 8;
  const int item = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (item >= total) return;
  const int split = item / (mt * nt);
  const int rem = item - split * (mt * nt);
  const int mi = rem / nt, ni = rem - (rem / nt) * nt;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)mi * WM;
  const int col0 = ni * NT;
  const int64_t k_beg = (int64_t)split * pps;
  const int64_t k_end = k_beg + pps < d ? k_beg + pps : d;
  const int nsteps = (int)((k_end - k_beg) / WK);  // host guarantees whole stages

  // staging: A: thread -> (probe row tid >> 1, 16-pixel half); B: NT / 256 (row, half) pairs.
  // Register pipeline two stages deep: the raw pixels, round(mean) bytes and W16 of stage
  // st + 2 are loaded while stage st's MFMAs run and stage st + 1 is converted into LDS,
  // so each global load has two stages of MFMA time (~2k cycles) to arrive.
  const int sr = tid >> 1, sh = (tid & 1) * PT;
  const int64_t arow = m0 + sr;
  const bool arow_ok = arow < b;
  const uint8_t* pa = P + (arow_ok ? arow : 0) * d + sh;
  constexpr int BR = NT >= 256 ? NT / 256 : 1;  // W (row, half) pairs per thread
  const bool bload = NT >= 256 || tid < 2 * NT;   // NT = 128: the first 256 threads
  struct Raw {
    uint4 p[NV], m[NV], w[BR][2 * NV];
  };
  auto load_raw = [&](int step, Raw& r) {
    const int64_t px0 = k_beg + (int64_t)step * WK;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      r.p[v] = arow_ok ? *reinterpret_cast<const uint4*>(pa + px0 + 16 * v) : make_uint4(0, 0, 0, 0);
      r.m[v] = *reinterpret_cast<const uint4*>(mean_u8 + px0 + sh + 16 * v);
    }
    if (bload) {
#pragma unroll
      for (int q = 0; q < BR; ++q) {
        const unsigned short* wrow = Wt16 + (int64_t)(col0 + sr + 256 * q) * d + px0 + sh;
#pragma unroll
        for (int v = 0; v < 2 * NV; ++v) r.w[q][v] = *reinterpret_cast<const uint4*>(wrow + 8 * v);
      }
    }
  };
  // p - round(mean) -> bf16 (exact: |p - mr| <= 255), the bf16 being the high half of the
  // exactly representable fp32 value; stored with W16 into LDS buffer buf
  auto convert_store = [&](const Raw& r, int buf) {
#pragma unroll
   for (int v = 0; v < NV; ++v) {
    const unsigned pw[4] = {r.p[v].x, r.p[v].y, r.p[v].z, r.p[v].w};
    const unsigned mw[4] = {r.m[v].x, r.m[v].y, r.m[v].z, r.m[v].w};
    unsigned pk[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned w = pw[q], m = mw[q];
      const float f0 = (float)(w & 0xffu) - (float)(m & 0xffu);
      const float f1 = (float)((w >> 8) & 0xffu) - (float)((m >> 8) & 0xffu);
      const float f2 = (float)((w >> 16) & 0xffu) - (float)((m >> 16) & 0xffu);
      const float f3 = (float)(w >> 24) - (float)(m >> 24);
      pk[2 * q] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
      pk[2 * q + 1] = __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u);
    }
    // padded rows past b must be zero (their slab rows are summed like the others)
    const uint4 a0 = arow_ok ? make_uint4(pk[0], pk[1], pk[2], pk[3]) : make_uint4(0, 0, 0, 0);
    const uint4 a1 = arow_ok ? make_uint4(pk[4], pk[5], pk[6], pk[7]) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(&sA[buf][sr * WS + sh + 16 * v]) = a0;
    *reinterpret_cast<uint4*>(&sA[buf][sr * WS + sh + 16 * v + 8]) = a1;
   }
    if (bload) {
#pragma unroll
      for (int q = 0; q < BR; ++q)
#pragma unroll
        for (int v = 0; v < 2 * NV; ++v) *reinterpret_cast<uint4*>(&sB[buf][(sr + 256 * q) * WS + sh + 8 * v]) = r.w[q][v];
    }
  };

  f32x16 acc[2][JB];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[i][j] = f32x16{};

  Raw r0, r1;
  if (nsteps > 0) load_raw(0, r0);
  if (nsteps > 1) load_raw(1, r1);
  if (nsteps > 0) convert_store(r0, 0);
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    // r1 holds stage st + 1 (loaded last iteration); refill r0 with stage st + 2
    if (st + 2 < nsteps) load_raw(st + 2, r0);
#pragma unroll
    for (int s = 0; s < WK / 16; ++s) {  // lane (r, h) holds A[r][16s + 8h + j], B[16s + 8h + j][r]
      bf16x8 a[2], w[JB];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&sA[buf][(wm * 64 + i * 32 + c32) * WS + 16 * s + 8 * h]);
#pragma unroll
      for (int j = 0; j < JB; ++j)
        w[j] = *reinterpret_cast<const bf16x8*>(&sB[buf][(wn * WN + j * 32 + c32) * WS + 16 * s + 8 * h]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], w[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nsteps) convert_store(r1, buf ^ 1);
    __syncthreads();
    r1 = r0;
  }

  float* out = part + (int64_t)split * bpad * ldw + col0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[row * ldw + wn * WN + j * 32 + c32] = acc[i][j][r];
      }
}

// ---------------------------------------------------------------------------------
// Fragment form (round 6): the wide kernel above staged BOTH operands
// through LDS.  Per 32x32x16 MFMA a wave read 768 B of fragments from LDS (2 A + 4 B per
// 8 MFMAs), which with the W16 and pixel stores kept the LDS busy ~1,900 of the 2,048
// MFMA cycles of a stage (MFMA busy 41 %), and each probe tile was read by two column tiles.
// Here W16 is kept in MFMA-fragment-native order (`Wf`, built once per model by
// bf16_frag_kernel): the 16 B a lane needs for one B fragment sit at ((ct * KB + kb) * 64
// + lane) * 16 B, so a wave's fragment is ONE contiguous 1 KiB global_load_dwordx4 straight
// into VGPRs, with no LDS round trip, prefetched four k-steps ahead in a register ring.
// Only the probes go through LDS (they need the p - round(mean) conversion, done once per
// pixel): a workgroup owns RM = 128 * MG probes x NT components, NT = 64 * NG, MG * NG = 8
// waves; each wave 128 probes x 64 components (4 x 2 accumulators of 32 x 32, 128 AGPRs),
// per k-step 4 A fragments from LDS (512 B per MFMA, 1,024 of the 2,048 cycles) and 2 B
// fragments from L2 (32 B/clk/CU).  At NT = ldw = 512 every probe tile is read once.
// Barriers are LDS-only (lgkmcnt(0) + s_barrier), so the B ring's loads stay in flight.
__device__ __forceinline__ void frag_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ML: round(mean)'s bytes of the split (pps <= kFragMeanLds) are copied into LDS once, so
// the stage loop issues only pixel and fragment loads (the 512 threads' per-stage mean loads
// were 2 of every 20 vector-memory instructions, all for the same 128 bytes).
constexpr int kFragMeanLds = 16384;
// NW = 4: a 256-thread workgroup (one wave per SIMD, 128 probes x 256 components at
// NT = 256), two per CU, so one workgroup's barrier is covered by the other's MFMAs.
template <int NT, int WK, bool ML, int NW = 8>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void project_bf16_frag_kernel(const uint8_t* __restrict__ P, int64_t b, int64_t d,
                                                                   const uint8_t* __restrict__ mean_u8,
                                                                   const uint4* __restrict__ Wf, int ldw,
                                                                   float* __restrict__ part, int64_t bpad,
                                                                   int64_t pps, int mt, int nt, int ns) {
  constexpr int NG = NT / 64;          // wave columns (64 components each)
  constexpr int MG = NW / NG;          // wave rows (128 probes each)
  constexpr int NTH = 64 * NW;         // threads
  constexpr int RM = 128 * MG;         // probes per workgroup
  constexpr int SUB = WK / 16;         // MFMA k-steps per stage
  constexpr int WS = WK + 8;           // LDS row stride (bf16): conflict-free ds_read_b128 / ds_write_b128
  constexpr int PT = RM * WK / NTH;    // pixels per thread per stage
  constexpr int TPR = WK / PT;         // threads per probe row
  constexpr int NV = PT / 16;          // uint4 of raw pixels per thread per stage
  constexpr int RD = 4;                // B ring depth (k-steps in flight)
  static_assert(NG * MG == NW && PT % 16 == 0 && TPR >= 1 && SUB % RD == 0, "frag tile");
  __shared__ __attribute__((aligned(16))) unsigned short sA[2][RM * WS];
  __shared__ __attribute__((aligned(16))) uint8_t sMean[ML ? kFragMeanLds : 16];

  // XCD-aware deal (as the wide kernel): XCD x takes the contiguous run of (split, m-tile,
  // n-tile) items [x * per, (x + 1) * per), split-major, so one K split's Wf slice streams
  // through one XCD's L2 for all its probe tiles
  const int total = mt * nt * ns;
  const int per = (total + 7) / 8;
  const int item = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (item >= total) return;
  const int split = item / (mt * nt);
  const int rem = item - split * (mt * nt);
  const int mi = rem / nt, ni = rem - (rem / nt) * nt;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int ng = wave % NG, mg = wave / NG;
  const int64_t m0 = (int64_t)mi * RM;
  const int col0 = ni * NT;
  const int64_t k_beg = (int64_t)split * pps;
  const int64_t k_end = k_beg + pps < d ? k_beg + pps : d;
  const int nsteps = (int)((k_end - k_beg) / WK);  // host guarantees whole stages
  const int nsub = nsteps * SUB;

  // probe staging: thread -> (row tid / TPR, PT pixels); raw bytes two stages ahead
  const int sr = tid / TPR, sh = (tid % TPR) * PT;
  const int64_t arow = m0 + sr;
  const bool arow_ok = arow < b;
  const uint8_t* pa = P + (arow_ok ? arow : 0) * d + sh;
  struct Raw {
    uint4 p[NV], m[NV];
  };
  // Every load in the main loop is unconditional (rows past b read row 0 and are zeroed
  // at conversion; steps past the end re-read the last one): a load under a branch makes
  // the compiler's vmcnt accounting path-dependent, and it then waited for ALL loads in
  // flight (the just-issued HBM pixel loads too) before each stage's first MFMA.
  auto load_raw = [&](int step, Raw& r) {
    const int64_t px0 = k_beg + (int64_t)step * WK;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      r.p[v] = *reinterpret_cast<const uint4*>(pa + px0 + 16 * v);
      if constexpr (!ML) r.m[v] = *reinterpret_cast<const uint4*>(mean_u8 + px0 + sh + 16 * v);
    }
  };
  auto convert_store = [&](const Raw& r, int step, int buf) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const unsigned pw[4] = {r.p[v].x, r.p[v].y, r.p[v].z, r.p[v].w};
      uint4 mq = r.m[v];
      if constexpr (ML) mq = *reinterpret_cast<const uint4*>(sMean + step * WK + sh + 16 * v);
      const unsigned mw[4] = {mq.x, mq.y, mq.z, mq.w};
      unsigned pk[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned w = pw[q], m = mw[q];
        const float f0 = (float)(w & 0xffu) - (float)(m & 0xffu);
        const float f1 = (float)((w >> 8) & 0xffu) - (float)((m >> 8) & 0xffu);
        const float f2 = (float)((w >> 16) & 0xffu) - (float)((m >> 16) & 0xffu);
        const float f3 = (float)(w >> 24) - (float)(m >> 24);
        pk[2 * q] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
        pk[2 * q + 1] = __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u);
      }
      const uint4 a0 = arow_ok ? make_uint4(pk[0], pk[1], pk[2], pk[3]) : make_uint4(0, 0, 0, 0);
      const uint4 a1 = arow_ok ? make_uint4(pk[4], pk[5], pk[6], pk[7]) : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(&sA[buf][sr * WS + sh + 16 * v]) = a0;
      *reinterpret_cast<uint4*>(&sA[buf][sr * WS + sh + 16 * v + 8]) = a1;
    }
  };

  // B fragments: wave columns ct0, ct0 + 1 (32 each); k-step g of this split is fragment
  // row kb0 + g
  const int64_t KB = d / 16;
  const int64_t ct0 = (col0 + ng * 64) / 32;
  const uint4* wb0 = Wf + (ct0 * KB + k_beg / 16) * 64 + lane;
  const uint4* wb1 = wb0 + KB * 64;
  uint4 ring[RD][2];
  auto load_b = [&](int g, uint4* dst) {
    dst[0] = wb0[(int64_t)g * 64];
    dst[1] = wb1[(int64_t)g * 64];
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  // (the host guarantees nsteps >= 1: splits are whole 64-pixel stages of d % 64 == 0)
  Raw r0, r1;
  if constexpr (ML) {
    for (int i = tid * 16; i < (int)(k_end - k_beg); i += NTH * 16)
      *reinterpret_cast<uint4*>(sMean + i) = *reinterpret_cast<const uint4*>(mean_u8 + k_beg + i);
    __syncthreads();
  }
  load_raw(0, r0);
#pragma unroll
  for (int g = 0; g < RD; ++g) load_b(g < nsub ? g : nsub - 1, ring[g]);
  load_raw(nsteps > 1 ? 1 : 0, r1);
  convert_store(r0, 0, 0);
  frag_lds_barrier();
  const unsigned short* arow_lds = &sA[0][(mg * 128 + c32) * WS + 8 * h];
  auto read_a = [&](int buf, int s, bf16x8 (&a)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(arow_lds + buf * (RM * WS) + i * 32 * WS + 16 * s);
  };
  // Order held by sched_barrier: without it the scheduler sank every ring refill below the
  // stage's last MFMA (next to the barrier), so each stage's first MFMA waited out a full
  // L2 round trip.  Per k-step: the k-step's A fragments are read, its 8 MFMAs issue, then
  // its ring slot is refilled four k-steps ahead.  The raw pixel registers alternate
  // between two sets by stage parity (the loop is unrolled by two), so no register copy
  // has to wait for the loads issued at the stage's start.
  auto run_stage = [&](int st, Raw& ld, Raw& cv) {
    const int buf = st & 1;
    load_raw(st + 2 < nsteps ? st + 2 : nsteps - 1, ld);
    bf16x8 acur[4], anxt[4];
    read_a(buf, 0, acur);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < SUB; ++s) {  // lane (r, h) holds A[r][16s + 8h + j], B[16s + 8h + j][r]
      if (s + 1 < SUB) read_a(buf, s + 1, anxt);
      // the next k-step's A reads issue before this k-step's MFMAs (8 MFMAs = 256 cycles of
      // cover for the LDS latency; the scheduler otherwise sank them below 7 of the 8)
      __builtin_amdgcn_sched_barrier(0);
      const int slot = s % RD;
      bf16x8 w0, w1;
      __builtin_memcpy(&w0, &ring[slot][0], 16);
      __builtin_memcpy(&w1, &ring[slot][1], 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[i], w0, acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(acur[i], w1, acc[i][1], 0, 0, 0);
      }
      const int g = st * SUB + s + RD;
      load_b(g < nsub ? g : nsub - 1, ring[slot]);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < SUB) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acur[i] = anxt[i];
      }
    }
    convert_store(cv, st + 1 < nsteps ? st + 1 : st, buf ^ 1);  // stage st + 1 (after the last: unread)
    frag_lds_barrier();
  };
  int st = 0;
  for (; st + 1 < nsteps; st += 2) {
    run_stage(st, r0, r1);
    run_stage(st + 1, r1, r0);
  }
  if (st < nsteps) run_stage(st, r0, r1);

  float* out = part + (int64_t)split * bpad * ldw + col0 + ng * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + mg * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < bpad) out[row * ldw + j * 32 + c32] = acc[i][j][r];
      }
}

// Wf[(ct * KB + kb) * 64 + lane] (16 B) = W16[32 ct + (lane & 31)][16 kb + 8 (lane >> 5) .. + 8]
__global__ void bf16_frag_kernel(const unsigned short* __restrict__ Wt16, int64_t d, int64_t total,
                                 uint4* __restrict__ Wf) {
  const int64_t KB = d / 16;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int ln = (int)(idx & 63);
    const int64_t rest = idx >> 6;
    const int64_t kb = rest % KB, ct = rest / KB;
    Wf[idx] = *reinterpret_cast<const uint4*>(Wt16 + (ct * 32 + (ln & 31)) * d + kb * 16 + 8 * (ln >> 5));
  }
}

bool bf16_frag_supported(int64_t d, int ldw) { return d % 64 == 0 && ldw % 128 == 0; }

hipError_t launch_bf16_frag(hipStream_t s, const unsigned short* Wt16, int64_t d, int ldw, void* Wf) {
  if (!bf16_frag_supported(d, ldw)) return hipErrorInvalidValue;
  const int64_t total = (int64_t)(ldw / 32) * (d / 16) * 64;
  hipLaunchKernelGGL(bf16_frag_kernel, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 65536)), dim3(256), 0, s,
                     Wt16, d, total, static_cast<uint4*>(Wf));
  return hipGetLastError();
}

// Wt16[c][px] = bf16(W[px][c]) (32 x 32 tiles through LDS), mean_r = round(mean).
__global__ void bf16_model_kernel(const float* __restrict__ W, const float* __restrict__ mean, int64_t d, int ldw,
                                  unsigned short* __restrict__ Wt16, float* __restrict__ mean_r) {
  __shared__ float t[32][33];
  const int64_t p0 = (int64_t)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int64_t px = p0 + r;
    t[r][tx] = px < d ? W[px * ldw + c0 + tx] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t px = p0 + tx;
    if (px < d) Wt16[(int64_t)(c0 + r) * d + px] = (unsigned short)bf16_bits(t[tx][r]);
  }
  if (blockIdx.y == 0 && threadIdx.x < 32 && p0 + threadIdx.x < d) mean_r[p0 + threadIdx.x] = rintf(mean[p0 + threadIdx.x]);
}

// corr_part[chunk][c] = sum over the chunk's pixels of (mean - round(mean)) W[px][c] (fp64).
__global__ void bf16_corr_kernel(const float* __restrict__ W, const float* __restrict__ mean, int64_t d, int ldw,
                                 int64_t chunk, double* __restrict__ corr_part) {
  const int c = threadIdx.x + blockIdx.y * blockDim.x;
  if (c >= ldw) return;
  const int64_t a = (int64_t)blockIdx.x * chunk;
  const int64_t e = a + chunk < d ? a + chunk : d;
  double s = 0.0;
  for (int64_t px = a; px < e; ++px) s += ((double)mean[px] - (double)rintf(mean[px])) * (double)W[px * ldw + c];
  corr_part[(int64_t)blockIdx.x * ldw + c] = s;
}

__global__ void bf16_corr_sum_kernel(const double* __restrict__ corr_part, int nchunk, int ldw, float* __restrict__ corr) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ldw) return;
  double s = 0.0;
  for (int z = 0; z < nchunk; ++z) s += corr_part[(int64_t)z * ldw + c];
  corr[c] = (float)s;
}

hipError_t launch_bf16_model(hipStream_t s, const float* W, const float* mean, int64_t d, int ldw,
                             unsigned short* Wt16, float* mean_r, float* corr, double* corr_part, int nchunk) {
  hipLaunchKernelGGL(bf16_model_kernel, dim3((unsigned)((d + 31) / 32), (unsigned)(ldw / 32)), dim3(256), 0, s, W,
                     mean, d, ldw, Wt16, mean_r);
  const int64_t chunk = (d + nchunk - 1) / nchunk;
  hipLaunchKernelGGL(bf16_corr_kernel, dim3((unsigned)nchunk, (unsigned)((ldw + 127) / 128)), dim3(128), 0, s, W,
                     mean, d, ldw, chunk, corr_part);
  hipLaunchKernelGGL(bf16_corr_sum_kernel, dim3((unsigned)((ldw + 127) / 128)), dim3(128), 0, s, corr_part, nchunk,
                     ldw, corr);
  return hipGetLastError();
}

// The wide form needs uint8 probes, whole 32-pixel stages per split, 16-byte aligned rows.
static bool bf16_wide_ok(int p_dtype, const void* P, int64_t d, int ldw, const uint8_t* mean_u8) {
  return mean_u8 && p_dtype == EF_U8 && d % WKS == 0 && ldw % 128 == 0 && (reinterpret_cast<uintptr_t>(P) & 15) == 0;
}

// round(mean) as bytes (the wide kernel's subtrahend); *bad counts entries outside 0..255
// (then the wide kernel is not used: its byte subtrahend could not represent them)
__global__ void mean_u8_kernel(const float* __restrict__ mean_r, int64_t d, uint8_t* __restrict__ out,
                               int* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d) return;
  const float v = mean_r[i];
  if (!(v >= 0.f && v <= 255.f)) atomicAdd(bad, 1);
  out[i] = (uint8_t)fminf(fmaxf(v, 0.f), 255.f);
}

hipError_t launch_mean_u8(hipStream_t s, const float* mean_r, int64_t d, uint8_t* out, int* bad) {
  hipLaunchKernelGGL(mean_u8_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, mean_r, d, out, bad);
  return hipGetLastError();
}

static bool use_frag(const void* Wf) {
#ifdef EF_DIAGNOSTICS  // EF_PROJ_FRAG=0: round 5's wide kernel (A/B)
  if (const char* e = getenv("EF_PROJ_FRAG")) return Wf && atoi(e) != 0;
#endif
  return Wf != nullptr;
}
// Frag-form launch shape: column tile NT (the widest of 512 / 256 / 128 dividing ldw),
// waves per workgroup NW (8, or 4 with two workgroups per CU), pixels per stage WK (128 at
// NT = 512: half the barriers per pixel; the 256 / 128-column forms would spill or exceed
// the LDS at 128), probes per workgroup RM, workgroups per CU.
struct FragCfg {
  int NT, NW, WK, RM, per_cu;
};
static FragCfg frag_cfg(int ldw, int64_t d) {
  FragCfg c;
  c.NT = ldw % 512 == 0 ? 512 : ldw % 256 == 0 ? 256 : 128;
  c.NW = 8;
#ifdef EF_DIAGNOSTICS  // EF_PROJ_NW=4: 256-thread workgroups of 128 x 256, two per CU (A/B)
  if (const char* e = getenv("EF_PROJ_NW"))
    if (atoi(e) == 4 && ldw % 256 == 0) c.NT = 256, c.NW = 4;
#endif
  c.WK = (c.NT == 512 && c.NW == 8 && d % 128 == 0) ? 128 : 64;  // (every split whole stages)
#ifdef EF_DIAGNOSTICS  // EF_PROJ_WK=64: 64-pixel stages at 512 columns (A/B)
  if (const char* e = getenv("EF_PROJ_WK"))
    if (atoi(e) == 64) c.WK = 64;
#endif
  c.RM = 128 * (c.NW / (c.NT / 64));
  c.per_cu = c.NW == 4 ? 2 : 1;
  return c;
}

int project_bf16_nsplit(int p_dtype, const void* P, const uint8_t* mean_u8, const void* Wf, int64_t bpad, int64_t d,
                        int ldw, int64_t* pix_per_split) {
  const int64_t steps = (d + HK - 1) / HK;
  if (bf16_wide_ok(p_dtype, P, d, ldw, mean_u8) && use_frag(Wf)) {
    const FragCfg fc = frag_cfg(ldw, d);
    const int FWK = fc.WK;
    const int64_t wsteps = d / FWK;
    const int64_t tiles = (bpad + fc.RM - 1) / fc.RM * (ldw / fc.NT);
    int64_t ns = (256 * fc.per_cu + tiles - 1) / tiles;  // every CU busy
    if (ns > wsteps) ns = wsteps;
    if (ns < 1) ns = 1;
    while ((tiles * ns) % 8 != 0 && ns < wsteps) ++ns;
    const int64_t steps_per = (wsteps + ns - 1) / ns;
    *pix_per_split = steps_per * FWK;
    return (int)((d + *pix_per_split - 1) / *pix_per_split);
  }
  if (bf16_wide_ok(p_dtype, P, d, ldw, mean_u8)) {
    const int64_t wsteps = d / WKS;
    const int nt = ldw % 256 == 0 ? ldw / 256 : ldw / 128;
    const int64_t tiles = (bpad + WM - 1) / WM * nt;
    // fill the 256 CUs with one workgroup each (an item count that is a multiple of 8
    // deals evenly over the XCDs; the launcher pads the grid otherwise)
    int64_t ns = (256 + tiles - 1) / tiles;
    if (ns > wsteps) ns = wsteps;
    if (ns < 1) ns = 1;
    while ((tiles * ns) % 8 != 0 && ns < wsteps) ++ns;
    const int64_t steps_per = (wsteps + ns - 1) / ns;
    *pix_per_split = steps_per * WKS;
    return (int)((d + *pix_per_split - 1) / *pix_per_split);
  }
  const int64_t tiles = bpad / HM * ((ldw + HN - 1) / HN);
  int64_t ns = (512 + tiles - 1) / tiles;  // ~2 workgroups per CU
  if (ns > steps) ns = steps;
  if (ns < 1) ns = 1;
  if (ns > 64) ns = 64;
  const int64_t steps_per = (steps + ns - 1) / ns;
  *pix_per_split = steps_per * HK;
  return (int)((d + *pix_per_split - 1) / *pix_per_split);
}

hipError_t launch_project_bf16(hipStream_t s, int p_dtype, const void* P, int64_t b, int64_t bpad, int64_t d,
                               const float* mean_r, const uint8_t* mean_u8, const unsigned short* Wt16,
                               const void* Wf, int ldw, float* part, int nsplit, int64_t pps) {
  if (ldw % HN != 0) return hipErrorInvalidValue;
  if (bf16_wide_ok(p_dtype, P, d, ldw, mean_u8) && use_frag(Wf)) {
    const FragCfg fc = frag_cfg(ldw, d);
    const int NT = fc.NT;
    const int nt = ldw / NT;
    const int mt = (int)((bpad + fc.RM - 1) / fc.RM);
    const int grid = (mt * nt * nsplit + 7) / 8 * 8;
    const int FWK = fc.WK;
    if (pps % FWK != 0) return hipErrorInvalidValue;
    const uint8_t* p8 = static_cast<const uint8_t*>(P);
    const uint4* wf = static_cast<const uint4*>(Wf);
    auto go = [&](auto kern, int threads) {
      hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(threads), 0, s, p8, b, d, mean_u8, wf, ldw, part, bpad, pps,
                         mt, nt, nsplit);
    };
    bool ml = pps <= kFragMeanLds;
#ifdef EF_DIAGNOSTICS  // EF_PROJ_MEAN_LDS=0: the per-stage global mean loads (A/B)
    if (const char* e = getenv("EF_PROJ_MEAN_LDS")) ml = ml && atoi(e) != 0;
#endif
    if (fc.NW == 4) {
      if (ml) go(project_bf16_frag_kernel<256, 64, true, 4>, 256);
      else go(project_bf16_frag_kernel<256, 64, false, 4>, 256);
    } else if (FWK == 128) {
      if (ml) go(project_bf16_frag_kernel<512, 128, true>, 512);
      else go(project_bf16_frag_kernel<512, 128, false>, 512);
    } else {
      if (NT == 512) go(project_bf16_frag_kernel<512, 64, false>, 512);
      else if (NT == 256) go(project_bf16_frag_kernel<256, 64, false>, 512);
      else go(project_bf16_frag_kernel<128, 64, false>, 512);
    }
    return hipGetLastError();
  }
  if (bf16_wide_ok(p_dtype, P, d, ldw, mean_u8)) {
    const bool n256 = ldw % 256 == 0;
    const int nt = n256 ? ldw / 256 : ldw / 128;
    const int mt = (int)((bpad + WM - 1) / WM);
    const int grid = (mt * nt * nsplit + 7) / 8 * 8;  // XCD deal over a multiple of 8
    if (bpad % WM != 0 || pps % WKS != 0) return hipErrorInvalidValue;
    const uint8_t* p8 = static_cast<const uint8_t*>(P);
    if (n256)
      hipLaunchKernelGGL((project_bf16_wide_kernel<256, WKS>), dim3((unsigned)grid), dim3(512), 0, s, p8, b, d, mean_u8,
                         Wt16, ldw, part, bpad, pps, mt, nt, nsplit);
    else
      hipLaunchKernelGGL((project_bf16_wide_kernel<128, WKS>), dim3((unsigned)grid), dim3(512), 0, s, p8, b, d, mean_u8,
                         Wt16, ldw, part, bpad, pps, mt, nt, nsplit);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)(bpad / HM), (unsigned)nsplit, (unsigned)(ldw / HN));
  const bool vec = (d % 16 == 0) && (pps % 16 == 0) && ((reinterpret_cast<uintptr_t>(P) & 15) == 0);
  if (p_dtype == EF_U8) {
    if (vec)
      hipLaunchKernelGGL((project_bf16_kernel<EF_U8, true>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw, part,
                         bpad, pps);
    else
      hipLaunchKernelGGL((project_bf16_kernel<EF_U8, false>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw,
                         part, bpad, pps);
  } else {
    if (vec)
      hipLaunchKernelGGL((project_bf16_kernel<EF_F32, true>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw,
                         part, bpad, pps);
    else
      hipLaunchKernelGGL((project_bf16_kernel<EF_F32, false>), grid, dim3(256), 0, s, P, b, d, mean_r, Wt16, ldw,
                         part, bpad, pps);
  }
  return hipGetLastError();
}

}  // namespace ef
