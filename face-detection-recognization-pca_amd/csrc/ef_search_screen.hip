// Single-bf16 screen, main pass, with the GALLERY operand in VGPRs (the C5
// headline scan, EF_OPT_SEARCH_SPLIT_BF16 = 3 at k > 128).  Same plan, workgroup tile
// (256 gallery rows x 256 probes), XCD deal and SearchWs contract (per chunk best key +
// runner-up) as search_wide16_kernel<.., false, true> (ef_search_wide.hip), whose collect
// pass still follows it; the per-(row, probe) fp32 score is the same chain of
// v_mfma_f32_16x16x32_bf16 steps in the same k order.
//
// search_wide16_kernel stages BOTH operands through LDS by LDS-DMA, 2 slices deep, one
// barrier + full DMA drain per 64-k slice; its ablations put the DMA + barrier share at
// ~10 points of the ~58 % a no-DMA form reached.  Here:
//   * wave w owns gallery rows 32w .. 32w + 31 of the tile (two 16-row A blocks) against
//     all 256 probes (sixteen 16-probe B blocks): 2 x 16 accumulators of 4 = 128 VGPRs;
//   * its A fragments (16 B per lane per block and k-step: slice-row chunk qd for k-step 0,
//     4 + qd for k-step 1, so each load instruction covers 64 contiguous bytes of 16 rows;
//     the probes pair the same chunks) are loaded by global_load_dwordx4 straight
//     into a 2-set register ring, one slice ahead (a third set spills: 48 registers of
//     running top-2 state sit beside the 128 accumulators): no LDS round trip for the
//     gallery, and no other wave reads them;
//   * only the probes go through LDS, by LDS-DMA into a 4-slice ring (3 slices ahead; the
//     probe tile is L2-resident), with the tile's |g|^2 (or 1/|g|) per wave alongside;
//   * every load in the loop is inline asm with explicit, exact vmcnt waits: per slice a
//     wave issues 4 gallery loads (slice it + 1), then 4 probe pieces + 1 aux piece (slice
//     it + 3), so before slice it's MFMAs exactly 14 younger operations may be outstanding
//     (vmcnt(14)), and before the slice's closing barrier 18 (the probes of it + 1 have
//     landed).  The compiler sees no
//     VMEM in the loop, so it never waits for all of them.
// The per-slice barrier stays (the probe ring's slots are recycled), but nothing waits for
// a DMA issued less than two slices earlier.
#include "ef_search_common.hpp"

#include <climits>

namespace ef {

namespace {

typedef short bf16x8s __attribute__((ext_vector_type(8)));
typedef float f32x4s __attribute__((ext_vector_type(4)));
typedef unsigned u32x4s __attribute__((ext_vector_type(4)));

constexpr int SR = kWide3RowTile;    // gallery rows per tile
constexpr int SP = kWide3ProbeTile;  // probes per workgroup
constexpr int SBK = 32;              // floats (64 bf16) per slice row
constexpr int SSL = SP * SBK;        // floats per probe slice (32 KiB)
constexpr int RING = 4;              // probe slices in LDS
constexpr int AUXW = 64;             // aux floats per wave and slot (32 rows, lanes 32-63 duplicate)

__device__ __forceinline__ float min3f(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ bf16x8s as_bf16(const u32x4s& v) {
  bf16x8s r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}
__device__ __forceinline__ bf16x8s as_bf16(const float4& v) {
  bf16x8s r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}

// 16 B at sbase + voff and at + 64 into two VGPR quads (vmcnt += 2)
__device__ __forceinline__ void gload32(u32x4s& lo, u32x4s& hi, unsigned voff, unsigned long long sbase) {
  asm volatile("global_load_dwordx4 %0, %2, %3\n\tglobal_load_dwordx4 %1, %2, %3 offset:64"
               : "=&v"(lo), "=&v"(hi)
               : "v"(voff), "s"(sbase)
               : "memory");
}
// the ring set's registers are ready (the asm ties them, so no use moves above the wait)
template <int N>
__device__ __forceinline__ void wait_vm(u32x4s (&g)[4]) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]) : "n"(N) : "memory");
}

// One gallery slice set: A fragments (row block rb, k-step ks) = g[2 rb + ks]
struct GSet {
  u32x4s g[4];
};

template <int KP, int METRIC>
__global__ __launch_bounds__(512, 1) void search_screen_kernel(const float* __restrict__ q1,
                                                               const float* __restrict__ G1,
                                                               const float* __restrict__ aux, int64_t n,
                                                               int n_ptiles, int tiles_per_chunk, int pblk,
                                                               int cblk, int64_t bpad, SearchWs ws) {
  static_assert(KP % SBK == 0, "whole slices");
  constexpr int NS = KP / SBK;
  __shared__ __attribute__((aligned(16))) float smem[RING * SSL + RING * 8 * AUXW];

  // the XCD deal of search_wide16_kernel's main pass
  const int total = gridDim.x;  // host guarantees total % 8 == 0
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  const int bsz = cblk * pblk;
  const int blk = lin / bsz, rr = lin - blk * bsz;
  const int nbp = n_ptiles / pblk;
  const int gc = (blk / nbp) * cblk + rr / pblk, pt = (blk % nbp) * pblk + rr % pblk;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qd = lane >> 4, r16 = lane & 15;

  const int64_t tiles_total = (n + SR - 1) / SR;
  const int64_t t0 = (int64_t)gc * tiles_per_chunk;
  const int64_t t1 = t0 + tiles_per_chunk < tiles_total ? t0 + tiles_per_chunk : tiles_total;
  const int64_t prow0 = (int64_t)pt * SP;  // this workgroup's first probe slot

  const float INF = __builtin_inff();
  if (t0 >= t1) {
    if (tid < SP) {
      ws.part_key[(int64_t)gc * bpad + prow0 + tid] = LLONG_MAX;
      ws.part_b2[(int64_t)gc * bpad + prow0 + tid] = INF;
    }
    return;
  }
  const int n_it = (int)((t1 - t0) * NS);  // host checks the 32-bit range
  const unsigned lds_base = lds_addr(smem);
  const unsigned long long gbase = uniform_ptr(G1), qbase = uniform_ptr(q1), abase = uniform_ptr(aux);

  // gallery rows of this lane's A fragments: 32 wave + 16 rb + r16 of the tile
  auto gload_set = [&](int it, GSet& s) {
    const int itc = it < n_it ? it : n_it - 1;  // past the end: re-read the last slice
    const int64_t t = t0 + itc / NS;
    const int sl = itc % NS;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      int64_t row = t * SR + 32 * wave + 16 * rb + r16;
      row = row < n ? row : n - 1;  // tail tile: masked at the epilogue
      const unsigned voff = (unsigned)((row * KP + sl * SBK + 4 * qd) * 4);
      gload32(s.g[2 * rb], s.g[2 * rb + 1], voff, gbase);
    }
  };
  // probe pieces of slice it (4 per wave: rows 8 j + (lane >> 3), j = 4 wave + jj, the
  // 16-B chunk swizzled by s(row) = 2 ((row >> 1) & 3): with the lanes' chunks qd / 4 + qd,
  // every ds_read_b128 lane group (MI355X_MICROARCH.md §LDS) then covers all 64 banks — each
  // of the row sets {0,2,12,14}, {4,6,8,10}, {1,3,13,15}, {5,7,9,11} meets s = {0,2,4,6})
  // + this wave's aux rows of the slice's tile
  auto dma_slice = [&](int it) {
    const int itc = it < n_it ? it : n_it - 1;
    const int64_t t = t0 + itc / NS;
    const int sl = itc % NS;
    const int slot = it & (RING - 1);
    const unsigned long long qb = qbase + (unsigned long long)(sl * SBK) * 4;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = wave * 4 + jj;
      const int row = j * 8 + (lane >> 3);
      const unsigned lch16 = (unsigned)(((lane & 7) ^ (((row >> 1) & 3) << 1)) * 16);
      const unsigned qoff = (unsigned)((prow0 + row) * KP * 4) + lch16;
      glds16s(qoff, qb, lds_base + (unsigned)((slot * SSL + j * 256) * 4));
    }
    int64_t arow = t * SR + 32 * wave + (lane & 31);
    arow = arow < n ? arow : n - 1;
    glds4s((unsigned)(arow * 4), abase, lds_base + (unsigned)((RING * SSL + (slot * 8 + wave) * AUXW) * 4));
  };

  float b1[16], b2[16];
  int i1[16];
#pragma unroll
  for (int pb = 0; pb < 16; ++pb) b1[pb] = INF, b2[pb] = INF, i1[pb] = INT_MAX;

  // 8 values of probe block pb (rows rowbase + 16 rb + 4 qd + r, increasing with (rb, r):
  // first minimum in lane) into the running (best, index, runner-up)
  auto consume = [&](const f32x4s& v0, const f32x4s& v1, int rowbase, int pb) {
    float mn = min3f(v0[0], v0[1], v0[2]);
    mn = min3f(mn, v0[3], v1[0]);
    mn = min3f(mn, v1[1], v1[2]);
    mn = fminf(mn, v1[3]);
    if (!__any(mn < b2[pb])) return;  // exact skip: no value here can change the top-2
    float m1 = INF, m2 = INF;
    int ir = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = e < 4 ? v0[e] : v1[e - 4];
      const bool lt = x < m1;
      m2 = __builtin_amdgcn_fmed3f(m1, x, m2);
      ir = lt ? 16 * (e >> 2) + (e & 3) : ir;
      m1 = lt ? x : m1;
    }
    const bool lt = m1 < b1[pb];
    b2[pb] = lt ? fminf(b1[pb], m2) : fminf(b2[pb], m1);
    i1[pb] = lt ? rowbase + ir + 4 * qd : i1[pb];
    b1[pb] = lt ? m1 : b1[pb];
  };

  f32x4s acc[2][16];
  const int sw = ((r16 >> 1) & 3) << 1;  // s(row) of every probe this lane reads
  const int ph = (qd ^ sw) * 4, pl = ((4 + qd) ^ sw) * 4;

  // one slice: MFMAs on set `cur`, after issuing the gallery loads of it + 1 into `nxt`
  auto run = [&](int it, GSet& cur, GSet& nxt) {
    gload_set(it + 1, nxt);
    dma_slice(it + 3);
    wait_vm<14>(cur.g);
    const int slot = it & (RING - 1);
    const int64_t t = t0 + it / NS;
    const int sl = it % NS;
    const float* sAux = smem + RING * SSL + (slot * 8 + wave) * AUXW;
    if (sl == 0) {
      // L2: start from -|g|^2 / 2 and accumulate q.g (-2 acc = |g|^2 - 2 q.g); cosine: 0
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        f32x4s a = {0.f, 0.f, 0.f, 0.f};
        if constexpr (METRIC == EF_METRIC_L2) {
          const float4 x = *reinterpret_cast<const float4*>(sAux + 16 * rb + 4 * qd);
          a = f32x4s{-0.5f * x.x, -0.5f * x.y, -0.5f * x.z, -0.5f * x.w};
        }
#pragma unroll
        for (int pb = 0; pb < 16; ++pb) acc[rb][pb] = a;
      }
    }
    const float* sq = smem + slot * SSL + r16 * SBK;
    const bf16x8s a00 = as_bf16(cur.g[0]), a01 = as_bf16(cur.g[1]);
    const bf16x8s a10 = as_bf16(cur.g[2]), a11 = as_bf16(cur.g[3]);
#pragma unroll
    for (int pb = 0; pb < 16; ++pb) {
      const bf16x8s bh = as_bf16(*reinterpret_cast<const float4*>(sq + 16 * pb * SBK + ph));
      const bf16x8s bl = as_bf16(*reinterpret_cast<const float4*>(sq + 16 * pb * SBK + pl));
      acc[0][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a00, bh, acc[0][pb], 0, 0, 0);
      acc[1][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a10, bh, acc[1][pb], 0, 0, 0);
      acc[0][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a01, bl, acc[0][pb], 0, 0, 0);
      acc[1][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a11, bl, acc[1][pb], 0, 0, 0);
    }
    if (sl == NS - 1) {
      const int tbase = (int)(t * SR) + 32 * wave;
      const bool tail = (t + 1) * SR > n;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const float4 x = *reinterpret_cast<const float4*>(sAux + 16 * rb + 4 * qd);
#pragma unroll
        for (int pb = 0; pb < 16; ++pb) {
          if constexpr (METRIC == EF_METRIC_L2) {
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[rb][pb][r] *= -2.f;
          } else {  // -(q.g) * (1/|g|)
            acc[rb][pb][0] *= -x.x;
            acc[rb][pb][1] *= -x.y;
            acc[rb][pb][2] *= -x.z;
            acc[rb][pb][3] *= -x.w;
          }
          if (tail) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (tbase + 16 * rb + 4 * qd + r >= n) acc[rb][pb][r] = INF;
          }
        }
      }
#pragma unroll
      for (int pb = 0; pb < 16; ++pb) consume(acc[0][pb], acc[1][pb], tbase, pb);
    }
    // the probes of slice it + 1 have landed (18 younger operations: G(it), D(it + 2),
    // G(it + 1), D(it + 3)); every wave is done with slot it before D(it + 4) refills it
    asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  // prologue: D(0) D(1) G(0) D(2), then D(0) landed (14 younger)
  GSet ga, gb;
  dma_slice(0);
  dma_slice(1);
  gload_set(0, ga);
  dma_slice(2);
  asm volatile("s_waitcnt vmcnt(14)\n\ts_barrier" ::: "memory");
  // two sets by iteration parity (unrolled, so each set is a fixed register range)
  int it = 0;
  for (; it + 1 < n_it; it += 2) {
    run(it, ga, gb);
    run(it + 1, gb, ga);
  }
  if (it < n_it) run(it, ga, gb);
  // drain: nothing may land in LDS after the merge below reuses it
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

  // the four row quarters (lanes r16, +16, +32, +48), then the eight waves via LDS
#pragma unroll
  for (int pb = 0; pb < 16; ++pb) {
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float ob1 = __shfl_xor(b1[pb], off);
      const int oi1 = __shfl_xor(i1[pb], off);
      const float ob2 = __shfl_xor(b2[pb], off);
      const bool other = ob1 < b1[pb] || (ob1 == b1[pb] && oi1 < i1[pb]);
      const float lose = other ? b1[pb] : ob1;
      b2[pb] = fminf(fminf(b2[pb], ob2), lose);
      if (other) { b1[pb] = ob1; i1[pb] = oi1; }
    }
  }
  float* xb = smem;  // [8 waves][256 probes] x (b1, b2, i1)
  if (qd == 0) {
#pragma unroll
    for (int pb = 0; pb < 16; ++pb) {
      const int o = ((wave * SP) + 16 * pb + r16) * 3;
      xb[o] = b1[pb];
      xb[o + 1] = b2[pb];
      xb[o + 2] = __int_as_float(i1[pb]);
    }
  }
  __syncthreads();
  if (tid < SP) {
    float B1 = xb[tid * 3], B2 = xb[tid * 3 + 1];
    int I1 = __float_as_int(xb[tid * 3 + 2]);
    for (int w = 1; w < 8; ++w) {
      const int o = (w * SP + tid) * 3;
      const float ob1 = xb[o], ob2 = xb[o + 1];
      const int oi1 = __float_as_int(xb[o + 2]);
      const bool other = ob1 < B1 || (ob1 == B1 && oi1 < I1);
      const float lose = other ? B1 : ob1;
      B2 = fminf(fminf(B2, ob2), lose);
      if (other) { B1 = ob1; I1 = oi1; }
    }
    const int64_t po = (int64_t)gc * bpad + prow0 + tid;
    ws.part_key[po] = I1 == INT_MAX ? LLONG_MAX : pack_key(B1, (unsigned)I1);
    ws.part_b2[po] = B2;
  }
}

}  // namespace

// Measured (round 6, profiles/r06/screen_vg_ab.txt; C5, 1M x 512, 4096 probes, same box,
// alternated): 4.34 / 4.35 ms per launch against 3.55 / 3.55 ms for search_wide16_kernel's
// main pass, keys identical, the same MFMA-busy cycles.  Counters: TA busy 45 % of the
// kernel's cycles against 30 % (a fragment-shaped register load touches 16 rows x 64 B per
// instruction, twice the lines per byte of an LDS-DMA piece's 8 rows x 128 B), waves waiting
// 37 % against 32 % of their cycles (one slice of register prefetch is all that fits beside
// the 128 accumulators and 48 registers of running top-2 state), MFMA busy 42 % against 55 %.
// Not the product path: kept for A/B in diagnostic builds (EF_SCREEN_VG=1).
bool screen_vg_enabled() {
#ifdef EF_DIAGNOSTICS  // EF_SCREEN_VG=1: this kernel for the screen's main pass (A/B)
  if (const char* e = getenv("EF_SCREEN_VG")) return atoi(e) != 0;
#endif
  return false;
}

// kh: floats per row of the single-bf16 copies (k / 2); the compiled widths 128 / 256
// (k = 256 / 512).  Same grid and plan checks as wide3_t.
hipError_t launch_search_screen(hipStream_t s, int kh, int metric, const SearchPlan& pl, const float* q1,
                                const float* G1, const float* aux, int64_t n, int64_t bpad, const SearchWs& ws) {
  const dim3 grid((unsigned)(pl.nchunks * pl.n_ptiles)), block(512);
  if (pl.n_ptiles % pl.pblk != 0 || pl.nchunks % pl.cblk != 0 || (pl.nchunks * pl.n_ptiles) % 8 != 0 ||
      (pl.nchunks * pl.n_ptiles / 8) % (pl.cblk * pl.pblk) != 0 || bpad % SP != 0)
    return hipErrorInvalidValue;
  // 32-bit byte offsets: probe rows and the gallery (G1 rows * kh * 4 < 2^32)
  if (bpad * (int64_t)kh * 4 >= ((int64_t)1 << 32) || n * (int64_t)kh * 4 >= ((int64_t)1 << 32) ||
      (int64_t)pl.tiles_per_chunk * (kh / SBK) >= ((int64_t)1 << 31))
    return hipErrorInvalidValue;
  const bool l2 = metric == EF_METRIC_L2;
  if (kh == 128) {
    if (l2)
      hipLaunchKernelGGL((search_screen_kernel<128, EF_METRIC_L2>), grid, block, 0, s, q1, G1, aux, n, pl.n_ptiles,
                         pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
    else
      hipLaunchKernelGGL((search_screen_kernel<128, EF_METRIC_COSINE>), grid, block, 0, s, q1, G1, aux, n,
                         pl.n_ptiles, pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
  } else if (kh == 256) {
    if (l2)
      hipLaunchKernelGGL((search_screen_kernel<256, EF_METRIC_L2>), grid, block, 0, s, q1, G1, aux, n, pl.n_ptiles,
                         pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
    else
      hipLaunchKernelGGL((search_screen_kernel<256, EF_METRIC_COSINE>), grid, block, 0, s, q1, G1, aux, n,
                         pl.n_ptiles, pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ef
