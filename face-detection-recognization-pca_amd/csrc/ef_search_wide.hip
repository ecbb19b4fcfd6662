// Distance GEMM + fused arg-best for wide features, KP in {256, 512} (BASELINE.json
// config 5: k = 512 eigenfaces) and any multiple of 128 above (KP = 0 instantiations: the
// full-rank per-person models of train-v5.py:539-545, k = face count).  Same contract as search_kernel in ef_search.hip (per
// chunk best key + runner-up into SearchWs, or COLLECT of the rows within a queued
// probe's threshold) so reduce_kernel / resolve_kernel finish it unchanged.
//
// At KP >= 256 a wave cannot keep its probes in registers (32 probes x 512 k = 256 VGPRs),
// so both operands stream through LDS, k-slice by k-slice:
//   * workgroup = 4 waves, tile = 128 gallery rows x 128 probes, k-slices of 32;
//     one LDS stage = 16 KiB of gallery + 16 KiB of probes, double-buffered (64 KiB),
//     filled by global_load_lds (no VGPR staging), 2 workgroups per CU;
//   * wave w owns probes [32w, 32w+32) of the tile (MFMA B operand, one ds_read_b128 per
//     4 k-steps) and all 128 rows as four 32-row A blocks: four independent accumulator
//     chains, 16 MFMAs per 5 ds_read_b128;
//   * 128-B slice rows are XOR-swizzled by ((row >> 1) & 7) on the source address, which
//     makes every ds_read_b128 lane group (MI355X_MICROARCH.md §LDS) conflict-free;
//   * the arg-best epilogue is the in-lane running (best, index, runner-up) of
//     ef_search.hip, once per 128-row tile (<= 6 % of the tile's MFMA time at KP = 256).
#include "ef_search_common.hpp"

#include <algorithm>
#include <climits>

namespace ef {

// Diagnostic builds only (timing, wrong results): EF_WIDE_ABL 1 = no per-slice barrier,
// 2 = no arg-best epilogue, 3 = no DMA after the first slices.
#ifndef EF_WIDE_ABL
#define EF_WIDE_ABL 0
#endif
#ifndef EF_WIDE_STAGGER  // wide16: n > 0 = the upper four waves issue their DMA after A block n - 1
#define EF_WIDE_STAGGER 2  // measured: 8.96 -> 8.76 ms at C5 (1: 8.83, 4: 9.03, 6: 9.36)
#endif
#ifndef EF_WIDE_INTERLEAVE
#define EF_WIDE_INTERLEAVE 0
#endif
#ifndef EF_WIDE_ROLES  // wide16: 1 = waves 0-3 issue every gallery DMA piece, 4-7 every probe piece (experiment)
#define EF_WIDE_ROLES 0
#endif
#ifndef EF_WIDE_SERP  // wide16: 1 = serpentine k-slice order over a sweep's tiles (experiment)
#define EF_WIDE_SERP 1  // with EF_WIDE3_PB 8: C5 HBM fetch 12.0 -> 8.1 GB per launch, same time (profiles/r04/c5_hbm_ab.txt)
#endif

constexpr int WR = kWideRowTile;    // gallery rows per tile
constexpr int WP = kWideProbeTile;  // probes per workgroup
constexpr int WBK = 32;             // k per slice
constexpr int WSL = WR * WBK;       // floats per gallery slice (= per probe slice)
static_assert(WR == 128 && WP == 128, "4 waves x 32 probes, 4 x 32-row blocks");

typedef short bf16x8w __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// min of three floats as one v_min3_f32, without the compiler's IEEE-mode canonicalisation
// of each input (scores are finite or +inf, never NaN)
__device__ __forceinline__ float min3_raw(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ bf16x8w as_bf16x8w(const float4& v) {
  bf16x8w r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}

// Row geometry of a sweep: KP > 0 is a compile-time row length (256 | 512); KP = 0 takes
// kp_rt, any multiple of 128 above 512 (full-rank per-person models, train-v5.py:539-545),
// at run time.  A sweep is (tile, slice) pairs flattened into one counter it; for KP = 0
// the split is a 32-bit division by a wave-uniform value (wide_t checks n_it < 2^31).
template <int KP>
struct WideGeom {
  int kp, ns;  // floats per row, 32-k slices per row
  __device__ __forceinline__ explicit WideGeom(int kp_rt) : kp(KP > 0 ? KP : kp_rt), ns((KP > 0 ? KP : kp_rt) / WBK) {}
  __device__ __forceinline__ int64_t tile(int64_t it) const {
    if constexpr (KP > 0) return it / (KP / WBK);
    else return (int64_t)((unsigned)it / (unsigned)ns);
  }
  __device__ __forceinline__ int slice(int64_t it) const {
    if constexpr (KP > 0) return (int)(it % (KP / WBK));
    else return (int)((unsigned)it % (unsigned)ns);
  }
};

template <int KP, int METRIC, bool COLLECT>
__global__ __launch_bounds__(256, 2) void search_wide_kernel(
    const float* __restrict__ qpad, const float* __restrict__ G, const float* __restrict__ aux, int64_t n,
    int n_ptiles, int tiles_per_chunk, int pblk, int cblk, int64_t bpad, SearchWs ws, int kp_rt) {
  const WideGeom<KP> geo(kp_rt);
  const int NS = geo.ns;  // slices per tile
  // [stage 0: gallery | probes][stage 1: gallery | probes][aux of even | odd tiles]
  // (aux is double-buffered by tile: the cosine epilogue reads it in the tile's last
  // slice, when the DMA of the next tile's first slice is already in flight)
  __shared__ __attribute__((aligned(16))) float smem[4 * WSL + 2 * WR];

  // one (gallery chunk gc, probe tile pt) work item
  auto body = [&](const int gc, const int pt, const int n_amb) {

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int c32 = lane & 31;

  const int64_t tiles_total = (n + WR - 1) / WR;
  const int64_t t0 = (int64_t)gc * tiles_per_chunk;
  const int64_t t1 = t0 + tiles_per_chunk < tiles_total ? t0 + tiles_per_chunk : tiles_total;
  const int64_t s0 = (int64_t)pt * WP + wave * 32 + c32;  // this lane's probe slot

  if (t0 >= t1) {
    if constexpr (!COLLECT) {
      if (h == 0) {
        ws.part_key[(int64_t)gc * bpad + s0] = LLONG_MAX;
        ws.part_b2[(int64_t)gc * bpad + s0] = __builtin_inff();
      }
    }
    return;
  }

  // DMA geometry: a slice is 16 pieces of 1 KiB (8 rows x 128 B); wave w issues pieces
  // 4w..4w+3 of the gallery slice and of the probe slice.  Lane l of piece j carries
  // row 8j + (l >> 3), physical 16-B chunk l & 7, which holds logical chunk
  // (l & 7) ^ ((row >> 1) & 7) = (l & 7) ^ ((4 * jj + (l >> 4)) & 7).
  // Per-lane byte offsets are fixed for the whole sweep (SGPR-base DMA: the slice's base
  // address is wave-uniform), so a slice's 8 DMAs cost no per-lane address arithmetic.
  const int prow = lane >> 3;
  unsigned goff[4], qoff[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int slot = pt * WP + (wave * 4 + jj) * 8 + prow;
    int qrow = slot;
    if constexpr (COLLECT) qrow = slot < n_amb ? ws.amb_list[slot] : 0;
    const unsigned lch16 = (unsigned)(((lane & 7) ^ ((4 * jj + (lane >> 4)) & 7)) * 16);
    goff[jj] = (unsigned)((wave * 4 + jj) * 8 + prow) * (geo.kp * 4) + lch16;
    qoff[jj] = (unsigned)qrow * (geo.kp * 4) + lch16;
  }
  const unsigned aoff = (unsigned)lane * 4;
  float thr = -__builtin_inff();
  if constexpr (COLLECT) {
    if (s0 < n_amb) thr = ws.thr[s0];
  }
  // settle these loads before the loop (a loop-merged wait would drain the LDS-DMA)
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) asm volatile("" ::"v"(qoff[jj]));
  asm volatile("" ::"v"(thr));

  const unsigned lds_base = lds_addr(smem);
  const int64_t n_it = (t1 - t0) * NS;
  // DMA of slice it into buffer buf, piece jj of this wave's four (+ the tile's aux).
  auto issue_piece = [&](int64_t it, int buf, int jj) {
    const int64_t t = t0 + geo.tile(it);
    const int sl = geo.slice(it);
    const int nrem = (int)((n - t * WR) < WR ? (n - t * WR) : WR);
    const unsigned long long gb = (unsigned long long)(size_t)(G + t * WR * geo.kp + sl * WBK);
    const unsigned long long qb = (unsigned long long)(size_t)(qpad + sl * WBK);
    const int j = wave * 4 + jj;
    unsigned go = goff[jj];
    if (nrem < WR) {  // tail tile: rows past the end re-read the last row (masked later)
      const unsigned row = go / (geo.kp * 4);
      go = (row < (unsigned)nrem ? row : (unsigned)(nrem - 1)) * (geo.kp * 4) + go % (geo.kp * 4);
    }
    glds16s(go, gb, lds_base + (unsigned)((buf * 2 * WSL + j * 256) * 4));
    glds16s(qoff[jj], qb, lds_base + (unsigned)((buf * 2 * WSL + WSL + j * 256) * 4));
    if (jj == 3 && sl == 0 && wave == 0) {  // the tile's ||g||^2 (L2) or 1/||g|| (cosine)
      const unsigned long long ab = (unsigned long long)(size_t)(aux + t * WR);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rr = 64 * q + lane;
        const unsigned ao = rr < nrem ? aoff + 256u * q : (unsigned)(nrem - 1) * 4;
        glds4s(ao, ab, lds_base + (unsigned)((4 * WSL + ((t - t0) & 1) * WR + 64 * q) * 4));
      }
    }
  };
  auto issue = [&](int64_t it, int buf) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) issue_piece(it, buf, jj);
  };

  const float INF = __builtin_inff();
  float b1 = INF, b2 = INF;
  int i1 = INT_MAX;
  auto consume = [&](const f32x16& v, int rowbase) {
    if constexpr (COLLECT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (v[r] <= thr) {
          const int pos = atomicAdd(&ws.cand_cnt[s0], 1);
          if (pos < kCandMax) ws.cand[s0 * kCandMax + pos] = rowbase + (r & 3) + 8 * (r >> 2) + 4 * h;
        }
      }
    } else {
      // uniform skip of blocks that cannot change the running top-2 (ef_search.hip consume)
      float mn = v[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mn = fminf(mn, v[r]);
      if (!__any(mn < b2)) return;
      float m1 = v[0], m2 = INF;
      int ir = 0;
#pragma unroll
      for (int r = 1; r < 16; ++r) {
        const bool lt = v[r] < m1;
        m2 = __builtin_amdgcn_fmed3f(m1, v[r], m2);
        ir = lt ? r : ir;
        m1 = lt ? v[r] : m1;
      }
      const bool lt = m1 < b1;
      b2 = lt ? fminf(b1, m2) : fminf(b2, m1);
      i1 = lt ? rowbase + (ir & 3) + 8 * (ir >> 2) + 4 * h : i1;
      b1 = lt ? m1 : b1;
    }
  };

  issue(0, 0);
  dma_wait_all();
  __syncthreads();

  const int sw = (c32 >> 1) & 7;  // swizzle key of rows c32 + 32 rb and of probe 32 w + c32
  f32x16 acc[4];
  for (int64_t it = 0; it < n_it; ++it) {
    const int buf = (int)(it & 1);
    const int sl = geo.slice(it);
    const float* const sAux = smem + 4 * WSL + (int)(geo.tile(it) & 1) * WR;
#if EF_WIDE_INTERLEAVE == 0
#if EF_WIDE_ABL == 3
    if (it + 1 < 2)
#else
    if (it + 1 < n_it)
#endif
      issue(it + 1, buf ^ 1);  // lands under this slice's MFMAs
#endif
    if (sl == 0) {
      // L2: start from -||g||^2 / 2 and accumulate q.g, so that -2 acc = ||g||^2 - 2 q.g
      // with the rounding of the chain scaled exactly by -2.  Cosine: start from 0.
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        acc[rb] = f32x16{};
        if constexpr (METRIC == EF_METRIC_L2) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 x = *reinterpret_cast<const float4*>(sAux + rb * 32 + 8 * q + 4 * h);
            acc[rb][4 * q] = -0.5f * x.x;
            acc[rb][4 * q + 1] = -0.5f * x.y;
            acc[rb][4 * q + 2] = -0.5f * x.z;
            acc[rb][4 * q + 3] = -0.5f * x.w;
          }
        }
      }
    }
    const float* sg = smem + buf * 2 * WSL;
    const float* sq = sg + WSL;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pch = ((h * 4 + j) ^ sw) * 4;  // lane half h owns k in [16h, 16h + 16) of the slice
      const float4 bq = *reinterpret_cast<const float4*>(sq + (wave * 32 + c32) * WBK + pch);
      float4 a[4];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) a[rb] = *reinterpret_cast<const float4*>(sg + (rb * 32 + c32) * WBK + pch);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rb].x, bq.x, acc[rb], 0, 0, 0);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rb].y, bq.y, acc[rb], 0, 0, 0);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rb].z, bq.z, acc[rb], 0, 0, 0);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rb].w, bq.w, acc[rb], 0, 0, 0);
#if EF_WIDE_INTERLEAVE
      // one DMA piece pair of slice it+1 per 16 MFMAs (buffer buf^1 was released by the
      // previous slice's barrier)
      if (it + 1 < n_it) issue_piece(it + 1, buf ^ 1, j);
#endif
    }
    if (sl == NS - 1) {
      const int64_t t = t0 + geo.tile(it);
      const int tbase = (int)(t * WR);
      const bool tail = (t + 1) * WR > n;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        if constexpr (METRIC == EF_METRIC_L2) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[rb][r] *= -2.f;
        } else {  // -(q.g) * (1/||g||)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 x = *reinterpret_cast<const float4*>(sAux + rb * 32 + 8 * q + 4 * h);
            acc[rb][4 * q] *= -x.x;
            acc[rb][4 * q + 1] *= -x.y;
            acc[rb][4 * q + 2] *= -x.z;
            acc[rb][4 * q + 3] *= -x.w;
          }
        }
        if (tail) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (tbase + rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h >= n) acc[rb][r] = INF;
        }
#if EF_WIDE_ABL == 2
        b1 = fminf(b1, acc[rb][0]);
        (void)tbase;
#else
        consume(acc[rb], tbase + rb * 32);  // blocks in row order (tie rule)
#endif
      }
    }
#if EF_WIDE_ABL != 1
    dma_wait_all();
    __syncthreads();  // slice it+1 landed; everyone is done reading buffer buf
#endif
  }

  if constexpr (!COLLECT) {
    const float ob1 = __shfl_xor(b1, 32);
    const int oi1 = __shfl_xor(i1, 32);
    const float ob2 = __shfl_xor(b2, 32);
    const bool other = ob1 < b1 || (ob1 == b1 && oi1 < i1);
    const float lose = other ? b1 : ob1;
    b2 = fminf(fminf(b2, ob2), lose);
    if (other) { b1 = ob1; i1 = oi1; }
    if (h == 0) {
      const int64_t o = (int64_t)gc * bpad + s0;
      ws.part_key[o] = i1 == INT_MAX ? LLONG_MAX : pack_key(b1, (unsigned)i1);
      ws.part_b2[o] = b2;
    }
  }
  };  // body
  if constexpr (COLLECT) {
    // collect pass: n_ptiles carries the collect plan's chunk count; the grid strides over
    // the (chunk, queued probe tile) items, so a handful of queued probes still spread over
    // the whole grid instead of one workgroup per main-pass chunk
    const int n_amb = *ws.amb_count;
    const int items = ((n_amb + 128 - 1) / 128) * n_ptiles;
    for (int item = blockIdx.x; item < items; item += gridDim.x) body(item % n_ptiles, item / n_ptiles, n_amb);
  } else {
    const int total = gridDim.x;  // host guarantees total % 8 == 0
    const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
    // (chunk, probe tile) blocks of cblk x pblk, one block per XCD (see search_plan)
    const int bsz = cblk * pblk;
    const int blk = lin / bsz, r = lin - blk * bsz;
    const int nbp = n_ptiles / pblk;
    body((blk / nbp) * cblk + r / pblk, (blk % nbp) * pblk + r % pblk, 0);
  }
}

// ---------------------------------------------------------------------------------------
// Split-bf16 wide scan, 256 gallery rows x 256 probes per workgroup (8 waves, 1 per CU).
// The split scan does 16/3 x the arithmetic of the fp32 one per LDS byte, so the 128 x 128
// tiles above would be bound by the L2 -> LDS stream (~25 B/clk/CU measured at C5); a
// 256 x 256 tile halves the streamed bytes per MFMA.  Wave w owns probes 64(w & 3) ..+64
// (two 32-probe B blocks) against rows 128(w >> 2) ..+128 (four 32-row A blocks): 8
// accumulator chains, each A fragment feeding both probe blocks (24 MFMAs per 12
// ds_read_b128 per 16 k).  The two row halves' running top-2 are merged through LDS at the
// end.  Same SearchWs contract as search_wide_kernel.
constexpr int W3R = 256;          // gallery rows per tile
constexpr int W3P = 256;          // probes per workgroup
constexpr int W3SL = W3R * WBK;   // floats per gallery slice (= per probe slice), 32 KiB
static_assert(W3R == kWide3RowTile && W3P == kWide3ProbeTile, "plan and kernel tiles agree");

template <int KP, int METRIC, bool COLLECT>
__global__ __launch_bounds__(512, 1) void search_wide3_kernel(
    const float* __restrict__ q3, const float* __restrict__ G3, const float* __restrict__ aux, int64_t n,
    int n_ptiles, int tiles_per_chunk, int pblk, int cblk, int64_t bpad, SearchWs ws, int kp_rt) {
  const WideGeom<KP> geo(kp_rt);
  const int NS = geo.ns;
  __shared__ __attribute__((aligned(16))) float smem[4 * W3SL + 2 * W3R];

  // one (gallery chunk gc, probe tile pt) work item
  auto body = [&](const int gc, const int pt, const int n_amb) {

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int pg = wave & 3, rh = wave >> 2;  // probe group (64 probes), row half (128 rows)

  const int64_t tiles_total = (n + W3R - 1) / W3R;
  const int64_t t0 = (int64_t)gc * tiles_per_chunk;
  const int64_t t1 = t0 + tiles_per_chunk < tiles_total ? t0 + tiles_per_chunk : tiles_total;
  int64_t sl0[2];  // this lane's probe slots
  sl0[0] = (int64_t)pt * W3P + 64 * pg + c32;
  sl0[1] = sl0[0] + 32;

  if (t0 >= t1) {
    if constexpr (!COLLECT) {
      if (h == 0 && rh == 0) {
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
          ws.part_key[(int64_t)gc * bpad + sl0[pb]] = LLONG_MAX;
          ws.part_b2[(int64_t)gc * bpad + sl0[pb]] = __builtin_inff();
        }
      }
    }
    return;
  }

  // DMA geometry (as search_wide_kernel): a slice is 32 pieces of 1 KiB (8 rows x 128 B)
  // for the gallery and 32 for the probes; wave w issues pieces 4w..4w+3 of each.
  const int prow = lane >> 3;
  unsigned goff[4], qoff[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int slot = pt * W3P + (wave * 4 + jj) * 8 + prow;
    int qrow = slot;
    if constexpr (COLLECT) qrow = slot < n_amb ? ws.amb_list[slot] : 0;
    const unsigned lch16 = (unsigned)(((lane & 7) ^ ((4 * jj + (lane >> 4)) & 7)) * 16);
    goff[jj] = (unsigned)((wave * 4 + jj) * 8 + prow) * (geo.kp * 4) + lch16;
    qoff[jj] = (unsigned)qrow * (geo.kp * 4) + lch16;
  }
  float thr[2] = {-__builtin_inff(), -__builtin_inff()};
  if constexpr (COLLECT) {
#pragma unroll
    for (int pb = 0; pb < 2; ++pb)
      if (sl0[pb] < n_amb) thr[pb] = ws.thr[sl0[pb]];
  }
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) asm volatile("" ::"v"(qoff[jj]));
  asm volatile("" ::"v"(thr[0]), "v"(thr[1]));

  const unsigned lds_base = lds_addr(smem);
  const int64_t n_it = (t1 - t0) * NS;
  auto issue = [&](int64_t it, int buf) {
    const int64_t t = t0 + geo.tile(it);
    const int sl = geo.slice(it);
    const int nrem = (int)((n - t * W3R) < W3R ? (n - t * W3R) : W3R);
    const unsigned long long gb = (unsigned long long)(size_t)(G3 + t * W3R * geo.kp + sl * WBK);
    const unsigned long long qb = (unsigned long long)(size_t)(q3 + sl * WBK);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = wave * 4 + jj;
      unsigned go = goff[jj];
      if (nrem < W3R) {  // tail tile: rows past the end re-read the last row (masked later)
        const unsigned row = go / (geo.kp * 4);
        go = (row < (unsigned)nrem ? row : (unsigned)(nrem - 1)) * (geo.kp * 4) + go % (geo.kp * 4);
      }
      glds16s(go, gb, lds_base + (unsigned)((buf * 2 * W3SL + j * 256) * 4));
      glds16s(qoff[jj], qb, lds_base + (unsigned)((buf * 2 * W3SL + W3SL + j * 256) * 4));
    }
    if (sl == 0 && wave == 0) {  // the tile's ||g||^2 (L2) or 1/||g|| (cosine)
      const unsigned long long ab = (unsigned long long)(size_t)(aux + t * W3R);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 64 * q + lane;
        const unsigned ao = r < nrem ? (unsigned)r * 4 : (unsigned)(nrem - 1) * 4;
        glds4s(ao, ab, lds_base + (unsigned)((4 * W3SL + ((t - t0) & 1) * W3R + 64 * q) * 4));
      }
    }
  };

  const float INF = __builtin_inff();
  float b1[2] = {INF, INF}, b2[2] = {INF, INF};
  int i1[2] = {INT_MAX, INT_MAX};
  auto consume = [&](const f32x16& v, int rowbase, int pb) {
    if constexpr (COLLECT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (v[r] <= thr[pb]) {
          const int pos = atomicAdd(&ws.cand_cnt[sl0[pb]], 1);
          if (pos < kCandMax) ws.cand[sl0[pb] * kCandMax + pos] = rowbase + (r & 3) + 8 * (r >> 2) + 4 * h;
        }
      }
    } else {
      float mn = v[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mn = fminf(mn, v[r]);
      if (!__any(mn < b2[pb])) return;  // exact skip (ef_search.hip consume)
      float m1 = v[0], m2 = INF;
      int ir = 0;
#pragma unroll
      for (int r = 1; r < 16; ++r) {
        const bool lt = v[r] < m1;
        m2 = __builtin_amdgcn_fmed3f(m1, v[r], m2);
        ir = lt ? r : ir;
        m1 = lt ? v[r] : m1;
      }
      const bool lt = m1 < b1[pb];
      b2[pb] = lt ? fminf(b1[pb], m2) : fminf(b2[pb], m1);
      i1[pb] = lt ? rowbase + (ir & 3) + 8 * (ir >> 2) + 4 * h : i1[pb];
      b1[pb] = lt ? m1 : b1[pb];
    }
  };

  issue(0, 0);
  dma_wait_all();
  __syncthreads();

  const int sw = (c32 >> 1) & 7;  // swizzle key of rows 32x + c32
  f32x16 acc[4][2];
  for (int64_t it = 0; it < n_it; ++it) {
    const int buf = (int)(it & 1);
    const int sl = geo.slice(it);
    const float* const sAux = smem + 4 * W3SL + (int)(geo.tile(it) & 1) * W3R + 128 * rh;
#if EF_WIDE_ABL == 3
    if (it + 1 < 2)  // diagnostic builds only: no slice DMA after the first (results invalid)
#else
    if (it + 1 < n_it)
#endif
      issue(it + 1, buf ^ 1);  // lands under this slice's MFMAs
    if (sl == 0) {
      // L2: start from -||g||^2 / 2 and accumulate q.g (-2 acc = ||g||^2 - 2 q.g); cosine: 0
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        f32x16 a = {};
        if constexpr (METRIC == EF_METRIC_L2) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 x = *reinterpret_cast<const float4*>(sAux + rb * 32 + 8 * q + 4 * h);
            a[4 * q] = -0.5f * x.x;
            a[4 * q + 1] = -0.5f * x.y;
            a[4 * q + 2] = -0.5f * x.z;
            a[4 * q + 3] = -0.5f * x.w;
          }
        }
        acc[rb][0] = a;
        acc[rb][1] = a;
      }
    }
    const float* sg = smem + buf * 2 * W3SL + (128 * rh + c32) * WBK;
    const float* sq = smem + buf * 2 * W3SL + W3SL + (64 * pg + c32) * WBK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ph = ((h * 4 + 2 * i) ^ sw) * 4, pl = ((h * 4 + 2 * i + 1) ^ sw) * 4;
      bf16x8w bh[2], bl[2];
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) {
        bh[pb] = as_bf16x8w(*reinterpret_cast<const float4*>(sq + pb * 32 * WBK + ph));
        bl[pb] = as_bf16x8w(*reinterpret_cast<const float4*>(sq + pb * 32 * WBK + pl));
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const bf16x8w ah = as_bf16x8w(*reinterpret_cast<const float4*>(sg + rb * 32 * WBK + ph));
        const bf16x8w al = as_bf16x8w(*reinterpret_cast<const float4*>(sg + rb * 32 * WBK + pl));
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[pb], acc[rb][pb], 0, 0, 0);
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[pb], acc[rb][pb], 0, 0, 0);
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[pb], acc[rb][pb], 0, 0, 0);
        }
      }
    }
    if (sl == NS - 1) {
      const int64_t t = t0 + geo.tile(it);
      const int tbase = (int)(t * W3R) + 128 * rh;
      const bool tail = (t + 1) * W3R > n;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
          if constexpr (METRIC == EF_METRIC_L2) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[rb][pb][r] *= -2.f;
          } else {  // -(q.g) * (1/||g||)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float4 x = *reinterpret_cast<const float4*>(sAux + rb * 32 + 8 * q + 4 * h);
              acc[rb][pb][4 * q] *= -x.x;
              acc[rb][pb][4 * q + 1] *= -x.y;
              acc[rb][pb][4 * q + 2] *= -x.z;
              acc[rb][pb][4 * q + 3] *= -x.w;
            }
          }
          if (tail) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (tbase + rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h >= n) acc[rb][pb][r] = INF;
          }
          consume(acc[rb][pb], tbase + rb * 32, pb);  // blocks in row order (tie rule)
        }
      }
    }
    dma_wait_all();
    __syncthreads();  // slice it+1 landed; everyone is done reading buffer buf
  }

  if constexpr (!COLLECT) {
    // lane halves (same probe, disjoint rows), then the two row halves through LDS
    float* xb = smem;  // [4 pg][2 pb][32] x (b1, b2, i1); the loop's last barrier freed LDS
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
      const float ob1 = __shfl_xor(b1[pb], 32);
      const int oi1 = __shfl_xor(i1[pb], 32);
      const float ob2 = __shfl_xor(b2[pb], 32);
      const bool other = ob1 < b1[pb] || (ob1 == b1[pb] && oi1 < i1[pb]);
      const float lose = other ? b1[pb] : ob1;
      b2[pb] = fminf(fminf(b2[pb], ob2), lose);
      if (other) { b1[pb] = ob1; i1[pb] = oi1; }
      if (rh == 1 && h == 0) {
        const int o = ((pg * 2 + pb) * 32 + c32) * 3;
        xb[o] = b1[pb];
        xb[o + 1] = b2[pb];
        xb[o + 2] = __int_as_float(i1[pb]);
      }
    }
    __syncthreads();
    if (rh == 0 && h == 0) {
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) {
        const int o = ((pg * 2 + pb) * 32 + c32) * 3;
        const float ob1 = xb[o], ob2 = xb[o + 1];
        const int oi1 = __float_as_int(xb[o + 2]);
        const bool other = ob1 < b1[pb] || (ob1 == b1[pb] && oi1 < i1[pb]);
        const float lose = other ? b1[pb] : ob1;
        b2[pb] = fminf(fminf(b2[pb], ob2), lose);
        if (other) { b1[pb] = ob1; i1[pb] = oi1; }
        const int64_t po = (int64_t)gc * bpad + sl0[pb];
        ws.part_key[po] = i1[pb] == INT_MAX ? LLONG_MAX : pack_key(b1[pb], (unsigned)i1[pb]);
        ws.part_b2[po] = b2[pb];
      }
    }
  }
  };  // body
  if constexpr (COLLECT) {
    // collect pass: n_ptiles carries the collect plan's chunk count; the grid strides over
    // the (chunk, queued probe tile) items, so a handful of queued probes still spread over
    // the whole grid instead of one workgroup per main-pass chunk
    const int n_amb = *ws.amb_count;
    const int items = ((n_amb + 256 - 1) / 256) * n_ptiles;
    for (int item = blockIdx.x; item < items; item += gridDim.x) body(item % n_ptiles, item / n_ptiles, n_amb);
  } else {
    const int total = gridDim.x;  // host guarantees total % 8 == 0
    const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
    const int bsz = cblk * pblk;
    const int blk = lin / bsz, rr = lin - blk * bsz;
    const int nbp = n_ptiles / pblk;
    body((blk / nbp) * cblk + rr / pblk, (blk % nbp) * pblk + rr % pblk, 0);
  }
}

// ---------------------------------------------------------------------------------------
// Split-bf16 wide scan on v_mfma_f32_16x16x32_bf16 (EF_OPT_SEARCH_SPLIT_BF16 = 1; 2 keeps
// search_wide3_kernel).  Same plan, tiles, DMA and SearchWs contract as search_wide3_kernel:
// 256 rows x 256 probes per workgroup, 8 waves, wave w = probes 64 (w & 3) ..+64 (four
// 16-probe B blocks pb) x rows 128 (w >> 2) ..+128 (eight 16-row A blocks rb).  Per 32-k
// slice lane (qd = lane >> 4, r16 = lane & 15) supplies row r16 of each A block and probe
// r16 of each B block for elements 8 qd .. 8 qd + 7 of the slice — chunk 2 qd (hi) and
// 2 qd + 1 (lo) of the 128-B slice row: 16 + 8 ds_read_b128 feed 96 MFMAs of 16 cycles
// (the 32x32x16 kernel: the same 24 reads for 48 MFMAs of 32 cycles).  Under the chip's
// clock on random bf16 operands the 16x16x32 shape delivers ~1.12-1.15x the FLOP/s of
// 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS give-back item 7).
// LDS swizzle: ds_read_b128 serves lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... in one
// LDS cycle each (MI355X_MICROARCH.md §LDS): rows 0-3 / 12-15 at chunk c meet rows 4-11 at
// chunk c + 2.  Physical chunk = logical ^ s(row) with s(row) = (row >> 1) & 5 (s in
// {0, 1, 4, 5}, so c ^ s and (c + 2) ^ s' never coincide within a lane group and the row
// pairs 2m, 2m + 1 fill both 32-bank halves): every group covers all 64 banks.  The wide3
// swizzle (row >> 1) & 7 would be 2-way conflicted here.
// Accumulator layout: acc[rb][pb][r] = row 16 rb + 4 qd + r of probe 16 pb + r16.
// HI1 (EF_OPT_SEARCH_SPLIT_BF16 = 3, the bf16 screen): the operands are the single-bf16
// copies of hi_rows_kernel (ef_search.hip) — per 64-element k slice, chunk 2q = elements
// 8q .. 8q + 7 and chunk 2q + 1 = elements 32 + 8q .. 32 + 8q + 7, so a slice row is the same
// 128 B, read by the same fragment code and swizzle: "hi" is the slice's first 32-k step,
// "lo" its second, two MFMAs per 64 k instead of three per 32 k.  Launched with the row
// length in 4-byte units (kp / 2); scores carry bf16 rounding of both operands, which the
// screen's bound (reduce_kernel<.., 2>) covers.
template <int KP, int METRIC, bool COLLECT, bool HI1 = false>
__global__ __launch_bounds__(512, 1) void search_wide16_kernel(
    const float* __restrict__ q3, const float* __restrict__ G3, const float* __restrict__ aux, int64_t n,
    int n_ptiles, int tiles_per_chunk, int pblk, int cblk, int64_t bpad, SearchWs ws, int kp_rt) {
  const WideGeom<KP> geo(kp_rt);
  const int NS = geo.ns;
  __shared__ __attribute__((aligned(16))) float smem[4 * W3SL + 2 * W3R];

  auto body = [&](const int gc, const int pt, const int n_amb) {

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qd = lane >> 4, r16 = lane & 15;
  const int pg = wave & 3, rh = wave >> 2;

  const int64_t tiles_total = (n + W3R - 1) / W3R;
  const int64_t t0 = (int64_t)gc * tiles_per_chunk;
  const int64_t t1 = t0 + tiles_per_chunk < tiles_total ? t0 + tiles_per_chunk : tiles_total;
  int64_t sl0[4];  // this lane's probe slots (probe 16 pb + r16 of the wave's 64)
#pragma unroll
  for (int pb = 0; pb < 4; ++pb) sl0[pb] = (int64_t)pt * W3P + 64 * pg + 16 * pb + r16;

  if (t0 >= t1) {
    if constexpr (!COLLECT) {
      if (qd == 0 && rh == 0) {
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          ws.part_key[(int64_t)gc * bpad + sl0[pb]] = LLONG_MAX;
          ws.part_b2[(int64_t)gc * bpad + sl0[pb]] = __builtin_inff();
        }
      }
    }
    return;
  }

  // DMA geometry of search_wide3_kernel with this kernel's swizzle: lane l of piece j
  // carries row 8 j + (l >> 3), physical chunk l & 7 = logical chunk (l & 7) ^ s(row),
  // s(row) = (row >> 1) & 5 = (4 jj + (l >> 4)) & 5.
  const int prow = lane >> 3;
#if EF_WIDE_ROLES
  // split roles: waves 0-3 carry the 32 gallery pieces of a slice (8 each, issued at the
  // slice's start: the gallery streams from HBM / MALL), waves 4-7 the 32 probe pieces
  // (L2-resident, issued at the stagger point)
  const bool gwave = wave < 4;
  unsigned off[8];
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int j = (wave & 3) * 8 + jj;
    const unsigned lch16 = (unsigned)(((lane & 7) ^ ((4 * jj + (lane >> 4)) & 5)) * 16);
    if (gwave) {
      off[jj] = (unsigned)(j * 8 + prow) * (geo.kp * 4) + lch16;
    } else {
      const int slot = pt * W3P + j * 8 + prow;
      int qrow = slot;
      if constexpr (COLLECT) qrow = slot < n_amb ? ws.amb_list[slot] : 0;
      off[jj] = (unsigned)qrow * (geo.kp * 4) + lch16;
    }
  }
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) asm volatile("" ::"v"(off[jj]));
#else
  unsigned goff[4], qoff[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int slot = pt * W3P + (wave * 4 + jj) * 8 + prow;
    int qrow = slot;
    if constexpr (COLLECT) qrow = slot < n_amb ? ws.amb_list[slot] : 0;
    const unsigned lch16 = (unsigned)(((lane & 7) ^ ((4 * jj + (lane >> 4)) & 5)) * 16);
    goff[jj] = (unsigned)((wave * 4 + jj) * 8 + prow) * (geo.kp * 4) + lch16;
    qoff[jj] = (unsigned)qrow * (geo.kp * 4) + lch16;
  }
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) asm volatile("" ::"v"(qoff[jj]));
#endif
  float thr[4] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  if constexpr (COLLECT) {
#pragma unroll
    for (int pb = 0; pb < 4; ++pb)
      if (sl0[pb] < n_amb) thr[pb] = ws.thr[sl0[pb]];
  }
  asm volatile("" ::"v"(thr[0]), "v"(thr[1]), "v"(thr[2]), "v"(thr[3]));

  const unsigned lds_base = lds_addr(smem);
  const int64_t n_it = (t1 - t0) * NS;
  // DMA piece p (0..7) of slice it into buffer buf: p >> 1 = this wave's piece jj, p & 1 =
  // gallery (0) or probes (1)
  auto issue_piece = [&](int64_t it, int buf, int p) {
    const int64_t t = t0 + geo.tile(it);
    int sl = geo.slice(it);
#if EF_WIDE_SERP
    // serpentine k order: odd tiles of the sweep walk the slices backwards, so the probe
    // slices used last by one tile are the first the next tile re-reads (L2 reuse)
    if ((t - t0) & 1) sl = NS - 1 - sl;
#endif
#if EF_WIDE_ROLES
    const int jj = p, j = (wave & 3) * 8 + jj;
    if (gwave) {
      const int nrem = (int)((n - t * W3R) < W3R ? (n - t * W3R) : W3R);
      const unsigned long long gb = (unsigned long long)(size_t)(G3 + t * W3R * geo.kp + sl * WBK);
      unsigned go = off[jj];
      if (nrem < W3R) {  // tail tile: rows past the end re-read the last row (masked later)
        const unsigned row = go / (geo.kp * 4);
        go = (row < (unsigned)nrem ? row : (unsigned)(nrem - 1)) * (geo.kp * 4) + go % (geo.kp * 4);
      }
      glds16s(go, gb, lds_base + (unsigned)((buf * 2 * W3SL + j * 256) * 4));
    } else {
      const unsigned long long qb = (unsigned long long)(size_t)(q3 + sl * WBK);
      glds16s(off[jj], qb, lds_base + (unsigned)((buf * 2 * W3SL + W3SL + j * 256) * 4));
    }
#else
    const int jj = p >> 1, j = wave * 4 + jj;
    if ((p & 1) == 0) {
      const int nrem = (int)((n - t * W3R) < W3R ? (n - t * W3R) : W3R);
      const unsigned long long gb = (unsigned long long)(size_t)(G3 + t * W3R * geo.kp + sl * WBK);
      unsigned go = goff[jj];
      if (nrem < W3R) {  // tail tile: rows past the end re-read the last row (masked later)
        const unsigned row = go / (geo.kp * 4);
        go = (row < (unsigned)nrem ? row : (unsigned)(nrem - 1)) * (geo.kp * 4) + go % (geo.kp * 4);
      }
      glds16s(go, gb, lds_base + (unsigned)((buf * 2 * W3SL + j * 256) * 4));
    } else {
      const unsigned long long qb = (unsigned long long)(size_t)(q3 + sl * WBK);
      glds16s(qoff[jj], qb, lds_base + (unsigned)((buf * 2 * W3SL + W3SL + j * 256) * 4));
    }
#endif
  };
  auto issue = [&](int64_t it, int buf) {
    const int64_t t = t0 + geo.tile(it);
    const int sl = geo.slice(it);
    const int nrem = (int)((n - t * W3R) < W3R ? (n - t * W3R) : W3R);
#pragma unroll
    for (int p = 0; p < 8; ++p) issue_piece(it, buf, p);
    if (sl == 0 && wave == 0) {  // the tile's ||g||^2 (L2) or 1/||g|| (cosine)
      const unsigned long long ab = (unsigned long long)(size_t)(aux + t * W3R);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 64 * q + lane;
        const unsigned ao = r < nrem ? (unsigned)r * 4 : (unsigned)(nrem - 1) * 4;
        glds4s(ao, ab, lds_base + (unsigned)((4 * W3SL + ((t - t0) & 1) * W3R + 64 * q) * 4));
      }
    }
  };

  const float INF = __builtin_inff();
  float b1[4] = {INF, INF, INF, INF}, b2[4] = {INF, INF, INF, INF};
  int i1[4] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX};
  // v[rb][r] = row rowbase + 16 rb + 4 qd + r (increasing with (rb, r): first-min in lane)
  auto consume = [&](const f32x4 (&v)[8], int rowbase, int pb) {
    if constexpr (COLLECT) {
#pragma unroll
      for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (v[rb][r] <= thr[pb]) {
            const int pos = atomicAdd(&ws.cand_cnt[sl0[pb]], 1);
            if (pos < kCandMax) ws.cand[sl0[pb] * kCandMax + pos] = rowbase + 16 * rb + 4 * qd + r;
          }
        }
    } else {
      // L2: v holds the raw accumulators a (score -2 a, exact): the block's best score is
      // -2 max(a), so the skip test needs 16 v_max3 and one multiply instead of 32
      // multiplies and 16 v_min3, and only a block that passes it scales its values.
      // Cosine: v holds the scores.  (fminf / fmaxf would re-canonicalise every MFMA
      // result first: one v_max_f32 x, x per input in IEEE mode)
      float mn;
      if constexpr (METRIC == EF_METRIC_L2) {
        float mx = v[0][0];
#pragma unroll
        for (int e = 1; e + 1 < 32; e += 2) mx = max3_raw(mx, v[e >> 2][e & 3], v[(e + 1) >> 2][(e + 1) & 3]);
        mn = -2.f * fmaxf(mx, v[7][3]);
      } else {
        mn = v[0][0];
#pragma unroll
        for (int e = 1; e + 1 < 32; e += 2) mn = min3_raw(mn, v[e >> 2][e & 3], v[(e + 1) >> 2][(e + 1) & 3]);
        mn = fminf(mn, v[7][3]);
      }
      if (!__any(mn < b2[pb])) return;  // exact skip (ef_search.hip consume)
      float m1 = INF, m2 = INF;
      int ir = 0;
#pragma unroll
      for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = METRIC == EF_METRIC_L2 ? -2.f * v[rb][r] : v[rb][r];
          const bool lt = x < m1;
          m2 = __builtin_amdgcn_fmed3f(m1, x, m2);
          ir = lt ? 16 * rb + r : ir;
          m1 = lt ? x : m1;
        }
      const bool lt = m1 < b1[pb];
      b2[pb] = lt ? fminf(b1[pb], m2) : fminf(b2[pb], m1);
      i1[pb] = lt ? rowbase + ir + 4 * qd : i1[pb];
      b1[pb] = lt ? m1 : b1[pb];
    }
  };

  issue(0, 0);
  dma_wait_all();
  __syncthreads();

  const int sw = (r16 >> 1) & 5;  // s(row) of every row / probe this lane reads
  const int ph = ((2 * qd) ^ sw) * 4, pl = ((2 * qd + 1) ^ sw) * 4;
  f32x4 acc[8][4];
  for (int64_t it = 0; it < n_it; ++it) {
    const int buf = (int)(it & 1);
    const int sl = geo.slice(it);
    const float* const sAux = smem + 4 * W3SL + (int)(geo.tile(it) & 1) * W3R + 128 * rh;
#if EF_WIDE_ABL == 3
    const bool more = it + 1 < 2;  // diagnostic builds only: no slice DMA after the first (results invalid)
#else
    const bool more = it + 1 < n_it;
#endif
#if EF_WIDE_STAGGER
    // waves w and w + 4 share a SIMD: the upper four issue their DMA burst half-way through
    // the slice, so each SIMD's MFMA pipe is fed by one wave while the other issues
    if (more && wave < 4) issue(it + 1, buf ^ 1);
#else
    if (more) issue(it + 1, buf ^ 1);  // lands under this slice's MFMAs
#endif
    if (sl == 0) {
      // L2: start from -||g||^2 / 2 and accumulate q.g (-2 acc = ||g||^2 - 2 q.g); cosine: 0
#pragma unroll
      for (int rb = 0; rb < 8; ++rb) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        if constexpr (METRIC == EF_METRIC_L2) {
          const float4 x = *reinterpret_cast<const float4*>(sAux + 16 * rb + 4 * qd);
          a = f32x4{-0.5f * x.x, -0.5f * x.y, -0.5f * x.z, -0.5f * x.w};
        }
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) acc[rb][pb] = a;
      }
    }
    const float* sg = smem + buf * 2 * W3SL + (128 * rh + r16) * WBK;
    const float* sq = smem + buf * 2 * W3SL + W3SL + (64 * pg + r16) * WBK;
    bf16x8w bh[4], bl[4];
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      bh[pb] = as_bf16x8w(*reinterpret_cast<const float4*>(sq + 16 * pb * WBK + ph));
      bl[pb] = as_bf16x8w(*reinterpret_cast<const float4*>(sq + 16 * pb * WBK + pl));
    }
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const bf16x8w ah = as_bf16x8w(*reinterpret_cast<const float4*>(sg + 16 * rb * WBK + ph));
      const bf16x8w al = as_bf16x8w(*reinterpret_cast<const float4*>(sg + 16 * rb * WBK + pl));
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        if constexpr (HI1) {  // k steps 0 and 1 of the 64-k slice
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[pb], acc[rb][pb], 0, 0, 0);
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bl[pb], acc[rb][pb], 0, 0, 0);
        } else {  // hi.hi' + hi.lo' + lo.hi'
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[pb], acc[rb][pb], 0, 0, 0);
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[pb], acc[rb][pb], 0, 0, 0);
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[pb], acc[rb][pb], 0, 0, 0);
        }
      }
#if EF_WIDE_STAGGER
      if (rb == EF_WIDE_STAGGER - 1 && more && wave >= 4) issue(it + 1, buf ^ 1);
#endif
    }
    if (sl == NS - 1) {
      const int64_t t = t0 + geo.tile(it);
      const int tbase = (int)(t * W3R) + 128 * rh;
      const bool tail = (t + 1) * W3R > n;
#pragma unroll
      for (int rb = 0; rb < 8; ++rb) {
        const float4 x = *reinterpret_cast<const float4*>(sAux + 16 * rb + 4 * qd);
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          // main pass, L2: the raw accumulators go to consume (see there); rows past the
          // gallery's end become -inf there (score +inf)
          constexpr bool raw = METRIC == EF_METRIC_L2 && !COLLECT;
          if constexpr (METRIC == EF_METRIC_L2) {
            if constexpr (!raw) {
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[rb][pb][r] *= -2.f;
            }
          } else {  // -(q.g) * (1/||g||)
            acc[rb][pb][0] *= -x.x;
            acc[rb][pb][1] *= -x.y;
            acc[rb][pb][2] *= -x.z;
            acc[rb][pb][3] *= -x.w;
          }
          if (tail) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (tbase + 16 * rb + 4 * qd + r >= n) acc[rb][pb][r] = raw ? -INF : INF;
          }
        }
      }
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        const f32x4 v[8] = {acc[0][pb], acc[1][pb], acc[2][pb], acc[3][pb],
                            acc[4][pb], acc[5][pb], acc[6][pb], acc[7][pb]};
#if EF_WIDE_ABL == 2
        {  // diagnostic builds only: the screen's min without the top-2 update (every
           // accumulator stays live, so no MFMA is dead code)
          float mn = v[0][0];
#pragma unroll
          for (int e = 1; e + 1 < 32; e += 2) mn = min3_raw(mn, v[e >> 2][e & 3], v[(e + 1) >> 2][(e + 1) & 3]);
          b1[pb] = fminf(b1[pb], fminf(mn, v[7][3]));
        }
#else
        consume(v, tbase, pb);
#endif
      }
    }
#if EF_WIDE_ABL != 1
    dma_wait_all();
    __syncthreads();  // slice it+1 landed; everyone is done reading buffer buf
#endif
  }

  if constexpr (!COLLECT) {
    // the four row quarters (lanes r16, +16, +32, +48), then the two row halves via LDS
    float* xb = smem;  // [4 pg][4 pb][16] x (b1, b2, i1); the loop's last barrier freed LDS
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
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
      if (rh == 1 && qd == 0) {
        const int o = ((pg * 4 + pb) * 16 + r16) * 3;
        xb[o] = b1[pb];
        xb[o + 1] = b2[pb];
        xb[o + 2] = __int_as_float(i1[pb]);
      }
    }
    __syncthreads();
    if (rh == 0 && qd == 0) {
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        const int o = ((pg * 4 + pb) * 16 + r16) * 3;
        const float ob1 = xb[o], ob2 = xb[o + 1];
        const int oi1 = __float_as_int(xb[o + 2]);
        const bool other = ob1 < b1[pb] || (ob1 == b1[pb] && oi1 < i1[pb]);
        const float lose = other ? b1[pb] : ob1;
        b2[pb] = fminf(fminf(b2[pb], ob2), lose);
        if (other) { b1[pb] = ob1; i1[pb] = oi1; }
        const int64_t po = (int64_t)gc * bpad + sl0[pb];
        ws.part_key[po] = i1[pb] == INT_MAX ? LLONG_MAX : pack_key(b1[pb], (unsigned)i1[pb]);
        ws.part_b2[po] = b2[pb];
      }
    }
  }
  };  // body
  if constexpr (COLLECT) {
    const int n_amb = *ws.amb_count;
    const int items = ((n_amb + 256 - 1) / 256) * n_ptiles;
    for (int item = blockIdx.x; item < items; item += gridDim.x) body(item % n_ptiles, item / n_ptiles, n_amb);
  } else {
    const int total = gridDim.x;  // host guarantees total % 8 == 0
    const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
    const int bsz = cblk * pblk;
    const int blk = lin / bsz, rr = lin - blk * bsz;
    const int nbp = n_ptiles / pblk;
    body((blk / nbp) * cblk + rr / pblk, (blk % nbp) * pblk + rr % pblk, 0);
  }
}

template <int KP, int M, bool HI1 = false>
static hipError_t wide3_t(hipStream_t s, bool collect, bool w16, const SearchPlan& pl, const float* q3,
                          const float* G3, const float* aux, int64_t n, int64_t bpad, const SearchWs& ws, int kp) {
  const dim3 grid((unsigned)(pl.nchunks * pl.n_ptiles)), block(512);
  if (pl.n_ptiles % pl.pblk != 0 || pl.nchunks % pl.cblk != 0 || (pl.nchunks * pl.n_ptiles) % 8 != 0 ||
      (pl.nchunks * pl.n_ptiles / 8) % (pl.cblk * pl.pblk) != 0 || bpad % W3P != 0)
    return hipErrorInvalidValue;  // the block deal would not be a bijection
  if (w16 || HI1) {
    if (collect)
      hipLaunchKernelGGL((search_wide16_kernel<KP, M, true, HI1>), dim3((unsigned)pl.c_grid), block, 0, s, q3, G3,
                         aux, n, pl.c_chunks, pl.c_tpc, pl.pblk, pl.cblk, bpad, ws, kp);
    else
      hipLaunchKernelGGL((search_wide16_kernel<KP, M, false, HI1>), grid, block, 0, s, q3, G3, aux, n, pl.n_ptiles,
                         pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws, kp);
  } else if (collect) {
    hipLaunchKernelGGL((search_wide3_kernel<KP, M, true>), dim3((unsigned)pl.c_grid), block, 0, s, q3, G3, aux, n,
                       pl.c_chunks, pl.c_tpc, pl.pblk, pl.cblk, bpad, ws, kp);
  } else {
    hipLaunchKernelGGL((search_wide3_kernel<KP, M, false>), grid, block, 0, s, q3, G3, aux, n, pl.n_ptiles,
                       pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws, kp);
  }
  return hipGetLastError();
}

template <int KP, int M>
static hipError_t wide_t(hipStream_t s, bool collect, int s3, const SearchPlan& pl, const float* qpad,
                         const float* G, const float* aux, int64_t n, int64_t bpad, const SearchWs& ws, int kp) {
  const dim3 grid((unsigned)(pl.nchunks * pl.n_ptiles)), block(256);
  if (pl.n_ptiles % pl.pblk != 0 || pl.nchunks % pl.cblk != 0 || (pl.nchunks * pl.n_ptiles) % 8 != 0 ||
      (pl.nchunks * pl.n_ptiles / 8) % (pl.cblk * pl.pblk) != 0)
    return hipErrorInvalidValue;  // the block deal would not be a bijection
  // 32-bit geometry of the kernels: probe rows addressed by unsigned byte offsets, and (KP = 0)
  // the flattened (tile, slice) counter of a sweep divided in 32 bits
  const int64_t ns = kp / WBK;
  if (kp % 128 != 0 || bpad * (int64_t)kp * 4 >= ((int64_t)1 << 31) ||
      (int64_t)std::max(pl.tiles_per_chunk, pl.c_tpc) * ns >= ((int64_t)1 << 31))
    return hipErrorInvalidValue;
  // plan from search_plan(.., true); s3 = 1: the 16x16x32 kernel, 2: the 32x32x16 one
  if (s3) return wide3_t<KP, M>(s, collect, s3 != 2, pl, qpad, G, aux, n, bpad, ws, kp);
  if (collect)
    hipLaunchKernelGGL((search_wide_kernel<KP, M, true>), dim3((unsigned)pl.c_grid), block, 0, s, qpad, G, aux, n,
                       pl.c_chunks, pl.c_tpc, pl.pblk, pl.cblk, bpad, ws, kp);
  else
    hipLaunchKernelGGL((search_wide_kernel<KP, M, false>), grid, block, 0, s, qpad, G, aux, n, pl.n_ptiles,
                       pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws, kp);
  return hipGetLastError();
}

hipError_t launch_search_wide(hipStream_t s, int kp, int metric, bool collect, int s3, const SearchPlan& pl,
                              const float* qpad, const float* G, const float* aux, int64_t n, int64_t bpad,
                              const SearchWs& ws) {
  const bool l2 = metric == EF_METRIC_L2;
  if (s3 == 3) {  // the bf16 screen on single-bf16 copies: rows of kp / 2 four-byte units
    const int kh = kp / 2;
    const int64_t ns = kh / WBK;
    if (kp % 128 != 0 || bpad * (int64_t)kh * 4 >= ((int64_t)1 << 31) ||
        (int64_t)std::max(pl.tiles_per_chunk, pl.c_tpc) * ns >= ((int64_t)1 << 31))
      return hipErrorInvalidValue;
    // main pass at the compiled widths: the gallery-in-VGPRs screen (ef_search_screen.hip)
    if (!collect && (kh == 128 || kh == 256) && screen_vg_enabled())
      return launch_search_screen(s, kh, metric, pl, qpad, G, aux, n, bpad, ws);
    switch (kp) {
      case 256:
        return l2 ? wide3_t<128, EF_METRIC_L2, true>(s, collect, true, pl, qpad, G, aux, n, bpad, ws, kh)
                  : wide3_t<128, EF_METRIC_COSINE, true>(s, collect, true, pl, qpad, G, aux, n, bpad, ws, kh);
      case 512:
        return l2 ? wide3_t<256, EF_METRIC_L2, true>(s, collect, true, pl, qpad, G, aux, n, bpad, ws, kh)
                  : wide3_t<256, EF_METRIC_COSINE, true>(s, collect, true, pl, qpad, G, aux, n, bpad, ws, kh);
      default:
        if (kp <= 512) return hipErrorInvalidValue;
        return l2 ? wide3_t<0, EF_METRIC_L2, true>(s, collect, true, pl, qpad, G, aux, n, bpad, ws, kh)
                  : wide3_t<0, EF_METRIC_COSINE, true>(s, collect, true, pl, qpad, G, aux, n, bpad, ws, kh);
    }
  }
  switch (kp) {
    case 256:
      return l2 ? wide_t<256, EF_METRIC_L2>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws, kp)
                : wide_t<256, EF_METRIC_COSINE>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws, kp);
    case 512:
      return l2 ? wide_t<512, EF_METRIC_L2>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws, kp)
                : wide_t<512, EF_METRIC_COSINE>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws, kp);
    default:  // k > 512: row length at run time
      if (kp <= 512) return hipErrorInvalidValue;
      return l2 ? wide_t<0, EF_METRIC_L2>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws, kp)
                : wide_t<0, EF_METRIC_COSINE>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws, kp);
  }
}

}  // namespace ef
