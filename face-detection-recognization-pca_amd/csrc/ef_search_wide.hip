// Distance GEMM + fused arg-best for wide features, KP in {256, 512} (BASELINE.json
// config 5: k = 512 eigenfaces).  Same contract as search_kernel in ef_search.hip (per
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

#include <climits>

namespace ef {

// Diagnostic builds only (timing, wrong results): EF_WIDE_ABL 1 = no per-slice barrier,
// 2 = no arg-best epilogue, 3 = no DMA after the first slices.
#ifndef EF_WIDE_ABL
#define EF_WIDE_ABL 0
#endif
#ifndef EF_WIDE_INTERLEAVE
#define EF_WIDE_INTERLEAVE 0
#endif

constexpr int WR = kWideRowTile;    // gallery rows per tile
constexpr int WP = kWideProbeTile;  // probes per workgroup
constexpr int WBK = 32;             // k per slice
constexpr int WSL = WR * WBK;       // floats per gallery slice (= per probe slice)
static_assert(WR == 128 && WP == 128, "4 waves x 32 probes, 4 x 32-row blocks");

typedef short bf16x8w __attribute__((ext_vector_type(8)));
__device__ __forceinline__ bf16x8w as_bf16x8w(const float4& v) {
  bf16x8w r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}

// S3: qpad and G are the split-bf16 copies (ef_search.hip: per 8 elements 16 B of hi, 16 B
// of lo) — same bytes per row, so the slice DMA is unchanged; each 32-k slice is two
// 16-k fragments (chunks 4h + 2i = hi, 4h + 2i + 1 = lo of lane half h), 3 bf16 MFMAs each.
template <int KP, int METRIC, bool COLLECT, bool S3 = false>
__global__ __launch_bounds__(256, 2) void search_wide_kernel(
    const float* __restrict__ qpad, const float* __restrict__ G, const float* __restrict__ aux, int64_t n,
    int n_ptiles, int tiles_per_chunk, int pblk, int cblk, int64_t bpad, SearchWs ws) {
  constexpr int NS = KP / WBK;  // slices per tile
  // [stage 0: gallery | probes][stage 1: gallery | probes][aux of even | odd tiles]
  // (aux is double-buffered by tile: the cosine epilogue reads it in the tile's last
  // slice, when the DMA of the next tile's first slice is already in flight)
  __shared__ __attribute__((aligned(16))) float smem[4 * WSL + 2 * WR];

  const int total = gridDim.x;  // host guarantees total % 8 == 0
  const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
  // (chunk, probe tile) blocks of cblk x pblk, one block per XCD (see search_plan)
  const int bsz = cblk * pblk;
  const int blk = lin / bsz, r = lin - blk * bsz;
  const int nbp = n_ptiles / pblk;
  const int gc = (blk / nbp) * cblk + r / pblk;
  const int pt = (blk % nbp) * pblk + r % pblk;

  int n_amb = 0;
  if constexpr (COLLECT) {
    n_amb = *ws.amb_count;
    if (pt * WP >= n_amb) return;  // uniform: nothing queued for this probe tile
  }

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
    goff[jj] = (unsigned)((wave * 4 + jj) * 8 + prow) * (KP * 4) + lch16;
    qoff[jj] = (unsigned)qrow * (KP * 4) + lch16;
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
    const int64_t t = t0 + it / NS;
    const int sl = (int)(it % NS);
    const int nrem = (int)((n - t * WR) < WR ? (n - t * WR) : WR);
    const unsigned long long gb = (unsigned long long)(size_t)(G + t * WR * KP + sl * WBK);
    const unsigned long long qb = (unsigned long long)(size_t)(qpad + sl * WBK);
    const int j = wave * 4 + jj;
    unsigned go = goff[jj];
    if (nrem < WR) {  // tail tile: rows past the end re-read the last row (masked later)
      const unsigned row = go / (KP * 4);
      go = (row < (unsigned)nrem ? row : (unsigned)(nrem - 1)) * (KP * 4) + go % (KP * 4);
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
    const int sl = (int)(it % NS);
    const float* const sAux = smem + 4 * WSL + (int)((it / NS) & 1) * WR;
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
    if constexpr (S3) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ph = ((h * 4 + 2 * i) ^ sw) * 4, pl = ((h * 4 + 2 * i + 1) ^ sw) * 4;
        const bf16x8w bh = as_bf16x8w(*reinterpret_cast<const float4*>(sq + (wave * 32 + c32) * WBK + ph));
        const bf16x8w bl = as_bf16x8w(*reinterpret_cast<const float4*>(sq + (wave * 32 + c32) * WBK + pl));
        bf16x8w ah[4], al[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          ah[rb] = as_bf16x8w(*reinterpret_cast<const float4*>(sg + (rb * 32 + c32) * WBK + ph));
          al[rb] = as_bf16x8w(*reinterpret_cast<const float4*>(sg + (rb * 32 + c32) * WBK + pl));
        }
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[rb], bh, acc[rb], 0, 0, 0);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[rb], bl, acc[rb], 0, 0, 0);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[rb], bh, acc[rb], 0, 0, 0);
      }
    } else
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
      const int64_t t = t0 + it / NS;
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
}

template <int KP, int M>
static hipError_t wide_t(hipStream_t s, bool collect, bool s3, const SearchPlan& pl, const float* qpad,
                         const float* G, const float* aux, int64_t n, int64_t bpad, const SearchWs& ws) {
  const dim3 grid((unsigned)(pl.nchunks * pl.n_ptiles)), block(256);
  if (pl.n_ptiles % pl.pblk != 0 || pl.nchunks % pl.cblk != 0 || (pl.nchunks * pl.n_ptiles) % 8 != 0 ||
      (pl.nchunks * pl.n_ptiles / 8) % (pl.cblk * pl.pblk) != 0)
    return hipErrorInvalidValue;  // the block deal would not be a bijection
  if (s3) {
    if (collect)
      hipLaunchKernelGGL((search_wide_kernel<KP, M, true, true>), grid, block, 0, s, qpad, G, aux, n, pl.n_ptiles,
                         pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
    else
      hipLaunchKernelGGL((search_wide_kernel<KP, M, false, true>), grid, block, 0, s, qpad, G, aux, n,
                         pl.n_ptiles, pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
  } else if (collect)
    hipLaunchKernelGGL((search_wide_kernel<KP, M, true>), grid, block, 0, s, qpad, G, aux, n, pl.n_ptiles,
                       pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
  else
    hipLaunchKernelGGL((search_wide_kernel<KP, M, false>), grid, block, 0, s, qpad, G, aux, n, pl.n_ptiles,
                       pl.tiles_per_chunk, pl.pblk, pl.cblk, bpad, ws);
  return hipGetLastError();
}

hipError_t launch_search_wide(hipStream_t s, int kp, int metric, bool collect, bool s3, const SearchPlan& pl,
                              const float* qpad, const float* G, const float* aux, int64_t n, int64_t bpad,
                              const SearchWs& ws) {
  const bool l2 = metric == EF_METRIC_L2;
  switch (kp) {
    case 256:
      return l2 ? wide_t<256, EF_METRIC_L2>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws)
                : wide_t<256, EF_METRIC_COSINE>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws);
    case 512:
      return l2 ? wide_t<512, EF_METRIC_L2>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws)
                : wide_t<512, EF_METRIC_COSINE>(s, collect, s3, pl, qpad, G, aux, n, bpad, ws);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace ef
