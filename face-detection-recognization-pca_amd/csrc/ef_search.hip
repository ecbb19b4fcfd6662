// Distance GEMM with fused arg-best epilogue.
//
// Replaces `cosine_similarity([f], face_features)` + `np.argmax`
// (scan-template-v4.py:274-275) and the per-row Python loop of useless/scan.py:122-127,
// batched over B probes, plus the north-star L2 argmin.
//
// Layout in HBM:  gallery G[n][KP] fp32 (k zero-padded to KP), gnorm2[n], ginv[n];
// probe features Qp[bpad][KP] (bpad a multiple of 256).
//
// Pass 1 — search_kernel (the hot kernel, v_mfma_f32_32x32x2_f32, exact fp32):
//   * workgroup = 8 waves = 256 probes; each wave keeps 32 probes (one 32-probe
//     B-operand block, KP/2 fp32 VGPRs, pre-scaled) in registers for the whole sweep;
//   * the workgroup sweeps one chunk of the gallery in 64-row tiles (two 32-row MFMA
//     blocks = two independent accumulator chains per wave) staged through
//     double-buffered LDS by LDS-DMA (global_load_lds, ef_dma.hpp), tile t+1's DMA in
//     flight under tile t's MFMAs;
//   * the gallery tile is the MFMA A operand so each lane's 16 accumulators hold 16
//     gallery rows of ONE probe: the arg-best is an in-lane running (best, index,
//     runner-up) with no cross-lane traffic until one __shfl_xor(32) at the end;
//   * K is permuted (lane half h owns k in [h*KP/2, (h+1)*KP/2)) so every A fragment is a
//     conflict-free ds_read_b128 feeding 4 MFMAs;
//   * blockIdx is remapped so the workgroups sharing a gallery chunk run on one XCD
//     (same blockIdx % 8) and hit its L2;
//   * each workgroup writes its per-probe (best key, runner-up score) for its chunk.
// Pass 2 — reduce_kernel: per probe, min over chunks -> winner + global runner-up; the
//   winner is re-scored in fp64 (difference form for L2).  A rigorous fp32 error bound
//   decides whether the runner-up could beat the winner; if so the probe is queued.
// Pass 3 (only for queued probes; a no-op launch otherwise) — the search kernel in
//   COLLECT mode gathers every row whose fp32 score is within the bound, and
//   resolve_kernel re-scores them in fp64 and keeps the lowest index among exact ties.
// Result: the argmin/argmax identity equals an fp64 evaluation with lowest-index
// tie-break (np.argmin / np.argmax semantics), independent of fp32 rounding.
//
// Split-bf16 scores (S3, EF_OPT_SEARCH_SPLIT_BF16): every fp32 operand x is carried as
// x = hi + lo + e with hi = bf16(x), lo = bf16(x - hi), |e| <= 2^-16 |x|, and the dot
// product is hi.hi' + hi.lo' + lo.hi' on v_mfma_f32_32x32x16_bf16 (products exact in fp32,
// fp32 accumulation): 3 bf16 MFMAs per 16 k instead of 8 fp32 ones, i.e. 16/3 x the
// arithmetic rate.  The gallery's split copy has the fp32 row's byte layout (per 8
// elements: 16 B of hi, 16 B of lo), so the tile DMA and the LDS reads are those of the
// fp32 kernel.  The pass-2 bound covers the dropped terms (lo.lo', e) and the longer
// chain; the winner is still re-scored from the fp32 gallery in fp64, so keys and match
// records equal the fp32 path's bit for bit whenever both resolve
// (tests/test_gpu_search_split.py; at the full C3 size, tests/test_gpu_c3_full.py).
#include "ef_search_common.hpp"

#include <climits>
#include <cstdlib>
#include <cmath>

namespace ef {

constexpr int TG = 64;  // gallery rows per LDS tile (two 32-row MFMA blocks)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// round-to-nearest-even fp32 -> bf16 bits (finite inputs) and back
__device__ __forceinline__ unsigned bf16_bits(float x) {
  const unsigned u = __float_as_uint(x);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_value(unsigned b) { return __uint_as_float(b << 16); }
// 8 consecutive fp32 values -> (hi, lo) bf16x8 fragments
__device__ __forceinline__ void split8(const float* x, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned h = bf16_bits(x[j]);
    hi[j] = (short)h;
    lo[j] = (short)bf16_bits(x[j] - bf16_value(h));
  }
}
__device__ __forceinline__ bf16x8 as_bf16x8(const float4& v) {
  bf16x8 r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}

// Workgroup = 8 waves x 32 probes = 256 probes (the gallery is swept Bpad/256 times).
// Each wave keeps its 32 probes as one B block (KP/2 VGPRs, pre-scaled) and runs the
// tile's two 32-row blocks as two independent accumulator chains; the arg-best epilogue
// is a branch-free top-2 in row order on registers.  <= 128 VGPRs -> 4 waves per SIMD.
// ABL (diagnostic builds only, results invalid): bit 1 skips the epilogue, bit 4 skips
// the per-tile wait + barrier.
template <int KP, int METRIC, bool COLLECT, bool S3 = false, int ABL = 0>
__global__ __launch_bounds__(512, 4) void search_kernel(
    const float* __restrict__ qpad, const float* __restrict__ G, const float* __restrict__ aux, int64_t n,
    int n_ptiles, int tiles_per_chunk, int64_t bpad, SearchWs ws) {
  constexpr int NW = 8;
  constexpr int KH = KP / 2;
  constexpr int CPR = KP / 4;                                          // 16-B chunks per row
  constexpr int SW = (CPR & 15) == 0 ? 16 : ((CPR & 7) == 0 ? 8 : 4);  // XOR swizzle width
  constexpr int NI = TG * CPR / 64;                                    // 1-KiB LDS-DMA pieces per tile
  constexpr int PPW = (NI + NW - 1) / NW;                              // pieces per wave
  constexpr int RP = 64 / CPR;                                         // rows per piece
  static_assert((NI % NW == 0 || NI < NW) && RP * CPR == 64 && TG == 64, "tile must be whole 1-KiB pieces");
  // KP = 128 (the k = 128 headline shape): no swizzle.  LDS piece p (1 KiB + 16 B pad)
  // holds row p of the tile's first 32-row block and row 32 + p of the second, so the
  // lane reading row c32 of either block uses one base (c32 * 1040 B) plus immediate
  // offsets — no per-read VALU address math, which costs MFMA issue cycles
  // (tools/micro/mfma_valu_probe.cpp) — and the 1040-B stride (260 = 4 mod 64 banks)
  // keeps every ds_read_b128 lane group conflict-free.  One full-wave DMA per piece.
  constexpr bool PAD = KP == 128;
  constexpr int PS = 2 * KP + 4;          // PAD: floats per piece (two rows + 16 B)
  constexpr int TGS = PAD ? 32 * PS : TG * KP;  // floats per tile buffer

  // Unpadded [TG][KP] tiles filled by global_load_lds (lane-linear 1-KiB pieces); the
  // chunk order inside each row is XOR-swizzled by (row & (SW-1)) on the SOURCE address so
  // the A-fragment ds_read_b128s (16 lanes = 16 rows, same logical chunk) hit distinct
  // banks.  All LDS lives in one array (a second __shared__ object can de-pipeline).
  __shared__ __attribute__((aligned(16))) float smem[2 * TGS + 2 * TG];
  float* const sG0 = smem;
  float* const sAux0 = smem + 2 * TGS;

  // one (gallery chunk gc, probe tile pt) work item
  auto body = [&](const int gc, const int pt, const int n_amb) {

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int lrow = lane / CPR, lc = lane % CPR;  // this lane's (row, chunk) inside a piece

  const int64_t tiles_total = (n + TG - 1) / TG;
  const int64_t t0 = (int64_t)gc * tiles_per_chunk;
  const int64_t t1 = t0 + tiles_per_chunk < tiles_total ? t0 + tiles_per_chunk : tiles_total;
  const int64_t s0 = (int64_t)pt * 256 + wave * 32 + c32;  // this lane's probe slot

  if (t0 >= t1) {  // empty chunk: publish "no candidate" so the reducer can skip it
    if constexpr (!COLLECT) {
      if (h == 0) {
        ws.part_key[(int64_t)gc * bpad + s0] = LLONG_MAX;
        ws.part_b2[(int64_t)gc * bpad + s0] = __builtin_inff();
      }
    }
    return;
  }

  // Issue the LDS-DMA of tile t into buffer buf.  Wave w fills pieces [w*PPW, (w+1)*PPW);
  // a piece is RP whole rows.  The swizzle splits into a lane constant and a wave-uniform
  // part: row & (SW-1) == ((j*RP) & (SW-1)) ^ (lrow & (SW-1)) for power-of-two RP, SW.
  // Rows past n (tail tile only) are clamped to a valid row and masked in the epilogue.
  const int lcx = lc ^ (lrow & (SW - 1));
  const unsigned lds_base = lds_addr(smem);
  // Full tiles use the SGPR-base DMA form: per piece one v_xor + one v_lshl_add (every VALU
  // instruction in this loop costs MFMA issue time); the tail tile clamps rows instead.
  auto issue_tile = [&](int64_t t, int buf) {
    const int nrem = (int)((n - t * TG) < TG ? (n - t * TG) : TG);
    if constexpr (PAD) {  // piece p = rows p (lanes 0-31) and 32 + p (lanes 32-63)
      const unsigned m0 = lds_base + (unsigned)(buf * TGS * 4);
      unsigned lid;  // re-derived in place (a loop-long VGPR would be spilled by hipcc)
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
      if (nrem == TG) {
        const unsigned long long gb = uniform_ptr(G + t * TG * KP);
        if (wave == 0) glds4s(lid * 4u, uniform_ptr(aux + t * TG), lds_base + (unsigned)((2 * TGS + buf * TG) * 4));
        const unsigned voff = ((lid >> 5) * 32 * KP + (lid & 31) * 4) * 4;
#pragma unroll
        for (int jj = 0; jj < PPW; ++jj) {
          const int p = wave * PPW + jj;
          glds16s(voff, gb + (unsigned long long)(p * KP * 4), m0 + (unsigned)(p * PS * 4));
        }
      } else {
        const float* gbase = G + t * TG * KP;
#pragma unroll
        for (int jj = 0; jj < PPW; ++jj) {
          const int p = wave * PPW + jj;
          int row = p + (int)(lid >> 5) * 32;
          row = row < nrem ? row : nrem - 1;
          glds16(gbase + row * KP + (lid & 31) * 4, m0 + (unsigned)(p * PS * 4));
        }
        if (wave == 0) {
          const int row = (int)lid < nrem ? (int)lid : nrem - 1;
          glds4(aux + t * TG + row, lds_base + (unsigned)((2 * TGS + buf * TG) * 4));
        }
      }
      return;
    }
    int lx = lcx, lr = lrow;
    asm volatile("" : "+v"(lx), "+v"(lr));  // recompute per tile (no hoisted per-piece VGPRs)
    if (nrem == TG) {
      const unsigned long long gb = uniform_ptr(G + t * TG * KP);
      const unsigned lro = (unsigned)(lr * KP * 4);
#pragma unroll
      for (int jj = 0; jj < PPW; ++jj) {
        const int j = wave * PPW + jj;
        if (NI >= NW || wave < NI) {  // uniform
          const int sj = (j * RP) & (SW - 1);
          glds16s(lro + ((unsigned)(lx ^ sj) << 4), gb + (unsigned long long)(j * RP * KP * 4),
                  lds_base + (unsigned)((buf * TGS + j * 256) * 4));
        }
      }
      if (wave == 0) glds4s((unsigned)lane * 4u, uniform_ptr(aux + t * TG), lds_base + (unsigned)((2 * TGS + buf * TG) * 4));
    } else {
      const float* gbase = G + t * TG * KP;  // wave-uniform
#pragma unroll
      for (int jj = 0; jj < PPW; ++jj) {
        const int j = wave * PPW + jj;
        if (NI >= NW || wave < NI) {  // uniform
          const int sj = (j * RP) & (SW - 1);
          int row = j * RP + lr;
          row = row < nrem ? row : nrem - 1;
          glds16(gbase + row * KP + ((lx ^ sj) << 2), lds_base + (unsigned)((buf * TGS + j * 256) * 4));
        }
      }
      if (wave == 0) {
        const int row = lane < nrem ? lane : nrem - 1;
        glds4(aux + t * TG + row, lds_base + (unsigned)((2 * TGS + buf * TG) * 4));  // one 4-B piece per lane
      }
    }
  };

  issue_tile(t0, 0);

  // Probe fragments (B operand): lane holds probe c32, k in [h*KH, h*KH+KH), pre-scaled
  // (exactly) so the chain yields the score: L2 acc = ||g||^2 + sum(-2q)g (the chain
  // starts from ||g||^2), cosine acc = -q.g (times 1/||g|| after the chain).
  constexpr float QS = METRIC == EF_METRIC_L2 ? -2.f : -1.f;
  // S3: the same k range as split (hi, lo) bf16x8 fragments, fragment i = k h*KH + 8i + [0, 8)
  constexpr int NF = KH / 8;
  float qb[S3 ? 1 : KH];
  bf16x8 qh[S3 ? NF : 1], ql[S3 ? NF : 1];
  {
    int64_t r0 = s0;
    bool v0 = true;
    if constexpr (COLLECT) {
      v0 = s0 < n_amb;
      r0 = v0 ? ws.amb_list[s0] : 0;
    }
    const float4* q0 = reinterpret_cast<const float4*>(qpad + r0 * KP + h * KH);
    if constexpr (S3) {
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const float4 a = v0 ? q0[2 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 b = v0 ? q0[2 * i + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float t[8] = {QS * a.x, QS * a.y, QS * a.z, QS * a.w, QS * b.x, QS * b.y, QS * b.z, QS * b.w};
        split8(t, qh[i], ql[i]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < KH / 4; ++j) {
        const float4 a = v0 ? q0[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        qb[4 * j] = QS * a.x; qb[4 * j + 1] = QS * a.y; qb[4 * j + 2] = QS * a.z; qb[4 * j + 3] = QS * a.w;
      }
    }
  }
  float thr = -__builtin_inff();
  if constexpr (COLLECT) {
    if (s0 < n_amb) thr = ws.thr[s0];
  }
  // Consume every probe register here, so hipcc places its waits for these loads before
  // the loop; otherwise its (loop-merged) wait state puts vmcnt(0) inside the tile loop,
  // which would also drain the asm LDS-DMA of the next tile.
  if constexpr (S3) {
#pragma unroll
    for (int i = 0; i < NF; ++i) asm volatile("" ::"v"(qh[i]), "v"(ql[i]));
  } else {
#pragma unroll
    for (int j = 0; j < KH; ++j) asm volatile("" ::"v"(qb[j]));
  }
  asm volatile("" ::"v"(thr));

  const float INF = __builtin_inff();
  float b1 = INF, b2 = INF;
  int i1 = INT_MAX;

  // Arg-best epilogue of one finished block of scores v (register r <-> row
  // rowbase + (r&3) + 8(r>>2) + 4h, increasing with r): branch-free top-2 in row order
  // (strict '<' keeps the lowest row on ties; v_med3 keeps the runner-up), then merged
  // into the running (best, index, runner-up).  COLLECT appends rows within thr instead.
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
      // Screen: a block whose minimum is not below the lane's runner-up changes neither
      // b1, b2 nor i1 (the update below would keep all three), so when no lane of the wave
      // has such a row the block is skipped on a uniform branch — ~8 v_min3 per 16 scores
      // instead of ~64 VALU ops, once the running top-2 has settled.
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

  // Accumulator start value: ||g||^2 of the block's rows for L2 (four float4 reads of the
  // staged norms match the register <-> row map), 0 for cosine.
  auto acc_init = [&](const float* tileA_blk) {
    f32x16 a = {};
    if constexpr (METRIC == EF_METRIC_L2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(tileA_blk + 8 * q + 4 * h);
        a[4 * q] = x.x;
        a[4 * q + 1] = x.y;
        a[4 * q + 2] = x.z;
        a[4 * q + 3] = x.w;
      }
    }
    return a;
  };

  dma_wait_all();
  __syncthreads();  // tile t0 landed

  for (int64_t t = t0; t < t1; ++t) {
    const int buf = (int)((t - t0) & 1);
    if (t + 1 < t1) issue_tile(t + 1, buf ^ 1);  // lands under this tile's MFMAs
    const float* tileG = sG0 + buf * TGS;
    const float* tileA = sAux0 + buf * TG;
    const bool tail = (t + 1) * TG > n;
    const int tbase = (int)(t * TG);
    int swz = PAD ? 0 : c32 & (SW - 1);  // rows c32 and 32 + c32 share (row & (SW-1)), SW <= 16
    // opaque per tile: stops hipcc hoisting all KH/4 swizzled addresses out of the loop
    if constexpr (!PAD) asm volatile("" : "+v"(swz));
    const float* arow0 = tileG + (PAD ? c32 * PS : c32 * KP);
    const float* arow1 = PAD ? arow0 + KP : tileG + (32 + c32) * KP;

    // both 32-row blocks at once: two independent accumulator chains sharing the B operand
    f32x16 acc0 = acc_init(tileA), acc1 = acc_init(tileA + 32);
    if constexpr (S3) {
      // fragment i: chunks 2i (hi) and 2i + 1 (lo) of this lane half's k range
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const int c0 = h * (CPR / 2) + 2 * i;
        const int ch = PAD ? c0 : c0 ^ swz, cl = PAD ? c0 + 1 : (c0 + 1) ^ swz;
        const bf16x8 ah = as_bf16x8(*reinterpret_cast<const float4*>(arow0 + ch * 4));
        const bf16x8 bh = as_bf16x8(*reinterpret_cast<const float4*>(arow1 + ch * 4));
        const bf16x8 al = as_bf16x8(*reinterpret_cast<const float4*>(arow0 + cl * 4));
        const bf16x8 bl = as_bf16x8(*reinterpret_cast<const float4*>(arow1 + cl * 4));
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, qh[i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, qh[i], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, ql[i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, ql[i], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, qh[i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl, qh[i], acc1, 0, 0, 0);
        if (i % 2 == 1) __builtin_amdgcn_sched_barrier(0);  // bound the A prefetch depth
      }
    } else
#pragma unroll
    for (int s = 0; s < KH; s += 4) {
      const int chunk = PAD ? h * (CPR / 2) + s / 4 : (h * (CPR / 2) + s / 4) ^ swz;
      const float4 a = *reinterpret_cast<const float4*>(arow0 + chunk * 4);
      const float4 b = *reinterpret_cast<const float4*>(arow1 + chunk * 4);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, qb[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b.x, qb[s], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, qb[s + 1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b.y, qb[s + 1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, qb[s + 2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b.z, qb[s + 2], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, qb[s + 3], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b.w, qb[s + 3], acc1, 0, 0, 0);
      if ((s / 4) % 2 == 1) __builtin_amdgcn_sched_barrier(0);  // bound the A prefetch depth
    }
    if constexpr (METRIC != EF_METRIC_L2) {  // cosine: -(q.g) * (1/||g||)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(tileA + 8 * q + 4 * h);
        const float4 y = *reinterpret_cast<const float4*>(tileA + 32 + 8 * q + 4 * h);
        acc0[4 * q] *= x.x; acc0[4 * q + 1] *= x.y; acc0[4 * q + 2] *= x.z; acc0[4 * q + 3] *= x.w;
        acc1[4 * q] *= y.x; acc1[4 * q + 1] *= y.y; acc1[4 * q + 2] *= y.z; acc1[4 * q + 3] *= y.w;
      }
    }
    if (tail) {  // uniform: only the last tile has rows past n
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tbase + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= n) acc0[r] = INF;
        if (row + 32 >= n) acc1[r] = INF;
      }
    }
    if constexpr (ABL & 1) {
      asm volatile("" ::"v"(acc0), "v"(acc1));
    } else {
      consume(acc0, tbase);  // rows of block 0 precede block 1 (row-order tie rule)
      consume(acc1, tbase + 32);
    }
    if constexpr (!(ABL & 4)) {
      dma_wait_all();
      __syncthreads();  // tile t+1 landed; everyone is done reading buffer buf
    }
  }

  if constexpr (!COLLECT) {
    // Merge the two lane halves (same probe, disjoint rows).
    const float ob1 = __shfl_xor(b1, 32);
    const int oi1 = __shfl_xor(i1, 32);
    const float ob2 = __shfl_xor(b2, 32);
    const bool other = ob1 < b1 || (ob1 == b1 && oi1 < i1);
    const float lose = other ? b1 : ob1;
    b2 = fminf(fminf(b2, ob2), lose);
    if (other) { b1 = ob1; i1 = oi1; }
    if (h == 0) {
      const int64_t o = (int64_t)gc * bpad;
      ws.part_key[o + s0] = i1 == INT_MAX ? LLONG_MAX : pack_key(b1, (unsigned)i1);
      ws.part_b2[o + s0] = b2;
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
    // XCD-aware mapping: blocks b and b+8 share an XCD; give each XCD a contiguous run of
    // (chunk, probe-tile) pairs so the probe tiles of one chunk are co-resident on it.
    const int total = gridDim.x;  // host guarantees total % 8 == 0
    const int lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
    const int gc = lin / n_ptiles;
    body(gc, lin - gc * n_ptiles, 0);
  }
}

// Split-bf16 scan on v_mfma_f32_16x16x32_bf16, KP = 128 (the C3 shape).  Same workgroup,
// tile, LDS layout (the padded two-row pieces) and SearchWs contract as search_kernel; the
// 16 x 16 shape is chosen because under the clock the chip holds on bf16 MFMA loads it
// delivers more FLOP/s than 32 x 32 at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS
// give-back item 7).  Lane l = (quarter qd = l >> 4, r16 = l & 15): it supplies row r16
// of each 16-row A block and probe r16 of each 16-probe B block for k-quarter qd, where
// quarter qd of step i is elements 32 qd + 8 i + [0, 8) (chunks 8 qd + 2i = hi, + 1 = lo
// of the row: one ds_read_b128 each, conflict-free on the 1040-B piece stride).  A wave
// keeps 32 probes as two B blocks (pb) and runs the tile's four 16-row blocks (rb) against
// both: 8 accumulators of 4 rows (row 16 rb + 4 qd + reg, probe 16 pb + r16), 96 MFMAs per
// 64-row tile.  Each lane carries the running top-2 of its two probes; the four quarters
// are merged by two shuffles at the end.
template <int METRIC, bool COLLECT>
__global__ __launch_bounds__(512, 4) void search16_kernel(
    const float* __restrict__ qpad, const float* __restrict__ G3, const float* __restrict__ aux, int64_t n,
    int n_ptiles, int tiles_per_chunk, int64_t bpad, SearchWs ws) {
  constexpr int KP = 128, PS = 2 * KP + 4, TGS = 32 * PS, PPW = 4;  // 8 waves x 4 pieces
  __shared__ __attribute__((aligned(16))) float smem[2 * TGS + 2 * TG];
  float* const sAux0 = smem + 2 * TGS;

  // one (gallery chunk gc, probe tile pt) work item
  auto body = [&](const int gc, const int pt, const int n_amb) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qd = lane >> 4, r16 = lane & 15;
  const int64_t tiles_total = (n + TG - 1) / TG;
  const int64_t t0 = (int64_t)gc * tiles_per_chunk;
  const int64_t t1 = t0 + tiles_per_chunk < tiles_total ? t0 + tiles_per_chunk : tiles_total;
  int64_t sl0[2];
  sl0[0] = (int64_t)pt * 256 + wave * 32 + r16;
  sl0[1] = sl0[0] + 16;

  if (t0 >= t1) {
    if constexpr (!COLLECT) {
      if (qd == 0) {
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
          ws.part_key[(int64_t)gc * bpad + sl0[pb]] = LLONG_MAX;
          ws.part_b2[(int64_t)gc * bpad + sl0[pb]] = __builtin_inff();
        }
      }
    }
    return;
  }

  // tile DMA: search_kernel's padded layout (piece p = rows p and 32 + p + 16 B)
  const unsigned lds_base = lds_addr(smem);
  auto issue_tile = [&](int64_t t, int buf) {
    const int nrem = (int)((n - t * TG) < TG ? (n - t * TG) : TG);
    const unsigned m0 = lds_base + (unsigned)(buf * TGS * 4);
    unsigned lid;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
    if (nrem == TG) {
      const unsigned long long gb = uniform_ptr(G3 + t * TG * KP);
      if (wave == 0) glds4s(lid * 4u, uniform_ptr(aux + t * TG), lds_base + (unsigned)((2 * TGS + buf * TG) * 4));
      const unsigned voff = ((lid >> 5) * 32 * KP + (lid & 31) * 4) * 4;
#pragma unroll
      for (int jj = 0; jj < PPW; ++jj) {
        const int p = wave * PPW + jj;
        // rows 4..11 of every 16 land with their 128-B quarter pairs swapped (see abase)
        glds16s(((p >> 2) & 3) - 1u < 2u ? voff ^ 128u : voff, gb + (unsigned long long)(p * KP * 4),
                m0 + (unsigned)(p * PS * 4));
      }
    } else {
      const float* gbase = G3 + t * TG * KP;
#pragma unroll
      for (int jj = 0; jj < PPW; ++jj) {
        const int p = wave * PPW + jj;
        int row = p + (int)(lid >> 5) * 32;
        row = row < nrem ? row : nrem - 1;
        glds16(gbase + row * KP + ((lid & 31) ^ (((p >> 2) & 3) - 1u < 2u ? 8u : 0u)) * 4, m0 + (unsigned)(p * PS * 4));
      }
      if (wave == 0) {
        const int row = (int)lid < nrem ? (int)lid : nrem - 1;
        glds4(aux + t * TG + row, lds_base + (unsigned)((2 * TGS + buf * TG) * 4));
      }
    }
  };
  issue_tile(t0, 0);

  // probes: lane's k-quarter of probes 16 pb + r16, pre-scaled like search_kernel
  constexpr float QS = METRIC == EF_METRIC_L2 ? -2.f : -1.f;
  bf16x8 qh[2][4], ql[2][4];
  float thr[2] = {-__builtin_inff(), -__builtin_inff()};
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    int64_t r0 = sl0[pb];
    bool v0 = true;
    if constexpr (COLLECT) {
      v0 = sl0[pb] < n_amb;
      r0 = v0 ? ws.amb_list[sl0[pb]] : 0;
      if (v0) thr[pb] = ws.thr[sl0[pb]];
    }
    const float4* q0 = reinterpret_cast<const float4*>(qpad + r0 * KP + qd * 32);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 a = v0 ? q0[2 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 b = v0 ? q0[2 * i + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float t[8] = {QS * a.x, QS * a.y, QS * a.z, QS * a.w, QS * b.x, QS * b.y, QS * b.z, QS * b.w};
      split8(t, qh[pb][i], ql[pb][i]);
    }
  }
#pragma unroll
  for (int pb = 0; pb < 2; ++pb)
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(qh[pb][i]), "v"(ql[pb][i]));
  asm volatile("" ::"v"(thr[0]), "v"(thr[1]));

  const float INF = __builtin_inff();
  float b1[2] = {INF, INF}, b2[2] = {INF, INF};
  int i1[2] = {INT_MAX, INT_MAX};
  // v[rb] = rows 16 rb + 4 qd + reg of probe block pb (increasing with (rb, reg))
  auto consume = [&](const f32x4 (&v)[4], int tbase, int pb) {
    if constexpr (COLLECT) {
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (v[rb][r] <= thr[pb]) {
            const int pos = atomicAdd(&ws.cand_cnt[sl0[pb]], 1);
            if (pos < kCandMax) ws.cand[sl0[pb] * kCandMax + pos] = tbase + 16 * rb + 4 * qd + r;
          }
        }
    } else {
      float mn = v[0][0];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) mn = fminf(mn, v[rb][r]);
      if (!__any(mn < b2[pb])) return;  // exact skip (search_kernel consume)
      float m1 = INF, m2 = INF;
      int ir = 0;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = v[rb][r];
          const bool lt = x < m1;
          m2 = __builtin_amdgcn_fmed3f(m1, x, m2);
          ir = lt ? 16 * rb + r : ir;
          m1 = lt ? x : m1;
        }
      const bool lt = m1 < b1[pb];
      b2[pb] = lt ? fminf(b1[pb], m2) : fminf(b2[pb], m1);
      i1[pb] = lt ? tbase + ir + 4 * qd : i1[pb];
      b1[pb] = lt ? m1 : b1[pb];
    }
  };

  dma_wait_all();
  __syncthreads();
  // lane's A base: row r16 of block rb lives in piece 16 (rb & 1) + r16, half rb >> 1.
  // ds_read_b128 serves lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... together
  // (MI355X_MICROARCH.md §LDS): quarters qd and qd + 1 of rows 4..11 vs 0-3 / 12-15 would
  // share banks on the 1040-B piece stride, so those rows hold their 128-B quarter pairs
  // swapped (chunk ^ 8, applied by the DMA) — every lane group then covers all 64 banks.
  const int qsw = ((r16 >> 2) - 1u) < 2u ? 8 : 0;
  const int abase = r16 * PS + ((8 * qd) ^ qsw) * 4;  // floats, + 16 PS (rb & 1) + KP (rb >> 1) + 8 i
  for (int64_t t = t0; t < t1; ++t) {
    const int buf = (int)((t - t0) & 1);
    if (t + 1 < t1) issue_tile(t + 1, buf ^ 1);
    const float* tileG = smem + buf * TGS + abase;
    const float* tileA = sAux0 + buf * TG;
    f32x4 acc[4][2];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
      if constexpr (METRIC == EF_METRIC_L2) {
        const float4 x = *reinterpret_cast<const float4*>(tileA + 16 * rb + 4 * qd);
        a = f32x4{x.x, x.y, x.z, x.w};
      }
      acc[rb][0] = a;
      acc[rb][1] = a;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const float* ar = tileG + 16 * PS * (rb & 1) + KP * (rb >> 1) + 8 * i;
        const bf16x8 ah = as_bf16x8(*reinterpret_cast<const float4*>(ar));
        const bf16x8 al = as_bf16x8(*reinterpret_cast<const float4*>(ar + 4));
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, qh[pb][i], acc[rb][pb], 0, 0, 0);
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, ql[pb][i], acc[rb][pb], 0, 0, 0);
          acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, qh[pb][i], acc[rb][pb], 0, 0, 0);
        }
      }
      if (i % 2 == 1) __builtin_amdgcn_sched_barrier(0);
    }
    const int tbase = (int)(t * TG);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      if constexpr (METRIC != EF_METRIC_L2) {  // cosine: -(q.g) * (1/||g||)
        const float4 x = *reinterpret_cast<const float4*>(tileA + 16 * rb + 4 * qd);
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
          acc[rb][pb][0] *= x.x; acc[rb][pb][1] *= x.y; acc[rb][pb][2] *= x.z; acc[rb][pb][3] *= x.w;
        }
      }
      if ((t + 1) * TG > n) {  // uniform: only the last tile has rows past n
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (tbase + 16 * rb + 4 * qd + r >= n) {
            acc[rb][0][r] = INF;
            acc[rb][1][r] = INF;
          }
      }
    }
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
      const f32x4 v[4] = {acc[0][pb], acc[1][pb], acc[2][pb], acc[3][pb]};
      consume(v, tbase, pb);
    }
    dma_wait_all();
    __syncthreads();
  }

  if constexpr (!COLLECT) {
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {  // merge the four row quarters
        const float ob1 = __shfl_xor(b1[pb], off);
        const int oi1 = __shfl_xor(i1[pb], off);
        const float ob2 = __shfl_xor(b2[pb], off);
        const bool other = ob1 < b1[pb] || (ob1 == b1[pb] && oi1 < i1[pb]);
        const float lose = other ? b1[pb] : ob1;
        b2[pb] = fminf(fminf(b2[pb], ob2), lose);
        if (other) { b1[pb] = ob1; i1[pb] = oi1; }
      }
      if (qd == 0) {
        const int64_t o = (int64_t)gc * bpad + sl0[pb];
        ws.part_key[o] = i1[pb] == INT_MAX ? LLONG_MAX : pack_key(b1[pb], (unsigned)i1[pb]);
        ws.part_b2[o] = b2[pb];
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
    const int gc = lin / n_ptiles;
    body(gc, lin - gc * n_ptiles, 0);
  }
}

// One wave per probe: winner over chunks, global runner-up, fp64 re-score, ambiguity test.
// KP = 0: row length kp_rt at run time (k > 512).
// S3: the scan's arithmetic — 0 fp32, 1 split bf16 (hi + lo), 2 single bf16 (the screen of
// EF_OPT_SEARCH_SPLIT_BF16 = 3) — which sets the bound below.
template <int KP, int METRIC, int S3 = 0>
__global__ __launch_bounds__(256) void reduce_kernel(const float* __restrict__ qpad, int64_t b, int64_t bpad,
                                                     int nchunks, const float* __restrict__ G, int64_t n,
                                                     int64_t g_offset, float gmax2, SearchWs ws,
                                                     long long* __restrict__ keys, int kp_rt) {
  const int kpv = KP > 0 ? KP : kp_rt;
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= b) return;
  long long kmin = LLONG_MAX;
  for (int c = lane; c < nchunks; c += 64) {
    const long long k = ws.part_key[(int64_t)c * bpad + p];
    kmin = k < kmin ? k : kmin;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const long long o = __shfl_xor(kmin, off);
    kmin = o < kmin ? o : kmin;
  }
  if (kmin == LLONG_MAX) {  // empty gallery
    if (lane == 0) {
      keys[p] = LLONG_MAX;
      if (ws.match) ws.match[p] = ef_match{__builtin_inf(), 0.0, LLONG_MAX};
    }
    return;
  }
  float r2 = __builtin_inff();
  for (int c = lane; c < nchunks; c += 64) {
    const long long k = ws.part_key[(int64_t)c * bpad + p];
    r2 = fminf(r2, ws.part_b2[(int64_t)c * bpad + p]);
    if (k != kmin && k != LLONG_MAX) r2 = fminf(r2, key_value(k));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) r2 = fminf(r2, __shfl_xor(r2, off));

  const float b1 = key_value(kmin);
  const unsigned row = (unsigned)(kmin & 0xffffffffll);
  const float* q = qpad + p * kpv;
  const double v = score64<KP, METRIC>(q, G + (int64_t)row * kpv, lane, kpv);
  // rigorous bound on |fp32 score - exact score| (fp32 FMA chain of KP terms,
  // fp32 ||g||^2 / 1/||g||, final rounding), doubled for the two compared scores
  float qq = 0.f;
  for (int c = lane; c < kpv; c += 64) qq = __builtin_fmaf(q[c], q[c], qq);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) qq += __shfl_xor(qq, off);
  const float u = 5.9604645e-08f;  // 2^-24
  const float qn = sqrtf(qq);
  float delta;
  if constexpr (S3 == 2) {
    // single-bf16 chain: |x - bf16(x)| <= 2^-8 |x| for both operands, so each product is
    // within (2 + 2^-8) 2^-8 |q||g| of the exact one (2.01 2^-8 taken); KP exact products +
    // the start value summed in fp32 (2u per add allowed), ||g||^2 itself to KP u
    const float es = 2.01f * 3.90625e-03f;  // 2.01 * 2^-8
    if constexpr (METRIC == EF_METRIC_L2) {
      const float gm = sqrtf(gmax2);
      delta = 2.f * (2.f * es * qn * gm + (kpv + 4) * 2.f * u * 1.01f * (2.02f * qn * gm + gmax2) +
                     kpv * u * gmax2 + 4.f * u * fabsf(b1)) + 1e-30f;
    } else {
      delta = 2.f * ((es + (kpv + 8) * 2.f * u) * 1.01f * qn) + 1e-30f;
    }
  } else if constexpr (S3 == 1) {
    // split-bf16 chain: dropped terms (lo.lo', hi.e', lo.e', e.q) <= 3.02 * 2^-16 |q||g| per
    // element, 3 KP exact products + the start value summed in fp32 (2u per add allowed, in
    // case the matrix core's adds do not round to nearest), ||g||^2 itself to KP u
    const float es = 3.05f * 1.5258789e-05f;  // 3.05 * 2^-16
    if constexpr (METRIC == EF_METRIC_L2) {
      const float gm = sqrtf(gmax2);
      delta = 2.f * (2.f * es * qn * gm + (3 * kpv + 4) * 2.f * u * 1.01f * (2.02f * qn * gm + gmax2) +
                     kpv * u * gmax2 + 4.f * u * fabsf(b1)) + 1e-30f;
    } else {
      delta = 2.f * ((es + (3 * kpv + 8) * 2.f * u) * 1.01f * qn) + 1e-30f;
    }
  } else if constexpr (METRIC == EF_METRIC_L2) {
    const float gm = sqrtf(gmax2);
    delta = 2.f * ((kpv + 4) * u * 1.01f * (2.f * qn * gm + gmax2) + 4.f * u * fabsf(b1));
  } else {
    delta = 2.f * ((kpv + 8) * u * 1.01f * qn) + 1e-30f;
  }
  delta *= 2.f;  // safety factor
  double qq64 = 0.0;  // tie-tolerance scale of the fp64 resolution (resolve_kernel)
  if (METRIC == EF_METRIC_L2 && ws.match) {
    for (int c = lane; c < kpv; c += 64) qq64 = fma((double)q[c], (double)q[c], qq64);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) qq64 += __shfl_xor(qq64, off);
  }
  if (lane == 0) {
    keys[p] = pack_key((float)v, (unsigned)(row + g_offset));
    if (ws.match)
      ws.match[p] = ef_match{v, METRIC == EF_METRIC_L2 ? qq64 + (double)gmax2 : 1.0,
                             pack_key((float)v, (unsigned)(row + g_offset))};
    if (r2 - b1 <= delta) {
      const int slot = atomicAdd(ws.amb_count, 1);
      ws.amb_list[slot] = (int)p;
      ws.thr[slot] = b1 + delta;
      ws.cand_cnt[slot] = 0;
    }
  }
}

// fp64 resolution of queued probes: lowest index among candidates whose fp64 score is
// within 1e-12 (relative) of the best — exact ties resolve like np.argmin/argmax.
template <int KP, int METRIC>
__global__ __launch_bounds__(256) void resolve_kernel(const float* __restrict__ qpad, const float* __restrict__ G,
                                                      int64_t n, int64_t g_offset, float gmax2, SearchWs ws,
                                                      long long* __restrict__ keys, int kp_rt) {
  const int kpv = KP > 0 ? KP : kp_rt;
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= *ws.amb_count) return;
  const int64_t p = ws.amb_list[slot];
  const float* q = qpad + p * kpv;
  const int cnt = ws.cand_cnt[slot];
  const bool overflow = cnt > kCandMax;
  const int64_t m = overflow ? n : cnt;
  auto row_of = [&](int64_t j) -> int64_t { return overflow ? j : (int64_t)ws.cand[slot * kCandMax + j]; };
  double vmin = INFINITY;
  for (int64_t j = 0; j < m; ++j) {
    const double v = score64<KP, METRIC>(q, G + row_of(j) * kpv, lane, kpv);
    vmin = v < vmin ? v : vmin;
  }
  double qq = 0.0;
  for (int c = lane; c < kpv; c += 64) qq = fma((double)q[c], (double)q[c], qq);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) qq += __shfl_xor(qq, off);
  const double scale = METRIC == EF_METRIC_L2 ? qq + (double)gmax2 : 1.0;
  const double tol = 1e-12 * (fabs(vmin) + scale);
  int64_t best_row = LLONG_MAX;
  double best_v = vmin;
  for (int64_t j = 0; j < m; ++j) {
    const int64_t r = row_of(j);
    const double v = score64<KP, METRIC>(q, G + r * kpv, lane, kpv);
    if (v <= vmin + tol && r < best_row) { best_row = r; best_v = v; }
  }
  if (lane == 0 && best_row != LLONG_MAX) {
    const long long key = pack_key((float)best_v, (unsigned)(best_row + g_offset));
    keys[p] = key;
    if (ws.match) {
      ws.match[p].score = best_v;
      ws.match[p].key = key;
    }
  }
}

// dst[rows_pad][kp] <- src[rows][k] with zero padding.
__global__ void pad_rows_kernel(const float* __restrict__ src, int64_t rows, int k, int64_t rows_pad,
                                float* __restrict__ dst, int kp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_pad * kp) return;
  const int64_t r = i / kp;
  const int c = (int)(i - r * kp);
  dst[i] = (r < rows && c < k) ? src[r * k + c] : 0.f;
}

// ||g||^2 and 1/||g|| per gallery row (K7: computed once at enrolment, not per probe as
// sklearn's cosine_similarity does, pairwise.py:1734), and max ||g||^2 for the bound.
__global__ void gallery_aux_kernel(const float* __restrict__ G, int64_t n, int kp, float* __restrict__ gnorm2,
                                   float* __restrict__ ginv) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  float s = 0.f;
  for (int c = lane; c < kp; c += 64) {
    const float v = G[row * kp + c];
    s = __builtin_fmaf(v, v, s);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) {
    gnorm2[row] = s;
    ginv[row] = s > 0.f ? 1.0f / sqrtf(s) : 0.f;
  }
}

// Split-bf16 copy of the gallery (S3 search): per 8 fp32 elements, 16 B of hi = bf16(x)
// then 16 B of lo = bf16(x - hi); same row bytes as the fp32 gallery.
__global__ void split_rows_kernel(const float* __restrict__ G, int64_t groups, uint4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= groups) return;
  const float4 a = reinterpret_cast<const float4*>(G)[2 * i];
  const float4 b = reinterpret_cast<const float4*>(G)[2 * i + 1];
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  unsigned hi[8], lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = bf16_bits(x[j]);
    lo[j] = bf16_bits(x[j] - bf16_value(hi[j]));
  }
  out[2 * i] = make_uint4(hi[0] | hi[1] << 16, hi[2] | hi[3] << 16, hi[4] | hi[5] << 16, hi[6] | hi[7] << 16);
  out[2 * i + 1] = make_uint4(lo[0] | lo[1] << 16, lo[2] | lo[3] << 16, lo[4] | lo[5] << 16, lo[6] | lo[7] << 16);
}

// Single-bf16 copy (the bf16 screen, EF_OPT_SEARCH_SPLIT_BF16 = 3; wide kernels): per 64
// fp32 elements, 128 B = eight 16-B chunks, chunk 2q = bf16(x[8q .. 8q + 7]) and chunk
// 2q + 1 = bf16(x[32 + 8q .. 32 + 8q + 7]) — the split copy's slice row bytes and fragment
// order, so search_wide16_kernel<.., HI1> reads it with the split code (half the bytes).
__global__ void hi_rows_kernel(const float* __restrict__ G, int64_t blocks, uint4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= blocks) return;
  const float4* x = reinterpret_cast<const float4*>(G) + 16 * i;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int e0 = (c & 1) * 32 + (c >> 1) * 8;  // first element of chunk c
    const float4 a = x[e0 / 4], b = x[e0 / 4 + 1];
    out[8 * i + c] = make_uint4(bf16_bits(a.x) | bf16_bits(a.y) << 16, bf16_bits(a.z) | bf16_bits(a.w) << 16,
                                bf16_bits(b.x) | bf16_bits(b.y) << 16, bf16_bits(b.z) | bf16_bits(b.w) << 16);
  }
}

// max ||g||^2 (one atomic per block; non-negative floats order as their bit patterns)
__global__ __launch_bounds__(256) void max_kernel(const float* __restrict__ x, int64_t n, unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) m = fmaxf(m, x[i]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(out, __float_as_uint(m));
  }
}

// ------------------------------------------------------------------------ launchers
SearchPlan search_plan(int64_t bpad, int64_t n, int kp, bool s3) {
  SearchPlan pl;
  const bool wide = kp > 128;
  const bool w3 = wide && s3;  // split-bf16 wide kernel: 256 x 256 tiles, one workgroup per CU
  pl.n_ptiles = (int)(bpad / (w3 ? kWide3ProbeTile : wide ? kWideProbeTile : kSearchProbeTile));
  const int64_t rows_per_tile = w3 ? kWide3RowTile : wide ? kWideRowTile : TG;
  const int64_t tiles = (n + rows_per_tile - 1) / rows_per_tile;
  // ~512 workgroups = one resident wave of them (2 per CU): every chunk is swept by a
  // workgroup that starts at launch, so there is no tail round (measured: 90.1 % vs 89.6 %
  // at 1M rows, 82 % vs 80.5 % at 125k rows for 2048); the chunk count is a multiple of 8
  // so the XCD remap is a bijection.  EF_SEARCH_WGS overrides (experiments).
#ifdef EF_DIAGNOSTICS
  static const int64_t target0 = [] { const char* e = getenv("EF_SEARCH_WGS"); return e ? atoll(e) : 512; }();
  int64_t target = target0;
#else
  int64_t target = 512;
#endif
  if (w3) target = 256;
  int64_t want = (target + pl.n_ptiles - 1) / pl.n_ptiles;
  if (want > tiles) want = tiles;
  if (want < 1) want = 1;
  pl.nchunks = (int)(((want + 7) / 8) * 8);
  pl.tiles_per_chunk = (int)((tiles + pl.nchunks - 1) / pl.nchunks);
  if (pl.tiles_per_chunk < 1) pl.tiles_per_chunk = 1;
  // Wide kernel: the probes stream through LDS with every gallery tile, so an XCD whose
  // workgroups span all probe tiles re-fetches them from beyond its L2 (32 tiles x 256 KiB
  // at C5 = 8 MiB > 4 MiB L2: 27x the gallery bytes measured).  Deal blocks of 8 probe
  // tiles x cblk chunks to each XCD instead: 2 MiB of probes stay L2-resident and each
  // chunk is read by n_ptiles / 8 XCDs.
  // The split-bf16 wide kernel's probe tiles are 256 x KP x 4 B (512 KiB at KP = 512): 4
  // of them per XCD keep 2 MiB of probes L2-resident.
  // collect plan: ~512 chunks (a few queued probes then spread over the whole chip; with
  // every probe tile queued the grid strides over all items, a main pass's work)
  pl.c_tpc = (int)std::max<int64_t>(1, (tiles + 511) / 512);
  pl.c_chunks = (int)((tiles + pl.c_tpc - 1) / pl.c_tpc);
  pl.c_grid = w3 ? 256 : 512;
#ifndef EF_WIDE3_PB  // probe tiles per XCD block of the split-bf16 wide scan (variant builds: experiments)
#define EF_WIDE3_PB 8
#endif
  const int pb = w3 ? EF_WIDE3_PB : 8;
  pl.pblk = pl.n_ptiles;
  pl.cblk = 1;
  if (wide && pl.n_ptiles % pb == 0 && pl.n_ptiles > pb) {
    const int64_t per_xcd = (int64_t)pl.nchunks * pl.n_ptiles / 8;
    if (per_xcd % pb == 0 && pl.nchunks % (per_xcd / pb) == 0) {
      pl.pblk = pb;
      pl.cblk = (int)(per_xcd / pb);
    }
  }
  return pl;
}

// Split-bf16 search (KP <= 128): S3 kernel on the split gallery G3 for the scan and the
// collect pass; reduce / resolve re-score from the fp32 gallery G as in the fp32 path.
// KP > 128: the wide kernel streams the probes too, so they are split into Q3 first.
// KP = 0: k > 512, row length kp at run time (wide kernels only).
template <int KP, int M>
static hipError_t search_s3_t(hipStream_t s, const SearchPlan& pl, const float* qpad, float* Q3, int64_t bpad,
                              int64_t b, const float* G, const float* G3, const float* aux, int64_t n,
                              int64_t g_offset, float gmax2, const SearchWs& ws, long long* keys, TimerEvt* tev,
                              ef_ctx* c, int kp) {
  if constexpr (KP > 128 || KP == 0) {
    if (!Q3) return hipErrorInvalidValue;
    // 16x16x32 split kernel unless the 32x32x16 one (2) or the single-bf16 screen (3) is asked for
    const int variant = c->opt_search_split_bf16 == 2 || c->opt_search_split_bf16 == 3 ? (int)c->opt_search_split_bf16 : 1;
    hipError_t e = variant == 3 ? launch_hi_rows(s, qpad, bpad, kp, Q3) : launch_split_rows(s, qpad, bpad, kp, Q3);
    if (e != hipSuccess) return e;
    timer_begin(c, EF_KERNEL_SEARCH, tev);
    e = launch_search_wide(s, kp, M, false, variant, pl, Q3, G3, aux, n, bpad, ws);
    timer_end(c, tev);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(ws.amb_count, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    const dim3 pgrid((unsigned)((b + 3) / 4));
    if (variant == 3)
      hipLaunchKernelGGL((reduce_kernel<KP, M, 2>), pgrid, dim3(256), 0, s, qpad, b, bpad, pl.nchunks, G, n,
                         g_offset, gmax2, ws, keys, kp);
    else
      hipLaunchKernelGGL((reduce_kernel<KP, M, 1>), pgrid, dim3(256), 0, s, qpad, b, bpad, pl.nchunks, G, n,
                         g_offset, gmax2, ws, keys, kp);
    e = launch_search_wide(s, kp, M, true, variant, pl, Q3, G3, aux, n, bpad, ws);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((resolve_kernel<KP, M>), pgrid, dim3(256), 0, s, qpad, G, n, g_offset, gmax2, ws, keys, kp);
    return hipGetLastError();
  } else {
    (void)Q3;
    const dim3 grid((unsigned)(pl.nchunks * pl.n_ptiles)), block(512);
    // KP = 128: the 16 x 16 x 32 kernel unless the 32 x 32 x 16 one is asked for (option 2)
    const bool k16 = KP == 128 && c->opt_search_split_bf16 != 2;
    timer_begin(c, EF_KERNEL_SEARCH, tev);
    if (k16)
      hipLaunchKernelGGL((search16_kernel<M, false>), grid, block, 0, s, qpad, G3, aux, n, pl.n_ptiles,
                         pl.tiles_per_chunk, bpad, ws);
    else
      hipLaunchKernelGGL((search_kernel<KP, M, false, true>), grid, block, 0, s, qpad, G3, aux, n, pl.n_ptiles,
                         pl.tiles_per_chunk, bpad, ws);
    timer_end(c, tev);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(ws.amb_count, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    const dim3 pgrid((unsigned)((b + 3) / 4));
    hipLaunchKernelGGL((reduce_kernel<KP, M, 1>), pgrid, dim3(256), 0, s, qpad, b, bpad, pl.nchunks, G, n,
                       g_offset, gmax2, ws, keys, kp);
    if (k16)
      hipLaunchKernelGGL((search16_kernel<M, true>), dim3((unsigned)pl.c_grid), block, 0, s, qpad, G3, aux, n,
                         pl.c_chunks, pl.c_tpc, bpad, ws);
    else
      hipLaunchKernelGGL((search_kernel<KP, M, true, true>), dim3((unsigned)pl.c_grid), block, 0, s, qpad, G3,
                         aux, n, pl.c_chunks, pl.c_tpc, bpad, ws);
    hipLaunchKernelGGL((resolve_kernel<KP, M>), pgrid, dim3(256), 0, s, qpad, G, n, g_offset, gmax2, ws, keys, kp);
    return hipGetLastError();
  }
}

template <int KP, int M>
static hipError_t search_t(hipStream_t s, const SearchPlan& pl, const float* qpad, float* Q3, int64_t bpad,
                           int64_t b, const float* G, const float* G3, const float* aux, int64_t n,
                           int64_t g_offset, float gmax2, const SearchWs& ws, long long* keys, bool timed_main,
                           TimerEvt* tev, ef_ctx* c, int kp) {
  constexpr bool wide = KP > 128 || KP == 0;
  if (G3) return search_s3_t<KP, M>(s, pl, qpad, Q3, bpad, b, G, G3, aux, n, g_offset, gmax2, ws, keys, tev, c, kp);
  const dim3 grid((unsigned)(pl.nchunks * pl.n_ptiles)), block(512);
  if (timed_main) timer_begin(c, EF_KERNEL_SEARCH, tev);
  if constexpr (wide) {
    const hipError_t e = launch_search_wide(s, kp, M, false, 0, pl, qpad, G, aux, n, bpad, ws);
    if (e != hipSuccess) return e;
  } else {
#ifdef EF_DIAGNOSTICS
  static const int abl = [] { const char* e = getenv("EF_SEARCH_ABL"); return e ? atoi(e) : 0; }();
#else
  constexpr int abl = 0;
#endif
  if (KP == 128 && M == EF_METRIC_L2 && abl > 0) {  // diagnostic build only: ablations (timing, wrong results)
#ifdef EF_DIAGNOSTICS
    auto k = abl == 1 ? search_kernel<KP, M, false, false, 1>
                      : abl == 4 ? search_kernel<KP, M, false, false, 4> : search_kernel<KP, M, false, false, 5>;
    hipLaunchKernelGGL(k, grid, block, 0, s, qpad, G, aux, n, pl.n_ptiles, pl.tiles_per_chunk, bpad, ws);
#endif
  } else {
    hipLaunchKernelGGL((search_kernel<KP, M, false>), grid, block, 0, s, qpad, G, aux, n, pl.n_ptiles,
                       pl.tiles_per_chunk, bpad, ws);
  }
  }
  if (timed_main) timer_end(c, tev);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(ws.amb_count, 0, sizeof(int), s);
  if (e != hipSuccess) return e;
  const dim3 pgrid((unsigned)((b + 3) / 4));
  hipLaunchKernelGGL((reduce_kernel<KP, M>), pgrid, dim3(256), 0, s, qpad, b, bpad, pl.nchunks, G, n, g_offset,
                     gmax2, ws, keys, kp);
  // queued (fp32-ambiguous) probes: collect + fp64 resolve; both exit at once when none
  if constexpr (wide) {
    e = launch_search_wide(s, kp, M, true, 0, pl, qpad, G, aux, n, bpad, ws);
    if (e != hipSuccess) return e;
  } else {
    hipLaunchKernelGGL((search_kernel<KP, M, true>), dim3((unsigned)pl.c_grid), block, 0, s, qpad, G, aux, n,
                       pl.c_chunks, pl.c_tpc, bpad, ws);
  }
  hipLaunchKernelGGL((resolve_kernel<KP, M>), pgrid, dim3(256), 0, s, qpad, G, n, g_offset, gmax2, ws, keys, kp);
  return hipGetLastError();
}

hipError_t launch_search(hipStream_t s, int kp, int metric, const SearchPlan& pl, const float* qpad, float* Q3,
                         int64_t bpad, int64_t b, const float* G, const float* G3, const float* aux, int64_t n,
                         int64_t g_offset, float gmax2, const SearchWs& ws, long long* keys, ef_ctx* c) {
  TimerEvt tev;
  tev.kernel = -1;
#define EF_SEARCH_CASE(KPV)                                                                                 \
  case KPV:                                                                                                 \
    return metric == EF_METRIC_L2                                                                           \
               ? search_t<KPV, EF_METRIC_L2>(s, pl, qpad, Q3, bpad, b, G, G3, aux, n, g_offset, gmax2, ws, keys, \
                                             true, &tev, c, kp)                                                   \
               : search_t<KPV, EF_METRIC_COSINE>(s, pl, qpad, Q3, bpad, b, G, G3, aux, n, g_offset, gmax2, ws, \
                                                 keys, true, &tev, c, kp);
  switch (kp) {
    EF_SEARCH_CASE(16)
    EF_SEARCH_CASE(32)
    EF_SEARCH_CASE(64)
    EF_SEARCH_CASE(128)
    EF_SEARCH_CASE(256)
    EF_SEARCH_CASE(512)
    default:  // k > 512 (a multiple of 128): the wide kernels with the row length at run time
      if (kp <= 512 || kp % 128 != 0) return hipErrorInvalidValue;
      return metric == EF_METRIC_L2
                 ? search_t<0, EF_METRIC_L2>(s, pl, qpad, Q3, bpad, b, G, G3, aux, n, g_offset, gmax2, ws, keys, true,
                                             &tev, c, kp)
                 : search_t<0, EF_METRIC_COSINE>(s, pl, qpad, Q3, bpad, b, G, G3, aux, n, g_offset, gmax2, ws, keys,
                                                 true, &tev, c, kp);
  }
#undef EF_SEARCH_CASE
}

__global__ void keys_fill_kernel(long long* keys, int64_t b, ef_match* match) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < b) {
    keys[i] = LLONG_MAX;
    if (match) match[i] = ef_match{__builtin_inf(), 0.0, LLONG_MAX};
  }
}

hipError_t launch_keys_none(hipStream_t s, long long* keys, int64_t b, ef_match* match) {
  hipLaunchKernelGGL(keys_fill_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, s, keys, b, match);
  return hipGetLastError();
}

hipError_t launch_pad_rows(hipStream_t s, const float* src, int64_t rows, int k, int64_t rows_pad, float* dst,
                           int kp) {
  const int64_t tot = rows_pad * kp;
  hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, src, rows, k,
                     rows_pad, dst, kp);
  return hipGetLastError();
}

hipError_t launch_split_rows(hipStream_t s, const float* G, int64_t n, int kp, void* out) {
  const int64_t groups = n * kp / 8;
  hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, G, groups,
                     static_cast<uint4*>(out));
  return hipGetLastError();
}

hipError_t launch_hi_rows(hipStream_t s, const float* G, int64_t n, int kp, void* out) {
  if (kp % 64 != 0) return hipErrorInvalidValue;
  const int64_t blocks = n * kp / 64;
  hipLaunchKernelGGL(hi_rows_kernel, dim3((unsigned)((blocks + 255) / 256)), dim3(256), 0, s, G, blocks,
                     static_cast<uint4*>(out));
  return hipGetLastError();
}

hipError_t launch_gallery_aux(hipStream_t s, const float* G, int64_t n, int kp, float* gnorm2, float* ginv,
                              unsigned* gmax2_bits) {
  hipError_t e = hipMemsetAsync(gmax2_bits, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gallery_aux_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, G, n, kp, gnorm2, ginv);
  hipLaunchKernelGGL(max_kernel, dim3(256), dim3(256), 0, s, gnorm2, n, gmax2_bits);
  return hipGetLastError();
}

}  // namespace ef
