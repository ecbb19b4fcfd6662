// Image side of the hot path.
//
// Ingest — train-v4.py:59-68 / scan-template-v4.py:257-263:
//     gray = cv2.cvtColor(img, COLOR_BGR2GRAY); face = cv2.resize(gray, (64, 64))
//   `resize_kernel` turns a ragged batch of decoded images (1 or 3 channels, any size)
//   into uint8 rows of any output size in one launch, with OpenCV 4.x's CV_8U arithmetic:
//   BT.601 fixed point Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14, and INTER_LINEAR as
//   resizeGeneric_ computes it for 8U (11-bit coefficients from float32 offsets, horizontal
//   int sums, vertical ((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2), plus its
//   identity copy and exact-2x INTER_AREA shortcuts.  Parity against OpenCV is unpinned
//   (OpenCV is absent here); the restatement is oracle/image_oracle.py.
//   Work per output pixel: 4 gathered source pixels (12 bytes for colour) + 1 byte out —
//   an L2/HBM-bound byte kernel, no GEMM.
//
// Template localiser — scan-template-v4.py:127-200:
//     cv2.matchTemplate(frame, resize(template, s), TM_CCOEFF_NORMED); cv2.minMaxLoc
//   for every (template, scale) problem of every model, against one grey frame.
//   The numerator is an exact integer correlation on the int8 matrix cores: with
//   I' = I - 128 and T' = T - 128 (exact int8), N = h*w,
//       N*sum(T I) - sum T * sum I  ==  N*sum(T' I') - sum T' * sum I'
//   (covariance is shift-invariant), so
//       P(y, x) = sum_{y'} sum_{x'} T'[y'][x'] I'[y+y'][x+x']
//   runs on v_mfma_i32_32x32x32_i8 and the window sums come from exact int64 integral
//   images.  Each template row y' contributes a Toeplitz product: for a 32-column block
//   of outputs starting at x0, P[y][x0+c] += sum_j I'[y+y'][x0+j] * B0[j][c] with
//   B0[j][c] = T'[y'][j-c] (0 outside [0, w)) — the frame rows are the plain A operand
//   and the banded template (precomputed once per template, "band") is the B operand.
//   Shift invariance of B0 means output block n uses B0's k-block kb-n at step kb, so a
//   wave carries four output blocks (128 columns) with ONE new B fragment per step.
//   Template rows are split in chunks of <= 128 (int32-exact: 128 * w * 2^14 < 2^31 for
//   w <= 1024) and templates wider than 352 in column pieces; the int32 partial slabs are
//   summed in int64 by `tm_score_kernel`, which applies OpenCV's TM_CCOEFF_NORMED
//   normalisation rule in float64 and reduces the first raster-order maximum with one
//   packed-key atomicMin per wave.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "ef_dma.hpp"
#include "ef_internal.hpp"
#include "ef_resize.hpp"

namespace ef {

typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

#define EF_TRY(expr)              \
  do {                            \
    int _rc = (expr);             \
    if (_rc != EF_OK) return _rc; \
  } while (0)
#define EF_HIP(ctx, expr, what)                          \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return hip_err(ctx, _e, what); \
  } while (0)

// ------------------------------------------------------------------------ ingest
struct ImgDesc {
  int64_t src_off;  // byte offset of the source image (rows of w * c bytes)
  int64_t dst_off;  // byte offset of the output image (oh rows of ow bytes)
  int h, w, c, oh, ow, pad;
};

template <bool RGB>
__device__ __forceinline__ int gray_at(const uint8_t* __restrict__ src, int w, int c, int y, int x) {
  const uint8_t* p = src + ((int64_t)y * w + x) * c;
  if (c == 1) return p[0];
  const int b = RGB ? p[2] : p[0], g = p[1], r = RGB ? p[0] : p[2];
  return (b * 1868 + g * 9617 + r * 4899 + 8192) >> 14;
}

// grid (ceil(max_out_pixels / 256), count); thread = one output pixel.
template <bool RGB>
__global__ __launch_bounds__(256) void resize_kernel(const uint8_t* __restrict__ src, const ImgDesc* __restrict__ desc,
                                                     uint8_t* __restrict__ dst) {
  const ImgDesc dd = desc[blockIdx.y];
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= dd.oh * dd.ow) return;
  const int dy = o / dd.ow, dx = o - (o / dd.ow) * dd.ow;
  const uint8_t* s = src + dd.src_off;
  const auto gray = [&](int y, int x) { return gray_at<RGB>(s, dd.w, dd.c, y, x); };
  const int v = resize_px(gray, dd.h, dd.w, dd.oh, dd.ow, dy, dx);
  dst[dd.dst_off + o] = (uint8_t)v;
}

static hipError_t launch_resize(hipStream_t s, const uint8_t* src, const ImgDesc* desc_dev, int count,
                                int64_t max_out, bool rgb, uint8_t* dst) {
  if (count == 0 || max_out == 0) return hipSuccess;
  const dim3 grid((unsigned)((max_out + 255) / 256), (unsigned)count);
  if (rgb)
    hipLaunchKernelGGL(resize_kernel<true>, grid, dim3(256), 0, s, src, desc_dev, dst);
  else
    hipLaunchKernelGGL(resize_kernel<false>, grid, dim3(256), 0, s, src, desc_dev, dst);
  return hipGetLastError();
}

// Interface used by the Haar pyramid (ef_haar.hip): grey single-channel ragged resize.
hipError_t launch_resize_gray(hipStream_t s, const uint8_t* src, const void* desc_dev, int count, int64_t max_out,
                              uint8_t* dst) {
  return launch_resize(s, src, static_cast<const ImgDesc*>(desc_dev), count, max_out, false, dst);
}
size_t img_desc_size() { return sizeof(ImgDesc); }
void img_desc_fill(void* d, int64_t src_off, int64_t dst_off, int h, int w, int c, int oh, int ow) {
  *static_cast<ImgDesc*>(d) = ImgDesc{src_off, dst_off, h, w, c, oh, ow, 0};
}

// ---------------------------------------------------------------- template localiser
constexpr int kTmChunk = 128;   // template rows per int32 partial
constexpr int kTmPiece = 352;   // template columns per piece (nkb <= 12)
constexpr int kTmTile = 128;    // output tile (rows = 4 waves x 32, cols = 4 blocks x 32)

struct TmProblem {
  int th, tw, hr, wr;
  int64_t tmpl_off;  // scaled template (uint8, th x tw) in the scaled buffer
  int64_t part_off;  // int32 offset of this problem's partial slabs [nparts][hr][wr]
  int64_t map_off;   // float offset of this problem's map (optional output)
  int nparts, pad;
};
struct TmPiece {
  int prob, px, wp, nkb;
  int64_t band_off;  // bytes: [th][nkb][64 lanes][16]
};
struct TmWork {
  int piece, part, ya, yb, y0, x0;
  int ncg;  // column groups of the output tile: 1 (128 x 128), 2 (64 x 256) or 4 (32 x 512)
};
struct TmStat {
  long long sT, varT;  // sum(T'), N*sum(T'^2) - sum(T')^2
};

// frame8 = I - 128 (int8) in a zero-padded [rows][pitch] image, and row prefix sums of I'
// and I'^2 (int64): one wave per integral-image row (row 0 is zero).
// The integral images are stored as T: int64, or wrapping uint32 when every template area n
// is < 2^18 — a window sum of I' (|.| <= 128 n < 2^31) and of I'^2 (<= 16384 n < 2^32) is
// then recovered exactly from the mod-2^32 corner differences, at half the bytes the
// score kernel's L2-bound corner gathers move.
template <typename T>
__global__ __launch_bounds__(256) void tm_rows_kernel(const uint8_t* __restrict__ f, int H, int W, int64_t ld,
                                                      int8_t* __restrict__ f8, int64_t pitch,
                                                      T* __restrict__ ii1, T* __restrict__ ii2,
                                                      unsigned long long* __restrict__ keys, int nkeys) {
  if (blockIdx.x == 0)  // reset the per-problem best keys (consumed by tm_score_kernel)
    for (int k = threadIdx.x; k < nkeys; k += 256) keys[k] = ~0ull;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row > H) return;
  const int64_t W1 = W + 1;
  T* r1 = ii1 + row * W1;
  T* r2 = ii2 + row * W1;
  if (row == 0) {
    for (int x = lane; x <= W; x += 64) r1[x] = r2[x] = 0;
    return;
  }
  const int y = row - 1;
  // 64-pixel chunks, lane = pixel (coalesced loads and stores), an inclusive wave scan per
  // chunk in int32 (|chunk sum of I'^2| <= 64 * 16384) carried into int64 row totals
  if (lane == 0) r1[0] = r2[0] = 0;
  long long c1 = 0, c2 = 0;
  for (int x0 = 0; x0 < W; x0 += 64) {
    const int x = x0 + lane;
    int e1 = 0, e2 = 0;
    if (x < W) {
      const int v = (int)f[(int64_t)y * ld + x] - 128;
      f8[(int64_t)y * pitch + x] = (int8_t)v;
      e1 = v;
      e2 = v * v;
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int t1 = __shfl_up(e1, off), t2 = __shfl_up(e2, off);
      if (lane >= off) {
        e1 += t1;
        e2 += t2;
      }
    }
    if (x < W) {
      r1[x + 1] = (T)(c1 + e1);
      r2[x + 1] = (T)(c2 + e2);
    }
    c1 += __shfl(e1, 63);
    c2 += __shfl(e2, 63);
  }
}

// Column prefix of the row sums: block = 16 columns x 64 row segments (a 641-column frame
// is 41 workgroups, not 11: the pass is latency-bound, so it wants many short segments).
constexpr int kColW = 16, kColSeg = 64;
template <typename T>
__global__ __launch_bounds__(1024) void tm_cols_kernel(int H, int W, T* __restrict__ ii1, T* __restrict__ ii2) {
  __shared__ T t1[kColSeg][kColW], t2[kColSeg][kColW];
  const int cx = threadIdx.x % kColW, sg = threadIdx.x / kColW;
  const int x = blockIdx.x * kColW + cx;
  const int64_t W1 = W + 1;
  const int per = (H + kColSeg - 1) / kColSeg;
  const int ya = 1 + sg * per, yb = ya + per < H + 1 ? ya + per : H + 1;
  T s1 = 0, s2 = 0;
  if (x <= W) {
#pragma unroll 4
    for (int y = ya; y < yb; ++y) {
      s1 += ii1[(int64_t)y * W1 + x];
      s2 += ii2[(int64_t)y * W1 + x];
    }
  }
  t1[sg][cx] = s1;
  t2[sg][cx] = s2;
  __syncthreads();
  T o1 = 0, o2 = 0;
  for (int q = 0; q < sg; ++q) {
    o1 += t1[q][cx];
    o2 += t2[q][cx];
  }
  if (x <= W) {
#pragma unroll 4
    for (int y = ya; y < yb; ++y) {
      o1 += ii1[(int64_t)y * W1 + x];
      o2 += ii2[(int64_t)y * W1 + x];
      ii1[(int64_t)y * W1 + x] = o1;
      ii2[(int64_t)y * W1 + x] = o2;
    }
  }
}

// Per problem: sum(T'), sum(T'^2) -> varT (exact int64).  One block per problem.
__global__ __launch_bounds__(256) void tm_stat_kernel(const uint8_t* __restrict__ scaled,
                                                      const TmProblem* __restrict__ probs, TmStat* __restrict__ st) {
  const TmProblem pb = probs[blockIdx.x];
  const int64_t n = (int64_t)pb.th * pb.tw;
  long long s1 = 0, s2 = 0;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const long long v = (long long)scaled[pb.tmpl_off + i] - 128;
    s1 += v;
    s2 += v * v;
  }
  __shared__ long long r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    st[blockIdx.x].sT = r1[0];
    st[blockIdx.x].varT = n * r2[0] - r1[0] * r1[0];
  }
}

// band[y'][kb][lane][j] = T'[y'][px + 32 kb + 16 (lane >> 5) + j - (lane & 31)] inside the
// piece's columns [0, wp), else 0 — the B-operand fragment (lane (c, h) holds
// B[16h + j][c]) of k-block kb.  grid (th, npieces), block 64 x nkb <= 1024 threads.
__global__ void tm_band_kernel(const uint8_t* __restrict__ scaled, const TmProblem* __restrict__ probs,
                               const TmPiece* __restrict__ pieces, uint8_t* __restrict__ bands) {
  const TmPiece pc = pieces[blockIdx.y];
  const TmProblem pb = probs[pc.prob];
  const int yy = blockIdx.x;
  if (yy >= pb.th) return;
  for (int t = threadIdx.x; t < 64 * pc.nkb; t += blockDim.x) {
    const int kb = t >> 6, lane = t & 63;
    const int c = lane & 31, hh = lane >> 5;
    union {
      int8_t b[16];
      i32x4 v;
    } u;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int q = 32 * kb + 16 * hh + j - c;  // template column inside the piece
      u.b[j] = (q >= 0 && q < pc.wp) ? (int8_t)((int)scaled[pb.tmpl_off + (int64_t)yy * pb.tw + pc.px + q] - 128)
                                     : (int8_t)0;
    }
    *reinterpret_cast<i32x4*>(bands + pc.band_off + ((int64_t)yy * pc.nkb + kb) * 1024 + lane * 16) = u.v;
  }
}

// One workgroup = one work item: an output tile of one problem (128 x 128, or 64 x 256 /
// 32 x 512 — below), template rows [ya, ya + J) of one column piece.  8 waves (2 per SIMD):
// wave w owns 32 output rows x the four 32-column blocks of one 128-column group (for the
// 128 x 128 tile: rows y0 + 32 (w & 3) + [0, 32), all 128 columns), and the template rows of
// parity w >> 2 — the two waves of a SIMD split the template rows and add their partial
// sums at the end.  Per template row a wave reads NKB + 3 A and NKB B fragments for
// 4 NKB MFMAs (the band's shift invariance: block n uses k-block kb - n).
// Operands live in LDS, filled by LDS-DMA one row PAIR per barrier, two pairs ahead:
//   * A ring: frame rows y0 + ya + q (q = 0 .. J + WROWS - 2) in slot q mod ring, each row
//     the 32 (nkb + 3) + 128 (ncg - 1) bytes the tile reads, slot stride SA = 16 (mod 256)
//     bytes, so the 16 rows a ds_read_b128 lane group touches fall in distinct banks; ring
//     = the slots of that stride the LDS region holds.  Pair p reads rows 2p .. 2p + WROWS
//     and prefetches rows 2p + WROWS + 3, 2p + WROWS + 4 (WROWS = the tile's output rows).
//   * B ring: the band slices of template rows 2p, 2p + 1 (nkb KiB each, lane-linear
//     fragments) in stage p % 3.
// Tile shapes (TmWork::ncg): 128 x 128, and for a map's last row band with one or two live
// 32-row blocks 32 x 512 or 64 x 256 — wave pair wr4 then owns column group wr4 & (ncg - 1)
// of row block wr4 / ncg, so no SIMD idles on dead rows (0.397 -> 0.383 ms per bench frame,
// profiles/r05/tm_tile_shape_ab.txt; three live row blocks as a 64 x 256 band plus a 32 x 512
// one measured no faster, profiles/r06/tm_split3_ab.txt).  In a map's last column tile each
// wave runs only its live 32-column blocks (NCB, a compile-time count per wave; 0.383 ->
// 0.368 ms per bench frame, profiles/r06/tm_live_cols_ab.txt).
// One barrier per template-row pair (half the barriers, and half the LDS fragment reads
// per MFMA, of a one-row-per-barrier, two-blocks-per-wave tiling).  The wide kernel
// (MAXNKB 12, one workgroup per CU) software-pipelines the pairs: the last 8 MFMAs of pair
// p run after the barrier, interleaved with the reads of pair p + 1's fragments, so the
// LDS round trip after a barrier is hidden under MFMAs (bench frame 0.418 -> 0.397 ms,
// profiles/r05/tm_pipeline_ab.txt); the narrow kernel (2 workgroups per CU) overlaps one
// workgroup's barrier with the other's MFMAs instead.
#ifndef EF_TM_PIPE  // software-pipelined pairs in the wide kernel (variant builds: 0 = off, A/B)
#define EF_TM_PIPE 1
#endif
constexpr int kTmRing = 144;  // A-ring slots (>= 133; 144 * 16 = 0 mod 256 keeps banks aligned)
constexpr int tm_max_sa(int maxnkb) { return (32 * (maxnkb + 3) + 255) / 256 * 256 + 16; }
constexpr int tm_lds_bytes(int maxnkb) { return kTmRing * tm_max_sa(maxnkb) + 3 * 2 * maxnkb * 1024 + 1024; }

// The wide kernel's software pipelining (tm_corr_kernel): which fragments the last T MFMAs
// of a template row use (kb-major sequence, block n on k-block kb - n), the order of the
// other fragments' reads (ea / eb, -1 = a tail fragment; ne of them), and the (kb, n) of
// each tail MFMA.
struct TmTail {
  bool a[16], b[16];
  int ea[16], eb[16], ne;
  int tk[32], tn[32];
};
// A wave with ncb live 32-column blocks (the map's last column tile: its columns past wr
// are dead) runs only blocks n < ncb — ncb·nkb MFMAs on A k-blocks 0 .. nkb + ncb - 2.
constexpr TmTail tm_tail(int nkb, int ncb, int t) {
  TmTail s{};
  int m = 0;
  for (int kb = 0; kb < nkb + ncb - 1; ++kb)
    for (int n = 0; n < ncb; ++n)
      if (kb - n >= 0 && kb - n < nkb) {
        if (m >= ncb * nkb - t) {
          s.a[kb] = s.b[kb - n] = true;
          s.tk[m - (ncb * nkb - t)] = kb;
          s.tn[m - (ncb * nkb - t)] = n;
        }
        ++m;
      }
  for (int kb = 0; kb < nkb + ncb - 1; ++kb) {  // consumption order: A[kb], then B[kb]
    s.ea[kb] = s.a[kb] ? -1 : s.ne++;
    s.eb[kb] = kb < nkb && !s.b[kb] ? s.ne++ : -1;
  }
  for (int kb = nkb + ncb - 1; kb < 16; ++kb) s.ea[kb] = s.eb[kb] = -1;  // A k-blocks no live block reads
  return s;
}

// position of MFMA (kb, n) in a template row's kb-major sequence
constexpr int tm_mfma_index(int nkb, int ncb, int kb, int n) {
  int m = 0;
  for (int k = 0; k < nkb + ncb - 1; ++k)
    for (int q = 0; q < ncb; ++q)
      if (k - q >= 0 && k - q < nkb) {
        if (k == kb && q == n) return m;
        ++m;
      }
  return m;
}
template <int NKB, int NCB, int T>
struct TmTailOf {
  static constexpr TmTail v = tm_tail(NKB, NCB, T);
};
// f(integral_constant<int, I>) for I = 0 .. N-1, unrolled by construction (no reliance on
// the loop unroller: a table lookup left in a rolled loop lands in scratch memory)
template <typename F, int... I>
__device__ __forceinline__ void tm_static_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

// MAXNKB: the largest k-block count of the launch's pieces (12 for 352-column pieces; the
// diagnostic build's EF_TM_PIECE = 96 runs MAXNKB = 5, whose 71 KiB of LDS let two
// workgroups share a CU).
template <int MAXNKB>
__global__ __launch_bounds__(512, MAXNKB <= 5 ? 2 : 1) void tm_corr_kernel(const int8_t* __restrict__ f8,
                                                                          int64_t pitch,
                                                                          const uint8_t* __restrict__ bands,
                                                                          const TmPiece* __restrict__ pieces,
                                                                          const TmWork* __restrict__ works,
                                                                          const TmProblem* __restrict__ probs,
                                                                          int* __restrict__ parts, int nwork) {
  constexpr int kTmMaxSA = tm_max_sa(MAXNKB), kTmMaxNkb = MAXNKB, kTmBStage = 2 * MAXNKB * 1024;
  static_assert(tm_lds_bytes(MAXNKB) >= 4 * 4 * 16 * 64 * 4, "the final reduction reuses the ring");
  __shared__ __attribute__((aligned(16))) uint8_t smem[tm_lds_bytes(MAXNKB)];
  const TmWork wk = works[blockIdx.x];
  const TmPiece pc = pieces[wk.piece];
  const TmProblem pb = probs[pc.prob];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr4 = wave & 3, par = wave >> 2;  // wave pair (SIMD), template-row parity
  const int r = lane & 31, h = lane >> 5;
  const int nkb = pc.nkb;
  // tile shape: wave pair wr4 owns 32-row block rb and 128-column group cg
  const int lc = wk.ncg == 4 ? 2 : wk.ncg == 2 ? 1 : 0;
  const int rb = wr4 >> lc, cg = wr4 & (wk.ncg - 1);
  const int WROWS = 32 * (4 >> lc);  // output rows of the tile
  const int RW = 32 * (nkb + 3) + 128 * (wk.ncg - 1);  // A-row bytes a tile reads
  const int SA = (RW + 255) / 256 * 256 + 16;  // slot stride = 16 (mod 256)
  const int nl = RW / 16;          // DMA lanes per A row (<= 54)
  const int ring = kTmRing * kTmMaxSA / SA;  // A-ring slots (host: >= WROWS + 6)
  // q mod ring for q < 4 ring (tm_tile_groups: 4 ring > J + WROWS + 6 > every slot index)
  auto wrap = [&](int q) {
    q -= q >= ring ? ring : 0;
    q -= q >= ring ? ring : 0;
    q -= q >= ring ? ring : 0;
    return q;
  };
  const int J = wk.yb - wk.ya;
  const int NP = (J + 1) / 2;      // template-row pairs
  const unsigned lds = lds_addr(smem);
  const unsigned ldsB = lds + (unsigned)(kTmRing * kTmMaxSA);
  const unsigned ldsD = ldsB + (unsigned)(3 * kTmBStage);  // dummy DMA target
  const int8_t* arow0 = f8 + (int64_t)(wk.y0 + wk.ya) * pitch + wk.x0 + pc.px + 16 * lane;  // + q * pitch
  const uint8_t* bsl0 = bands + pc.band_off + (int64_t)wk.ya * nkb * 1024 + 16 * lane;     // + j * nkb KiB
  // Row blocks past hr and column groups past wr are skipped per wave (uniform); NKB is a
  // compile-time constant so the k-block loop unrolls and the fragment reads are static.
  const bool wact = wk.y0 + 32 * rb < pb.hr && wk.x0 + 128 * cg < pb.wr;
  i32x16 acc[4] = {};
  auto run = [&](auto nkb_c, auto ncb_c) {
    constexpr int NKB = decltype(nkb_c)::value;
    constexpr int NCB = decltype(ncb_c)::value;  // live 32-column blocks of this wave (1..4)
    constexpr int NKA = NKB + NCB - 1;           // A k-blocks those blocks read
    constexpr int NPC = 2 * NKB + 2;       // DMA pieces per pair: 2 NKB band slices + 2 A rows
    constexpr int Q = (NPC + 7) / 8;       // DMA instructions per wave per pair
    // Pair p's operands: band slices of rows 2p, 2p+1 into stage p % 3 and A rows
    // q = 2p + WROWS - 1, 2p + WROWS (completing the windows of rows 2p, 2p + 1); wave w issues
    // pieces w, w + 8, ..., padded with harmless dummy DMAs to exactly Q instructions, so
    // "pair p landed" is a vmcnt of Q x (pairs issued after it).
    auto issue_piece = [&](int p, int i) {
      const int pi = wave + 8 * i;
      if (pi < 2 * NKB) {
        const int rr = pi / NKB, kb = pi - (pi / NKB) * NKB, j = 2 * p + rr;
        if (j < J)
          glds16(bsl0 + ((int64_t)j * NKB + kb) * 1024,
                 ldsB + (unsigned)((p % 3) * kTmBStage + (rr * kTmMaxNkb + kb) * 1024));
        else
          glds16(bsl0, ldsD);
      } else if (pi < NPC) {
        const int q = 2 * p + WROWS - 1 + (pi - 2 * NKB);
        if (q < J + WROWS - 1) {
          if (lane < nl) glds16(arow0 + (int64_t)q * pitch, lds + (unsigned)(wrap(q) * SA));
        } else {
          glds16(bsl0, ldsD);
        }
      } else {
        glds16(bsl0, ldsD);
      }
    };
    auto issue = [&](int p) {
#pragma unroll
      for (int i = 0; i < Q; ++i) issue_piece(p, i);
    };
    for (int q = wave; q < WROWS - 1; q += 8)
      if (lane < nl) glds16(arow0 + (int64_t)q * pitch, lds + (unsigned)(q * SA));
    issue(0);
    if (NP > 1) {
      issue(1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(Q) : "memory");
    } else {
      dma_wait_all();
    }
    __syncthreads();
#ifdef EF_TM_STAMP
    unsigned long long ph[5] = {0, 0, 0, 0, 0};
    unsigned long long tq = __builtin_amdgcn_s_memtime();
#define EF_STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ph[i] += t_ - tq; tq = t_; } while (0)
#else
#define EF_STAMP(i) do {} while (0)
#endif
    if constexpr (EF_TM_PIPE && MAXNKB > 5) {  // (the 2-workgroup narrow kernel overlaps by occupancy)
    // Software-pipelined pairs: the barrier of pair p sits before its last T MFMAs, and
    // the fragments of pair p + 1 that those MFMAs do not use are read right after it, so
    // their LDS round trip runs under the tail instead of the pipe idling between the
    // barrier and the next pair's first MFMA; the tail's own fragments (the highest A and B
    // k-blocks, needed last by the next pair) are re-read after it.  One register set.
    // Stage p % 3 is rewritten by pair p + 3's DMA, issued during pair p + 1 — after this
    // barrier, by which every wave has completed its reads of stage p (lgkmcnt(0) below).
    constexpr int NM = NCB * NKB;                           // MFMAs per template row
#ifndef EF_TM_TAIL  // (variant builds: A/B of the tail length)
#define EF_TM_TAIL 8
#endif
    // MFMAs after the barrier (at least one: the tail is where pair p + 1's reads go)
    constexpr int T = NM / 2 < 1 ? 1 : NM / 2 < EF_TM_TAIL ? NM / 2 : EF_TM_TAIL;
    static_assert(T <= 32, "TmTail holds 32 tail MFMAs");
    using Tail = TmTailOf<NKB, NCB, T>;
    i32x4 A[NKA], B[NKB];
    // fragment reads of pair p: the tail's (LATE) or the others, in consumption order
    auto frag_read = [&](int p, auto late_c) {
      constexpr bool LATE = decltype(late_c)::value;
      const int j = 2 * p + par;
      const uint8_t* aslot = smem + wrap(j + 32 * rb + r) * SA + 16 * h + 128 * cg;
      const uint8_t* bst = smem + kTmRing * kTmMaxSA + (p % 3) * kTmBStage + par * kTmMaxNkb * 1024 + 16 * lane;
      tm_static_for(
          [&](auto kc) {
            constexpr int kb = decltype(kc)::value;
            if constexpr (Tail::v.a[kb] == LATE) A[kb] = *reinterpret_cast<const i32x4*>(aslot + 32 * kb);
            if constexpr (kb < NKB && Tail::v.b[kb] == LATE) B[kb] = *reinterpret_cast<const i32x4*>(bst + kb * 1024);
          },
          std::make_integer_sequence<int, NKA>{});
    };
    // MFMAs [LO, HI) of a row's sequence (kb-major; block n uses k-block kb - n).  With
    // dma, pair p + 2's pieces go between the first NM - T at evenly spaced positions.
    auto mfmas = [&](auto lo_c, auto hi_c, bool dma, int p) {
      constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
      if constexpr (LO == 0)  // pieces placed before the first MFMA (short rows: NM - T < Q + 1)
        tm_static_for(
            [&](auto ic) {
              constexpr int i = decltype(ic)::value;
              if constexpr ((i + 1) * (NM - T) / (Q + 1) == 0)
                if (dma) issue_piece(p + 2, i);
            },
            std::make_integer_sequence<int, Q>{});
      tm_static_for(
          [&](auto kc) {
            constexpr int kb = decltype(kc)::value;
            tm_static_for(
                [&](auto nc) {
                  constexpr int n = decltype(nc)::value, m = tm_mfma_index(NKB, NCB, kb, n);
                  if constexpr (kb - n >= 0 && kb - n < NKB && m >= LO && m < HI) {
                    acc[n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[kb], B[kb - n], acc[n], 0, 0, 0);
                    tm_static_for(
                        [&](auto ic) {
                          constexpr int i = decltype(ic)::value;
                          if constexpr (m + 1 == (i + 1) * (NM - T) / (Q + 1)) {
                            __builtin_amdgcn_sched_barrier(0);
                            if (dma) issue_piece(p + 2, i);
                            __builtin_amdgcn_sched_barrier(0);
                          }
                        },
                        std::make_integer_sequence<int, Q>{});
                  }
                },
                std::make_integer_sequence<int, NCB>{});
          },
          std::make_integer_sequence<int, NKA>{});
    };
    if (wact && par < J) {
      frag_read(0, std::false_type{});
      frag_read(0, std::true_type{});
    }
    for (int p = 0; p < NP; ++p) {
      const bool ahead = p + 2 < NP;
      const int j = 2 * p + par;
      const bool act = wact && j < J;
      if (act)
        mfmas(std::integral_constant<int, 0>{}, std::integral_constant<int, NM - T>{}, ahead, p);
      else if (ahead)
        issue(p + 2);
      __builtin_amdgcn_sched_barrier(0);  // (MFMAs are not memory ops: keep them on their side)
      EF_STAMP(1);
      if (ahead)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(Q) : "memory");  // pair p + 1 landed
      else
        dma_wait_all();
      EF_STAMP(2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();  // pair p + 1 visible to every wave; stage p read by every wave
      __builtin_amdgcn_sched_barrier(0);
      EF_STAMP(3);
      if (act) {
        // pair p + 1's non-tail fragments spread evenly between this pair's tail MFMAs (a
        // wave whose rows end here reads harmless stale slots it never uses)
        const int j1 = j + 2;
        const uint8_t* aslot = smem + wrap(j1 + 32 * rb + r) * SA + 16 * h + 128 * cg;
        const uint8_t* bst =
            smem + kTmRing * kTmMaxSA + ((p + 1) % 3) * kTmBStage + par * kTmMaxNkb * 1024 + 16 * lane;
        tm_static_for(
            [&](auto tc) {
              constexpr int t = decltype(tc)::value;
              tm_static_for(
                  [&](auto kc) {
                    constexpr int kb = decltype(kc)::value;
                    if constexpr (Tail::v.ea[kb] >= 0 && Tail::v.ea[kb] * T / Tail::v.ne == t)
                      A[kb] = *reinterpret_cast<const i32x4*>(aslot + 32 * kb);
                    if constexpr (kb < NKB && Tail::v.eb[kb] >= 0 && Tail::v.eb[kb] * T / Tail::v.ne == t)
                      B[kb] = *reinterpret_cast<const i32x4*>(bst + kb * 1024);
                  },
                  std::make_integer_sequence<int, NKA>{});
              __builtin_amdgcn_sched_barrier(0);
              constexpr int tk = Tail::v.tk[t], tn = Tail::v.tn[t];
              acc[tn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[tk], B[tk - tn], acc[tn], 0, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            },
            std::make_integer_sequence<int, T>{});
        frag_read(p + 1, std::true_type{});  // the tail's own fragments, needed last by pair p + 1
      }
      EF_STAMP(0);  // "issue" = the next pair's reads + this pair's tail MFMAs
    }
    } else {
    for (int p = 0; p < NP; ++p) {
      const bool ahead = p + 2 < NP;
      const int j = 2 * p + par;
      EF_STAMP(0);
      if (wact && j < J) {
        const uint8_t* aslot = smem + wrap(j + 32 * rb + r) * SA + 16 * h + 128 * cg;
        const uint8_t* bst = smem + kTmRing * kTmMaxSA + (p % 3) * kTmBStage + par * kTmMaxNkb * 1024 + 16 * lane;
        i32x4 A[NKA], B[NKB];
#pragma unroll
        for (int kb = 0; kb < NKA; ++kb) {  // in the order the MFMAs consume them
          A[kb] = *reinterpret_cast<const i32x4*>(aslot + 32 * kb);
          if (kb < NKB) B[kb] = *reinterpret_cast<const i32x4*>(bst + kb * 1024);
        }
        // pair p+2's DMA pieces are issued between the MFMAs (evenly spaced), not as a burst
        // after the barrier: a burst of 32 LDS-DMA instructions per CU kept every wave in
        // its issue phase (~800 cycles per pair) with the MFMA pipe idle
        int m = 0;
#pragma unroll
        for (int i = 0; i < Q; ++i)  // pieces placed before the first MFMA (short rows)
          if ((i + 1) * (NCB * NKB) / (Q + 1) == 0 && ahead) issue_piece(p + 2, i);
#pragma unroll
        for (int kb = 0; kb < NKA; ++kb)
#pragma unroll
          for (int n = 0; n < NCB; ++n)
            if (kb - n >= 0 && kb - n < NKB) {
              acc[n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[kb], B[kb - n], acc[n], 0, 0, 0);
              ++m;
#pragma unroll
              for (int i = 0; i < Q; ++i)
                if (m == (i + 1) * (NCB * NKB) / (Q + 1)) {
                  __builtin_amdgcn_sched_barrier(0);
                  if (ahead) issue_piece(p + 2, i);
                  __builtin_amdgcn_sched_barrier(0);
                }
            }
      } else if (ahead) {
        issue(p + 2);
      }
      EF_STAMP(1);
      if (ahead)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(Q) : "memory");  // pair p + 1 landed
      else
        dma_wait_all();
      EF_STAMP(2);
      __syncthreads();  // ... for every wave; everyone is done with stage p % 3 and its slots
      EF_STAMP(3);
    }
    }
#ifdef EF_TM_STAMP
    if (blockIdx.x % 97 == 0 && lane == 0 && (wave == 0 || wave == 4))
      printf("tmstamp blk %d wave %d nkb %d pairs %d issue %llu mfma %llu vmwait %llu barrier %llu\n", (int)blockIdx.x,
             wave, NKB, NP, ph[0], ph[1], ph[2], ph[3]);
#endif
#undef EF_STAMP
  };
  // live column blocks of this wave's column group: a map's last column tile runs only
  // those (waves with none are inactive and run the 4-block loop for its DMA and barriers)
  const int ncb = __builtin_amdgcn_readfirstlane(wact ? min(4, (pb.wr - wk.x0 - 128 * cg + 31) / 32) : 4);
  auto run_nkb = [&](auto nkb_c) {
    switch (ncb) {
      case 1: run(nkb_c, std::integral_constant<int, 1>{}); break;
      case 2: run(nkb_c, std::integral_constant<int, 2>{}); break;
      case 3: run(nkb_c, std::integral_constant<int, 3>{}); break;
      default: run(nkb_c, std::integral_constant<int, 4>{}); break;
    }
  };
  switch (nkb) {
#define EF_TM_NKB(V)                                     \
  case V:                                                \
    if constexpr (V <= MAXNKB) run_nkb(std::integral_constant<int, V>{}); \
    break;
    EF_TM_NKB(1) EF_TM_NKB(2) EF_TM_NKB(3) EF_TM_NKB(4) EF_TM_NKB(5) EF_TM_NKB(6)
    EF_TM_NKB(7) EF_TM_NKB(8) EF_TM_NKB(9) EF_TM_NKB(10) EF_TM_NKB(11) EF_TM_NKB(12)
#undef EF_TM_NKB
    default:
      break;
  }
  // the odd-row waves hand their partial sums to the even-row waves through LDS (the ring
  // is free: the loop ended with a barrier after every DMA landed)
  int* red = reinterpret_cast<int*>(smem) + (wr4 * 4 * 16 * 64);
  if (par == 1 && wact) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int g = 0; g < 16; ++g) red[(n * 16 + g) * 64 + lane] = acc[n][g];
  }
  __syncthreads();
  if (par == 1 || !wact) return;
  int* out = parts + pb.part_off + (int64_t)wk.part * pb.hr * pb.wr;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int x = wk.x0 + 128 * cg + 32 * n + r;
    if (x >= pb.wr) continue;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int y = wk.y0 + 32 * rb + (g & 3) + 8 * (g >> 2) + 4 * h;
      if (y < pb.hr) out[(int64_t)y * pb.wr + x] = acc[n][g] + red[(n * 16 + g) * 64 + lane];
    }
  }
}

// OpenCV's TM_CCOEFF_NORMED rule (templmatch.cpp common_matchTemplate) on exact integers.
// sqT = sqrt((double)varT), hoisted per problem (the same correctly rounded value).
__device__ __forceinline__ float tm_score(long long numN, long long varI, long long varT, double sqT) {
  if (varT == 0) return 1.f;  // flat template: all ones
  const double t = __dmul_rn(sqrt((double)varI), sqT);
  const double num = (double)numN;
  const double an = fabs(num);
  double rr;
  if (an < t)
    rr = __ddiv_rn(num, t);
  else if (an < __dmul_rn(t, 1.125))
    rr = num > 0 ? 1.0 : (num < 0 ? -1.0 : 0.0);
  else
    rr = 0.0;
  return __double2float_rn(rr);
}

// Max-first, then lowest raster index: min over ~orderable(score) << 32 | index.
__device__ __forceinline__ unsigned long long tm_key(float v, unsigned idx) {
  const unsigned b = __float_as_uint(v == 0.f ? 0.f : v);
  const unsigned o = (b & 0x80000000u) ? ~b : (b | 0x80000000u);  // ascending order
  return ((unsigned long long)(~o) << 32) | idx;
}

// grid (blocks per problem, nprob): score every position (grid-stride), optional map,
// then one packed-key atomicMin per block for the first raster-order maximum.
template <typename T>
__global__ __launch_bounds__(256) void tm_score_kernel(const TmProblem* __restrict__ probs,
                                                       const TmStat* __restrict__ st, const int* __restrict__ parts,
                                                       const T* __restrict__ ii1, const T* __restrict__ ii2, int W,
                                                       float* __restrict__ maps,
                                                       unsigned long long* __restrict__ keys) {
  const TmProblem pb = probs[blockIdx.y];
  const TmStat ts = st[blockIdx.y];
  const double sqT = sqrt((double)ts.varT);
  const int64_t npos = (int64_t)pb.hr * pb.wr;
  const long long n = (long long)pb.th * pb.tw;
  const int64_t W1 = W + 1;
  unsigned long long key = ~0ull;
  // rows are strided over the blocks of this problem, columns over the threads (no 64-bit
  // index division per position)
  // two positions (x, x + 256) per thread per pass: both positions' loads are in flight
  // before either's fp64 normalisation (the kernel is load-latency bound)
  for (int y = blockIdx.x; y < pb.hr; y += gridDim.x) {
    const int64_t a0 = (int64_t)y * W1, b0 = (int64_t)(y + pb.th) * W1;
    const int64_t row = (int64_t)y * pb.wr;
    for (int x = threadIdx.x; x < pb.wr; x += 512) {
      const bool two = x + 256 < pb.wr;
      long long P[2] = {0, 0}, sI[2], sI2[2];
      const int* pp = parts + pb.part_off + row + x;
      for (int q = 0; q < pb.nparts; ++q) {
        P[0] += pp[(int64_t)q * npos];
        if (two) P[1] += pp[(int64_t)q * npos + 256];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t a = a0 + x + 256 * u, b = b0 + x + 256 * u;
        T d1 = 0, d2 = 0;
        if (u == 0 || two) {
          if constexpr (std::is_same<T, unsigned>::value) {
            // 32-bit byte offsets from the uniform base (the images hold < 2^30 entries):
            // base + zext(offset) addressing instead of 64-bit address arithmetic per load
            auto ld = [](const unsigned* p, int64_t e) {
              return *reinterpret_cast<const unsigned*>(reinterpret_cast<const char*>(p) + (uint32_t)e * 4u);
            };
            d1 = ld(ii1, b + pb.tw) - ld(ii1, a + pb.tw) - ld(ii1, b) + ld(ii1, a);
            d2 = ld(ii2, b + pb.tw) - ld(ii2, a + pb.tw) - ld(ii2, b) + ld(ii2, a);
          } else {
            d1 = ii1[b + pb.tw] - ii1[a + pb.tw] - ii1[b] + ii1[a];
            d2 = ii2[b + pb.tw] - ii2[a + pb.tw] - ii2[b] + ii2[a];
          }
        }
        // uint32: d1 is the two's-complement window sum, d2 the (non-negative) one
        sI[u] = std::is_same<T, long long>::value ? (long long)d1 : (long long)(int)d1;
        sI2[u] = (long long)d2;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
        const int64_t i = row + x + 256 * u;
        long long numN, varI;
        if constexpr (std::is_same<T, unsigned>::value) {
          // every template area < 2^18: |sI|, |sT| <= 128 n < 2^25 and sI2 <= 16384 n < 2^32,
          // so the window terms are 32 x 32 -> 64-bit products (n * P keeps a 64-bit P)
          const int n32 = (int)n, sI32 = (int)sI[u], sT32 = (int)ts.sT;
          numN = (long long)n32 * P[u] - (long long)sT32 * sI32;
          varI = (long long)((unsigned long long)(unsigned)n32 * (unsigned)sI2[u]) - (long long)sI32 * sI32;
        } else {
          numN = n * P[u] - ts.sT * sI[u];
          varI = n * sI2[u] - sI[u] * sI[u];
        }
        const float v = tm_score(numN, varI, ts.varT, sqT);
        if (maps) maps[pb.map_off + i] = v;
        const unsigned long long k = tm_key(v, (unsigned)i);
        key = k < key ? k : key;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(key, off);
    key = o < key ? o : key;
  }
  __shared__ unsigned long long red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = key;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = red[0];
    for (int w = 1; w < 4; ++w) m = red[w] < m ? red[w] : m;
    if (m != ~0ull) atomicMin(keys + blockIdx.y, m);
  }
}


// ------------------------------------------------------------------ ctx state
struct TmState {
  int H = 0, W = 0, nprob = 0, nwork = 0, max_nkb = 0;
  bool ii64 = false;  // int64 integral images (some template area >= 2^18, or EF_TM_II64)
  int64_t pitch = 0, max_pos = 0, map_total = 0;
  std::vector<TmProblem> probs;
  DevBuf raw, scaled, bands, d_probs, d_pieces, d_works, d_stat, parts, f8, ii1, ii2, keys, frame_stage, maps;
};

void tm_release(ef_ctx* c) {
  if (!c || !c->tm) return;
  TmState* t = static_cast<TmState*>(c->tm);
  DevBuf* bufs[] = {&t->raw,   &t->scaled, &t->bands, &t->d_probs, &t->d_pieces, &t->d_works, &t->d_stat,
                    &t->parts, &t->f8,     &t->ii1,   &t->ii2,     &t->keys,     &t->frame_stage, &t->maps};
  for (DevBuf* b : bufs) release(*b);
  delete t;
  c->tm = nullptr;
}

static int64_t rup(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// Column groups of a tile whose row band has nrb live 32-row blocks: 4 (32 x 512) for one,
// 2 (64 x 256) for two, when the kernel's A ring holds that shape's window (WROWS + 6
// slots at its wider slot stride; tm_corr_kernel), else 1 (128 x 128).
static int tm_tile_groups(int nrb, int nkb, int maxnkb) {
  for (int g = nrb == 1 ? 4 : nrb == 2 ? 2 : 1; g > 1; g >>= 1) {
    const int rw = 32 * (nkb + 3) + 128 * (g - 1);
    const int sa = (rw + 255) / 256 * 256 + 16;
    const int ring = kTmRing * tm_max_sa(maxnkb) / sa;
    // window + prefetch, and the kernel's wrap() (three conditional subtracts) covers every
    // slot index (< 128 template rows + the tile's rows + 6)
    if (ring >= 32 * (4 / g) + 6 && 4 * ring > 128 + 32 * (4 / g) + 6 && rw <= 1024) return g;
  }
  return 1;
}

}  // namespace ef

using namespace ef;

extern "C" {

int ef_preprocess(ef_ctx* c, const uint8_t* data, const int64_t* offsets, const int32_t* heights,
                  const int32_t* widths, const int32_t* channels, int64_t count, int32_t out_h, int32_t out_w,
                  uint8_t* out, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if (count < 0 || out_h <= 0 || out_w <= 0 || (count > 0 && (!data || !offsets || !heights || !widths || !out)))
    return set_err(c, EF_E_INVALID, "ef_preprocess: bad arguments");
  if (count == 0) return EF_OK;
  if (count > 65535) return set_err(c, EF_E_INVALID, "ef_preprocess: at most 65535 images per call");
  EF_HIP(c, hipSetDevice(c->device), "hipSetDevice");
  const bool dev = flags & EF_MEM_DEVICE;
  std::vector<ImgDesc> desc((size_t)count);
  int64_t src_bytes = 0;
  for (int64_t i = 0; i < count; ++i) {
    const int ch = channels ? channels[i] : 1;
    if (heights[i] <= 0 || widths[i] <= 0 || (ch != 1 && ch != 3 && ch != 4) || offsets[i] < 0)
      return set_err(c, EF_E_INVALID, "ef_preprocess: image " + std::to_string(i) + " has a bad shape");
    desc[i] = ImgDesc{offsets[i], i * (int64_t)out_h * out_w, heights[i], widths[i], ch, out_h, out_w, 0};
    const int64_t end = offsets[i] + (int64_t)heights[i] * widths[i] * ch;
    src_bytes = end > src_bytes ? end : src_bytes;
  }
  // metadata + (host) pixels staged in one scratch buffer
  const size_t dbytes = rup((int64_t)desc.size() * sizeof(ImgDesc), 256);
  const size_t obytes = (size_t)count * out_h * out_w;
  const size_t need = dbytes + (dev ? 0 : rup(src_bytes, 256) + rup(obytes, 256));
  EF_TRY(ensure(c, c->p_stage, need));
  char* base = static_cast<char*>(c->p_stage.p);
  ImgDesc* ddesc = reinterpret_cast<ImgDesc*>(base);
  const uint8_t* src = data;
  uint8_t* dst = out;
  EF_HIP(c, hipMemcpyAsync(ddesc, desc.data(), desc.size() * sizeof(ImgDesc), hipMemcpyHostToDevice, c->stream),
         "H2D descriptors");
  if (!dev) {
    uint8_t* s = reinterpret_cast<uint8_t*>(base + dbytes);
    EF_HIP(c, hipMemcpyAsync(s, data, src_bytes, hipMemcpyHostToDevice, c->stream), "H2D images");
    src = s;
    dst = reinterpret_cast<uint8_t*>(base + dbytes + rup(src_bytes, 256));
  }
  TimerEvt tev;
  timer_begin(c, EF_KERNEL_INGEST, &tev);
  EF_HIP(c, launch_resize(c->stream, src, ddesc, (int)count, (int64_t)out_h * out_w, flags & EF_IMG_RGB, dst),
         "resize kernel");
  timer_end(c, &tev);
  if (!dev) {
    EF_HIP(c, hipMemcpyAsync(out, dst, obytes, hipMemcpyDeviceToHost, c->stream), "D2H faces");
  }
  // descriptors live in scratch that the next call may overwrite: always wait
  EF_HIP(c, hipStreamSynchronize(c->stream), "sync");
  return EF_OK;
}

// Width of the integral images (host-only, API v7).  uint32 (wrapping) sums need every
// template area < 2^18 (window sums of I'^2 <= 16384 * area < 2^32) AND fewer than 2^30
// integral entries, (H + 1)(W + 1): tm_score_kernel<unsigned> forms byte offsets as
// uint32(entry) * 4 (a 32k x 32k frame wrapped them).  Otherwise int64.
int ef_tm_sums_bits(int32_t frame_h, int32_t frame_w, int64_t max_template_area) {
  if (frame_h <= 0 || frame_w <= 0 || max_template_area < 0) return EF_E_INVALID;
  if (max_template_area >= (int64_t)1 << 18) return 64;
  if ((int64_t)(frame_h + 1) * (int64_t)(frame_w + 1) >= (int64_t)1 << 30) return 64;
  return 32;
}

int ef_tm_prepare(ef_ctx* c, const uint8_t* templ_data, const int64_t* templ_offsets, const int32_t* templ_h,
                  const int32_t* templ_w, int32_t n_templates, const int32_t* prob_templ, const int32_t* prob_h,
                  const int32_t* prob_w, int32_t n_problems, int32_t frame_h, int32_t frame_w, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if (n_templates < 0 || n_problems < 0 || frame_h <= 0 || frame_w <= 0 ||
      (n_templates > 0 && (!templ_data || !templ_offsets || !templ_h || !templ_w)) ||
      (n_problems > 0 && (!prob_templ || !prob_h || !prob_w)))
    return set_err(c, EF_E_INVALID, "ef_tm_prepare: bad arguments");
  if (n_problems > 65535) return set_err(c, EF_E_INVALID, "ef_tm_prepare: at most 65535 problems");
  EF_HIP(c, hipSetDevice(c->device), "hipSetDevice");
  tm_release(c);
  TmState* t = new TmState();
  c->tm = t;
  t->H = frame_h;
  t->W = frame_w;
  t->nprob = n_problems;
  t->pitch = rup((int64_t)frame_w + 640, 64);  // a 512-column tile's rows read past the frame
  t->ii64 = c->opt_tm_int64 != 0;
  if (ef_tm_sums_bits(frame_h, frame_w, 1) == 64) t->ii64 = true;  // frame-size rule alone
  const bool dev = flags & EF_MEM_DEVICE;

  int64_t raw_bytes = 0;
  for (int i = 0; i < n_templates; ++i) {
    if (templ_h[i] <= 0 || templ_w[i] <= 0 || templ_offsets[i] < 0)
      return set_err(c, EF_E_INVALID, "ef_tm_prepare: template " + std::to_string(i) + " has a bad shape");
    const int64_t e = templ_offsets[i] + (int64_t)templ_h[i] * templ_w[i];
    raw_bytes = e > raw_bytes ? e : raw_bytes;
  }
  int piece_w = kTmPiece;  // template columns per piece
#ifdef EF_DIAGNOSTICS
  if (const char* e = std::getenv("EF_TM_PIECE")) piece_w = std::max(1, std::min(kTmPiece, std::atoi(e)));
#endif
  std::vector<ImgDesc> rd;
  std::vector<TmPiece> pieces;
  std::vector<TmWork> works;
  int64_t scaled_bytes = 0, part_elems = 0, band_bytes = 0, map_total = 0, max_pos = 0;
  int max_h = 0;
  for (int p = 0; p < n_problems; ++p) {
    const int ti = prob_templ[p], th = prob_h[p], tw = prob_w[p];
    if (ti < 0 || ti >= n_templates || th <= 0 || tw <= 0 || th > frame_h || tw > frame_w || tw > 4096)
      return set_err(c, EF_E_INVALID, "ef_tm_prepare: problem " + std::to_string(p) + " is invalid");
    TmProblem pb{};
    pb.th = th;
    pb.tw = tw;
    pb.hr = frame_h - th + 1;
    pb.wr = frame_w - tw + 1;
    pb.tmpl_off = scaled_bytes;
    rd.push_back(ImgDesc{templ_offsets[ti], scaled_bytes, templ_h[ti], templ_w[ti], 1, th, tw, 0});
    scaled_bytes += rup((int64_t)th * tw, 16);
    const int npiece = (tw + piece_w - 1) / piece_w;
    const int nchunk = (th + kTmChunk - 1) / kTmChunk;
    pb.nparts = npiece * nchunk;
    pb.part_off = part_elems;
    part_elems += (int64_t)pb.nparts * pb.hr * pb.wr;
    pb.map_off = map_total;
    map_total += (int64_t)pb.hr * pb.wr;
    max_pos = std::max<int64_t>(max_pos, (int64_t)pb.hr * pb.wr);
    max_h = std::max(max_h, th);
    if (ef_tm_sums_bits(frame_h, frame_w, (int64_t)th * tw) == 64) t->ii64 = true;
    for (int q = 0; q < npiece; ++q) {
      TmPiece pc{};
      pc.prob = p;
      pc.px = q * piece_w;
      pc.wp = std::min(piece_w, tw - pc.px);
      pc.nkb = (pc.wp + 31 + 31) / 32;
      t->max_nkb = std::max(t->max_nkb, pc.nkb);
      pc.band_off = band_bytes;
      band_bytes += (int64_t)th * pc.nkb * 1024;
      pieces.push_back(pc);
    }
    t->probs.push_back(pb);
  }
  // work items, once the launch's kernel (narrow or wide A ring) is known
  const int kmax = t->max_nkb <= 5 ? 5 : 12;
  for (int pi = 0; pi < (int)pieces.size(); ++pi) {
    const TmPiece& pc = pieces[pi];
    const TmProblem& pb = t->probs[pc.prob];
    const int npiece = (pb.tw + piece_w - 1) / piece_w, nchunk = (pb.th + kTmChunk - 1) / kTmChunk;
    const int q = pc.px / piece_w;
    for (int ch = 0; ch < nchunk; ++ch)
      for (int y0 = 0; y0 < pb.hr; y0 += kTmTile) {
        // the map's last row band: with one or two live 32-row blocks the tile turns into
        // 32 x 512 or 64 x 256 (4 or 2 column groups), so its waves are not left idle
        const int nrb = std::min(4, (pb.hr - y0 + 31) / 32);
        const int ncg = tm_tile_groups(nrb, pc.nkb, kmax);
        for (int x0 = 0; x0 < pb.wr; x0 += kTmTile * ncg)
          works.push_back(
              TmWork{pi, ch * npiece + q, ch * kTmChunk, std::min(pb.th, (ch + 1) * kTmChunk), y0, x0, ncg});
      }
  }
  // longest work items first, so the short ones fill the tail: per template row a tile's
  // fullest wave runs ncb * nkb MFMAs (~32 cycles each; ncb its live column blocks) plus
  // ~650 cycles of LDS round trip and barrier (DESIGN K11)
  auto cost = [&](const TmWork& w) {
    const TmPiece& pc = pieces[w.piece];
    const int ncb = (int)std::min<int64_t>(4, (t->probs[pc.prob].wr - w.x0 + 31) / 32);
    return (int64_t)(w.yb - w.ya) * (32 * ncb * pc.nkb + 650);
  };
  std::stable_sort(works.begin(), works.end(), [&](const TmWork& a, const TmWork& b) { return cost(a) > cost(b); });
  t->nwork = (int)works.size();
  t->max_pos = max_pos;
  t->map_total = map_total;
  hipStream_t s = c->stream;
  EF_TRY(ensure(c, t->raw, std::max<int64_t>(raw_bytes, 16)));
  EF_TRY(ensure(c, t->scaled, std::max<int64_t>(scaled_bytes, 16)));
  EF_TRY(ensure(c, t->bands, std::max<int64_t>(band_bytes, 16)));
  EF_TRY(ensure(c, t->d_probs, std::max<size_t>(t->probs.size() * sizeof(TmProblem), 16)));
  EF_TRY(ensure(c, t->d_pieces, std::max<size_t>(pieces.size() * sizeof(TmPiece), 16)));
  EF_TRY(ensure(c, t->d_works, std::max<size_t>(works.size() * sizeof(TmWork), 16)));
  EF_TRY(ensure(c, t->d_stat, std::max<size_t>((size_t)n_problems * sizeof(TmStat), 16)));
  EF_TRY(ensure(c, t->parts, std::max<int64_t>(part_elems * 4, 16)));
  EF_TRY(ensure(c, t->keys, std::max<size_t>((size_t)n_problems * 8, 16)));
  EF_TRY(ensure(c, t->f8, (size_t)(frame_h + kTmTile + 32) * t->pitch));
  EF_TRY(ensure(c, t->ii1, (size_t)(frame_h + 1) * (frame_w + 1) * 8));
  EF_TRY(ensure(c, t->ii2, (size_t)(frame_h + 1) * (frame_w + 1) * 8));
  EF_TRY(ensure(c, t->frame_stage, (size_t)frame_h * frame_w));
  EF_HIP(c, hipMemsetAsync(t->f8.p, 0, t->f8.bytes, s), "memset frame");
  if (raw_bytes > 0)
    EF_HIP(c, hipMemcpyAsync(t->raw.p, templ_data, raw_bytes, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s),
           "templates");
  if (n_problems > 0) {
    ImgDesc* drd = nullptr;
    EF_TRY(ensure(c, c->p_stage, rd.size() * sizeof(ImgDesc)));
    drd = static_cast<ImgDesc*>(c->p_stage.p);
    EF_HIP(c, hipMemcpyAsync(drd, rd.data(), rd.size() * sizeof(ImgDesc), hipMemcpyHostToDevice, s), "H2D desc");
    EF_HIP(c, hipMemcpyAsync(t->d_probs.p, t->probs.data(), t->probs.size() * sizeof(TmProblem),
                             hipMemcpyHostToDevice, s), "H2D problems");
    EF_HIP(c, hipMemcpyAsync(t->d_pieces.p, pieces.data(), pieces.size() * sizeof(TmPiece), hipMemcpyHostToDevice, s),
           "H2D pieces");
    EF_HIP(c, hipMemcpyAsync(t->d_works.p, works.data(), works.size() * sizeof(TmWork), hipMemcpyHostToDevice, s),
           "H2D works");
    int64_t max_out = 0;
    for (auto& d : rd) max_out = std::max<int64_t>(max_out, (int64_t)d.oh * d.ow);
    EF_HIP(c, launch_resize(s, static_cast<const uint8_t*>(t->raw.p), drd, (int)rd.size(), max_out, false,
                            static_cast<uint8_t*>(t->scaled.p)), "resize templates");
    hipLaunchKernelGGL(tm_stat_kernel, dim3((unsigned)n_problems), dim3(256), 0, s,
                       static_cast<const uint8_t*>(t->scaled.p), static_cast<const TmProblem*>(t->d_probs.p),
                       static_cast<TmStat*>(t->d_stat.p));
    hipLaunchKernelGGL(tm_band_kernel, dim3((unsigned)max_h, (unsigned)pieces.size()), dim3(256), 0, s,
                       static_cast<const uint8_t*>(t->scaled.p), static_cast<const TmProblem*>(t->d_probs.p),
                       static_cast<const TmPiece*>(t->d_pieces.p), static_cast<uint8_t*>(t->bands.p));
    EF_HIP(c, hipGetLastError(), "template prepare kernels");
  }
  EF_HIP(c, hipStreamSynchronize(s), "sync");  // host vectors and staged descriptors go out of scope
  return EF_OK;
}

int ef_tm_match(ef_ctx* c, const uint8_t* frame, int64_t frame_ld, float* best_out, int32_t* x_out, int32_t* y_out,
                float* maps_out, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  TmState* t = static_cast<TmState*>(c->tm);
  if (!t) return set_err(c, EF_E_STATE, "ef_tm_match: call ef_tm_prepare first");
  if (!frame || frame_ld < t->W) return set_err(c, EF_E_INVALID, "ef_tm_match: bad frame");
  EF_HIP(c, hipSetDevice(c->device), "hipSetDevice");
  const bool dev = flags & EF_MEM_DEVICE;
  hipStream_t s = c->stream;
  const int H = t->H, W = t->W;
  const uint8_t* f = frame;
  if (!dev) {
    EF_HIP(c, hipMemcpy2DAsync(t->frame_stage.p, W, frame, frame_ld, W, H, hipMemcpyHostToDevice, s), "H2D frame");
    f = static_cast<const uint8_t*>(t->frame_stage.p);
    frame_ld = W;
  }
  int8_t* f8 = static_cast<int8_t*>(t->f8.p);
  unsigned long long* keys = static_cast<unsigned long long*>(t->keys.p);
  TimerEvt tev;
  timer_begin(c, EF_KERNEL_TMATCH, &tev);
  const dim3 rgrid((unsigned)((H + 1 + 3) / 4)), cgrid((unsigned)((W + 1 + kColW - 1) / kColW));
  // The integral images' column pass runs on a side stream beside the correlation kernel
  // (it needs only the row pass; the score kernel joins both): its 8 KiB blocks fit next to
  // a correlation workgroup's 147 KiB of LDS.
  bool side = t->nprob > 0 && t->nwork > 0;
#ifdef EF_DIAGNOSTICS
  if (std::getenv("EF_TM_NOSIDE")) side = false;  // A/B: column pass in line
#endif
  if (side) {
    if (!c->tm_side) EF_HIP(c, hipStreamCreateWithFlags(&c->tm_side, hipStreamNonBlocking), "tm side stream");
    for (int i = 0; i < 2; ++i)
      if (!c->tm_side_ev[i]) EF_HIP(c, hipEventCreateWithFlags(&c->tm_side_ev[i], hipEventDisableTiming), "tm event");
  }
  hipStream_t cs = side ? c->tm_side : s;  // the column pass's stream
  if (t->ii64) {
    long long* ii1 = static_cast<long long*>(t->ii1.p);
    long long* ii2 = static_cast<long long*>(t->ii2.p);
    hipLaunchKernelGGL(tm_rows_kernel<long long>, rgrid, dim3(256), 0, s, f, H, W, frame_ld, f8, t->pitch, ii1, ii2,
                       keys, t->nprob);
    if (side) {
      EF_HIP(c, hipEventRecord(c->tm_side_ev[0], s), "rows done");
      EF_HIP(c, hipStreamWaitEvent(cs, c->tm_side_ev[0], 0), "side waits rows");
    }
    hipLaunchKernelGGL(tm_cols_kernel<long long>, cgrid, dim3(1024), 0, cs, H, W, ii1, ii2);
  } else {
    unsigned* ii1 = static_cast<unsigned*>(t->ii1.p);
    unsigned* ii2 = static_cast<unsigned*>(t->ii2.p);
    hipLaunchKernelGGL(tm_rows_kernel<unsigned>, rgrid, dim3(256), 0, s, f, H, W, frame_ld, f8, t->pitch, ii1, ii2,
                       keys, t->nprob);
    if (side) {
      EF_HIP(c, hipEventRecord(c->tm_side_ev[0], s), "rows done");
      EF_HIP(c, hipStreamWaitEvent(cs, c->tm_side_ev[0], 0), "side waits rows");
    }
    hipLaunchKernelGGL(tm_cols_kernel<unsigned>, cgrid, dim3(1024), 0, cs, H, W, ii1, ii2);
  }
  if (side) EF_HIP(c, hipEventRecord(c->tm_side_ev[1], cs), "cols done");
  if (t->nprob > 0) {
    if (t->nwork > 0) {
      bool narrow = t->max_nkb <= 5;
#ifdef EF_DIAGNOSTICS
      if (std::getenv("EF_TM_WIDE")) narrow = false;  // A/B: one workgroup per CU
#endif
      auto corr = narrow ? tm_corr_kernel<5> : tm_corr_kernel<12>;
      hipLaunchKernelGGL(corr, dim3((unsigned)t->nwork), dim3(512), 0, s, f8, t->pitch,
                         static_cast<const uint8_t*>(t->bands.p), static_cast<const TmPiece*>(t->d_pieces.p),
                         static_cast<const TmWork*>(t->d_works.p), static_cast<const TmProblem*>(t->d_probs.p),
                         static_cast<int*>(t->parts.p), t->nwork);
    }
    float* maps = nullptr;
    if (maps_out) {
      if (dev) {
        maps = maps_out;
      } else {
        EF_TRY(ensure(c, t->maps, (size_t)t->map_total * 4));
        maps = static_cast<float*>(t->maps.p);
      }
    }
    if (side) EF_HIP(c, hipStreamWaitEvent(s, c->tm_side_ev[1], 0), "score waits cols");
    const int64_t sblk = 64;  // row-strided blocks per problem
    const dim3 sgrid((unsigned)sblk, (unsigned)t->nprob);
    const TmProblem* dp = static_cast<const TmProblem*>(t->d_probs.p);
    const TmStat* dst = static_cast<const TmStat*>(t->d_stat.p);
    const int* dparts = static_cast<const int*>(t->parts.p);
    if (t->ii64)
      hipLaunchKernelGGL(tm_score_kernel<long long>, sgrid, dim3(256), 0, s, dp, dst, dparts,
                         static_cast<const long long*>(t->ii1.p), static_cast<const long long*>(t->ii2.p), W, maps,
                         keys);
    else
      hipLaunchKernelGGL(tm_score_kernel<unsigned>, sgrid, dim3(256), 0, s, dp, dst, dparts,
                         static_cast<const unsigned*>(t->ii1.p), static_cast<const unsigned*>(t->ii2.p), W, maps,
                         keys);
    timer_end(c, &tev);
    EF_HIP(c, hipGetLastError(), "template match kernels");
    std::vector<unsigned long long> hk((size_t)t->nprob);
    EF_HIP(c, hipMemcpyAsync(hk.data(), keys, hk.size() * 8, hipMemcpyDeviceToHost, s), "D2H keys");
    if (maps_out && !dev)
      EF_HIP(c, hipMemcpyAsync(maps_out, maps, (size_t)t->map_total * 4, hipMemcpyDeviceToHost, s), "D2H maps");
    EF_HIP(c, hipStreamSynchronize(s), "sync");
    for (int p = 0; p < t->nprob; ++p) {
      const unsigned o = ~(unsigned)(hk[p] >> 32);
      const unsigned b = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
      float v;
      std::memcpy(&v, &b, 4);
      const unsigned idx = (unsigned)(hk[p] & 0xffffffffu);
      if (best_out) best_out[p] = v;
      if (x_out) x_out[p] = (int32_t)(idx % (unsigned)t->probs[p].wr);
      if (y_out) y_out[p] = (int32_t)(idx / (unsigned)t->probs[p].wr);
    }
  } else {
    timer_end(c, &tev);
    EF_HIP(c, hipStreamSynchronize(s), "sync");
  }
  return EF_OK;
}

int ef_tm_info(ef_ctx* c, int32_t* n_problems, int64_t* map_elems, int32_t* result_h, int32_t* result_w) {
  if (!c) return EF_E_INVALID;
  TmState* t = static_cast<TmState*>(c->tm);
  if (!t) return set_err(c, EF_E_STATE, "ef_tm_info: call ef_tm_prepare first");
  if (n_problems) *n_problems = t->nprob;
  if (map_elems) *map_elems = t->map_total;
  for (int p = 0; p < t->nprob; ++p) {
    if (result_h) result_h[p] = t->probs[p].hr;
    if (result_w) result_w[p] = t->probs[p].wr;
  }
  return EF_OK;
}

}  // extern "C"
