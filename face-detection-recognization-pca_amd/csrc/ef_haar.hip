// Haar cascade face detector: the
//     face_cascade.detectMultiScale(gray, scaleFactor=1.1, minNeighbors=5, minSize=(30, 30))
// of detection-v4.py:18, :50-55, evaluated the way OpenCV 4.x's CascadeClassifierImpl runs
// a stump-based HAAR cascade (cascadedetect.cpp), for a cascade the caller loads (the
// reference's haarcascade_frontalface_default.xml ships inside OpenCV, which is absent
// here, so parity is unpinned; tests use synthetic cascades against oracle/haar_oracle.py).
//
// Per frame, all on the GPU except the final rectangle grouping:
//   1. pyramid: one ragged resize launch builds every layer (W/s, H/s) of the scale list
//      (INTER_LINEAR rules of ef_image.hip; OpenCV uses INTER_LINEAR_EXACT here — the one
//      documented deviation);
//   2. integral images of every layer (int32, as OpenCV's CV_32S sum) and of its squares
//      (uint32 with wrap-around, as OpenCV's: window sums are differences mod 2^32 and a
//      window's sum of squares fits); row scan per wave, column scan per 64-column strip;
//   3. `haar_stage0_kernel`: one thread per window origin of every layer — variance
//      normalisation (HaarEvaluator::setWindow: nf = area * sqsum - sum^2 over the window
//      shrunk by one pixel, 1/sqrt(nf) as float, reject when area / sqrt(nf) >= 0.1) and
//      the first stage, result -1 / 0 / 1;
//   4. `haar_rows_kernel`: CascadeClassifierInvoker's scan order — a stage-0 rejection
//      skips the next x position — resolved per (layer, row) from the stage-0 results,
//      compacting the surviving windows into a work list;
//   5. `haar_cascade_kernel`: the remaining stages in groups (1-2, 3-5, 6-9, 10-14, 15-..),
//      one launch per group over the compacted survivors of the previous one (thread per
//      window), so waves stay full as the cascade rejects; accepted windows appended as
//      candidates;
// then the host sorts the candidates into OpenCV's (scale, y, x) order and runs
// cv::groupRectangles(minNeighbors, eps = 0.2) (connected components of SimilarRects,
// averaged rectangles, neighbour threshold, nested-rectangle filter).
// Float arithmetic follows predictOrderedStump: feature = w0*S0 + w1*S1 (+ w2*S2) in
// float (no contraction), times the float normalisation factor, compared with the stump
// threshold; the stage sum accumulates the float leaves in double.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "ef_internal.hpp"

namespace ef {

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

struct HaarFeat {
  int x[3], y[3], w[3], h[3];
  float wt[3];
  int nr;
};
struct HaarStump {
  int feat;
  float thr, left, right;
};
// One stump with its feature inlined (stump order): what the split cascade kernel stages
// into LDS per stage, so a stump costs no dependent scalar loads of the stump and feature
// tables (those miss the scalar cache: the tables are ~180 KB for a frontal-face cascade).
// src[r - 1][k]: corner k of rect r (0 (x, y), 1 (x + w, y), 2 (x, y + h), 3 (x + w, y + h))
// equals corner src of rect 0, or -1 (its own gather) — e.g. a half rect sharing the
// whole rect's right edge; the split kernel reuses rect 0's loaded value.
struct HaarRec {
  float thr, left, right;
  int nr;
  int x[3], y[3], w[3], h[3];
  float wt[3];
  int pad;
  signed char src[2][4];
};
struct HaarStage {
  int first, count;
  float thr;
  int pad;
};
struct HaarLayer {
  int w, h, nx, ny, step;
  float scale;
  int64_t pix_off, ii_off, res_off;
};
struct HaarCand {
  int layer, y, x;
  float vnf;  // the window's normalisation factor (stage 0's haar_norm), carried along the lists
};

// ------------------------------------------------------------------ integral images
// Row prefix sums of one layer row per wave (row 0 of the integral image is zero).
__global__ __launch_bounds__(256) void haar_rows_ii_kernel(const uint8_t* __restrict__ pix,
                                                           const HaarLayer* __restrict__ L, int* __restrict__ ii1,
                                                           unsigned* __restrict__ ii2) {
  const HaarLayer ly = L[blockIdx.y];
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row > ly.h) return;
  const int64_t W1 = ly.w + 1;
  int* r1 = ii1 + ly.ii_off + row * W1;
  unsigned* r2 = ii2 + ly.ii_off + row * W1;
  if (row == 0) {
    for (int x = lane; x <= ly.w; x += 64) r1[x] = 0, r2[x] = 0u;
    return;
  }
  const uint8_t* src = pix + ly.pix_off + (int64_t)(row - 1) * ly.w;
  // 64-pixel chunks, lane = pixel (coalesced), an inclusive wave scan per chunk carried
  // into the row totals (CV_32S sum / wrapping sqsum: the same values mod 2^32)
  if (lane == 0) r1[0] = r2[0] = 0;
  unsigned c1 = 0, c2 = 0;
  for (int x0 = 0; x0 < ly.w; x0 += 64) {
    const int x = x0 + lane;
    unsigned e1 = 0, e2 = 0;
    if (x < ly.w) {
      const unsigned v = src[x];
      e1 = v;
      e2 = v * v;
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned t1 = __shfl_up(e1, off), t2 = __shfl_up(e2, off);
      if (lane >= off) {
        e1 += t1;
        e2 += t2;
      }
    }
    if (x < ly.w) {
      r1[x + 1] = (int)(c1 + e1);
      r2[x + 1] = c2 + e2;
    }
    c1 += __shfl(e1, 63);
    c2 += __shfl(e2, 63);
  }
}

// Column prefix: block = 64 columns x 16 row segments of one layer.
__global__ __launch_bounds__(1024) void haar_cols_ii_kernel(const HaarLayer* __restrict__ L, int* __restrict__ ii1,
                                                            unsigned* __restrict__ ii2) {
  const HaarLayer ly = L[blockIdx.y];
  __shared__ int t1[16][64];
  __shared__ unsigned t2[16][64];
  const int cx = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int x = blockIdx.x * 64 + cx;
  if (blockIdx.x * 64 > ly.w) return;  // uniform per block
  const int64_t W1 = ly.w + 1;
  int* a1 = ii1 + ly.ii_off;
  unsigned* a2 = ii2 + ly.ii_off;
  const int per = (ly.h + 15) / 16;
  const int ya = 1 + sg * per, yb = ya + per < ly.h + 1 ? ya + per : ly.h + 1;
  int s1 = 0;
  unsigned s2 = 0;
  if (x <= ly.w)
    for (int y = ya; y < yb; ++y) {
      s1 += a1[y * W1 + x];
      s2 += a2[y * W1 + x];
    }
  t1[sg][cx] = s1;
  t2[sg][cx] = s2;
  __syncthreads();
  int o1 = 0;
  unsigned o2 = 0;
  for (int q = 0; q < sg; ++q) {
    o1 += t1[q][cx];
    o2 += t2[q][cx];
  }
  if (x <= ly.w)
    for (int y = ya; y < yb; ++y) {
      o1 += a1[y * W1 + x];
      o2 += a2[y * W1 + x];
      a1[y * W1 + x] = o1;
      a2[y * W1 + x] = o2;
    }
}

// ------------------------------------------------------------------ cascade evaluation
template <typename T>
__device__ __forceinline__ T box(const T* ii, int64_t W1, int x, int y, int w, int h) {
  return ii[(int64_t)(y + h) * W1 + x + w] - ii[(int64_t)y * W1 + x + w] - ii[(int64_t)(y + h) * W1 + x] +
         ii[(int64_t)y * W1 + x];
}

// HaarEvaluator::setWindow: the float normalisation factor, or 0 for a rejected window.
__device__ __forceinline__ float haar_norm(const int* ii1, const unsigned* ii2, int64_t W1, int x, int y, int ww,
                                           int wh) {
  const double area = (double)((ww - 2) * (wh - 2));
  const int s = box(ii1, W1, x + 1, y + 1, ww - 2, wh - 2);
  const unsigned q = box(ii2, W1, x + 1, y + 1, ww - 2, wh - 2);
  const double nf = __dsub_rn(__dmul_rn(area, (double)q), __dmul_rn((double)s, (double)s));
  if (!(nf > 0.0)) return 0.f;
  const float v = __double2float_rn(__ddiv_rn(1.0, sqrt(nf)));
  return __dmul_rn(area, (double)v) < 0.1 ? v : 0.f;
}

// One stage (predictOrderedStump's inner loop): true when the window passes it.
__device__ __forceinline__ bool haar_stage(const int* ii1, int64_t W1, int x, int y, float vnf,
                                           const HaarStage& st, const HaarRec* __restrict__ recs) {
  double tmp = 0.0;
  for (int i = 0; i < st.count; ++i) {
    const HaarRec f = recs[st.first + i];  // stump + feature in one (wave-uniform) record
    float val = __fmul_rn(f.wt[0], (float)box(ii1, W1, x + f.x[0], y + f.y[0], f.w[0], f.h[0]));
    val = __fadd_rn(val, __fmul_rn(f.wt[1], (float)box(ii1, W1, x + f.x[1], y + f.y[1], f.w[1], f.h[1])));
    if (f.wt[2] != 0.f)
      val = __fadd_rn(val, __fmul_rn(f.wt[2], (float)box(ii1, W1, x + f.x[2], y + f.y[2], f.w[2], f.h[2])));
    val = __fmul_rn(val, vnf);
    tmp = __dadd_rn(tmp, (double)(val < f.thr ? f.left : f.right));
  }
  return !(tmp < (double)st.thr);
}

// Pass 1: variance + first stage for every visitable window origin of every layer (grid (pos/256,
// layers)); res = -1 (low variance), 0 (rejected by stage 0), 1 (passed stage 0).
__global__ __launch_bounds__(256) void haar_stage0_kernel(const HaarLayer* __restrict__ L,
                                                          const int* __restrict__ ii1,
                                                          const unsigned* __restrict__ ii2,
                                                          const HaarStage* __restrict__ stages,
                                                          const HaarRec* __restrict__ recs, int ww, int wh,
                                                          signed char* __restrict__ res, float* __restrict__ vn) {
  const HaarLayer ly = L[blockIdx.y];
  // only the origins the invoker can visit: x and y multiples of the layer's step (a
  // step-2 layer has a quarter of its origins evaluated; the rest are never read)
  const int nxs = (ly.nx + ly.step - 1) / ly.step, nys = (ly.ny + ly.step - 1) / ly.step;
  const int64_t ps = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (ps >= (int64_t)nxs * nys) return;
  const int ys = (int)(ps / nxs);
  const int y = ys * ly.step, x = (int)(ps - (int64_t)ys * nxs) * ly.step;
  const int64_t p = (int64_t)y * ly.nx + x;
  const int64_t W1 = ly.w + 1;
  const int* a1 = ii1 + ly.ii_off;
  const float vnf = haar_norm(a1, ii2 + ly.ii_off, W1, x, y, ww, wh);
  signed char r = -1;
  if (vnf != 0.f) r = haar_stage(a1, W1, x, y, vnf, stages[0], recs) ? 1 : 0;
  res[ly.res_off + p] = r;
  vn[ly.res_off + p] = vnf;
}

// Pass 2: the invoker's x walk for each (layer, evaluated row): positions 0, step, ...
// with one extra step after a stage-0 rejection; survivors of stage 0 go to the list.
// One wave per row, 16 rows per workgroup: 64 positions per chunk are loaded coalesced,
// the walk's recurrence (position i+1 is visited unless i was visited and rejected) is
// solved in closed form on the wave-uniform ballot masks, and the workgroup appends all
// its rows' survivors with ONE atomicAdd (count pass, then write pass).  A thread-per-row
// walk of dependent byte loads with per-survivor atomics took ~150 us per 640x480 frame;
// one atomic per chunk still ~90 us (a single counter serialises them).
constexpr int kHaarRowWaves = 16;
constexpr int kHaarMaxLayers = 255;

__device__ __forceinline__ unsigned long long haar_walk(unsigned long long rej, bool& v) {
  // within a run of rejected positions the walk visits every other one from the run's
  // first (visited) position; right after a run it visits unless the run's last position
  // was visited.  A position is a run start when the one before it is not rejected (or,
  // for bit 0, when the carried-in position is visited).
  const unsigned long long EVEN = 0x5555555555555555ull;
  const unsigned long long R = v ? rej : (rej & ~1ull);  // an unvisited bit 0 cannot skip
  const unsigned long long S = R & ~(R << 1);             // run starts
  const unsigned long long RE = R & ~(R + (S & EVEN));    // runs that start at even bits
  const unsigned long long E = (RE & EVEN) | (R & ~RE & ~EVEN);  // even offset in its run
  unsigned long long vis = (R & E) | (~R & ~((R & E) << 1));
  if (!v) vis &= ~1ull;
  v = !(((vis >> 63) & 1ull) && ((rej >> 63) & 1ull));
  return vis;
}

__global__ __launch_bounds__(1024) void haar_rows_kernel(const HaarLayer* __restrict__ L, int nlayers,
                                                         const int* __restrict__ row_start,
                                                         const signed char* __restrict__ res,
                                                         const float* __restrict__ vn,
                                                         HaarCand* __restrict__ work, int* __restrict__ nwork,
                                                         int cap) {
  __shared__ int rs[kHaarMaxLayers + 1];
  __shared__ int woff[kHaarRowWaves];
  for (int i = threadIdx.x; i <= nlayers; i += blockDim.x) rs[i] = row_start[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gr = blockIdx.x * kHaarRowWaves + wave;  // evaluated row of this wave
  const bool live = gr < rs[nlayers];
  int li = 0;
  if (live)
    while (rs[li + 1] <= gr) ++li;
  const HaarLayer ly = L[li];
  const int y = live ? (gr - rs[li]) * ly.step : 0;
  const signed char* rr = res + ly.res_off + (int64_t)y * ly.nx;
  const int npos = live ? (ly.nx + ly.step - 1) / ly.step : 0;  // visited candidates: x = i * step
  auto chunk = [&](int c0, bool& v) {
    const int i = c0 + lane;
    const signed char r = i < npos ? rr[(int64_t)i * ly.step] : (signed char)-1;
    const unsigned long long rej = __ballot(r == 0);
    const unsigned long long pas = __ballot(r > 0);
    return haar_walk(rej, v) & pas;
  };
  int total = 0;
  bool v = true;
  for (int c0 = 0; c0 < npos; c0 += 64) total += __popcll(chunk(c0, v));
  if (lane == 0) woff[wave] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    int sum = 0;
    for (int w = 0; w < kHaarRowWaves; ++w) {
      const int t = woff[w];
      woff[w] = sum;
      sum += t;
    }
    const int base = sum ? atomicAdd(nwork, sum) : 0;
    for (int w = 0; w < kHaarRowWaves; ++w) woff[w] += base;
  }
  __syncthreads();
  int k = woff[wave];
  v = true;
  for (int c0 = 0; c0 < npos; c0 += 64) {
    const unsigned long long surv = chunk(c0, v);
    if ((surv >> lane) & 1ull) {
      const int kk = k + __popcll(surv & ((1ull << lane) - 1ull));
      const int x = (c0 + lane) * ly.step;
      if (kk < cap) work[kk] = HaarCand{li, y, x, vn[ly.res_off + (int64_t)y * ly.nx + x]};
    }
    k += __popcll(surv);
  }
}

// Pass 3: stages [s0, s1) for each window of the input list; survivors go to the output
// list (the candidates after the last group).  Grid sized by the host's upper bound, the
// live count read from device memory.
__global__ __launch_bounds__(256) void haar_cascade_kernel(const HaarLayer* __restrict__ L,
                                                           const int* __restrict__ ii1,
                                                           const unsigned* __restrict__ ii2,
                                                           const HaarStage* __restrict__ stages, int s0, int s1,
                                                           const HaarRec* __restrict__ recs, int ww, int wh,
                                                           const HaarCand* __restrict__ in, const int* __restrict__ nin,
                                                           int cap, HaarCand* __restrict__ out, int* __restrict__ nout) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = min(*nin, cap);
  if (i >= n) return;
  const HaarCand w = in[i];
  const HaarLayer ly = L[w.layer];
  const int64_t W1 = ly.w + 1;
  const int* a1 = ii1 + ly.ii_off;
  const float vnf = w.vnf;  // == haar_norm(a1, ii2 + ly.ii_off, W1, w.x, w.y, ww, wh)
  for (int s = s0; s < s1; ++s)
    if (!haar_stage(a1, W1, w.x, w.y, vnf, stages[s], recs)) return;
  const int k = atomicAdd(nout, 1);
  if (k < cap) out[k] = w;
}

// The feature value of predictOrderedStump (same int box sums, same float operations in
// the same order) with rect 1/2 corners that coincide with rect 0's taken from rect 0's
// loads instead of gathered again (the split kernel is gather-bound).
__device__ __forceinline__ float haar_feature_shared(const int* __restrict__ a1, int64_t W1, int wx, int wy,
                                                     const HaarRec& f) {
  const int64_t b0 = (int64_t)(wy + f.y[0]) * W1 + wx + f.x[0], h0 = (int64_t)f.h[0] * W1;
  const int c[4] = {a1[b0], a1[b0 + f.w[0]], a1[b0 + h0], a1[b0 + h0 + f.w[0]]};
  float val = __fmul_rn(f.wt[0], (float)(c[3] - c[1] - c[2] + c[0]));
#pragma unroll
  for (int r = 1; r < 3; ++r) {
    if (r == 2 && f.wt[2] == 0.f) break;
    const int64_t br = (int64_t)(wy + f.y[r]) * W1 + wx + f.x[r], hr = (int64_t)f.h[r] * W1;
    const int64_t off[4] = {br, br + f.w[r], br + hr, br + hr + f.w[r]};
    int v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int sc = f.src[r - 1][k];
      if (sc < 0)
        v[k] = a1[off[k]];
      else
        v[k] = sc == 0 ? c[0] : (sc == 1 ? c[1] : (sc == 2 ? c[2] : c[3]));
    }
    val = __fadd_rn(val, __fmul_rn(f.wt[r], (float)(v[3] - v[1] - v[2] + v[0])));
  }
  return val;
}

// Pass 3, split form: a workgroup of 4 waves takes 64 windows (lane = window, as above, so
// each stump's integral-image gathers stay coalesced over neighbouring windows) and wave q
// evaluates stumps q, q+4, q+8, ... of every stage, read from LDS records (stump + its
// feature inlined, staged 256 at a time); the four partial sums are combined in LDS.  4x the waves of the thread-per-window form and a quarter of the serial stump
// chain per stage — the late groups have few windows and ~100-200 stumps per stage.  Only
// used for cascades whose stage sums are exact in double in any association (checked at
// ef_haar_set_cascade), so the decisions equal predictOrderedStump's sequential sum.
// NQ waves per workgroup (4, 8 or 16): the late groups hold a few thousand windows, so
// the kernel is bound by the latency of each wave's serial stump chain — more waves per
// window block and 4 stumps' gathers in flight per wave (unrolled) shorten it.
constexpr int kHaarRecChunk = 256;
template <int NQ>
__global__ __launch_bounds__(NQ * 64) void haar_cascade_split_kernel(const HaarLayer* __restrict__ L,
                                                                 const int* __restrict__ ii1,
                                                                 const unsigned* __restrict__ ii2,
                                                                 const HaarStage* __restrict__ stages, int s0, int s1,
                                                                 const HaarRec* __restrict__ recs, int ww, int wh,
                                                                 const HaarCand* __restrict__ in,
                                                                 const int* __restrict__ nin, int cap,
                                                                 HaarCand* __restrict__ out, int* __restrict__ nout) {
  __shared__ double part[NQ][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int n = min(*nin, cap);
  const int i = blockIdx.x * 64 + lane;
  if (blockIdx.x * 64 >= n) return;  // uniform over the workgroup
  const bool valid = i < n;
  const HaarCand w = in[valid ? i : blockIdx.x * 64];
  const HaarLayer ly = L[w.layer];
  const int64_t W1 = ly.w + 1;
  const int* a1 = ii1 + ly.ii_off;
  const float vnf = w.vnf;  // == haar_norm(a1, ii2 + ly.ii_off, W1, w.x, w.y, ww, wh)
  bool alive = valid;
  __shared__ HaarRec srec[kHaarRecChunk];
  for (int st = s0; st < s1; ++st) {
    const HaarStage sg = stages[st];
    double tmp = 0.0;
    for (int c0 = 0; c0 < sg.count; c0 += kHaarRecChunk) {
      const int cn = min(kHaarRecChunk, sg.count - c0);
      {  // stage the chunk's records (dword-wise, coalesced)
        const int* src = reinterpret_cast<const int*>(recs + sg.first + c0);
        int* dst = reinterpret_cast<int*>(srec);
        for (int e = threadIdx.x; e < cn * (int)(sizeof(HaarRec) / 4); e += NQ * 64) dst[e] = src[e];
      }
      __syncthreads();
      if (alive) {
#pragma unroll 4
        for (int t = q; t < cn; t += NQ) {  // wave q: every NQ-th stump (the sum is order-free)
          const HaarRec& f = srec[t];
          float val = haar_feature_shared(a1, W1, w.x, w.y, f);
          val = __fmul_rn(val, vnf);
          tmp = __dadd_rn(tmp, (double)(val < f.thr ? f.left : f.right));
        }
      }
      __syncthreads();  // the chunk is consumed before the next one is staged
    }
    part[q][lane] = tmp;
    __syncthreads();
    if (alive) {
      double tot = part[0][lane];
#pragma unroll
      for (int r = 1; r < NQ; ++r) tot = __dadd_rn(tot, part[r][lane]);
      alive = !(tot < (double)sg.thr);
    }
    if (!__syncthreads_or(alive)) return;  // every window of the workgroup rejected
  }
  if (alive && q == 0) {
    const int k = atomicAdd(nout, 1);
    if (k < cap) out[k] = w;
  }
}

// ------------------------------------------------------------------ host side
struct HaarState {
  int ww = 0, wh = 0, nstages = 0;
  bool order_free = false;  // every stage sum is exact in double in any order (see set_cascade)
  DevBuf stages, recs;
  DevBuf pix, ii1, ii2, res, vn, layers, rowstart, work, cand, counters, frame, desc;
};

void haar_release(ef_ctx* c) {
  if (!c || !c->haar) return;
  HaarState* h = static_cast<HaarState*>(c->haar);
  DevBuf* bufs[] = {&h->stages, &h->recs, &h->pix, &h->ii1,      &h->ii2,     &h->res, &h->vn,
                    &h->layers, &h->rowstart, &h->work, &h->cand, &h->counters, &h->frame, &h->desc};
  for (DevBuf* b : bufs) release(*b);
  delete h;
  c->haar = nullptr;
}

static int cv_round(double v) { return (int)std::lrint(v); }

struct RectI {
  int x, y, w, h;
};

// cv::groupRectangles(rects, thr, eps): SimilarRects components numbered by lowest member,
// averaged per class, classes with <= thr members dropped, then the nested-rectangle filter.
static std::vector<RectI> group_rectangles(const std::vector<RectI>& rects, int thr, double eps) {
  if (thr <= 0 || rects.empty()) return rects;
  const int n = (int)rects.size();
  std::vector<int> parent(n);
  for (int i = 0; i < n; ++i) parent[i] = i;
  auto find = [&](int i) {
    while (parent[i] != i) {
      parent[i] = parent[parent[i]];
      i = parent[i];
    }
    return i;
  };
  auto similar = [&](const RectI& a, const RectI& b) {
    const double delta = eps * (std::min(a.w, b.w) + std::min(a.h, b.h)) * 0.5;
    return std::abs(a.x - b.x) <= delta && std::abs(a.y - b.y) <= delta &&
           std::abs(a.x + a.w - b.x - b.w) <= delta && std::abs(a.y + a.h - b.y - b.h) <= delta;
  };
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (similar(rects[i], rects[j])) {
        const int ri = find(i), rj = find(j);
        if (ri != rj) parent[std::max(ri, rj)] = std::min(ri, rj);
      }
  std::vector<int> label(n), cls_of_root(n, -1);
  int nc = 0;
  for (int i = 0; i < n; ++i) {
    const int r = find(i);
    if (cls_of_root[r] < 0) cls_of_root[r] = nc++;
    label[i] = cls_of_root[r];
  }
  std::vector<long long> acc((size_t)nc * 4, 0);
  std::vector<int> cnt(nc, 0);
  for (int i = 0; i < n; ++i) {
    long long* a = &acc[(size_t)label[i] * 4];
    a[0] += rects[i].x;
    a[1] += rects[i].y;
    a[2] += rects[i].w;
    a[3] += rects[i].h;
    cnt[label[i]]++;
  }
  std::vector<RectI> rr(nc);
  for (int c = 0; c < nc; ++c) {
    const float s = 1.f / (float)cnt[c];
    const long long* a = &acc[(size_t)c * 4];
    rr[c] = RectI{(int)std::lrint((float)a[0] * s), (int)std::lrint((float)a[1] * s), (int)std::lrint((float)a[2] * s),
                  (int)std::lrint((float)a[3] * s)};
  }
  std::vector<RectI> out;
  for (int i = 0; i < nc; ++i) {
    const RectI r1 = rr[i];
    const int n1 = cnt[i];
    if (n1 <= thr) continue;
    int j = 0;
    for (; j < nc; ++j) {
      const int n2 = cnt[j];
      if (j == i || n2 <= thr) continue;
      const RectI r2 = rr[j];
      const int dx = cv_round(r2.w * eps), dy = cv_round(r2.h * eps);
      if (r1.x >= r2.x - dx && r1.y >= r2.y - dy && r1.x + r1.w <= r2.x + r2.w + dx &&
          r1.y + r1.h <= r2.y + r2.h + dy && (n2 > std::max(3, n1) || n1 < 3))
        break;
    }
    if (j == nc) out.push_back(r1);
  }
  return out;
}

}  // namespace ef

using namespace ef;

extern "C" {

int ef_haar_set_cascade(ef_ctx* c, int32_t win_w, int32_t win_h, int32_t n_features, const int32_t* rects,
                        const float* weights, int32_t n_stages, const int32_t* stage_count,
                        const float* stage_threshold, int32_t n_stumps, const int32_t* stump_feature,
                        const float* stump_threshold, const float* stump_left, const float* stump_right) {
  if (!c) return EF_E_INVALID;
  if (win_w < 3 || win_h < 3 || n_features < 1 || n_stages < 1 || n_stumps < 1 || !rects || !weights ||
      !stage_count || !stage_threshold || !stump_feature || !stump_threshold || !stump_left || !stump_right)
    return set_err(c, EF_E_INVALID, "ef_haar_set_cascade: bad arguments");
  std::vector<HaarFeat> f((size_t)n_features);
  for (int i = 0; i < n_features; ++i) {
    HaarFeat& q = f[i];
    q.nr = 0;
    for (int k = 0; k < 3; ++k) {
      const int* r = rects + ((size_t)i * 3 + k) * 4;
      q.x[k] = r[0], q.y[k] = r[1], q.w[k] = r[2], q.h[k] = r[3];
      q.wt[k] = weights[(size_t)i * 3 + k];
      if (k == 2 && q.wt[k] == 0.f) q.x[k] = q.y[k] = q.w[k] = q.h[k] = 0;
      if (q.wt[k] != 0.f || k < 2) {
        if (q.x[k] < 0 || q.y[k] < 0 || q.w[k] < 0 || q.h[k] < 0 || q.x[k] + q.w[k] > win_w ||
            q.y[k] + q.h[k] > win_h)
          return set_err(c, EF_E_INVALID, "ef_haar_set_cascade: feature " + std::to_string(i) +
                                              " has a rectangle outside the window (tilted features are not supported)");
        ++q.nr;
      }
    }
  }
  std::vector<HaarStage> st((size_t)n_stages);
  int first = 0;
  for (int s = 0; s < n_stages; ++s) {
    if (stage_count[s] < 1) return set_err(c, EF_E_INVALID, "ef_haar_set_cascade: empty stage");
    st[s] = HaarStage{first, stage_count[s], stage_threshold[s], 0};
    first += stage_count[s];
  }
  if (first != n_stumps) return set_err(c, EF_E_INVALID, "ef_haar_set_cascade: stage counts do not add up to n_stumps");
  std::vector<HaarStump> sp((size_t)n_stumps);
  for (int i = 0; i < n_stumps; ++i) {
    if (stump_feature[i] < 0 || stump_feature[i] >= n_features)
      return set_err(c, EF_E_INVALID, "ef_haar_set_cascade: stump feature index out of range");
    sp[i] = HaarStump{stump_feature[i], stump_threshold[i], stump_left[i], stump_right[i]};
  }
  // Can a stage's sum of leaf values (floats, accumulated in double) be formed in any
  // association?  Every value is a multiple of the smallest nonzero leaf's ulp u, so every
  // partial sum is too; if the sum of |leaf| maxima stays <= 2^53 u, every partial sum is
  // an exactly representable double and the order does not matter.
  bool order_free = true;
  for (int s = 0; s < n_stages && order_free; ++s) {
    double u = 0.0, bound = 0.0;
    for (int t = st[s].first; t < st[s].first + st[s].count; ++t) {
      const float lv[2] = {sp[t].left, sp[t].right};
      for (float v : lv) {
        if (!std::isfinite(v)) order_free = false;
        if (v == 0.f) continue;
        int e = 0;
        (void)std::frexp((double)v, &e);  // |v| in [2^(e-1), 2^e): float ulp 2^(e-24)
        const double ul = std::ldexp(1.0, e - 24);
        u = u == 0.0 ? ul : std::min(u, ul);
      }
      bound += std::max(std::fabs((double)sp[t].left), std::fabs((double)sp[t].right));
    }
    if (u > 0.0 && bound > std::ldexp(u, 53)) order_free = false;
  }
  EF_HIP(c, hipSetDevice(c->device), "hipSetDevice");
  haar_release(c);
  HaarState* h = new HaarState();
  c->haar = h;
  h->ww = win_w;
  h->wh = win_h;
  h->nstages = n_stages;
  h->order_free = order_free && !c->opt_haar_ordered;
  EF_TRY(ensure(c, h->stages, st.size() * sizeof(HaarStage)));
  EF_HIP(c, hipMemcpy(h->stages.p, st.data(), st.size() * sizeof(HaarStage), hipMemcpyHostToDevice), "H2D stages");
  std::vector<HaarRec> rc((size_t)n_stumps);
  for (int i = 0; i < n_stumps; ++i) {
    const HaarFeat& q = f[sp[i].feat];
    HaarRec& r = rc[i];
    r.thr = sp[i].thr, r.left = sp[i].left, r.right = sp[i].right, r.nr = q.nr, r.pad = 0;
    for (int k = 0; k < 3; ++k) r.x[k] = q.x[k], r.y[k] = q.y[k], r.w[k] = q.w[k], r.h[k] = q.h[k], r.wt[k] = q.wt[k];
    auto corner = [&](int rr, int k, int& cx, int& cy) {
      cx = r.x[rr] + ((k & 1) ? r.w[rr] : 0);
      cy = r.y[rr] + ((k & 2) ? r.h[rr] : 0);
    };
    for (int rr = 1; rr < 3; ++rr)
      for (int k = 0; k < 4; ++k) {
        int x1, y1;
        corner(rr, k, x1, y1);
        r.src[rr - 1][k] = -1;
        for (int m = 0; m < 4; ++m) {
          int x0, y0;
          corner(0, m, x0, y0);
          if (x0 == x1 && y0 == y1) {
            r.src[rr - 1][k] = (signed char)m;
            break;
          }
        }
      }
  }
  EF_TRY(ensure(c, h->recs, rc.size() * sizeof(HaarRec)));
  EF_HIP(c, hipMemcpy(h->recs.p, rc.data(), rc.size() * sizeof(HaarRec), hipMemcpyHostToDevice), "H2D records");
  return EF_OK;
}

int ef_haar_detect(ef_ctx* c, const uint8_t* gray, int32_t H, int32_t W, int64_t ld, double scale_factor,
                   int32_t min_neighbors, int32_t min_w, int32_t min_h, int32_t max_w, int32_t max_h,
                   int32_t* rects_out, int32_t max_rects, int32_t* n_rects, int32_t* cand_out, int32_t max_cand,
                   int32_t* n_cand, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  HaarState* h = static_cast<HaarState*>(c->haar);
  if (!h) return set_err(c, EF_E_STATE, "ef_haar_detect: call ef_haar_set_cascade first");
  if (!gray || H < 1 || W < 1 || ld < W || !(scale_factor > 1.0) || !n_rects || (max_rects > 0 && !rects_out))
    return set_err(c, EF_E_INVALID, "ef_haar_detect: bad arguments");
  EF_HIP(c, hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  const int mw = (max_w > 0 && max_h > 0) ? max_w : W, mh = (max_w > 0 && max_h > 0) ? max_h : H;
  // detectMultiScaleNoGrouping's scale list and FeatureEvaluator::updateScaleData's layers
  std::vector<HaarLayer> layers;
  std::vector<float> scales;
  for (double factor = 1.0;; factor *= scale_factor) {
    const int sw = cv_round(h->ww * factor), sh = cv_round(h->wh * factor);
    if (sw > mw || sh > mh) break;
    if (sw < min_w || sh < min_h) continue;
    scales.push_back((float)factor);
  }
  int64_t pix = 0, ii = 0, resn = 0;
  for (float sc : scales) {
    HaarLayer ly{};
    ly.w = cv_round((float)W / sc);
    ly.h = cv_round((float)H / sc);
    ly.nx = std::max(ly.w + 1 - h->ww, 0);
    ly.ny = std::max(ly.h + 1 - h->wh, 0);
    ly.step = sc >= 2.f ? 1 : 2;
    ly.scale = sc;
    ly.pix_off = pix;
    ly.ii_off = ii;
    ly.res_off = resn;
    pix += (int64_t)ly.w * ly.h;
    ii += (int64_t)(ly.w + 1) * (ly.h + 1);
    resn += (int64_t)ly.nx * ly.ny;
    if (ly.nx > 0 && ly.ny > 0) layers.push_back(ly);
  }
  *n_rects = 0;
  if (n_cand) *n_cand = 0;
  if (layers.empty()) return EF_OK;
  const int nl = (int)layers.size();
  if (nl > kHaarMaxLayers)
    return set_err(c, EF_E_INVALID, "ef_haar_detect: more than " + std::to_string(kHaarMaxLayers) +
                                        " pyramid layers (scale factor too close to 1)");
  std::vector<int> row_start(nl + 1, 0);
  for (int i = 0; i < nl; ++i) row_start[i + 1] = row_start[i] + (layers[i].ny + layers[i].step - 1) / layers[i].step;
  // candidate / work-list capacity: every window origin the invoker can visit (a 1080p
  // frame at minSize 30 has ~3.5 M; a cascade whose stage 0 passes most of them must not
  // overflow a fixed list)
  int64_t visitable = 0;
  for (const auto& ly : layers)
    visitable += (int64_t)((ly.nx + ly.step - 1) / ly.step) * ((ly.ny + ly.step - 1) / ly.step);
  if (visitable > INT_MAX / 2) return set_err(c, EF_E_INVALID, "ef_haar_detect: frame too large");
  const int cap = (int)std::max<int64_t>(visitable, 1024);
  EF_TRY(ensure(c, h->pix, pix));
  EF_TRY(ensure(c, h->ii1, ii * 4));
  EF_TRY(ensure(c, h->ii2, ii * 4));
  EF_TRY(ensure(c, h->res, std::max<int64_t>(resn, 16)));
  EF_TRY(ensure(c, h->vn, std::max<int64_t>(resn * 4, 16)));
  EF_TRY(ensure(c, h->layers, layers.size() * sizeof(HaarLayer)));
  EF_TRY(ensure(c, h->rowstart, row_start.size() * sizeof(int)));
  EF_TRY(ensure(c, h->work, (size_t)cap * sizeof(HaarCand)));
  EF_TRY(ensure(c, h->cand, (size_t)cap * sizeof(HaarCand)));
  EF_TRY(ensure(c, h->counters, 64));
  EF_TRY(ensure(c, h->desc, layers.size() * img_desc_size()));
  const uint8_t* src = gray;
  if (!(flags & EF_MEM_DEVICE) || ld != W) {
    EF_TRY(ensure(c, h->frame, (size_t)H * W));
    EF_HIP(c, hipMemcpy2DAsync(h->frame.p, W, gray, ld, W, H,
                               (flags & EF_MEM_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s),
           "frame");
    src = static_cast<const uint8_t*>(h->frame.p);
  }
  std::vector<char> desc(layers.size() * img_desc_size());
  int64_t max_out = 0;
  for (int i = 0; i < nl; ++i) {
    img_desc_fill(desc.data() + i * img_desc_size(), 0, layers[i].pix_off, H, W, 1, layers[i].h, layers[i].w);
    max_out = std::max<int64_t>(max_out, (int64_t)layers[i].w * layers[i].h);
  }
  EF_HIP(c, hipMemcpyAsync(h->desc.p, desc.data(), desc.size(), hipMemcpyHostToDevice, s), "H2D desc");
  EF_HIP(c, hipMemcpyAsync(h->layers.p, layers.data(), layers.size() * sizeof(HaarLayer), hipMemcpyHostToDevice, s),
         "H2D layers");
  EF_HIP(c, hipMemcpyAsync(h->rowstart.p, row_start.data(), row_start.size() * sizeof(int), hipMemcpyHostToDevice, s),
         "H2D rows");
  EF_HIP(c, hipMemsetAsync(h->counters.p, 0, 64, s), "memset");
  TimerEvt tev;
  timer_begin(c, EF_KERNEL_HAAR, &tev);
  EF_HIP(c, launch_resize_gray(s, src, h->desc.p, nl, max_out, static_cast<uint8_t*>(h->pix.p)), "pyramid");
  const HaarLayer* dl = static_cast<const HaarLayer*>(h->layers.p);
  int* ii1 = static_cast<int*>(h->ii1.p);
  unsigned* ii2 = static_cast<unsigned*>(h->ii2.p);
  int maxh = 0, maxw = 0;
  int64_t maxpos = 0;
  for (auto& ly : layers) {
    maxh = std::max(maxh, ly.h);
    maxw = std::max(maxw, ly.w);
    maxpos = std::max<int64_t>(maxpos, (int64_t)((ly.nx + ly.step - 1) / ly.step) * ((ly.ny + ly.step - 1) / ly.step));
  }
  const uint8_t* lp = static_cast<const uint8_t*>(h->pix.p);
  hipLaunchKernelGGL(haar_rows_ii_kernel, dim3((unsigned)((maxh + 1 + 3) / 4), (unsigned)nl), dim3(256), 0, s, lp, dl,
                     ii1, ii2);
  hipLaunchKernelGGL(haar_cols_ii_kernel, dim3((unsigned)((maxw + 1 + 63) / 64), (unsigned)nl), dim3(1024), 0, s, dl,
                     ii1, ii2);
  const HaarStage* dst = static_cast<const HaarStage*>(h->stages.p);
  const HaarRec* drc = static_cast<const HaarRec*>(h->recs.p);
  signed char* res = static_cast<signed char*>(h->res.p);
  hipLaunchKernelGGL(haar_stage0_kernel, dim3((unsigned)((maxpos + 255) / 256), (unsigned)nl), dim3(256), 0, s, dl, ii1,
                     ii2, dst, drc, h->ww, h->wh, res, static_cast<float*>(h->vn.p));
  int* cnt = static_cast<int*>(h->counters.p);
  HaarCand* work = static_cast<HaarCand*>(h->work.p);
  HaarCand* cand = static_cast<HaarCand*>(h->cand.p);
  hipLaunchKernelGGL(haar_rows_kernel, dim3((unsigned)((row_start[nl] + kHaarRowWaves - 1) / kHaarRowWaves)),
                     dim3(64 * kHaarRowWaves), 0, s, dl, nl,
                     static_cast<const int*>(h->rowstart.p), res, static_cast<const float*>(h->vn.p), work, cnt,
                     cap);
  int hc[16] = {0};
  EF_HIP(c, hipMemcpyAsync(hc, cnt, sizeof(int), hipMemcpyDeviceToHost, s), "D2H work count");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
  if (hc[0] > cap) return set_err(c, EF_E_INVALID, "ef_haar_detect: work-list capacity exceeded");
  // stage groups; the lists ping-pong between work and cand, counters cnt[g]
  // EF_HAAR_GROUPS="1,4,8,14" (experiments): first stage of each group, ascending, <= 14.
  // Default {1, 4, 8, 14} (tools/haar_groups.sh, 640x480 synthetic frontal cascade, ms per
  // frame): 1,3,6,10,15 0.532; 1,4,8,14 0.490; 1,6,12 0.487; 1,4,9 0.497; eleven or twelve
  // groups 0.61-0.64 — fewer, longer groups win until the dead lanes of a long group cost
  // more than a launch and a compaction.
  static const std::vector<int> groups = [] {
    std::vector<int> g;
#ifdef EF_DIAGNOSTICS
    if (const char* e = getenv("EF_HAAR_GROUPS")) {
      for (const char* p = e; *p;) {
        const int v = atoi(p);
        if (v >= 1 && (g.empty() || v > g.back()) && g.size() < 14) g.push_back(v);
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
      }
    }
#endif
    if (g.empty() || g[0] != 1) g = {1, 4, 8, 14};
    g.push_back(1 << 30);
    return g;
  }();
  // every group takes the split form when the cascade's stage sums are order-free
  // (measured, 640x480 synthetic frontal cascade with LDS stump records and 8 waves: split
  // from group 1 0.637 ms, from stage 3 0.652, from stage 6 0.673 per frame)
#ifdef EF_DIAGNOSTICS  // experiments: first split-form stage group, waves per split workgroup
  static const int kHaarSplitFrom = [] { const char* e = getenv("EF_HAAR_SPLIT_FROM"); return e ? atoi(e) : 1; }();
  static const int split_waves = [] {
    const char* e = getenv("EF_HAAR_SPLITW");
    const int v = e ? atoi(e) : 8;
    return v == 4 || v == 16 ? v : 8;
  }();
#else
  constexpr int kHaarSplitFrom = 1, split_waves = 8;
#endif
  int gi = 0;
  const int live = hc[0];  // upper bound of every group's input
  HaarCand* bin = work;
  HaarCand* bout = cand;
  for (; groups[gi] < h->nstages; ++gi) {
    const int s0 = groups[gi], s1 = std::min(groups[gi + 1], h->nstages);
    if (live > 0 && h->order_free && s0 >= kHaarSplitFrom) {
      const dim3 g((unsigned)((live + 63) / 64));
      if (split_waves == 16)
        hipLaunchKernelGGL(haar_cascade_split_kernel<16>, g, dim3(1024), 0, s, dl, ii1, ii2, dst, s0, s1, drc, h->ww,
                           h->wh, bin, cnt + gi, cap, bout, cnt + gi + 1);
      else if (split_waves == 8)
        hipLaunchKernelGGL(haar_cascade_split_kernel<8>, g, dim3(512), 0, s, dl, ii1, ii2, dst, s0, s1, drc, h->ww,
                           h->wh, bin, cnt + gi, cap, bout, cnt + gi + 1);
      else
        hipLaunchKernelGGL(haar_cascade_split_kernel<4>, g, dim3(256), 0, s, dl, ii1, ii2, dst, s0, s1, drc, h->ww,
                           h->wh, bin, cnt + gi, cap, bout, cnt + gi + 1);
    } else if (live > 0)
      hipLaunchKernelGGL(haar_cascade_kernel, dim3((unsigned)((live + 255) / 256)), dim3(256), 0, s, dl, ii1, ii2, dst,
                         s0, s1, drc, h->ww, h->wh, bin, cnt + gi, cap, bout, cnt + gi + 1);
    std::swap(bin, bout);
  }
  timer_end(c, &tev);
  EF_HIP(c, hipGetLastError(), "haar kernels");
  EF_HIP(c, hipMemcpyAsync(hc, cnt, 16 * sizeof(int), hipMemcpyDeviceToHost, s), "D2H counts");
  EF_HIP(c, hipStreamSynchronize(s), "sync");
#ifdef EF_DIAGNOSTICS
  if (getenv("EF_HAAR_DEBUG")) {
    fprintf(stderr, "[ef_haar] stage-group inputs:");
    for (int g = 0; g <= gi; ++g) fprintf(stderr, " %d", hc[g]);
    fprintf(stderr, "\n");
  }
#endif
  hc[1] = hc[gi];  // survivors of the last group (all of stage 0's when the cascade has 1 stage)
  cand = bin;
  if (hc[1] > cap) return set_err(c, EF_E_INVALID, "ef_haar_detect: candidate capacity exceeded");
  std::vector<HaarCand> hcand((size_t)hc[1]);
  if (hc[1] > 0)
    EF_HIP(c, hipMemcpy(hcand.data(), cand, hcand.size() * sizeof(HaarCand), hipMemcpyDeviceToHost), "D2H cand");
  // OpenCV's order: scale, then y, then x
  std::sort(hcand.begin(), hcand.end(), [](const HaarCand& a, const HaarCand& b) {
    return a.layer != b.layer ? a.layer < b.layer : (a.y != b.y ? a.y < b.y : a.x < b.x);
  });
  std::vector<RectI> rects;
  rects.reserve(hcand.size());
  for (const HaarCand& q : hcand) {
    const float sc = layers[q.layer].scale;
    rects.push_back(RectI{(int)std::lrint((float)q.x * sc), (int)std::lrint((float)q.y * sc),
                          cv_round(h->ww * sc), cv_round(h->wh * sc)});
  }
  if (n_cand) *n_cand = (int32_t)rects.size();
  if (cand_out)
    for (int i = 0; i < (int)rects.size() && i < max_cand; ++i) {
      cand_out[4 * i] = rects[i].x, cand_out[4 * i + 1] = rects[i].y;
      cand_out[4 * i + 2] = rects[i].w, cand_out[4 * i + 3] = rects[i].h;
    }
  const std::vector<RectI> g = group_rectangles(rects, min_neighbors, 0.2);
  *n_rects = (int32_t)g.size();
  for (int i = 0; i < (int)g.size() && i < max_rects; ++i) {
    rects_out[4 * i] = g[i].x, rects_out[4 * i + 1] = g[i].y, rects_out[4 * i + 2] = g[i].w, rects_out[4 * i + 3] = g[i].h;
  }
  return EF_OK;
}

}  // extern "C"
