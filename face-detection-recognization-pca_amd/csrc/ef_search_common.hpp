// Device helpers shared by the search kernels (ef_search.hip, ef_search_wide.hip).
#pragma once

#include "ef_dma.hpp"
#include "ef_internal.hpp"

namespace ef {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ long long pack_key(float v, unsigned idx) {
  if (v == 0.0f) v = 0.0f;  // canonical +0 so that -0 and +0 tie on index
  int b = __float_as_int(v);
  int s = b >= 0 ? b : (b ^ 0x7FFFFFFF);
  return (long long)(((unsigned long long)(unsigned)s << 32) | (unsigned long long)idx);
}
__device__ __forceinline__ float key_value(long long key) {
  const int s = (int)(key >> 32);
  return __int_as_float(s >= 0 ? s : (s ^ 0x7FFFFFFF));
}


// fp64 score of gallery row `row` for probe q (L2: squared distance in difference form;
// cosine: -q.g/(|q||g|), 0 for a zero vector — sklearn normalize semantics).
// KP = 0: the row length is kp_rt (k > 512, any multiple of 128).
template <int KP, int METRIC>
__device__ __forceinline__ double score64(const float* __restrict__ q, const float* __restrict__ g, int lane,
                                          int kp_rt = KP) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  auto term = [&](int c) {
    const double qv = q[c], gv = g[c];
    if constexpr (METRIC == EF_METRIC_L2) {
      const double dv = qv - gv;
      s0 = fma(dv, dv, s0);
    } else {
      s0 = fma(qv, gv, s0);
      s1 = fma(qv, qv, s1);
      s2 = fma(gv, gv, s2);
    }
  };
  if constexpr (KP > 0) {
#pragma unroll
    for (int c = lane; c < KP; c += 64) term(c);
  } else {
    for (int c = lane; c < kp_rt; c += 64) term(c);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off);
    if constexpr (METRIC != EF_METRIC_L2) {
      s1 += __shfl_xor(s1, off);
      s2 += __shfl_xor(s2, off);
    }
  }
  if constexpr (METRIC == EF_METRIC_L2) {
    return s0;
  } else {
    return (s1 > 0.0 && s2 > 0.0) ? -(s0 / (sqrt(s1) * sqrt(s2))) : 0.0;
  }
}

// Wide search (KP in {256, 512}, or KP = 0 with a run-time row length kp > 512, a
// multiple of 128): probes streamed through LDS with the gallery.
constexpr int kWideRowTile = 128;    // gallery rows per tile
constexpr int kWideProbeTile = 128;  // probes per workgroup
constexpr int kWide3RowTile = 256;    // split-bf16 wide kernel: gallery rows per tile
constexpr int kWide3ProbeTile = 256;  // split-bf16 wide kernel: probes per workgroup
// s3: qpad and G are the split-bf16 copies (split-bf16 scan); 1 = the 16x16x32 kernel,
// 2 = the 32x32x16 one (EF_OPT_SEARCH_SPLIT_BF16), 0 = the fp32 scan
hipError_t launch_search_wide(hipStream_t s, int kp, int metric, bool collect, int s3, const SearchPlan& pl,
                              const float* qpad, const float* G, const float* aux, int64_t n, int64_t bpad,
                              const SearchWs& ws);
// the single-bf16 screen's main pass with the gallery operand in VGPRs (ef_search_screen.hip;
// kh = k / 2 in {128, 256}); screen_vg_enabled: the product default (diagnostic A/B knob)
bool screen_vg_enabled();
hipError_t launch_search_screen(hipStream_t s, int kh, int metric, const SearchPlan& pl, const float* q1,
                                const float* G1, const float* aux, int64_t n, int64_t bpad, const SearchWs& ws);

}  // namespace ef
