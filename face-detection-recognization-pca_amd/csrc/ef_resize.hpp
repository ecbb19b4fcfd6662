// OpenCV 4.x resize arithmetic for CV_8U grey sources (shared by ef_image.hip's ragged
// resize and ef_jpeg.hip's fused decode -> grey -> resize): INTER_LINEAR as resizeGeneric_
// computes it (11-bit coefficients from float32 offsets, horizontal int sums, vertical
// ((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2), plus the identity copy and the exact-2x
// INTER_AREA shortcut.  Restated in oracle/image_oracle.py.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ef {

// One axis of OpenCV's INTER_LINEAR setup (resizeGeneric_): source pair and 11-bit
// weights.  Horizontal: borders clamp the index AND zero the fraction; vertical: only
// the source rows clamp.  Separate roundings as in the reference (no FMA contraction).
__device__ __forceinline__ void lin_axis(int dpos, int n_in, int n_out, bool zero_borders, int& i0, int& i1,
                                         int& c0, int& c1) {
  const double scale = __ddiv_rn(1.0, __ddiv_rn((double)n_out, (double)n_in));  // 1 / inv_scale
  float f = __double2float_rn(__dadd_rn(__dmul_rn(__dadd_rn((double)dpos, 0.5), scale), -0.5));
  int s = (int)floorf(f);
  f = __fsub_rn(f, (float)s);
  if (zero_borders) {
    if (s < 0) { f = 0.f; s = 0; }
    if (s >= n_in - 1) { f = 0.f; s = n_in - 1; }
  }
  c0 = __float2int_rn(__fmul_rn(__fsub_rn(1.f, f), 2048.f));
  c1 = __float2int_rn(__fmul_rn(f, 2048.f));
  i0 = s < 0 ? 0 : (s > n_in - 1 ? n_in - 1 : s);
  i1 = s + 1 < 0 ? 0 : (s + 1 > n_in - 1 ? n_in - 1 : s + 1);
}

// Output pixel (dy, dx) of an (oh, ow) resize of an (h, w) grey source read through
// gray(y, x).
template <class Gray>
__device__ __forceinline__ int resize_px(const Gray& gray, int h, int w, int oh, int ow, int dy, int dx) {
  if (oh == h && ow == w) return gray(dy, dx);  // dsize == ssize: copy
  if (h == 2 * oh && w == 2 * ow) {              // INTER_AREA fast path (exact 2x)
    const int y = 2 * dy, x = 2 * dx;
    return (gray(y, x) + gray(y, x + 1) + gray(y + 1, x) + gray(y + 1, x + 1) + 2) >> 2;
  }
  int x0, x1, a0, a1, y0, y1, b0, b1;
  lin_axis(dx, w, ow, true, x0, x1, a0, a1);
  lin_axis(dy, h, oh, false, y0, y1, b0, b1);
  const int d0 = gray(y0, x0) * a0 + gray(y0, x1) * a1;
  const int d1 = gray(y1, x0) * a0 + gray(y1, x1) * a1;
  const int v = (((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

}  // namespace ef
