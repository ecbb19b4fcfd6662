// Probe projection f = (p - mean) . W  (SURVEY.md K6).
//
// Replaces project_face_to_eigenspace (useless/scan.py:93-96) and the folded
// scaler.transform + pca.transform of extract_face_features (scan-template-v4.py:265-266),
// batched over B probes.  uint8 pixels are converted and mean-subtracted while they are
// staged into LDS (the centred matrix is never materialised in HBM).
//
// GEMM M=B probes, N=KPW (64|128) components, K=d pixels on v_mfma_f32_32x32x2_f32.
// Workgroup tile 128 probes x KPW, BK=32 pixels per stage, double-buffered LDS with
// register-staged prefetch.  K is split over gridDim.y into fp32 partial slabs that a
// second kernel sums in a fixed order (deterministic) straight into the padded probe
// buffer the search kernel reads.
#include "ef_internal.hpp"

namespace ef {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = kProjRowTile;  // 128 probes
constexpr int BK = 32;            // pixels per stage
constexpr int SA = BK + 4;        // LDS row stride of the pixel tile (conflict-free b128 reads)

// KPW = columns of this workgroup's tile (64 | 128); ldw = total padded columns of W and of
// the partial slabs (KPW, or a multiple of 128 with gridDim.z = ldw / 128 column tiles).
// FAST (uint8 probes, d and the split a whole number of 32-pixel stages, 16-B aligned
// rows): every load in the main loop is unconditional — rows past b read row b - 1 and are
// zeroed at conversion, the prefetch after the last stage re-reads it — so the loop has no
// branches and the compiler's vmcnt accounting stays exact (a load under a branch made it
// wait for every load in flight; the generic form also carries the per-element fallback).
template <int KPW, int PDT, bool VEC, bool FAST = false>
__global__ __launch_bounds__(256, 2) void project_kernel(const void* __restrict__ Pv, int64_t b,
                                                         int64_t d, const float* __restrict__ mu,
                                                         const float* __restrict__ W, int ldw,
                                                         float* __restrict__ part, int64_t bpad,
                                                         int64_t pix_per_split) {
  constexpr int WAVES_M = KPW == 128 ? 2 : 4;
  constexpr int RW = BM / WAVES_M;            // rows per wave (64 | 32)
  constexpr int AB = RW / 32;                 // A blocks per wave
  constexpr int CW = KPW / (4 / WAVES_M);     // cols per wave (64)
  constexpr int BB = CW / 32;                 // B blocks per wave
  constexpr int SW = KPW;                     // LDS row stride of the W tile
  constexpr int W4 = BK * KPW / 4;            // float4s per W tile
  constexpr int W4_PT = W4 / 256;

  __shared__ __attribute__((aligned(16))) float sA[2][BM * SA];
  __shared__ __attribute__((aligned(16))) float sW[2][BK * SW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, c32 = lane & 31;
  const int wm = wave / (4 / WAVES_M), wn = wave % (4 / WAVES_M);
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int col0 = blockIdx.z * KPW;
  const int64_t k_beg = (int64_t)blockIdx.y * pix_per_split;
  int64_t k_end = k_beg + pix_per_split;
  if (k_end > d) k_end = d;
  const int nsteps = (int)((k_end - k_beg + BK - 1) / BK);

  // pixel staging: thread -> (row, 16-pixel half).  load_stage only issues the global
  // loads (raw pixels, mean, W) into registers; the uint8 -> float conversion and the mean
  // subtraction happen in store_stage, after the stage's MFMAs, so the loads' latency is
  // hidden under them instead of being waited for before the first MFMA.
  const int pr = tid >> 1, ph = (tid & 1) * 16;
  float pv[16];
  float muv[16];
  uint4 raw = make_uint4(0u, 0u, 0u, 0u);
  bool raw_ok = false;
  float4 wv[W4_PT];

  const bool row_ok = m0 + pr < b;
  auto load_stage = [&](int step) {
    const int64_t kb = k_beg + (int64_t)step * BK;
    const int64_t row = m0 + pr;
    const int64_t px0 = kb + ph;
    const bool full = VEC && row < b && px0 + 16 <= k_end;
    if constexpr (PDT == EF_U8) {
      const uint8_t* P = reinterpret_cast<const uint8_t*>(Pv);
      raw_ok = full;
      if (full) {
        raw = *reinterpret_cast<const uint4*>(P + row * d + px0);
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          pv[j] = (row < b && px0 + j < k_end) ? (float)P[row * d + px0 + j] : 0.f;
      }
    } else {
      const float* P = reinterpret_cast<const float*>(Pv);
      if (full) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 v = *reinterpret_cast<const float4*>(P + row * d + px0 + 4 * j);
          pv[4 * j] = v.x; pv[4 * j + 1] = v.y; pv[4 * j + 2] = v.z; pv[4 * j + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) pv[j] = (row < b && px0 + j < k_end) ? P[row * d + px0 + j] : 0.f;
      }
    }
    // mean of this thread's 16 pixels (0 on padded rows / pixels, which stay 0)
    if (full) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 m = *reinterpret_cast<const float4*>(mu + px0 + 4 * j);
        muv[4 * j] = m.x; muv[4 * j + 1] = m.y; muv[4 * j + 2] = m.z; muv[4 * j + 3] = m.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) muv[j] = (row < b && px0 + j < k_end) ? mu[px0 + j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < W4_PT; ++j) {
      const int idx = tid + 256 * j;
      const int kr = idx / (KPW / 4), c4 = idx % (KPW / 4);
      const int64_t px = kb + kr;
      wv[j] = px < k_end ? reinterpret_cast<const float4*>(W + px * ldw + col0)[c4]
                         : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_stage = [&](int buf) {
    if constexpr (PDT == EF_U8) {
      if (raw_ok) {
        const unsigned w4[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) pv[j] = (float)((w4[j >> 2] >> (8 * (j & 3))) & 0xffu);
      }
    }
    // mean subtraction fused into the operand staging (K2)
#pragma unroll
    for (int j = 0; j < 16; ++j) pv[j] -= muv[j];
    float* a = &sA[buf][pr * SA + ph];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<float4*>(a + 4 * j) = make_float4(pv[4 * j], pv[4 * j + 1], pv[4 * j + 2], pv[4 * j + 3]);
#pragma unroll
    for (int j = 0; j < W4_PT; ++j) {
      const int idx = tid + 256 * j;
      const int kr = idx / (KPW / 4), c4 = idx % (KPW / 4);
      *reinterpret_cast<float4*>(&sW[buf][kr * SW + c4 * 4]) = wv[j];
    }
  };

  // FAST forms (no branch, no per-element fallback); the staged registers are a value
  // (FastRaw) rather than the captured arrays, which the compiler kept in scratch here
  struct FastRaw {
    uint4 raw;
    float4 mu[4];
    float4 w[W4_PT];
  };
  auto load_fast = [&](int step) {
    FastRaw r;
    const int64_t kb = k_beg + (int64_t)step * BK;
    const int64_t px0 = kb + ph;
    const uint8_t* P = reinterpret_cast<const uint8_t*>(Pv);
    r.raw = *reinterpret_cast<const uint4*>(P + (row_ok ? m0 + pr : b - 1) * d + px0);
#pragma unroll
    for (int j = 0; j < 4; ++j) r.mu[j] = *reinterpret_cast<const float4*>(mu + px0 + 4 * j);
#pragma unroll
    for (int j = 0; j < W4_PT; ++j) {
      const int idx = tid + 256 * j;
      const int kr = idx / (KPW / 4), c4 = idx % (KPW / 4);
      r.w[j] = reinterpret_cast<const float4*>(W + (kb + kr) * ldw + col0)[c4];
    }
    return r;
  };
  auto store_fast = [&](const FastRaw& r, int buf) {
    const unsigned w4[4] = {r.raw.x, r.raw.y, r.raw.z, r.raw.w};
    float* a = &sA[buf][pr * SA + ph];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned u = w4[j];
      const float4 m = r.mu[j];
      const float4 v = row_ok ? make_float4((float)(u & 0xffu) - m.x, (float)((u >> 8) & 0xffu) - m.y,
                                            (float)((u >> 16) & 0xffu) - m.z, (float)(u >> 24) - m.w)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(a + 4 * j) = v;
    }
#pragma unroll
    for (int j = 0; j < W4_PT; ++j) {
      const int idx = tid + 256 * j;
      const int kr = idx / (KPW / 4), c4 = idx % (KPW / 4);
      *reinterpret_cast<float4*>(&sW[buf][kr * SW + c4 * 4]) = r.w[j];
    }
  };

  f32x16 acc[AB][BB];
#pragma unroll
  for (int i = 0; i < AB; ++i)
#pragma unroll
    for (int j = 0; j < BB; ++j) acc[i][j] = f32x16{};

  if (nsteps > 0) {
    if constexpr (FAST) {
      store_fast(load_fast(0), 0);
    } else {
      load_stage(0);
      store_stage(0);
    }
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const bool more = st + 1 < nsteps;  // (FAST: the last prefetch re-reads the last stage)
    FastRaw fr;
    if constexpr (FAST)
      fr = load_fast(st + 1 < nsteps ? st + 1 : st);
    else if (more)
      load_stage(st + 1);
    // the next stage's loads issue before this stage's MFMAs (the scheduler would sink
    // them next to the stores and wait out their latency there)
    if constexpr (FAST) __builtin_amdgcn_sched_barrier(0);
    // k permutation inside the stage: lane half h owns pixels [16h, 16h+16)
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 4) {
      float4 a[AB];
#pragma unroll
      for (int i = 0; i < AB; ++i)
        a[i] = *reinterpret_cast<const float4*>(&sA[buf][(wm * RW + i * 32 + c32) * SA + 16 * h + s4]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float bv[BB];
#pragma unroll
        for (int j = 0; j < BB; ++j) bv[j] = sW[buf][(16 * h + s4 + e) * SW + wn * CW + j * 32 + c32];
#pragma unroll
        for (int i = 0; i < AB; ++i) {
          const float av = e == 0 ? a[i].x : e == 1 ? a[i].y : e == 2 ? a[i].z : a[i].w;
#pragma unroll
          for (int j = 0; j < BB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    // (and their conversion stays after the MFMAs: hoisted above them it waits for the loads)
    if constexpr (FAST) __builtin_amdgcn_sched_barrier(0);
    if constexpr (FAST)
      store_fast(fr, buf ^ 1);
    else if (more)
      store_stage(buf ^ 1);
    __syncthreads();
  }

  // partial slab [split][bpad][KPW]; col = lane&31, row = (r&3) + 8(r>>2) + 4h
  float* out = part + (int64_t)blockIdx.y * bpad * ldw + col0;
#pragma unroll
  for (int i = 0; i < AB; ++i)
#pragma unroll
    for (int j = 0; j < BB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * RW + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wn * CW + j * 32 + c32;
        out[row * ldw + col] = acc[i][j][r];
      }
}

// qpad[row][c] = sum_z part[z][row][c] (c < kp, rows < bpad; fixed z order);
// f_out[row][c] for row < b, c < k when requested.
// corr (bf16 model only): per-column correction subtracted after the sum.
__global__ void project_reduce_kernel(const float* __restrict__ part, int nsplit, int64_t b,
                                      int64_t bpad, int kpw, int k, int kp, const float* __restrict__ corr,
                                      float* __restrict__ qpad, float* __restrict__ f_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= bpad * kp) return;
  const int64_t row = i / kp;
  const int c = (int)(i - row * kp);
  float s = 0.f;
  if (row < b && c < k)
  {
    for (int z = 0; z < nsplit; ++z) s += part[((int64_t)z * bpad + row) * kpw + c];
    if (corr) s -= corr[c];
  }
  qpad[i] = s;
  if (f_out && row < b && c < k) f_out[row * k + c] = s;
}

int project_nsplit(int64_t bpad, int64_t d, int kpw, int64_t* pix_per_split) {
  const int64_t mtiles = bpad / BM * (kpw > 128 ? kpw / 128 : 1);
  int64_t ns = (512 + mtiles - 1) / mtiles;  // ~2 workgroups per CU
  const int64_t steps = (d + BK - 1) / BK;
  if (ns > steps) ns = steps;
  if (ns < 1) ns = 1;
  if (ns > 64) ns = 64;
  const int64_t steps_per = (steps + ns - 1) / ns;
  *pix_per_split = steps_per * BK;
  return (int)((d + *pix_per_split - 1) / *pix_per_split);
}

template <int KPW, int PDT>
static hipError_t proj_t(hipStream_t s, const void* P, int64_t b, int64_t bpad, int64_t d,
                         const float* mean, const float* W, int ldw, float* part, int nsplit, int64_t pps) {
  const dim3 grid((unsigned)(bpad / BM), (unsigned)nsplit, (unsigned)(ldw / KPW));
  const bool vec = (d % 16 == 0) && ((reinterpret_cast<uintptr_t>(P) & 15) == 0) && (pps % 16 == 0);
  bool fast = PDT == EF_U8 && vec && d % BK == 0 && pps % BK == 0 && b >= 1;
#ifdef EF_DIAGNOSTICS  // EF_PROJ_FAST=0: the generic kernel (A/B)
  if (const char* e = getenv("EF_PROJ_FAST")) fast = fast && atoi(e) != 0;
#endif
  if (fast)
    hipLaunchKernelGGL((project_kernel<KPW, PDT, true, true>), grid, dim3(256), 0, s, P, b, d, mean, W, ldw, part,
                       bpad, pps);
  else if (vec)
    hipLaunchKernelGGL((project_kernel<KPW, PDT, true>), grid, dim3(256), 0, s, P, b, d, mean, W, ldw, part,
                       bpad, pps);
  else
    hipLaunchKernelGGL((project_kernel<KPW, PDT, false>), grid, dim3(256), 0, s, P, b, d, mean, W, ldw,
                       part, bpad, pps);
  return hipGetLastError();
}

hipError_t launch_project(hipStream_t s, int kpw, int p_dtype, const void* P, int64_t b,
                          int64_t bpad, int64_t d, const float* mean, const float* W, float* part,
                          int nsplit, int64_t pps) {
  if (kpw == 64)
    return p_dtype == EF_U8 ? proj_t<64, EF_U8>(s, P, b, bpad, d, mean, W, kpw, part, nsplit, pps)
                            : proj_t<64, EF_F32>(s, P, b, bpad, d, mean, W, kpw, part, nsplit, pps);
  if (kpw % 128 == 0)
    return p_dtype == EF_U8 ? proj_t<128, EF_U8>(s, P, b, bpad, d, mean, W, kpw, part, nsplit, pps)
                            : proj_t<128, EF_F32>(s, P, b, bpad, d, mean, W, kpw, part, nsplit, pps);
  return hipErrorInvalidValue;
}

hipError_t launch_project_reduce(hipStream_t s, const float* part, int nsplit, int64_t b,
                                 int64_t bpad, int kpw, int k, int kp, const float* corr, float* qpad,
                                 float* f_out) {
  const int64_t tot = bpad * kp;
  hipLaunchKernelGGL(project_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, part,
                     nsplit, b, bpad, kpw, k, kp, corr, qpad, f_out);
  return hipGetLastError();
}

}  // namespace ef
