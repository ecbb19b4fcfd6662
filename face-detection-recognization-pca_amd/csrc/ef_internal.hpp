// Internal declarations shared by the libeigenface translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../../include/eigenface.h"

namespace ef {

// ---- padded widths ------------------------------------------------------------------
// Gallery / probe features are stored with k zero-padded to KP in {16,32,64,128,256,512},
// beyond 512 to a multiple of 128 (zero padding is exact for dot products and distances).
// k > 512 arises from full-rank per-person models (train-v5.py:539-545 sets
// n_components = face count).  The search kernels address a probe row with a 32-bit byte
// offset, so a launch covers at most 2^31 / (4 KP) probes (longer batches run in pieces).
constexpr int kMaxFeatureK = 1 << 16;
inline int feature_pad(int k) {
  if (k <= 16) return 16;
  if (k <= 32) return 32;
  if (k <= 64) return 64;
  if (k <= 128) return 128;
  if (k <= 256) return 256;
  if (k <= 512) return 512;
  if (k <= kMaxFeatureK) return (k + 127) / 128 * 128;
  return -1;
}
// The projection GEMM writes KPW = 64 or a multiple of 128 columns (128-column tiles).
inline int proj_pad(int kp) { return kp <= 64 ? 64 : (kp + 127) / 128 * 128; }

constexpr int kSearchProbeTile = 256;   // probes per search workgroup (4 waves x 64)
constexpr int kProjRowTile = 128;       // probes per projection workgroup
constexpr int kJacobiMax = 88;          // largest (even) order the LDS Jacobi handles
constexpr int kCandMax = 32;            // fp64 re-rank candidates kept per ambiguous probe

// Workspace of one search call (device pointers).
struct SearchWs {
  long long* part_key;  // [nchunks][bpad] best (score, row) per chunk
  float* part_b2;       // [nchunks][bpad] runner-up score per chunk
  int* amb_count;       // probes queued for fp64 resolution
  int* amb_list;        // [bpad] probe of each queued slot
  float* thr;           // [bpad] fp32 score threshold of each slot
  int* cand;            // [bpad][kCandMax] candidate rows
  int* cand_cnt;        // [bpad]
  ef_match* match;      // [b] exact merge records (fp64 winner score), may be null
};

struct SearchPlan {
  int n_ptiles = 0, nchunks = 0, tiles_per_chunk = 0;
  // wide kernel: (chunk, probe tile) pairs are dealt to XCDs in blocks of cblk chunks x
  // pblk probe tiles, so one XCD's L2 holds pblk probe tiles instead of all of them
  int pblk = 0, cblk = 1;
  // collect pass (queued probes only): c_grid workgroups stride over (c_chunks chunks of
  // c_tpc tiles) x (queued probe tiles) items
  int c_chunks = 1, c_tpc = 1, c_grid = 8;
};

// one launch of a (possibly piecewise) search: probes [off, off + b), launched and planned
// with bpad = round_up(b, 256) rows (ef_api.hip search_pieces)
struct SearchPiece {
  int64_t off, b, bpad;
};

// ---- device buffer ------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct TimerEvt {
  hipEvent_t a, b;
  int kernel;
};

}  // namespace ef

struct ef_ctx {
  int device = 0;
  // tunables set with ef_set_option (include/eigenface.h EF_OPT_*)
  int64_t opt_fit_max_iters = 500;
  int64_t opt_fit_fp32_coarse = 1;
  int64_t opt_cov_slab_bytes = (int64_t)8 << 30;
  int64_t opt_tm_int64 = 0;
  int64_t opt_haar_ordered = 0;
  int64_t opt_jpeg_chunk_bits = 0;
  int64_t opt_search_split_bf16 = 0;
  int g3_layout = 0;  // what G3 holds: 1 split (hi + lo) rows, 3 single-bf16 rows
  int64_t opt_jpeg_part_files = 8192;
  int64_t opt_fit_chebyshev = 1;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;

  // recognition model (p - mean) . W
  int64_t d = 0;
  int k = 0, kp = 0, kpw = 0;
  ef::DevBuf mean;  // float[d]
  ef::DevBuf W;     // float[d][kpw]
  bool bf16 = false;   // EF_MODEL_BF16: project with W16 on bf16 MFMA
  ef::DevBuf W16;      // bf16[kpw][d]
  ef::DevBuf W16f;     // W16 in MFMA-fragment order (frag-form projection), when supported
  bool w16f_ok = false;
  ef::DevBuf mean_r;   // float[d] round(mean)
  ef::DevBuf mean_u8;  // uint8[d] round(mean) (wide bf16 kernel) + int counter
  bool mean_u8_ok = false;  // every round(mean) in 0..255
  ef::DevBuf corr;     // float[kpw] (mean - round(mean)).W

  // gallery
  int64_t n_gallery = 0, g_offset = 0;
  int g_k = 0, g_kp = 0;
  ef::DevBuf G;      // float[n][g_kp]
  ef::DevBuf gnorm2; // float[n]  ||g||^2
  ef::DevBuf ginv;   // float[n]  1/||g|| (0 for a zero row)
  ef::DevBuf gmax2;  // uint (float bits) max ||g||^2
  ef::DevBuf G3;     // split-bf16 copy of G (same bytes), built on the first split search
  bool g3_valid = false;
  float gmax2_host = 0.f;

  // per-call scratch (grown on demand, never shrunk)
  ef::DevBuf q_pad;     // float[bpad][kp]
  ef::DevBuf q3;        // split-bf16 probes [bpad][kp] (wide split-bf16 scans)
  ef::DevBuf keys;      // int64[bpad]
  ef::DevBuf search_ws; // SearchWs carve-out
  ef::DevBuf p_stage;   // probe pixels staged from host
  ef::DevBuf proj_part; // float[nsplit][bpad][kpw]
  ef::DevBuf feats_dev; // float[b][k] staging for host output

  std::vector<ef::DevBuf> fit_pool;  // ef_fit workspaces, reused across calls (ef_trim frees)

  // JPEG decode (ef_jpeg.hip): device workspace, host-output staging, and two upload slots
  // (a pinned host buffer + its device copy each): the host stages batch i + 1 into one slot
  // — the next part of a call, or the next call — while the device decodes batch i from
  // the other.  up_done[s]: the upload that last read pinned slot s (copy stream);
  // ws_free[s]: the last kernel that read device slot s (compute stream); done: the last
  // decode's kernels (a call on another stream, or a reallocation, waits for it).
  ef::DevBuf jpeg_ws, jpeg_out, jpeg_rows;
  ef::DevBuf jpeg_up[2];
  void* jpeg_pinned[2] = {nullptr, nullptr};
  size_t jpeg_pinned_bytes[2] = {0, 0};
  hipEvent_t jpeg_up_done[2] = {nullptr, nullptr};
  hipEvent_t jpeg_ws_free[2] = {nullptr, nullptr};
  hipEvent_t jpeg_done = nullptr;
  hipStream_t jpeg_copy = nullptr;  // upload stream (created on first use)
  // the fit's side stream (created on first use): work off the critical path of the
  // subspace iteration, e.g. the int8 digit planes of C during the coarse phase
  hipStream_t fit_side = nullptr;
  hipEvent_t fit_side_ev[2] = {nullptr, nullptr};
  // the template localiser's side stream (created on first use): the integral images' column
  // pass runs beside the correlation kernel
  hipStream_t tm_side = nullptr;
  hipEvent_t tm_side_ev[2] = {nullptr, nullptr};
  int jpeg_slot = 0;                // slot of the next staged batch

  void* tm = nullptr;    // template-localiser state (ef_image.hip TmState), ef_tm_prepare
  void* haar = nullptr;  // Haar cascade state (ef_haar.hip HaarState), ef_haar_set_cascade

  // multi-GPU: RCCL communicator (ef_comm_init), null when single-rank
  void* comm = nullptr;
  int comm_size = 1, comm_rank = 0;
  ef::DevBuf match_local;  // ef_match[b] this rank's records
  ef::DevBuf match_all;    // ef_match[comm_size][b] gathered records
  ef::DevBuf q_local;      // float[cpad][kp] this rank's slice of the projected probes

  bool timing = false;
  std::vector<ef::TimerEvt> pending;
  double t_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t t_n[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

namespace ef {

int set_err(ef_ctx* c, int code, const std::string& msg);
void tm_release(ef_ctx* c);
void haar_release(ef_ctx* c);
int hip_err(ef_ctx* c, hipError_t e, const char* what);
int ensure(ef_ctx* c, DevBuf& b, size_t bytes);
void release(DevBuf& b);
void timer_begin(ef_ctx* c, int kernel, TimerEvt* t);
void timer_end(ef_ctx* c, TimerEvt* t);
// events created but not recorded: the launcher records them itself around the kernels
// (t->kernel < 0 when timing is off); timer_commit queues them for ef_timing_get
void timer_arm(ef_ctx* c, int kernel, TimerEvt* t);
void timer_commit(ef_ctx* c, TimerEvt* t);

// ---- launchers (defined in the .hip files) -------------------------------------------
SearchPlan search_plan(int64_t bpad, int64_t n, int kp, bool s3);
std::vector<SearchPiece> search_pieces(int64_t b, int kp);
// G3: split-bf16 copy of G (EF_OPT_SEARCH_SPLIT_BF16) or null for the fp32 kernels; Q3: scratch
// [bpad][kp] for the split probes (kp > 128 with G3 only)
hipError_t launch_search(hipStream_t s, int kp, int metric, const SearchPlan& pl, const float* qpad, float* Q3,
                         int64_t bpad, int64_t b, const float* G, const float* G3, const float* aux, int64_t n,
                         int64_t g_offset, float gmax2, const SearchWs& ws, long long* keys, ef_ctx* c);
hipError_t launch_split_rows(hipStream_t s, const float* G, int64_t n, int kp, void* out);
// single-bf16 copy for the bf16 screen (EF_OPT_SEARCH_SPLIT_BF16 = 3), kp % 64 == 0
hipError_t launch_hi_rows(hipStream_t s, const float* G, int64_t n, int kp, void* out);
hipError_t launch_keys_none(hipStream_t s, long long* keys, int64_t b, ef_match* match);
// keys[b] (+ merged[b]) <- exact arg-best over parts x b match records (ef_comm.hip)
hipError_t launch_matches_merge(hipStream_t s, const ef_match* parts, int nparts, int64_t b, long long* keys,
                                ef_match* merged);
void comm_release(ef_ctx* c);
// ragged resize (ef_image.hip) from device descriptors written by img_desc_fill: the Haar
// pyramid and the JPEG ingest (BGR order for 3-channel sources)
hipError_t launch_resize_gray(hipStream_t s, const uint8_t* src, const void* desc_dev, int count, int64_t max_out,
                              uint8_t* dst);
size_t img_desc_size();
void img_desc_fill(void* d, int64_t src_off, int64_t dst_off, int h, int w, int c, int oh, int ow);
// wait for every queued JPEG upload and decode of the context (ef_jpeg.hip)
hipError_t jpeg_quiesce(ef_ctx* c);
// hipFuncSetAttribute(fn, MaxDynamicSharedMemorySize, bytes) once per (kernel, device),
// thread-safe (several contexts may launch the same kernel on different devices)
hipError_t allow_dynamic_lds(const void* fn, int bytes);

// Runs fn(0) .. fn(n - 1) on a process-wide pool of host worker threads (created once, at
// most 15, plus the calling thread, which takes tasks too) and returns when all are done.
// Jobs from concurrent callers run one at a time.  Spawning threads per call cost ~1-2 ms
// per 16 threads in the sandboxed containers, as much as the host work it split.
void host_parallel(int n, const std::function<void(int)>& fn);
int host_threads();  // EF_OPT_HOST_THREADS (the job's CPU share)
// all-gather over the attached communicator on ctx->stream (bytes per rank)
int comm_allgather(ef_ctx* c, const void* send, void* recv, size_t bytes_per_rank);
hipError_t launch_pad_rows(hipStream_t s, const float* src, int64_t rows, int k, int64_t rows_pad,
                           float* dst, int kp);
hipError_t launch_gallery_aux(hipStream_t s, const float* G, int64_t n, int kp, float* gnorm2,
                              float* ginv, unsigned* gmax2_bits);

hipError_t launch_project(hipStream_t s, int kpw, int p_dtype, const void* P, int64_t b,
                          int64_t bpad, int64_t d, const float* mean, const float* W,
                          float* part, int nsplit, int64_t pix_per_split);
int project_nsplit(int64_t bpad, int64_t d, int kpw, int64_t* pix_per_split);
hipError_t launch_project_reduce(hipStream_t s, const float* part, int nsplit, int64_t b,
                                 int64_t bpad, int kpw, int k, int kp, const float* corr, float* qpad,
                                 float* f_out);
// bf16 model (EF_MODEL_BF16): W16 [kpw][d] bf16, round(mean), fp64-derived correction row
hipError_t launch_bf16_model(hipStream_t s, const float* W, const float* mean, int64_t d, int ldw,
                             unsigned short* Wt16, float* mean_r, float* corr, double* corr_part, int nchunk);
int project_bf16_nsplit(int p_dtype, const void* P, const uint8_t* mean_u8, const void* Wf, int64_t bpad, int64_t d,
                        int ldw, int64_t* pix_per_split);
hipError_t launch_project_bf16(hipStream_t s, int p_dtype, const void* P, int64_t b, int64_t bpad, int64_t d,
                               const float* mean_r, const uint8_t* mean_u8, const unsigned short* Wt16,
                               const void* Wf, int ldw, float* part, int nsplit, int64_t pps);
// fragment-native copy of W16 for the frag-form projection (d % 64 == 0, ldw % 128 == 0)
bool bf16_frag_supported(int64_t d, int ldw);
hipError_t launch_bf16_frag(hipStream_t s, const unsigned short* Wt16, int64_t d, int ldw, void* Wf);
hipError_t launch_mean_u8(hipStream_t s, const float* mean_r, int64_t d, uint8_t* out, int* bad);

}  // namespace ef
