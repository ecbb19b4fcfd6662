// C ABI: context, recognition model, gallery, search, timing (include/eigenface.h).
#include <climits>
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <set>
#include <utility>
#include <vector>

#include "ef_internal.hpp"

#include <atomic>

namespace ef {

int set_err(ef_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_err(ef_ctx* c, hipError_t e, const char* what) {
  return set_err(c, e == hipErrorOutOfMemory ? EF_E_NOMEM : EF_E_HIP,
                 std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(ef_ctx* c, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return EF_OK;
  release(b);
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) {
    b.p = nullptr;
    b.bytes = 0;
    return hip_err(c, e, "hipMalloc");
  }
  b.bytes = bytes;
  return EF_OK;
}

void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

void timer_begin(ef_ctx* c, int kernel, TimerEvt* t) {
  t->kernel = -1;
  if (!c->timing) return;
  if (hipEventCreate(&t->a) != hipSuccess) return;
  if (hipEventCreate(&t->b) != hipSuccess) { (void)hipEventDestroy(t->a); return; }
  t->kernel = kernel;
  (void)hipEventRecord(t->a, c->stream);
}

void timer_arm(ef_ctx* c, int kernel, TimerEvt* t) {
  t->kernel = -1;
  if (!c->timing) return;
  if (hipEventCreate(&t->a) != hipSuccess) return;
  if (hipEventCreate(&t->b) != hipSuccess) { (void)hipEventDestroy(t->a); return; }
  t->kernel = kernel;
}

void timer_commit(ef_ctx* c, TimerEvt* t) {
  if (t->kernel >= 0) c->pending.push_back(*t);
}

void timer_end(ef_ctx* c, TimerEvt* t) {
  if (t->kernel < 0) return;
  (void)hipEventRecord(t->b, c->stream);
  c->pending.push_back(*t);
}

static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

#define EF_TRY(expr)                         \
  do {                                       \
    int _rc = (expr);                        \
    if (_rc != EF_OK) return _rc;            \
  } while (0)
#define EF_HIP(ctx, expr, what)                           \
  do {                                                    \
    hipError_t _e = (expr);                               \
    if (_e != hipSuccess) return hip_err(ctx, _e, what);  \
  } while (0)

// The pieces search_local launches for b probes of kp floats: whole 256-probe tiles, at
// most as many per piece as keep a probe row's byte offset below 2^31 (the kernels' 32-bit
// offsets).  Piece i covers probes [off, off + b) and is launched with bpad =
// round_up(b, 256) rows, and its plan is built from that same bpad — never from the
// caller's q_pad row count, which can be larger (the sharded projection pads
// R * ceil(b / R) rows): a plan whose probe-tile count differs from the launch's row count
// makes the kernels' part_key stride disagree between chunks.
std::vector<SearchPiece> search_pieces(int64_t b, int kp) {
  std::vector<SearchPiece> v;
  const int64_t row_bytes = (int64_t)kp * 4;
  const int64_t piece = std::max<int64_t>(kSearchProbeTile, ((int64_t)INT_MAX / row_bytes) / kSearchProbeTile * kSearchProbeTile);
  for (int64_t off = 0; off < b; off += piece) {
    const int64_t bi = std::min(piece, b - off);
    v.push_back(SearchPiece{off, bi, round_up(bi, kSearchProbeTile)});
  }
  return v;
}

// Search the probes already in ctx->q_pad (at least round_up(b, 256) rows, kp = ctx->g_kp)
// of this rank's gallery: keys_dev[b] and, when match_dev is non-null, the fp64 match
// records, piece by piece (search_pieces).
static int search_local(ef_ctx* c, int64_t bpad, int64_t b, int metric, long long* keys_dev, ef_match* match_dev) {
  if (c->n_gallery == 0) {
    EF_HIP(c, launch_keys_none(c->stream, keys_dev, b, match_dev), "keys");
    return EF_OK;
  }
  if (bpad < round_up(b, kSearchProbeTile))
    return set_err(c, EF_E_INVALID, "search: probe buffer shorter than the batch");
  const std::vector<SearchPiece> pieces = search_pieces(b, c->g_kp);
  std::vector<SearchPlan> plans;
  int64_t bpad_max = 0;
  size_t parts = 0;
  for (const SearchPiece& p : pieces) {
    // a shorter last piece's plan may have more chunks
    plans.push_back(search_plan(p.bpad, c->n_gallery, c->g_kp, c->opt_search_split_bf16 != 0));
    bpad_max = std::max(bpad_max, p.bpad);
    parts = std::max(parts, (size_t)plans.back().nchunks * (size_t)p.bpad);
  }
  // workspace carve-out (16-byte aligned pieces), sized for the largest piece
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t nkb = al(parts * 8), nb2 = al(parts * 4);
  const size_t ncnt = al(16), nlist = al((size_t)bpad_max * 4), nthr = al((size_t)bpad_max * 4);
  const size_t ncand = al((size_t)bpad_max * kCandMax * 4), ncc = al((size_t)bpad_max * 4);
  EF_TRY(ensure(c, c->search_ws, nkb + nb2 + ncnt + nlist + nthr + ncand + ncc));
  char* base = static_cast<char*>(c->search_ws.p);
  SearchWs ws;
  ws.part_key = reinterpret_cast<long long*>(base);
  base += nkb;
  ws.part_b2 = reinterpret_cast<float*>(base);
  base += nb2;
  ws.amb_count = reinterpret_cast<int*>(base);
  base += ncnt;
  ws.amb_list = reinterpret_cast<int*>(base);
  base += nlist;
  ws.thr = reinterpret_cast<float*>(base);
  base += nthr;
  ws.cand = reinterpret_cast<int*>(base);
  base += ncand;
  ws.cand_cnt = reinterpret_cast<int*>(base);
  const float* aux = static_cast<const float*>(metric == EF_METRIC_L2 ? c->gnorm2.p : c->ginv.p);
  const float* G3 = nullptr;
  float* Q3 = nullptr;
  if (c->opt_search_split_bf16) {  // split-bf16 scan
    if (c->g_kp > 128) {
      EF_TRY(ensure(c, c->q3, (size_t)bpad_max * c->g_kp * sizeof(float)));
      Q3 = static_cast<float*>(c->q3.p);
    }
    // the bf16 screen (3) runs on single-bf16 rows (wide kernels, k > 128); every other split
    // scan on the split (hi + lo) rows
    const int layout = c->opt_search_split_bf16 == 3 && c->g_kp > 128 ? 3 : 1;
    if (!c->g3_valid || c->g3_layout != layout) {
      EF_TRY(ensure(c, c->G3, (size_t)c->n_gallery * c->g_kp * sizeof(float)));
      const float* Gp = static_cast<const float*>(c->G.p);
      EF_HIP(c, layout == 3 ? launch_hi_rows(c->stream, Gp, c->n_gallery, c->g_kp, c->G3.p)
                            : launch_split_rows(c->stream, Gp, c->n_gallery, c->g_kp, c->G3.p),
             "split gallery");
      c->g3_valid = true;
      c->g3_layout = layout;
    }
    G3 = static_cast<const float*>(c->G3.p);
  }
  for (size_t i = 0; i < pieces.size(); ++i) {
    const SearchPiece& p = pieces[i];
    ws.match = match_dev ? match_dev + p.off : nullptr;
    EF_HIP(c,
           launch_search(c->stream, c->g_kp, metric, plans[i], static_cast<const float*>(c->q_pad.p) + p.off * c->g_kp,
                         Q3, p.bpad, p.b, static_cast<const float*>(c->G.p), G3, aux, c->n_gallery, c->g_offset,
                         c->gmax2_host, ws, keys_dev + p.off, c),
           "search");
  }
  return EF_OK;
}

// Search ctx->q_pad: this rank's shard, then (communicator attached) the exact merge of
// every rank's match records (ef_comm.hip).  match_dev (optional) receives the records
// of the (global) winners.
static int search_qpad(ef_ctx* c, int64_t bpad, int64_t b, int metric, long long* keys_dev, ef_match* match_dev) {
  if (!c->comm || c->comm_size == 1) return search_local(c, bpad, b, metric, keys_dev, match_dev);
  EF_TRY(ensure(c, c->match_local, (size_t)b * sizeof(ef_match)));
  EF_TRY(ensure(c, c->match_all, (size_t)b * c->comm_size * sizeof(ef_match)));
  ef_match* loc = static_cast<ef_match*>(c->match_local.p);
  ef_match* all = static_cast<ef_match*>(c->match_all.p);
  EF_TRY(search_local(c, bpad, b, metric, keys_dev, loc));
  EF_TRY(comm_allgather(c, loc, all, (size_t)b * sizeof(ef_match)));
  EF_HIP(c, launch_matches_merge(c->stream, all, c->comm_size, b, keys_dev, match_dev), "matches merge");
  return EF_OK;
}

// Project b probes (device pointer P) into ctx->q_pad; optional feature output (device).
static int project_dev(ef_ctx* c, const void* P, int dtype, int64_t b, int64_t bpad, float* f_dev, DevBuf* dst) {
  EF_TRY(ensure(c, *dst, (size_t)bpad * c->kp * sizeof(float)));
  if (b == 0) {  // this rank's slice of a sharded projection can be empty
    EF_HIP(c, hipMemsetAsync(dst->p, 0, (size_t)bpad * c->kp * sizeof(float), c->stream), "zero features");
    return EF_OK;
  }
  int64_t pps = 0;
  const uint8_t* mu8 = c->mean_u8_ok ? static_cast<const uint8_t*>(c->mean_u8.p) : nullptr;
  const void* wf = c->w16f_ok ? c->W16f.p : nullptr;
  const int ns = c->bf16 ? project_bf16_nsplit(dtype, P, mu8, wf, bpad, c->d, c->kpw, &pps)
                         : project_nsplit(bpad, c->d, c->kpw, &pps);
  EF_TRY(ensure(c, c->proj_part, (size_t)ns * bpad * c->kpw * sizeof(float)));
  TimerEvt t;
  timer_begin(c, EF_KERNEL_PROJECT, &t);
  if (c->bf16) {
    EF_HIP(c,
           launch_project_bf16(c->stream, dtype, P, b, bpad, c->d, static_cast<const float*>(c->mean_r.p),
                               mu8, static_cast<const unsigned short*>(c->W16.p), wf,
                               c->kpw,
                               static_cast<float*>(c->proj_part.p), ns, pps),
           "project kernel (bf16)");
  } else {
    EF_HIP(c,
           launch_project(c->stream, c->kpw, dtype, P, b, bpad, c->d, static_cast<const float*>(c->mean.p),
                          static_cast<const float*>(c->W.p), static_cast<float*>(c->proj_part.p), ns, pps),
           "project kernel");
  }
  timer_end(c, &t);
  EF_HIP(c,
         launch_project_reduce(c->stream, static_cast<const float*>(c->proj_part.p), ns, b, bpad, c->kpw,
                               c->k, c->kp, c->bf16 ? static_cast<const float*>(c->corr.p) : nullptr,
                               static_cast<float*>(dst->p), f_dev),
         "project reduce");
  return EF_OK;
}

// Features of the whole batch in ctx->q_pad for the search.  With a communicator attached
// rank r projects probes [r*cs, (r+1)*cs), cs = ceil(b / ranks), and one all-gather of the
// (cs x kp) slices assembles the batch (rows past b are zero); otherwise the whole batch.
// Returns the padded row count of q_pad in *bpad_out.  f_dev (optional) gets this rank's
// rows only when sharded, so the fused path keeps the unsharded projection for it.
static int project_for_search(ef_ctx* c, const void* Pd, int dtype, int64_t b, float* f_dev, int64_t* bpad_out) {
  if (!c->comm || c->comm_size == 1 || f_dev) {
    const int64_t bpad = round_up(b, kSearchProbeTile);
    EF_TRY(project_dev(c, Pd, dtype, b, bpad, f_dev, &c->q_pad));
    *bpad_out = bpad;
    return EF_OK;
  }
  const int64_t R = c->comm_size, cs = (b + R - 1) / R;
  const int64_t lo = std::min<int64_t>(b, c->comm_rank * cs), hi = std::min<int64_t>(b, (c->comm_rank + 1) * cs);
  const size_t esz = dtype == EF_U8 ? 1 : 4;
  const void* Pl = static_cast<const char*>(Pd) + (size_t)lo * c->d * esz;
  EF_TRY(project_dev(c, Pl, dtype, hi - lo, round_up(cs, kSearchProbeTile), nullptr, &c->q_local));
  const int64_t rows = R * cs, bpad = round_up(rows, kSearchProbeTile);
  EF_TRY(ensure(c, c->q_pad, (size_t)bpad * c->kp * sizeof(float)));
  float* q = static_cast<float*>(c->q_pad.p);
  EF_TRY(comm_allgather(c, c->q_local.p, q, (size_t)cs * c->kp * sizeof(float)));
  if (bpad > rows)
    EF_HIP(c, hipMemsetAsync(q + rows * c->kp, 0, (size_t)(bpad - rows) * c->kp * sizeof(float), c->stream), "pad");
  *bpad_out = bpad;
  return EF_OK;
}

static int stage_probes(ef_ctx* c, const void* P, int dtype, int64_t b, uint32_t flags, const void** Pd) {
  if (flags & EF_MEM_DEVICE) {
    *Pd = P;
    return EF_OK;
  }
  const size_t bytes = (size_t)b * c->d * (dtype == EF_U8 ? 1 : 4);
  EF_TRY(ensure(c, c->p_stage, bytes));
  EF_HIP(c, hipMemcpyAsync(c->p_stage.p, P, bytes, hipMemcpyHostToDevice, c->stream), "H2D probes");
  *Pd = c->p_stage.p;
  return EF_OK;
}

namespace {
class HostPool {
 public:
  explicit HostPool(int workers) {
    for (int i = 0; i < workers; ++i) threads_.emplace_back([this] { loop(); });
  }
  void run(int n, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> job(job_mu_);  // one job at a time
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      done_ = 0;
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(mu_);
    while (next_ < n_) {  // the caller takes tasks too (and finishes the job alone if
      const int i = next_++;  // the workers are gone, e.g. in a forked child)
      lk.unlock();
      fn(i);
      lk.lock();
      ++done_;
    }
    done_cv_.wait(lk, [&] { return done_ == n_; });
    fn_ = nullptr;
    n_ = 0;
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return fn_ && next_ < n_; });
      const int i = next_++;
      const std::function<void(int)>* f = fn_;
      lk.unlock();
      (*f)(i);  // the job cannot end before this task is counted
      lk.lock();
      if (++done_ == n_) done_cv_.notify_all();
    }
  }
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, done_ = 0;
  std::vector<std::thread> threads_;
};
}  // namespace

// Host worker count (EF_OPT_HOST_THREADS, process-wide): the job's CPU share.  The machine's
// hardware_concurrency() is the wrong size on a shared host (256 on the GPU pool's boxes,
// whose one-GPU jobs get 16 CPUs), so the default is min(16, hardware threads) and the
// Python layer sets the share it sees (OMP_NUM_THREADS, else the affinity mask).
static std::atomic<int> g_host_threads{0};
int host_threads() {
  const int v = g_host_threads.load(std::memory_order_relaxed);
  if (v > 0) return v;
  return (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
}

void host_parallel(int n, const std::function<void(int)>& fn) {
  if (n <= 1) {
    if (n == 1) fn(0);
    return;
  }
  // never destroyed: the workers block on the condition variable until the process exits
  // (sized on first use; the caller takes tasks too, so n tasks always finish)
  static HostPool* pool = new HostPool(std::max(0, std::min(host_threads(), 64) - 1));
  pool->run(n, fn);
}

hipError_t allow_dynamic_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;  // (kernel, device)
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({fn, dev})) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert({fn, dev});
  return e;
}

}  // namespace ef

using namespace ef;

extern "C" {

int ef_api_version(void) { return EF_API_VERSION; }

int ef_search_schedule(int64_t b, int32_t k, int64_t n, int32_t split_bf16, int64_t* pieces_out, int32_t max_pieces,
                       int32_t* n_pieces) {
  if (b < 0 || k < 1 || k > 65536 || n < 1 || !n_pieces || max_pieces < 0 || (max_pieces > 0 && !pieces_out))
    return EF_E_INVALID;
  const int kp = feature_pad(k);
  const std::vector<SearchPiece> pieces = search_pieces(b, kp);
  *n_pieces = (int32_t)pieces.size();
  for (size_t i = 0; i < pieces.size() && (int64_t)i < max_pieces; ++i) {
    const SearchPlan pl = search_plan(pieces[i].bpad, n, kp, split_bf16 != 0);
    int64_t* o = pieces_out + 6 * i;
    o[0] = pieces[i].off;
    o[1] = pieces[i].b;
    o[2] = pieces[i].bpad;
    o[3] = pl.n_ptiles;
    o[4] = pl.nchunks;
    o[5] = (int64_t)pl.tiles_per_chunk;
  }
  return EF_OK;
}

int ef_device_count(int* out) {
  if (!out) return EF_E_INVALID;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return EF_OK;
}

int ef_create(int device, ef_ctx** out) {
  if (!out) return EF_E_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return EF_E_HIP;
  if (device < 0 || device >= n) return EF_E_INVALID;
  if (hipSetDevice(device) != hipSuccess) return EF_E_HIP;
  ef_ctx* c = new ef_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return EF_E_HIP;
  }
  c->stream = c->own_stream;
  *out = c;
  return EF_OK;
}

void ef_destroy(ef_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)jpeg_quiesce(c);
  for (auto& t : c->pending) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  DevBuf* bufs[] = {&c->mean,      &c->W,         &c->W16,       &c->W16f,      &c->mean_r,    &c->mean_u8, &c->corr,
                    &c->G,         &c->G3,        &c->q3,        &c->gnorm2,    &c->ginv,    &c->gmax2,
                    &c->q_pad,     &c->keys,      &c->search_ws, &c->p_stage,   &c->proj_part,
                    &c->feats_dev, &c->jpeg_ws,   &c->jpeg_out,  &c->jpeg_rows, &c->jpeg_up[0], &c->jpeg_up[1]};
  for (DevBuf* b : bufs) release(*b);
  for (int i = 0; i < 2; ++i) {
    if (c->jpeg_pinned[i]) (void)hipHostFree(c->jpeg_pinned[i]);
    if (c->jpeg_up_done[i]) (void)hipEventDestroy(c->jpeg_up_done[i]);
    if (c->jpeg_ws_free[i]) (void)hipEventDestroy(c->jpeg_ws_free[i]);
  }
  if (c->jpeg_done) (void)hipEventDestroy(c->jpeg_done);
  if (c->jpeg_copy) (void)hipStreamDestroy(c->jpeg_copy);
  for (int i = 0; i < 2; ++i)
    if (c->fit_side_ev[i]) (void)hipEventDestroy(c->fit_side_ev[i]);
  if (c->fit_side) (void)hipStreamDestroy(c->fit_side);
  for (int i = 0; i < 2; ++i)
    if (c->tm_side_ev[i]) (void)hipEventDestroy(c->tm_side_ev[i]);
  if (c->tm_side) (void)hipStreamDestroy(c->tm_side);
  for (auto& b : c->fit_pool) release(b);
  comm_release(c);
  tm_release(c);
  haar_release(c);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

const char* ef_last_error(const ef_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ef_set_stream(ef_ctx* c, void* s) {
  if (!c) return EF_E_INVALID;
  c->stream = static_cast<hipStream_t>(s);  // NULL = the default stream
  return EF_OK;
}

int ef_get_stream(const ef_ctx* c, void** out) {
  if (!c || !out) return EF_E_INVALID;
  *out = static_cast<void*>(c->stream);
  return EF_OK;
}

int ef_use_own_stream(ef_ctx* c) {
  if (!c) return EF_E_INVALID;
  c->stream = c->own_stream;
  return EF_OK;
}

int ef_synchronize(ef_ctx* c) {
  if (!c) return EF_E_INVALID;
  EF_HIP(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  return EF_OK;
}

int ef_trim(ef_ctx* c) {
  if (!c) return EF_E_INVALID;
  EF_HIP(c, hipSetDevice(c->device), "hipSetDevice");
  EF_HIP(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  EF_HIP(c, jpeg_quiesce(c), "jpeg quiesce");
  for (auto& b : c->fit_pool) release(b);
  c->fit_pool.clear();
  release(c->jpeg_ws);
  release(c->jpeg_out);
  release(c->jpeg_rows);
  release(c->jpeg_up[0]);
  release(c->jpeg_up[1]);
  for (int i = 0; i < 2; ++i) {
    if (c->jpeg_pinned[i]) (void)hipHostFree(c->jpeg_pinned[i]);
    c->jpeg_pinned[i] = nullptr;
    c->jpeg_pinned_bytes[i] = 0;
  }
  return EF_OK;
}

int ef_model_set(ef_ctx* c, const float* mean, const float* W, int64_t d, int32_t k, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if (!mean || !W || d < 1 || k < 1) return set_err(c, EF_E_INVALID, "ef_model_set: bad arguments");
  const int kp = feature_pad(k);
  if (kp < 0) return set_err(c, EF_E_INVALID, "ef_model_set: k > 65536 is not supported");
  (void)hipSetDevice(c->device);
  const bool bf16 = (flags & EF_MODEL_BF16) != 0;
  const int kpw = bf16 ? (kp + 127) / 128 * 128 : proj_pad(kp);  // bf16 kernel: 128-column tiles
  EF_TRY(ensure(c, c->mean, (size_t)d * sizeof(float)));
  EF_TRY(ensure(c, c->W, (size_t)d * kpw * sizeof(float)));
  const hipMemcpyKind kind = (flags & EF_MEM_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  EF_HIP(c, hipMemcpyAsync(c->mean.p, mean, (size_t)d * sizeof(float), kind, c->stream), "copy mean");
  const float* wsrc = W;
  DevBuf tmp;
  if (!(flags & EF_MEM_DEVICE)) {
    EF_TRY(ensure(c, tmp, (size_t)d * k * sizeof(float)));
    hipError_t e = hipMemcpyAsync(tmp.p, W, (size_t)d * k * sizeof(float), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) { release(tmp); return hip_err(c, e, "copy W"); }
    wsrc = static_cast<const float*>(tmp.p);
  }
  hipError_t e = launch_pad_rows(c->stream, wsrc, d, k, d, static_cast<float*>(c->W.p), kpw);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  release(tmp);
  if (e != hipSuccess) return hip_err(c, e, "pad W");
  if (bf16) {
    const int ldw = kpw;
    EF_TRY(ensure(c, c->W16, (size_t)ldw * d * sizeof(unsigned short)));
    EF_TRY(ensure(c, c->mean_r, (size_t)d * sizeof(float)));
    EF_TRY(ensure(c, c->corr, (size_t)ldw * sizeof(float)));
    const int nchunk = 256;
    DevBuf cp;
    EF_TRY(ensure(c, cp, (size_t)nchunk * ldw * sizeof(double)));
    e = launch_bf16_model(c->stream, static_cast<const float*>(c->W.p), static_cast<const float*>(c->mean.p), d, ldw,
                          static_cast<unsigned short*>(c->W16.p), static_cast<float*>(c->mean_r.p),
                          static_cast<float*>(c->corr.p), static_cast<double*>(cp.p), nchunk);
    int bad = 1;
    int* bad_dev = reinterpret_cast<int*>(static_cast<char*>(c->mean_u8.p));
    if (e == hipSuccess) {
      const size_t off = ((size_t)d + 255) & ~size_t(255);
      const int rc = ensure(c, c->mean_u8, off + 16);
      if (rc != EF_OK) { release(cp); return rc; }
      bad_dev = reinterpret_cast<int*>(static_cast<char*>(c->mean_u8.p) + off);
      e = hipMemsetAsync(bad_dev, 0, sizeof(int), c->stream);
      if (e == hipSuccess)
        e = launch_mean_u8(c->stream, static_cast<const float*>(c->mean_r.p), d, static_cast<uint8_t*>(c->mean_u8.p),
                           bad_dev);
      if (e == hipSuccess) e = hipMemcpyAsync(&bad, bad_dev, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    release(cp);
    if (e != hipSuccess) return hip_err(c, e, "bf16 model");
    c->mean_u8_ok = bad == 0;
    c->w16f_ok = false;
    if (bf16_frag_supported(d, ldw)) {
      EF_TRY(ensure(c, c->W16f, (size_t)ldw * d * sizeof(unsigned short)));
      EF_HIP(c, launch_bf16_frag(c->stream, static_cast<const unsigned short*>(c->W16.p), d, ldw, c->W16f.p),
             "bf16 fragment model");
      EF_HIP(c, hipStreamSynchronize(c->stream), "sync");
      c->w16f_ok = true;
    }
  }
  c->bf16 = bf16;
  c->d = d;
  c->k = k;
  c->kp = kp;
  c->kpw = kpw;
  return EF_OK;
}

int ef_project(ef_ctx* c, const void* P, int32_t dtype, int64_t b, float* F, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if (c->d == 0) return set_err(c, EF_E_STATE, "ef_project: no model (call ef_model_set)");
  if (!P || !F || b < 0 || (dtype != EF_U8 && dtype != EF_F32))
    return set_err(c, EF_E_INVALID, "ef_project: bad arguments");
  if (b == 0) return EF_OK;
  (void)hipSetDevice(c->device);
  const int64_t bpad = round_up(b, kSearchProbeTile);
  const void* Pd = nullptr;
  EF_TRY(stage_probes(c, P, dtype, b, flags, &Pd));
  float* fdev = F;
  if (!(flags & EF_MEM_DEVICE)) {
    EF_TRY(ensure(c, c->feats_dev, (size_t)b * c->k * sizeof(float)));
    fdev = static_cast<float*>(c->feats_dev.p);
  }
  EF_TRY(project_dev(c, Pd, dtype, b, bpad, fdev, &c->q_pad));
  if (!(flags & EF_MEM_DEVICE)) {
    EF_HIP(c, hipMemcpyAsync(F, fdev, (size_t)b * c->k * sizeof(float), hipMemcpyDeviceToHost, c->stream),
           "D2H features");
    EF_HIP(c, hipStreamSynchronize(c->stream), "sync");
  }
  return EF_OK;
}

int ef_gallery_set(ef_ctx* c, const float* G, int64_t n, int32_t k, int64_t offset, uint32_t flags) {
  if (!c) return EF_E_INVALID;
  if ((!G && n > 0) || n < 0 || k < 1 || offset < 0 || n + offset > (int64_t)UINT_MAX)
    return set_err(c, EF_E_INVALID, "ef_gallery_set: bad arguments");
  const int kp = feature_pad(k);
  if (kp < 0) return set_err(c, EF_E_INVALID, "ef_gallery_set: k > 65536 is not supported");
  (void)hipSetDevice(c->device);
  c->n_gallery = 0;
  c->g3_valid = false;
  if (n > 0) {
    EF_TRY(ensure(c, c->G, (size_t)n * kp * sizeof(float)));
    EF_TRY(ensure(c, c->gnorm2, (size_t)n * sizeof(float)));
    EF_TRY(ensure(c, c->ginv, (size_t)n * sizeof(float)));
    EF_TRY(ensure(c, c->gmax2, 16));
    const hipMemcpyKind kind = (flags & EF_MEM_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (k == kp) {
      EF_HIP(c, hipMemcpyAsync(c->G.p, G, (size_t)n * k * sizeof(float), kind, c->stream), "copy gallery");
    } else {
      const float* src = G;
      DevBuf tmp;
      if (!(flags & EF_MEM_DEVICE)) {
        EF_TRY(ensure(c, tmp, (size_t)n * k * sizeof(float)));
        hipError_t e = hipMemcpyAsync(tmp.p, G, (size_t)n * k * sizeof(float), hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) { release(tmp); return hip_err(c, e, "copy gallery"); }
        src = static_cast<const float*>(tmp.p);
      }
      hipError_t e = launch_pad_rows(c->stream, src, n, k, n, static_cast<float*>(c->G.p), kp);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      release(tmp);
      if (e != hipSuccess) return hip_err(c, e, "pad gallery");
    }
    EF_HIP(c,
           launch_gallery_aux(c->stream, static_cast<const float*>(c->G.p), n, kp,
                              static_cast<float*>(c->gnorm2.p), static_cast<float*>(c->ginv.p),
                              static_cast<unsigned*>(c->gmax2.p)),
           "gallery norms");
    EF_HIP(c, hipMemcpyAsync(&c->gmax2_host, c->gmax2.p, sizeof(float), hipMemcpyDeviceToHost, c->stream),
           "D2H gmax2");
    EF_HIP(c, hipStreamSynchronize(c->stream), "sync");
  }
  c->n_gallery = n;
  c->g_offset = offset;
  c->g_k = k;
  c->g_kp = kp;
  return EF_OK;
}

// ef_search / ef_search_matches: keys (and/or match records) of b probe features.
static int search_impl(ef_ctx* c, const float* Q, int64_t b, int32_t metric, int64_t* keys, ef_match* match,
                       uint32_t flags, const char* fn) {
  if (!c) return EF_E_INVALID;
  if (c->g_k == 0) return set_err(c, EF_E_STATE, std::string(fn) + ": no gallery (call ef_gallery_set)");
  if (!Q || (!keys && !match) || b < 0 || (metric != EF_METRIC_L2 && metric != EF_METRIC_COSINE))
    return set_err(c, EF_E_INVALID, std::string(fn) + ": bad arguments");
  if (b == 0) return EF_OK;
  (void)hipSetDevice(c->device);
  const bool dev = flags & EF_MEM_DEVICE;
  const int64_t bpad = round_up(b, kSearchProbeTile);
  EF_TRY(ensure(c, c->q_pad, (size_t)bpad * c->g_kp * sizeof(float)));
  const float* qsrc = Q;
  if (!dev) {
    EF_TRY(ensure(c, c->p_stage, (size_t)b * c->g_k * sizeof(float)));
    EF_HIP(c, hipMemcpyAsync(c->p_stage.p, Q, (size_t)b * c->g_k * sizeof(float), hipMemcpyHostToDevice, c->stream),
           "H2D queries");
    qsrc = static_cast<const float*>(c->p_stage.p);
  }
  EF_HIP(c, launch_pad_rows(c->stream, qsrc, b, c->g_k, bpad, static_cast<float*>(c->q_pad.p), c->g_kp),
         "pad queries");
  EF_TRY(ensure(c, c->keys, (size_t)bpad * sizeof(long long) + (size_t)b * sizeof(ef_match)));
  long long* kdev = (dev && keys) ? reinterpret_cast<long long*>(keys) : static_cast<long long*>(c->keys.p);
  ef_match* mdev = nullptr;
  if (match) mdev = dev ? match : reinterpret_cast<ef_match*>(static_cast<char*>(c->keys.p) + bpad * sizeof(long long));
  EF_TRY(search_qpad(c, bpad, b, metric, kdev, mdev));
  if (!dev) {
    if (keys)
      EF_HIP(c, hipMemcpyAsync(keys, kdev, (size_t)b * sizeof(long long), hipMemcpyDeviceToHost, c->stream),
             "D2H keys");
    if (match)
      EF_HIP(c, hipMemcpyAsync(match, mdev, (size_t)b * sizeof(ef_match), hipMemcpyDeviceToHost, c->stream),
             "D2H matches");
    EF_HIP(c, hipStreamSynchronize(c->stream), "sync");
  }
  return EF_OK;
}

static int recognize_impl(ef_ctx* c, const void* P, int32_t dtype, int64_t b, int32_t metric, int64_t* keys,
                          ef_match* match, float* feats, uint32_t flags, const char* fn) {
  if (!c) return EF_E_INVALID;
  const std::string f(fn);
  if (c->d == 0) return set_err(c, EF_E_STATE, f + ": no model (call ef_model_set)");
  if (c->g_k == 0) return set_err(c, EF_E_STATE, f + ": no gallery (call ef_gallery_set)");
  if (c->g_k != c->k) return set_err(c, EF_E_INVALID, f + ": gallery k != model k");
  if (!P || (!keys && !match) || b < 0 || (dtype != EF_U8 && dtype != EF_F32) ||
      (metric != EF_METRIC_L2 && metric != EF_METRIC_COSINE))
    return set_err(c, EF_E_INVALID, f + ": bad arguments");
  if (b == 0) return EF_OK;
  (void)hipSetDevice(c->device);
  const bool dev = flags & EF_MEM_DEVICE;
  const void* Pd = nullptr;
  EF_TRY(stage_probes(c, P, dtype, b, flags, &Pd));
  float* fdev = nullptr;
  if (feats) {
    if (dev) {
      fdev = feats;
    } else {
      EF_TRY(ensure(c, c->feats_dev, (size_t)b * c->k * sizeof(float)));
      fdev = static_cast<float*>(c->feats_dev.p);
    }
  }
  int64_t bpad = 0;
  EF_TRY(project_for_search(c, Pd, dtype, b, fdev, &bpad));
  EF_TRY(ensure(c, c->keys, (size_t)bpad * sizeof(long long) + (size_t)b * sizeof(ef_match)));
  long long* kdev = (dev && keys) ? reinterpret_cast<long long*>(keys) : static_cast<long long*>(c->keys.p);
  ef_match* mdev = nullptr;
  if (match) mdev = dev ? match : reinterpret_cast<ef_match*>(static_cast<char*>(c->keys.p) + bpad * sizeof(long long));
  EF_TRY(search_qpad(c, bpad, b, metric, kdev, mdev));
  if (!dev) {
    if (keys)
      EF_HIP(c, hipMemcpyAsync(keys, kdev, (size_t)b * sizeof(long long), hipMemcpyDeviceToHost, c->stream),
             "D2H keys");
    if (match)
      EF_HIP(c, hipMemcpyAsync(match, mdev, (size_t)b * sizeof(ef_match), hipMemcpyDeviceToHost, c->stream),
             "D2H matches");
    if (feats)
      EF_HIP(c, hipMemcpyAsync(feats, fdev, (size_t)b * c->k * sizeof(float), hipMemcpyDeviceToHost, c->stream),
             "D2H features");
    EF_HIP(c, hipStreamSynchronize(c->stream), "sync");
  }
  return EF_OK;
}

int ef_search(ef_ctx* c, const float* Q, int64_t b, int32_t metric, int64_t* keys, uint32_t flags) {
  if (c && !keys) return set_err(c, EF_E_INVALID, "ef_search: bad arguments");
  return search_impl(c, Q, b, metric, keys, nullptr, flags, "ef_search");
}

int ef_search_matches(ef_ctx* c, const float* Q, int64_t b, int32_t metric, ef_match* out, uint32_t flags) {
  if (c && !out) return set_err(c, EF_E_INVALID, "ef_search_matches: bad arguments");
  return search_impl(c, Q, b, metric, nullptr, out, flags, "ef_search_matches");
}

int ef_recognize(ef_ctx* c, const void* P, int32_t dtype, int64_t b, int32_t metric, int64_t* keys, float* feats,
                 uint32_t flags) {
  if (c && !keys) return set_err(c, EF_E_INVALID, "ef_recognize: bad arguments");
  return recognize_impl(c, P, dtype, b, metric, keys, nullptr, feats, flags, "ef_recognize");
}

int ef_recognize_matches(ef_ctx* c, const void* P, int32_t dtype, int64_t b, int32_t metric, ef_match* out,
                         float* feats, uint32_t flags) {
  if (c && !out) return set_err(c, EF_E_INVALID, "ef_recognize_matches: bad arguments");
  return recognize_impl(c, P, dtype, b, metric, nullptr, out, feats, flags, "ef_recognize_matches");
}

int ef_set_option(ef_ctx* c, int32_t option, int64_t value) {
  if (!c) return EF_E_INVALID;
  switch (option) {
    case EF_OPT_FIT_MAX_ITERS:
      if (value < 1) return set_err(c, EF_E_INVALID, "EF_OPT_FIT_MAX_ITERS must be >= 1");
      c->opt_fit_max_iters = value;
      return EF_OK;
    case EF_OPT_FIT_FP32_COARSE:
      if (value < 0 || value > 2) return set_err(c, EF_E_INVALID, "EF_OPT_FIT_FP32_COARSE must be 0, 1 or 2");
      c->opt_fit_fp32_coarse = value;
      return EF_OK;
    case EF_OPT_COV_SLAB_BYTES:
      if (value < 1) return set_err(c, EF_E_INVALID, "EF_OPT_COV_SLAB_BYTES must be >= 1");
      c->opt_cov_slab_bytes = value;
      return EF_OK;
    case EF_OPT_TM_INT64_SUMS:
      c->opt_tm_int64 = value != 0;
      return EF_OK;
    case EF_OPT_HAAR_ORDERED:
      c->opt_haar_ordered = value != 0;
      return EF_OK;
    case EF_OPT_JPEG_CHUNK_BITS:
      if (value < 0 || value > (1 << 24) || value % 32)
        return set_err(c, EF_E_INVALID, "EF_OPT_JPEG_CHUNK_BITS must be 0 or a multiple of 32 up to 2^24");
      c->opt_jpeg_chunk_bits = value;
      return EF_OK;
    case EF_OPT_JPEG_PART_FILES:
      if (value < 1) return set_err(c, EF_E_INVALID, "EF_OPT_JPEG_PART_FILES must be >= 1");
      c->opt_jpeg_part_files = value;
      return EF_OK;
    case EF_OPT_FIT_CHEBYSHEV:
      c->opt_fit_chebyshev = value != 0;
      return EF_OK;
    case EF_OPT_SEARCH_SPLIT_BF16:
      if (value < 0 || value > 3) return set_err(c, EF_E_INVALID, "EF_OPT_SEARCH_SPLIT_BF16 must be 0, 1, 2 or 3");
      c->opt_search_split_bf16 = value;
      return EF_OK;
    case EF_OPT_HOST_THREADS:
      if (value < 0 || value > 256) return set_err(c, EF_E_INVALID, "EF_OPT_HOST_THREADS must be 0..256");
      g_host_threads.store((int)value, std::memory_order_relaxed);
      return EF_OK;
    default:
      return set_err(c, EF_E_INVALID, "ef_set_option: unknown option " + std::to_string(option));
  }
}

int ef_get_option(const ef_ctx* c, int32_t option, int64_t* value) {
  if (!c || !value) return EF_E_INVALID;
  switch (option) {
    case EF_OPT_FIT_MAX_ITERS: *value = c->opt_fit_max_iters; return EF_OK;
    case EF_OPT_FIT_FP32_COARSE: *value = c->opt_fit_fp32_coarse; return EF_OK;
    case EF_OPT_COV_SLAB_BYTES: *value = c->opt_cov_slab_bytes; return EF_OK;
    case EF_OPT_TM_INT64_SUMS: *value = c->opt_tm_int64; return EF_OK;
    case EF_OPT_HAAR_ORDERED: *value = c->opt_haar_ordered; return EF_OK;
    case EF_OPT_JPEG_CHUNK_BITS: *value = c->opt_jpeg_chunk_bits; return EF_OK;
    case EF_OPT_SEARCH_SPLIT_BF16: *value = c->opt_search_split_bf16; return EF_OK;
    case EF_OPT_JPEG_PART_FILES: *value = c->opt_jpeg_part_files; return EF_OK;
    case EF_OPT_FIT_CHEBYSHEV: *value = c->opt_fit_chebyshev; return EF_OK;
    case EF_OPT_HOST_THREADS: *value = host_threads(); return EF_OK;
    default: return EF_E_INVALID;
  }
}

void ef_keys_decode(const int64_t* keys, int64_t b, int32_t metric, float* best, int64_t* idx) {
  for (int64_t i = 0; i < b; ++i) {
    const int64_t key = keys[i];
    if (key == EF_KEY_NONE) {
      if (best) best[i] = NAN;
      if (idx) idx[i] = -1;
      continue;
    }
    const int32_t s = (int32_t)(key >> 32);
    const int32_t bits = s >= 0 ? s : (s ^ 0x7FFFFFFF);
    float v;
    std::memcpy(&v, &bits, sizeof(v));
    if (best) best[i] = metric == EF_METRIC_COSINE ? -v : v;
    if (idx) idx[i] = (int64_t)(uint32_t)(key & 0xffffffffll);
  }
}

int ef_timing_enable(ef_ctx* c, int on) {
  if (!c) return EF_E_INVALID;
  c->timing = on != 0;
  return EF_OK;
}

static int timing_drain(ef_ctx* c) {
  if (c->pending.empty()) return EF_OK;
  EF_HIP(c, hipStreamSynchronize(c->stream), "sync");
  for (auto& t : c->pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess && t.kernel >= 0 && t.kernel < 8) {
      c->t_ms[t.kernel] += ms;
      c->t_n[t.kernel] += 1;
    }
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  c->pending.clear();
  return EF_OK;
}

int ef_timing_get(ef_ctx* c, int32_t kernel, double* total_ms, int64_t* launches) {
  if (!c || kernel < 0 || kernel >= 8) return EF_E_INVALID;
  EF_TRY(timing_drain(c));
  if (total_ms) *total_ms = c->t_ms[kernel];
  if (launches) *launches = c->t_n[kernel];
  return EF_OK;
}

int ef_timing_reset(ef_ctx* c) {
  if (!c) return EF_E_INVALID;
  EF_TRY(timing_drain(c));
  for (int i = 0; i < 8; ++i) {
    c->t_ms[i] = 0;
    c->t_n[i] = 0;
  }
  return EF_OK;
}

}  // extern "C"
