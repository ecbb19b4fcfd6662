// Exact cross-shard arg-best merge and the in-library RCCL communicator
// (include/eigenface.h: ef_matches_merge, ef_comm_*).
//
// Sharding: rank r owns gallery rows [lo_r, hi_r) (global offsets in its
// keys).  Each rank's search emits one match record per probe — the winner's fp64 score,
// the tie-tolerance scale and the packed key — and one all-gather of the records
// (24 B x b per rank, latency-bound at b = 4096) lets every rank merge them exactly: the
// lowest global index among the parts whose fp64 score is within 1e-12 of the minimum,
// the rule ef_search's resolve_kernel applies inside one gallery.  This replaces the
// reference's best-over-models loop (scan-template-v4.py:297-319, strict '>' in model
// order) by an order-independent exact reduction.
//
// What "exact" covers: the merged row equals the single-gallery arg-best whenever the
// competing rows' fp64 scores are exactly equal (lowest global index wins, np.argmin's
// rule) or differ by more than the 1e-12 relative tie window.  Inside that window — fp64
// rounding noise of the score evaluation itself, where np.argmin's own answer depends on
// summation order — a shard reports the lowest index of ITS window (measured from its own
// minimum, scaled by its own max‖g‖²), so a row that is in the global window but not in
// its shard's can lose to another shard's row.  Closing that would need a second
// exchange round for a difference below fp64 evaluation error; it is not done.
//
// RCCL is loaded at run time (dlopen): a process that already mapped a librccl (torch's)
// reuses it, and libeigenface keeps no link-time dependency on it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <climits>
#include <cmath>
#include <cstring>

#include "ef_internal.hpp"

namespace ef {

// ---------------------------------------------------------------------------- merge
__host__ __device__ inline long long merge_pack_key(float v, unsigned idx) {
  if (v == 0.0f) v = 0.0f;  // canonical +0 (ef_search_common.hpp pack_key)
  int b;
  memcpy(&b, &v, sizeof b);
  const int s = b >= 0 ? b : (b ^ 0x7FFFFFFF);
  return (long long)(((unsigned long long)(unsigned)s << 32) | (unsigned long long)idx);
}

__host__ __device__ inline void merge_one(const ef_match* parts, int nparts, int64_t b, int64_t p, long long* key,
                                          ef_match* merged) {
  double vmin = INFINITY, sc = 0.0;
  bool any = false;
  for (int r = 0; r < nparts; ++r) {
    const ef_match& m = parts[(int64_t)r * b + p];
    if (m.key == LLONG_MAX) continue;
    any = true;
    vmin = m.score < vmin ? m.score : vmin;
    sc = m.scale > sc ? m.scale : sc;
  }
  if (!any) {
    *key = LLONG_MAX;
    if (merged) *merged = ef_match{INFINITY, 0.0, LLONG_MAX};
    return;
  }
  const double tol = 1e-12 * (fabs(vmin) + sc);
  long long best_idx = LLONG_MAX;
  double best_v = vmin;
  for (int r = 0; r < nparts; ++r) {
    const ef_match& m = parts[(int64_t)r * b + p];
    if (m.key == LLONG_MAX || !(m.score <= vmin + tol)) continue;
    const long long idx = m.key & 0xffffffffll;
    if (idx < best_idx) best_idx = idx, best_v = m.score;
  }
  *key = merge_pack_key((float)best_v, (unsigned)best_idx);
  if (merged) *merged = ef_match{best_v, sc, *key};
}

__global__ void matches_merge_kernel(const ef_match* __restrict__ parts, int nparts, int64_t b,
                                     long long* __restrict__ keys, ef_match* __restrict__ merged) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= b) return;
  merge_one(parts, nparts, b, p, keys + p, merged ? merged + p : nullptr);
}

hipError_t launch_matches_merge(hipStream_t s, const ef_match* parts, int nparts, int64_t b, long long* keys,
                                ef_match* merged) {
  if (b <= 0) return hipSuccess;
  hipLaunchKernelGGL(matches_merge_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, s, parts, nparts, b, keys,
                     merged);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- RCCL
namespace {
struct Rccl {
  bool tried = false, ok = false;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  if (r.tried) return r;
  r.tried = true;
  void* h = nullptr;
  for (const char* name : {"librccl.so.1", "librccl.so"}) {
    h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);  // the copy the process already mapped (torch's)
    if (h) break;
  }
  for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
    if (h) break;
    h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
  }
  if (!h) return r;
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
  r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.error_string;
  return r;
}

int rccl_err(ef_ctx* c, ncclResult_t e, const char* what) {
  return set_err(c, EF_E_HIP, std::string(what) + ": " + rccl().error_string(e));
}
}  // namespace

void comm_release(ef_ctx* c) {
  if (c->comm && rccl().ok) (void)rccl().comm_destroy(static_cast<ncclComm_t>(c->comm));
  c->comm = nullptr;
  c->comm_size = 1;
  c->comm_rank = 0;
  release(c->match_local);
  release(c->match_all);
  release(c->q_local);
}

int comm_allgather(ef_ctx* c, const void* send, void* recv, size_t bytes_per_rank) {
  const ncclResult_t e = rccl().all_gather(send, recv, bytes_per_rank, ncclUint8, static_cast<ncclComm_t>(c->comm),
                                           c->stream);
  return e == ncclSuccess ? EF_OK : rccl_err(c, e, "ncclAllGather");
}

}  // namespace ef

using namespace ef;

extern "C" {

int ef_matches_merge(ef_ctx* c, const ef_match* parts, int32_t nparts, int64_t b, int64_t* keys_out,
                     ef_match* merged_out, uint32_t flags) {
  if (!parts || !keys_out || nparts < 1 || b < 0) return c ? set_err(c, EF_E_INVALID, "ef_matches_merge: bad arguments")
                                                           : EF_E_INVALID;
  if (flags & EF_MEM_DEVICE) {
    if (!c) return EF_E_INVALID;
    (void)hipSetDevice(c->device);
    const hipError_t e = launch_matches_merge(c->stream, parts, nparts, b, reinterpret_cast<long long*>(keys_out),
                                              merged_out);
    return e == hipSuccess ? EF_OK : hip_err(c, e, "matches merge");
  }
  for (int64_t p = 0; p < b; ++p)
    merge_one(parts, nparts, b, p, reinterpret_cast<long long*>(keys_out + p), merged_out ? merged_out + p : nullptr);
  return EF_OK;
}

int ef_comm_unique_id(void* id_out) {
  if (!id_out) return EF_E_INVALID;
  if (!rccl().ok) return EF_E_STATE;
  ncclUniqueId id;
  if (rccl().get_unique_id(&id) != ncclSuccess) return EF_E_HIP;
  static_assert(sizeof(ncclUniqueId) == EF_UNIQUE_ID_BYTES, "RCCL unique id size");
  memcpy(id_out, &id, sizeof id);
  return EF_OK;
}

int ef_comm_init(ef_ctx* c, int32_t nranks, int32_t rank, const void* unique_id) {
  if (!c) return EF_E_INVALID;
  if (nranks < 1 || rank < 0 || rank >= nranks || !unique_id)
    return set_err(c, EF_E_INVALID, "ef_comm_init: bad arguments");
  if (!rccl().ok) return set_err(c, EF_E_STATE, "ef_comm_init: RCCL (librccl.so.1) could not be loaded");
  (void)hipSetDevice(c->device);
  comm_release(c);
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof id);
  ncclComm_t comm = nullptr;
  const ncclResult_t e = rccl().comm_init_rank(&comm, nranks, id, rank);
  if (e != ncclSuccess) return rccl_err(c, e, "ncclCommInitRank");
  c->comm = comm;
  c->comm_size = nranks;
  c->comm_rank = rank;
  return EF_OK;
}

int ef_comm_destroy(ef_ctx* c) {
  if (!c) return EF_E_INVALID;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  comm_release(c);
  return EF_OK;
}

int ef_comm_info(const ef_ctx* c, int32_t* nranks, int32_t* rank) {
  if (!c) return EF_E_INVALID;
  if (nranks) *nranks = c->comm ? c->comm_size : 1;
  if (rank) *rank = c->comm ? c->comm_rank : 0;
  return EF_OK;
}

}  // extern "C"
