/*
 * eigenface.h — C ABI of libeigenface.so, the MI355X (gfx950) eigenfaces engine.
 *
 * The reference (saladbkp/face-detection-recognization-PCA) has no FFI: its hot
 * path is Python calling NumPy/LAPACK and scikit-learn.  Each entry point below
 * replaces one of those call sites; the Python host layer
 * (face-detection-recognization-pca_amd/eigenface) binds them with ctypes and
 * keeps the reference's Python surface (INTEGRATION.md shows the bindings).
 *
 * Conventions
 *   - Every function returns EF_OK (0) or a negative EF_E_* code; the message is
 *     available from ef_last_error(ctx) until the next call on that ctx.
 *   - Sizes are int64_t, matrices are row-major and dense (leading dimension =
 *     row length) unless stated otherwise.
 *   - Pointer arguments are HOST pointers unless EF_MEM_DEVICE is set in
 *     `flags`, in which case they are device pointers on the ctx's device
 *     (e.g. torch-ROCm data_ptr()).  Host-pointer calls are synchronous on
 *     return; device-pointer calls are stream-ordered on the ctx's stream and
 *     return without synchronising.
 *   - A ctx is not thread-safe.  One process per GPU.
 */
#ifndef EIGENFACE_H_
#define EIGENFACE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EF_API_VERSION 7

/* status codes */
#define EF_OK 0
#define EF_E_INVALID (-1) /* bad argument / unsupported shape            */
#define EF_E_HIP (-2)     /* HIP runtime error                           */
#define EF_E_STATE (-3)   /* call out of order (no model / no gallery)   */
#define EF_E_NOMEM (-4)   /* device allocation failed                    */
#define EF_E_NUMERIC (-5) /* eigensolver did not converge / non-finite   */

/* element types */
#define EF_U8 0
#define EF_F32 1
#define EF_F64 2

/* similarity metrics (ef_search) */
#define EF_METRIC_L2 0     /* argmin ||q-g||^2, lowest index on ties (north star)           */
#define EF_METRIC_COSINE 1 /* argmax q.g/(|q||g|), first max wins (scan-template-v4.py:274-275) */

/* flags */
#define EF_FIT_STANDARDIZE 0x1u /* StandardScaler before PCA (train-v4.py:131)                */
#define EF_MODEL_BF16 0x2u      /* ef_model_set: project on bf16 MFMA (config 5), fp32 features */
#define EF_MEM_DEVICE 0x100u    /* pointer args are device pointers, call is asynchronous    */
#define EF_IMG_RGB 0x200u       /* ef_preprocess: 3/4-channel pixels are RGB(A), not BGR(A)  */

/* kernels whose device time can be queried with ef_timing_get */
#define EF_KERNEL_SEARCH 0  /* distance GEMM + fused arg-best   */
#define EF_KERNEL_PROJECT 1 /* (p - mean).W projection GEMM     */
#define EF_KERNEL_TMATCH 2  /* template localiser, one frame    */
#define EF_KERNEL_INGEST 3  /* grey + resize of one image batch */
#define EF_KERNEL_HAAR 4    /* Haar cascade detection, one frame (GPU part) */
#define EF_KERNEL_JPEG 5    /* JPEG entropy decode + IDCT + colour, one batch */
#define EF_KERNEL_SYRK 6    /* the fit's int8 covariance/Gram SYRK, all passes of one fit */
#define EF_KERNEL_JPEG_HOST 7 /* host staging of one ef_jpeg_ingest part (marker parse, destuff, tables):
                                wall time on the host, not a device kernel (API v7) */

/* No-result sentinel in a key array (empty gallery). */
#define EF_KEY_NONE INT64_MAX

typedef struct ef_ctx ef_ctx;

/* ---------------------------------------------------------------- context */
int ef_api_version(void);
int ef_device_count(int* out);
int ef_create(int device, ef_ctx** out);
void ef_destroy(ef_ctx* ctx);
const char* ef_last_error(const ef_ctx* ctx);
/* Launch on an external hipStream_t, e.g. torch.cuda.current_stream().cuda_stream;
 * NULL means the default (null) stream.  ef_use_own_stream restores the ctx's own
 * non-blocking stream (the default after ef_create). */
int ef_set_stream(ef_ctx* ctx, void* hip_stream);
int ef_use_own_stream(ef_ctx* ctx);
/* The hipStream_t the ctx launches on now (*out; NULL = the default stream): lets a caller
 * order its own stream after an asynchronous EF_MEM_DEVICE call (hipStreamWaitEvent, or
 * torch.cuda.ExternalStream + wait_stream). */
int ef_get_stream(const ef_ctx* ctx, void** out);
int ef_synchronize(ef_ctx* ctx);
/* ef_fit keeps its device workspaces (operand copies, covariance, subspace blocks) in
 * the context between calls, so repeated fits do not pay hipMalloc/hipFree; ef_trim
 * frees them (ef_destroy does too). */
int ef_trim(ef_ctx* ctx);

/* -------------------------------------------------------------------- fit
 * Replaces manual_pca (useless/train.py:56-128) and, with EF_FIT_STANDARDIZE,
 * StandardScaler.fit_transform + PCA(svd_solver='full').fit_transform
 * (train-v4.py:126-146).  X is n x d uint8 pixels (train-v4.py:68,73).
 * Computes mean -> centre(+scale) -> covariance (Gram A.A^T/(n-1) when n<d,
 * A^T.A/(n-1) otherwise) -> symmetric eigensolve -> back-project -> unit
 * eigenfaces with the sklearn svd_flip sign rule -> training projection.
 * k is clamped to min(n, d) as manual_pca does (useless/train.py:114).
 * Outputs (host or device, all float64; NULL skips an optional output):
 *   mean_out[d]        column mean of X (train-v4.py:127, useless/train.py:70)
 *   var_out[d]         population variance (StandardScaler.var_)        optional
 *   scale_out[d]       StandardScaler.scale_ (1 for constant pixels)     optional
 *   components_out[k*d] eigenfaces as rows (pca.components_; manual_pca's
 *                      eigenfaces matrix is its transpose)
 *   eigvals_out[k]     covariance eigenvalues, descending (explained_variance_)
 *   proj_out[n*k]      training projection (projected_data / face_features) optional
 *   total_var_out[1]   trace of the covariance                         optional
 *   k_out[1]           number of components actually produced          optional
 *   iters_out[1]       eigensolver iterations (0 = direct Jacobi)       optional
 */
int ef_fit(ef_ctx* ctx, const uint8_t* X, int64_t n, int64_t d, int32_t k, uint32_t flags,
           double* mean_out, double* var_out, double* scale_out, double* components_out,
           double* eigvals_out, double* proj_out, double* total_var_out, int32_t* k_out,
           int32_t* iters_out);
/* ef_fit for any element type: x_dtype EF_U8 (= ef_fit), EF_F32 or EF_F64 — manual_pca's
 * float64 faces (useless/train.py:40, :56-128) and ManualPCA.fit on standardised,
 * non-integral data (scripts/manual/train-v2.py:16-42, fed by ManualStandardScaler :53-72).
 * Float input: fp64 two-pass column statistics, covariance / Gram, back-projection and
 * training projection on the fp64 MFMA GEMM with centring (and 1/scale) in the operand
 * loads; uint8 input keeps the exact integer kernels. */
int ef_fit_ex(ef_ctx* ctx, const void* X, int32_t x_dtype, int64_t n, int64_t d, int32_t k, uint32_t flags,
              double* mean_out, double* var_out, double* scale_out, double* components_out,
              double* eigvals_out, double* proj_out, double* total_var_out, int32_t* k_out,
              int32_t* iters_out);
/* Column mean and population variance of X (n x d, EF_U8 / EF_F32 / EF_F64), float64 out:
 * ManualStandardScaler.fit (np.mean / np.std, scripts/manual/train-v2.py:58-64) and
 * StandardScaler.fit's statistics (train-v4.py:131).  uint8: exact integer sums; float:
 * two passes in fp64 (sum, then sum of (x - mean) and (x - mean)^2, sklearn's
 * _incremental_mean_and_var form).  var_out may be NULL. */
int ef_colstats(ef_ctx* ctx, const void* X, int32_t x_dtype, int64_t n, int64_t d, uint32_t flags,
                double* mean_out, double* var_out);
/* The fit's CholQR factor alone (API v7): Li = L^-1 (row-major, zeros above the diagonal)
 * for G = L L^T, 1 <= m <= 256, G row-major with row stride ldg >= m; host pointers.  A
 * pivot <= tol_rel * max diag(G) sets *info = -(column + 1) and leaves Li as given;
 * *info = 0 on success. */
int ef_chol_inv(ef_ctx* ctx, const double* G, int32_t m, int64_t ldg, double tol_rel, double* Li, int32_t* info);

/* ---------------------------------------------------- sample-sharded fit (API v6)
 * The fit collective of SURVEY §8(e): rank r holds uint8 rows X_r (n_r x d) on its GPU.
 * ef_fit_shard_stats: the exact integer pieces of the local rows —
 *   sum_out[d] = sum x, sumsq_out[d] = sum x^2 (uint64) per pixel,
 *   cross_out[d*d] (int64) = X'_r^T X'_r with X' = X - 128 (the upper 64 x 64 blocks exact,
 *   the rest of the matrix unspecified);
 * the caller sums the three arrays over ranks (an all-reduce, integer sum — e.g. RCCL
 * int64 over xGMI), then every rank calls
 * ef_fit_from_stats with the sums and n_total = sum n_r: mean / var / scale / components /
 *   eigenvalues / total variance exactly as ef_fit computes them on the concatenated rows
 *   (the same integers give the same covariance, bit for bit), covariance path only
 *   (n_total >= d; EF_FIT_STANDARDIZE as in ef_fit);
 * ef_fit_transform: the training projection (projected_data / fit_transform output) of
 *   local rows with a fitted model (mean[d], scale[d] or NULL = no StandardScaler,
 *   comps[k*d]) — the rows ef_fit's proj_out would hold for them.
 * Host pointers unless EF_MEM_DEVICE (then every array argument is a device pointer). */
int ef_fit_shard_stats(ef_ctx* ctx, const uint8_t* X, int64_t n, int64_t d, uint64_t* sum_out, uint64_t* sumsq_out,
                       int64_t* cross_out, uint32_t flags);
int ef_fit_from_stats(ef_ctx* ctx, const uint64_t* sum, const uint64_t* sumsq, const int64_t* cross, int64_t n_total,
                      int64_t d, int32_t k, uint32_t flags, double* mean_out, double* var_out, double* scale_out,
                      double* components_out, double* eigvals_out, double* total_var_out, int32_t* k_out,
                      int32_t* iters_out);
int ef_fit_transform(ef_ctx* ctx, const uint8_t* X, int64_t n, int64_t d, const double* mean, const double* scale,
                     const double* components, int32_t k, uint32_t flags, double* proj_out);

/* --------------------------------------------------------------- projection
 * Recognition model f = (p - mean) . W  (useless/scan.py:93-96; sklearn
 * scaler.transform + pca.transform folded, scan-template-v4.py:265-266).
 * mean[d], W[d*k] float32, row-major (d rows of k), 1 <= k <= 65536 (k > 512 is padded
 * to a multiple of 128: the full-rank per-person models of train-v5.py:539-545).  Kept
 * resident.
 * EF_MODEL_BF16: f = (p - round(mean)).bf16(W) - (mean - round(mean)).W with
 * fp32 accumulation (exact bf16 inputs for uint8 pixels; only W is rounded). */
int ef_model_set(ef_ctx* ctx, const float* mean, const float* W, int64_t d, int32_t k, uint32_t flags);
/* P[b*d] pixels (EF_U8 or EF_F32) -> F[b*k] float32. */
int ef_project(ef_ctx* ctx, const void* P, int32_t p_dtype, int64_t b, float* F, uint32_t flags);

/* ------------------------------------------------------------------ search
 * Gallery rows G[n*k] float32 (face_features / projected_data), kept resident; any
 * 1 <= k <= 65536 (as ef_model_set).
 * global_offset is added to every returned index (row sharding across ranks). */
int ef_gallery_set(ef_ctx* ctx, const float* G, int64_t n, int32_t k, int64_t global_offset,
                   uint32_t flags);
/* Q[b*k] float32 probe features -> keys[b].  A key packs the exact fp32 score
 * of the winning row in its high 32 bits (order-preserving) and the global
 * row index in its low 32 bits, so min over keys == argbest with lowest-index
 * tie-break; an all-reduce(MIN) over ranks combines sharded galleries. */
int ef_search(ef_ctx* ctx, const float* Q, int64_t b, int32_t metric, int64_t* keys, uint32_t flags);
/* Fused pipeline: project P then search; feats (b*k float32) optional. */
int ef_recognize(ef_ctx* ctx, const void* P, int32_t p_dtype, int64_t b, int32_t metric,
                 int64_t* keys, float* feats, uint32_t flags);
/* Host-side key decoding: L2 -> squared distance, COSINE -> similarity;
 * EF_KEY_NONE -> idx -1, best NaN. */
void ef_keys_decode(const int64_t* keys, int64_t b, int32_t metric, float* best, int64_t* idx);
/* Host-side introspection (no ctx, no GPU): the launches a search of b probes of k features
 * over an n-row gallery makes.  A batch whose padded probe block would pass 2 GiB (k > 512)
 * is searched in pieces of whole 256-probe tiles.  *n_pieces = the piece count; for the
 * first max_pieces pieces, pieces_out[6*i ..] = {first probe, probes, padded rows the
 * piece is launched with, probe tiles of its plan, gallery chunks, row tiles per chunk}.
 * split_bf16 as EF_OPT_SEARCH_SPLIT_BF16.  (API v6) */
int ef_search_schedule(int64_t b, int32_t k, int64_t n, int32_t split_bf16, int64_t* pieces_out, int32_t max_pieces,
                       int32_t* n_pieces);

/* ------------------------------------------------ exact cross-shard arg-best
 * A key's fp32 score cannot order two shards' winners whose fp64 scores differ by less
 * than one fp32 ulp, and a MIN over keys would then fall back to the lower index.  The
 * match record of a probe carries the winner's fp64 score, so shards merge exactly:
 *   score  fp64 score of the winning row (L2: squared distance; COSINE: -similarity;
 *          +inf with key == EF_KEY_NONE for an empty shard)
 *   scale  tie-tolerance scale (L2: |q|^2 + max |g|^2 of the shard; COSINE: 1)
 *   key    the packed key of ef_search (global row index in the low 32 bits)
 * Merging picks, per probe, the lowest global index among the parts whose score is within
 * 1e-12 * (|min score| + max scale) of the minimum — the rule a single engine applies to
 * its fp32-ambiguous candidates (np.argmin / np.argmax first-index semantics,
 * scan-template-v4.py:274-275). */
typedef struct ef_match {
  double score;
  double scale;
  int64_t key;
} ef_match;
int ef_search_matches(ef_ctx* ctx, const float* Q, int64_t b, int32_t metric, ef_match* out, uint32_t flags);
int ef_recognize_matches(ef_ctx* ctx, const void* P, int32_t p_dtype, int64_t b, int32_t metric, ef_match* out,
                         float* feats, uint32_t flags);
/* parts: nparts x b records (part-major) -> keys_out[b] (and merged records in merged_out,
 * optional).  Host pointers: computed on the host, ctx may be NULL (usable without a GPU).
 * EF_MEM_DEVICE: device pointers, stream-ordered on ctx's stream. */
int ef_matches_merge(ef_ctx* ctx, const ef_match* parts, int32_t nparts, int64_t b, int64_t* keys_out,
                     ef_match* merged_out, uint32_t flags);

/* ------------------------------------------------------------- multi-GPU (RCCL)
 * Row-sharded gallery across the ranks of one job, one process per GPU:
 * rank r sets its shard with ef_gallery_set(..., global_offset = first global row).
 * Once a communicator is attached, ef_search / ef_recognize (and the _matches forms) on
 * every rank return the GLOBAL result: each rank searches its shard, the match records
 * are all-gathered over RCCL (xGMI) and merged exactly (ef_matches_merge) on the ctx's
 * stream.  ef_recognize additionally splits the projection: rank r projects probes
 * [r*c, (r+1)*c), c = ceil(b / nranks), and the features are all-gathered.  Every rank
 * must make the same calls with the same b and metric (collectives).  RCCL is loaded at
 * run time (librccl.so.1); EF_E_STATE if it is unavailable.
 * ef_comm_unique_id: rank 0 creates the id (EF_UNIQUE_ID_BYTES bytes) and the caller
 * broadcasts it (e.g. over torch.distributed or MPI). */
#define EF_UNIQUE_ID_BYTES 128
int ef_comm_unique_id(void* id_out);
int ef_comm_init(ef_ctx* ctx, int32_t nranks, int32_t rank, const void* unique_id);
int ef_comm_destroy(ef_ctx* ctx);
int ef_comm_info(const ef_ctx* ctx, int32_t* nranks, int32_t* rank);

/* ------------------------------------------------------------------ options
 * Per-context tunables (defaults in brackets). */
#define EF_OPT_FIT_MAX_ITERS 1   /* subspace-iteration cap [500]; reaching it unconverged -> EF_E_NUMERIC */
#define EF_OPT_FIT_FP32_COARSE 2 /* 1 [default]: a coarse phase of reduced-precision C.Q products while
                                    the Ritz values still move (self-correcting; split-bf16 matrix-core
                                    products for a 256-wide block, fp32 otherwise); 2: the same with
                                    fp32 products; 0: fp64 products throughout */
#define EF_OPT_COV_SLAB_BYTES 3  /* device budget of the int32 covariance partial sums [8 GiB];
                                    smaller budgets run the multi-pass int64 schedule */
#define EF_OPT_TM_INT64_SUMS 4   /* 1: int64 integral images in the template localiser [0: auto] */
#define EF_OPT_HAAR_ORDERED 5    /* 1: sequential stage sums even when reassociation is exact [0] */
#define EF_OPT_JPEG_CHUNK_BITS 6 /* entropy-decode chunk per GPU thread, bits (multiple of 32) [0: auto] */
#define EF_OPT_SEARCH_SPLIT_BF16 7 /* 1: gallery scans on bf16 MFMA with split (hi + lo) fp32 operands
                                      and a widened error bound; identities and scores are still
                                      fp64-resolved, so results equal the fp32 scan's [0]; 2: the same
                                      with the 32x32x16 kernel at k in (64, 128] (comparison); 3: at
                                      k > 128 a single-bf16 screen (one bf16 MFMA per product, fp32
                                      accumulation, a bf16-wide bound) — still fp64-resolved, same
                                      results, fewer MFMAs; more probes reach the resolution when
                                      the best two rows are within ~2% (k <= 128: as 1) */
#define EF_OPT_JPEG_PART_FILES 8   /* ef_jpeg_ingest decodes in parts of this many files, staging
                                      part i + 1 on a host thread while part i decodes [8192] */
#define EF_OPT_FIT_CHEBYSHEV 9     /* 1 [default]: the subspace iteration advances a Chebyshev
                                      three-term recurrence on [0, theta_m] between Rayleigh-Ritz
                                      steps; 0: one shifted power step per iteration */
#define EF_OPT_HOST_THREADS 10     /* host worker threads for the JPEG parse / destuff, PROCESS-WIDE
                                      (any context sets it) [0: min(16, hardware threads)]; the
                                      Python Engine sets the job's CPU share (API v7) */
int ef_set_option(ef_ctx* ctx, int32_t option, int64_t value);
int ef_get_option(const ef_ctx* ctx, int32_t option, int64_t* value);

/* ------------------------------------------------------------------ ingest
 * Replaces the per-image cv2.cvtColor(img, COLOR_BGR2GRAY) + cv2.resize(gray, (w, h))
 * (INTER_LINEAR) of train-v4.py:59-68 and scan-template-v4.py:257-263 for a ragged
 * batch of decoded images in one launch, with OpenCV's CV_8U fixed-point arithmetic
 * (parity against OpenCV unpinned: OpenCV is not installed where this was built).
 * Image i: heights[i] x widths[i] x channels[i] (1, 3 = BGR, 4 = BGRA; EF_IMG_RGB for
 * RGB order; channels NULL = all 1) uint8 pixels at data + offsets[i], row-major.
 * out: count x out_h x out_w uint8 (the probe / training row layout, train-v4.py:68).
 * data/out are host pointers, or device pointers with EF_MEM_DEVICE; the metadata
 * arrays are always host arrays.  At most 65535 images per call. */
int ef_preprocess(ef_ctx* ctx, const uint8_t* data, const int64_t* offsets, const int32_t* heights,
                  const int32_t* widths, const int32_t* channels, int64_t count, int32_t out_h,
                  int32_t out_w, uint8_t* out, uint32_t flags);

/* ------------------------------------------------------------------ JPEG decode
 * Replaces the per-file cv2.imread of the ingest paths (train-v4.py:59 IMREAD_COLOR;
 * useless/train.py:33 and scan-template-v4.py:52 IMREAD_GRAYSCALE) for a batch of
 * JPEG files: image i is sizes[i] bytes at data + offsets[i] (data is always a host
 * pointer).  Decoded on the GPU with libjpeg-turbo's default arithmetic (islow IDCT,
 * fancy upsampling, its YCbCr->RGB tables), so the pixels equal what imread returns:
 *   EF_JPEG_GRAY  h x w luma (libjpeg JCS_GRAYSCALE output, IMREAD_GRAYSCALE)
 *   EF_JPEG_BGR   h x w x 3 BGR (IMREAD_COLOR)
 * written at out + out_offsets[i] (host, or device with EF_MEM_DEVICE — then the
 * pixels can go straight into ef_preprocess with EF_MEM_DEVICE).  Supported: sequential
 * Huffman (SOF0/SOF1) 8-bit, 1 or 3 components, luma at the maximal sampling factors,
 * chroma at 1x or 2x horizontally and vertically (4:4:4, 4:2:2, 4:2:0), one scan,
 * restart intervals.  status[i] (optional) is 0, or EF_JPEG_E_UNSUPPORTED /
 * EF_JPEG_E_CORRUPT for a file the caller must decode on the host (nothing is written
 * for it).  ef_jpeg_info parses the headers on the host (no context, no GPU). */
#define EF_JPEG_GRAY 0
#define EF_JPEG_BGR 1
#define EF_JPEG_E_UNSUPPORTED (-10)
#define EF_JPEG_E_CORRUPT (-11)
int ef_jpeg_info(const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int32_t count, int32_t* heights,
                 int32_t* widths, int32_t* components, int32_t* status);
int ef_jpeg_decode(ef_ctx* ctx, const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int32_t count,
                   int32_t mode, uint8_t* out, const int64_t* out_offsets, int32_t* status, uint32_t flags);
/* Fused ingest (train-v4.py:59-68 for a batch of files): decode, then ef_preprocess's
 * grey + INTER_LINEAR resize to out_h x out_w computed straight from the decoded planes
 * (the same pixels as ef_jpeg_decode followed by ef_preprocess).  out: count x out_h x out_w
 * uint8 rows (host, or device with EF_MEM_DEVICE); the row of a file with status[i] != 0 is
 * zero and the caller decodes that file itself.  status is final on return.  With
 * EF_MEM_DEVICE the rows are stream-ordered on ctx's stream and the call returns once the
 * decode is queued (no host wait), so the next call's host-side parse overlaps this
 * decode; ef_jpeg_decode with EF_MEM_DEVICE behaves the same.  Host outputs return complete. */
int ef_jpeg_ingest(ef_ctx* ctx, const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int32_t count,
                   int32_t mode, int32_t out_h, int32_t out_w, uint8_t* out, int32_t* status, uint32_t flags);

/* -------------------------------------------------------- template localiser
 * Replaces template_match_all_models' inner loops (scan-template-v4.py:127-200):
 * for every problem p = (template t, scaled size h x w):
 *   R_p = cv2.matchTemplate(frame, cv2.resize(template_t, (w, h)), TM_CCOEFF_NORMED)
 *   (best, (x, y)) = cv2.minMaxLoc(R_p) maximum (first in raster order).
 * The correlation is exact (int8 matrix cores, int64 sums); the normalisation follows
 * OpenCV's rule in float64, R is float32.  ef_tm_prepare uploads the grey templates
 * (templ_h[i] x templ_w[i] at templ_data + templ_offsets[i]), resizes them on the GPU
 * and builds the resident operands for a frame_h x frame_w frame; ef_tm_match then
 * runs one frame (row stride frame_ld bytes) and returns per problem best_out, x_out,
 * y_out (each optional) and, if maps_out is non-NULL, every R_p concatenated
 * (sizes from ef_tm_info).  Host pointers unless EF_MEM_DEVICE. */
int ef_tm_prepare(ef_ctx* ctx, const uint8_t* templ_data, const int64_t* templ_offsets,
                  const int32_t* templ_h, const int32_t* templ_w, int32_t n_templates,
                  const int32_t* prob_templ, const int32_t* prob_h, const int32_t* prob_w,
                  int32_t n_problems, int32_t frame_h, int32_t frame_w, uint32_t flags);
int ef_tm_match(ef_ctx* ctx, const uint8_t* frame, int64_t frame_ld, float* best_out, int32_t* x_out,
                int32_t* y_out, float* maps_out, uint32_t flags);
int ef_tm_info(ef_ctx* ctx, int32_t* n_problems, int64_t* map_elems, int32_t* result_h,
               int32_t* result_w);
/* Host-only (API v7): the integral-image width ef_tm_prepare picks for a frame_h x frame_w
 * frame whose largest template area is max_template_area: 32 (wrapping uint32 sums) when
 * every area is < 2^18 and (frame_h + 1)(frame_w + 1) < 2^30, else 64 (int64 sums); the
 * EF_OPT_TM_INT64_SUMS option forces 64 per context.  EF_E_INVALID on bad sizes. */
int ef_tm_sums_bits(int32_t frame_h, int32_t frame_w, int64_t max_template_area);

/* --------------------------------------------------------- Haar cascade detector
 * Replaces face_cascade.detectMultiScale(gray, scaleFactor, minNeighbors, minSize)
 * (detection-v4.py:18, :50-55) for a stump-based HAAR cascade as OpenCV stores it
 * (stages of depth-1 trees over up-to-3-rectangle features, no tilted features):
 *   features i: rects[i][k] = {x, y, w, h} in window coordinates, weights[i][k] (k < 3,
 *               weight 0 = unused third rectangle);
 *   stages s:   stage_count[s] consecutive stumps, stage_threshold[s];
 *   stumps j:   feature index, threshold, left leaf (value < threshold), right leaf.
 * ef_haar_detect runs the image pyramid, variance normalisation and cascade on the GPU
 * and cv::groupRectangles(min_neighbors, 0.2) on the host; rects_out holds up to
 * max_rects {x, y, w, h}, *n_rects the total; cand_out (optional) the ungrouped
 * candidates in OpenCV's (scale, y, x) order.  max_w/max_h <= 0 means the frame size.
 * The frame is a host pointer (row stride ld) unless EF_MEM_DEVICE.  Parity against
 * OpenCV is unpinned (OpenCV and its cascade files are absent where this was built);
 * OpenCV's pyramid uses INTER_LINEAR_EXACT, this one INTER_LINEAR. */
int ef_haar_set_cascade(ef_ctx* ctx, int32_t win_w, int32_t win_h, int32_t n_features, const int32_t* rects,
                        const float* weights, int32_t n_stages, const int32_t* stage_count,
                        const float* stage_threshold, int32_t n_stumps, const int32_t* stump_feature,
                        const float* stump_threshold, const float* stump_left, const float* stump_right);
int ef_haar_detect(ef_ctx* ctx, const uint8_t* gray, int32_t h, int32_t w, int64_t ld, double scale_factor,
                   int32_t min_neighbors, int32_t min_w, int32_t min_h, int32_t max_w, int32_t max_h,
                   int32_t* rects_out, int32_t max_rects, int32_t* n_rects, int32_t* cand_out, int32_t max_cand,
                   int32_t* n_cand, uint32_t flags);

/* ------------------------------------------------------------------ timing
 * Device time of each launch of a kernel, measured with hipEvents on the
 * stream the kernel is launched on. */
int ef_timing_enable(ef_ctx* ctx, int on);
int ef_timing_get(ef_ctx* ctx, int32_t kernel_id, double* total_ms, int64_t* launches);
int ef_timing_reset(ef_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* EIGENFACE_H_ */
