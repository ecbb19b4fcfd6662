"""Thin Python layer over the C ABI: one ``Engine`` per GPU.

Arrays may be NumPy (host; the call copies in/out and synchronises) or torch-ROCm
CUDA tensors (device; zero-copy, stream-ordered, no synchronisation).  One call must
not mix the two.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import sys
from dataclasses import dataclass

import numpy as np

from . import _native as N

METRICS = {"l2": N.EF_METRIC_L2, "cosine": N.EF_METRIC_COSINE}


def _is_dev(x):
    return x is not None and hasattr(x, "data_ptr") and getattr(x, "is_cuda", False)


def _host(x, dtype):
    a = np.ascontiguousarray(x, dtype=dtype)
    return a, a.ctypes.data


def _dev(x, torch_dtype):
    if x.dtype != torch_dtype:
        raise TypeError(f"expected {torch_dtype}, got {x.dtype}")
    if not x.is_contiguous():
        x = x.contiguous()
    return x, x.data_ptr()


_OPTIONS = {"fit_max_iters": N.EF_OPT_FIT_MAX_ITERS, "fit_fp32_coarse": N.EF_OPT_FIT_FP32_COARSE,
            "cov_slab_bytes": N.EF_OPT_COV_SLAB_BYTES, "tm_int64_sums": N.EF_OPT_TM_INT64_SUMS,
            "haar_ordered": N.EF_OPT_HAAR_ORDERED, "jpeg_chunk_bits": N.EF_OPT_JPEG_CHUNK_BITS,
            "search_split_bf16": N.EF_OPT_SEARCH_SPLIT_BF16, "jpeg_part_files": N.EF_OPT_JPEG_PART_FILES,
            "fit_chebyshev": N.EF_OPT_FIT_CHEBYSHEV, "host_threads": N.EF_OPT_HOST_THREADS}


def host_cpu_share():
    """The job's CPU share for the library's host workers: OMP_NUM_THREADS when set (the
    GPU pool presets it to the job's share), else the affinity mask, capped at 16."""
    share = None
    v = os.environ.get("OMP_NUM_THREADS", "")
    if v.strip().isdigit() and int(v) > 0:
        share = int(v)
    if share is None:
        try:
            share = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            share = os.cpu_count() or 1
    return max(1, min(16, share))


def _option(o):
    return _OPTIONS[o] if isinstance(o, str) else int(o)


def _metric(m):
    if isinstance(m, str):
        return METRICS[m.lower()]
    return int(m)


@dataclass
class FitResult:
    """Outputs of the GPU fit (float64).  ``components`` is k x d (rows =
    eigenfaces, sklearn ``components_``); manual_pca's ``eigenfaces`` is its
    transpose."""

    mean: np.ndarray
    var: np.ndarray
    scale: np.ndarray
    components: np.ndarray
    eigenvalues: np.ndarray
    projection: np.ndarray | None
    total_var: float
    k: int
    iters: int


_TORCH_READY = False


def _init_torch_first():
    """torch's HIP runtime must come up before this process's first libeigenface context,
    or torch reports no GPU afterwards (seen on the MI355X boxes) — so when torch is
    installed it is initialised here, whether or not the caller imported it yet."""
    global _TORCH_READY
    if _TORCH_READY:
        return
    _TORCH_READY = True
    torch = sys.modules.get("torch")
    if torch is None:
        import importlib.util
        if importlib.util.find_spec("torch") is None:
            return
        import torch
    if torch.cuda.is_available():
        torch.cuda.init()


class Engine:
    """A libeigenface context bound to one HIP device."""

    def __init__(self, device: int = 0):
        self._lib = N.lib()
        _init_torch_first()
        h = C.c_void_p()
        rc = self._lib.ef_create(int(device), C.byref(h))
        if rc != N.EF_OK:
            raise N.EigenfaceError(rc, f"ef_create(device={device}) failed (no usable HIP device?)")
        self._h = h
        self.device = int(device)
        self._chk(self._lib.ef_set_option(h, N.EF_OPT_HOST_THREADS, host_cpu_share()))
        # The engine's own stream is a torch pool stream when torch is present: pool streams
        # live as long as the process, so a tensor marked with record_stream (_torch_order)
        # never outlives the stream it was recorded on.  A stream the library created would
        # be destroyed by close() while such a tensor, freed later, still records an event
        # on it (a host crash at free time).
        self._pool_stream = None
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_available():
            self._pool_stream = torch.cuda.Stream(device=self.device)
            self._chk(self._lib.ef_set_stream(h, C.c_void_p(self._pool_stream.cuda_stream)))
        self.model_k = None
        self.model_d = None
        self.gallery_n = 0
        self.gallery_k = None
        # Owner tokens of the resident model / gallery: whoever uploads them last owns them.
        # Callers that cache "my model is resident" (EigenfacePCA, recognize_face_with_model)
        # compare their token with these instead of assuming nobody else replaced it.
        self.model_owner = None
        self.gallery_owner = None

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.ef_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc):
        return N.check(self._h, rc)

    def set_stream(self, stream_handle):
        """Launch on an external hipStream_t (int handle, e.g. torch's
        ``current_stream().cuda_stream``; 0 is the default stream)."""
        self._chk(self._lib.ef_set_stream(self._h, C.c_void_p(int(stream_handle) or None)))

    def use_own_stream(self):
        """Back to the engine's own non-blocking stream (its torch pool stream, or the
        library's stream without torch)."""
        if self._pool_stream is not None:
            self.set_stream(self._pool_stream.cuda_stream)
        else:
            self._chk(self._lib.ef_use_own_stream(self._h))

    def synchronize(self):
        self._chk(self._lib.ef_synchronize(self._h))

    def stream_handle(self) -> int:
        """The hipStream_t the engine launches on (0 = the default stream)."""
        s = C.c_void_p()
        self._chk(self._lib.ef_get_stream(self._h, C.byref(s)))
        return int(s.value or 0)

    @contextlib.contextmanager
    def _torch_order(self, *tensors):
        """Stream order of a call on device tensors when the engine runs on its own stream:
        the engine's stream first waits for torch's current stream (the inputs' producers),
        then torch's current stream waits for the engine's (the outputs' consumers), and
        every tensor the call reads or writes — inputs included, e.g. a dtype-converted
        temporary that dies when the wrapper returns — is marked as used on the engine's
        stream, so the caching allocator hands its memory to no other stream before the
        engine's kernels are done.  The mark is made only on streams that live as long as
        the process (the engine's torch pool stream, the default stream): a tensor freed
        after its stream was destroyed would crash the allocator; on a caller's external
        stream (set_stream) inputs are safe to reuse on torch's current stream only.  No
        host wait either way; a no-op when the engine already runs on torch's stream."""
        import torch
        h = self.stream_handle()
        cur = torch.cuda.current_stream(self.device)
        if h == cur.cuda_stream:
            yield
            return
        pool = self._pool_stream
        if pool is not None and h == pool.cuda_stream:
            ext = pool
        else:
            ext = torch.cuda.ExternalStream(h, device=self.device) if h else torch.cuda.default_stream(self.device)
        ext.wait_stream(cur)
        yield
        cur.wait_stream(ext)
        if ext is pool or not h:
            for t in tensors:
                if t is not None:
                    t.record_stream(ext)

    def trim(self):
        """Free the fit workspaces the context keeps between fits (ef_trim)."""
        self._chk(self._lib.ef_trim(self._h))

    def chol_inv(self, G, tol_rel=1e-13, Li=None):
        """The fit's CholQR factor alone (ef_chol_inv): (Li, info) with Li = L^-1 for
        G = L L^T (1 <= m <= 256).  On a failed pivot info = -(column + 1) and Li is returned
        as given (zeros by default)."""
        G = np.ascontiguousarray(G, dtype=np.float64)
        m = int(G.shape[0])
        L = np.zeros((m, m), np.float64) if Li is None else np.array(Li, dtype=np.float64, order="C", copy=True)
        info = C.c_int32(0)
        self._chk(self._lib.ef_chol_inv(self._h, G.ctypes.data, m, int(G.shape[1]), float(tol_rel), L.ctypes.data,
                                        C.byref(info)))
        return L, int(info.value)

    def set_option(self, option, value):
        """Context tunable (include/eigenface.h EF_OPT_*): "fit_max_iters",
        "fit_fp32_coarse", "cov_slab_bytes", "tm_int64_sums", "haar_ordered", "jpeg_chunk_bits",
        "search_split_bf16", "jpeg_part_files", "fit_chebyshev", "host_threads" (process-wide) or
        the code."""
        self._chk(self._lib.ef_set_option(self._h, _option(option), int(value)))

    def get_option(self, option):
        v = C.c_int64(0)
        self._chk(self._lib.ef_get_option(self._h, _option(option), C.byref(v)))
        return int(v.value)

    # --------------------------------------------------------------- multi-GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        """A fresh RCCL unique id (rank 0 creates it; broadcast it to the other ranks)."""
        buf = C.create_string_buffer(N.EF_UNIQUE_ID_BYTES)
        rc = N.lib().ef_comm_unique_id(buf)
        if rc != N.EF_OK:
            raise N.EigenfaceError(rc, "ef_comm_unique_id failed (RCCL unavailable?)")
        return bytes(buf.raw)

    def comm_init(self, nranks: int, rank: int, unique_id: bytes):
        """Attach an in-library RCCL communicator (ef_comm_init): from now on search /
        recognize return the global result over the row-sharded gallery."""
        if len(unique_id) != N.EF_UNIQUE_ID_BYTES:
            raise ValueError("unique_id must be EF_UNIQUE_ID_BYTES bytes")
        buf = C.create_string_buffer(bytes(unique_id), N.EF_UNIQUE_ID_BYTES)
        self._chk(self._lib.ef_comm_init(self._h, int(nranks), int(rank), buf))

    def comm_destroy(self):
        self._chk(self._lib.ef_comm_destroy(self._h))

    def comm_info(self):
        n, r = C.c_int32(0), C.c_int32(0)
        self._chk(self._lib.ef_comm_info(self._h, C.byref(n), C.byref(r)))
        return int(n.value), int(r.value)

    # ------------------------------------------------------------------------ fit
    @staticmethod
    def _fit_input(X):
        """(array, pointer, EF dtype, on device) of fit input: uint8 pixels (exact integer
        kernels) or float32 / float64 data (fp64 loaders; include/eigenface.h ef_fit_ex)."""
        if _is_dev(X):
            import torch
            codes = {torch.uint8: N.EF_U8, torch.float32: N.EF_F32, torch.float64: N.EF_F64}
            if X.dtype not in codes:
                raise TypeError(f"fit input must be uint8, float32 or float64, got {X.dtype}")
            x, xp = _dev(X, X.dtype)
            return x, xp, codes[X.dtype], True
        a = np.asarray(X)
        if a.dtype == np.uint8:
            code, dt = N.EF_U8, np.uint8
        elif a.dtype == np.float32:
            code, dt = N.EF_F32, np.float32
        else:
            code, dt = N.EF_F64, np.float64
        x, xp = _host(a, dt)
        return x, xp, code, False

    def fit(self, X, n_components: int, standardize: bool = False, projection: bool = True) -> FitResult:
        """GPU eigenfaces fit of faces X (n x d); see include/eigenface.h ef_fit / ef_fit_ex.

        X is uint8 pixels, or float32 / float64 data (e.g. ManualStandardScaler output,
        scripts/manual/train-v2.py:194-197).  It may be a host array or a device torch
        tensor; for a device X the outputs stay on the device (float64 torch tensors,
        EF_MEM_DEVICE)."""
        x, xp, xdt, dev = self._fit_input(X)
        if dev:
            import torch
        if x.ndim != 2:
            raise ValueError("X must be 2-D (n_samples, n_pixels)")
        n, d = (int(v) for v in x.shape)
        k = int(n_components)
        kk = min(k, n if n < d else d)
        if dev:
            def alloc(*shape):
                return torch.empty(shape, dtype=torch.float64, device=x.device)

            def ptr(a):
                return a.data_ptr()
        else:
            def alloc(*shape):
                return np.empty(shape)

            def ptr(a):
                return a.ctypes.data
        mean, var, scale = alloc(d), alloc(d), alloc(d)
        comps, eig = alloc(kk, d), alloc(kk)
        proj = alloc(n, kk) if projection else None
        tv = alloc(1)
        k_out = C.c_int32(0)
        it = C.c_int32(0)
        flags = (N.EF_FIT_STANDARDIZE if standardize else 0) | (N.EF_MEM_DEVICE if dev else 0)
        with (self._torch_order(x, mean, var, scale, comps, eig, proj, tv) if dev else contextlib.nullcontext()):
            self._chk(self._lib.ef_fit_ex(
                self._h, xp, xdt, n, d, k, flags, ptr(mean), ptr(var), ptr(scale), ptr(comps), ptr(eig),
                ptr(proj) if proj is not None else None, ptr(tv), C.byref(k_out), C.byref(it)))
        if dev:
            self.synchronize()
        return FitResult(mean, var, scale, comps, eig, proj, float(tv[0]), int(k_out.value), int(it.value))

    def colstats(self, X):
        """Column mean and population variance (float64) of X (n x d, uint8 / float32 /
        float64; ef_colstats): np.mean / np.var(axis=0) on the GPU — exact integer sums for
        uint8, two-pass fp64 for floats.  Host input -> numpy, device input -> tensors."""
        x, xp, xdt, dev = self._fit_input(X)
        if x.ndim != 2 or x.shape[0] < 1 or x.shape[1] < 1:
            raise ValueError("X must be 2-D (n_samples >= 1, n_features >= 1)")
        n, d = (int(v) for v in x.shape)
        if dev:
            import torch
            mean = torch.empty(d, dtype=torch.float64, device=x.device)
            var = torch.empty(d, dtype=torch.float64, device=x.device)
            with self._torch_order(x, mean, var):
                self._chk(self._lib.ef_colstats(self._h, xp, xdt, n, d, N.EF_MEM_DEVICE, mean.data_ptr(),
                                                var.data_ptr()))
            self.synchronize()
            return mean, var
        mean, var = np.empty(d), np.empty(d)
        self._chk(self._lib.ef_colstats(self._h, xp, xdt, n, d, 0, mean.ctypes.data, var.ctypes.data))
        return mean, var

    # --------------------------------------------------------- sample-sharded fit
    def fit_shard_stats(self, X):
        """ef_fit_shard_stats: the exact integer pieces of this rank's uint8 rows X (n x d) —
        (sum x [d], sum x^2 [d], X'^T X' [d, d] with X' = X - 128, upper 64-blocks exact) as
        int64 arrays: torch tensors on X's device for a device X, numpy otherwise.  Summed
        over ranks they are the pieces of the whole set (distributed.sharded_fit)."""
        x, xp, xdt, dev = self._fit_input(X)
        if xdt != N.EF_U8 or x.ndim != 2:
            raise TypeError("fit_shard_stats takes 2-D uint8 pixels")
        n, d = (int(v) for v in x.shape)
        if dev:
            import torch
            s1 = torch.empty(d, dtype=torch.int64, device=x.device)
            s2 = torch.empty(d, dtype=torch.int64, device=x.device)
            cr = torch.empty((d, d), dtype=torch.int64, device=x.device)
            with self._torch_order(x, s1, s2, cr):
                self._chk(self._lib.ef_fit_shard_stats(self._h, xp, n, d, s1.data_ptr(), s2.data_ptr(),
                                                       cr.data_ptr(), N.EF_MEM_DEVICE))
            return s1, s2, cr
        s1, s2 = np.empty(d, np.int64), np.empty(d, np.int64)
        cr = np.empty((d, d), np.int64)
        self._chk(self._lib.ef_fit_shard_stats(self._h, xp, n, d, s1.ctypes.data, s2.ctypes.data, cr.ctypes.data, 0))
        return s1, s2, cr

    def fit_from_stats(self, sums, sumsqs, cross, n_total: int, n_components: int, standardize: bool = False) -> FitResult:
        """ef_fit_from_stats: the fit (covariance path, n_total >= d) from the pieces of
        fit_shard_stats summed over every rank — equal to fit() on the concatenated rows bit
        for bit (projection None: see fit_transform_rows).  Device pieces give device
        (float64 torch) outputs."""
        if _is_dev(sums):
            import torch
            s1, p1 = _dev(sums, torch.int64)
            s2, p2 = _dev(sumsqs, torch.int64)
            cr, p3 = _dev(cross, torch.int64)
            d = int(s1.shape[0])
            kk = min(int(n_components), d)

            def alloc(*shape):
                return torch.empty(shape, dtype=torch.float64, device=s1.device)

            def ptr(a):
                return a.data_ptr()
            flags = N.EF_MEM_DEVICE
        else:
            s1, p1 = _host(np.asarray(sums), np.int64)
            s2, p2 = _host(np.asarray(sumsqs), np.int64)
            cr, p3 = _host(np.asarray(cross), np.int64)
            d = int(s1.shape[0])
            kk = min(int(n_components), d)

            def alloc(*shape):
                return np.empty(shape)

            def ptr(a):
                return a.ctypes.data
            flags = 0
        if tuple(cr.shape) != (d, d) or tuple(s2.shape) != (d,):
            raise ValueError(f"pieces must be sum[{d}], sumsq[{d}], cross[{d}, {d}]")
        mean, var, scale = alloc(d), alloc(d), alloc(d)
        comps, eig, tv = alloc(kk, d), alloc(kk), alloc(1)
        k_out, it = C.c_int32(0), C.c_int32(0)
        flags |= N.EF_FIT_STANDARDIZE if standardize else 0
        ctx = self._torch_order(s1, s2, cr, mean, var, scale, comps, eig, tv) if flags & N.EF_MEM_DEVICE \
            else contextlib.nullcontext()
        with ctx:
            self._chk(self._lib.ef_fit_from_stats(self._h, p1, p2, p3, int(n_total), d, int(n_components), flags,
                                                  ptr(mean), ptr(var), ptr(scale), ptr(comps), ptr(eig), ptr(tv),
                                                  C.byref(k_out), C.byref(it)))
        if flags & N.EF_MEM_DEVICE:
            self.synchronize()
        return FitResult(mean, var, scale, comps, eig, None, float(tv[0]), int(k_out.value), int(it.value))

    def fit_transform_rows(self, X, result: FitResult, standardize: bool = False):
        """ef_fit_transform: the training projection of uint8 rows X with a fitted model —
        the rows fit()'s projection holds for them (the sample-sharded fit projects each
        rank's own rows)."""
        x, xp, xdt, dev = self._fit_input(X)
        if xdt != N.EF_U8 or x.ndim != 2:
            raise TypeError("fit_transform_rows takes 2-D uint8 pixels")
        n, d = (int(v) for v in x.shape)
        k = int(result.k)
        if dev:
            import torch
            mean, pm = _dev(result.mean, torch.float64)
            comps, pc = _dev(result.components, torch.float64)
            sc, ps = _dev(result.scale, torch.float64) if standardize else (None, None)
            out = torch.empty((n, k), dtype=torch.float64, device=x.device)
            with self._torch_order(x, mean, comps, sc, out):
                self._chk(self._lib.ef_fit_transform(self._h, xp, n, d, pm, ps, pc, k, N.EF_MEM_DEVICE,
                                                     out.data_ptr()))
            return out
        mean, pm = _host(np.asarray(result.mean), np.float64)
        comps, pc = _host(np.asarray(result.components), np.float64)
        sc, ps = _host(np.asarray(result.scale), np.float64) if standardize else (None, None)
        out = np.empty((n, k))
        self._chk(self._lib.ef_fit_transform(self._h, xp, n, d, pm, ps, pc, k, 0, out.ctypes.data))
        return out

    # ----------------------------------------------------------------- projection
    def set_model(self, mean, W, precision="fp32", owner=None):
        """Resident recognition model f = (p - mean) . W, W is d x k (k <= 512).

        precision="bf16" projects on bf16 MFMA (BASELINE.json config 5):
        f = (p - round(mean)).bf16(W) - (mean - round(mean)).W, fp32 accumulation;
        features, gallery search and arg-best stay fp32 (fp64-resolved)."""
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        if _is_dev(W):
            import torch
            m, mp = _dev(mean, torch.float32)
            w, wp = _dev(W, torch.float32)
            flags = N.EF_MEM_DEVICE
        else:
            m, mp = _host(mean, np.float32)
            w, wp = _host(W, np.float32)
            flags = 0
        d, k = w.shape
        if m.shape[0] != d:
            raise ValueError("mean and W disagree on d")
        if precision == "bf16":
            flags |= N.EF_MODEL_BF16
        self.model_owner = None  # a failed upload leaves no valid owner
        self._chk(self._lib.ef_model_set(self._h, mp, wp, d, k, flags))
        if flags:
            self.synchronize()
        self.model_d, self.model_k = int(d), int(k)
        self.model_owner = owner if owner is not None else object()

    def _dev_pixels(self, P):
        """Validated device probe pixels: (b, model_d) uint8 or float32, contiguous."""
        import torch
        if P.dtype not in (torch.uint8, torch.float32):
            raise TypeError(f"probe pixels must be uint8 or float32, got {P.dtype}")
        if P.ndim != 2 or P.shape[1] != self.model_d:
            raise ValueError(f"P must be (b, {self.model_d}), got {tuple(P.shape)}")
        p, pp = _dev(P, P.dtype)
        return p, pp, (N.EF_U8 if P.dtype == torch.uint8 else N.EF_F32)

    @staticmethod
    def _dev_out(t, shape, dtype, what):
        if t.dtype != dtype or tuple(t.shape) != tuple(shape) or not t.is_contiguous():
            raise ValueError(f"{what} must be a contiguous {dtype} tensor of shape {tuple(shape)}")
        return t

    def project(self, P, out=None):
        if self.model_k is None:
            raise RuntimeError("no model: call set_model first")
        if _is_dev(P):
            import torch
            p, pp, dtype = self._dev_pixels(P)
            b = p.shape[0]
            if out is None:
                out = torch.empty((b, self.model_k), dtype=torch.float32, device=p.device)
            self._dev_out(out, (b, self.model_k), torch.float32, "out")
            with self._torch_order(p, out):
                self._chk(self._lib.ef_project(self._h, pp, dtype, b, out.data_ptr(), N.EF_MEM_DEVICE))
            return out
        p = np.asarray(P)
        dtype = N.EF_U8 if p.dtype == np.uint8 else N.EF_F32
        p, pp = _host(p, np.uint8 if dtype == N.EF_U8 else np.float32)
        if p.ndim != 2 or p.shape[1] != self.model_d:
            raise ValueError("P must be (b, d)")
        b = p.shape[0]
        f = np.empty((b, self.model_k), dtype=np.float32)
        self._chk(self._lib.ef_project(self._h, pp, dtype, b, f.ctypes.data, 0))
        return f

    # --------------------------------------------------------------------- search
    def set_gallery(self, G, global_offset: int = 0, owner=None):
        if _is_dev(G):
            import torch
            g, gp = _dev(G, torch.float32)
            flags = N.EF_MEM_DEVICE
        else:
            g, gp = _host(G, np.float32)
            flags = 0
        if g.ndim != 2:
            raise ValueError("gallery must be 2-D (n, k)")
        n, k = g.shape
        self.gallery_owner = None
        self._chk(self._lib.ef_gallery_set(self._h, gp, n, k, int(global_offset), flags))
        self.gallery_n, self.gallery_k = int(n), int(k)
        self.gallery_owner = owner if owner is not None else object()

    def search_keys(self, Q, metric="l2", keys=None):
        """Packed keys (int64) of the best gallery row per probe."""
        mt = _metric(metric)
        if self.gallery_k is None:
            raise RuntimeError("no gallery: call set_gallery first")
        if _is_dev(Q):
            import torch
            q, qp = _dev(Q, torch.float32)
            if q.ndim != 2 or q.shape[1] != self.gallery_k:
                raise ValueError(f"Q must be (b, {self.gallery_k}), got {tuple(q.shape)}")
            b = q.shape[0]
            if keys is None:
                keys = torch.empty(b, dtype=torch.int64, device=q.device)
            self._dev_out(keys, (b,), torch.int64, "keys")
            with self._torch_order(q, keys):
                self._chk(self._lib.ef_search(self._h, qp, b, mt, keys.data_ptr(), N.EF_MEM_DEVICE))
            return keys
        q, qp = _host(Q, np.float32)
        if q.ndim != 2 or q.shape[1] != self.gallery_k:
            raise ValueError(f"Q must be (b, {self.gallery_k}), got {q.shape}")
        b = q.shape[0]
        k = np.empty(b, dtype=np.int64)
        self._chk(self._lib.ef_search(self._h, qp, b, mt, k.ctypes.data, 0))
        return k

    def search(self, Q, metric="l2"):
        """Return (idx int64, best float32): L2 -> squared distance, cosine -> similarity."""
        keys = self.search_keys(Q, metric)
        if _is_dev(keys):
            keys = keys.cpu().numpy()
        return decode_keys(keys, metric)

    def recognize_keys(self, P, metric="l2", keys=None, feats=None):
        """Fused projection + search (device or host)."""
        mt = _metric(metric)
        if self.model_k is None or self.gallery_k is None:
            raise RuntimeError("recognize needs a model and a gallery")
        if _is_dev(P):
            import torch
            p, pp, dtype = self._dev_pixels(P)
            b = p.shape[0]
            if keys is None:
                keys = torch.empty(b, dtype=torch.int64, device=p.device)
            self._dev_out(keys, (b,), torch.int64, "keys")
            fp = None
            if feats is not None:
                fp = self._dev_out(feats, (b, self.model_k), torch.float32, "feats").data_ptr()
            with self._torch_order(p, keys, feats):
                self._chk(self._lib.ef_recognize(self._h, pp, dtype, b, mt, keys.data_ptr(), fp, N.EF_MEM_DEVICE))
            return keys
        p = np.asarray(P)
        dtype = N.EF_U8 if p.dtype == np.uint8 else N.EF_F32
        p, pp = _host(p, np.uint8 if dtype == N.EF_U8 else np.float32)
        if p.ndim != 2 or p.shape[1] != self.model_d:
            raise ValueError(f"P must be (b, {self.model_d}), got {p.shape}")
        b = p.shape[0]
        k = np.empty(b, dtype=np.int64)
        fp = None
        if feats is not None:
            if not (isinstance(feats, np.ndarray) and feats.dtype == np.float32 and feats.shape == (b, self.model_k)
                    and feats.flags.c_contiguous):
                raise ValueError(f"feats must be a contiguous float32 array of shape {(b, self.model_k)}")
            fp = feats.ctypes.data
        self._chk(self._lib.ef_recognize(self._h, pp, dtype, b, mt, k.ctypes.data, fp, 0))
        return k

    # ------------------------------------------------------- exact match records
    def search_matches(self, Q, metric="l2", out=None):
        """ef_search_matches: per-probe (fp64 score, scale, key) records (numpy structured
        array of N.MATCH_DTYPE on the host; an (b, 3) int64 tensor for device input)."""
        return self._matches(Q, metric, out, search=True)

    def recognize_matches(self, P, metric="l2", out=None):
        """ef_recognize_matches: projection + search, returning match records."""
        return self._matches(P, metric, out, search=False)

    def _matches(self, X, metric, out, search):
        mt = _metric(metric)
        if self.gallery_k is None:
            raise RuntimeError("no gallery: call set_gallery first")
        if not search and self.model_k is None:
            raise RuntimeError("recognize needs a model and a gallery")
        if _is_dev(X):
            import torch
            if search:
                x, xp = _dev(X, torch.float32)
                if x.ndim != 2 or x.shape[1] != self.gallery_k:
                    raise ValueError(f"Q must be (b, {self.gallery_k}), got {tuple(x.shape)}")
            else:
                x, xp, dtype = self._dev_pixels(X)
            b = x.shape[0]
            if out is None:
                out = torch.empty((b, 3), dtype=torch.int64, device=x.device)
            self._dev_out(out, (b, 3), torch.int64, "out")
            with self._torch_order(x, out):
                if search:
                    self._chk(self._lib.ef_search_matches(self._h, xp, b, mt, out.data_ptr(), N.EF_MEM_DEVICE))
                else:
                    self._chk(self._lib.ef_recognize_matches(self._h, xp, dtype, b, mt, out.data_ptr(), None,
                                                             N.EF_MEM_DEVICE))
            return out
        if search:
            x, xp = _host(X, np.float32)
            want = self.gallery_k
        else:
            x = np.asarray(X)
            dtype = N.EF_U8 if x.dtype == np.uint8 else N.EF_F32
            x, xp = _host(x, np.uint8 if dtype == N.EF_U8 else np.float32)
            want = self.model_d
        # the C side reads b * want elements from the host pointer: a narrower or 1-D
        # input would be read past its end
        if x.ndim != 2 or x.shape[1] != want:
            raise ValueError(f"{'Q' if search else 'P'} must be (b, {want}), got {x.shape}")
        b = x.shape[0]
        res = np.empty(b, dtype=N.MATCH_DTYPE)
        if search:
            self._chk(self._lib.ef_search_matches(self._h, xp, b, mt, res.ctypes.data, 0))
        else:
            self._chk(self._lib.ef_recognize_matches(self._h, xp, dtype, b, mt, res.ctypes.data, None, 0))
        return res

    def merge_matches(self, parts, b, keys=None):
        """Device merge (ef_matches_merge, EF_MEM_DEVICE) of gathered records: ``parts`` is
        an (nparts*b, 3) int64 tensor (part-major) -> int64 keys[b]."""
        import torch
        b = int(b)
        if not (isinstance(parts, torch.Tensor) and parts.is_cuda):
            raise TypeError("parts must be a device tensor (use merge_matches_host for host records)")
        if parts.dtype != torch.int64 or parts.ndim != 2 or parts.shape[1] != 3 or not parts.is_contiguous():
            raise ValueError(f"parts must be a contiguous (nparts*b, 3) int64 tensor, got "
                             f"{parts.dtype} {tuple(parts.shape)}")
        if b < 0 or (b and parts.shape[0] % b) or (b == 0 and parts.shape[0]):
            raise ValueError(f"parts has {parts.shape[0]} records, not a multiple of b = {b}")
        nparts = parts.shape[0] // b if b else 0
        if keys is None:
            keys = torch.empty(b, dtype=torch.int64, device=parts.device)
        elif not (keys.dtype == torch.int64 and tuple(keys.shape) == (b,) and keys.is_contiguous()
                  and keys.device == parts.device):
            raise ValueError(f"keys must be a contiguous int64 tensor of shape ({b},) on {parts.device}")
        if b:
            with self._torch_order(parts, keys):
                self._chk(self._lib.ef_matches_merge(self._h, parts.data_ptr(), nparts, b, keys.data_ptr(), None,
                                                     N.EF_MEM_DEVICE))
        return keys

    def recognize(self, P, metric="l2", return_features=False):
        """Project probes P (uint8/float32 pixels) and return (idx, best[, feats])."""
        p = np.asarray(P)
        feats = np.empty((p.shape[0], self.model_k), dtype=np.float32) if return_features else None
        keys = self.recognize_keys(p, metric, feats=feats)
        idx, best = decode_keys(keys, metric)
        return (idx, best, feats) if return_features else (idx, best)

    # ---------------------------------------------------------------------- images
    PREPROCESS_CHUNK = 65535

    def preprocess(self, images, size=(64, 64), rgb=False, out=None):
        """Grey + INTER_LINEAR resize of a ragged batch (include/eigenface.h
        ef_preprocess): ``images`` is a list of uint8 arrays (h, w) or (h, w, 3|4)
        (BGR unless ``rgb``); ``size`` is cv2's (width, height).  Returns an
        (n, height*width) uint8 array (or fills device tensor ``out``)."""
        ow, oh = int(size[0]), int(size[1])
        n = len(images)
        if n == 0:
            return np.empty((0, oh * ow), np.uint8)
        if n > self.PREPROCESS_CHUNK:  # ef_preprocess takes at most 65535 images per call
            res = np.empty((n, oh * ow), np.uint8) if out is None else None
            for a in range(0, n, self.PREPROCESS_CHUNK):
                e = min(n, a + self.PREPROCESS_CHUNK)
                part = self.preprocess(images[a:e], size, rgb, None if out is None else out[a:e])
                if res is not None:
                    res[a:e] = part
            return out if out is not None else res
        arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
        hs = np.array([a.shape[0] for a in arrs], np.int32)
        ws = np.array([a.shape[1] for a in arrs], np.int32)
        cs = np.array([1 if a.ndim == 2 else a.shape[2] for a in arrs], np.int32)
        sizes = np.array([a.size for a in arrs], np.int64)
        offs = np.zeros(n, np.int64)
        offs[1:] = np.cumsum(sizes)[:-1]
        buf = np.concatenate([a.reshape(-1) for a in arrs])
        flags = N.EF_IMG_RGB if rgb else 0
        if out is not None:  # device output: stage the pixels on the device too
            import torch
            dbuf = torch.from_numpy(buf).to(out.device)
            with self._torch_order(out, dbuf):
                self._chk(self._lib.ef_preprocess(self._h, dbuf.data_ptr(), offs.ctypes.data, hs.ctypes.data,
                                                  ws.ctypes.data, cs.ctypes.data, n, oh, ow, out.data_ptr(),
                                                  flags | N.EF_MEM_DEVICE))
            return out
        res = np.empty((n, oh * ow), np.uint8)
        self._chk(self._lib.ef_preprocess(self._h, buf.ctypes.data, offs.ctypes.data, hs.ctypes.data,
                                          ws.ctypes.data, cs.ctypes.data, n, oh, ow, res.ctypes.data, flags))
        return res

    # ----------------------------------------------------------------- JPEG decode
    def decode_jpegs(self, blobs, mode="bgr"):
        """GPU decode of a batch of JPEG files (include/eigenface.h ef_jpeg_decode):
        ``blobs`` are the files' bytes; ``mode`` "bgr" (cv2.imread IMREAD_COLOR) or "gray"
        (IMREAD_GRAYSCALE).  Returns a list of uint8 arrays, None where the GPU decoder
        does not take the file (progressive, CMYK, ...; ``status`` says why)."""
        m = _jpeg_mode(mode)
        n = len(blobs)
        if n == 0:
            return []
        packed = _pack_blobs(blobs)
        data, offs, sizes, _keep = packed
        h, w, _, st = jpeg_info(blobs, _packed=packed)
        ch = 1 if m == N.EF_JPEG_GRAY else 3
        px = np.where(st == 0, h.astype(np.int64) * w * ch, 0)
        ooff = np.zeros(n, np.int64)
        ooff[1:] = np.cumsum(px)[:-1]
        out = np.empty(max(1, int(px.sum())), np.uint8)
        self._chk(self._lib.ef_jpeg_decode(self._h, data, offs.ctypes.data, sizes.ctypes.data, n, m,
                                           out.ctypes.data, ooff.ctypes.data, st.ctypes.data, 0))
        res = []
        for i in range(n):
            if st[i] != 0:
                res.append(None)
                continue
            a = out[ooff[i]:ooff[i] + px[i]]
            res.append(a.reshape(h[i], w[i]) if ch == 1 else a.reshape(h[i], w[i], 3))
        return res

    def ingest_jpegs(self, blobs, size=(64, 64), mode="bgr", out=None):
        """Fused GPU decode + grey + INTER_LINEAR resize of JPEG files
        (ef_jpeg_ingest): (rows uint8 (n, h*w) — or device tensor ``out`` filled —,
        status int32 (n,)).  Rows of files with status != 0 are zero.  With ``out`` the
        call returns once the decode is queued on the engine's stream (status is final);
        torch's current stream is ordered after it (no host wait), so torch work on ``out``
        queued afterwards sees the decoded rows, and back-to-back calls overlap one batch's
        host staging with the previous batch's decode."""
        m = _jpeg_mode(mode)
        ow, oh = int(size[0]), int(size[1])
        n = len(blobs)
        st = np.zeros(n, np.int32)
        if n == 0:
            return np.empty((0, oh * ow), np.uint8), st
        data, offs, sizes, _keep = _pack_blobs(blobs)
        if out is not None:
            import torch
            o, op = _dev(out, torch.uint8)
            self._dev_out(o, (n, oh * ow), torch.uint8, "out")
            with self._torch_order(o):
                self._chk(self._lib.ef_jpeg_ingest(self._h, data, offs.ctypes.data, sizes.ctypes.data, n, m,
                                                   oh, ow, op, st.ctypes.data, N.EF_MEM_DEVICE))
            return out, st
        rows = np.empty((n, oh * ow), np.uint8)
        self._chk(self._lib.ef_jpeg_ingest(self._h, data, offs.ctypes.data, sizes.ctypes.data, n, m,
                                           oh, ow, rows.ctypes.data, st.ctypes.data, 0))
        return rows, st

    def tm_prepare(self, templates, problems, frame_shape):
        """Resident template-localiser operands (ef_tm_prepare).  ``templates``: list of
        grey uint8 (h, w) arrays; ``problems``: list of (template index, height, width)
        scaled sizes; ``frame_shape``: (H, W)."""
        arrs = [np.ascontiguousarray(t, dtype=np.uint8) for t in templates]
        nt = len(arrs)
        th = np.array([a.shape[0] for a in arrs], np.int32)
        tw = np.array([a.shape[1] for a in arrs], np.int32)
        sizes = np.array([a.size for a in arrs], np.int64)
        offs = np.zeros(nt, np.int64)
        if nt > 1:
            offs[1:] = np.cumsum(sizes)[:-1]
        buf = np.concatenate([a.reshape(-1) for a in arrs]) if nt else np.zeros(1, np.uint8)
        pr = np.asarray(problems, dtype=np.int64).reshape(-1, 3)
        pt, ph, pw = (np.ascontiguousarray(pr[:, i], dtype=np.int32) for i in range(3))
        H, W = (int(v) for v in frame_shape)
        self._chk(self._lib.ef_tm_prepare(self._h, buf.ctypes.data, offs.ctypes.data, th.ctypes.data,
                                          tw.ctypes.data, nt, pt.ctypes.data, ph.ctypes.data, pw.ctypes.data,
                                          len(pr), H, W, 0))
        self._tm = (len(pr), H, W, pr.copy())

    def tm_match(self, frame, maps=False):
        """Run the prepared problems on one grey frame: (best float32[P], x int32[P],
        y int32[P]) and, with ``maps``, the list of TM_CCOEFF_NORMED result maps."""
        if getattr(self, "_tm", None) is None:
            raise RuntimeError("call tm_prepare first")
        npb, H, W, _ = self._tm
        f = np.ascontiguousarray(frame, dtype=np.uint8)
        if f.shape != (H, W):
            raise ValueError(f"frame must be {(H, W)}, got {f.shape}")
        best = np.empty(npb, np.float32)
        xs = np.empty(npb, np.int32)
        ys = np.empty(npb, np.int32)
        mp = None
        if maps:
            n = C.c_int32(0)
            tot = C.c_int64(0)
            hr = np.empty(max(npb, 1), np.int32)
            wr = np.empty(max(npb, 1), np.int32)
            self._chk(self._lib.ef_tm_info(self._h, C.byref(n), C.byref(tot), hr.ctypes.data, wr.ctypes.data))
            flat = np.empty(tot.value, np.float32)
            mp = flat
        self._chk(self._lib.ef_tm_match(self._h, f.ctypes.data, W, best.ctypes.data, xs.ctypes.data,
                                        ys.ctypes.data, mp.ctypes.data if mp is not None else None, 0))
        if not maps:
            return best, xs, ys
        out, o = [], 0
        for p in range(npb):
            m = int(hr[p]) * int(wr[p])
            out.append(flat[o:o + m].reshape(int(hr[p]), int(wr[p])))
            o += m
        return best, xs, ys, out

    # --------------------------------------------------------------------- timing
    def timing(self, on=True):
        self._chk(self._lib.ef_timing_enable(self._h, 1 if on else 0))

    def timing_reset(self):
        self._chk(self._lib.ef_timing_reset(self._h))

    def timing_get(self, kernel="search"):
        kid = {"search": N.EF_KERNEL_SEARCH, "project": N.EF_KERNEL_PROJECT, "tmatch": N.EF_KERNEL_TMATCH,
               "ingest": N.EF_KERNEL_INGEST, "haar": N.EF_KERNEL_HAAR, "jpeg": N.EF_KERNEL_JPEG,
               "syrk": N.EF_KERNEL_SYRK, "jpeg_host": N.EF_KERNEL_JPEG_HOST}[kernel]
        ms = C.c_double(0)
        n = C.c_int64(0)
        self._chk(self._lib.ef_timing_get(self._h, kid, C.byref(ms), C.byref(n)))
        return float(ms.value), int(n.value)


def decode_keys(keys, metric="l2"):
    """(idx int64, best float32) from packed keys; EF_KEY_NONE -> (-1, nan)."""
    k = np.ascontiguousarray(keys, dtype=np.int64)
    b = k.shape[0]
    idx = np.empty(b, dtype=np.int64)
    best = np.empty(b, dtype=np.float32)
    N.lib().ef_keys_decode(k.ctypes.data, b, _metric(metric), best.ctypes.data, idx.ctypes.data)
    return idx, best


def merge_matches_host(parts, b):
    """Host merge (ef_matches_merge without a context; no GPU needed): ``parts`` is an
    array of N.MATCH_DTYPE (nparts*b, part-major) or its (nparts*b, 3) int64 view."""
    p = np.ascontiguousarray(parts)
    if p.dtype != np.dtype(N.MATCH_DTYPE):
        p = np.ascontiguousarray(p, dtype=np.int64)
        if p.ndim != 2 or p.shape[1] != 3:
            raise ValueError(f"parts must be (nparts*b, 3) int64 or MATCH_DTYPE records, got {p.shape}")
        p = p.view(N.MATCH_DTYPE).reshape(-1)
    b = int(b)
    if b < 0 or (b and p.shape[0] % b) or (b == 0 and p.shape[0]):
        raise ValueError(f"{p.shape[0]} records is not a multiple of b = {b}")
    nparts = p.shape[0] // b if b else 0
    keys = np.empty(b, dtype=np.int64)
    if b:
        rc = N.lib().ef_matches_merge(None, p.ctypes.data, nparts, b, keys.ctypes.data, None, 0)
        if rc != N.EF_OK:
            raise N.EigenfaceError(rc, "ef_matches_merge failed")
    return keys


def _jpeg_mode(mode):
    try:
        return {"bgr": N.EF_JPEG_BGR, "color": N.EF_JPEG_BGR, "gray": N.EF_JPEG_GRAY, "grey": N.EF_JPEG_GRAY}[mode]
    except KeyError:
        raise ValueError(f"unknown JPEG output mode {mode!r} (bgr | gray)") from None


def _bytes_data_offset():
    """Offset of a bytes object's payload from id(): CPython's PyBytesObject layout,
    verified once (0 disables the fast path)."""
    probe = b"eigenface-probe"
    off = sys.getsizeof(b"") - 1
    try:
        if C.string_at(id(probe) + off, len(probe)) == probe:
            return off
    except Exception:  # pragma: no cover - non-CPython
        pass
    return 0


_BYTES_OFF = None


def _pack_blobs(blobs):
    """Address the files in place (no concatenation): (base pointer, int64 offsets from it,
    int64 sizes, keep-alive list).  The C ABI reads file i at base + offsets[i]."""
    global _BYTES_OFF
    if _BYTES_OFF is None:
        _BYTES_OFF = _bytes_data_offset()
    n = len(blobs)
    sizes = np.fromiter(map(len, blobs), np.int64, n)
    if _BYTES_OFF and set(map(type, blobs)) == {bytes}:  # payload address = id + header
        addrs = np.fromiter(map(id, blobs), np.int64, n) + _BYTES_OFF
        keep = blobs
    else:
        keep = [np.frombuffer(b, np.uint8) if len(b) else np.zeros(1, np.uint8) for b in blobs]
        addrs = np.fromiter((v.ctypes.data for v in keep), np.int64, n)
    base = int(addrs.min()) if n else 0
    return base, addrs - base, sizes, keep


def jpeg_info(blobs, _packed=None):
    """Header parse on the host (ef_jpeg_info, no GPU): (height, width, components,
    status) int32 arrays; status 0 = the GPU decoder takes the file."""
    data, offs, sizes, _keep = _packed if _packed is not None else _pack_blobs(blobs)
    n = len(sizes)
    h, w, c, st = (np.zeros(n, np.int32) for _ in range(4))
    if n:
        rc = N.lib().ef_jpeg_info(data, offs.ctypes.data, sizes.ctypes.data, n, h.ctypes.data,
                                  w.ctypes.data, c.ctypes.data, st.ctypes.data)
        if rc != N.EF_OK:
            raise N.EigenfaceError(rc, "ef_jpeg_info failed")
    return h, w, c, st


def device_count() -> int:
    n = C.c_int(0)
    N.lib().ef_device_count(C.byref(n))
    return int(n.value)
