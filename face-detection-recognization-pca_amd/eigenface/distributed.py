"""Gallery row sharding across GPUs (one process per GPU, torch.distributed).

Rank r owns gallery rows [lo_r, hi_r) and searches them with global row offsets.  Its
search returns one *match record* per probe (include/eigenface.h ``ef_match``: the
winner's fp64 score, the tie-tolerance scale and the packed key), and one all-gather of
the records (24 B per probe and rank: 96 KiB per rank at B = 4096 — latency-bound; RCCL
over xGMI with backend "nccl", gloo on CPU) lets every rank merge them exactly with
``ef_matches_merge``: the lowest global index among the ranks whose fp64 score is within
1e-12 of the best.  A MIN over the packed fp32 keys alone would order two ranks' winners
only to fp32 resolution and break sub-ulp differences by index; the fp64 record makes the
sharded arg-best equal the single-engine one for exact ties and for any
two rows whose fp64 scores differ by more than the 1e-12 relative tie window (inside it —
fp64 evaluation noise — each shard resolves its own window first; csrc/ef_comm.hip).

The projection model is replicated; the probe batch's projection is split by rows across
ranks and the (B x k) fp32 features are all-gathered (2 MiB at B = 4096, k = 128), so no
rank repeats another's projection work.

``merge="min"`` is the north star's exchange instead: each rank's packed
fp32 key per probe and ONE all-reduce(MIN) of B x 8 B — no record gather, no merge launch.
It equals the exact merge except where two ranks' winners tie in fp32 but not in fp64 (a
sub-ulp difference: the MIN then keeps the lower index; tests/test_distributed_cpu.py
shows both cases), so "exact" stays the default.

The same exchange also exists inside the library (``Engine.comm_init`` /
``ef_comm_init``: RCCL driven from C, for callers of the C ABI); this module is the
torch.distributed form.

This is the logical analogue of recognize_face_all_models' best-over-models loop
(scan-template-v4.py:297-319), made exact and independent of shard order.
"""
from __future__ import annotations

import numpy as np

from . import _native as N


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous, balanced row range [lo, hi) of a rank."""
    return n_total * rank // world, n_total * (rank + 1) // world


def pack_keys(values, idx):
    """Host mirror of the kernel key format (include/eigenface.h ef_search)."""
    v = np.ascontiguousarray(values, dtype=np.float32).copy()
    v[v == 0] = 0.0  # canonical +0
    b = v.view(np.int32).astype(np.int64)
    s = np.where(b >= 0, b, b ^ 0x7FFFFFFF)
    return (s << 32) | (np.asarray(idx, dtype=np.int64) & 0xFFFFFFFF)


def make_matches(score, scale, idx):
    """Host match records (N.MATCH_DTYPE) from fp64 scores (L2 squared distance or
    -cosine; +inf = no row), tie scales and global row indices."""
    score = np.asarray(score, dtype=np.float64)
    m = np.empty(score.shape[0], dtype=N.MATCH_DTYPE)
    m["score"] = score
    m["scale"] = scale
    fin = np.isfinite(score)
    keys = pack_keys(np.where(fin, score, 0.0).astype(np.float32), idx)
    m["key"] = np.where(fin, keys, N.EF_KEY_NONE)
    return m


def _as_records_tensor(m):
    """(b, 3) int64 tensor view of match records (numpy structured array or tensor)."""
    import torch
    if isinstance(m, torch.Tensor):
        return m
    a = np.ascontiguousarray(m, dtype=N.MATCH_DTYPE)
    return torch.from_numpy(a.view(np.int64).reshape(-1, 3).copy())


class ShardedGallery:
    """One rank's shard of a row-partitioned gallery.

    ``local_matches(Q, metric) -> match records`` defaults to the rank's
    :class:`eigenface.Engine` (device tensors in, a (b, 3) int64 device tensor out)."""

    def __init__(self, engine, gallery_local, n_total: int, rank: int, world: int, group=None,
                 local_matches=None, local_project=None, merge: str = "exact"):
        if merge not in ("exact", "min"):
            raise ValueError(f"merge must be 'exact' or 'min', not {merge!r}")
        self.merge = merge
        self.rank, self.world, self.n_total, self.group = rank, world, n_total, group
        self.lo, self.hi = shard_range(n_total, rank, world)
        if gallery_local is not None and len(gallery_local) != self.hi - self.lo:
            raise ValueError(f"rank {rank}: expected {self.hi - self.lo} rows, got {len(gallery_local)}")
        self.engine = engine
        if engine is not None and gallery_local is not None:
            engine.set_gallery(gallery_local, global_offset=self.lo)
        # one rank with the engine's own search: its keys are already global (no records,
        # no merge launch)
        self._direct = world == 1 and engine is not None and local_matches is None and local_project is None
        self._local_is_engine = local_matches is None
        self._local = local_matches or (lambda q, m: engine.search_matches(q, m))
        self._project = local_project or (lambda p, out=None: engine.project(p, out=out))
        self._fbuf = {}
        self._rbuf = {}

    # ---------------------------------------------------------------- exchange
    def _gather_merge(self, rec, b, keys=None):
        """All-gather every rank's records and merge them exactly -> int64 keys[b]."""
        import torch
        import torch.distributed as dist

        rec = _as_records_tensor(rec)
        if self.world == 1:
            parts = rec
        else:
            key = (b, str(rec.device))
            if key not in self._rbuf:
                self._rbuf[key] = torch.empty((self.world * b, 3), dtype=torch.int64, device=rec.device)
            parts = self._rbuf[key]
            if rec.is_cuda and not _device_collectives(self.group):  # gloo: gather on host
                chunks = [torch.empty((b, 3), dtype=torch.int64) for _ in range(self.world)]
                dist.all_gather(chunks, rec.cpu(), group=self.group)
                parts.copy_(torch.cat(chunks))
            elif rec.is_cuda:  # RCCL over xGMI, stream-ordered on torch's current stream
                dist.all_gather_into_tensor(parts, rec, group=self.group)
            else:
                dist.all_gather(list(parts.chunk(self.world)), rec, group=self.group)
        if parts.is_cuda and self.engine is not None:
            return self.engine.merge_matches(parts, b, keys)
        from .engine import merge_matches_host
        out = torch.from_numpy(merge_matches_host(parts.cpu().numpy(), b))
        if keys is not None:
            keys.copy_(out)
            return keys
        return out

    def _min_reduce(self, local_keys, keys=None):
        """merge="min": one all-reduce(MIN) of the ranks' packed keys -> int64 keys[b]."""
        import torch
        import torch.distributed as dist

        k = local_keys if isinstance(local_keys, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(local_keys, dtype=np.int64))
        if self.world > 1:
            if k.is_cuda and not _device_collectives(self.group):  # gloo: reduce on host
                t = k.cpu()
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
                k.copy_(t)
            else:  # RCCL over xGMI, stream-ordered on torch's current stream (or gloo, CPU)
                dist.all_reduce(k, op=dist.ReduceOp.MIN, group=self.group)
        if keys is not None:
            keys.copy_(k)
            return keys
        return k

    def _local_keys(self, Q, metric):
        """This rank's packed keys (global row indices) of its best row per probe."""
        if self.engine is not None and self._local_is_engine:
            return self.engine.search_keys(Q, metric)
        rec = self._local(Q, metric)
        if isinstance(rec, np.ndarray) and rec.dtype.names:
            return np.ascontiguousarray(rec["key"], dtype=np.int64).copy()
        return _as_records_tensor(rec)[:, 2].contiguous()

    def search_keys(self, Q, metric="l2", keys=None):
        """Global packed keys of the best row per probe (all ranks get the same keys)."""
        if self._direct:
            return self.engine.search_keys(Q, metric, keys=keys)
        if self.merge == "min":
            return self._min_reduce(self._local_keys(Q, metric), keys)
        b = int(Q.shape[0])
        return self._gather_merge(self._local(Q, metric), b, keys)

    def _allgather_rows(self, loc, out):
        """out[(world*c), k] <- concat over ranks of loc[c, k] (rank order)."""
        import torch
        import torch.distributed as dist

        if loc.is_cuda and not _device_collectives(self.group):  # gloo: gather on host
            parts = [torch.empty_like(loc, device="cpu") for _ in range(self.world)]
            dist.all_gather(parts, loc.cpu(), group=self.group)
            out.copy_(torch.cat(parts))
        elif loc.is_cuda:  # RCCL over xGMI, stream-ordered on torch's current stream
            dist.all_gather_into_tensor(out, loc, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.world)), loc, group=self.group)
        return out

    def project_sharded(self, P):
        """Features of the whole probe batch: rank r projects rows [r*c, (r+1)*c) (c =
        ceil(B/world)) straight into its slice buffer, then one all-gather of the (c x k)
        slices.  Row order equals P's; rows past B (zero padding) are dropped."""
        import torch
        import torch.distributed as dist

        b = int(P.shape[0])
        c = (b + self.world - 1) // self.world
        lo, hi = min(b, self.rank * c), min(b, (self.rank + 1) * c)
        f = None
        if self.engine is not None:
            kk = int(self.engine.model_k)
        else:  # host hook (tests): k from the projected slice, agreed by every rank
            f = self._project(P[lo:hi]) if hi > lo else None
            t = torch.tensor([0 if f is None else int(f.shape[1])], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            kk = int(t.item())
        key = (c, kk, str(P.device))
        if key not in self._fbuf:
            self._fbuf[key] = (torch.zeros((c, kk), dtype=torch.float32, device=P.device),
                               torch.empty((self.world * c, kk), dtype=torch.float32, device=P.device))
        loc, full = self._fbuf[key]
        if hi > lo:
            if f is None:
                f = self._project(P[lo:hi], out=loc[: hi - lo])
            if not isinstance(f, torch.Tensor) or f.data_ptr() != loc.data_ptr():
                loc[: hi - lo].copy_(torch.as_tensor(np.ascontiguousarray(f) if not isinstance(f, torch.Tensor) else f))
        self._allgather_rows(loc, full)
        return full[:b]

    def recognize_keys(self, P, metric="l2", keys=None, shard_projection=True):
        """Projection + local search + exact merge.  world > 1 with a device (or CPU
        tensor) batch: the projection is split across ranks (project_sharded); otherwise
        the engine's fused ef_recognize_matches runs the whole batch."""
        import torch

        if self._direct:
            return self.engine.recognize_keys(P, metric, keys=keys)
        b = int(P.shape[0])
        if self.merge == "min":
            if self.world > 1 and shard_projection and isinstance(P, torch.Tensor):
                return self._min_reduce(self._local_keys(self.project_sharded(P), metric), keys)
            return self._min_reduce(self.engine.recognize_keys(P, metric), keys)  # replicated projection
        if self.world == 1 or not shard_projection or not isinstance(P, torch.Tensor):
            return self._gather_merge(self.engine.recognize_matches(P, metric), b, keys)
        q = self.project_sharded(P)
        return self._gather_merge(self._local(q, metric), b, keys)

    def exchange_ms(self, b: int, k: int, device, reps: int = 20) -> float:
        """Milliseconds per step of this rank's collectives alone — the feature all-gather of
        ceil(b / world) x k fp32 rows per rank and the all-gather of b fp64 match records
        (merge="min": the all-reduce of b packed keys instead) —
        on the same transport as recognize_keys (RCCL stream-ordered, or gloo through the
        host), averaged over `reps` after one warm-up.  The caller takes the max over ranks."""
        import time

        import torch
        import torch.distributed as dist

        c = (b + self.world - 1) // self.world
        loc = torch.zeros((c, k), dtype=torch.float32, device=device)
        full = torch.empty((self.world * c, k), dtype=torch.float32, device=device)
        rec = torch.zeros((b, 3), dtype=torch.int64, device=device)
        gloo = not _device_collectives(self.group)
        parts = torch.empty((self.world * b, 3), dtype=torch.int64, device=device)

        kmin = torch.zeros(b, dtype=torch.int64, device=device)

        def one():
            self._allgather_rows(loc, full)
            if self.merge == "min":
                self._min_reduce(kmin)
            elif gloo:
                chunks = [torch.empty((b, 3), dtype=torch.int64) for _ in range(self.world)]
                dist.all_gather(chunks, rec.cpu(), group=self.group)
                parts.copy_(torch.cat(chunks))
            else:
                dist.all_gather_into_tensor(parts, rec, group=self.group)

        one()
        torch.cuda.synchronize(device)
        dist.barrier(group=self.group)
        t = time.perf_counter()
        for _ in range(reps):
            one()
        torch.cuda.synchronize(device)
        return (time.perf_counter() - t) / reps * 1e3


# ------------------------------------------------------------------ sharded fit
def _device_collectives(group=None):
    """True when ``group``'s backend reduces device tensors (RCCL, "nccl" on ROCm); every
    other backend (gloo) reduces host tensors.  The one predicate ShardedGallery and the
    sharded fit use."""
    import torch.distributed as dist
    return dist.get_backend(group) == "nccl"


def allreduce_fit_stats(pieces, group=None, device=None):
    """Sum the exact integer fit pieces (sum x, sum x^2, X'^T X'; int64) over the ranks of
    ``group`` in place: an integer sum, so the result is exact in any order.  RCCL reduces
    device tensors (host pieces — a host X_local — travel through ``device``, default the
    current GPU, and are copied back); gloo reduces host copies.  Of X'^T X' only the upper
    64-blocks travel (d % 64 == 0)."""
    import torch
    import torch.distributed as dist

    on_device = _device_collectives(group)
    if on_device and device is None:
        device = torch.device("cuda", torch.cuda.current_device())

    def reduce(t):
        if not on_device and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, group=group)
            t.copy_(h)
        elif on_device and not t.is_cuda and torch.device(device).type != t.device.type:
            h = t.to(device)
            dist.all_reduce(h, group=group)
            t.copy_(h.cpu())
        elif on_device and not t.is_cuda:  # (tests: a host "device")
            h = t.clone()
            dist.all_reduce(h, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=group)

    out = []
    for t in pieces:
        if not isinstance(t, torch.Tensor):
            t = torch.from_numpy(np.ascontiguousarray(t, dtype=np.int64))
        d = t.shape[0]
        if t.ndim == 2 and d % 64 == 0:
            # X'^T X': only its upper 64 x 64 blocks are specified (and read by the covariance
            # finalize), so only they travel — half the bytes of the d x d matrix
            nb = d // 64
            iu = torch.triu_indices(nb, nb, device=t.device)
            blocks = t.view(nb, 64, nb, 64).permute(0, 2, 1, 3)
            packed = blocks[iu[0], iu[1]].contiguous()
            reduce(packed)
            blocks[iu[0], iu[1]] = packed
        else:
            reduce(t)
        out.append(t)
    return out


def sharded_fit(engine, X_local, n_components: int, standardize: bool = False, group=None, projection: bool = True,
                stats_fn=None, fit_fn=None, transform_fn=None):
    """The sample-sharded fit of SURVEY.md §8(e) (the fit collective): every rank holds the
    uint8 rows X_local of its shard; each computes the exact integer pieces of its rows
    (``Engine.fit_shard_stats``: sum x, sum x^2 and X'^T X' with X' = X - 128), one
    all-reduce(sum) per piece adds them up (the d x d piece is 2 GiB at d = 16384:
    bandwidth-bound over xGMI, beside a SYRK of n_total / world rows), and every rank runs
    the covariance-path fit from the sums (``Engine.fit_from_stats``) — bit-identical to
    ``Engine.fit`` on the concatenated rows, because the same integers give the same
    covariance (only the upper 64-blocks of X'^T X' are reduced: 1 GiB at d = 16384) — then projects its own rows (``Engine.fit_transform_rows``).  Returns the
    FitResult with ``projection`` = this rank's rows.  The ``*_fn`` hooks replace the
    engine calls (CPU tests)."""
    import torch
    import torch.distributed as dist

    stats_fn = stats_fn or engine.fit_shard_stats
    fit_fn = fit_fn or engine.fit_from_stats
    transform_fn = transform_fn or engine.fit_transform_rows
    n_local = int(X_local.shape[0])
    n = torch.tensor([n_local], dtype=torch.int64)
    dev = None
    if _device_collectives(group):
        dev = X_local.device if isinstance(X_local, torch.Tensor) and X_local.is_cuda else \
            torch.device("cuda", torch.cuda.current_device())
        n = n.to(dev)
    dist.all_reduce(n, group=group)
    n_total = int(n.item())
    pieces = allreduce_fit_stats(stats_fn(X_local), group, device=dev)
    if not isinstance(X_local, torch.Tensor) or not X_local.is_cuda:
        pieces = [p.cpu().numpy() if isinstance(p, torch.Tensor) else p for p in pieces]
    res = fit_fn(*pieces, n_total, n_components, standardize)
    if projection and n_local > 0:
        res.projection = transform_fn(X_local, res, standardize)
    return res
