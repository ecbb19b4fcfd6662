"""Gallery row sharding across GPUs (one process per GPU, torch.distributed).

Rank r owns gallery rows [lo_r, hi_r) and searches them with global row offsets, so
its per-probe packed key (order-preserving score << 32 | global row) is directly
comparable with every other rank's.  One all-reduce(MIN) over the B int64 keys (RCCL
over xGMI with backend "nccl"; gloo on CPU) yields the global arg-best with the
lowest-index tie-break.  The projection model is replicated; the
probe batch's projection is split by rows across ranks and the (B x k) fp32 features
are all-gathered (2 MiB at B = 4096, k = 128), so no rank repeats another's projection
work — at 8 ranks a replicated projection would be ~20 % of each rank's step.

This is the logical analogue of recognize_face_all_models' best-over-models loop
(scan-template-v4.py:297-319), made exact: a MIN over keys instead of a strict '>'
scan, so the result does not depend on shard order.
"""
from __future__ import annotations

import numpy as np


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


class ShardedGallery:
    """One rank's shard of a row-partitioned gallery.

    ``local_search(Q, metric) -> int64 keys`` defaults to the rank's
    :class:`eigenface.Engine` (device tensors in, device keys out)."""

    def __init__(self, engine, gallery_local, n_total: int, rank: int, world: int, group=None,
                 local_search=None, local_project=None):
        self.rank, self.world, self.n_total, self.group = rank, world, n_total, group
        self.lo, self.hi = shard_range(n_total, rank, world)
        if gallery_local is not None and len(gallery_local) != self.hi - self.lo:
            raise ValueError(f"rank {rank}: expected {self.hi - self.lo} rows, got {len(gallery_local)}")
        self.engine = engine
        if engine is not None and gallery_local is not None:
            engine.set_gallery(gallery_local, global_offset=self.lo)
        self._local = local_search or (lambda q, m, keys=None: engine.search_keys(q, m, keys=keys))
        self._project = local_project or (lambda p, out=None: engine.project(p, out=out))
        self._fbuf = {}

    def _allreduce_min(self, k):
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return k
        if not isinstance(k, torch.Tensor):
            k = torch.from_numpy(np.ascontiguousarray(k))
        if k.is_cuda and dist.get_backend(self.group) != "nccl":  # gloo: reduce on host
            h = k.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MIN, group=self.group)
            k.copy_(h)
        else:  # RCCL over xGMI, stream-ordered on torch's current stream
            dist.all_reduce(k, op=dist.ReduceOp.MIN, group=self.group)
        return k

    def search_keys(self, Q, metric="l2", keys=None):
        import torch

        k = self._local(Q, metric, keys=keys) if keys is not None else self._local(Q, metric)
        if not isinstance(k, torch.Tensor):
            k = torch.from_numpy(np.ascontiguousarray(k))
        return self._allreduce_min(k)

    def _allgather_rows(self, loc, out):
        """out[(world*c), k] <- concat over ranks of loc[c, k] (rank order)."""
        import torch
        import torch.distributed as dist

        if loc.is_cuda and dist.get_backend(self.group) != "nccl":  # gloo: gather on host
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
        """Projection + local search + all-reduce.  world > 1 with a device (or CPU
        tensor) batch: the projection is split across ranks (project_sharded);
        otherwise the engine's fused ef_recognize runs the whole batch."""
        import torch

        if self.world == 1 or not shard_projection or not isinstance(P, torch.Tensor):
            return self._allreduce_min(self.engine.recognize_keys(P, metric, keys=keys))
        q = self.project_sharded(P)
        k = self._local(q, metric, keys=keys) if keys is not None else self._local(q, metric)
        if not isinstance(k, torch.Tensor):
            k = torch.from_numpy(np.ascontiguousarray(k))
        return self._allreduce_min(k)
