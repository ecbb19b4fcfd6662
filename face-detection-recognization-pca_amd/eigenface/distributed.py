"""Gallery row sharding across GPUs (one process per GPU, torch.distributed).

Rank r owns gallery rows [lo_r, hi_r) and searches them with global row offsets, so
its per-probe packed key (order-preserving score << 32 | global row) is directly
comparable with every other rank's.  One all-reduce(MIN) over the B int64 keys (RCCL
over xGMI with backend "nccl"; gloo on CPU) yields the global arg-best with the
lowest-index tie-break — the only data-path collective.  The probe
batch and the projection model are replicated (projection is < 2 % of the flops).

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
                 local_search=None):
        self.rank, self.world, self.n_total, self.group = rank, world, n_total, group
        self.lo, self.hi = shard_range(n_total, rank, world)
        if gallery_local is not None and len(gallery_local) != self.hi - self.lo:
            raise ValueError(f"rank {rank}: expected {self.hi - self.lo} rows, got {len(gallery_local)}")
        self.engine = engine
        if engine is not None and gallery_local is not None:
            engine.set_gallery(gallery_local, global_offset=self.lo)
        self._local = local_search or (lambda q, m, keys=None: engine.search_keys(q, m, keys=keys))

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

    def recognize_keys(self, P, metric="l2", keys=None):
        """Fused projection + local search + all-reduce (engine path)."""
        return self._allreduce_min(self.engine.recognize_keys(P, metric, keys=keys))
