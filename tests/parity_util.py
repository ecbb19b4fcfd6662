"""What the search engine guarantees, as test assertions.

The engine resolves every probe's arg-best in fp64 (ef_search.hip reduce_kernel /
resolve_kernel): the returned row is the lowest index among the rows whose fp64 score is
within 1e-12 * (|best| + scale) of the best, with scale = ||q||^2 + max ||g||^2 for L2 and,
for cosine, scores -cos(q, g) (ef_search_common.hpp score64) with scale 1.  So:

* every probe whose fp64 top-2 gap exceeds that window must get exactly the oracle's
  first-arg-best row (np.argmin / np.argmax semantics) — no fraction floor;
* every other probe must get a row inside the window.

The checker scores in fp64 with the expanded form (||q||^2 + ||g||^2 - 2 q.g, or unit-row
dot products for cosine); its evaluation error is ~1e-15 of the scale, 1000x below the
window, so the 1.1x margin on the window absorbs it.
"""
import numpy as np

from oracle import eigenface_oracle as orc

WINDOW = 1e-12
MARGIN = 1.1


def top2(q, g, metric, chunk_rows=131072, chunk_probes=512):
    """fp64 (first-best index, best, runner-up) per probe over all gallery rows, scores as
    'smaller is better' (L2: squared distance; cosine: -cos in unit terms)."""
    q64 = np.asarray(q, np.float64)
    b = len(q64)
    idx = np.zeros(b, np.int64)
    best = np.full(b, np.inf)
    second = np.full(b, np.inf)
    if metric == "cosine":
        q64 = orc._unit_rows(q64)
    for p0 in range(0, b, chunk_probes):
        qs = q64[p0:p0 + chunk_probes]
        qq = (qs ** 2).sum(1)
        bi, bb, bs = idx[p0:p0 + chunk_probes], best[p0:p0 + chunk_probes], second[p0:p0 + chunk_probes]
        for a in range(0, len(g), chunk_rows):
            g64 = np.asarray(g[a:a + chunk_rows], np.float64)
            if metric == "l2":
                s = qq[:, None] + (g64 ** 2).sum(1)[None, :] - 2.0 * (qs @ g64.T)
            else:
                s = -(qs @ orc._unit_rows(g64).T)
            j = np.argmin(s, axis=1)  # first minimum inside the chunk
            cb = s[np.arange(len(qs)), j]
            if s.shape[1] > 1:
                s[np.arange(len(qs)), j] = np.inf
                c2 = s.min(axis=1)
            else:
                c2 = np.full(len(qs), np.inf)
            new = cb < bb  # strictly better: earlier chunks keep exact ties (first index)
            bs[:] = np.where(new, np.minimum(bb, c2), np.minimum(bs, cb))
            bi[:] = np.where(new, a + j, bi)
            bb[:] = np.where(new, cb, bb)
    return idx, best, second


def gmax2_of(g, chunk=131072):
    return max(((np.asarray(g[a:a + chunk], np.float64) ** 2).sum(1).max() for a in range(0, len(g), chunk)),
               default=0.0)


def window(q, g, metric, best, gmax2=None):
    """The engine's tie window per probe, in the checker's units."""
    q64 = np.asarray(q, np.float64)
    qn2 = (q64 ** 2).sum(1)
    if metric == "l2":
        scale = qn2 + (gmax2_of(g) if gmax2 is None else gmax2)
        return WINDOW * (np.abs(best) + scale)
    # cosine: resolve_kernel's fp64 score is -cos (score64: -q.g / (|q| |g|)), window
    # 1e-12 (|score| + 1)
    return WINDOW * (np.abs(best) + 1.0)


def chosen_scores(q, g, idx, metric):
    """fp64 scores of the rows the engine chose (same units as top2)."""
    q64 = np.asarray(q, np.float64)
    gi = np.asarray(g[idx], np.float64)
    if metric == "l2":
        return ((q64 - gi) ** 2).sum(1)
    return -(orc._unit_rows(q64) * orc._unit_rows(gi)).sum(1)


def assert_exact_argbest(q, g, idx, metric, ref=None, min_clear=None, gmax2=None):
    """The guarantee above.  ref: precomputed top2(q, g, metric).  Returns the boolean
    mask of probes outside the tie window (asserted exact)."""
    ref_idx, best, second = ref if ref is not None else top2(q, g, metric)
    idx = np.asarray(idx)
    w = MARGIN * window(q, g, metric, best, gmax2)
    mine = chosen_scores(q, g, idx, metric)
    bad = ~(mine - best <= w)
    assert not bad.any(), f"{metric}: {bad.sum()} probes chose a row outside the tie window " \
                          f"(first {np.flatnonzero(bad)[:5]})"
    clear = (second - best) > w
    miss = clear & (idx != ref_idx)
    assert not miss.any(), f"{metric}: {miss.sum()} of {clear.sum()} clear probes differ from the fp64 " \
                           f"first-arg-best (first {np.flatnonzero(miss)[:5]})"
    if min_clear is not None:
        assert clear.mean() >= min_clear, clear.mean()
    return clear


def top2_device(q, g, metric, chunk_rows=131072):
    """top2 with torch fp64 GEMMs on the GPU: an independent fp64 checker (rocBLAS, not
    the engine's kernels) for full-size batches the host cannot score in seconds
    (4096 probes x 1M rows).  Same units and semantics as top2 outside ties."""
    import torch
    dev = torch.device("cuda")
    q64 = torch.as_tensor(np.asarray(q), device=dev).double()
    if metric == "cosine":
        q64 = q64 / q64.norm(dim=1, keepdim=True).clamp_min(1e-300)
    qq = (q64 * q64).sum(1)
    b = q64.shape[0]
    best = torch.full((b,), float("inf"), dtype=torch.float64, device=dev)
    second = best.clone()
    idx = torch.zeros(b, dtype=torch.int64, device=dev)
    for a in range(0, len(g), chunk_rows):
        gc = g[a:a + chunk_rows]
        g64 = (gc if isinstance(gc, torch.Tensor) else torch.as_tensor(np.asarray(gc))).to(dev).double()
        if metric == "l2":
            s = qq[:, None] + (g64 * g64).sum(1)[None, :] - 2.0 * (q64 @ g64.T)
        else:
            s = -(q64 @ (g64 / g64.norm(dim=1, keepdim=True).clamp_min(1e-300)).T)
        if s.shape[1] > 1:
            v, j = torch.topk(s, 2, dim=1, largest=False)
            cb, c2, cj = v[:, 0], v[:, 1], j[:, 0]
        else:
            cb, c2, cj = s[:, 0], torch.full_like(s[:, 0], float("inf")), torch.zeros(b, dtype=torch.int64, device=dev)
        new = cb < best
        second = torch.where(new, torch.minimum(best, c2), torch.minimum(second, cb))
        idx = torch.where(new, a + cj, idx)
        best = torch.where(new, cb, best)
        del s
    return idx.cpu().numpy(), best.cpu().numpy(), second.cpu().numpy()


def plant_rivals(G, q, anchors, seed, avoid=()):
    """Near-tie stress: for probe i, a copy of gallery row anchors[i] whose
    coordinate of largest |q - g| is moved by 1..64 ulps (random direction), written over a
    row in the other half of the gallery (a different chunk).  Its fp64 score differs from
    the anchor's by ~1e-10..1e-7 of the scale: far inside fp32 (and bf16) rounding of the
    scan scores, far outside the 1e-12 tie window.  Returns (G2, rival rows)."""
    rng = np.random.default_rng(seed)
    n = len(G)
    G2 = G.copy()
    used = set(int(a) for a in anchors) | set(int(a) for a in avoid)
    rivals = np.empty(len(anchors), np.int64)
    for i, a in enumerate(anchors):
        r = (int(a) + n // 2) % n
        while r in used:
            r = (r + 1) % n
        used.add(r)
        rivals[i] = r
    g = G[anchors].copy()
    diff = np.abs(np.asarray(q, np.float32) - g)
    col = np.argmax(diff, axis=1)
    steps = rng.integers(1, 65, len(anchors)) * rng.choice([-1, 1], len(anchors))
    bits = g[np.arange(len(anchors)), col].view(np.int32).astype(np.int64) + steps
    g[np.arange(len(anchors)), col] = bits.astype(np.int32).view(np.float32)
    G2[rivals] = g
    return G2, rivals
