"""CPU oracle for the Haar cascade face detector — TEST INFRASTRUCTURE ONLY.

Restates ``face_cascade.detectMultiScale(gray, scaleFactor=1.1, minNeighbors=5,
minSize=(30, 30))`` (detection-v4.py:18, :50-55) the way OpenCV 4.x's
``CascadeClassifierImpl`` evaluates a stump-based HAAR cascade (objdetect
cascadedetect.cpp: detectMultiScaleNoGrouping, FeatureEvaluator::updateScaleData,
HaarEvaluator::setWindow / OptFeature::calc, predictOrderedStump,
CascadeClassifierInvoker, groupRectangles + SimilarRects, GROUP_EPS = 0.2).

Parity is UNPINNED: OpenCV (4.8.1.78, useless/requirements.txt:3) is not installed,
so neither its outputs nor the cascade file the reference loads
(cv2.data.haarcascades + 'haarcascade_frontalface_default.xml') exist here.  Tests
use synthetic cascades.  One documented deviation: OpenCV builds its image pyramid
with INTER_LINEAR_EXACT; this restatement (and the GPU) use the INTER_LINEAR rules of
image_oracle.resize_linear.

Only tests/ may import this module.
"""
from __future__ import annotations

import numpy as np

from .image_oracle import resize_linear

GROUP_EPS = 0.2


def cv_round(v):
    """cvRound: round half to even (lrint)."""
    return int(np.rint(v))


def scale_list(win, img_size, scale_factor=1.1, min_size=(0, 0), max_size=None):
    """detectMultiScaleNoGrouping's factor loop: float32 scales."""
    ww, wh = win
    W, H = img_size
    mw, mh = (W, H) if not max_size or max_size == (0, 0) else max_size
    out = []
    factor = 1.0
    while True:
        sw, sh = cv_round(ww * factor), cv_round(wh * factor)
        if sw > mw or sh > mh:
            break
        if not (sw < min_size[0] or sh < min_size[1]):
            out.append(np.float32(factor))
        factor *= scale_factor
    return out


def layer_size(img_size, sc):
    """updateScaleData: sz = (cvRound(W / sc), cvRound(H / sc)) in float arithmetic."""
    W, H = img_size
    return cv_round(np.float32(W) / sc), cv_round(np.float32(H) / sc)


def _integral(a):
    ii = np.zeros((a.shape[0] + 1, a.shape[1] + 1), dtype=np.int64)
    ii[1:, 1:] = a.astype(np.int64).cumsum(0).cumsum(1)
    return ii


def _box(ii, ys, xs, x, y, w, h):
    return ii[ys + y + h, xs + x + w] - ii[ys + y, xs + x + w] - ii[ys + y + h, xs + x] + ii[ys + y, xs + x]


def eval_layer(layer, cascade):
    """runAt for every window origin of one pyramid layer: result per (y, x) origin —
    -1 (setWindow: low variance), -stage (rejected at that stage; 0 = first stage) or 1."""
    ww, wh = cascade["win"]
    h, w = layer.shape
    ny, nx = h + 1 - wh, w + 1 - ww
    if ny <= 0 or nx <= 0:
        return np.zeros((0, 0), np.int64)
    ii = _integral(layer)
    sq = _integral(layer.astype(np.int64) ** 2)
    ys, xs = np.meshgrid(np.arange(ny), np.arange(nx), indexing="ij")
    area = float((ww - 2) * (wh - 2))
    s = _box(ii, ys, xs, 1, 1, ww - 2, wh - 2).astype(np.float64)
    q = _box(sq, ys, xs, 1, 1, ww - 2, wh - 2).astype(np.float64)
    nf = area * q - s * s
    with np.errstate(divide="ignore", invalid="ignore"):
        vnf = np.where(nf > 0, 1.0 / np.sqrt(np.where(nf > 0, nf, 1.0)), 1.0).astype(np.float32)
    ok = (nf > 0) & (area * vnf.astype(np.float64) < 0.1)
    res = np.full((ny, nx), -1, np.int64)
    alive = ok.copy()
    res[alive] = 1
    feats = cascade["features"]
    for si, (sthr, stumps) in enumerate(cascade["stages"]):
        tmp = np.zeros((ny, nx), np.float64)
        for fi, thr, left, right in stumps:
            val = np.zeros((ny, nx), np.float32)
            for k, (rx, ry, rw, rh, wt) in enumerate(feats[fi]):
                if k == 2 and wt == 0:
                    continue
                term = np.float32(wt) * _box(ii, ys, xs, rx, ry, rw, rh).astype(np.float32)
                val = term if k == 0 else (val + term).astype(np.float32)
            val = (val * vnf).astype(np.float32)
            tmp += np.where(val < np.float32(thr), np.float32(left), np.float32(right)).astype(np.float64)
        rej = alive & (tmp < np.float64(np.float32(sthr)))
        res[rej] = -si
        alive &= ~rej
    return res


def candidates(gray, cascade, scale_factor=1.1, min_size=(0, 0), max_size=None):
    """detectMultiScaleNoGrouping: raw rectangles in (scale, y, x) order, with the
    invoker's skip (a stage-0 rejection skips the next x position)."""
    H, W = gray.shape
    ww, wh = cascade["win"]
    out = []
    for sc in scale_list((ww, wh), (W, H), scale_factor, min_size, max_size):
        lw, lh = layer_size((W, H), sc)
        layer = resize_linear(gray, (lw, lh))
        res = eval_layer(layer, cascade)
        if res.size == 0:
            continue
        step = 1 if sc >= 2 else 2
        win = (cv_round(ww * sc), cv_round(wh * sc))
        for y in range(0, res.shape[0], step):
            x = 0
            while x < res.shape[1]:
                r = res[y, x]
                if r > 0:
                    out.append((cv_round(np.float32(x) * sc), cv_round(np.float32(y) * sc), win[0], win[1]))
                if r == 0:
                    x += step
                x += step
    return out


def _similar(a, b, eps):
    delta = eps * (min(a[2], b[2]) + min(a[3], b[3])) * 0.5
    return (abs(a[0] - b[0]) <= delta and abs(a[1] - b[1]) <= delta and
            abs(a[0] + a[2] - b[0] - b[2]) <= delta and abs(a[1] + a[3] - b[1] - b[3]) <= delta)


def partition(rects, eps):
    """cv::partition with SimilarRects.  Its union-find result is the set of connected
    components of the (symmetric) similarity graph, and its final pass numbers the
    classes in order of their lowest member index — so any union-find gives the same
    labels."""
    n = len(rects)
    parent = list(range(n))

    def find(i):
        while parent[i] != i:
            parent[i] = parent[parent[i]]
            i = parent[i]
        return i

    for i in range(n):
        for j in range(i + 1, n):
            if _similar(rects[i], rects[j], eps):
                ri, rj = find(i), find(j)
                if ri != rj:
                    parent[max(ri, rj)] = min(ri, rj)
    labels, roots = [], {}
    for i in range(n):
        r = find(i)
        if r not in roots:
            roots[r] = len(roots)
        labels.append(roots[r])
    return labels, len(roots)


def group_rectangles(rects, group_threshold, eps=GROUP_EPS):
    """cv::groupRectangles(rectList, groupThreshold, eps)."""
    if group_threshold <= 0 or not rects:
        return list(rects)
    labels, nc = partition(rects, eps)
    acc = [[0, 0, 0, 0] for _ in range(nc)]
    cnt = [0] * nc
    for r, c in zip(rects, labels):
        for k in range(4):
            acc[c][k] += r[k]
        cnt[c] += 1
    rr = []
    for c in range(nc):
        s = np.float32(1.0) / np.float32(cnt[c])
        rr.append(tuple(cv_round(np.float32(acc[c][k]) * s) for k in range(4)))
    out = []
    for i in range(nc):
        r1, n1 = rr[i], cnt[i]
        if n1 <= group_threshold:
            continue
        keep = True
        for j in range(nc):
            n2 = cnt[j]
            if j == i or n2 <= group_threshold:
                continue
            r2 = rr[j]
            dx, dy = cv_round(r2[2] * eps), cv_round(r2[3] * eps)
            if (r1[0] >= r2[0] - dx and r1[1] >= r2[1] - dy and r1[0] + r1[2] <= r2[0] + r2[2] + dx and
                    r1[1] + r1[3] <= r2[1] + r2[3] + dy and (n2 > max(3, n1) or n1 < 3)):
                keep = False
                break
        if keep:
            out.append(r1)
    return out


def detect_multi_scale(gray, cascade, scale_factor=1.1, min_neighbors=5, min_size=(30, 30), max_size=None):
    """face_cascade.detectMultiScale(gray, scaleFactor, minNeighbors, minSize) (detection-v4.py:50-55)."""
    return group_rectangles(candidates(gray, cascade, scale_factor, min_size, max_size), min_neighbors)
