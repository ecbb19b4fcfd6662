"""CPU oracle for the image side of the hot path — TEST INFRASTRUCTURE ONLY.

Restates, in NumPy integer / float64 arithmetic, the OpenCV calls the reference makes
around the eigenfaces path:

  * ingest  (train-v4.py:59-68, scan-template-v4.py:257-263):
        cv2.cvtColor(img, COLOR_BGR2GRAY) -> cv2.resize(gray, (64, 64))   [INTER_LINEAR]
  * template localiser (scan-template-v4.py:127-200):
        cv2.resize(template, (int(w*s), int(h*s))) for s in (0.8, 1.0, 1.2)
        cv2.matchTemplate(frame, t, TM_CCOEFF_NORMED) -> cv2.minMaxLoc -> corner rule
        (is_detection_in_corner, :75-125) -> best over templates/scales (strict '>')
        -> keep if > 0.6.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg use
this module; the product path runs the HIP kernels (``eigenface.image``).

Third-party algorithm: OpenCV (opencv-python 4.8.1.78, useless/requirements.txt:3) is
NOT installed here and no reference test pins its outputs, so these restatements are
**parity unpinned** against OpenCV itself.  They follow OpenCV 4.x's published CV_8U
code paths:

  * cvtColor BGR2GRAY, CV_8U: Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14
    (imgproc color_rgb: yuv_shift = 14, R2Y/G2Y/B2Y).
  * resize INTER_LINEAR, CV_8U (imgproc resize.cpp, resizeGeneric_ with
    HResizeLinear<uchar,int,short,2048> / VResizeLinear<uchar,int,short,
    FixedPtCast<...,22>>; IPP is off by default for the non-bit-exact resize):
      - dsize == ssize: copy;
      - exact 2x downscale in both axes: INTER_AREA fast path, (a+b+c+d+2) >> 2;
      - otherwise, per output column: fx = float((dx+0.5)*scale_x - 0.5),
        sx = floor(fx), fx -= sx; sx < 0 -> (sx, fx) = (0, 0); sx >= W-1 ->
        (sx, fx) = (W-1, 0); alpha = (rint((1-fx)*2048), rint(fx*2048)) as float32
        products; rows: fy likewise but NOT zeroed at the borders, source rows
        clamped to [0, H-1]; horizontal D = S[sx]*a0 + S[sx+1]*a1 (int);
        vertical dst = (((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2.
  * matchTemplate TM_CCOEFF_NORMED: OpenCV computes the cross-correlation in float32
    (DFT) and normalises with double integral images.  The restatement here is the
    exact form of the same quantity: with N = h*w, integers
        numN  = N * sum(T*I_win) - sum(T) * sum(I_win)
        varT  = N * sum(T^2)     - sum(T)^2
        varI  = N * sum(I_win^2) - sum(I_win)^2
    and OpenCV's clamp rule on t = sqrt(varI) * sqrt(varT) (float64):
        |numN| < t -> numN / t;  |numN| < 1.125 t -> sign(numN);  else 0,
    a flat template gives an all-ones map; stored as float32.  minMaxLoc returns the
    first maximum in raster order.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "bgr2gray",
    "resize_linear",
    "preprocess",
    "match_template_ccoeff_normed",
    "match_template_fft",
    "min_max_loc_max",
    "is_detection_in_corner",
    "scaled_sizes",
    "template_match_all_models",
]


def bgr2gray(img):
    """cv2.cvtColor(img, COLOR_BGR2GRAY) for uint8 (train-v4.py:65)."""
    a = np.asarray(img)
    if a.ndim == 2:
        return a.astype(np.uint8)
    a = a.astype(np.int32)
    return ((a[..., 0] * 1868 + a[..., 1] * 9617 + a[..., 2] * 4899 + 8192) >> 14).astype(np.uint8)


def _coeffs(n_in, n_out, zero_borders):
    """Source index pairs and 11-bit weights of one axis (OpenCV resizeGeneric_ setup)."""
    scale = 1.0 / (float(n_out) / float(n_in))  # inv_scale = dsize/ssize; scale = 1/inv_scale
    f = ((np.arange(n_out, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if zero_borders:
        lo = s < 0
        f[lo] = 0.0
        s[lo] = 0
        hi = s >= n_in - 1
        f[hi] = 0.0
        s[hi] = n_in - 1
    c0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    c1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    i0 = np.clip(s, 0, n_in - 1)
    i1 = np.clip(s + 1, 0, n_in - 1)
    return i0, i1, c0, c1


def resize_linear(img, dsize):
    """cv2.resize(img, dsize=(w, h)) with the default INTER_LINEAR, uint8 2-D."""
    src = np.asarray(img, dtype=np.uint8)
    w_out, h_out = int(dsize[0]), int(dsize[1])
    h_in, w_in = src.shape
    if (h_in, w_in) == (h_out, w_out):
        return src.copy()
    if w_in == 2 * w_out and h_in == 2 * h_out:  # INTER_AREA fast path (exact 2x)
        s = src.astype(np.int32)
        q = s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2]
        return ((q + 2) >> 2).astype(np.uint8)
    x0, x1, a0, a1 = _coeffs(w_in, w_out, True)
    y0, y1, b0, b1 = _coeffs(h_in, h_out, False)
    s = src.astype(np.int64)
    rows = s[:, x0] * a0 + s[:, x1] * a1  # HResizeLinear, (h_in, w_out)
    d0 = rows[y0] >> 4
    d1 = rows[y1] >> 4
    v = ((b0[:, None] * d0) >> 16) + ((b1[:, None] * d1) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def preprocess(img, size=(64, 64)):
    """train-v4.py:65-68: gray (if 3-channel BGR) -> resize -> flatten."""
    return resize_linear(bgr2gray(img), size).reshape(-1)


def _box(ii, h, w):
    return ii[h:, w:] - ii[:-h, w:] - ii[h:, :-w] + ii[:-h, :-w]


def _integral(a):
    ii = np.zeros((a.shape[0] + 1, a.shape[1] + 1), dtype=np.int64)
    ii[1:, 1:] = a.cumsum(0).cumsum(1)
    return ii


def match_template_ccoeff_normed(frame, templ):
    """cv2.matchTemplate(frame, templ, TM_CCOEFF_NORMED) (scan-template-v4.py:183), exact
    integer form + OpenCV's normalisation rule; float32 (H-h+1, W-w+1)."""
    I = np.asarray(frame, dtype=np.int64)
    T = np.asarray(templ, dtype=np.int64)
    H, W = I.shape
    h, w = T.shape
    hr, wr = H - h + 1, W - w + 1
    n = h * w
    sT, sT2 = int(T.sum()), int((T * T).sum())
    varT = n * sT2 - sT * sT
    if varT == 0:  # templNorm < DBL_EPSILON: all ones
        return np.ones((hr, wr), np.float32)
    # sum(T * I_win): exact int64 correlation, one template row at a time
    P = np.zeros((hr, wr), dtype=np.int64)
    for yy in range(h):
        rows = I[yy:yy + hr]
        for xx in range(w):
            t = T[yy, xx]
            if t:
                P += t * rows[:, xx:xx + wr]
    sI = _box(_integral(I), h, w)
    sI2 = _box(_integral(I * I), h, w)
    numN = n * P - sT * sI
    varI = n * sI2 - sI * sI
    return _normalise(numN, varI, varT)


def _normalise(numN, varI, varT):
    t = np.sqrt(varI.astype(np.float64)) * np.sqrt(np.float64(varT))
    num = numN.astype(np.float64)
    an = np.abs(num)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(an < t, num / np.where(t > 0, t, 1.0),
                     np.where(an < t * 1.125, np.sign(num), 0.0))
    return r.astype(np.float32)


def match_template_fft(frame, templ):
    """CPU baseline only (bench.py cpu_baseline leg): TM_CCOEFF_NORMED the way OpenCV
    evaluates it on the CPU — the cross-correlation by FFT (float64 here, float32 DFT in
    OpenCV), window sums from integral images, the same normalisation rule."""
    from scipy.signal import fftconvolve
    I = np.asarray(frame, dtype=np.float64)
    T = np.asarray(templ, dtype=np.float64)
    h, w = T.shape
    n = h * w
    corr = fftconvolve(I, T[::-1, ::-1], mode="valid")
    Ii = np.asarray(frame, dtype=np.int64)
    sI = _box(_integral(Ii), h, w).astype(np.float64)
    sI2 = _box(_integral(Ii * Ii), h, w).astype(np.float64)
    sT, sT2 = T.sum(), (T * T).sum()
    varT = n * sT2 - sT * sT
    if varT == 0:
        return np.ones(corr.shape, np.float32)
    num = n * corr - sT * sI
    t = np.sqrt(np.maximum(n * sI2 - sI * sI, 0.0)) * np.sqrt(varT)
    an = np.abs(num)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(an < t, num / np.where(t > 0, t, 1.0), np.where(an < t * 1.125, np.sign(num), 0.0))
    return r.astype(np.float32)


def min_max_loc_max(R):
    """(max_val, (x, y)) of cv2.minMaxLoc: first maximum in raster order."""
    R = np.asarray(R)
    i = int(np.argmax(R))
    y, x = divmod(i, R.shape[1])
    return float(R[y, x]), (x, y)


def is_detection_in_corner(det, frame_width, frame_height, corner_threshold=0.15, border_threshold=0.05):
    """scan-template-v4.py:75-125."""
    x, y, w, h = det["x"], det["y"], det["width"], det["height"]
    corner_w = int(frame_width * corner_threshold)
    corner_h = int(frame_height * corner_threshold)
    border_w = int(frame_width * border_threshold)
    border_h = int(frame_height * border_threshold)
    cx = x + w // 2
    cy = y + h // 2
    if x < border_w or y < border_h or (x + w) > (frame_width - border_w) or (y + h) > (frame_height - border_h):
        return True
    if cx < corner_w and cy < corner_h:
        return True
    if cx > (frame_width - corner_w) and cy < corner_h:
        return True
    if cx < corner_w and cy > (frame_height - corner_h):
        return True
    if cx > (frame_width - corner_w) and cy > (frame_height - corner_h):
        return True
    return False


def scaled_sizes(th, tw, fh, fw, scales=(0.8, 1.0, 1.2)):
    """scan-template-v4.py:160-168: [(scale, new_w, new_h)] that are not skipped."""
    out = []
    for s in scales:
        nw, nh = int(tw * s), int(th * s)
        if nw < 20 or nh < 20 or nw > fw or nh > fh:
            continue
        out.append((s, nw, nh))
    return out


def template_match_all_models(frame, models, threshold=0.6):
    """scan-template-v4.py:127-200.  models: {person: [template uint8 2-D, ...]} in
    iteration order; returns the detections list (x, y, width, height, person_name,
    confidence, scale)."""
    fh, fw = frame.shape[:2]
    found = []
    for person, templates in models.items():
        if not templates:
            continue
        best, best_score = None, 0.0
        for t in templates:
            for s, nw, nh in scaled_sizes(t.shape[0], t.shape[1], fh, fw):
                st = resize_linear(t, (nw, nh))
                R = match_template_ccoeff_normed(frame, st)
                mv, (mx, my) = min_max_loc_max(R)
                if mv > best_score:
                    cand = {"x": mx, "y": my, "width": nw, "height": nh, "person_name": person,
                            "confidence": mv, "scale": s}
                    if not is_detection_in_corner(cand, fw, fh):
                        best_score = mv
                        best = cand
        if best and best_score > threshold:
            found.append(best)
    return found
