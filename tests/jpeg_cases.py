"""Synthetic JPEG files for the decoder tests, encoded with Pillow (libjpeg-turbo).

The expected pixels are Pillow's own libjpeg-turbo decode of the same bytes — the
library cv2.imread wraps (OpenCV bundles libjpeg-turbo), with the same defaults (islow
IDCT, fancy upsampling).  Grey output is libjpeg's JCS_GRAYSCALE (Pillow draft("L")),
what cv2.IMREAD_GRAYSCALE returns; colour is RGB reversed to BGR (IMREAD_COLOR)."""
import io

import numpy as np

try:
    from PIL import Image
except ImportError:  # pragma: no cover - Pillow is part of the image
    Image = None


def smooth_image(h, w, ch, seed):
    """Photograph-like content: low-frequency gradients + a little noise."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    out = []
    for c in range(ch):
        a, b, p = rng.uniform(0.02, 0.2, 3)
        v = 128 + 90 * np.sin(a * x + p) * np.cos(b * y + 2 * p) + rng.normal(0, 6, (h, w))
        out.append(np.clip(np.rint(v), 0, 255).astype(np.uint8))
    return out[0] if ch == 1 else np.stack(out, 2)


def noise_image(h, w, ch, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (h, w) if ch == 1 else (h, w, ch), dtype=np.uint8)


def encode(arr, **kw):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="JPEG", **kw)
    return b.getvalue()


def decode_ref(blob, mode):
    """Pillow/libjpeg-turbo decode: "gray" -> (h, w); "bgr" -> (h, w, 3)."""
    im = Image.open(io.BytesIO(blob))
    if mode == "gray":
        im.draft("L", im.size)
        return np.asarray(im.convert("L") if im.mode != "L" else im, dtype=np.uint8)
    if im.mode == "L":
        g = np.asarray(im, dtype=np.uint8)
        return np.repeat(g[..., None], 3, axis=2)
    return np.ascontiguousarray(np.asarray(im.convert("RGB"), dtype=np.uint8)[..., ::-1])


SIZES = [(1, 1), (1, 17), (17, 1), (2, 2), (3, 5), (8, 8), (9, 9), (15, 16), (16, 15), (33, 47), (64, 64),
         (100, 100), (121, 250), (250, 121)]


def corpus(seed=0):
    """(name, bytes) pairs over sampling factors, qualities, restart intervals, sizes."""
    out = []
    k = seed
    for (h, w) in SIZES:
        for sub in (0, 1, 2):  # Pillow: 0 = 4:4:4, 1 = 4:2:2, 2 = 4:2:0
            for q in (12, 75, 97):
                k += 1
                img = smooth_image(h, w, 3, k) if k % 3 else noise_image(h, w, 3, k)
                out.append((f"c{h}x{w}_s{sub}_q{q}", encode(img, quality=q, subsampling=sub)))
        k += 1
        out.append((f"g{h}x{w}", encode(smooth_image(h, w, 1, k), quality=80)))
        k += 1
        out.append((f"gn{h}x{w}", encode(noise_image(h, w, 1, k), quality=100)))
    for (h, w) in [(40, 56), (64, 64), (97, 131)]:
        for sub in (0, 2):
            for rb in (1, 3):
                k += 1
                out.append((f"r{h}x{w}_s{sub}_rb{rb}", encode(smooth_image(h, w, 3, k), quality=85, subsampling=sub,
                                                             restart_marker_blocks=rb)))
        k += 1
        out.append((f"rg{h}x{w}", encode(smooth_image(h, w, 1, k), quality=60, restart_marker_rows=1)))
    k += 1
    out.append(("opt", encode(smooth_image(70, 90, 3, k), quality=90, optimize=True)))
    return out
