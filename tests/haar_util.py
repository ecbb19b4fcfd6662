"""Synthetic HAAR cascades and frames for the detector tests (no OpenCV cascade file
exists here: haarcascade_frontalface_default.xml ships inside OpenCV, which is absent)."""
import numpy as np


def synth_cascade(seed=0, win=(24, 24), n_feat=40, stages=(3, 5, 7, 9), loose=0.0):
    """Random 2/3-rectangle edge/line features with OpenCV-style weights; stump
    thresholds ~ typical normalised feature values; stage thresholds permissive enough
    that every stage both passes and rejects windows on structured frames."""
    rng = np.random.default_rng(seed)
    ww, wh = win
    feats = []
    for _ in range(n_feat):
        w = int(rng.integers(2, ww // 2)) * 2 // 2
        h = int(rng.integers(2, wh // 2))
        x = int(rng.integers(0, ww - 2 * w + 1))
        y = int(rng.integers(0, wh - h + 1))
        if rng.random() < 0.5:  # two-rectangle edge feature: whole * -1 + half * 2
            feats.append([(x, y, 2 * w, h, -1.0), (x + w, y, w, h, 2.0)])
        else:  # three-rectangle line feature (x3 weight on the middle third)
            w3 = max(1, (2 * w) // 3)
            feats.append([(x, y, 3 * w3, h, -1.0), (x + w3, y, w3, h, 3.0), (0, 0, 0, 0, 0.0)][:2 + int(rng.random() < 0.3)])
    st = []
    fi = 0
    for si, n in enumerate(stages):
        stumps = []
        for _ in range(n):
            thr = float(np.float32(rng.normal(0.0, 0.02)))
            left, right = float(np.float32(rng.uniform(-1, 0.2))), float(np.float32(rng.uniform(-0.2, 1)))
            stumps.append((fi % n_feat, thr, left, right))
            fi += 1
        st.append((float(np.float32(-0.35 * n + loose)), stumps))
    return {"win": win, "features": feats, "stages": st}


def synth_frame(seed=0, shape=(120, 160)):
    """Grey frame with smooth background, bright/dark boxes and noise (structure for the
    features, flat patches for the variance rejection)."""
    rng = np.random.default_rng(seed)
    H, W = shape
    yy, xx = np.mgrid[0:H, 0:W]
    f = 90 + 40 * np.sin(xx / 17.0) * np.cos(yy / 23.0)
    for _ in range(8):
        y0, x0 = rng.integers(0, H - 20), rng.integers(0, W - 20)
        h, w = rng.integers(10, 40), rng.integers(10, 40)
        f[y0:y0 + h, x0:x0 + w] += rng.uniform(-60, 60)
    f += rng.normal(0, 6, f.shape)
    f[: H // 6, : W // 6] = 128  # flat corner: low-variance windows
    return np.clip(np.rint(f), 0, 255).astype(np.uint8)


def cascade_xml(c):
    """Write a cascade dict in OpenCV's opencv-cascade-classifier XML layout."""
    ww, wh = c["win"]
    out = ['<?xml version="1.0"?>', "<opencv_storage>", '<cascade type_id="opencv-cascade-classifier">',
           "<stageType>BOOST</stageType>", "<featureType>HAAR</featureType>", f"<height>{wh}</height>",
           f"<width>{ww}</width>", f"<stageNum>{len(c['stages'])}</stageNum>", "<stages>"]
    for thr, stumps in c["stages"]:
        out += ["<_>", f"<maxWeakCount>{len(stumps)}</maxWeakCount>", f"<stageThreshold>{thr!r}</stageThreshold>",
                "<weakClassifiers>"]
        for fi, t, l, r in stumps:
            out.append(f"<_><internalNodes>\n 0 -1 {fi} {t!r}</internalNodes><leafValues>\n {l!r} {r!r}</leafValues></_>")
        out += ["</weakClassifiers>", "</_>"]
    out += ["</stages>", "<features>"]
    for f in c["features"]:
        out.append("<_><rects>" + "".join(f"<_>\n {x} {y} {w} {h} {wt!r}</_>" for x, y, w, h, wt in f) + "</rects></_>")
    out += ["</features>", "</cascade>", "</opencv_storage>"]
    return "\n".join(out)
