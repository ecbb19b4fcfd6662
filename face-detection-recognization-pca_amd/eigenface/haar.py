"""Haar cascade face detector on the GPU: a drop-in for the
``cv2.CascadeClassifier(...).detectMultiScale(gray, scaleFactor=1.1, minNeighbors=5,
minSize=(30, 30))`` call of detection-v4.py:18, :50-55.

``load_cascade`` reads OpenCV's cascade XML (the ``opencv-cascade-classifier`` format of
``cv2.data.haarcascades``; BOOST stages of HAAR stumps, no tilted features) into plain
arrays; ``CascadeClassifier.detectMultiScale`` runs the pyramid, variance normalisation
and the cascade on the GPU (``ef_haar_detect``) and returns cv2's result layout — an
``(n, 4)`` int32 array of ``x, y, w, h``, or an empty tuple when nothing is found.

OpenCV (and so its cascade files) is not installed where this was built: parity against
OpenCV's detector is unpinned.  One documented deviation: OpenCV resizes its pyramid with
INTER_LINEAR_EXACT, this engine with INTER_LINEAR.
"""
from __future__ import annotations

import ctypes as C
import xml.etree.ElementTree as ET

import numpy as np

from .pca import get_engine


def _nums(text):
    return [float(v) for v in text.split()]


def load_cascade(path):
    """OpenCV cascade XML -> {"win": (w, h), "features": [[(x, y, w, h, weight), ...]],
    "stages": [(threshold, [(feature, threshold, left, right), ...])]}."""
    root = ET.parse(path).getroot()
    cas = root.find("cascade")
    if cas is None:
        raise ValueError(f"{path}: not an opencv-cascade-classifier file (old-format cascades are not supported)")
    if (cas.findtext("stageType") or "").strip() != "BOOST" or (cas.findtext("featureType") or "").strip() != "HAAR":
        raise ValueError(f"{path}: only BOOST / HAAR cascades are supported")
    win = (int(cas.findtext("width")), int(cas.findtext("height")))
    stages = []
    for st in cas.find("stages"):
        thr = float(st.findtext("stageThreshold"))
        stumps = []
        for wc in st.find("weakClassifiers"):
            nodes = _nums(wc.findtext("internalNodes"))
            leaves = _nums(wc.findtext("leafValues"))
            if len(nodes) != 4 or len(leaves) != 2:
                raise ValueError(f"{path}: only depth-1 trees (stumps) are supported")
            stumps.append((int(nodes[2]), nodes[3], leaves[0], leaves[1]))
        stages.append((thr, stumps))
    feats = []
    for f in cas.find("features"):
        if int(f.findtext("tilted") or 0):
            raise ValueError(f"{path}: tilted features are not supported")
        rects = [tuple(_nums(r.text)) for r in f.find("rects")]
        feats.append([(int(r[0]), int(r[1]), int(r[2]), int(r[3]), r[4]) for r in rects])
    return {"win": win, "features": feats, "stages": stages}


class CascadeClassifier:
    """cv2.CascadeClassifier lookalike backed by libeigenface (one GPU per process)."""

    def __init__(self, filename=None, cascade=None, device=0, engine=None):
        self.engine = engine if engine is not None else get_engine(device)
        self.cascade = None
        if filename is not None:
            self.load(filename)
        elif cascade is not None:
            self.set_cascade(cascade)

    def empty(self):
        return self.cascade is None

    def load(self, filename):
        self.set_cascade(load_cascade(filename))
        return True

    def set_cascade(self, cascade):
        feats = cascade["features"]
        nf = len(feats)
        rects = np.zeros((nf, 3, 4), np.int32)
        wts = np.zeros((nf, 3), np.float32)
        for i, f in enumerate(feats):
            if not 2 <= len(f) <= 3:
                raise ValueError("HAAR features have 2 or 3 rectangles")
            for k, (x, y, w, h, wt) in enumerate(f):
                rects[i, k] = (x, y, w, h)
                wts[i, k] = wt
        counts = np.array([len(s[1]) for s in cascade["stages"]], np.int32)
        sthr = np.array([s[0] for s in cascade["stages"]], np.float32)
        st = [sp for s in cascade["stages"] for sp in s[1]]
        sf = np.array([p[0] for p in st], np.int32)
        st_thr = np.array([p[1] for p in st], np.float32)
        sl = np.array([p[2] for p in st], np.float32)
        sr = np.array([p[3] for p in st], np.float32)
        e = self.engine
        e._chk(e._lib.ef_haar_set_cascade(e._h, int(cascade["win"][0]), int(cascade["win"][1]), nf, rects.ctypes.data,
                                          wts.ctypes.data, len(counts), counts.ctypes.data, sthr.ctypes.data, len(st),
                                          sf.ctypes.data, st_thr.ctypes.data, sl.ctypes.data, sr.ctypes.data))
        self.cascade = cascade

    def detect(self, image, scaleFactor=1.1, minNeighbors=3, minSize=(), maxSize=(), return_candidates=False):
        """(rects (n, 4) int32, candidates (m, 4) int32 or None)."""
        if self.cascade is None:
            raise RuntimeError("no cascade loaded")
        g = np.ascontiguousarray(image, dtype=np.uint8)
        if g.ndim != 2:
            raise ValueError("detectMultiScale expects a grey image (cv2.cvtColor(frame, COLOR_BGR2GRAY))")
        H, W = g.shape
        mn = tuple(minSize) if minSize else (0, 0)
        mx = tuple(maxSize) if maxSize else (0, 0)
        cap = 4096
        e = self.engine
        while True:
            out = np.empty((cap, 4), np.int32)
            cand = np.empty((cap, 4), np.int32) if return_candidates else None
            n, nc = C.c_int32(0), C.c_int32(0)
            e._chk(e._lib.ef_haar_detect(e._h, g.ctypes.data, H, W, W, float(scaleFactor), int(minNeighbors),
                                         int(mn[0]), int(mn[1]), int(mx[0]), int(mx[1]), out.ctypes.data, cap,
                                         C.byref(n), cand.ctypes.data if cand is not None else None,
                                         cap if cand is not None else 0, C.byref(nc), 0))
            if n.value <= cap and (cand is None or nc.value <= cap):
                break
            cap = max(n.value, nc.value)
        rects = out[: n.value].copy()
        return rects, (cand[: nc.value].copy() if cand is not None else None)

    def detectMultiScale(self, image, scaleFactor=1.1, minNeighbors=3, flags=0, minSize=(), maxSize=()):
        """cv2.CascadeClassifier.detectMultiScale: (n, 4) int32 array, or () if none."""
        rects, _ = self.detect(image, scaleFactor, minNeighbors, minSize, maxSize)
        return rects if len(rects) else ()


def _frames_from_video(path):
    """(frames iterator, fps, total_frames) via OpenCV's VideoCapture (video decode is host
    I/O outside this engine; without OpenCV, pass decoded frames instead)."""
    import cv2  # noqa: F401 - optional dependency, raises ImportError when absent

    cap = cv2.VideoCapture(path)
    if not cap.isOpened():
        return None, 0.0, 0

    def gen():
        while True:
            ok, fr = cap.read()
            if not ok:
                break
            yield fr
        cap.release()

    return gen(), cap.get(cv2.CAP_PROP_FPS), int(cap.get(cv2.CAP_PROP_FRAME_COUNT))


def detect_faces_and_save_data(video_or_frames, output_face_dir, output_json_path, cascade,
                               fps=0.0, total_frames=None, video_path=None, device=0):
    """detection-v4.py:8-114: per frame grey (GPU, BT.601 fixed point) -> detectMultiScale(
    1.1, 5, (30, 30)) on the GPU -> face crops ``face_{id:06d}_frame_{n:06d}.jpg`` and the
    ``{person}_faces_detection.json`` layout.  ``video_or_frames`` is a
    video path (needs OpenCV for decoding) or an iterable of BGR uint8 frames."""
    import json
    import os
    from datetime import datetime

    from .compat import _save_bgr_jpg

    clf = cascade if isinstance(cascade, CascadeClassifier) else CascadeClassifier(cascade, device=device)
    if isinstance(video_or_frames, str):
        frames, fps, total_frames = _frames_from_video(video_or_frames)
        if frames is None:
            print(f"Error: Could not open video {video_or_frames}")
            return None
        video_path = video_or_frames
    else:
        frames = video_or_frames
    os.makedirs(output_face_dir, exist_ok=True)
    eng = get_engine(device)
    faces, face_id, n = [], 0, 0
    for frame in frames:
        frame = np.ascontiguousarray(frame, dtype=np.uint8)
        gray = eng.preprocess([frame], (frame.shape[1], frame.shape[0]))[0].reshape(frame.shape[:2])
        found = clf.detectMultiScale(gray, scaleFactor=1.1, minNeighbors=5, minSize=(30, 30))
        for (x, y, w, h) in found:
            fn = f"face_{face_id:06d}_frame_{n:06d}.jpg"
            fp = os.path.join(output_face_dir, fn)
            _save_bgr_jpg(fp, frame[y:y + h, x:x + w])
            faces.append({"face_id": face_id, "frame_number": n, "timestamp": n / fps if fps > 0 else 0,
                          "x": int(x), "y": int(y), "width": int(w), "height": int(h),
                          "center_x": int(x + w // 2), "center_y": int(y + h // 2), "area": int(w * h),
                          "image_path": fp, "image_filename": fn})
            face_id += 1
        n += 1
    info = {"video_path": video_path, "total_frames": total_frames if total_frames is not None else n, "fps": fps,
            "total_faces_detected": len(faces), "processing_date": datetime.now().isoformat(), "faces": faces}
    os.makedirs(os.path.dirname(os.path.abspath(output_json_path)), exist_ok=True)
    with open(output_json_path, "w", encoding="utf-8") as f:
        json.dump(info, f, indent=2, ensure_ascii=False)
    return info


__all__ = ["load_cascade", "CascadeClassifier", "detect_faces_and_save_data"]
