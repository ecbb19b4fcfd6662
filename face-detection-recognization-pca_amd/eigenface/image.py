"""Image side of the hot path on the GPU.

* ``preprocess_faces``   — the per-image ``cv2.cvtColor(BGR2GRAY)`` + ``cv2.resize(64, 64)``
                           of train-v4.py:59-68 / scan-template-v4.py:257-263, for a whole
                           ragged batch in one launch (``ef_preprocess``).
* ``match_template``     — ``cv2.matchTemplate(frame, templ, TM_CCOEFF_NORMED)``
                           (scan-template-v4.py:183), exact integer correlation on the int8
                           matrix cores (``ef_tm_prepare`` / ``ef_tm_match``).
* ``TemplateLocaliser``  — ``MultiModelFaceScanner.template_match_all_models``
                           (scan-template-v4.py:127-200): every model's templates at scales
                           0.8/1.0/1.2, minMaxLoc, the corner/border rule (:75-125), best per
                           model with a strict '>' and the 0.6 threshold.  Templates, their
                           scaled copies and banded operands stay resident; each frame is one
                           ``ef_tm_match`` call.

OpenCV is not installed where this was built, so parity against OpenCV's own outputs is
unpinned; the arithmetic follows OpenCV 4.x's CV_8U paths (stated in DESIGN.md) and the
tests hold the GPU to a NumPy restatement of them bit for bit.
"""
from __future__ import annotations

import numpy as np

from .pca import get_engine

SCALES = (0.8, 1.0, 1.2)  # scan-template-v4.py:161


def preprocess_faces(images, size=(64, 64), rgb=False, device=0):
    """uint8 (n, h*w) face rows from decoded images (BGR or grey; ``rgb`` for RGB order)."""
    return get_engine(device).preprocess(images, size, rgb=rgb)


def is_detection_in_corner(det, frame_width, frame_height, corner_threshold=0.15, border_threshold=0.05):
    """scan-template-v4.py:75-125 (host integer logic)."""
    x, y, w, h = det["x"], det["y"], det["width"], det["height"]
    corner_w, corner_h = int(frame_width * corner_threshold), int(frame_height * corner_threshold)
    border_w, border_h = int(frame_width * border_threshold), int(frame_height * border_threshold)
    cx, cy = x + w // 2, y + h // 2
    if x < border_w or y < border_h or (x + w) > (frame_width - border_w) or (y + h) > (frame_height - border_h):
        return True
    if cx < corner_w and cy < corner_h:
        return True
    if cx > (frame_width - corner_w) and cy < corner_h:
        return True
    if cx < corner_w and cy > (frame_height - corner_h):
        return True
    return cx > (frame_width - corner_w) and cy > (frame_height - corner_h)


def scaled_sizes(th, tw, fh, fw, scales=SCALES):
    """scan-template-v4.py:160-168: the (scale, new_w, new_h) that are not skipped."""
    out = []
    for s in scales:
        nw, nh = int(tw * s), int(th * s)
        if nw < 20 or nh < 20 or nw > fw or nh > fh:
            continue
        out.append((s, nw, nh))
    return out


def match_template(frame, templ, device=0):
    """cv2.matchTemplate(frame, templ, cv2.TM_CCOEFF_NORMED) -> float32 map."""
    f = np.ascontiguousarray(frame, dtype=np.uint8)
    t = np.ascontiguousarray(templ, dtype=np.uint8)
    if f.ndim != 2 or t.ndim != 2 or t.shape[0] > f.shape[0] or t.shape[1] > f.shape[1]:
        raise ValueError("grey frame and a template no larger than it are required")
    eng = get_engine(device)
    eng.tm_prepare([t], [(0, t.shape[0], t.shape[1])], f.shape)
    return eng.tm_match(f, maps=True)[3][0]


class TemplateLocaliser:
    """All (model, template, scale) problems of the reference's live loop, prepared once
    for a frame size and evaluated per frame on the GPU.

    ``models``: ``{person_name: [grey uint8 template, ...]}`` in the reference's model
    order (its first 5 detection faces per model, scan-template-v4.py:45-55)."""

    def __init__(self, models, frame_shape, scales=SCALES, device=0):
        self.frame_shape = (int(frame_shape[0]), int(frame_shape[1]))
        self.engine = get_engine(device)
        fh, fw = self.frame_shape
        self.templates, self.problems, self.meta = [], [], []
        for person, templates in models.items():
            for t in templates or []:
                t = np.ascontiguousarray(t, dtype=np.uint8)
                ti = len(self.templates)
                self.templates.append(t)
                for s, nw, nh in scaled_sizes(t.shape[0], t.shape[1], fh, fw, scales):
                    self.problems.append((ti, nh, nw))
                    self.meta.append((person, s, nw, nh))
        self.persons = list(models)
        self._prepared = False

    def _prepare(self):
        if not self._prepared:
            self.engine.tm_prepare(self.templates, self.problems, self.frame_shape)
            self._prepared = True

    def match(self, frame):
        """Per problem (max_val float32, x, y) of TM_CCOEFF_NORMED on ``frame``."""
        self._prepare()
        if not self.problems:
            return np.empty(0, np.float32), np.empty(0, np.int32), np.empty(0, np.int32)
        return self.engine.tm_match(frame)

    def template_match_all_models(self, frame, threshold=0.6):
        """scan-template-v4.py:127-200: best non-corner match per model above threshold."""
        fh, fw = self.frame_shape
        best_v, xs, ys = self.match(frame)
        found = []
        per_person = {}
        for (person, s, nw, nh), v, x, y in zip(self.meta, best_v, xs, ys):
            per_person.setdefault(person, []).append((float(v), int(x), int(y), nw, nh, s))
        for person in self.persons:
            best, best_score = None, 0.0
            for v, x, y, nw, nh, s in per_person.get(person, []):
                if v > best_score:
                    cand = {"x": x, "y": y, "width": nw, "height": nh, "person_name": person,
                            "confidence": v, "scale": s}
                    if not is_detection_in_corner(cand, fw, fh):
                        best_score = v
                        best = cand
            if best and best_score > threshold:
                found.append(best)
        return found
