"""GPU Haar cascade detector (ef_haar_detect) against oracle/haar_oracle.py on synthetic
cascades: identical candidate windows (pyramid, variance normalisation, stage sums,
skip rule) and identical grouped rectangles.  Parity against OpenCV is unpinned (no
OpenCV / cascade file here)."""
import numpy as np
import pytest

from haar_util import cascade_xml, synth_cascade, synth_frame
from oracle import haar_oracle as ho

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,shape,sf,mn,mns", [
    (0, (120, 160), 1.1, (30, 30), 5),
    (1, (96, 128), 1.2, (24, 24), 3),
    (2, (150, 100), 1.05, (0, 0), 2),
    (3, (60, 61), 1.3, (0, 0), 1),
])
def test_detect_matches_oracle(seed, shape, sf, mn, mns):
    from eigenface.haar import CascadeClassifier
    c = synth_cascade(seed, loose=0.3 * (seed % 2))
    f = synth_frame(seed, shape)
    clf = CascadeClassifier(cascade=c)
    rects, cand = clf.detect(f, sf, mns, mn, return_candidates=True)
    ref_cand = ho.candidates(f, c, sf, mn)
    assert [tuple(r) for r in cand] == ref_cand
    ref = ho.group_rectangles(ref_cand, mns)
    assert [tuple(r) for r in rects] == ref
    assert len(ref_cand) > 0  # the synthetic cascade accepts windows on these frames


def test_detect_multi_scale_surface(tmp_path):
    """cv2-style call on a cascade loaded from OpenCV's XML layout; () when nothing."""
    from eigenface.haar import CascadeClassifier
    c = synth_cascade(4, loose=0.5)
    p = tmp_path / "cascade.xml"
    p.write_text(cascade_xml(c))
    clf = CascadeClassifier(str(p))
    assert not clf.empty()
    f = synth_frame(4, (120, 160))
    out = clf.detectMultiScale(f, scaleFactor=1.1, minNeighbors=5, minSize=(30, 30))
    ref = ho.detect_multi_scale(f, c, 1.1, 5, (30, 30))
    if ref:
        assert out.dtype == np.int32 and [tuple(r) for r in out] == ref
    else:
        assert out == ()
    flat = np.full((80, 80), 100, np.uint8)  # no variance anywhere: nothing detected
    assert clf.detectMultiScale(flat) == ()


def test_detect_faces_and_save_data_layout(tmp_path):
    """detection-v4.py's crops + JSON layout from BGR frames."""
    import json
    import os
    from eigenface.haar import CascadeClassifier, detect_faces_and_save_data
    c = synth_cascade(0)
    frames = []
    for s in range(3):
        g = synth_frame(s, (120, 160))
        frames.append(np.stack([g, g, g], -1))
    out_json = tmp_path / "p" / "p_faces_detection.json"
    info = detect_faces_and_save_data(frames, str(tmp_path / "p"), str(out_json), CascadeClassifier(cascade=c), fps=25.0)
    data = json.load(open(out_json))
    assert data["total_frames"] == 3 and data["fps"] == 25.0
    assert data["total_faces_detected"] == len(data["faces"]) == len(info["faces"])
    exp = sum(len(ho.detect_multi_scale(f[..., 0], c, 1.1, 5, (30, 30))) for f in frames)
    assert len(data["faces"]) == exp
    for i, face in enumerate(data["faces"]):
        assert face["face_id"] == i and os.path.exists(face["image_path"])
        assert set(face) == {"face_id", "frame_number", "timestamp", "x", "y", "width", "height", "center_x",
                             "center_y", "area", "image_path", "image_filename"}


@pytest.mark.parametrize("tiny_leaf,nst,shape,seed", [(False, 12, (120, 160), 7), (True, 12, (120, 160), 7),
                                                      (False, 20, (150, 200), 8)])
def test_long_cascade_split_and_ordered_paths(tiny_leaf, nst, shape, seed):
    """A 12- or 20-stage cascade reaches the late stage groups (stages 1-3 in the split
    kernel, 4 on in the LDS-patch kernel when the stage sums are order-free; a 1e-12 leaf
    value makes them order-dependent and forces the sequential thread-per-window form) —
    every form must equal the oracle's candidates."""
    from eigenface.haar import CascadeClassifier
    c = synth_cascade(seed, n_feat=60, stages=tuple(range(3, 3 + 2 * nst, 2)), loose=2.0 if nst <= 12 else 2.7)
    if tiny_leaf:
        thr, stumps = c["stages"][7]
        f, t, left, right = stumps[0]
        stumps[0] = (f, t, float(np.float32(1e-12)), right)
    f = synth_frame(3, shape)
    clf = CascadeClassifier(cascade=c)
    rects, cand = clf.detect(f, 1.1, 2, (0, 0), return_candidates=True)
    ref_cand = ho.candidates(f, c, 1.1, (0, 0))
    assert len(ref_cand) > 0  # windows survive every stage, so the late groups ran
    assert [tuple(r) for r in cand] == ref_cand
    if len(ref_cand) <= 2000:  # the oracle's grouping is quadratic in pure Python
        assert [tuple(r) for r in rects] == ho.group_rectangles(ref_cand, 2)
