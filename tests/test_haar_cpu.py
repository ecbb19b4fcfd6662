"""CPU checks of the Haar detector's oracle and host logic: cv::groupRectangles
restatement, the invoker's skip rule, scale list, and the product's cascade-XML loader."""
import numpy as np

from haar_util import cascade_xml, synth_cascade, synth_frame
from oracle import haar_oracle as ho


def test_group_rectangles_rules():
    a = [(10, 10, 30, 30)] * 6 + [(11, 10, 30, 31)]          # one cluster of 7
    b = [(100, 100, 40, 40)] * 3                             # below the neighbour threshold
    inner = [(14, 14, 20, 20)] * 6                           # inside the first (n2 > max(3, n1))
    got = ho.group_rectangles(a + b + inner, 5)
    assert got == [(10, 10, 30, 30)]
    # averaging uses float 1/n and round-half-even
    assert ho.group_rectangles([(0, 0, 10, 10), (1, 1, 11, 11)] * 3, 2) == [(0, 0, 10, 10)]
    assert ho.group_rectangles(a, 0) == a


def test_partition_numbers_classes_by_lowest_member():
    rects = [(0, 0, 10, 10), (200, 200, 10, 10), (1, 0, 10, 10), (200, 201, 10, 10), (500, 0, 10, 10)]
    labels, n = ho.partition(rects, 0.2)
    assert labels == [0, 1, 0, 1, 2] and n == 3


def test_scale_list_matches_min_size_rule():
    sc = ho.scale_list((24, 24), (640, 480), 1.1, (30, 30))
    assert abs(sc[0] - 1.331) < 1e-6 and round(24 * float(sc[0])) >= 30
    assert round(24 * float(sc[-1])) <= 480 and round(24 * float(sc[-1]) * 1.1) > 480


def test_candidates_skip_rule():
    """A stage-0 rejection skips the next x position (CascadeClassifierInvoker)."""
    c = synth_cascade(1)
    f = synth_frame(1, (60, 80))
    res = ho.eval_layer(f, c)
    cand = ho.candidates(f, c, 1.1, (24, 24), (24, 24))  # one scale: factor 1
    exp = []
    for y in range(0, res.shape[0], 2):
        x = 0
        while x < res.shape[1]:
            if res[y, x] > 0:
                exp.append((x, y, 24, 24))
            x += 4 if res[y, x] == 0 else 2
    assert cand == exp
    assert (res == -1).any() and (res == 0).any() and (res == 1).any()


def test_load_cascade_roundtrip(tmp_path):
    from eigenface.haar import load_cascade
    c = synth_cascade(2)
    p = tmp_path / "c.xml"
    p.write_text(cascade_xml(c))
    got = load_cascade(str(p))
    assert got["win"] == c["win"]
    assert [[tuple(r) for r in f] for f in got["features"]] == [[tuple(r) for r in f] for f in c["features"]]
    assert got["stages"] == c["stages"]
