"""JPEG header parse (ef_jpeg_info, host-only, no GPU) against Pillow's view of the same
files: dimensions, component count, and which files the GPU decoder takes."""
import io

import numpy as np

import jpeg_cases as J


def test_info_matches_pillow_over_corpus():
    from eigenface.engine import jpeg_info
    cases = J.corpus()
    h, w, c, st = jpeg_info([b for _, b in cases])
    assert (st == 0).all()
    for (name, b), hh, ww, cc in zip(cases, h, w, c):
        from PIL import Image
        im = Image.open(io.BytesIO(b))
        assert (im.height, im.width) == (hh, ww), name
        assert cc == (1 if im.mode == "L" else 3), name


def test_info_statuses():
    from PIL import Image
    from eigenface.engine import jpeg_info
    prog = J.encode(J.smooth_image(16, 16, 3, 0), progressive=True)
    b = io.BytesIO()
    Image.fromarray(J.smooth_image(16, 16, 3, 1)).convert("CMYK").save(b, format="JPEG")
    png = io.BytesIO()
    Image.fromarray(J.smooth_image(8, 8, 3, 2)).save(png, format="PNG")
    _, _, _, st = jpeg_info([prog, b.getvalue(), png.getvalue(), b"", b"\xff\xd8"])
    np.testing.assert_array_equal(st, [-10, -10, -11, -11, -11])
