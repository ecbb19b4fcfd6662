"""CPU checks of the image-side oracle (oracle/image_oracle.py) and the host logic of
eigenface.image: OpenCV-rule restatements of cvtColor/resize/matchTemplate (parity
against OpenCV itself is unpinned: OpenCV is not installed) and the reference's
scale/corner rules (scan-template-v4.py:75-125, :160-168)."""
import numpy as np
import pytest

from oracle import image_oracle as io


def test_bgr2gray_fixed_point():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [10, 200, 30]]],
                  np.uint8)
    g = io.bgr2gray(px)[0]
    # (1868 B + 9617 G + 4899 R + 8192) >> 14
    assert list(g) == [29, 150, 76, 255, 0, (10 * 1868 + 200 * 9617 + 30 * 4899 + 8192) >> 14]


def test_resize_identity_area_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    np.testing.assert_array_equal(io.resize_linear(img, (53, 37)), img)
    big = rng.integers(0, 256, (64, 96), dtype=np.uint8)
    q = big.astype(int)
    ref = (q[0::2, 0::2] + q[0::2, 1::2] + q[1::2, 0::2] + q[1::2, 1::2] + 2) >> 2
    np.testing.assert_array_equal(io.resize_linear(big, (48, 32)), ref)
    for shape, size in [((100, 100), (64, 64)), ((31, 17), (64, 64)), ((224, 230), (64, 64)), ((7, 200), (50, 3))]:
        flat = np.full(shape, 173, np.uint8)
        np.testing.assert_array_equal(io.resize_linear(flat, size), np.full(size[::-1], 173, np.uint8))


def test_resize_close_to_float_bilinear():
    """The fixed-point result stays within 1 of an exact float64 bilinear evaluation."""
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (100, 90), dtype=np.uint8)
    out = io.resize_linear(img, (64, 64)).astype(float)

    def axis(n_in, n_out):
        f = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        s = np.floor(f).astype(int)
        a = f - s
        return np.clip(s, 0, n_in - 1), np.clip(s + 1, 0, n_in - 1), a
    y0, y1, fy = axis(100, 64)
    x0, x1, fx = axis(90, 64)
    im = img.astype(float)
    top = im[y0][:, x0] * (1 - fx) + im[y0][:, x1] * fx
    bot = im[y1][:, x0] * (1 - fx) + im[y1][:, x1] * fx
    ref = top * (1 - fy[:, None]) + bot * fy[:, None]
    assert np.abs(out - ref).max() <= 1.0


def _ncc_float(frame, t):
    H, W = frame.shape
    h, w = t.shape
    tt = t - t.mean()
    out = np.zeros((H - h + 1, W - w + 1))
    for y in range(H - h + 1):
        for x in range(W - w + 1):
            win = frame[y:y + h, x:x + w].astype(float)
            ww = win - win.mean()
            den = np.sqrt((ww * ww).sum() * (tt * tt).sum())
            out[y, x] = (ww * tt).sum() / den if den > 0 else 0.0
    return out


def test_match_template_matches_float_ncc_and_planted_location():
    rng = np.random.default_rng(2)
    frame = rng.integers(0, 256, (40, 50), dtype=np.uint8)
    t = frame[11:11 + 9, 23:23 + 12].copy()
    R = io.match_template_ccoeff_normed(frame, t)
    assert R.shape == (32, 39) and R.dtype == np.float32
    np.testing.assert_allclose(R, _ncc_float(frame, t), atol=1e-6)
    v, (x, y) = io.min_max_loc_max(R)
    assert (x, y) == (23, 11) and v == pytest.approx(1.0, abs=1e-7)


def test_match_template_flat_cases():
    frame = np.full((20, 30), 9, np.uint8)
    frame[5:, 10:] = np.arange(15 * 20).reshape(15, 20) % 251
    t = np.full((4, 6), 200, np.uint8)
    np.testing.assert_array_equal(io.match_template_ccoeff_normed(frame, t), np.ones((17, 25), np.float32))
    t2 = np.arange(24, dtype=np.uint8).reshape(4, 6)
    R = io.match_template_ccoeff_normed(frame, t2)
    assert np.all(R[:2, :5] == 0.0)  # flat windows score 0 (OpenCV rule)


def test_min_max_loc_first_in_raster_order():
    R = np.zeros((4, 5), np.float32)
    R[2, 1] = R[1, 3] = 0.5
    assert io.min_max_loc_max(R) == (0.5, (3, 1))


def test_host_rules_match_oracle():
    from eigenface import image as im
    rng = np.random.default_rng(3)
    for _ in range(500):
        fw, fh = int(rng.integers(100, 700)), int(rng.integers(100, 500))
        d = {"x": int(rng.integers(0, fw)), "y": int(rng.integers(0, fh)),
             "width": int(rng.integers(10, 200)), "height": int(rng.integers(10, 200))}
        assert im.is_detection_in_corner(d, fw, fh) == io.is_detection_in_corner(d, fw, fh)
        th, tw = int(rng.integers(5, 400)), int(rng.integers(5, 400))
        assert im.scaled_sizes(th, tw, fh, fw) == io.scaled_sizes(th, tw, fh, fw)
