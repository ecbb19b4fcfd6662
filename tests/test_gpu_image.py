"""GPU ingest (grey + resize) and template localiser against oracle/image_oracle.py,
bit for bit (integer work: exact; scores: the same float64 operations, stored float32).
Parity against OpenCV itself is unpinned (OpenCV is not installed); the oracle restates
OpenCV 4.x's CV_8U arithmetic."""
import numpy as np
import pytest

from oracle import image_oracle as io

pytestmark = pytest.mark.gpu

SHAPES = [(100, 100), (64, 64), (128, 128), (224, 230), (31, 17), (7, 200), (1, 1), (65, 130), (300, 41)]


@pytest.mark.parametrize("size", [(64, 64), (128, 128), (50, 3), (100, 100)])
def test_preprocess_grey_matches_oracle(eng, size):
    rng = np.random.default_rng(size[0])
    imgs = [rng.integers(0, 256, s, dtype=np.uint8) for s in SHAPES]
    out = eng.preprocess(imgs, size)
    assert out.shape == (len(imgs), size[0] * size[1])
    for i, im in enumerate(imgs):
        np.testing.assert_array_equal(out[i], io.preprocess(im, size), err_msg=f"image {i} {im.shape}")


def test_preprocess_colour_bgr_rgb_bgra(eng):
    rng = np.random.default_rng(7)
    imgs = [rng.integers(0, 256, s + (3,), dtype=np.uint8) for s in SHAPES]
    out = eng.preprocess(imgs, (64, 64))
    for i, im in enumerate(imgs):
        np.testing.assert_array_equal(out[i], io.preprocess(im, (64, 64)))
    rgb = eng.preprocess([im[..., ::-1].copy() for im in imgs], (64, 64), rgb=True)
    np.testing.assert_array_equal(rgb, out)
    bgra = [np.concatenate([im, rng.integers(0, 256, im.shape[:2] + (1,), dtype=np.uint8)], 2) for im in imgs]
    np.testing.assert_array_equal(eng.preprocess(bgra, (64, 64)), out)


def test_preprocess_mixed_batch_into_device_tensor(eng):
    import torch
    rng = np.random.default_rng(8)
    imgs = [rng.integers(0, 256, SHAPES[i % len(SHAPES)] + ((3,) if i % 2 else ()), dtype=np.uint8)
            for i in range(200)]
    out = torch.empty((200, 64 * 64), dtype=torch.uint8, device="cuda")
    eng.preprocess(imgs, (64, 64), out=out)
    torch.cuda.synchronize()
    ref = np.stack([io.preprocess(im) for im in imgs])
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_preprocess_bad_shape_raises(eng):
    from eigenface import EigenfaceError
    with pytest.raises(EigenfaceError):
        eng.preprocess([np.zeros((4, 4, 2), np.uint8)], (8, 8))


CASES = [  # frame (H, W), template (h, w)
    ((40, 50), (9, 12)),
    ((96, 160), (20, 24)),
    ((150, 200), (33, 70)),
    ((170, 420), (140, 30)),    # > 128 template rows: two int32 chunks
    ((60, 500), (21, 380)),     # > 352 template columns: two pieces
    ((300, 300), (1, 1)),
    ((33, 33), (33, 33)),       # 1 x 1 result
    ((200, 300), (40, 130)),    # widest 5-k-block piece: the 71 KiB correlation kernel
    ((200, 300), (40, 131)),    # narrowest 6-k-block piece: the 148 KiB kernel
    ((160, 600), (140, 40)),    # one live row block: 32 x 512 tiles, narrow kernel
    ((160, 640), (135, 200)),   # one live row block: 32 x 512 tiles, 148 KiB kernel
    ((200, 600), (150, 180)),   # two live row blocks: 64 x 256 tiles, 148 KiB kernel
    ((100, 640), (80, 400)),    # 32 x 512 tiles over two column pieces
    ((150, 700), (100, 360)),   # 64 x 256 tiles over two column pieces
    ((300, 500), (215, 90)),    # three live row blocks, one live column block, narrow kernel
    ((300, 449), (220, 150)),   # three live row blocks, two live column blocks, 148 KiB kernel
    ((300, 420), (213, 160)),   # three live row blocks, one live column block, 148 KiB kernel
]


@pytest.mark.parametrize("fs,ts", CASES)
def test_match_template_map_bit_exact(eng, fs, ts):
    rng = np.random.default_rng(fs[0] * 7 + ts[1])
    frame = rng.integers(0, 256, fs, dtype=np.uint8)
    y, x = rng.integers(0, fs[0] - ts[0] + 1), rng.integers(0, fs[1] - ts[1] + 1)
    t = frame[y:y + ts[0], x:x + ts[1]].copy()
    other = rng.integers(0, 256, ts, dtype=np.uint8)
    eng.tm_prepare([t, other], [(0,) + ts, (1,) + ts], fs)
    best, xs, ys, maps = eng.tm_match(frame, maps=True)
    for p, tt in enumerate((t, other)):
        R = io.match_template_ccoeff_normed(frame, tt)
        np.testing.assert_array_equal(maps[p], R)
        v, (mx, my) = io.min_max_loc_max(R)
        assert (best[p], xs[p], ys[p]) == (np.float32(v), mx, my)
    if ts != (1, 1):
        assert (xs[0], ys[0]) == (x, y)


def _random_case(seed):
    """A random (frame, template) shape whose oracle map costs <= ~1e9 multiply-adds:
    covers both correlation kernels, all three tile shapes (the last row band's live 32-row
    blocks), column pieces (> 352 template columns) and row chunks (> 128 template rows)."""
    rng = np.random.default_rng(1000 + seed)
    while True:
        H, W = int(rng.integers(24, 300)), int(rng.integers(40, 720))
        h, w = int(rng.integers(1, H + 1)), int(rng.integers(1, min(W, 480) + 1))
        if (H - h + 1) * (W - w + 1) * h * w <= 1e9:
            return rng, (H, W), (h, w)


@pytest.mark.parametrize("seed", range(40))
def test_match_template_random_shapes(eng, seed):
    """Random shapes, maps bit-exact to the oracle and the first raster-order maximum —
    with and without the map output (the keys-only path scores without writing maps)."""
    rng, fs, ts = _random_case(seed)
    frame = rng.integers(0, 256, fs, dtype=np.uint8)
    y, x = rng.integers(0, fs[0] - ts[0] + 1), rng.integers(0, fs[1] - ts[1] + 1)
    t = frame[y:y + ts[0], x:x + ts[1]].copy()
    other = rng.integers(0, 256, ts, dtype=np.uint8)
    eng.tm_prepare([t, other], [(0,) + ts, (1,) + ts], fs)
    best, xs, ys, maps = eng.tm_match(frame, maps=True)
    best2, xs2, ys2 = eng.tm_match(frame)
    for p, tt in enumerate((t, other)):
        R = io.match_template_ccoeff_normed(frame, tt)
        np.testing.assert_array_equal(maps[p], R)
        v, (mx, my) = io.min_max_loc_max(R)
        assert (best[p], xs[p], ys[p]) == (np.float32(v), mx, my)
        assert (best2[p], xs2[p], ys2[p]) == (best[p], xs[p], ys[p])


def test_match_template_extreme_pixels_and_flat(eng):
    """All-0/255 pixels stress the int32 partial bound; flat template -> ones; flat
    frame windows -> 0."""
    rng = np.random.default_rng(5)
    frame = (rng.integers(0, 2, (200, 420)) * 255).astype(np.uint8)
    frame[:60, :100] = 77
    t = (rng.integers(0, 2, (150, 360)) * 255).astype(np.uint8)
    flat = np.full((20, 30), 9, np.uint8)
    small = rng.integers(0, 256, (12, 10), dtype=np.uint8)
    eng.tm_prepare([t, flat, small], [(0, 150, 360), (1, 20, 30), (2, 12, 10)], frame.shape)
    best, xs, ys, maps = eng.tm_match(frame, maps=True)
    np.testing.assert_array_equal(maps[0], io.match_template_ccoeff_normed(frame, t))
    np.testing.assert_array_equal(maps[1], np.ones((181, 391), np.float32))
    R2 = io.match_template_ccoeff_normed(frame, small)
    np.testing.assert_array_equal(maps[2], R2)
    assert np.all(maps[2][:40, :80] == 0)


@pytest.mark.parametrize("force64", [False, True])
@pytest.mark.parametrize("ts", [(511, 512), (520, 510)])
def test_match_template_integral_width(eng, monkeypatch, ts, force64):
    """Integral images are wrapping uint32 while every template area is < 2^18 and int64
    otherwise (or with the EF_OPT_TM_INT64_SUMS option).  (511, 512) is the largest uint32 case: on the
    all-0 region (I' = -128) the window sum of I'^2 is 16384 * 261632, just below 2^32;
    (520, 510) has area >= 2^18 and must take the int64 form."""
    eng.set_option("tm_int64_sums", 1 if force64 else 0)
    rng = np.random.default_rng(ts[0])
    frame = (rng.integers(0, 2, (560, 540)) * 255).astype(np.uint8)
    frame[:530, :525] = 0
    frame[300:, 200:] = rng.integers(0, 256, (260, 340), dtype=np.uint8)
    t = frame[25:25 + ts[0], 12:12 + ts[1]].copy()
    try:
        eng.tm_prepare([t], [(0,) + ts], frame.shape)
        best, xs, ys, maps = eng.tm_match(frame, maps=True)
    finally:
        eng.set_option("tm_int64_sums", 0)
    R = io.match_template_ccoeff_normed(frame, t)
    np.testing.assert_array_equal(maps[0], R)
    v, (mx, my) = io.min_max_loc_max(R)
    assert (best[0], xs[0], ys[0]) == (np.float32(v), mx, my) == (np.float32(v), 12, 25)


def test_match_template_frame_past_uint32_offsets(eng):
    """a 32767 x 32767 frame has (H + 1)(W + 1) = 2^30 integral entries,
    so the uint32 form's byte offsets (uint32(entry) * 4) would wrap; ef_tm_prepare must
    pick int64 sums (ef_tm_sums_bits) even though the template area is tiny.  A random
    frame with the template cut from its far corner: the maximum (1.0) must be found there,
    with the first-max position of minMaxLoc."""
    import eigenface._native as nat
    H = W = 32767
    assert nat.lib().ef_tm_sums_bits(H, W, 24 * 24) == 64
    rng = np.random.default_rng(99)
    frame = rng.integers(0, 256, (H, W), dtype=np.uint8)
    y0, x0 = 32700, 32720
    t = frame[y0:y0 + 24, x0:x0 + 24].copy()
    eng.tm_prepare([t], [(0, 24, 24)], frame.shape)
    best, xs, ys = eng.tm_match(frame)
    assert (int(xs[0]), int(ys[0])) == (x0, y0)
    R = io.match_template_ccoeff_normed(frame[y0 - 8:y0 + 40, x0 - 8:x0 + 40], t)
    assert best[0] == np.float32(R.max()) == R[8, 8]
    eng.tm_prepare([t], [(0, 24, 24)], (32, 32))  # release the ~20 GB of operands
    del frame


def test_scaled_templates_resized_on_gpu(eng):
    """Problems at 0.8/1.2 scale: the GPU resizes the template (INTER_LINEAR) first."""
    from eigenface.image import scaled_sizes
    rng = np.random.default_rng(11)
    frame = rng.integers(0, 256, (120, 160), dtype=np.uint8)
    t = rng.integers(0, 256, (41, 37), dtype=np.uint8)
    probs = [(0, nh, nw) for _, nw, nh in scaled_sizes(41, 37, 120, 160)]
    assert len(probs) == 3
    eng.tm_prepare([t], probs, frame.shape)
    best, xs, ys, maps = eng.tm_match(frame, maps=True)
    for p, (_, nh, nw) in enumerate(probs):
        R = io.match_template_ccoeff_normed(frame, io.resize_linear(t, (nw, nh)))
        np.testing.assert_array_equal(maps[p], R)


def test_template_localiser_matches_reference_loop():
    """TemplateLocaliser.template_match_all_models == the oracle restatement of
    scan-template-v4.py:127-200 (scales, minMaxLoc, corner rule, strict '>', 0.6)."""
    from eigenface.image import TemplateLocaliser
    rng = np.random.default_rng(12)
    frame = rng.integers(0, 256, (180, 240), dtype=np.uint8)
    models = {
        "alice": [frame[60:100, 90:125].copy(), rng.integers(0, 256, (30, 30), dtype=np.uint8)],
        "bob": [rng.integers(0, 256, (25, 40), dtype=np.uint8)],
        "carol": [frame[2:40, 3:40].copy()],  # best match sits in the corner/border: skipped
    }
    loc = TemplateLocaliser(models, frame.shape)
    got = loc.template_match_all_models(frame)
    ref = io.template_match_all_models(frame, models)
    assert [(d["person_name"], d["x"], d["y"], d["width"], d["height"], d["scale"]) for d in got] == \
           [(d["person_name"], d["x"], d["y"], d["width"], d["height"], d["scale"]) for d in ref]
    for a, b in zip(got, ref):
        assert np.float32(a["confidence"]) == np.float32(b["confidence"])
    assert got and got[0]["person_name"] == "alice" and (got[0]["x"], got[0]["y"]) == (90, 60)
    # a second frame reuses the prepared operands
    frame2 = np.roll(frame, 7, axis=1)
    got2 = loc.template_match_all_models(frame2)
    ref2 = io.template_match_all_models(frame2, models)
    assert [(d["person_name"], d["x"], d["y"]) for d in got2] == [(d["person_name"], d["x"], d["y"]) for d in ref2]
