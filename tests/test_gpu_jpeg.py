"""GPU JPEG decode (include/eigenface.h ef_jpeg_decode / ef_jpeg_ingest) against
libjpeg-turbo, bit for bit.  The oracle is Pillow's libjpeg-turbo decode of the same
bytes (tests/jpeg_cases.py): the library behind cv2.imread, which the reference calls
per file (train-v4.py:59, useless/train.py:33, scan-template-v4.py:52)."""
import io

import numpy as np
import pytest

import jpeg_cases as J
from oracle import image_oracle as io_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def corpus():
    return J.corpus()


@pytest.mark.parametrize("mode", ["bgr", "gray"])
def test_decode_matches_libjpeg_turbo(eng, corpus, mode):
    got = eng.decode_jpegs([b for _, b in corpus], mode)
    for (name, b), g in zip(corpus, got):
        ref = J.decode_ref(b, mode)
        assert g is not None, name
        np.testing.assert_array_equal(g, ref, err_msg=f"{mode} {name}")


def _progressive():
    return J.encode(J.smooth_image(40, 40, 3, 1), quality=80, progressive=True)


def _cmyk():
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(J.smooth_image(16, 16, 3, 2)).convert("CMYK").save(b, format="JPEG")
    return b.getvalue()


def test_unsupported_and_corrupt_files_are_reported(eng):
    good = J.encode(J.smooth_image(30, 20, 3, 3), quality=90)
    blobs = [good, _progressive(), _cmyk(), b"\xff\xd8\xff\xe0garbage", b"", good[:40], good]
    from eigenface.engine import jpeg_info
    _, _, _, st = jpeg_info(blobs)
    assert st[0] == 0 and st[6] == 0
    assert st[1] == -10 and st[2] == -10           # progressive, CMYK: EF_JPEG_E_UNSUPPORTED
    assert st[3] == -11 and st[4] == -11 and st[5] == -11  # EF_JPEG_E_CORRUPT
    got = eng.decode_jpegs(blobs, "bgr")
    ref = J.decode_ref(good, "bgr")
    np.testing.assert_array_equal(got[0], ref)
    np.testing.assert_array_equal(got[6], ref)
    assert all(g is None for g in got[1:6])


def test_damaged_entropy_data_decodes_without_fault(eng):
    """Flipped bits and a truncated scan: libjpeg warns and feeds zeros; the decoder must
    stay in bounds (shape right, no fault) — the pixel values of a damaged stream are not
    pinned."""
    rng = np.random.default_rng(5)
    blobs = []
    for k in range(40):
        b = bytearray(J.encode(J.smooth_image(48, 64, 3, k), quality=70, subsampling=k % 3))
        sos = b.find(b"\xff\xda")
        for _ in range(8):
            i = int(rng.integers(sos + 14, len(b) - 2))
            b[i] ^= 1 << int(rng.integers(0, 8))
        blobs.append(bytes(b if k % 2 else b[:len(b) * 3 // 4]))
    got = eng.decode_jpegs(blobs, "bgr")
    for g in got:
        assert g is None or g.shape == (48, 64, 3)
    # the engine is still healthy
    good = J.encode(J.smooth_image(20, 20, 3, 9))
    np.testing.assert_array_equal(eng.decode_jpegs([good], "bgr")[0], J.decode_ref(good, "bgr"))


@pytest.mark.parametrize("mode", ["bgr", "gray"])
def test_ingest_equals_decode_then_preprocess(eng, corpus, mode):
    """ef_jpeg_ingest (decode -> grey -> INTER_LINEAR 64x64 on the GPU, no host round
    trip) equals libjpeg's pixels through the resize oracle."""
    blobs = [b for _, b in corpus] + [_progressive()]
    rows, st = eng.ingest_jpegs(blobs, (64, 64), mode)
    assert (st[:-1] == 0).all() and st[-1] == -10
    assert not rows[-1].any()
    for i, (name, b) in enumerate(corpus):
        np.testing.assert_array_equal(rows[i], io_oracle.preprocess(J.decode_ref(b, mode), (64, 64)),
                                      err_msg=f"{mode} {name}")


def test_ingest_into_device_tensor_large_batch(eng):
    import torch
    n = 3000
    blobs = [J.encode(J.smooth_image(90 + k % 23, 70 + k % 17, 3, k), quality=60 + k % 40, subsampling=k % 3,
                      **({"restart_marker_blocks": 1 + k % 4} if k % 5 == 0 else {})) for k in range(n)]
    out = torch.empty((n, 64 * 64), dtype=torch.uint8, device="cuda")
    _, st = eng.ingest_jpegs(blobs, (64, 64), "bgr", out=out)
    torch.cuda.synchronize()
    assert (st == 0).all()
    rows = out.cpu().numpy()
    for i in range(0, n, 97):
        np.testing.assert_array_equal(rows[i], io_oracle.preprocess(J.decode_ref(blobs[i], "bgr"), (64, 64)))


def test_ingest_parts_host_output_status(eng):
    """The ingest decodes in parts (EF_OPT_JPEG_PART_FILES; the next part staged on a host thread):
    statuses and rows land at every part's offsets, host and device outputs agree, and
    files the decoder does not take (progressive) give zero rows in any part."""
    import torch
    n = 2500
    blobs = [J.encode(J.smooth_image(60 + k % 29, 50 + k % 31, 3, k), quality=70 + k % 25, subsampling=k % 3)
             for k in range(n)]
    bad = [5, 1023, 1024, 1700, 2499]
    for i in bad:
        blobs[i] = _progressive()
    eng.set_option("jpeg_part_files", 1024)  # three parts
    try:
        rows, st = eng.ingest_jpegs(blobs, (64, 64), "gray")
        one_rows, one_st = None, None
        eng.set_option("jpeg_part_files", 8192)  # one part
        one_rows, one_st = eng.ingest_jpegs(blobs, (64, 64), "gray")
    finally:
        eng.set_option("jpeg_part_files", 8192)
    np.testing.assert_array_equal(one_st, st)
    np.testing.assert_array_equal(one_rows, rows)
    assert [i for i in range(n) if st[i] != 0] == bad
    assert all(st[i] == -10 for i in bad)
    assert not rows[bad].any()
    out = torch.empty((n, 64 * 64), dtype=torch.uint8, device="cuda")
    eng.set_option("jpeg_part_files", 1000)
    try:
        _, st2 = eng.ingest_jpegs(blobs, (64, 64), "gray", out=out)
    finally:
        eng.set_option("jpeg_part_files", 8192)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st2, st)
    np.testing.assert_array_equal(out.cpu().numpy(), rows)
    for i in [0, 1022, 1025, 1699, 1701, 2498]:
        np.testing.assert_array_equal(rows[i], io_oracle.preprocess(J.decode_ref(blobs[i], "gray"), (64, 64)))


@pytest.mark.parametrize("chunk_bits", [64, 512])
def test_unconverged_rounds_finish_on_device(eng, corpus, chunk_bits):
    """Chunks far shorter than the self-synchronisation distance: the queued rounds do not
    reach the fixed point (64-bit chunks need one round per chunk, ~1100 on this corpus), so
    jpeg_finish_kernel completes every segment sequentially on the device — still bit-exact."""
    blobs = [b for _, b in corpus]
    eng.set_option("jpeg_chunk_bits", chunk_bits)
    try:
        got = eng.decode_jpegs(blobs, "bgr")
        rows, st = eng.ingest_jpegs(blobs, (64, 64), "gray")
    finally:
        eng.set_option("jpeg_chunk_bits", 0)
    assert (st == 0).all()
    for (name, b), g, r in zip(corpus, got, rows):
        np.testing.assert_array_equal(g, J.decode_ref(b, "bgr"), err_msg=f"{chunk_bits} {name}")
        np.testing.assert_array_equal(r, io_oracle.preprocess(J.decode_ref(b, "gray"), (64, 64)),
                                      err_msg=f"{chunk_bits} {name}")


def test_back_to_back_device_ingests(eng):
    """Device-output ingests return once queued: consecutive calls alternate the two upload
    slots, the next call's staging overlapping this call's decode.  Four calls of different
    batches (and sizes, so buffers grow in between) into separate tensors, one sync at the
    end: every row equals a synchronous host-output ingest of the same batch."""
    import torch
    batches = []
    for c, n in enumerate([700, 1300, 400, 1300]):
        batches.append([J.encode(J.smooth_image(40 + (k * 7 + c) % 90, 50 + (k * 3 + c) % 70, 3, 1000 * c + k),
                                 quality=55 + (k + c) % 45, subsampling=(k + c) % 3) for k in range(n)])
    outs = [torch.empty((len(b), 32 * 32), dtype=torch.uint8, device="cuda") for b in batches]
    sts = [eng.ingest_jpegs(b, (32, 32), "bgr", out=o)[1] for b, o in zip(batches, outs)]
    torch.cuda.synchronize()
    for b, o, st in zip(batches, outs, sts):
        ref, ref_st = eng.ingest_jpegs(b, (32, 32), "bgr")
        np.testing.assert_array_equal(st, ref_st)
        np.testing.assert_array_equal(o.cpu().numpy(), ref)
    for i in range(0, len(batches[1]), 101):
        np.testing.assert_array_equal(outs[1][i].cpu().numpy(),
                                      io_oracle.preprocess(J.decode_ref(batches[1][i], "bgr"), (32, 32)))


def test_device_ingest_ordered_on_torch_stream(eng):
    """A device-output ingest on the engine's own stream orders torch's current stream
    after the decode (event wait, no host sync): torch work queued after the call — a
    clone, and a reduction read after only a stream-level synchronize — sees the decoded
    rows, and the output's memory is not reused while the decode still writes it."""
    import torch
    eng.use_own_stream()
    blobs = [J.encode(J.smooth_image(60 + k % 50, 70 + k % 40, 3, 500 + k), quality=80, subsampling=k % 3)
             for k in range(900)]
    ref, ref_st = eng.ingest_jpegs(blobs, (32, 32), "bgr")
    out = torch.empty((len(blobs), 32 * 32), dtype=torch.uint8, device="cuda")
    st = eng.ingest_jpegs(blobs, (32, 32), "bgr", out=out)[1]
    copy = out.clone()                      # queued on torch's stream right after the call
    total = out.to(torch.int64).sum()
    del out                                 # its block may be reused only after the decode
    junk = torch.full((len(blobs), 32 * 32), 7, dtype=torch.uint8, device="cuda")
    torch.cuda.current_stream().synchronize()
    np.testing.assert_array_equal(st, ref_st)
    np.testing.assert_array_equal(copy.cpu().numpy(), ref)
    assert int(total) == int(ref.astype(np.int64).sum())
    assert int(junk.sum()) == 7 * junk.numel()


def test_ingest_wide_sources_read_planes_directly(eng):
    """Sources whose band of rows exceeds the fused resize's LDS budget (large frames) take its
    direct-read path; small ones in the same call the LDS-staged path — both equal libjpeg's
    pixels through the resize oracle, for 4:2:0, 4:2:2, 4:4:4 and grey files."""
    blobs = [J.encode(J.smooth_image(1200, 1500, 3, 31), quality=85, subsampling=0),
             J.encode(J.smooth_image(900, 1700, 3, 32), quality=75, subsampling=1),
             J.encode(J.smooth_image(1100, 640, 3, 33), quality=90, subsampling=2),
             J.encode(J.smooth_image(700, 1300, 1, 34), quality=80),
             J.encode(J.smooth_image(130, 170, 3, 35), quality=95, subsampling=2)]
    for mode in ("bgr", "gray"):
        rows, st = eng.ingest_jpegs(blobs, (64, 64), mode)
        assert (st == 0).all()
        for i, b in enumerate(blobs):
            np.testing.assert_array_equal(rows[i], io_oracle.preprocess(J.decode_ref(b, mode), (64, 64)),
                                          err_msg=f"{mode} file {i}")
