"""CPU-side checks of the C-ABI library: it loads, exports every entry point that
include/eigenface.h declares, and its host-only helpers behave (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "eigenface.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ef_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_api():
    names = _declared()
    for n in ("ef_create", "ef_destroy", "ef_fit", "ef_model_set", "ef_project", "ef_gallery_set",
              "ef_search", "ef_recognize", "ef_keys_decode", "ef_timing_get"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from eigenface import _native
    lib = _native.lib()
    for n in _declared():
        assert hasattr(lib, n), n
    assert set(_native.EXPORTED_SYMBOLS) == set(_declared())
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    for n in _declared():
        assert re.search(rf"\bT {n}$", out, re.M), n


def test_library_is_gfx950_code_object():
    from eigenface import _native
    data = open(_native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle target id


def test_one_hip_runtime_per_process():
    """Opening libeigenface before anything imported torch must not map a second HIP
    runtime when torch comes in later (two runtimes: the one that initialises second
    sees no GPU — the drop-in trainers' subprocess failure on the box)."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from eigenface import _native; _native.lib()\n"
            "import torch\n"
            "maps = open('/proc/self/maps').read().split('\\n')\n"
            "paths = {l.split()[-1] for l in maps if 'libamdhip64' in l}\n"
            "print(len(paths), sorted(paths))\n") % os.path.join(ROOT, "face-detection-recognization-pca_amd")
    r = subprocess.run([__import__("sys").executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("1 "), r.stdout


def test_api_version_and_no_device_here():
    from eigenface import _native
    lib = _native.lib()
    assert lib.ef_api_version() == 7
    n = ctypes.c_int(-1)
    assert lib.ef_device_count(ctypes.byref(n)) == 0
    if n.value == 0:  # build container: creating a context must fail cleanly, not crash
        h = ctypes.c_void_p()
        assert lib.ef_create(0, ctypes.byref(h)) != 0
        from eigenface import Engine, EigenfaceError
        with pytest.raises(EigenfaceError):
            Engine(0)


def test_key_decode_roundtrip_order_and_ties():
    """Packed keys: high 32 bits order-preserving score, low 32 bits index."""
    from eigenface import decode_keys

    def pack(v, i):
        b = np.float32(v).view(np.int32).item()
        if v == 0:
            b = 0
        s = b if b >= 0 else b ^ 0x7FFFFFFF
        return (s << 32) | i

    vals = [-3.5, -1e-30, 0.0, 1e-30, 2.0, 7.25, np.inf]
    keys = np.array([pack(v, 10 + j) for j, v in enumerate(vals)], dtype=np.int64)
    assert np.all(np.diff(keys) > 0)  # signed int64 order == score order
    idx, best = decode_keys(keys, "l2")
    np.testing.assert_array_equal(idx, 10 + np.arange(len(vals)))
    np.testing.assert_array_equal(best, np.array(vals, np.float32))
    # equal scores: lower index is the smaller key (np.argmin tie-break)
    assert pack(1.5, 3) < pack(1.5, 4)
    # cosine keys hold -similarity
    idx, sim = decode_keys(np.array([pack(-0.75, 2)], np.int64), "cosine")
    assert idx[0] == 2 and sim[0] == np.float32(0.75)
    idx, best = decode_keys(np.array([(1 << 63) - 1], np.int64), "l2")
    assert idx[0] == -1 and np.isnan(best[0])


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    from eigenface import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(_native.NativeLibraryError):
        _native.lib()


def test_product_package_does_not_import_oracle():
    pkg = os.path.join(ROOT, "face-detection-recognization-pca_amd", "eigenface")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            assert "oracle" not in open(os.path.join(pkg, f)).read().replace("no oracle", ""), f


def test_product_library_reads_no_environment_knobs():
    """Experiment knobs and ablations live in the diagnostic build (make diag,
    -DEF_DIAGNOSTICS) only: the product library never calls getenv, so no environment
    variable can change its numerics or kernel choice."""
    from eigenface import _native
    out = subprocess.run(["nm", "-D", "--undefined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    assert not re.search(r"\bgetenv\b", out)


def test_host_match_merge_is_exact():
    """ef_matches_merge on the host (no GPU): fp64 scores decide across parts even when
    their fp32 keys tie; exact ties and near-ties within 1e-12 go to the lowest index;
    empty parts are ignored; all-empty gives EF_KEY_NONE."""
    from eigenface import _native as N, decode_keys, merge_matches_host
    from eigenface.distributed import pack_keys

    b = 5
    inf = np.inf
    none = N.EF_KEY_NONE
    # part 0 rows 0..99, part 1 rows 100..199
    s0 = np.array([1.0, 2.0, 3.0, inf, 5.0])
    s1 = np.array([1.0 - 1e-9, 2.0, 3.0 + 1e-13, inf, 4.0])
    i0 = np.array([7, 8, 9, 0, 11])
    i1 = np.array([107, 5, 109, 0, 111])
    recs = np.zeros(2 * b, dtype=N.MATCH_DTYPE)
    for r, (s, i) in enumerate([(s0, i0), (s1, i1)]):
        recs["score"][r * b:(r + 1) * b] = s
        recs["scale"][r * b:(r + 1) * b] = 1.0
        keys = pack_keys(np.where(np.isinf(s), 0, s).astype(np.float32), i)
        keys[np.isinf(s)] = none
        recs["key"][r * b:(r + 1) * b] = keys
    # fp32 keys of probe 0 tie (1 - 1e-9 rounds to 1.0f): the key MIN would pick row 7
    assert np.float32(1.0 - 1e-9) == np.float32(1.0)
    out = merge_matches_host(recs, b)
    idx, best = decode_keys(out, "l2")
    np.testing.assert_array_equal(idx, [107, 5, 9, -1, 111])
    assert best[4] == np.float32(4.0)
    assert out[3] == none


def _hostless_engine(model_d=None, model_k=None, gallery_k=None):
    """An Engine whose context was never created (no GPU here): the input checks run
    before any C call, so a call that reaches the library would fail on the NULL ctx."""
    from eigenface import Engine
    e = object.__new__(Engine)
    from eigenface import _native
    e._lib = _native.lib()
    e._h = ctypes.c_void_p()
    e.model_d, e.model_k, e.gallery_k, e.gallery_n = model_d, model_k, gallery_k, 0
    return e


def test_match_record_api_checks_shapes_before_the_c_call():
    """search_matches / recognize_matches on host arrays: the C side reads b x k (or
    b x d) elements from the pointer, so a narrower or 1-D input must raise first."""
    e = _hostless_engine()
    with pytest.raises(RuntimeError):
        e.search_matches(np.zeros((4, 8), np.float32))
    e = _hostless_engine(gallery_k=8)
    with pytest.raises(RuntimeError):
        e.recognize_matches(np.zeros((4, 16), np.uint8))
    e = _hostless_engine(model_d=16, model_k=8, gallery_k=8)
    for bad in (np.zeros((4, 7), np.float32), np.zeros(8, np.float32), np.zeros((2, 4, 8), np.float32)):
        with pytest.raises(ValueError):
            e.search_matches(bad)
    for bad in (np.zeros((4, 15), np.uint8), np.zeros(16, np.uint8), np.zeros((4, 8), np.float32)):
        with pytest.raises(ValueError):
            e.recognize_matches(bad)


def test_host_merge_checks_record_shapes():
    from eigenface import _native as N, merge_matches_host
    recs = np.zeros(6, dtype=N.MATCH_DTYPE)
    with pytest.raises(ValueError):
        merge_matches_host(recs, 4)  # 6 records are not a multiple of b = 4
    with pytest.raises(ValueError):
        merge_matches_host(np.zeros((6, 2), np.int64), 3)
    recs["key"] = N.EF_KEY_NONE
    recs["score"] = np.inf
    assert (merge_matches_host(recs, 3) == N.EF_KEY_NONE).all()


def test_search_schedule_plans_each_piece_from_its_launched_rows():
    """every search launch's plan must be built from the row count the
    piece is launched with.  The sharded projection pads its feature block to
    round_up(R * ceil(b / R), 256) rows (b = 4096, R = 3: 4352), more than the
    round_up(b, 256) = 4096 rows the kernels are told about; a plan built from the larger
    count gives a part_key stride the kernels do not use.  ef_search_schedule reports what
    search_local launches (host arithmetic, no GPU)."""
    from eigenface import _native
    lib = _native.lib()
    i32 = ctypes.c_int32

    def sched(b, k, n, split):
        cnt = i32(-1)
        assert lib.ef_search_schedule(b, k, n, split, None, 0, ctypes.byref(cnt)) == 0
        out = np.zeros((max(cnt.value, 1), 6), np.int64)
        assert lib.ef_search_schedule(b, k, n, split, out.ctypes.data, cnt.value, ctypes.byref(cnt)) == 0
        return out[:cnt.value]

    def kp_of(k):
        for p in (16, 32, 64, 128, 256, 512):
            if k <= p:
                return p
        return -(-k // 128) * 128

    for b, k, n, split in [(4096, 128, 1_000_000, 0), (4096, 512, 1_000_000, 3), (4096, 512, 1_000_000, 0),
                           (1, 64, 10, 0), (257, 16, 5000, 1), (8200, 65536, 20_000, 1), (8200, 65536, 20_000, 0),
                           (3000, 601, 7001, 3), (70_000, 1024, 1000, 0), (1366, 128, 333_334, 0)]:
        p = sched(b, k, n, split)
        kp = kp_of(k)
        assert p[0, 0] == 0 and p[:, 1].sum() == b
        np.testing.assert_array_equal(p[1:, 0], np.cumsum(p[:-1, 1]))        # contiguous pieces
        np.testing.assert_array_equal(p[:, 2], -(-p[:, 1] // 256) * 256)      # rows = round_up(b_i, 256)
        assert np.all(p[:, 2] * kp * 4 <= 2**31 - 1) or len(p) == 1 and p[0, 2] == 256
        tile = 256 if kp <= 128 or split else 128                               # probes per workgroup
        np.testing.assert_array_equal(p[:, 3] * tile, p[:, 2])                  # plan == launch
        assert np.all(p[:, 4] % 8 == 0) and np.all(p[:, 4] * p[:, 5] * (64 if kp <= 128 else 128 if not split else 256)
                                                    >= n)
    assert lib.ef_search_schedule(10, 0, 10, 0, None, 0, ctypes.byref(i32())) != 0


def test_tm_integral_width_rule():
    """the wrapping uint32 integral images index bytes as
    uint32(entry) * 4, so ef_tm_prepare must pick int64 sums once a frame has 2^30 or more
    integral entries, (H + 1)(W + 1), as well as for template areas >= 2^18."""
    from eigenface import _native
    lib = _native.lib()
    assert lib.ef_tm_sums_bits(480, 640, 150 * 360) == 32
    assert lib.ef_tm_sums_bits(480, 640, (1 << 18) - 1) == 32
    assert lib.ef_tm_sums_bits(480, 640, 1 << 18) == 64
    # the frame-size edge: 32768 x 32767 entries stay uint32, 32768 x 32768 = 2^30 do not
    assert lib.ef_tm_sums_bits(32767, 32766, 16) == 32   # 32768 * 32767 < 2^30
    assert lib.ef_tm_sums_bits(32767, 32767, 16) == 64   # 32768 * 32768 = 2^30
    assert lib.ef_tm_sums_bits(1 << 20, 1023, 16) == 64  # tall frames too
    assert lib.ef_tm_sums_bits(0, 640, 16) < 0


def test_host_cpu_share_rule(monkeypatch):
    """the library's host workers (JPEG parse / destuff) are sized to the
    job's CPU share — OMP_NUM_THREADS as the GPU pool presets it, else the affinity mask —
    not to the machine's hardware threads (256 on the pool's boxes), capped at 16."""
    from eigenface.engine import host_cpu_share
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert host_cpu_share() == 16
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert host_cpu_share() == 3
    monkeypatch.setenv("OMP_NUM_THREADS", "256")
    assert host_cpu_share() == 16
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert host_cpu_share() == max(1, min(16, len(os.sched_getaffinity(0))))
