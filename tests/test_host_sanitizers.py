"""Host sanitizer build of the C ABI (host ASan/UBSan builds of the C-ABI shim).

`make -C face-detection-recognization-pca_amd asan` compiles every source with
AddressSanitizer + UndefinedBehaviorSanitizer on the host code and links
tests/native/host_fuzz.cpp, which fuzzes the entry points that run without a GPU: the
JPEG marker parser behind every batched decode (ef_jpeg_info: seed files from Pillow plus
deterministic mutations — bit flips, marker injection, length tampering, truncation,
splices — one file per call and a batch call), the host merge of match records and the
key decoder.  Any sanitizer report aborts the process."""
import os
import subprocess

import pytest

import jpeg_cases as J

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "face-detection-recognization-pca_amd")
BIN = os.path.join(PKG, "build_asan", "host_fuzz")


def test_host_fuzz_under_asan_ubsan(tmp_path):
    jobs = str(min(8, os.cpu_count() or 4))
    r = subprocess.run(["make", "-C", PKG, "-j", jobs, "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("asan build failed:\n" + r.stdout[-2000:] + r.stderr[-2000:])
    seeds = []
    for i, (name, blob) in enumerate(J.corpus()):
        if i % 4:
            continue
        p = tmp_path / f"seed{i}.jpg"
        p.write_bytes(blob)
        seeds.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([BIN, "6000"] + seeds, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "clean" in r.stdout
