"""The C ABI with no Python in the calling process (include/eigenface.h is the drop-in
boundary; INTEGRATION.md shows the cgo / JNI / N-API bindings that would call it the same
way): tests/native/c_pipeline.c fits, projects and recognises through libeigenface.so and
checks every result against double-precision arithmetic of its own."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "face-detection-recognization-pca_amd", "eigenface", "_lib")

pytestmark = pytest.mark.gpu


def test_c_caller_fit_project_recognise(tmp_path):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = tmp_path / "c_pipeline"
    subprocess.run([cc, "-O2", "-std=c11", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "c_pipeline.c"), "-o", str(exe),
                    "-L", LIBDIR, "-leigenface", f"-Wl,-rpath,{LIBDIR}", "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr
    assert "C_PIPELINE_OK" in r.stdout
    assert "300/300 identities equal the double brute force" in r.stdout
