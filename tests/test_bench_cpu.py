"""bench.py's launcher logic without a GPU: --gpus must agree with a torchrun WORLD_SIZE,
and the self-launch (WORLD_SIZE unset, --gpus N > 1) starts N rank processes with the
torchrun environment and propagates a failing rank's exit code."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_must_match_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "disagrees with WORLD_SIZE=2" in r.stderr


def test_gpus_must_be_positive():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "0"], capture_output=True, text=True, timeout=120,
                       env=_env())
    assert r.returncode == 2


def test_self_launch_sets_rank_env_and_propagates_failure():
    """Here every rank finds no GPU and exits 2: the parent must report it (not 0), and
    each rank must have seen its own RANK / LOCAL_RANK and the common WORLD_SIZE."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-timeout", "200"], capture_output=True,
                       text=True, timeout=300, env=_env())
    assert r.returncode == 2, r.stderr[-2000:]
    assert "no GPU visible" in r.stderr


def test_launch_ranks_passes_environment(tmp_path, monkeypatch):
    """launch_ranks itself: the children get the torchrun contract variables."""
    sys.path.insert(0, ROOT)
    import importlib
    bench = importlib.import_module("bench")
    script = tmp_path / "child.py"
    script.write_text("import os, sys\n"
                      "out = os.path.join(%r, 'r' + os.environ['RANK'])\n"
                      "open(out, 'w').write(' '.join(os.environ[k] for k in "
                      "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')))\n"
                      "sys.exit(0 if os.environ['RANK'] != '1' else 5)\n" % str(tmp_path))
    monkeypatch.setattr(bench, "__file__", str(script))
    rc = bench.launch_ranks(3, [], timeout_s=60)
    assert rc == 5
    port = None
    for r in range(3):
        f = tmp_path / f"r{r}"
        if not f.exists():  # rank 1 failing may stop a later rank before it writes
            continue
        rank, local, world, addr, p = f.read_text().split()
        assert (rank, local, world, addr) == (str(r), str(r), "3", "127.0.0.1")
        assert port in (None, p)
        port = p


def test_tmatch_executed_work_model():
    """bench.tmatch_executed_ops: whole output row bands (128 rows; 32 / 64 for a last row
    band with one / two live 32-row blocks — the 32 x 512 / 64 x 256 tiles), the map's
    columns rounded up to whole 32-column blocks (a wave runs only its live column blocks),
    band columns rounded up to 32-column k-blocks (DESIGN K11)."""
    sys.path.insert(0, ROOT)
    import importlib
    bench = importlib.import_module("bench")
    # output exactly one tile (128 x 128), template 40 x 33: band 33 + 31 = 64 columns
    H, W, h, w = 127 + 40, 127 + 33, 40, 33
    ex = bench.tmatch_executed_ops([(0, h, w)], H, W)
    assert ex == 2.0 * 128 * 128 * h * 64
    # one more output column opens a second tile column with one live 32-column block
    assert bench.tmatch_executed_ops([(0, h, w)], H, W + 1) == 2.0 * 128 * 160 * h * 64
    # one live output row across 417 columns: one 32 x 512 tile, 14 live column blocks
    assert bench.tmatch_executed_ops([(0, h, w)], h, w + 416) == 2.0 * 32 * 448 * h * 64
    # 168 rows x 256 columns: a full 128-row band, then 40 rows = two live row blocks in
    # one 64 x 256 tile
    assert bench.tmatch_executed_ops([(0, h, w)], 167 + h, 255 + w) == 2.0 * (128 * 256 + 64 * 256) * h * 64
    # 160 rows x 256 columns: the last band has one live row block, a 32 x 512 tile with
    # 8 live column blocks
    assert bench.tmatch_executed_ops([(0, h, w)], 159 + h, 255 + w) == 2.0 * (128 * 256 + 32 * 256) * h * 64
    # 200 rows: the last band has three live row blocks, a whole 128 x 128 tile row
    assert bench.tmatch_executed_ops([(0, h, w)], 199 + h, 255 + w) == 2.0 * (128 * 256 + 128 * 256) * h * 64


def test_ingest_touched_bytes_model():
    """bench.ingest_touched_bytes: the copy path touches every line of the crop; a 4x
    downscale only the lines of its sampled rows (2 per output row)."""
    sys.path.insert(0, ROOT)
    import importlib
    bench = importlib.import_module("bench")
    # 64 x 64 grey copy at a line-aligned offset: every byte, 32 lines + the output
    assert bench.ingest_touched_bytes([0], [64], [64], [1]) == 64 * 64 + 64 * 64
    # 256 x 256 grey -> 64 x 64: 128 distinct source rows of 256 B (2 lines each)
    rows = np.unique(np.concatenate(bench._lin_src(64, 256)))
    assert rows.size == 128
    assert bench.ingest_touched_bytes([0], [256], [256], [1]) == 128 * 256 + 64 * 64
