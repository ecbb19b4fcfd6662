"""bench.py's N > 1 path end to end: the script launches its own rank
processes (no torchrun), the ranks shard the gallery, project their slices of the probe
batch, exchange features and fp64 match records and merge; rank 0 prints the JSON line
with the max-over-ranks step time.  The box has one GPU, so the two ranks share it and
exchange through gloo (RCCL needs one GPU per rank) — the same code path as the nccl run
apart from the collective's transport."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(args, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    return r


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("metric", ["l2", "cosine"])
def test_bench_two_ranks_one_gpu(metric):
    r = _run(["--gpus", "2", "--backend", "gloo", "--gallery", "200000", "--metric", metric, "--no-cpu",
              "--no-fit", "--no-image", "--no-c2", "--no-split", "--steps", "3", "--warmup", "1", "--repeats", "2",
              "--launch-timeout", "240"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2
    assert rec["check"]["planted_match"] == 1.0
    assert rec["check"]["ranks_agree"] is True
    assert rec["config"]["rows_per_rank"] == 100_000
    assert rec["steps"] == 3 and len(rec["repeats_ms_per_step"]) == 2
    assert rec["value"] > 0 and rec["cpu_baseline"] is None
    # the collectives alone (gloo through the host here: an upper bound of RCCL's share)
    assert rec["exchange_ms_per_step"] > 0 and 0 < rec["exchange_share_of_step"]
    # the north star's single all-reduce(MIN) on the same step: same keys on this data
    om = rec["other_merge"]
    assert om["merge"] == "min" and om["keys_identical"] is True and om["ms_per_step"] > 0
    assert om["exchange_ms_per_step"] > 0
    print(f"2 ranks / one GPU, gloo: step {rec['ms_per_step']} ms, exchange {rec['exchange_ms_per_step']} ms "
          f"({100 * rec['exchange_share_of_step']:.1f} %); merge=min: step {om['ms_per_step']} ms, "
          f"exchange {om['exchange_ms_per_step']} ms")


@pytest.mark.parametrize("ranks,gallery", [(4, 200_000), (3, 200_003)])
def test_bench_more_ranks_one_gpu(ranks, gallery):
    """Rehearsal of the driver's N = 4 run (and an uneven 3-way split: shards of 66667 /
    66668 rows, the probe slices 1366 / 1365) on the one card: every rank's keys agree and
    every planted probe finds its row across the shard boundaries."""
    r = _run(["--gpus", str(ranks), "--backend", "gloo", "--gallery", str(gallery), "--no-cpu", "--no-fit",
              "--no-image", "--no-c2", "--no-split", "--steps", "2", "--warmup", "1", "--repeats", "1",
              "--launch-timeout", "240"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == ranks
    assert rec["check"]["planted_match"] == 1.0
    assert rec["check"]["ranks_agree"] is True
    assert rec["config"]["rows_per_rank"] in (gallery // ranks, -(-gallery // ranks))


def test_bench_rejects_gpus_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "disagrees with WORLD_SIZE" in r.stderr


def test_bench_nccl_refuses_shared_gpu():
    """--backend nccl with more ranks than GPUs: every rank refuses and the launcher exits
    non-zero instead of hanging in RCCL init."""
    import torch
    n = torch.cuda.device_count()
    r = _run(["--gpus", str(n + 1), "--backend", "nccl", "--gallery", "10000", "--no-cpu", "--no-fit", "--no-image",
              "--no-c2", "--no-split", "--steps", "1", "--launch-timeout", "120"], timeout=180)
    assert r.returncode != 0
    assert "only" in r.stderr and "GPU(s) are visible" in r.stderr
