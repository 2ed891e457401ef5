"""bench.py's N > 1 entry point as the driver runs it (`python bench.py --gpus N`, no torchrun):
bench.py starts the N ranks itself (torch.distributed.run as a child process) and rank 0 prints
exactly one JSON line.  On CPU the ranks run the ``--cpu-plumbing`` path (gloo, the ids all-gather
through adaptive_amd.distributed.gather_rows, max-over-ranks timing, the rank topology and the
neighbour-shard cross-check) -- no GPU, no decode.  N = 8 is the node the driver's scaling run uses."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_spawns_its_own_ranks(n):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--cpu-plumbing",
                        "--batch", "8", "--max-len", "5"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks_seen"] == n and d["backend"] == "gloo"
    assert d["gathered_ok"] is True
    assert len(d["regions_s"]) >= 5
    # what the GPU line carries for N > 1 too: every rank listed once, and every rank's re-decode of its
    # neighbour's shard equal to the gathered rows (AND over the ranks)
    ranks = d["rank_devices"]["ranks"]
    assert sorted(r["rank"] for r in ranks) == list(range(n))
    assert sorted(r["local_rank"] for r in ranks) == list(range(n))
    assert d["cross_check"]["ok"] is True


def test_bench_refuses_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-plumbing"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
