"""CPU: bench.py starts its own ranks for --gpus N (the driver's multi-GPU run invokes the script
directly, without a launcher).  --dry-run stops every rank right after the gloo group forms, before
any GPU work, so the launch logic runs here."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    return r, lines


def test_gpus2_spawns_two_gloo_ranks():
    r, lines = _run("--gpus", "2", "--dry-run")
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout: the relay keeps the channel clean
    d = json.loads(lines[0])
    assert d["dry_run"] and d["n_gpus"] == 2 and d["world_size"] == 2
    assert sorted(x["rank"] for x in d["ranks"]) == [0, 1]
    assert all(x["world_size"] == 2 for x in d["ranks"])


def test_gpus1_runs_in_process():
    r, lines = _run("--gpus", "1", "--dry-run")
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(lines[-1])
    assert d["world_size"] == 1 and d["ranks"] == [{"rank": 0, "world_size": 1}]
    assert "torch.distributed.run" not in r.stderr


def test_failing_rank_fails_the_launch():
    """A rank that exits non-zero (here: an unknown flag, so argparse exits 2 in every rank) makes the
    parent exit non-zero -- never a silent success."""
    r, lines = _run("--gpus", "2", "--dry-run", "--no-such-flag")
    assert r.returncode != 0
