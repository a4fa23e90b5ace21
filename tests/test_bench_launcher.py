"""CPU (gloo): `bench.py --gpus N` run directly starts its N ranks itself
(launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set before anything
touches a GPU); the ranks form a process group, time is max-reduced and
bit-exactness min-reduced, and only rank 0 prints the one JSON line.  The
GPU work itself is replaced by the --launcher-selftest stub."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_spawns_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launcher-selftest"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["selftest"] is True
    assert out["max_elapsed"] == 2.0  # rank 1 reported 2.0, rank 0 1.0: the max over ranks
    assert out["bit_exact"] is True
