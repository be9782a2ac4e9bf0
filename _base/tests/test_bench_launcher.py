"""bench.py's own N-rank launch on CPU: `--gpus N` without a
launcher starts N ranks, they rendezvous over gloo, gather one packed
trajectory buffer per episode and rank 0 prints one JSON line with the
per-rank values (the GPU leg is stubbed with --stub)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=240, env=e)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_launcher_yields_n_ranks_gloo():
    r = _bench(["--gpus", "3", "--stub", "--steps", "40", "--warmup", "0", "--colloids", "128"])
    assert r.returncode == 0, r.stderr
    line = _line(r.stdout)
    assert line["n_gpus"] == 3 and line["world"] == 3
    assert len(line["per_rank_value"]) == 3
    assert line["value"] > 0
    # 20-slice episodes of 128 agents: features 12 B + action 8 + logp 4 + reward 4,
    # plus the one-byte kill flag
    assert line["gather"]["bytes_per_rank"] == 20 * 128 * 28 + 1
    assert line["gather"]["per_run"] == 2


def test_launcher_rejects_world_mismatch():
    r = _bench(["--gpus", "1", "--stub"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr
