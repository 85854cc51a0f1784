"""CPU: `bench.py --gpus N` started without a torch.distributed launcher starts the N rank
processes itself (a torch.distributed.run child, 127.0.0.1 rendezvous), and the rank-0 line
reports N ranks joined; the launch probe checks it with gloo and never touches a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    env["GSR_DIST_BACKEND"] = "gloo"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_and_joins_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints, the launcher relays it once
    assert lines[0]["n_gpus"] == n and lines[0]["ranks_joined"] == n
    assert lines[0]["backend"] == "gloo"


def test_gpus_must_match_world_size():
    """Under an outer launcher, a --gpus that disagrees with WORLD_SIZE is an error."""
    r = _run(["--gpus", "2", "--launch-probe"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stderr + r.stdout)


def test_single_rank_probe():
    r = _run(["--launch-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["n_gpus"] == 1 and line["ranks_joined"] == 1
