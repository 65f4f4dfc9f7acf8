"""bench.py launch contract on the CPU host (gloo): ``--gpus N`` starts N rank
processes itself and the rendezvous sees exactly N ranks; a launcher / flag
mismatch or too few devices fail loudly instead of measuring fewer GPUs."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                          text=True, timeout=timeout, cwd="/tmp")


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--check-launch"], {"TCA_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout  # only rank 0 prints
    d = json.loads(line[0])
    assert d == {"check_launch": True, "world": n, "ranks_seen": n, "self_launched": True}


def test_launcher_world_mismatch_fails():
    r = _run(["--gpus", "3", "--check-launch"], {"WORLD_SIZE": "2", "TCA_DIST_BACKEND": "gloo"})
    assert r.returncode != 0 and "wrong GPU count" in r.stderr


def test_too_few_devices_fails():
    # no GPU on this host: --gpus 2 must refuse instead of measuring on fewer devices
    r = _run(["--gpus", "2", "--check-launch"])
    assert r.returncode != 0 and "GPU(s) are visible" in r.stderr


def test_single_rank_check():
    r = _run(["--check-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["world"] == 1
