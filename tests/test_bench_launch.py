"""bench.py's rank launch (no GPU needed): `--gpus N` without a launcher starts N ranks itself
(RANK / LOCAL_RANK / WORLD_SIZE / 127.0.0.1 rendezvous), and under a launcher it refuses a
WORLD_SIZE that differs from --gpus. Both checks run before any GPU call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=120)


def test_gpus_n_plans_n_ranks():
    r = _run(["--gpus", "4", "--config", "c4", "--print-launch"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert [d["RANK"] for d in plan["ranks"]] == ["0", "1", "2", "3"]
    assert [d["LOCAL_RANK"] for d in plan["ranks"]] == ["0", "1", "2", "3"]
    assert {d["WORLD_SIZE"] for d in plan["ranks"]} == {"4"}
    assert {d["MASTER_ADDR"] for d in plan["ranks"]} == {"127.0.0.1"}
    assert len({d["MASTER_PORT"] for d in plan["ranks"]}) == 1
    # the children run this script with the same arguments (minus the test hook)
    assert plan["cmd"][1:] == [BENCH, "--gpus", "4", "--config", "c4"]


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_gpus_zero_is_refused():
    r = _run(["--gpus", "0"])
    assert r.returncode == 2
