"""CPU: `python bench.py --gpus N` launches N ranks by itself (one process per GPU, the
environment torch.distributed.run would give them) when no launcher set WORLD_SIZE, and the
ranks rendezvous (gloo, no GPU work: --launch-selftest)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("n", (2, 3))
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-selftest"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    ranks = out["ranks"]
    assert [d["rank"] for d in ranks] == list(range(n))
    assert [d["local_rank"] for d in ranks] == list(range(n))
    assert {d["world"] for d in ranks} == {n}
    assert len({d["pid"] for d in ranks}) == n  # one process per rank
    assert len({d["master"] for d in ranks}) == 1 and ranks[0]["master"].startswith("127.0.0.1:")


def test_gpus_1_runs_in_process():
    r = _run(["--gpus", "1", "--launch-selftest"])
    assert r.returncode == 0, r.stderr
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["ranks"][0]["pid"] > 0


def test_launcher_world_size_must_match():
    """Under a launcher (WORLD_SIZE set) a different --gpus is an error, not a silent N=1 line."""
    r = _run(["--gpus", "4", "--launch-selftest"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus=4" in r.stderr


@pytest.mark.parametrize("n", (2, 3))
def test_distributed_mismatch_is_refused(n):
    """A distributed iterate that differs from the single-GPU one on every executor path
    (mismatch injected on rank 1 through the real verification chain,
    mlamg.distributed.verify_paths) ends the run non-zero with no value line."""
    r = _run(["--gpus", str(n), "--verify-selftest"],
             env_extra={"MLAMG_INJECT_MISMATCH_RANK": "1"})
    assert r.returncode == 4, (r.returncode, r.stderr[-2000:])
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "REFUSED" in r.stderr


def test_distributed_verification_passes_without_mismatch():
    r = _run(["--gpus", "2", "--verify-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["verify_selftest"] and out["cycle_graph"] and out["overlap"]


def test_failing_rank_fails_the_launch():
    """A rank that dies makes the launcher stop the others and exit with its status (rank 0
    would otherwise wait in the rendezvous)."""
    r = _run(["--gpus", "3", "--launch-selftest"], env_extra={"MLAMG_SELFTEST_FAIL_RANK": "1"})
    assert r.returncode == 3
