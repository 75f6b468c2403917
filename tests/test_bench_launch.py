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


def test_phase_sequence_completes():
    """Every rank walks the distributed bench's phases (mlamg.distributed.DIST_PHASES) under the
    watchdog and marks each on stderr, rank-tagged."""
    r = _run(["--gpus", "2", "--phase-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["phase_selftest"] and out["phases"][0] == "init"
    for rank in (0, 1):
        for ph in out["phases"]:
            assert f"[mlamg rank {rank}/2] phase {ph} " in r.stderr, (rank, ph)
        assert f"[mlamg rank {rank}/2] done" in r.stderr


@pytest.mark.parametrize("phase", ("uid_broadcast", "warmup"))
def test_stalled_rank_exits_nonzero_naming_its_phase(phase):
    """VERDICT r04 Next #2: a rank that hangs (test hook MLAMG_SELFTEST_STALL=1:<phase>) is
    ended by its watchdog when the phase overruns its budget: it prints the phase it was in and
    exits non-zero (EXIT_DIST_TIMEOUT); the launcher then stops the other rank, which is waiting
    in the next phase's barrier (a phase with twice the budget, so the stalled rank's watchdog
    fires first). Nothing re-executes or restarts."""
    r = _run(["--gpus", "2", "--phase-selftest"],
             env_extra={"MLAMG_SELFTEST_STALL": f"1:{phase}",
                        "MLAMG_PHASE_TIMEOUT_SCALE": "0.01", "MLAMG_DIST_TIMEOUT_S": "60"})
    assert r.returncode == 5, (r.returncode, r.stderr[-3000:])
    assert f"[mlamg rank 1/2] FAILED in phase {phase}" in r.stderr, r.stderr[-3000:]
    assert "exceeded its budget" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_gloo_timeout_names_the_waiting_phase():
    """The peer side: with the watchdog budgets long, the rank waiting for a stalled peer hits
    the gloo collective timeout (MLAMG_DIST_TIMEOUT_S) in the next phase's barrier and exits
    non-zero naming that phase; the launcher's SIGTERM then makes the stalled rank dump its
    threads' stacks (faulthandler) before it dies — its last marker names the phase it hung in."""
    r = _run(["--gpus", "2", "--phase-selftest"],
             env_extra={"MLAMG_SELFTEST_STALL": "1:timed", "MLAMG_DIST_TIMEOUT_S": "5"})
    assert r.returncode == 6, (r.returncode, r.stderr[-3000:])
    assert "[mlamg rank 0/2] FAILED in phase roofline" in r.stderr, r.stderr[-3000:]
    assert "[mlamg rank 1/2] test hook: stalling in phase timed" in r.stderr
    assert "selftest_stall_point" in r.stderr  # rank 1's stack dump on SIGTERM
