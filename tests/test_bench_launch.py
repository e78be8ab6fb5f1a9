"""bench.py's multi-rank launch path on the CPU (--dry-run: gloo process groups, no HIP).

`bench.py --gpus N` outside a launcher must start N ranks itself (torch.distributed.run as a
child process) and report n_gpus = N; under a launcher whose WORLD_SIZE differs from --gpus it
must refuse (exit 2) instead of printing a line with the wrong n_gpus.  At N = 1 the per-step
collective runs too (world-1 process group), so 1 -> N efficiency compares equal work.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout, cwd="/tmp")


def _line(out):
    lines = [ln for ln in out.strip().splitlines() if ln.strip()]
    # stdout is exactly one JSON line (rank 0's); library banners (RCCL's version lines at
    # communicator creation) and logs go to stderr
    assert len(lines) == 1 and lines[0].startswith("{"), out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_dry_run_reports_the_ranks_it_ran(n):
    r = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1", "--prewarm-ms", "20"],
             _env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == n and d["dry_run"] is True
    assert d["config"]["parallelism"] == f"dp{n}"
    assert d["config"]["global_batch"] == n * d["config"]["batch_per_gpu"]
    assert d["steps"] == 3 and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["cpu_baseline"] is None and d["scaling"] == "weak"


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "1", "--dry-run", "--steps", "1"],
             _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0", "--dry-run"], _env(), timeout=120)
    assert r.returncode == 2


def test_prewarm_runs_the_same_collectives_on_every_rank():
    """The pre-warm runs for a wall-clock budget with the per-step collective inside: ranks of
    different speed must still run the same number of steps (round 6: a per-rank time loop ran
    different numbers of all-gathers: a hang at N = 2 was seen once under gloo, and RCCL
    hangs on it).  Rank 1 starts its budget 40 ms later; the line reports every rank's count."""
    r = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--prewarm-ms", "60"],
             _env(BENCH_DRY_SKEW_MS="40"), timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    assert len(d["prewarm_steps"]) == 2 and d["prewarm_steps"][0] == d["prewarm_steps"][1] > 0
