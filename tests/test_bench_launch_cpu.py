"""CPU: `python bench.py --gpus N` starts N ranks itself (no external launcher) and refuses a
WORLD_SIZE that disagrees with --gpus.  The ranks join a gloo group and never touch a GPU
(--launch-check); the same launch path starts the measured ranks on a GPU node."""
import json
import os
import subprocess
import sys

from conftest import REPO


def _run(args, extra_env=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update({"DRT_BENCH_BACKEND": "gloo", "OMP_NUM_THREADS": "1"}, **(extra_env or {}))
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks_joined"] == 2, rec


def test_bench_world_size_mismatch_refused():
    r = _run(["--gpus", "4", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, (r.returncode, r.stderr[-2000:])


def test_bench_gpus1_runs_in_process():
    r = _run(["--gpus", "1", "--launch-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
