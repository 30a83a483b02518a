"""bench.py as the driver runs it for the scaling curve: `python bench.py --gpus N` (no torchrun
environment) launches N rank processes itself and relays rank 0's one JSON line; a torchrun world
that disagrees with --gpus is refused with a dp_error line.  Exercised on the host path
(`--device cpu`: gloo, eager, tiny batch) — the same launcher, rendezvous, max-over-ranks timing
and data-parallel wrapper as the GPU run, without a GPU (reference step: torch/train.py:85-100)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=280):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "2"
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd="/tmp")
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    return p.returncode, lines, p.stderr


SMALL = ["--device", "cpu", "--batch", "2", "--steps", "2", "--warmup", "1"]


@pytest.mark.timeout(300)
def test_launcher_spawns_ranks_and_relays_one_line():
    rc, lines, err = _run(["--gpus", "2"] + SMALL)
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    assert len(d["ms_per_step_per_rank"]) == 2 and all(v > 0 for v in d["ms_per_step_per_rank"])
    # the job's time is the slowest rank's
    assert d["ms_per_step"] == pytest.approx(max(d["ms_per_step_per_rank"]))
    assert d["value"] == pytest.approx(4 * 2 / (d["ms_per_step"] * 2 / 1e3), rel=1e-6)
    assert "overlapped buckets" in d["dp"]
    assert "launching 2 ranks" in err


@pytest.mark.timeout(300)
def test_launcher_single_allreduce_mode():
    rc, lines, err = _run(["--gpus", "2", "--dp-overlap", "0"] + SMALL)
    assert rc == 0, err[-3000:]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and "one post-backward all-reduce" in d["dp"]


@pytest.mark.timeout(300)
def test_one_gpu_runs_in_process():
    rc, lines, err = _run(["--gpus", "1"] + SMALL)
    assert rc == 0, err[-3000:]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["dp"] is None and d["config"]["parallelism"] == "dp1"
    assert "launching" not in err


@pytest.mark.timeout(120)
def test_world_size_mismatch_is_refused():
    rc, lines, _ = _run(["--gpus", "1"] + SMALL, {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] is None and "WORLD_SIZE=2" in d["dp_error"]
