"""bench.py's `--gpus N` launcher on CPU: a plain `python bench.py --gpus 2` must start two
ranks itself (torch.distributed.run, one process per rank, the reference's launcher
scripts/script_train.sh:33), and rank 0 must report `n_gpus: 2` after both ranks ran the
barrier-bracketed timed region. `--selftest` swaps the GPU step for a stub CPU step on gloo."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--selftest", *args],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_two_ranks_launched_by_bench():
    r = _run("--gpus", "2", "--steps", "3", "--warmup", "1")
    assert r["n_gpus"] == 2
    assert r["ranks_seen"] == 2
    assert r["steps"] == 3 and r["warmup"] == 1


def test_single_rank_stays_in_process():
    r = _run("--gpus", "1", "--steps", "2", "--warmup", "0")
    assert r["n_gpus"] == 1 and r["ranks_seen"] == 1


@pytest.mark.parametrize("mode", ["--sweep", "--train"])
def test_modes_parse_through_the_launcher(mode):
    # the sweep / training modes take the same launcher path (the stub step replaces them)
    r = _run("--gpus", "2", mode, "--steps", "1", "--warmup", "0")
    assert r["n_gpus"] == 2 and r["ranks_seen"] == 2
