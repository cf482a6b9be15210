"""bench.py's multi-rank launcher on CPU: `python bench.py --gpus 2` started directly (no WORLD_SIZE) must run two
ranks through torch.distributed.run as a child process, and every rank must see a world of 2 (gloo here; the
GPU box uses the same path with RCCL)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *extra], capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


@pytest.mark.timeout(300)
def test_gpus2_launches_two_ranks():
    r = _run("--gpus", "2", "--launch-check")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout          # ONE JSON line, from rank 0
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2 and lines[0]["backend"] == "gloo"
    # every sub-line of the default run (configs[2] - [4], re-simulation) runs on both ranks at world 2
    from bench import SUBLINES
    sub = lines[0]["secondary"]
    assert list(sub) == [wl for wl, _ in SUBLINES]
    for wl, res in sub.items():
        assert "error" not in res, (wl, res)
        assert res["ranks_seen"] == 2 and res["n_gpus"] == 2, (wl, res)


@pytest.mark.timeout(120)
def test_gpus_disagreeing_with_world_size_fails():
    r = _run("--gpus", "2", "--launch-check", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
