"""bench.py's own rank launcher, on CPU: `--gpus N`
without torch.distributed.run starts N rank processes itself; with
--launch-dry-run each rank reports its environment without touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env=None, timeout=120):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=e)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_launch_dry_run_ranks(n):
    p = run(["--gpus", str(n), "--launch-dry-run"])
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert sorted(int(x["RANK"]) for x in lines) == list(range(n))
    assert all(x["LOCAL_RANK"] == x["RANK"] for x in lines)
    assert {x["WORLD_SIZE"] for x in lines} == {str(n)}
    assert {x["MASTER_ADDR"] for x in lines} == {"127.0.0.1"}
    assert len({x["MASTER_PORT"] for x in lines}) == 1
    assert all(x["RT_BENCH_LAUNCHED"] == "1" for x in lines)


def test_launch_rank_failure_propagates():
    p = run(["--gpus", "4", "--launch-dry-run"], env={"RT_BENCH_DRY_FAIL": "2:5"})
    assert p.returncode == 5
    assert "rank 2 exited 5" in p.stderr


def test_launch_fails_fast_without_gpus():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has GPUs")
    p = run(["--gpus", "2", "--steps", "3"], timeout=60)
    assert p.returncode == 2
    assert "GPU(s) visible" in p.stderr
