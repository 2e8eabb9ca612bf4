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


VIS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def fake_topology(root, gpus, cpus=1):
    """A KFD topology directory: `cpus` CPU nodes (simd_count 0) first, then
    `gpus` GPU nodes, as /sys/class/kfd/kfd/topology/nodes lays them out."""
    os.makedirs(root, exist_ok=True)
    for i in range(cpus + gpus):
        d = os.path.join(root, str(i))
        os.makedirs(d, exist_ok=True)
        simd = 0 if i < cpus else 1024
        with open(os.path.join(d, "properties"), "w") as fp:
            fp.write(f"cpu_cores_count {16 if i < cpus else 0}\nsimd_count {simd}\nmax_waves_per_simd 8\n")
    return str(root)


@pytest.fixture
def topo8(tmp_path):
    return fake_topology(tmp_path / "nodes", 8)


def run(args, env=None, timeout=120):
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT") + VIS}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=e)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_launch_dry_run_ranks(n, topo8):
    p = run(["--gpus", str(n), "--launch-dry-run"], env={"RT_KFD_TOPOLOGY": topo8})
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert sorted(int(x["RANK"]) for x in lines) == list(range(n))
    assert all(x["LOCAL_RANK"] == x["RANK"] for x in lines)
    assert {x["WORLD_SIZE"] for x in lines} == {str(n)}
    assert {x["MASTER_ADDR"] for x in lines} == {"127.0.0.1"}
    assert len({x["MASTER_PORT"] for x in lines}) == 1
    assert all(x["RT_BENCH_LAUNCHED"] == "1" for x in lines)


def test_launch_rank_failure_propagates(topo8):
    p = run(["--gpus", "4", "--launch-dry-run"], env={"RT_BENCH_DRY_FAIL": "2:5", "RT_KFD_TOPOLOGY": topo8})
    assert p.returncode == 5
    assert "rank 2 exited 5" in p.stderr


def test_launch_fails_fast_without_gpus(tmp_path):
    # a topology with one GPU: --gpus 2 stops before starting any rank
    p = run(["--gpus", "2", "--steps", "3"], env={"RT_KFD_TOPOLOGY": fake_topology(tmp_path / "one", 1)}, timeout=60)
    assert p.returncode == 2
    assert "only 1 GPU(s) visible" in p.stderr


def test_launch_parent_never_loads_hip(topo8, tmp_path):
    """The launcher's count path (not a dry run's shortcut: the same code runs
    for every --gpus N > 1) leaves the parent without torch or the HIP
    runtime mapped when it starts the ranks."""
    maps = tmp_path / "parent_maps.txt"
    p = run(["--gpus", "2", "--launch-dry-run"], env={"RT_KFD_TOPOLOGY": topo8, "RT_BENCH_LAUNCH_MAPS": str(maps)})
    assert p.returncode == 0, p.stderr
    text = maps.read_text()
    assert "python" in text  # the parent's own mappings were recorded
    for lib in ("libamdhip64", "libtorch", "libhsa-runtime64", "librccl", "libamd_smi"):
        assert lib not in text, lib


@pytest.mark.parametrize("env,want", [
    ({}, 8),
    ({"HIP_VISIBLE_DEVICES": "0,1,2"}, 3),
    ({"CUDA_VISIBLE_DEVICES": "5"}, 1),
    ({"ROCR_VISIBLE_DEVICES": "1,3,5,7", "HIP_VISIBLE_DEVICES": "0,2"}, 2),
    ({"ROCR_VISIBLE_DEVICES": "1,3", "HIP_VISIBLE_DEVICES": "0,1,2"}, 2),
    ({"HIP_VISIBLE_DEVICES": "0,9,1"}, 1),  # stops at the first invalid index
    ({"HIP_VISIBLE_DEVICES": ""}, 0),
    ({"HIP_VISIBLE_DEVICES": "GPU-3a5c7e9b11d13f15"}, 1),
])
def test_visible_gpu_count(topo8, monkeypatch, env, want):
    sys.path.insert(0, ROOT)
    import bench
    for k in VIS:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("RT_KFD_TOPOLOGY", topo8)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert bench.visible_gpu_count() == want


def test_visible_gpu_count_without_topology(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("RT_KFD_TOPOLOGY", str(tmp_path / "absent"))
    assert bench.visible_gpu_count() is None
