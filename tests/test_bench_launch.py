"""bench.py's launch contract on CPU: ``--gpus N`` without a launcher starts N
ranks through torch.distributed.run (one process per GPU, as the driver
launches it), and a --gpus / WORLD_SIZE mismatch fails loudly instead of
silently benchmarking one rank."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for (k, v) in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_2_without_launcher_spawns_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"], capture_output=True, text=True,
                       timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["gpus"] == 2 for x in lines)


def test_gpus_must_match_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"], capture_output=True, text=True,
                       timeout=60, env=_env(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=4" in r.stderr


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--launch-probe"], capture_output=True, text=True, timeout=60,
                       env=_env())
    assert r.returncode == 0
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"rank": 0, "world": 1, "gpus": 1}


def test_launch_command_and_cpu_pool():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_command(["--gpus", "8", "--steps", "3"], 8, 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    old = os.environ.get("OMP_NUM_THREADS")
    try:
        os.environ["OMP_NUM_THREADS"] = "3"
        assert bench.cpu_pool_size(0) == min(3, len(os.sched_getaffinity(0)))
        assert bench.cpu_pool_size(2) <= 2
    finally:
        if old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = old
    info = bench.cpu_host_info()
    assert info["host_cpu_count"] == os.cpu_count()
