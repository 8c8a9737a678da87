"""bench.py's N-rank path rehearsed on one GPU: `--gpus 2` launches two ranks
through torch.distributed.run (as the driver does for N > 1), here with a
gloo group and both ranks on cuda:0 (MASTIC_BENCH_BACKEND / _DEVICE); the C2
steps merge the ranks' agg shares, the full job folds and merges its slices,
and the north_star leg splits its job over the ranks (strong scaling) with
heavy hitters equal to the plaintext ones."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_two_ranks_on_one_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTIC_BENCH_BACKEND="gloo", MASTIC_BENCH_DEVICE="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--reports", "1024", "--total-reports", "2048", "--north-star-reports", "16384", "--cpu-baseline", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["full_job"]["job_reports"] == 4096
    ns = d["north_star"]
    assert "error" not in ns, ns
    assert ns["n_gpus"] == 2 and ns["scaling"] == "strong" and ns["job_reports"] == 16384
    assert ns["heavy_hitters_equal_plaintext"] is True
    for c in (d["comm"], ns["comm"]):  # the merge path the line was measured with
        assert c["backend"] == "gloo-rehearsal" and c["nranks"] == 2
        assert [x["rank"] for x in c["devices"]] == [0, 1]


def test_bench_two_ranks_through_the_library_comm_on_one_gpu():
    """`--gpus 2` on one GPU with the library's own communicator path (not the
    gloo merge): the MASTIC_RCCL_LIB test hook binds the shared-memory RCCL
    stand-in (tests/host/fake_rccl.cpp), so bench.py's lib_comm_init, the C2
    steps' and the full job's mastic_allgather_fold and the north_star sweep's
    CommMerge (mastic_aggregate_merged per level) run at two ranks exactly as
    on the driver's node; the line says which transport carried them."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fake = os.path.join(ROOT, "tests", "host", "_build", "libfake_rccl.so")
    assert os.path.exists(fake), "run __graft_entry__.build() first"
    env = dict(os.environ, MASTIC_BENCH_DEVICE="0", MASTIC_RCCL_LIB=fake)
    env.pop("MASTIC_BENCH_BACKEND", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--reports", "1024", "--total-reports", "2048", "--north-star-reports", "16384", "--cpu-baseline", "0",
           "--standalone", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["full_job"]["job_reports"] == 4096 and "mastic_allgather_fold" in d["full_job"]["what"]
    ns = d["north_star"]
    assert "error" not in ns, ns
    assert ns["n_gpus"] == 2 and ns["job_reports"] == 16384 and ns["heavy_hitters_equal_plaintext"] is True
    for c in (d["comm"], ns["comm"]):
        assert c["backend"] == "rccl-stand-in" and c["nranks"] == 2
        assert [x["rank"] for x in c["devices"]] == [0, 1]


def _run_bench(args, timeout=500):
    env = dict(os.environ, MASTIC_BENCH_BACKEND="gloo", MASTIC_BENCH_DEVICE="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    # the failing rank's own traceback, not only the launcher's tail
    first = "\n".join(l for l in r.stderr.splitlines() if l.startswith("[rank0]") or "Error" in l)[:4000]
    assert r.returncode == 0, first + "\n...\n" + r.stderr[-1500:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    # a rank whose north_star leg raised prints its traceback and leaves the
    # others' collectives ("Connection closed by peer"): show every rank's
    tb = [l for l in r.stderr.splitlines() if "Error" in l or "Traceback" in l or l.lstrip().startswith("File ")]
    assert "error" not in d.get("north_star", {}), (d["north_star"], "\n".join(tb)[-6000:])
    return d


def test_bench_four_ranks_uneven_job_on_one_gpu():
    """`--gpus 4` (four ranks through torch.distributed.run, gloo, one GPU,
    6 GiB of HBM budget per rank): C2 steps with the merge, and the
    north_star leg over a job of 16,387 reports, which four ranks cannot split
    evenly (split_bounds: 4,096 / 4,097 / 4,097 / 4,097); the heavy hitters
    and sampled levels' aggregates equal the plaintext ones."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = _run_bench(["--gpus", "4", "--steps", "1", "--warmup", "1", "--reports", "512", "--total-reports", "512",
                    "--north-star-reports", "16387", "--cpu-baseline", "0", "--memory-budget-gb", "6"])
    assert d["n_gpus"] == 4 and d["value"] > 0
    ns = d["north_star"]
    assert ns["n_gpus"] == 4 and ns["job_reports"] == 16387
    assert ns["heavy_hitters"] > 0 and ns["heavy_hitters_equal_plaintext"] is True


def test_bench_four_ranks_one_rank_without_reports():
    """A split sweep job of 3 reports over 4 ranks: rank 0 holds none
    (split_bounds gives it [0, 0)), so at every level it contributes zero
    shares through SweepMerge.total(have_results=False) to the same
    collectives as the other ranks.  The job's heavy hitters (every attribute
    with weight >= the threshold of 1) and sampled levels' aggregates equal
    the plaintext ones."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # (--standalone 0: this case is about the empty rank; four ranks sharing one GPU take ~100 s
    # per sweep of 32 merged levels already)
    d = _run_bench(["--gpus", "4", "--config", "c2sweep", "--split", "1", "--reports", "3", "--steps", "1",
                    "--warmup", "0", "--cpu-baseline", "0", "--memory-budget-gb", "2", "--standalone", "0"])
    c = d["config"]
    assert d["n_gpus"] == 4 and c["job_reports"] == 3 and c["reports_this_rank"] == 0
    assert c["heavy_hitters_equal_plaintext"] is True


def test_bench_under_torchrun_uses_the_library_communicator():
    """The driver's N > 1 launch path at one rank: torch.distributed.run starts
    bench.py, the ranks form a gloo control group, and every agg-share merge
    (C2 steps, the full job, the north_star sweep's per-level totals) goes
    through the library's own RCCL communicator (mastic_comm_init with one
    rank, mastic_aggregate_merged / mastic_allgather_fold, CommMerge)."""
    import socket
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1",
           "--warmup", "1", "--reports", "1024", "--total-reports", "2048", "--north-star-reports", "16384",
           "--cpu-baseline", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert "mastic_allgather_fold" in d["full_job"]["what"]
    ns = d["north_star"]
    assert "error" not in ns, ns
    assert ns["job_reports"] == 16384 and ns["heavy_hitters_equal_plaintext"] is True
    for c in (d["comm"], ns["comm"]):
        assert c["backend"] == "rccl" and c["nranks"] == 1 and len(c["devices"]) == 1
    # the sponge kernels' and the level kernel's own rates (Mastic.set_serial_sponges)
    for ab in (d["roofline_absorb"], ns["roofline_absorb"]):
        assert ab["standalone"]["frac"] > 0 and ab["standalone"]["level_kernel_frac_alone"] > 0


def test_bench_exits_nonzero_when_a_rank_cannot_join():
    """No silent fallback: under torch.distributed.run with the nccl backend, a
    rank whose library communicator cannot be created (injected) makes the
    run exit non-zero with no bench line, instead of switching to another
    merge transport."""
    import socket
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1",
           "--warmup", "0", "--reports", "512", "--total-reports", "512", "--north-star", "0", "--cpu-baseline", "0"]
    env = dict(os.environ, MASTIC_BENCH_COMM_FAIL_RANK="0")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "no silent fallback" in r.stderr
