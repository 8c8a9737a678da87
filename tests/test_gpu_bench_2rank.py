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
    assert ns["n_gpus"] == 2 and ns["scaling"] == "strong" and ns["job_reports"] == 16384
    assert ns["heavy_hitters_equal_plaintext"] is True
