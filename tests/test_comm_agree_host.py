"""The N-rank decision of the collective calls' agreement round
(csrc/comm_agree.hpp, mastic_hip.hip comm_agree; include/mastic_hip.h
"failure model"), on the host under ASan/UBSan with 8 simulated ranks: no
rank ever proceeds to the data all-gather unless every rank is ready; a rank
whose local work failed returns its own code, every other rank the lowest
failing rank's; calls that disagree on the entry point or the share geometry
(or a corrupted record) give EINVAL on every rank.  The GPU side of the same
code runs at world 1 in tests/test_gpu_comm.py (RCCL refuses two ranks on one
device; the driver's 8-GPU node runs it for real)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "host", "comm_agree_host.cpp")

WANT = {
    "all ready": "0,0,0,0,0,0,0,0",
    "enomem on rank 5": "-12,-12,-12,-12,-12,-12,-12,-12",
    "einval 2, enomem 6": "-22,-22,-22,-22,-22,-22,-12,-22",
    "geometry on rank 3": "-22,-22,-22,-22,-22,-22,-22,-22",
    "entry point on rank 7": "-22,-22,-22,-22,-22,-22,-22,-22",
    "bad record on rank 1": "-22,-22,-22,-22,-22,-22,-22,-22",
    "failure and mismatch": "-5,-5,-5,-5,-5,-5,-5,-5",
    "world 1": "0",
    "world 1 enomem": "-12",
    "zero elements": "0,0,0,0",
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_agreement_round_decisions_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "comm_agree_host")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-o", exe, SRC])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    got = {ln[5:30].strip(): ln[30:].strip().split("=", 1)[1] for ln in r.stdout.splitlines() if ln.startswith("case ")}
    assert got == WANT
    assert r.stdout.rstrip().endswith("comm_agree_host: OK")
