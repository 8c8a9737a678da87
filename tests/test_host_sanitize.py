"""Host AddressSanitizer / UBSan build and fuzz of the library's untrusted-
input decoders, on the CPU: the collector-supplied agg param
(csrc/host_tree.hpp: decode + prefix tree, the code build_tree runs before
uploading the tree) and the instantiation parameters (csrc/params.hpp
mc_derive, run by mastic_ctx_create).  tests/host/fuzz_host.cpp holds the
cases; every malformed agg param must return EINVAL with the reference's
ValueError text (poc/vidpf.py:229-239, poc/mastic.py:413-420), and no
sanitizer report may occur (-fno-sanitize-recover: the first one aborts)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "host", "fuzz_host.cpp")

WANT = {
    "empty": "rc=-22 err=agg param too short",
    "six bytes": "rc=-22 err=agg param too short",
    "truncated body": "rc=-22 err=agg param has incorrect length",
    "oversized body": "rc=-22 err=agg param has incorrect length",
    "count >= 2^31": "rc=-22 err=agg param has incorrect length",
    "level == bits": "rc=-22 err=level too deep",
    "weight check flag 2": "rc=-22 err=invalid weight check flag",
    "zero prefixes": "rc=-22 err=empty candidate prefix list",
    "non-zero tail bits": "rc=-22 err=prefix with incorrect length",
    "duplicate prefixes": "rc=-22 err=candidate prefixes are non-unique",
    "tree too large": "rc=-12 err=agg param tree too large",
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_decoders_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "fuzz_host")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-o", exe, SRC])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    lines = {ln[5:33].strip(): ln[33:].strip() for ln in r.stdout.splitlines() if ln.startswith("case ")}
    for (name, want) in WANT.items():
        assert lines.get(name) == want, (name, lines.get(name))
    assert lines["valid"].startswith("rc=0")
    assert r.stdout.rstrip().endswith("fuzz_host: OK")
