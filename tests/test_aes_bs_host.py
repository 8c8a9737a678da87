"""The bitsliced AES-128 counter stream of tools/aes_bs.hpp (the measured
alternative to the level kernel's LDS T-table AES, DESIGN.md §5 "Bitsliced
AES") is correct before it is timed: compiled for the host and checked
against a byte-wise FIPS-197 AES -- the Boyar-Peralta S-box circuit over all
256 inputs, the FIPS-197 C.1 known answer through the counter-mode input
transform, and 200 random (key, seed, counter base) batches of 32 blocks of
XofFixedKeyAes128.hash_block (vdaf-13).  tools/aes_bs_mb.hip times the same
header on gfx950."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "host", "aes_bs_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_bitsliced_aes_matches_fips197(tmp_path):
    exe = str(tmp_path / "aes_bs_check")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-fsanitize=undefined", "-fno-sanitize-recover=all",
                           "-o", exe, SRC])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert r.stdout.strip() == "ok"
