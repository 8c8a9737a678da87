"""The MASTIC_RCCL_LIB test hook on the CPU (no GPU calls): the library binds
the named library instead of RCCL -- never falling back to RCCL when it
cannot be loaded -- and tests/host/fake_rccl.cpp (the shared-memory stand-in
tests/test_gpu_comm_nrank.py runs N ranks on one GPU with) exports the eight
entry points the library binds and hands out ids."""
import ctypes
import os
import subprocess
import sys

from conftest import PKG_ROOT, ROOT

FAKE = os.path.join(ROOT, "tests", "host", "_build", "libfake_rccl.so")

_PROBE = r"""
import sys
sys.path.insert(0, %(pkg)r)
from mastic_amd import _lib
import ctypes
buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
rc = _lib.lib().mastic_comm_unique_id(buf)
print("RC", rc, buf.raw[:4].hex())
"""


def _probe(env_value):
    env = dict(os.environ)
    env["MASTIC_RCCL_LIB"] = env_value
    r = subprocess.run([sys.executable, "-c", _PROBE % {"pkg": PKG_ROOT}], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return [ln for ln in r.stdout.splitlines() if ln.startswith("RC")][0].split()


def test_fake_exports_the_bound_entry_points():
    if not os.path.exists(FAKE):
        import __graft_entry__
        __graft_entry__.build_fake_rccl()
    lib = ctypes.CDLL(FAKE)
    for name in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommGetAsyncError", "ncclCommAbort", "ncclCommFinalize",
                 "ncclCommDestroy", "ncclAllGather", "ncclGetErrorString"):
        assert hasattr(lib, name), name


def test_hook_binds_the_named_library_without_fallback():
    if not os.path.exists(FAKE):
        import __graft_entry__
        __graft_entry__.build_fake_rccl()
    # the fake's id starts with its magic "FRCC" (little-endian 0x46524343)
    assert _probe(FAKE) == ["RC", "0", "43435246"]
    # a library that cannot be loaded: ENODEV, not RCCL's id
    assert _probe(os.path.join(ROOT, "tests", "host", "_build", "no_such_rccl.so"))[:2] == ["RC", "-19"]
