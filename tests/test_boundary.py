"""CPU-side checks of the drop-in boundary (no compute calls without a GPU):
the C-ABI library loads, exports every symbol include/mastic_hip.h declares,
and the product fails loudly (no CPU fallback) when no gfx950 device exists."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "mastic_hip.h")).read()
    return sorted(set(re.findall(r"\b(mastic_[a-z_0-9]+)\s*\(", text)))


def _lib_path():
    from mastic_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.LIB_PATH


def test_header_and_binding_agree():
    from mastic_amd import _lib
    assert _header_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib_path())
    for name in _header_symbols():
        assert hasattr(lib, name), name


def test_library_is_gfx950_code_object():
    data = open(_lib_path(), "rb").read()
    assert b"gfx950" in data
    assert b"k_eval_aes" in data and b"k_node_proof" in data and b"k_absorb" in data


def test_no_cpu_fallback_without_device():
    """Without a GPU, creating a context raises instead of computing on the CPU."""
    import mastic_amd
    from mastic_amd import _lib
    lib = ctypes.CDLL(_lib_path())
    n = ctypes.c_int(0)
    hip = ctypes.CDLL("libamdhip64.so")
    if hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.MasticError):
        mastic_amd.MasticCount(4)
    del lib


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "draft-mouris-cfrg-mastic_amd")
    for dirpath, _dirs, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                text = open(os.path.join(dirpath, f), errors="replace").read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", text).replace("CPU oracle", ""), f
