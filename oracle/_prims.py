"""ctypes binding of oracle/prims.c (TEST INFRASTRUCTURE, see oracle/__init__.py).

The shared library is built into ``oracle/_build/`` by ``oracle/Makefile``
(``__graft_entry__.build()`` runs it); if it is missing we compile it on
demand with gcc so the CPU test suite is self-contained.
"""
import ctypes
import os
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle_prims.so")
_lock = threading.Lock()
_lib = None


def build() -> str:
    os.makedirs(os.path.dirname(_SO), exist_ok=True)
    src = os.path.join(_HERE, "prims.c")
    if (not os.path.exists(_SO)) or os.path.getmtime(_SO) < os.path.getmtime(src):
        tmp = _SO + ".%d.tmp" % os.getpid()
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", tmp, src])
        os.replace(tmp, _SO)
    return _SO


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                l = ctypes.CDLL(build())
                l.oracle_turboshake128.argtypes = [
                    ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint8,
                    ctypes.c_char_p, ctypes.c_size_t]
                l.oracle_aes128_expand.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
                l.oracle_aes128_encrypt.argtypes = [
                    ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
                l.oracle_fixed_key_aes_blocks.argtypes = [
                    ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64,
                    ctypes.c_size_t, ctypes.c_char_p]
                _lib = l
    return _lib


def turboshake128(msg: bytes, domain: int, out_len: int) -> bytes:
    out = ctypes.create_string_buffer(out_len)
    lib().oracle_turboshake128(msg, len(msg), domain, out, out_len)
    return out.raw


def aes128_expand(key: bytes) -> bytes:
    assert len(key) == 16
    rk = ctypes.create_string_buffer(176)
    lib().oracle_aes128_expand(key, rk)
    return rk.raw


def aes128_encrypt(round_keys: bytes, block: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().oracle_aes128_encrypt(round_keys, block, out)
    return out.raw


def fixed_key_aes_blocks(round_keys: bytes, seed: bytes, first_ctr: int, nblocks: int) -> bytes:
    out = ctypes.create_string_buffer(16 * nblocks)
    lib().oracle_fixed_key_aes_blocks(round_keys, seed, first_ctr, nblocks, out)
    return out.raw
