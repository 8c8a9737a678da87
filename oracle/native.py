"""Native multithreaded CPU baseline of prep_init (TEST INFRASTRUCTURE, see
oracle/__init__.py): the ctypes binding of ``oracle/native_prep.c``.

``prep_init_native`` runs ``Mastic.prep_init`` (poc/mastic.py:205-318) for a
batch of reports on the host's cores: the VIDPF evaluation, node proofs,
binders, counter check, eval proof, beta share and truncated out shares in C
(AES-NI, 64-bit Keccak, one thread per report range); the weight check's FLP
query (and joint randomness) through this package's Python restatement, the
same calls ``oracle/mastic.py`` makes.  bench.py times it as the
``cpu_baseline.native`` point beside the poc-faithful Python port; tests check
it against the Python oracle and the reference's golden vectors.
"""
import ctypes
import os
import subprocess
import threading

from .dst import (USAGE_CONVERT, USAGE_EVAL_PROOF, USAGE_EXTEND, USAGE_NODE_PROOF, USAGE_ONEHOT_CHECK,
                  USAGE_PAYLOAD_CHECK, dst, dst_alg)
from .flp import Count, Histogram, MultihotCountVec, Sum, SumVec

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libnative_prep.so")
_lock = threading.Lock()
_lib = None


def build() -> str:
    os.makedirs(os.path.dirname(_SO), exist_ok=True)
    src = os.path.join(_HERE, "native_prep.c")
    if (not os.path.exists(_SO)) or os.path.getmtime(_SO) < os.path.getmtime(src):
        tmp = _SO + ".%d.tmp" % os.getpid()
        subprocess.check_call(["gcc", "-O3", "-fPIC", "-shared", "-pthread", "-o", tmp, src])
        os.replace(tmp, _SO)
    return _SO


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                l = ctypes.CDLL(build())
                P, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
                l.native_prep_vidpf.restype = i32
                l.native_prep_vidpf.argtypes = [i32, i32, i32, i32, i32, i32, ctypes.c_char_p, i32, i32,
                                                ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz),
                                                ctypes.c_char_p, sz, sz, ctypes.c_char_p, ctypes.c_char_p, i32,
                                                ctypes.c_char_p, i32, i32, P, P, P]
                l.native_has_aesni.restype = i32
                _lib = l
    return _lib


def truncation(valid):
    """(tgroup, tlimit) of FlpBBCGGI19.truncate: groups of tgroup consecutive
    measurement elements decoded from bits, over the first tlimit elements."""
    if isinstance(valid, Sum):
        return (valid.bits, valid.bits)
    if isinstance(valid, SumVec):
        return (valid.bits, valid.length * valid.bits)
    if isinstance(valid, (Histogram, MultihotCountVec)):
        return (1, valid.length)
    assert isinstance(valid, Count)
    return (1, valid.MEAS_LEN)


def prep_init_native(o, verify_key: bytes, ctx: bytes, agg_id: int, agg_param, nonces: bytes, pubs: bytes,
                     ins: bytes, threads: int, times=None):
    """prep_init of n reports (wire encodings in) with an oracle Mastic `o`.
    Returns (prep_shares: list of bytes (test_vec_encode_prep_share),
    out_shares: bytes, n x len(prefixes) x (1 + OUTPUT_LEN) encoded elements).
    If ``times`` is a dict, the wall seconds of the C part (VIDPF, binders,
    eval proof: ``native_c_s``) and of the Python FLP part (``flp_py_s``) are
    added to it."""
    import time
    (level, prefixes, do_weight_check) = agg_param
    n = len(nonces) // 16
    f = o.field
    vl = o.vidpf.VALUE_LEN
    (tg, tl) = truncation(o.flp.valid)
    pbytes = (level + 1 + 7) // 8
    enc_p = bytearray()
    for p in prefixes:
        v = 0
        for b in p:
            v = (v << 1) | int(bool(b))
        enc_p += (v << (8 * pbytes - len(p))).to_bytes(pbytes, "big")
    ID = o.ID
    dsts = [dst(ctx, USAGE_EXTEND), dst(ctx, USAGE_CONVERT), dst(ctx, USAGE_NODE_PROOF),
            dst_alg(ctx, USAGE_ONEHOT_CHECK, ID), dst_alg(ctx, USAGE_PAYLOAD_CHECK, ID),
            dst_alg(ctx, USAGE_EVAL_PROOF, ID)]
    darr = (ctypes.c_char_p * 6)(*dsts)
    dlen = (ctypes.c_size_t * 6)(*[len(d) for d in dsts])
    psz = o.vidpf.public_share_size()
    isz = o.input_share_size(agg_id)
    row = len(prefixes) * (1 + -(-tl // tg)) * f.ENCODED_SIZE
    ev = ctypes.create_string_buffer(max(32 * n, 1))
    bs = ctypes.create_string_buffer(max(vl * f.ENCODED_SIZE * n, 1))
    out = ctypes.create_string_buffer(max(row * n, 1))
    t0 = time.perf_counter()
    rc = lib().native_prep_vidpf(8 * f.ENCODED_SIZE, o.vidpf.BITS, vl, agg_id, level, len(prefixes),
                                 bytes(enc_p), tg, tl, darr, dlen, verify_key, len(verify_key), n, nonces, pubs,
                                 psz, ins, isz, threads, ev, bs, out)
    t1 = time.perf_counter()
    if rc != 0:
        raise ValueError("native_prep_vidpf: bad arguments")
    shares = []
    for i in range(n):
        eval_proof = ev.raw[32 * i:32 * (i + 1)]
        jr_part = verifier = None
        if do_weight_check:
            # the FLP part of prep_init, as oracle/mastic.py (poc/mastic.py:236-256)
            nonce = nonces[16 * i:16 * (i + 1)]
            isd = o.decode_input_share(agg_id, ins[isz * i:isz * (i + 1)])
            (_key, proof_share, seed, peer_part) = o.expand_input_share(ctx, agg_id, isd)
            beta_share = f.decode_vec(bs.raw[vl * f.ENCODED_SIZE * i:vl * f.ENCODED_SIZE * (i + 1)])
            query_rand = o.query_rand(verify_key, ctx, nonce, level)
            joint_rand = []
            if o.flp.JOINT_RAND_LEN > 0:
                jr_part = o.joint_rand_part(ctx, seed, beta_share[1:], nonce)
                parts = [jr_part, peer_part] if agg_id == 0 else [peer_part, jr_part]
                joint_rand = o.joint_rand(ctx, o.joint_rand_seed(ctx, parts))
            verifier = o.flp.query(beta_share[1:], proof_share, query_rand, joint_rand, 2)
        shares.append(o.test_vec_encode_prep_share((eval_proof, verifier, jr_part)))
    if times is not None:
        times["native_c_s"] = times.get("native_c_s", 0.0) + t1 - t0
        times["flp_py_s"] = times.get("flp_py_s", 0.0) + time.perf_counter() - t1
    return (shares, out.raw[:row * n])


def has_aesni() -> bool:
    return bool(lib().native_has_aesni())
