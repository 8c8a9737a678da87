"""poc/mastic_hip.py -- the reference-side binding a poc maintainer would add
next to ``poc/mastic.py`` to route a batch of ``Mastic.prep_init`` calls
(mastic.py:205-318) through the GPU library (C ABI: include/mastic_hip.h).

It reads only what the poc's ``Mastic`` object already holds (``ID``,
``vidpf.BITS``, ``flp.valid`` and its parameters) and the poc's own wire
encoders (``encode_agg_param`` :413-435, ``test_vec_encode_public_share``
:531-535, ``test_vec_encode_input_share`` :516-529), and returns the prep
shares in ``test_vec_encode_prep_share``'s encoding (:543-552).  Plain ctypes,
no dependency beyond the standard library.  ``tests/test_gpu_integration_stub.py``
drives it with the poc-shaped restatement under ``oracle/`` standing in for
``poc/mastic.py`` and checks the reference's golden vectors through it.
"""
import ctypes

ABI_VERSION = 4  # include/mastic_hip.h MASTIC_ABI_VERSION
_EINVAL = -22


class MasticParams(ctypes.Structure):
    _fields_ = [("circuit", ctypes.c_uint32), ("bits", ctypes.c_uint32), ("length", ctypes.c_uint32),
                ("sum_vec_bits", ctypes.c_uint32), ("max_measurement", ctypes.c_uint64),
                ("chunk_length", ctypes.c_uint32), ("device", ctypes.c_int32)]


class MasticSizes(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint32) for name in (
        "field_bytes", "value_len", "meas_len", "output_len", "proof_len", "verifier_len",
        "joint_rand_len", "query_rand_len", "prove_rand_len", "rand_size", "public_share_size")] + [
        ("input_share_size", ctypes.c_uint32 * 2),
        ("prep_share_size", ctypes.c_uint32 * 2),
        ("algorithm_id", ctypes.c_uint32),
    ]


def load(path="libmastic_hip.so"):
    """Bind the library's entry points this stub uses."""
    lib = ctypes.CDLL(path)
    P, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.mastic_abi_version.restype = i32
    lib.mastic_abi_version.argtypes = []
    if lib.mastic_abi_version() != ABI_VERSION:
        raise ImportError("libmastic_hip ABI %d, this stub expects %d" % (lib.mastic_abi_version(), ABI_VERSION))
    lib.mastic_ctx_create.restype = i32
    lib.mastic_ctx_create.argtypes = [ctypes.POINTER(MasticParams), ctypes.POINTER(P)]
    lib.mastic_ctx_destroy.restype = None
    lib.mastic_ctx_destroy.argtypes = [P]
    lib.mastic_last_error.restype = ctypes.c_char_p
    lib.mastic_last_error.argtypes = [P]
    lib.mastic_get_sizes.restype = i32
    lib.mastic_get_sizes.argtypes = [P, ctypes.POINTER(MasticSizes)]
    lib.mastic_prep_init_batch.restype = i32
    lib.mastic_prep_init_batch.argtypes = [P, ctypes.c_char_p, sz,       # verify key, length
                                           ctypes.c_char_p, sz,          # application ctx
                                           i32, ctypes.c_char_p, sz,     # agg_id, encoded agg param
                                           sz, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,  # n, reports
                                           P, P, P, P]                   # prep shares, jr seeds, out shares, status
    return lib


def _params(mastic, device):
    """mastic_params from a poc Mastic instance (mastic.py:567-614)."""
    circuit = mastic.ID & 0xFF
    valid = mastic.flp.valid
    p = MasticParams(circuit=circuit, bits=mastic.vidpf.BITS, device=device)
    if circuit == 2:                  # Sum(field, max_measurement)
        p.max_measurement = valid.max_measurement
    elif circuit == 3:                # SumVec(field, length, bits, chunk_length)
        (p.length, p.sum_vec_bits, p.chunk_length) = (valid.length, valid.bits, valid.chunk_length)
    elif circuit == 4:                # Histogram(field, length, chunk_length)
        (p.length, p.chunk_length) = (valid.length, valid.chunk_length)
    elif circuit == 5:                # MultihotCountVec(field, length, max_weight, chunk_length)
        (p.length, p.max_measurement, p.chunk_length) = (valid.length, valid.max_weight, valid.chunk_length)
    return p


class MasticHip:
    """One GPU context for one poc Mastic instance."""

    def __init__(self, lib, mastic, device=0):
        self.lib = lib
        self.mastic = mastic
        self.params = _params(mastic, device)
        self.ctx = ctypes.c_void_p()
        rc = lib.mastic_ctx_create(ctypes.byref(self.params), ctypes.byref(self.ctx))
        if rc != 0:
            raise RuntimeError("mastic_ctx_create failed (%d): needs an MI355X (gfx950)" % rc)
        self.sizes = MasticSizes()
        self._check(lib.mastic_get_sizes(self.ctx, ctypes.byref(self.sizes)))

    def close(self):
        if self.ctx:
            self.lib.mastic_ctx_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    __del__ = close

    def _check(self, rc):
        if rc != 0:
            msg = (self.lib.mastic_last_error(self.ctx) or b"").decode(errors="replace")
            if rc == _EINVAL:
                raise ValueError(msg)       # the poc's ValueError cases (mastic.py:205-230)
            raise RuntimeError("%s (%d)" % (msg, rc))

    def prep_init_batch(self, verify_key, ctx, agg_id, agg_param, reports):
        """``[Mastic.prep_init(verify_key, ctx, agg_id, agg_param, nonce,
        public_share, input_share)[1] for (nonce, public_share, input_shares)
        in reports]``, encoded as ``test_vec_encode_prep_share``."""
        m = self.mastic
        enc_ap = m.encode_agg_param(agg_param)
        nonces = b"".join(r[0] for r in reports)
        pubs = b"".join(m.test_vec_encode_public_share(r[1]) for r in reports)
        ins = b"".join(m.test_vec_encode_input_share(r[2]) for r in reports)
        psz = self.sizes.prep_share_size[1 if agg_param[2] else 0]
        n = len(reports)
        prep_shares = ctypes.create_string_buffer(max(psz * n, 1))
        self._check(self.lib.mastic_prep_init_batch(self.ctx, verify_key, len(verify_key), ctx, len(ctx), agg_id,
                                                    enc_ap, len(enc_ap), n, nonces, pubs, ins,
                                                    prep_shares, None, None, None))
        return [prep_shares.raw[psz * i: psz * (i + 1)] for i in range(n)]
