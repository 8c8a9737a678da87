"""poc/mastic_hip.py -- the reference-side binding a poc maintainer would add
next to ``poc/mastic.py`` to route a batch of the aggregator loop
(examples.py:49-74) through the GPU library (C ABI: include/mastic_hip.h):

    poc per report                                 this binding, per batch
    ---------------------------------------------  ---------------------------------------
    Mastic.prep_init          mastic.py:205-318    MasticHip.prep_init_batch
    Mastic.prep_shares_to_prep mastic.py:320-362   MasticHip.prep_shares_to_prep_batch
    Mastic.prep_next          mastic.py:364-377    (the poc's own, on the returned states)
    Mastic.agg_init + agg_update  :379-388         MasticHip.aggregate (GPU fold of the
                                                   out shares still in HBM)

It reads only what the poc's ``Mastic`` object already holds (``ID``,
``vidpf.BITS``, ``field``, ``flp`` and its ``valid`` parameters) and the poc's
own wire encoders (``encode_agg_param`` :413-435, ``test_vec_encode_public_share``
:531-535, ``test_vec_encode_input_share`` :516-529, ``test_vec_encode_prep_share``
:543-552), and returns the poc's own types: ``prep_init_batch`` returns one
``(prep_state, prep_share)`` per report exactly as ``prep_init`` does, with
``prep_state = (truncated_out_share, joint_rand_seed)`` as field elements of
``mastic.field`` / bytes (mastic.py:311-318), so the rest of a poc driver
(``prep_next``, ``unshard``) runs unchanged.  Plain ctypes, nothing beyond the
standard library.  ``tests/test_gpu_integration_stub.py`` runs the loop of
examples.py:49-74 through it on every golden vector.
"""
import ctypes

ABI_VERSION = 6  # include/mastic_hip.h MASTIC_ABI_VERSION
_EINVAL = -22
PROOF_SIZE = 32  # mastic.py:31 (eval proofs, joint-rand parts and seeds)
# mastic_decide_batch's per-report codes (include/mastic_hip.h)
DECIDE_VIDPF_FAIL, DECIDE_OK, DECIDE_FLP_FAIL = 0, 1, 2


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
    P, sz, i32, cp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p
    lib.mastic_abi_version.restype = i32
    lib.mastic_abi_version.argtypes = []
    if lib.mastic_abi_version() != ABI_VERSION:
        raise ImportError("libmastic_hip ABI %d, this stub expects %d" % (lib.mastic_abi_version(), ABI_VERSION))
    sigs = {
        "mastic_ctx_create": (i32, [ctypes.POINTER(MasticParams), ctypes.POINTER(P)]),
        "mastic_ctx_destroy": (None, [P]),
        "mastic_last_error": (cp, [P]),
        "mastic_get_sizes": (i32, [P, ctypes.POINTER(MasticSizes)]),
        # ctx, verify key + length, application ctx + length, agg_id, encoded agg param + length,
        # n, nonces, public shares, input shares -> prep shares, jr seeds, out shares, status
        "mastic_prep_init_batch": (i32, [P, cp, sz, cp, sz, i32, cp, sz, sz, cp, cp, cp, P, P, P, P]),
        # ctx, application ctx + length, encoded agg param + length, n, leader / helper prep shares
        # -> prep messages, per-report decide codes
        "mastic_decide_batch": (i32, [P, cp, sz, cp, sz, sz, cp, cp, P, P]),
        # ctx, agg_id, valid mask (n bytes or NULL) -> agg share (encode_vec)
        "mastic_aggregate": (i32, [P, i32, P, P]),
    }
    for (name, (res, args)) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
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
    """One GPU context for one poc Mastic instance.  The context keeps each
    aggregator's last ``prep_init_batch`` results (out shares included) in
    HBM until ``aggregate`` folds them."""

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
        self._n = [None, None]  # reports of each aggregator's last prep_init_batch

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

    def _decode_prep_share(self, do_weight_check, data):
        """test_vec_encode_prep_share's bytes (mastic.py:543-552) -> the poc's
        ``(eval_proof, verifier_share, joint_rand_part)`` tuple (:300-318)."""
        m = self.mastic
        eval_proof = data[:PROOF_SIZE]
        if not do_weight_check:
            return (eval_proof, None, None)
        rest = data[PROOF_SIZE:]
        jr_part = None
        if m.flp.JOINT_RAND_LEN > 0:
            (jr_part, rest) = (rest[:PROOF_SIZE], rest[PROOF_SIZE:])
        return (eval_proof, m.field.decode_vec(rest), jr_part)

    def prep_init_batch(self, verify_key, ctx, agg_id, agg_param, reports):
        """``[Mastic.prep_init(verify_key, ctx, agg_id, agg_param, nonce,
        public_share, input_share) for (nonce, public_share, input_shares)
        in reports]`` (mastic.py:205-318): one ``(prep_state, prep_share)``
        per report, in the poc's types.  ``reports`` holds each report's
        ``input_shares[agg_id]``."""
        m = self.mastic
        (_level, prefixes, do_weight_check) = agg_param
        enc_ap = m.encode_agg_param(agg_param)
        nonces = b"".join(r[0] for r in reports)
        pubs = b"".join(m.test_vec_encode_public_share(r[1]) for r in reports)
        ins = b"".join(m.test_vec_encode_input_share(r[2]) for r in reports)
        n = len(reports)
        psz = self.sizes.prep_share_size[1 if do_weight_check else 0]
        osz = len(prefixes) * (1 + self.sizes.output_len) * self.sizes.field_bytes
        prep_shares = ctypes.create_string_buffer(max(psz * n, 1))
        jr_seeds = ctypes.create_string_buffer(max(PROOF_SIZE * n, 1))
        out_shares = ctypes.create_string_buffer(max(osz * n, 1))
        status = (ctypes.c_int32 * max(n, 1))()
        self._check(self.lib.mastic_prep_init_batch(self.ctx, verify_key, len(verify_key), ctx, len(ctx), agg_id,
                                                    enc_ap, len(enc_ap), n, nonces, pubs, ins,
                                                    prep_shares, jr_seeds, out_shares, status))
        self._n[agg_id] = n
        with_seed = do_weight_check and m.flp.JOINT_RAND_LEN > 0  # mastic.py:236-248
        out = []
        for i in range(n):
            if status[i] != 0:  # FlpBBCGGI19.query aborted (t^P == 1): the poc raises there
                raise Exception("FLP query failed for report %d" % i)
            truncated = m.field.decode_vec(out_shares.raw[osz * i:osz * (i + 1)])
            jr_seed = jr_seeds.raw[PROOF_SIZE * i:PROOF_SIZE * (i + 1)] if with_seed else None
            prep_share = self._decode_prep_share(do_weight_check, prep_shares.raw[psz * i:psz * (i + 1)])
            out.append(((truncated, jr_seed), prep_share))
        return out

    def prep_shares_to_prep_batch(self, ctx, agg_param, prep_shares):
        """``[Mastic.prep_shares_to_prep(ctx, agg_param, [leader, helper])
        for (leader, helper) in prep_shares]`` (mastic.py:320-362) decided on
        the GPU.  Returns ``(prep_msgs, failures)``: the poc's prep message
        per report (the joint-rand seed, or None) and, per report, None or the
        Exception the poc would raise ('VIDPF verification failed' /
        'FLP verification failed')."""
        m = self.mastic
        enc_ap = m.encode_agg_param(agg_param)
        n = len(prep_shares)
        enc = [b"".join(m.test_vec_encode_prep_share(p[a]) for p in prep_shares) for a in range(2)]
        msgs = ctypes.create_string_buffer(max(PROOF_SIZE * n, 1))
        codes = ctypes.create_string_buffer(max(n, 1))
        self._check(self.lib.mastic_decide_batch(self.ctx, ctx, len(ctx), enc_ap, len(enc_ap), n, enc[0], enc[1],
                                                 msgs, codes))
        with_msg = agg_param[2] and m.flp.JOINT_RAND_LEN > 0
        prep_msgs, failures = [], []
        for i in range(n):
            code = codes.raw[i]
            failures.append(None if code == DECIDE_OK else
                            Exception("VIDPF verification failed" if code == DECIDE_VIDPF_FAIL else
                                      "FLP verification failed"))
            prep_msgs.append(msgs.raw[PROOF_SIZE * i:PROOF_SIZE * (i + 1)] if with_msg else None)
        return (prep_msgs, failures)

    def aggregate(self, agg_id, agg_param, valid=None):
        """``agg_init`` + ``agg_update`` (mastic.py:379-388) over the out
        shares of this aggregator's last ``prep_init_batch``, folded on the
        GPU (they never left HBM); ``valid[i]`` false leaves report i out
        (the reports whose prep_shares_to_prep / prep_next failed).  Returns
        the poc's agg share (field elements)."""
        m = self.mastic
        n = self._n[agg_id]
        if n is None:
            raise ValueError("no prep_init_batch for this aggregator")
        mask = None
        if valid is not None:
            if len(valid) != n:
                raise ValueError("valid mask has incorrect length")
            mask = bytes(int(bool(v)) for v in valid)
        nbytes = len(agg_param[1]) * (1 + self.sizes.output_len) * self.sizes.field_bytes
        agg = ctypes.create_string_buffer(max(nbytes, 1))
        self._check(self.lib.mastic_aggregate(self.ctx, agg_id, mask, agg))
        return m.field.decode_vec(agg.raw[:nbytes])
