"""Mastic VDAF on MI355X — the drop-in for the reference's ``Mastic`` class.

Mirrors ``poc/mastic.py`` (class ``Mastic`` :52-559, instantiations
:567-614): same method names, argument meaning, return types and error
behaviour (``ValueError`` for malformed inputs, ``Exception`` for failed
verification).  The per-report methods are batches of one; the ``*_batch``
methods are the production path and keep everything in wire encodings
(``test_vec/mastic`` format).  All cryptography runs in the HIP kernels
behind ``libmastic_hip.so``; this module only (de)serialises.
"""
import ctypes
import itertools

import numpy as np

from . import _lib
from .field import Field64, Field128

PROOF_SIZE = 32
CIRCUIT_IDS = {"Count": 1, "Sum": 2, "SumVec": 3, "Histogram": 4, "MultihotCountVec": 5}


def _check(ctx_ptr, rc):
    if rc != 0:
        msg = _lib.lib().mastic_last_error(ctx_ptr) if ctx_ptr else b""
        text = (msg or b"").decode(errors="replace") or "mastic error"
        if rc == -22:
            raise ValueError(text)
        raise _lib.MasticError(rc, text)


def _pack_path(path) -> bytes:
    """MSB-first bit packing (PrefixTreeIndex.encode, poc/vidpf.py:33-39)."""
    return np.packbits(np.fromiter(path, dtype=bool, count=len(path))).tobytes()


def _pack_bits_lsb(bits) -> bytes:
    out = bytearray((len(bits) + 7) // 8)
    for (i, b) in enumerate(bits):
        out[i // 8] |= int(bool(b)) << (i % 8)
    return bytes(out)


class VidpfInfo:
    """The parts of ``poc/vidpf.py``'s ``Vidpf`` object that drivers read
    through ``mastic.vidpf`` (constants :85-100, index helpers :418-427); the
    VIDPF itself runs in the HIP kernels."""

    KEY_SIZE = 16
    NONCE_SIZE = 16
    RAND_SIZE = 32

    def __init__(self, field, bits: int, value_len: int):
        self.field = field
        self.BITS = bits
        self.VALUE_LEN = value_len

    def test_index_from_int(self, value: int, length: int):
        """poc/vidpf.py:418-422 (MSB first)."""
        assert length <= self.BITS
        return tuple((value >> (length - 1 - i)) & 1 != 0 for i in range(length))

    def prefixes_for_level(self, level: int):
        """poc/vidpf.py:424-427"""
        return tuple(self.test_index_from_int(value, level + 1) for value in range(2 ** level))


class Mastic:
    """Mastic(bits, valid) with the validity circuit given as (name, params)."""

    ID = 0xFFFFFFFF
    VERIFY_KEY_SIZE = 32
    NONCE_SIZE = 16
    SHARES = 2
    ROUNDS = 1
    test_vec_name = "Mastic"

    def __init__(self, bits: int, circuit: str, length: int = 0, sum_vec_bits: int = 0,
                 max_measurement: int = 0, chunk_length: int = 0, device: int = 0):
        self.circuit = circuit
        self.params = _lib.MasticParams(CIRCUIT_IDS[circuit], bits, length, sum_vec_bits,
                                        max_measurement, chunk_length, device)
        self._ctx = ctypes.c_void_p()
        rc = _lib.lib().mastic_ctx_create(ctypes.byref(self.params), ctypes.byref(self._ctx))
        if rc != 0:
            raise _lib.MasticError(rc, "mastic_ctx_create failed (needs an MI355X / gfx950 device; "
                                       "there is no CPU fallback)")
        sz = _lib.MasticSizes()
        _check(self._ctx, _lib.lib().mastic_get_sizes(self._ctx, ctypes.byref(sz)))
        self.sizes = sz
        self.field = Field64 if sz.field_bytes == 8 else Field128
        self.BITS = bits
        self.VALUE_LEN = sz.value_len
        self.MEAS_LEN = sz.meas_len
        self.OUTPUT_LEN = sz.output_len
        self.PROOF_LEN = sz.proof_len
        self.VERIFIER_LEN = sz.verifier_len
        self.JOINT_RAND_LEN = sz.joint_rand_len
        self.RAND_SIZE = sz.rand_size
        self.ID = sz.algorithm_id
        self.length = length
        self.sum_vec_bits = sum_vec_bits
        self.max_measurement = max_measurement
        self.chunk_length = chunk_length
        self.vidpf = VidpfInfo(self.field, bits, sz.value_len)
        if circuit == "Sum":
            self._wbits = max_measurement.bit_length()
            self._offset = 2 ** self._wbits - 1 - max_measurement
        elif circuit == "MultihotCountVec":
            self._wbits = max_measurement.bit_length()
            self._offset = 2 ** self._wbits - 1 - max_measurement

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx:
            _lib.lib().mastic_ctx_destroy(ctx)
            self._ctx = None

    # ------------------------------------------------------------ circuits
    def encode_measurement(self, weight):
        """Valid.encode (vdaf_poc.flp_bbcggi19) -> MEAS_LEN field elements."""
        F = self.field
        c = self.circuit
        if c == "Count":
            return [F(int(weight))]
        if c == "Sum":
            if not 0 <= weight <= self.max_measurement:
                raise ValueError("measurement out of range")
            return (F.encode_into_bit_vector(weight, self._wbits)
                    + F.encode_into_bit_vector(weight + self._offset, self._wbits))
        if c == "SumVec":
            if len(weight) != self.length:
                raise ValueError("incorrect measurement length")
            return [x for v in weight for x in F.encode_into_bit_vector(int(v), self.sum_vec_bits)]
        if c == "Histogram":
            if not 0 <= weight < self.length:
                raise ValueError("bucket out of range")
            return [F(int(i == weight)) for i in range(self.length)]
        if len(weight) != self.length:
            raise ValueError("incorrect measurement length")
        total = sum(int(bool(x)) for x in weight)
        if total > self.max_measurement:
            raise ValueError("measurement weight too large")
        return [F(int(bool(x))) for x in weight] + F.encode_into_bit_vector(self._offset + total, self._wbits)

    def decode_result(self, output, num_measurements):
        """Valid.decode."""
        if self.circuit in ("Count", "Sum"):
            return output[0].int()
        return [x.int() for x in output]

    # --------------------------------------------------------- wire sizes
    def public_share_size(self):
        return self.sizes.public_share_size

    def input_share_size(self, agg_id):
        return self.sizes.input_share_size[agg_id]

    def prep_share_size(self, weight_check):
        return self.sizes.prep_share_size[1 if weight_check else 0]

    # ------------------------------------------------------ batch (native)
    def shard_batch(self, ctx: bytes, alphas, weights, nonces: bytes, rands: bytes):
        """Client shard of n reports on the GPU.  Returns the wire encodings
        (public_shares, input_shares_0, input_shares_1) as bytes."""
        n = len(alphas)
        ab = (self.BITS + 7) // 8
        a = bytearray(ab * n)
        for (i, alpha) in enumerate(alphas):
            if len(alpha) != self.BITS:
                raise ValueError("alpha out of range")
            a[ab * i: ab * (i + 1)] = _pack_path(alpha)
        betas = b"".join(self.field.encode_vec(self.encode_measurement(w)) for w in weights)
        return self.shard_encoded(ctx, n, bytes(a), betas, nonces, rands)

    def shard_encoded(self, ctx: bytes, n: int, alphas: bytes, betas: bytes, nonces: bytes, rands: bytes):
        if len(nonces) != 16 * n or len(rands) != self.RAND_SIZE * n:
            raise ValueError("nonce / randomness has incorrect length")
        pub = np.empty(self.sizes.public_share_size * n, np.uint8)
        in0 = np.empty(self.sizes.input_share_size[0] * n, np.uint8)
        in1 = np.empty(self.sizes.input_share_size[1] * n, np.uint8)
        _check(self._ctx, _lib.lib().mastic_shard_batch(
            self._ctx, ctx, len(ctx), n, _lib.buf(alphas), _lib.buf(betas), _lib.buf(nonces),
            _lib.buf(rands), _lib.buf(pub), _lib.buf(in0), _lib.buf(in1)))
        return (pub.tobytes(), in0.tobytes(), in1.tobytes())

    def prep_init_batch(self, verify_key: bytes, ctx: bytes, agg_id: int, agg_param, nonces: bytes,
                        public_shares: bytes, input_shares: bytes, want_out_shares=True):
        """prep_init for n reports (wire in, wire out).  Returns
        (prep_shares bytes, jr_seeds bytes, out_shares bytes or None, status int32 array)."""
        enc = self.encode_agg_param(agg_param) if not isinstance(agg_param, (bytes, bytearray)) else bytes(agg_param)
        (level, count, wc) = self._agg_param_header(enc)
        n = len(nonces) // 16
        self._check_verify_key(verify_key)
        if len(public_shares) != n * self.sizes.public_share_size:
            raise ValueError("public shares have incorrect length")
        if len(input_shares) != n * self.sizes.input_share_size[agg_id]:
            raise ValueError("input shares have incorrect length")
        ps = np.empty(n * self.prep_share_size(wc), np.uint8)
        js = np.empty(n * 32, np.uint8)
        ow = count * (1 + self.OUTPUT_LEN) * self.field.ENCODED_SIZE
        out = np.empty(n * ow, np.uint8) if want_out_shares else None
        st = np.empty(n, np.int32)
        _check(self._ctx, _lib.lib().mastic_prep_init_batch(
            self._ctx, verify_key, len(verify_key), ctx, len(ctx), agg_id, enc, len(enc), n, _lib.buf(nonces),
            _lib.buf(public_shares), _lib.buf(input_shares), _lib.buf(ps), _lib.buf(js), _lib.buf(out),
            _lib.buf(st)))
        return (ps.tobytes(), js.tobytes(), None if out is None else out.tobytes(), st)

    def decide_batch(self, ctx: bytes, agg_param, prep_shares_0: bytes, prep_shares_1: bytes):
        """prep_shares_to_prep for n report pairs -> (prep_msgs bytes, status uint8 array)."""
        enc = self.encode_agg_param(agg_param) if not isinstance(agg_param, (bytes, bytearray)) else bytes(agg_param)
        (_level, _count, wc) = self._agg_param_header(enc)
        psz = self.prep_share_size(wc)
        n = len(prep_shares_0) // psz
        if len(prep_shares_0) != n * psz or len(prep_shares_1) != n * psz:
            raise ValueError("prep shares have incorrect length")
        msgs = np.zeros(32 * n, np.uint8)
        valid = np.empty(n, np.uint8)
        _check(self._ctx, _lib.lib().mastic_decide_batch(
            self._ctx, ctx, len(ctx), enc, len(enc), n, _lib.buf(prep_shares_0), _lib.buf(prep_shares_1),
            _lib.buf(msgs), _lib.buf(valid)))
        return (msgs.tobytes(), valid)

    def decide_results(self, ctx: bytes, n: int):
        """prep_shares_to_prep + prep_next of both aggregators' last
        prep_init_device (same reports and agg param) on the GPU
        (``mastic_decide_results``) -> (accept uint8 array, decide codes)."""
        acc = np.empty(n, np.uint8)
        code = np.empty(n, np.uint8)
        _check(self._ctx, _lib.lib().mastic_decide_results(self._ctx, ctx, len(ctx), _lib.buf(acc), _lib.buf(code)))
        return (acc, code)

    def select_timing(self, agg_id: int):
        """Make last_timing* report agg_id's last prep_init (waits for it)."""
        _check(self._ctx, _lib.lib().mastic_prep_result(self._ctx, agg_id, None, None, None, None))

    def aggregate_to(self, agg_id: int, valid, dev_ptr: int, stream: int = 0):
        """``mastic_aggregate_device_on_stream``: fold into caller-owned device memory
        (e.g. a torch tensor's ``data_ptr()``); the share stays in HBM.
        ``stream`` is the hipStream_t handle whose queued work last touched
        the buffer (0 = the null stream)."""
        v = None if valid is None else np.ascontiguousarray(np.asarray(valid, dtype=np.uint8))
        _check(self._ctx, _lib.lib().mastic_aggregate_device_on_stream(
            self._ctx, agg_id, _lib.buf(v), ctypes.c_void_p(dev_ptr), ctypes.c_void_p(stream or None)))

    # ------------------------------- multi-GPU merge (library-owned RCCL)
    @staticmethod
    def comm_unique_id() -> bytes:
        """``mastic_comm_unique_id``: rank 0 creates the communicator id and
        hands it to the other ranks by any channel."""
        buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
        rc = _lib.lib().mastic_comm_unique_id(buf)
        if rc != 0:
            raise _lib.MasticError(rc, "mastic_comm_unique_id failed")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, unique_id: bytes, timeout_ms: int = 0):
        """``mastic_comm_init_timeout``: join this ctx to an RCCL communicator
        of ``nranks`` GPUs (collective; one process per GPU).  ``timeout_ms``
        bounds the init and every later wait on the communicator (0: the
        library's default, MASTIC_COMM_TIMEOUT_MS); a peer that does not join
        in time raises MasticError (ETIMEDOUT) instead of hanging."""
        if len(unique_id) != _lib.COMM_ID_BYTES:
            raise ValueError("communicator id has incorrect length")
        _check(self._ctx, _lib.lib().mastic_comm_init_timeout(self._ctx, nranks, rank, _lib.buf(bytes(unique_id)),
                                                              int(timeout_ms)))

    def comm_info(self):
        """(nranks, rank) of the ctx's communicator ((1, 0) without one)."""
        (n, r) = (ctypes.c_int(), ctypes.c_int())
        _check(self._ctx, _lib.lib().mastic_comm_info(self._ctx, ctypes.byref(n), ctypes.byref(r)))
        return (n.value, r.value)

    def comm_destroy(self):
        _check(self._ctx, _lib.lib().mastic_comm_destroy(self._ctx))

    def allgather_fold(self, dev_local: int, n_local: int, n_elems: int, dev_out: int, stream: int = 0):
        """``mastic_allgather_fold`` on device pointers: dev_out = the mod-p
        sum of every rank's n_local shares of n_elems elements."""
        _check(self._ctx, _lib.lib().mastic_allgather_fold(
            self._ctx, ctypes.c_void_p(dev_local or None), n_local, n_elems, ctypes.c_void_p(dev_out or None),
            ctypes.c_void_p(stream or None)))

    def merge_host(self, shares: bytes, n_local: int, n_elems: int) -> bytes:
        """``mastic_merge_host``: the mod-p sum over the communicator's ranks
        of n_local encode_vec shares of n_elems elements each (host bytes)."""
        if len(shares) != n_local * n_elems * self.field.ENCODED_SIZE:
            raise ValueError("shares have incorrect length")
        out = np.empty(n_elems * self.field.ENCODED_SIZE, np.uint8)
        _check(self._ctx, _lib.lib().mastic_merge_host(self._ctx, _lib.buf(bytes(shares)), n_local, n_elems,
                                                       _lib.buf(out)))
        return out.tobytes()

    def aggregate_merged(self, agg_ids, n_elems: int, valid=None, zeros=False) -> bytes:
        """``mastic_aggregate_merged``: the sum over the communicator's ranks
        (and over ``agg_ids``) of the GPU folds of the last prep_init's out
        shares, as encode_vec bytes (Mastic.agg_update + merge, mastic.py:384-397).
        ``zeros``: this rank ran no prep_init and contributes agg_init's
        zeros (the call is collective)."""
        mask = 0
        for a in agg_ids:
            if a not in (0, 1):
                raise ValueError("invalid aggregator ID")
            mask |= 1 << a
        if zeros:
            mask |= 4  # MASTIC_MERGE_ZEROS
        out = np.empty(n_elems * self.field.ENCODED_SIZE, np.uint8)
        v = None if valid is None else np.ascontiguousarray(np.asarray(valid, dtype=np.uint8))
        _check(self._ctx, _lib.lib().mastic_aggregate_merged(self._ctx, mask, _lib.buf(v), n_elems, _lib.buf(out)))
        return out.tobytes()

    def aggregate_device(self, agg_id: int, agg_param, valid=None, raw=False):
        """Fold the out shares of the last prep_init(_batch) of agg_id on the GPU
        (raw=True: the agg share as encode_vec bytes, without decoding)."""
        enc = self.encode_agg_param(agg_param) if not isinstance(agg_param, (bytes, bytearray)) else bytes(agg_param)
        (_level, count, _wc) = self._agg_param_header(enc)
        out = np.empty(count * (1 + self.OUTPUT_LEN) * self.field.ENCODED_SIZE, np.uint8)
        v = None if valid is None else np.ascontiguousarray(np.asarray(valid, dtype=np.uint8))
        _check(self._ctx, _lib.lib().mastic_aggregate(self._ctx, agg_id, _lib.buf(v), _lib.buf(out)))
        return out.tobytes() if raw else self.field.decode_vec(out.tobytes())

    # ------------------------------------------- device-resident batches
    def reports_shard(self, ctx: bytes, alphas_packed: bytes, betas: bytes, nonces: bytes, rands: bytes):
        """Shard n reports on the GPU and keep them resident in HBM."""
        n = len(nonces) // 16
        rep = Reports(self, n)
        _check(self._ctx, _lib.lib().mastic_reports_shard(
            rep._ptr, ctx, len(ctx), _lib.buf(alphas_packed), _lib.buf(betas), _lib.buf(nonces), _lib.buf(rands)))
        return rep

    def reports_upload(self, nonces: bytes, public_shares: bytes, input_shares_0=None, input_shares_1=None):
        rep = Reports(self, len(nonces) // 16)
        _check(self._ctx, _lib.lib().mastic_reports_upload(
            rep._ptr, _lib.buf(nonces), _lib.buf(public_shares), _lib.buf(input_shares_0),
            _lib.buf(input_shares_1)))
        return rep

    def prep_init_device(self, reports, verify_key: bytes, ctx: bytes, agg_id: int, agg_param):
        """Enqueue prep_init for resident reports; results stay in HBM."""
        enc = self.encode_agg_param(agg_param) if not isinstance(agg_param, (bytes, bytearray)) else bytes(agg_param)
        self._check_verify_key(verify_key)
        _check(self._ctx, _lib.lib().mastic_prep_init(self._ctx, reports._ptr, verify_key, len(verify_key), ctx,
                                                      len(ctx), agg_id, enc, len(enc)))

    def prep_result(self, reports, agg_id: int, agg_param, want_out_shares=False):
        """Wire results of the last prep_init_device for agg_id:
        (prep_shares bytes, jr_seeds bytes, out_shares bytes or None, status int32 array)."""
        enc = self.encode_agg_param(agg_param) if not isinstance(agg_param, (bytes, bytearray)) else bytes(agg_param)
        (_level, count, wc) = self._agg_param_header(enc)
        n = reports.n
        ps = np.empty(n * self.prep_share_size(wc), np.uint8)
        js = np.empty(n * 32, np.uint8)
        out = np.empty(n * count * (1 + self.OUTPUT_LEN) * self.field.ENCODED_SIZE, np.uint8) \
            if want_out_shares else None
        st = np.empty(n, np.int32)
        _check(self._ctx, _lib.lib().mastic_prep_result(self._ctx, agg_id, _lib.buf(ps), _lib.buf(js),
                                                        _lib.buf(out), _lib.buf(st)))
        return (ps.tobytes(), js.tobytes(), None if out is None else out.tobytes(), st)

    def synchronize(self):
        _check(self._ctx, _lib.lib().mastic_synchronize(self._ctx))

    def last_timing(self):
        """(eval_ms, eval_launches, absorb_ms, absorb_launches, total_ms) of the last prep_init."""
        e, a, t = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        ne, na = ctypes.c_int(), ctypes.c_int()
        _check(self._ctx, _lib.lib().mastic_last_timing(self._ctx, ctypes.byref(e), ctypes.byref(ne),
                                                        ctypes.byref(a), ctypes.byref(na), ctypes.byref(t)))
        return (e.value, ne.value, a.value, na.value, t.value)

    def last_timing3(self):
        """(aes_ms, aes_launches, proof_ms, proof_launches, absorb_ms, absorb_launches, total_ms)."""
        v = [ctypes.c_double() for _ in range(4)]
        k = [ctypes.c_int() for _ in range(3)]
        _check(self._ctx, _lib.lib().mastic_last_timing3(
            self._ctx, ctypes.byref(v[0]), ctypes.byref(k[0]), ctypes.byref(v[1]), ctypes.byref(k[1]),
            ctypes.byref(v[2]), ctypes.byref(k[2]), ctypes.byref(v[3])))
        return (v[0].value, k[0].value, v[1].value, k[1].value, v[2].value, k[2].value, v[3].value)

    def tree_stats(self, agg_param):
        enc = self.encode_agg_param(agg_param) if not isinstance(agg_param, (bytes, bytearray)) else bytes(agg_param)
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._ctx, _lib.lib().mastic_tree_stats(self._ctx, enc, len(enc), ctypes.byref(a),
                                                       ctypes.byref(b), ctypes.byref(c)))
        return (a.value, b.value, c.value)

    def set_memory_budget(self, nbytes: int):
        """HBM budget for one prep_init's work buffers (``mastic_set_memory_budget``;
        0 = 75 % of the free HBM).  Several contexts sharing one GPU (ranks of a
        one-GPU rehearsal) each take a slice."""
        _check(self._ctx, _lib.lib().mastic_set_memory_budget(self._ctx, ctypes.c_uint64(int(nbytes))))

    def set_test_hooks(self, force_slow_blk: int = -1, fail_allocs: int = 0):
        """Result-preserving test hooks of this context (``mastic_set_test_hooks``):
        hand the payload fast path over to the exact next_vec stream at convert
        block ``force_slow_blk`` (-1: off), and make the next ``fail_allocs``
        result / cache-slot allocations fail as if HBM were exhausted (the
        ENOMEM recovery path).  Outputs are identical either way.  Returns how
        many injected failures the previous setting had not yet used."""
        rc = _lib.lib().mastic_set_test_hooks(self._ctx, int(force_slow_blk), int(fail_allocs))
        if rc < 0:
            _check(self._ctx, rc)
        return rc

    def set_test_sponge_delay(self, delay_us: int):
        """Test hook (``mastic_set_test_sponge_delay``): the next prep_init
        that records empty timing marks on the binder-sponge stream (a
        frontier-cache hit) first holds that stream for ``delay_us``
        microseconds, so those marks complete late.  Results are unaffected."""
        _check(self._ctx, _lib.lib().mastic_set_test_sponge_delay(self._ctx, int(delay_us)))

    def set_serial_sponges(self, on=None) -> bool:
        """Measurement schedule (``mastic_set_serial_sponges``): with ``on``
        True every binder-sponge launch runs alone on the GPU (the level
        kernels wait for it), so ``last_timing3`` times the sponge kernels and
        the level kernel each by itself; False restores the overlapped
        schedule, None only queries.  Results are identical either way.
        Returns the previous setting."""
        rc = _lib.lib().mastic_set_serial_sponges(self._ctx, -1 if on is None else int(bool(on)))
        if rc < 0:
            _check(self._ctx, rc)
        return bool(rc)

    def set_frontier_cache(self, on: bool):
        """Keep each prep_init's per-level binder inputs and last frontier in HBM so
        that the next level of a sweep evaluates only its new level (C ABI
        mastic_set_frontier_cache); results are identical either way."""
        _check(self._ctx, _lib.lib().mastic_set_frontier_cache(self._ctx, 1 if on else 0, None))

    def last_prep_was_cached(self) -> bool:
        v = ctypes.c_int()
        _check(self._ctx, _lib.lib().mastic_set_frontier_cache(self._ctx, -1, ctypes.byref(v)))
        return bool(v.value)

    def proof_tree(self, agg_id: int, ctx: bytes, n: int):
        """Merkle tree over the eval proofs of the last prep_init of agg_id
        over n reports (proof-aggregation mode, see mastic_amd.proof_agg):
        list of levels, leaves first, each a list of 32-byte nodes."""
        from .proof_agg import level_sizes
        sizes = level_sizes(n)
        out = np.empty(32 * max(1, sum(sizes)), np.uint8)
        _check(self._ctx, _lib.lib().mastic_proof_tree(self._ctx, agg_id, ctx, len(ctx), _lib.buf(out), sum(sizes)))
        raw = out.tobytes()
        levels, off = [], 0
        for m in sizes:
            levels.append([raw[32 * (off + i):32 * (off + i + 1)] for i in range(m)])
            off += m
        return levels

    def work_bytes(self, agg_param):
        """HBM work bytes per report of one prep_init at this agg param
        (batches larger than the memory budget allows are run in chunks)."""
        enc = self.encode_agg_param(agg_param) if not isinstance(agg_param, (bytes, bytearray)) else bytes(agg_param)
        v = ctypes.c_uint64()
        _check(self._ctx, _lib.lib().mastic_work_bytes(self._ctx, enc, len(enc), ctypes.byref(v)))
        return v.value

    @staticmethod
    def _check_verify_key(verify_key):
        """The verify key is XofTurboShake128's seed, length-prefixed with one
        byte (mastic.py:302-306,499-510): the poc accepts any length below 256
        (its driver passes 16 bytes, examples.py:38,176)."""
        if not isinstance(verify_key, (bytes, bytearray)):
            raise TypeError("verify key must be bytes")
        if len(verify_key) > 255:
            raise ValueError("verify key has incorrect length")

    @staticmethod
    def _agg_param_header(enc: bytes):
        if len(enc) < 7:
            raise ValueError("agg param too short")
        return (int.from_bytes(enc[:2], "big"), int.from_bytes(enc[2:6], "big"), bool(enc[-1]))

    # ------------------------------------------- reference API (one report)
    def shard(self, ctx, measurement, nonce, rand):
        """poc/mastic.py:91-185"""
        if len(nonce) != self.NONCE_SIZE:
            raise ValueError("incorrect nonce size")
        if len(rand) != self.RAND_SIZE:
            raise ValueError("randomness has incorrect length")
        (alpha, weight) = measurement
        (pub, in0, in1) = self.shard_batch(ctx, [alpha], [weight], nonce, rand)
        return (self.decode_public_share(pub), [self.decode_input_share(0, in0), self.decode_input_share(1, in1)])

    def is_valid(self, agg_param, previous_agg_params) -> bool:
        """poc/mastic.py:187-203"""
        (level, _prefixes, do_weight_check) = agg_param
        weight_checked = ((do_weight_check and len(previous_agg_params) == 0)
                          or (not do_weight_check and any(p[2] for p in previous_agg_params)))
        level_increased = len(previous_agg_params) == 0 or level > previous_agg_params[-1][0]
        return weight_checked and level_increased

    def prep_init(self, verify_key, ctx, agg_id, agg_param, nonce, public_share, input_share):
        """poc/mastic.py:205-318 (routed to the GPU as a batch of one)."""
        if agg_id not in (0, 1):
            raise ValueError("invalid aggregator ID")
        (level, prefixes, wc) = agg_param
        if len(public_share) != self.BITS:
            raise ValueError("corrections words has incorrect length")
        for p in prefixes:
            if len(p) != level + 1:
                raise ValueError("prefix with incorrect length")
        pub = self.encode_public_share(public_share)
        ins = self.test_vec_encode_input_share(input_share)
        (ps, js, out, st) = self.prep_init_batch(verify_key, ctx, agg_id, agg_param, nonce, pub, ins)
        if st[0] != 0:
            raise ValueError("test point is a root of unity")
        prep_share = self.decode_prep_share(wc, ps)
        jr_seed = js[:32] if (wc and self.JOINT_RAND_LEN > 0) else None
        return ((self.field.decode_vec(out), jr_seed), prep_share)

    def prep_shares_to_prep(self, ctx, agg_param, prep_shares):
        """poc/mastic.py:320-362"""
        if len(prep_shares) != 2:
            raise ValueError("unexpected number of prep shares")
        (_level, _prefixes, wc) = agg_param
        for ps in prep_shares:
            if wc and ps[1] is None:
                raise ValueError("expected FLP verifier shares")
            if wc and self.JOINT_RAND_LEN > 0 and ps[2] is None:
                raise ValueError("expected FLP joint randomness parts")
        enc0 = self.test_vec_encode_prep_share(prep_shares[0] if wc else (prep_shares[0][0], None, None))
        enc1 = self.test_vec_encode_prep_share(prep_shares[1] if wc else (prep_shares[1][0], None, None))
        (msgs, valid) = self.decide_batch(ctx, agg_param, enc0, enc1)
        if valid[0] == 0:
            raise Exception("VIDPF verification failed")
        if valid[0] == 2:
            raise Exception("FLP verification failed")
        if not wc or self.JOINT_RAND_LEN == 0:
            return None
        return msgs[:32]

    def prep_next(self, _ctx, prep_state, prep_msg):
        """poc/mastic.py:364-377"""
        (truncated, jr_seed) = prep_state
        if jr_seed is not None:
            if prep_msg is None:
                raise ValueError("expected joint rand confirmation")
            if prep_msg != jr_seed:
                raise Exception("joint rand confirmation failed")
        return truncated

    def agg_init(self, agg_param):
        return self.field.zeros(len(agg_param[1]) * (1 + self.OUTPUT_LEN))

    def agg_update(self, agg_param, agg_share, out_share):
        return [a + b for (a, b) in zip(agg_share, out_share)]

    def merge(self, agg_param, agg_shares):
        agg = self.agg_init(agg_param)
        for s in agg_shares:
            agg = self.agg_update(agg_param, agg, s)
        return agg

    def unshard(self, agg_param, agg_shares, num_measurements):
        """poc/mastic.py:399-411"""
        agg = self.merge(agg_param, agg_shares)
        k = 1 + self.OUTPUT_LEN
        return [self.decode_result(agg[i + 1:i + k], agg[i].int()) for i in range(0, len(agg), k)]

    # ----------------------------------------------------------- encodings
    def encode_agg_param(self, agg_param) -> bytes:
        """poc/mastic.py:413-435"""
        (level, prefixes, do_weight_check) = agg_param
        if not 0 <= level < 2 ** 16:
            raise ValueError("level out of range")
        if not 0 <= len(prefixes) < 2 ** 32:
            raise ValueError("number of prefixes out of range")
        out = level.to_bytes(2, "big") + len(prefixes).to_bytes(4, "big")
        out += b"".join(_pack_path(p) for p in prefixes)
        return out + bytes([int(bool(do_weight_check))])

    def decode_agg_param(self, enc: bytes):
        (level, count, wc) = self._agg_param_header(enc)
        plen = (level + 1 + 7) // 8
        if len(enc) != 6 + plen * count + 1:
            raise ValueError("agg param has incorrect length")
        prefixes = []
        for i in range(count):
            b = enc[6 + plen * i: 6 + plen * (i + 1)]
            prefixes.append(tuple(bool((b[j // 8] >> (7 - j % 8)) & 1) for j in range(level + 1)))
        return (level, tuple(prefixes), wc)

    def encode_public_share(self, cws) -> bytes:
        """Vidpf.encode_public_share (poc/vidpf.py:382-394)."""
        if isinstance(cws, (bytes, bytearray)):
            return bytes(cws)
        out = _pack_bits_lsb(list(itertools.chain.from_iterable(cw[1] for cw in cws)))
        out += b"".join(cw[0] for cw in cws)
        out += b"".join(self.field.encode_vec(cw[2]) for cw in cws)
        return out + b"".join(cw[3] for cw in cws)

    def decode_public_share(self, data: bytes):
        if len(data) != self.sizes.public_share_size:
            raise ValueError("public share has incorrect length")
        B = self.BITS
        nb = (2 * B + 7) // 8
        bits = [bool((data[i // 8] >> (i % 8)) & 1) for i in range(2 * B)]
        pos = nb
        seeds = [data[pos + 16 * i: pos + 16 * (i + 1)] for i in range(B)]
        pos += 16 * B
        wl = self.VALUE_LEN * self.field.ENCODED_SIZE
        ws = [self.field.decode_vec(data[pos + wl * i: pos + wl * (i + 1)]) for i in range(B)]
        pos += wl * B
        proofs = [data[pos + 32 * i: pos + 32 * (i + 1)] for i in range(B)]
        return [(seeds[i], [bits[2 * i], bits[2 * i + 1]], ws[i], proofs[i]) for i in range(B)]

    test_vec_encode_public_share = encode_public_share

    def test_vec_encode_input_share(self, input_share) -> bytes:
        """poc/mastic.py:516-529"""
        if isinstance(input_share, (bytes, bytearray)):
            return bytes(input_share)
        (key, proof_share, seed, peer) = input_share
        out = key
        if proof_share is not None:
            out += self.field.encode_vec(proof_share)
        if seed is not None:
            out += seed
        if peer is not None:
            out += peer
        return out

    def decode_input_share(self, agg_id, data: bytes):
        if len(data) != self.sizes.input_share_size[agg_id]:
            raise ValueError("input share has incorrect length")
        key, rest = data[:16], data[16:]
        proof_share = seed = peer = None
        if agg_id == 0:
            k = self.PROOF_LEN * self.field.ENCODED_SIZE
            proof_share, rest = self.field.decode_vec(rest[:k]), rest[k:]
        if agg_id == 1 or self.JOINT_RAND_LEN > 0:
            seed, rest = rest[:32], rest[32:]
        if self.JOINT_RAND_LEN > 0:
            peer = rest[:32]
        return (key, proof_share, seed, peer)

    def test_vec_encode_prep_share(self, prep_share) -> bytes:
        """poc/mastic.py:543-552"""
        (eval_proof, verifier, jr_part) = prep_share
        out = eval_proof
        if jr_part is not None:
            out += jr_part
        if verifier is not None:
            out += self.field.encode_vec(verifier)
        return out

    def decode_prep_share(self, weight_check, data: bytes):
        if len(data) != self.prep_share_size(weight_check):
            raise ValueError("prep share has incorrect length")
        ep, rest = data[:32], data[32:]
        if not weight_check:
            return (ep, None, None)
        jp = None
        if self.JOINT_RAND_LEN > 0:
            jp, rest = rest[:32], rest[32:]
        return (ep, self.field.decode_vec(rest), jp)

    def test_vec_encode_prep_msg(self, msg) -> bytes:
        return msg if msg is not None else b""

    def test_vec_encode_agg_share(self, agg_share) -> bytes:
        return self.field.encode_vec(agg_share) if len(agg_share) else b""


class Reports:
    """A batch of reports resident in HBM (wire encodings)."""

    def __init__(self, mastic, n):
        self._m = mastic
        self._parent = None
        self._ptr = ctypes.c_void_p()
        _check(mastic._ctx, _lib.lib().mastic_reports_create(mastic._ctx, n, ctypes.byref(self._ptr)))
        self.n = n

    def view(self, first: int, count: int):
        """Reports first..first+count-1 of this batch, sharing its HBM
        (``mastic_reports_view``); keeps this batch alive."""
        v = Reports.__new__(Reports)
        v._m = self._m
        v._ptr = ctypes.c_void_p()
        _check(self._m._ctx, _lib.lib().mastic_reports_view(self._ptr, first, count, ctypes.byref(v._ptr)))
        v.n = count
        v._parent = self
        return v

    def upload(self, nonces: bytes, public_shares: bytes, input_shares_0=None, input_shares_1=None):
        """Overwrite this batch's reports in place (``mastic_reports_upload``);
        a view and the batch it views share HBM, so either sees the new data."""
        _check(self._m._ctx, _lib.lib().mastic_reports_upload(
            self._ptr, _lib.buf(nonces), _lib.buf(public_shares), _lib.buf(input_shares_0),
            _lib.buf(input_shares_1)))

    def download(self):
        m = self._m
        n = self.n
        nonces = np.empty(16 * n, np.uint8)
        pub = np.empty(m.sizes.public_share_size * n, np.uint8)
        in0 = np.empty(m.sizes.input_share_size[0] * n, np.uint8)
        in1 = np.empty(m.sizes.input_share_size[1] * n, np.uint8)
        _check(m._ctx, _lib.lib().mastic_reports_download(self._ptr, _lib.buf(nonces), _lib.buf(pub),
                                                          _lib.buf(in0), _lib.buf(in1)))
        return (nonces.tobytes(), pub.tobytes(), in0.tobytes(), in1.tobytes())

    def __del__(self):
        if getattr(self, "_ptr", None):
            _lib.lib().mastic_reports_destroy(self._ptr)
            self._ptr = None


class MasticCount(Mastic):
    """poc/mastic.py:567-574"""
    test_vec_name = "MasticCount"

    def __init__(self, bits: int, device: int = 0):
        super().__init__(bits, "Count", device=device)


class MasticSum(Mastic):
    """poc/mastic.py:577-584"""
    test_vec_name = "MasticSum"

    def __init__(self, bits: int, max_measurement: int, device: int = 0):
        super().__init__(bits, "Sum", max_measurement=max_measurement, device=device)


class MasticSumVec(Mastic):
    """poc/mastic.py:587-594"""
    test_vec_name = "MasticSumVec"

    def __init__(self, bits: int, length: int, sum_vec_bits: int, chunk_length: int, device: int = 0):
        super().__init__(bits, "SumVec", length=length, sum_vec_bits=sum_vec_bits,
                         chunk_length=chunk_length, device=device)


class MasticHistogram(Mastic):
    """poc/mastic.py:597-604"""
    test_vec_name = "MasticHistogram"

    def __init__(self, bits: int, length: int, chunk_length: int, device: int = 0):
        super().__init__(bits, "Histogram", length=length, chunk_length=chunk_length, device=device)


class MasticMultihotCountVec(Mastic):
    """poc/mastic.py:607-614"""
    test_vec_name = "MasticMultihotCountVec"

    def __init__(self, bits: int, length: int, max_weight: int, chunk_length: int, device: int = 0):
        super().__init__(bits, "MultihotCountVec", length=length, max_measurement=max_weight,
                         chunk_length=chunk_length, device=device)


def from_test_vec(tv: dict, device: int = 0) -> Mastic:
    bits = tv["vidpf_bits"]
    if "max_measurement" in tv:
        return MasticSum(bits, tv["max_measurement"], device=device)
    if "max_weight" in tv:
        return MasticMultihotCountVec(bits, tv["length"], tv["max_weight"], tv["chunk_length"], device=device)
    if "bits" in tv:
        return MasticSumVec(bits, tv["length"], tv["bits"], tv["chunk_length"], device=device)
    if "length" in tv:
        return MasticHistogram(bits, tv["length"], tv["chunk_length"], device=device)
    return MasticCount(bits, device=device)
