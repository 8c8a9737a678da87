"""Mastic VDAF (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates ``poc/mastic.py`` (class ``Mastic`` :52-559 and the instantiations
:567-614) with the same per-report control flow.  Adds the wire decoders the
poc lacks (input share, prep share, agg param) so golden vectors can be
replayed.
"""
from .common import (concat, decode_path_msb_first, encode_path_msb_first, front,
                     from_be_bytes, to_be_bytes, to_le_bytes, vec_add, vec_sub)
from .dst import (USAGE_EVAL_PROOF, USAGE_JOINT_RAND, USAGE_JOINT_RAND_PART,
                  USAGE_JOINT_RAND_SEED, USAGE_ONEHOT_CHECK, USAGE_PAYLOAD_CHECK,
                  USAGE_PROOF_SHARE, USAGE_PROVE_RAND, USAGE_QUERY_RAND, dst_alg)
from .field import Field64, Field128
from .flp import Count, FlpBBCGGI19, Histogram, MultihotCountVec, Sum, SumVec
from .vidpf import PROOF_SIZE, Vidpf, bfs_nodes
from .xof import XofTurboShake128


class Mastic:
    xof = XofTurboShake128
    ID = 0xFFFFFFFF
    VERIFY_KEY_SIZE = XofTurboShake128.SEED_SIZE
    NONCE_SIZE = 16
    SHARES = 2
    ROUNDS = 1
    test_vec_name = "Mastic"

    def __init__(self, bits: int, valid):
        """poc/mastic.py:81-89"""
        self.field = valid.field
        self.flp = FlpBBCGGI19(valid)
        self.vidpf = Vidpf(valid.field, bits, 1 + valid.MEAS_LEN)
        self.RAND_SIZE = self.vidpf.RAND_SIZE + 2 * self.xof.SEED_SIZE
        if self.flp.JOINT_RAND_LEN > 0:
            self.RAND_SIZE += self.xof.SEED_SIZE

    # ---------------------------------------------------------- client
    def shard(self, ctx, measurement, nonce, rand):
        """poc/mastic.py:91-185"""
        use_jr = self.flp.JOINT_RAND_LEN > 0
        (vidpf_rand, rand) = front(self.vidpf.RAND_SIZE, rand)
        (prove_rand_seed, rand) = front(self.xof.SEED_SIZE, rand)
        (helper_seed, rand) = front(self.xof.SEED_SIZE, rand)
        leader_seed = None
        if use_jr:
            (leader_seed, rand) = front(self.xof.SEED_SIZE, rand)
        if len(rand) != 0:
            raise ValueError("randomness has incorrect length")
        (alpha, weight) = measurement
        beta = [self.field(1)] + self.flp.encode(weight)
        (cws, keys) = self.vidpf.gen(alpha, beta, ctx, nonce, vidpf_rand)
        joint_rand = []
        parts = [None, None]
        if use_jr:
            lb = self.vidpf.get_beta_share(0, cws, keys[0], ctx, nonce)
            hb = self.vidpf.get_beta_share(1, cws, keys[1], ctx, nonce)
            parts = [self.joint_rand_part(ctx, leader_seed, lb[1:], nonce),
                     self.joint_rand_part(ctx, helper_seed, hb[1:], nonce)]
            joint_rand = self.joint_rand(ctx, self.joint_rand_seed(ctx, parts))
        proof = self.flp.prove(beta[1:], self.prove_rand(ctx, prove_rand_seed), joint_rand)
        leader_proof_share = vec_sub(proof, self.helper_proof_share(ctx, helper_seed))
        input_shares = [
            (keys[0], leader_proof_share, leader_seed, parts[1]),
            (keys[1], None, helper_seed, parts[0]),
        ]
        return (cws, input_shares)

    def is_valid(self, agg_param, previous_agg_params) -> bool:
        """poc/mastic.py:187-203"""
        (level, _prefixes, do_weight_check) = agg_param
        weight_checked = ((do_weight_check and len(previous_agg_params) == 0)
                          or (not do_weight_check
                              and any(p[2] for p in previous_agg_params)))
        level_increased = (len(previous_agg_params) == 0
                           or level > previous_agg_params[-1][0])
        return weight_checked and level_increased

    # ----------------------------------------------------- aggregators
    def prep_init(self, verify_key, ctx, agg_id, agg_param, nonce, cws, input_share):
        """poc/mastic.py:205-318"""
        (level, prefixes, do_weight_check) = agg_param
        (key, proof_share, seed, peer_part) = self.expand_input_share(ctx, agg_id, input_share)
        (out_share, root) = self.vidpf.eval_with_siblings(
            agg_id, cws, key, level, prefixes, ctx, nonce)

        jr_part = None
        jr_seed = None
        verifier_share = None
        if do_weight_check:
            beta_share = self.vidpf.get_beta_share(agg_id, cws, key, ctx, nonce)
            query_rand = self.query_rand(verify_key, ctx, nonce, level)
            joint_rand = []
            if self.flp.JOINT_RAND_LEN > 0:
                assert seed is not None and peer_part is not None
                jr_part = self.joint_rand_part(ctx, seed, beta_share[1:], nonce)
                parts = [jr_part, peer_part] if agg_id == 0 else [peer_part, jr_part]
                jr_seed = self.joint_rand_seed(ctx, parts)
                joint_rand = self.joint_rand(ctx, jr_seed)
            verifier_share = self.flp.query(beta_share[1:], proof_share, query_rand,
                                            joint_rand, 2)

        payload_binder = []
        onehot_binder = []
        for n in bfs_nodes(root):
            if n.left is not None and n.right is not None:
                payload_binder.append(self.field.encode_vec(
                    vec_sub(n.w, vec_add(n.left.w, n.right.w))))
            onehot_binder.append(n.proof)
        payload_check = self.xof(b"", dst_alg(ctx, USAGE_PAYLOAD_CHECK, self.ID),
                                 concat(payload_binder)).next(PROOF_SIZE)
        onehot_check = self.xof(b"", dst_alg(ctx, USAGE_ONEHOT_CHECK, self.ID),
                                concat(onehot_binder)).next(PROOF_SIZE)
        counter_check = self.field.encode_vec(
            [root.left.w[0] + root.right.w[0] + self.field(agg_id)])
        eval_proof = self.xof(verify_key, dst_alg(ctx, USAGE_EVAL_PROOF, self.ID),
                              onehot_check + counter_check + payload_check).next(PROOF_SIZE)

        truncated = []
        for val_share in out_share:
            truncated += [val_share[0]] + self.flp.truncate(val_share[1:])
        return ((truncated, jr_seed), (eval_proof, verifier_share, jr_part))

    def prep_shares_to_prep(self, ctx, agg_param, prep_shares):
        """poc/mastic.py:320-362"""
        (_level, _prefixes, do_weight_check) = agg_param
        if len(prep_shares) != 2:
            raise ValueError("unexpected number of prep shares")
        (ep0, vs0, jp0) = prep_shares[0]
        (ep1, vs1, jp1) = prep_shares[1]
        if ep0 != ep1:
            raise Exception("VIDPF verification failed")
        if not do_weight_check:
            return None
        if vs0 is None or vs1 is None:
            raise ValueError("expected FLP verifier shares")
        if not self.flp.decide(vec_add(vs0, vs1)):
            raise Exception("FLP verification failed")
        if self.flp.JOINT_RAND_LEN == 0:
            return None
        if jp0 is None or jp1 is None:
            raise ValueError("expected FLP joint randomness parts")
        return self.joint_rand_seed(ctx, [jp0, jp1])

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
        """poc/mastic.py:379-382"""
        return self.field.zeros(len(agg_param[1]) * (1 + self.flp.OUTPUT_LEN))

    def agg_update(self, agg_param, agg_share, out_share):
        """poc/mastic.py:384-388"""
        return vec_add(agg_share, out_share)

    def merge(self, agg_param, agg_shares):
        """poc/mastic.py:390-397"""
        agg = self.agg_init(agg_param)
        for s in agg_shares:
            agg = vec_add(agg, s)
        return agg

    def unshard(self, agg_param, agg_shares, num_measurements):
        """poc/mastic.py:399-411"""
        agg = self.merge(agg_param, agg_shares)
        result = []
        while len(agg) > 0:
            (chunk, agg) = front(self.flp.OUTPUT_LEN + 1, agg)
            result.append(self.flp.decode(chunk[1:], chunk[0].int()))
        return result

    # ------------------------------------------------------ encodings
    def encode_agg_param(self, agg_param) -> bytes:
        """poc/mastic.py:413-435"""
        (level, prefixes, do_weight_check) = agg_param
        if not 0 <= level < 2 ** 16:
            raise ValueError("level out of range")
        if not 0 <= len(prefixes) < 2 ** 32:
            raise ValueError("number of prefixes out of range")
        out = to_be_bytes(level, 2) + to_be_bytes(len(prefixes), 4)
        for p in prefixes:
            out += encode_path_msb_first(p)
        return out + to_be_bytes(int(do_weight_check), 1)

    def decode_agg_param(self, data: bytes):
        level = from_be_bytes(data[:2])
        count = from_be_bytes(data[2:6])
        plen = (level + 1 + 7) // 8
        if len(data) != 6 + plen * count + 1:
            raise ValueError("agg param has incorrect length")
        prefixes = tuple(decode_path_msb_first(data[6 + plen * i: 6 + plen * (i + 1)], level + 1)
                         for i in range(count))
        return (level, prefixes, bool(data[-1]))

    def expand_input_share(self, ctx, agg_id, input_share):
        """poc/mastic.py:437-450"""
        (key, proof_share, seed, peer_part) = input_share
        if agg_id != 0:
            assert seed is not None
            proof_share = self.helper_proof_share(ctx, seed)
        return (key, proof_share, seed, peer_part)

    def helper_proof_share(self, ctx, seed):
        """poc/mastic.py:452-459"""
        return self.xof.expand_into_vec(self.field, seed, dst_alg(ctx, USAGE_PROOF_SHARE, self.ID),
                                        b"", self.flp.PROOF_LEN)

    def prove_rand(self, ctx, seed):
        """poc/mastic.py:461-468"""
        return self.xof.expand_into_vec(self.field, seed, dst_alg(ctx, USAGE_PROVE_RAND, self.ID),
                                        b"", self.flp.PROVE_RAND_LEN)

    def joint_rand_part(self, ctx, seed, weight_share, nonce):
        """poc/mastic.py:470-481"""
        return self.xof.derive_seed(seed, dst_alg(ctx, USAGE_JOINT_RAND_PART, self.ID),
                                    nonce + self.field.encode_vec(weight_share))

    def joint_rand_seed(self, ctx, parts):
        """poc/mastic.py:483-488"""
        return self.xof.derive_seed(b"", dst_alg(ctx, USAGE_JOINT_RAND_SEED, self.ID), concat(parts))

    def joint_rand(self, ctx, seed):
        """poc/mastic.py:490-497"""
        return self.xof.expand_into_vec(self.field, seed, dst_alg(ctx, USAGE_JOINT_RAND, self.ID),
                                        b"", self.flp.JOINT_RAND_LEN)

    def query_rand(self, verify_key, ctx, nonce, level):
        """poc/mastic.py:499-510"""
        return self.xof.expand_into_vec(self.field, verify_key,
                                        dst_alg(ctx, USAGE_QUERY_RAND, self.ID),
                                        nonce + to_le_bytes(level, 2), self.flp.QUERY_RAND_LEN)

    # ------------------------------------------- test-vector encodings
    def test_vec_set_type_param(self, test_vec):
        test_vec["vidpf_bits"] = int(self.vidpf.BITS)
        return ["vidpf_bits"] + self.flp.test_vec_set_type_param(test_vec)

    def test_vec_encode_input_share(self, input_share) -> bytes:
        """poc/mastic.py:516-529"""
        (key, proof_share, seed, peer_part) = input_share
        out = key
        if proof_share is not None:
            out += self.field.encode_vec(proof_share)
        if seed is not None:
            out += seed
        if peer_part is not None:
            out += peer_part
        return out

    def test_vec_encode_public_share(self, cws) -> bytes:
        return self.vidpf.encode_public_share(cws)

    def test_vec_encode_agg_share(self, agg_share) -> bytes:
        return self.field.encode_vec(agg_share) if len(agg_share) > 0 else b""

    def test_vec_encode_prep_share(self, prep_share) -> bytes:
        """poc/mastic.py:543-552 (note: jr part precedes the verifier share)."""
        (eval_proof, verifier_share, jr_part) = prep_share
        out = eval_proof
        if jr_part is not None:
            out += jr_part
        if verifier_share is not None:
            out += self.field.encode_vec(verifier_share)
        return out

    def test_vec_encode_prep_msg(self, prep_msg) -> bytes:
        return prep_msg if prep_msg is not None else b""

    # ------------------------------------------------------ decoders
    def input_share_size(self, agg_id: int) -> int:
        n = self.vidpf.KEY_SIZE
        if agg_id == 0:
            n += self.flp.PROOF_LEN * self.field.ENCODED_SIZE
            if self.flp.JOINT_RAND_LEN > 0:
                n += 2 * self.xof.SEED_SIZE
        else:
            n += self.xof.SEED_SIZE
            if self.flp.JOINT_RAND_LEN > 0:
                n += self.xof.SEED_SIZE
        return n

    def decode_input_share(self, agg_id: int, data: bytes):
        if len(data) != self.input_share_size(agg_id):
            raise ValueError("input share has incorrect length")
        (key, rest) = front(self.vidpf.KEY_SIZE, data)
        proof_share = None
        seed = None
        peer = None
        if agg_id == 0:
            plen = self.flp.PROOF_LEN * self.field.ENCODED_SIZE
            (enc, rest) = front(plen, rest)
            proof_share = self.field.decode_vec(enc)
        if agg_id == 1 or self.flp.JOINT_RAND_LEN > 0:
            (seed, rest) = front(self.xof.SEED_SIZE, rest)
        if self.flp.JOINT_RAND_LEN > 0:
            (peer, rest) = front(self.xof.SEED_SIZE, rest)
        return (key, proof_share, seed, peer)

    def prep_share_size(self, do_weight_check: bool) -> int:
        n = PROOF_SIZE
        if do_weight_check:
            n += self.flp.VERIFIER_LEN * self.field.ENCODED_SIZE
            if self.flp.JOINT_RAND_LEN > 0:
                n += self.xof.SEED_SIZE
        return n

    def decode_prep_share(self, do_weight_check: bool, data: bytes):
        if len(data) != self.prep_share_size(do_weight_check):
            raise ValueError("prep share has incorrect length")
        (eval_proof, rest) = front(PROOF_SIZE, data)
        if not do_weight_check:
            return (eval_proof, None, None)
        jr_part = None
        if self.flp.JOINT_RAND_LEN > 0:
            (jr_part, rest) = front(self.xof.SEED_SIZE, rest)
        return (eval_proof, self.field.decode_vec(rest), jr_part)


class MasticCount(Mastic):
    """poc/mastic.py:567-574"""
    ID = 0xFFFF0001
    test_vec_name = "MasticCount"

    def __init__(self, bits: int):
        super().__init__(bits, Count(Field64))


class MasticSum(Mastic):
    """poc/mastic.py:577-584"""
    ID = 0xFFFF0002
    test_vec_name = "MasticSum"

    def __init__(self, bits: int, max_measurement: int):
        super().__init__(bits, Sum(Field64, max_measurement))


class MasticSumVec(Mastic):
    """poc/mastic.py:587-594"""
    ID = 0xFFFF0003
    test_vec_name = "MasticSumVec"

    def __init__(self, bits: int, length: int, sum_vec_bits: int, chunk_length: int):
        super().__init__(bits, SumVec(Field128, length, sum_vec_bits, chunk_length))


class MasticHistogram(Mastic):
    """poc/mastic.py:597-604"""
    ID = 0xFFFF0004
    test_vec_name = "MasticHistogram"

    def __init__(self, bits: int, length: int, chunk_length: int):
        super().__init__(bits, Histogram(Field128, length, chunk_length))


class MasticMultihotCountVec(Mastic):
    """poc/mastic.py:607-614"""
    ID = 0xFFFF0005
    test_vec_name = "MasticMultihotCountVec"

    def __init__(self, bits: int, length: int, max_weight: int, chunk_length: int):
        super().__init__(bits, MultihotCountVec(Field128, length, max_weight, chunk_length))


def from_test_vec(tv: dict) -> Mastic:
    """Instantiate the Mastic variant a reference test vector was made with."""
    bits = tv["vidpf_bits"]
    if "max_measurement" in tv:
        return MasticSum(bits, tv["max_measurement"])
    if "max_weight" in tv:
        return MasticMultihotCountVec(bits, tv["length"], tv["max_weight"], tv["chunk_length"])
    if "bits" in tv:
        return MasticSumVec(bits, tv["length"], tv["bits"], tv["chunk_length"])
    if "length" in tv:
        return MasticHistogram(bits, tv["length"], tv["chunk_length"])
    return MasticCount(bits)
