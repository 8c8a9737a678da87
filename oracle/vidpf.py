"""VIDPF (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates ``poc/vidpf.py`` (class ``Vidpf`` :84-470) with the same per-node
control flow: key generation ``gen`` (:103-211), evaluation with siblings
``eval_with_siblings`` (:213-261), ``get_beta_share`` (:263-279),
``eval_next`` (:281-325), ``extend`` (:330-350), ``convert`` (:352-364),
``node_proof`` (:366-380) and ``encode_public_share`` (:382-394).  Adds the
wire decoder the poc lacks (``decode_public_share``).
"""
import itertools
import random

from .common import (encode_path_msb_first, pack_bits, to_le_bytes, unpack_bits,
                     vec_add, vec_neg, vec_sub, xor)
from .dst import USAGE_CONVERT, USAGE_EXTEND, USAGE_NODE_PROOF, dst
from .xof import XofFixedKeyAes128, XofTurboShake128

PROOF_SIZE = 32


class Node:
    """One evaluated node of an aggregator's share of the prefix tree
    (PrefixTreeEntry, poc/vidpf.py:60-81)."""
    __slots__ = ("seed", "ctrl", "w", "proof", "left", "right")

    def __init__(self, seed, ctrl, w, proof):
        self.seed = seed
        self.ctrl = ctrl
        self.w = w
        self.proof = proof
        self.left = None
        self.right = None


def index_encode(path) -> bytes:
    """PrefixTreeIndex.encode (poc/vidpf.py:33-39): MSB-first bit packing."""
    return encode_path_msb_first(path)


class Vidpf:
    KEY_SIZE = XofFixedKeyAes128.SEED_SIZE
    NONCE_SIZE = XofFixedKeyAes128.SEED_SIZE
    RAND_SIZE = 2 * XofFixedKeyAes128.SEED_SIZE

    def __init__(self, field, bits: int, value_len: int):
        self.field = field
        self.BITS = bits
        self.VALUE_LEN = value_len

    # ------------------------------------------------------------ gen
    def gen(self, alpha, beta, ctx: bytes, nonce: bytes, rand: bytes):
        """poc/vidpf.py:103-211"""
        if len(alpha) != self.BITS:
            raise ValueError("alpha out of range")
        if len(beta) != self.VALUE_LEN:
            raise ValueError("incorrect beta length")
        if len(nonce) != self.NONCE_SIZE:
            raise ValueError("incorrect nonce size")
        if len(rand) != self.RAND_SIZE:
            raise ValueError("randomness has incorrect length")
        keys = [rand[:self.KEY_SIZE], rand[self.KEY_SIZE:]]
        seeds = list(keys)
        ctrls = [False, True]
        cws = []
        for i in range(self.BITS):
            bit = bool(alpha[i])
            keep = int(bit)
            lose = 1 - keep
            (s0, t0) = self.extend(seeds[0], ctx, nonce)
            (s1, t1) = self.extend(seeds[1], ctx, nonce)
            seed_cw = xor(s0[lose], s1[lose])
            ctrl_cw = [t0[0] ^ t1[0] ^ (not bit), t0[1] ^ t1[1] ^ bit]
            if ctrls[0]:
                s0[keep] = xor(s0[keep], seed_cw)
                t0[keep] ^= ctrl_cw[keep]
            if ctrls[1]:
                s1[keep] = xor(s1[keep], seed_cw)
                t1[keep] ^= ctrl_cw[keep]
            (seeds[0], w0) = self.convert(s0[keep], ctx, nonce)
            (seeds[1], w1) = self.convert(s1[keep], ctx, nonce)
            ctrls = [t0[keep], t1[keep]]
            w_cw = vec_add(vec_sub(beta, w0), w1)
            if ctrls[1]:
                w_cw = vec_neg(w_cw)
            path = tuple(alpha[:i + 1])
            proof_cw = xor(self.node_proof(seeds[0], ctx, path),
                           self.node_proof(seeds[1], ctx, path))
            cws.append((seed_cw, ctrl_cw, w_cw, proof_cw))
        return (cws, keys)

    # ----------------------------------------------------------- eval
    def eval_with_siblings(self, agg_id, cws, key, level, prefixes, ctx, nonce):
        """poc/vidpf.py:213-261"""
        if agg_id not in (0, 1):
            raise ValueError("invalid aggregator ID")
        if len(cws) != self.BITS:
            raise ValueError("corrections words has incorrect length")
        if not 0 <= level < self.BITS:
            raise ValueError("level too deep")
        for p in prefixes:
            if len(p) != level + 1:
                raise ValueError("prefix with incorrect length")
        if len(set(tuple(p) for p in prefixes)) != len(prefixes):
            raise ValueError("candidate prefixes are non-unique")
        root = Node(key, bool(agg_id), [], b"")
        out_share = []
        for prefix in prefixes:
            n = root
            for (i, bit) in enumerate(prefix):
                parent_path = tuple(prefix[:i])
                if n.left is None:
                    n.left = self.eval_next(n, cws[i], ctx, nonce, parent_path + (False,))
                if n.right is None:
                    n.right = self.eval_next(n, cws[i], ctx, nonce, parent_path + (True,))
                n = n.right if bit else n.left
            out_share.append(n.w if agg_id == 0 else vec_neg(n.w))
        return (out_share, root)

    def get_beta_share(self, agg_id, cws, key, ctx, nonce):
        """poc/vidpf.py:263-279"""
        root = Node(key, bool(agg_id), [], b"")
        l = self.eval_next(root, cws[0], ctx, nonce, (False,))
        r = self.eval_next(root, cws[0], ctx, nonce, (True,))
        share = vec_add(l.w, r.w)
        return vec_neg(share) if agg_id == 1 else share

    def eval_next(self, node, cw, ctx, nonce, path):
        """poc/vidpf.py:281-325"""
        (seed_cw, ctrl_cw, w_cw, proof_cw) = cw
        keep = int(bool(path[-1]))
        (s, t) = self.extend(node.seed, ctx, nonce)
        if node.ctrl:
            s[keep] = xor(s[keep], seed_cw)
            t[keep] ^= ctrl_cw[keep]
        (next_seed, w) = self.convert(s[keep], ctx, nonce)
        next_ctrl = t[keep]
        if next_ctrl:
            w = vec_add(w, w_cw)
        proof = self.node_proof(next_seed, ctx, path)
        if next_ctrl:
            proof = xor(proof, proof_cw)
        return Node(next_seed, next_ctrl, w, proof)

    def verify(self, proof0: bytes, proof1: bytes) -> bool:
        return proof0 == proof1

    def extend(self, seed, ctx, nonce):
        """poc/vidpf.py:330-350"""
        xof = XofFixedKeyAes128(seed, dst(ctx, USAGE_EXTEND), nonce)
        s = [bytearray(xof.next(self.KEY_SIZE)), bytearray(xof.next(self.KEY_SIZE))]
        t = [bool(s[0][0] & 1), bool(s[1][0] & 1)]
        s[0][0] &= 0xFE
        s[1][0] &= 0xFE
        return ([bytes(s[0]), bytes(s[1])], t)

    def convert(self, seed, ctx, nonce):
        """poc/vidpf.py:352-364"""
        xof = XofFixedKeyAes128(seed, dst(ctx, USAGE_CONVERT), nonce)
        next_seed = xof.next(XofFixedKeyAes128.SEED_SIZE)
        return (next_seed, xof.next_vec(self.field, self.VALUE_LEN))

    def node_proof(self, seed, ctx, path) -> bytes:
        """poc/vidpf.py:366-380"""
        binder = to_le_bytes(self.BITS, 2) + to_le_bytes(len(path) - 1, 2) + index_encode(path)
        return XofTurboShake128(seed, dst(ctx, USAGE_NODE_PROOF), binder).next(PROOF_SIZE)

    # ------------------------------------------------------- encoding
    def encode_public_share(self, cws) -> bytes:
        """poc/vidpf.py:382-394"""
        out = pack_bits(list(itertools.chain.from_iterable(cw[1] for cw in cws)))
        out += b"".join(cw[0] for cw in cws)
        out += b"".join(self.field.encode_vec(cw[2]) for cw in cws)
        out += b"".join(cw[3] for cw in cws)
        return out

    def public_share_size(self) -> int:
        return ((2 * self.BITS + 7) // 8 + self.BITS * (16 + PROOF_SIZE)
                + self.BITS * self.VALUE_LEN * self.field.ENCODED_SIZE)

    def decode_public_share(self, data: bytes):
        """Inverse of encode_public_share (the poc has no decoder)."""
        if len(data) != self.public_share_size():
            raise ValueError("public share has incorrect length")
        nb = (2 * self.BITS + 7) // 8
        ctrl = unpack_bits(data[:nb], 2 * self.BITS)
        pos = nb
        seeds = [data[pos + 16 * i: pos + 16 * (i + 1)] for i in range(self.BITS)]
        pos += 16 * self.BITS
        wlen = self.VALUE_LEN * self.field.ENCODED_SIZE
        ws = [self.field.decode_vec(data[pos + wlen * i: pos + wlen * (i + 1)])
              for i in range(self.BITS)]
        pos += wlen * self.BITS
        proofs = [data[pos + 32 * i: pos + 32 * (i + 1)] for i in range(self.BITS)]
        return [(seeds[i], [ctrl[2 * i], ctrl[2 * i + 1]], ws[i], proofs[i])
                for i in range(self.BITS)]

    # -------------------------------------------------------- helpers
    def is_prefix(self, x, y, level) -> bool:
        return tuple(x) == tuple(y[:level + 1])

    def test_input_rand(self):
        return tuple(bool(random.randrange(2)) for _ in range(self.BITS))

    def test_input_zero(self):
        return tuple([False] * self.BITS)

    def test_index_from_int(self, value: int, length: int):
        assert length <= self.BITS
        return tuple((value >> (length - 1 - i)) & 1 != 0 for i in range(length))

    def prefixes_for_level(self, level: int):
        return tuple(self.test_index_from_int(v, level + 1) for v in range(2 ** level))

    def test_eval(self, agg_id, cws, key, level, prefixes, ctx, nonce):
        """poc/vidpf.py:429-470: out shares + SHA3-256 over node proofs (BFS)."""
        import hashlib
        (out_share, root) = self.eval_with_siblings(agg_id, cws, key, level, prefixes, ctx, nonce)
        h = hashlib.sha3_256()
        for n in bfs_nodes(root):
            h.update(n.proof)
        return (out_share, h.digest())


def bfs_nodes(root):
    """Breadth-first order of every evaluated node below the root, the order
    the reference uses for its binders (poc/mastic.py:263-275)."""
    q = []
    if root.left is not None:
        q.append(root.left)
    if root.right is not None:
        q.append(root.right)
    i = 0
    while i < len(q):
        n = q[i]
        i += 1
        if n.left is not None:
            q.append(n.left)
        if n.right is not None:
            q.append(n.right)
    return q
