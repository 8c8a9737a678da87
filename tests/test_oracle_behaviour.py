"""Behavioural tests of the CPU oracle, re-expressing the reference's own unit
tests (poc/tests/test_vidpf.py, poc/tests/test_mastic.py) so the oracle is
pinned by behaviour as well as by the golden bytes."""
import os
import random

import pytest

from oracle.common import vec_add
from oracle.field import Field64, Field128
from oracle.mastic import MasticCount, MasticSum, MasticSumVec
from oracle.vidpf import Vidpf

CTX = b"some application"


def _rand(n, rng):
    return bytes(rng.getrandbits(8) for _ in range(n))


def run_vdaf(mastic, agg_param, measurements, rng):
    """In-process shard -> prep -> aggregate -> unshard (vdaf_poc.test_utils
    run_vdaf semantics, used by poc/tests/test_mastic.py:178-337)."""
    vk = _rand(mastic.VERIFY_KEY_SIZE, rng)
    agg = [mastic.agg_init(agg_param) for _ in range(2)]
    for meas in measurements:
        nonce = _rand(16, rng)
        (cws, ins) = mastic.shard(CTX, meas, nonce, _rand(mastic.RAND_SIZE, rng))
        states, shares = zip(*[mastic.prep_init(vk, CTX, a, agg_param, nonce, cws, ins[a])
                               for a in range(2)])
        msg = mastic.prep_shares_to_prep(CTX, agg_param, list(shares))
        for a in range(2):
            agg[a] = mastic.agg_update(agg_param, agg[a], mastic.prep_next(CTX, states[a], msg))
    return mastic.unshard(agg_param, agg, len(measurements))


def test_is_valid_truth_table():
    """poc/tests/test_mastic.py:11-68"""
    m = MasticCount(4)
    assert m.is_valid((0, ((False,),), True), [])
    assert m.is_valid((2, ((True, False, False),), True), [])
    assert not m.is_valid((0, ((False,),), False), [])
    assert m.is_valid((1, ((False, True),), False), [(0, ((False,),), True)])
    assert not m.is_valid((1, ((False, True),), True), [(0, ((False,),), True)])
    assert not m.is_valid((1, ((False, True),), True), [(0, ((False,),), False)])
    assert not m.is_valid((1, ((True, False),), False), [(0, ((False,),), False)])
    assert not m.is_valid((1, ((True, False),), False), [(2, ((True, False, False),), True)])


def test_end_to_end_count_and_sum():
    """poc/tests/test_mastic.py:179-337 (Count / Sum / SumVec cases)."""
    rng = random.Random(1)
    m = MasticCount(2)
    ix = m.vidpf.test_index_from_int
    meas = [(ix(0b10, 2), 1), (ix(0b00, 2), 1), (ix(0b11, 2), 1), (ix(0b01, 2), 1), (ix(0b11, 2), 1)]
    assert run_vdaf(m, (0, (ix(0, 1), ix(1, 1)), True), meas, rng) == [2, 3]
    m = MasticSum(2, 3)
    meas = [(ix(0b10, 2), 1), (ix(0b00, 2), 2), (ix(0b11, 2), 3), (ix(0b01, 2), 0), (ix(0b11, 2), 3)]
    assert run_vdaf(m, (1, (ix(0b00, 2), ix(0b01, 2), ix(0b11, 2)), True), meas, rng) == [2, 0, 6]
    m = MasticSumVec(16, 3, 2, 3)
    ix = m.vidpf.test_index_from_int
    meas = [(ix(0b1111000011110000, 16), [0, 2, 1]), (ix(0b1111000011110001, 16), [1, 3, 0]),
            (ix(0b0111000011110000, 16), [3, 3, 3])]
    assert run_vdaf(m, (14, (ix(0b111100001111000, 15),), True), meas, rng) == [[1, 5, 1]]


def test_vidpf_eval_invariants():
    """poc/tests/test_vidpf.py:12-62: on-path seeds differ / ctrl shares of one;
    off-path seeds equal / ctrl shares of zero; node proofs always agree."""
    from oracle.vidpf import Node
    rng = random.Random(2)
    v = Vidpf(Field128, 5, 1)
    nonce = _rand(16, rng)
    alpha = tuple(bool(rng.getrandbits(1)) for _ in range(5))
    (pub, keys) = v.gen(alpha, [Field128(1)], CTX, nonce, _rand(32, rng))
    for on_path in (True, False):
        nodes = [Node(keys[0], False, [], b""), Node(keys[1], True, [], b"")]
        for i in range(5):
            path = alpha[:i + 1] if on_path else alpha[:i] + (not alpha[i],)
            nodes = [v.eval_next(nodes[a], pub[i], CTX, nonce, path) for a in range(2)]
            assert (nodes[0].seed != nodes[1].seed) == on_path
            assert (nodes[0].ctrl != nodes[1].ctrl) == on_path
            assert nodes[0].proof == nodes[1].proof
            if not on_path:
                break


def test_vidpf_exhaustive_small():
    """poc/tests/test_vidpf.py:155-191 style: every prefix of every level."""
    rng = random.Random(3)
    v = Vidpf(Field64, 4, 2)
    nonce = _rand(16, rng)
    alpha = (True, False, True, True)
    beta = [Field64(1), Field64(7)]
    (pub, keys) = v.gen(alpha, beta, CTX, nonce, _rand(32, rng))
    for level in range(4):
        prefixes = v.prefixes_for_level(level)
        outs, proofs = [], []
        for a in range(2):
            (o, pf) = v.test_eval(a, pub, keys[a], level, prefixes, CTX, nonce)
            outs.append(o)
            proofs.append(pf)
        assert proofs[0] == proofs[1]
        for (p, x, y) in zip(prefixes, outs[0], outs[1]):
            want = beta if v.is_prefix(p, alpha, level) else [Field64(0)] * 2
            assert vec_add(x, y) == want


@pytest.mark.parametrize("tweak", ["counter", "weight"])
def test_malformed_payload_rejected(tweak):
    """poc/tests/test_mastic.py:71-175: a tweaked CW payload breaks the eval
    proof from the tweaked level on (the weight tweak at level 0 only from
    level 1, because the payload check needs interior nodes)."""
    rng = random.Random(4)
    bits = 5
    m = MasticCount(bits)
    vk = _rand(32, rng)
    nonce = _rand(16, rng)
    (pub, ins) = m.shard(CTX, ((True,) * bits, True), nonce, _rand(m.RAND_SIZE, rng))
    bad_level = 2
    (s, c, w, pf) = pub[bad_level]
    w = list(w)
    w[0 if tweak == "counter" else 1] += Field64(1)
    pub = list(pub)
    pub[bad_level] = (s, c, w, pf)
    for level in range(bits):
        ap = (level, ((True,) * (level + 1),), False)
        shares = [m.prep_init(vk, CTX, a, ap, nonce, pub, ins[a])[1] for a in range(2)]
        if level < bad_level:
            m.prep_shares_to_prep(CTX, ap, shares)
        else:
            with pytest.raises(Exception):
                m.prep_shares_to_prep(CTX, ap, shares)
