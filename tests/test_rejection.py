"""Rejection sampling in next_vec (poc/vidpf.py:352-364 via vdaf_poc.xof
next_vec) on real data.  No reference vector reaches it; the
fixtures tests/golden/rejection_{f64,f128}.json (tests/rejection/make_fixture.py)
hold reports whose level-0 VIDPF node has a convert-stream candidate with top
word 0xffffffff: for Field64 (C2's Mastic(32, Sum 255)) a candidate >= p that
next_vec rejects, for Field128 (C4's Histogram circuit) the GPU fast path's
handover trigger.  CPU: the oracle reproduces the fixture and the candidate is
really there.  GPU: shard, prep_init of both aggregators (the level kernel
hands over to the exact stream by itself, nothing forced), decide and out
shares are bit-identical to the fixture."""
import json
import os

import pytest

from conftest import GOLDEN

FIXTURES = ["rejection_f64.json", "rejection_f128.json"]


def _load(name):
    return json.load(open(os.path.join(GOLDEN, name)))


def _oracle(fx):
    from oracle import mastic as om
    if fx["circuit"] == "MasticSum":
        return om.MasticSum(fx["bits"], 255)
    return om.MasticHistogram(fx["bits"], 64, 8)


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_has_the_candidate_and_oracle_reproduces_it(name):
    from oracle.dst import USAGE_CONVERT, dst
    from oracle.xof import XofFixedKeyAes128
    fx = _load(name)
    o = _oracle(fx)
    ctx, nonce = bytes.fromhex(fx["ctx"]), bytes.fromhex(fx["nonce"])
    rj = fx["rejection"]
    key0 = bytes.fromhex(rj["key0"])
    assert bytes.fromhex(fx["rand"])[:16] == key0
    (s, _t) = o.vidpf.extend(key0, ctx, nonce)
    xof = XofFixedKeyAes128(s[rj["child"]], dst(ctx, USAGE_CONVERT), nonce)
    xof.next(16)
    enc = o.field.ENCODED_SIZE
    raw = [int.from_bytes(xof.next(enc), "little") for _ in range(o.vidpf.VALUE_LEN)]
    c = raw[rj["candidate"]]
    assert c >> (8 * enc - 32) == 0xFFFFFFFF
    assert (c >= o.field.MODULUS) == rj["rejected"]
    if enc == 8:
        assert rj["rejected"], "the Field64 fixture must hold a rejected candidate"
        # next_vec skipped it: the node's payload is the candidates without it
        (_seed, w) = o.vidpf.convert(s[rj["child"]], ctx, nonce)
        want = [x for x in raw if x < o.field.MODULUS]
        assert [x.int() for x in w[:len(want)]] == want
    for r in fx["reports"]:
        alpha = tuple(bool(b) for b in r["alpha"])
        (cws, ins) = o.shard(ctx, (alpha, r["weight"]), nonce, bytes.fromhex(fx["rand"]))
        assert o.test_vec_encode_public_share(cws).hex() == r["public_share"]
        assert [o.test_vec_encode_input_share(x).hex() for x in ins] == r["input_shares"]
    vk = bytes.fromhex(fx["verify_key"])
    for p in fx["prep"]:
        ap = o.decode_agg_param(bytes.fromhex(p["agg_param"]))
        for (r, want) in zip(fx["reports"], p["reports"]):
            cws = o.vidpf.decode_public_share(bytes.fromhex(r["public_share"]))
            for a in range(2):
                isd = o.decode_input_share(a, bytes.fromhex(r["input_shares"][a]))
                (st, sh) = o.prep_init(vk, ctx, a, ap, nonce, cws, isd)
                assert o.test_vec_encode_prep_share(sh).hex() == want["prep_share_%d" % a]


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_gpu_matches_rejection_fixture(name):
    import mastic_amd
    fx = _load(name)
    if fx["circuit"] == "MasticSum":
        m = mastic_amd.MasticSum(fx["bits"], 255)
    else:
        m = mastic_amd.MasticHistogram(fx["bits"], 64, 8)
    ctx, nonce = bytes.fromhex(fx["ctx"]), bytes.fromhex(fx["nonce"])
    reps = fx["reports"]
    n = len(reps)
    # client shard on the GPU (k_shard's convert of the on-path child)
    (pub, in0, in1) = m.shard_batch(ctx, [tuple(bool(b) for b in r["alpha"]) for r in reps],
                                    [r["weight"] for r in reps], nonce * n, bytes.fromhex(fx["rand"]) * n)
    assert pub.hex() == "".join(r["public_share"] for r in reps)
    assert in0.hex() == "".join(r["input_shares"][0] for r in reps)
    assert in1.hex() == "".join(r["input_shares"][1] for r in reps)
    vk = bytes.fromhex(fx["verify_key"])
    for p in fx["prep"]:
        ap = bytes.fromhex(p["agg_param"])
        shares = []
        for a in range(2):
            (ps, _js, out, st) = m.prep_init_batch(vk, ctx, a, ap, nonce * n, pub, in0 if a == 0 else in1)
            assert list(st) == [0] * n
            assert ps.hex() == "".join(w["prep_share_%d" % a] for w in p["reports"])
            assert out.hex() == "".join(w["out_share_%d" % a] for w in p["reports"])
            shares.append(ps)
        (msgs, valid) = m.decide_batch(ctx, ap, shares[0], shares[1])
        assert list(valid) == [1] * n
        for (i, w) in enumerate(p["reports"]):
            if w["prep_msg"]:
                assert msgs[32 * i:32 * (i + 1)].hex() == w["prep_msg"]
