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


@pytest.mark.gpu
@pytest.mark.parametrize("force_slow", [None, 0, 3])
@pytest.mark.parametrize("name", FIXTURES)
def test_gpu_cache_hit_recomputes_rejected_parent(name, force_slow):
    """Frontier-cache hit over the fixture's rejected node: at level 1 both
    level-0 nodes are parents, and the cached call recomputes each parent's
    payload from its cached convert seed -- for report B through the real
    rejection (the exact next_vec stream), and with the force_slow_blk test
    hook (mastic_set_test_hooks) through a forced handover at a payload block.  Prep shares and out shares
    of the hit equal a context without the cache and the oracle."""
    import mastic_amd
    fx = _load(name)

    def mk():
        if fx["circuit"] == "MasticSum":
            return mastic_amd.MasticSum(fx["bits"], 255)
        return mastic_amd.MasticHistogram(fx["bits"], 64, 8)
    m_on, m_off = mk(), mk()
    if force_slow is not None:
        for m in (m_on, m_off):
            m.set_test_hooks(force_slow_blk=force_slow)
    m_on.set_frontier_cache(True)
    o = _oracle(fx)
    ctx, nonce = bytes.fromhex(fx["ctx"]), bytes.fromhex(fx["nonce"])
    reps = fx["reports"]
    n = len(reps)
    pub = bytes.fromhex("".join(r["public_share"] for r in reps))
    ins = [bytes.fromhex("".join(r["input_shares"][a] for r in reps)) for a in range(2)]
    dev_on = m_on.reports_upload(nonce * n, pub, ins[0], ins[1])
    dev_off = m_off.reports_upload(nonce * n, pub, ins[0], ins[1])
    vk = bytes.fromhex(fx["verify_key"])
    F, T = False, True
    ap0 = (0, ((F,), (T,)), False)
    ap1 = (1, ((F, F), (F, T), (T, F), (T, T)), False)
    for agg_id in range(2):
        for ap in (ap0, ap1):
            m_on.prep_init_device(dev_on, vk, ctx, agg_id, ap)
            m_off.prep_init_device(dev_off, vk, ctx, agg_id, ap)
            a = m_on.prep_result(dev_on, agg_id, ap, want_out_shares=True)
            b = m_off.prep_result(dev_off, agg_id, ap, want_out_shares=True)
            if ap is ap1:
                assert m_on.last_prep_was_cached(), "level 1 should extend the cached level-0 tree"
            assert a[0] == b[0] and a[2] == b[2], (ap[0], agg_id)
            psz = len(a[0]) // n
            for (i, r) in enumerate(reps):
                cws = o.vidpf.decode_public_share(bytes.fromhex(r["public_share"]))
                isd = o.decode_input_share(agg_id, bytes.fromhex(r["input_shares"][agg_id]))
                (_st, sh) = o.prep_init(vk, ctx, agg_id, ap, nonce, cws, isd)
                assert a[0][psz * i:psz * (i + 1)] == o.test_vec_encode_prep_share(sh), (ap[0], agg_id, i)
