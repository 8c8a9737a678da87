"""Parity of the HIP path (through the C ABI) with the CPU oracle and the
reference's golden vectors.  Bit-exact everywhere: all of this is integer,
byte and GF(p) arithmetic.

Sizes: the golden vectors; random reports for every circuit at sizes the
oracle finishes in seconds; the C2 bench shape (BITS 32, Sum 255) with a
large prefix set checked through size-independent properties plus one report
replayed in the oracle.
"""
import json
import os
import random

import pytest

from conftest import golden_files

pytestmark = pytest.mark.gpu

CTX = b"some application"


@pytest.fixture(scope="module")
def mastic_amd():
    import mastic_amd
    from mastic_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libmastic_hip.so missing: build() was not run")
    try:
        mastic_amd.MasticCount(2)
    except _lib.MasticError as e:
        if e.code == -19:
            pytest.skip("no gfx950 device")
        raise
    return mastic_amd


def _oracle_for(m):
    from oracle import mastic as om
    c = m.circuit
    if c == "Count":
        return om.MasticCount(m.BITS)
    if c == "Sum":
        return om.MasticSum(m.BITS, m.max_measurement)
    if c == "SumVec":
        return om.MasticSumVec(m.BITS, m.length, m.sum_vec_bits, m.chunk_length)
    if c == "Histogram":
        return om.MasticHistogram(m.BITS, m.length, m.chunk_length)
    return om.MasticMultihotCountVec(m.BITS, m.length, m.max_measurement, m.chunk_length)


# ------------------------------------------------------------ golden vectors
@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_golden_vector_on_gpu(mastic_amd, path):
    tv = json.load(open(path))
    m = mastic_amd.from_test_vec(tv)
    ctx = bytes.fromhex(tv["ctx"])
    vk = bytes.fromhex(tv["verify_key"])
    ap = m.decode_agg_param(bytes.fromhex(tv["agg_param"]))
    reps = tv["prep"]
    # client shard on the GPU
    alphas = [tuple(r["measurement"][0]) for r in reps]
    weights = [r["measurement"][1] for r in reps]
    nonces = b"".join(bytes.fromhex(r["nonce"]) for r in reps)
    rands = b"".join(bytes.fromhex(r["rand"]) for r in reps)
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rands)
    assert pub == b"".join(bytes.fromhex(r["public_share"]) for r in reps)
    assert in0 == b"".join(bytes.fromhex(r["input_shares"][0]) for r in reps)
    assert in1 == b"".join(bytes.fromhex(r["input_shares"][1]) for r in reps)
    # prep_init, both aggregators
    shares = []
    for a in range(2):
        ins = in0 if a == 0 else in1
        (ps, js, out, st) = m.prep_init_batch(vk, ctx, a, ap, nonces, pub, ins)
        assert list(st) == [0] * len(reps)
        assert ps == b"".join(bytes.fromhex(r["prep_shares"][0][a]) for r in reps)
        want_out = b"".join(b"".join(bytes.fromhex(x) for x in r["out_shares"][a]) for r in reps)
        assert out == want_out
        shares.append(ps)
        agg = m.aggregate_device(a, ap)
        assert m.test_vec_encode_agg_share(agg).hex() == tv["agg_shares"][a]
    (msgs, valid) = m.decide_batch(ctx, ap, shares[0], shares[1])
    assert list(valid) == [1] * len(reps)
    for (i, r) in enumerate(reps):
        if r["prep_messages"][0]:
            assert msgs[32 * i:32 * (i + 1)].hex() == r["prep_messages"][0]
    aggs = [m.aggregate_device(a, ap) for a in range(2)]
    assert m.unshard(ap, aggs, len(reps)) == tv["agg_result"]


def test_reference_shaped_api_one_report(mastic_amd):
    """The per-report methods mirror poc/mastic.py and agree with the oracle."""
    tv = json.load(open(golden_files()[4]))  # MasticHistogram_0
    m = mastic_amd.from_test_vec(tv)
    o = _oracle_for(m)
    ctx = bytes.fromhex(tv["ctx"])
    vk = bytes.fromhex(tv["verify_key"])
    ap = m.decode_agg_param(bytes.fromhex(tv["agg_param"]))
    rep = tv["prep"][0]
    meas = (tuple(rep["measurement"][0]), rep["measurement"][1])
    nonce = bytes.fromhex(rep["nonce"])
    rand = bytes.fromhex(rep["rand"])
    (cws, ins) = m.shard(ctx, meas, nonce, rand)
    (ocws, oins) = o.shard(ctx, meas, nonce, rand)
    assert m.encode_public_share(cws) == o.test_vec_encode_public_share(ocws)
    states, shares = [], []
    for a in range(2):
        (st, sh) = m.prep_init(vk, ctx, a, ap, nonce, cws, ins[a])
        (ost, osh) = o.prep_init(vk, ctx, a, ap, nonce, ocws, oins[a])
        assert m.test_vec_encode_prep_share(sh) == o.test_vec_encode_prep_share(osh)
        assert [x.int() for x in st[0]] == [x.int() for x in ost[0]]
        assert st[1] == ost[1]
        states.append(st)
        shares.append(sh)
    msg = m.prep_shares_to_prep(ctx, ap, shares)
    assert msg == o.prep_shares_to_prep(ctx, ap, [o.decode_prep_share(True, m.test_vec_encode_prep_share(s))
                                                  for s in shares])
    outs = [m.prep_next(ctx, states[a], msg) for a in range(2)]
    assert m.unshard(ap, outs, 1) == o.unshard(ap, [[o.field(x.int()) for x in y] for y in outs], 1)


# ------------------------------------------------------------ random parity
def _random_reports(m, rng, n):
    alphas, weights = [], []
    for _ in range(n):
        alphas.append(tuple(bool(rng.getrandbits(1)) for _ in range(m.BITS)))
        c = m.circuit
        if c == "Count":
            weights.append(rng.randrange(2))
        elif c == "Sum":
            weights.append(rng.randrange(m.max_measurement + 1))
        elif c == "SumVec":
            weights.append([rng.randrange(2 ** m.sum_vec_bits) for _ in range(m.length)])
        elif c == "Histogram":
            weights.append(rng.randrange(m.length))
        else:
            k = rng.randrange(m.max_measurement + 1)
            idx = set(rng.sample(range(m.length), k))
            weights.append([i in idx for i in range(m.length)])
    nonces = bytes(rng.getrandbits(8) for _ in range(16 * n))
    rands = bytes(rng.getrandbits(8) for _ in range(m.RAND_SIZE * n))
    return alphas, weights, nonces, rands


def _random_agg_param(m, rng, alphas, level, nprefix, weight_check):
    cand = set(tuple(a[:level + 1]) for a in alphas)
    while len(cand) < nprefix and len(cand) < 2 ** (level + 1):
        cand.add(tuple(bool(rng.getrandbits(1)) for _ in range(level + 1)))
    pre = list(cand)[:nprefix]
    rng.shuffle(pre)
    return (level, tuple(pre), weight_check)


def _check_against_oracle(m, o, ctx, vk, ap, alphas, weights, nonces, rands, check_shard=True):
    n = len(alphas)
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rands)
    ps_sz, is_sz = m.public_share_size(), [m.input_share_size(0), m.input_share_size(1)]
    gpu = {}
    for a in range(2):
        gpu[a] = m.prep_init_batch(vk, ctx, a, ap, nonces, pub, in0 if a == 0 else in1)
        assert list(gpu[a][3]) == [0] * n
    oshares = [[], []]
    for i in range(n):
        nonce = nonces[16 * i:16 * (i + 1)]
        meas = (alphas[i], weights[i])
        if check_shard:
            (ocws, oins) = o.shard(ctx, meas, nonce, rands[m.RAND_SIZE * i:m.RAND_SIZE * (i + 1)])
            assert o.test_vec_encode_public_share(ocws) == pub[ps_sz * i:ps_sz * (i + 1)]
            assert o.test_vec_encode_input_share(oins[0]) == in0[is_sz[0] * i:is_sz[0] * (i + 1)]
            assert o.test_vec_encode_input_share(oins[1]) == in1[is_sz[1] * i:is_sz[1] * (i + 1)]
        else:
            ocws = o.vidpf.decode_public_share(pub[ps_sz * i:ps_sz * (i + 1)])
            oins = [o.decode_input_share(0, in0[is_sz[0] * i:is_sz[0] * (i + 1)]),
                    o.decode_input_share(1, in1[is_sz[1] * i:is_sz[1] * (i + 1)])]
        for a in range(2):
            (ost, osh) = o.prep_init(vk, ctx, a, ap, nonce, ocws, oins[a])
            enc = o.test_vec_encode_prep_share(osh)
            (ps, js, out, _st) = gpu[a]
            assert ps[len(enc) * i:len(enc) * (i + 1)] == enc, "prep share %d agg %d" % (i, a)
            ow = len(out) // n
            assert out[ow * i:ow * (i + 1)] == o.field.encode_vec(ost[0]), "out share %d agg %d" % (i, a)
            if ost[1] is not None:
                assert js[32 * i:32 * (i + 1)] == ost[1]
            oshares[a].append(enc)
    (msgs, valid) = m.decide_batch(ctx, ap, gpu[0][0], gpu[1][0])
    assert list(valid) == [1] * n
    for i in range(n):
        omsg = o.prep_shares_to_prep(ctx, ap, [o.decode_prep_share(ap[2], oshares[a][i]) for a in range(2)])
        if omsg is not None:
            assert msgs[32 * i:32 * (i + 1)] == omsg
    return gpu


CASES = [
    ("Count", dict(bits=6)),
    ("Sum", dict(bits=5, max_measurement=13)),
    ("SumVec", dict(bits=4, length=5, sum_vec_bits=3, chunk_length=4)),
    ("Histogram", dict(bits=5, length=7, chunk_length=3)),
    ("MultihotCountVec", dict(bits=4, length=6, max_measurement=3, chunk_length=2)),
]


@pytest.mark.parametrize("circuit,kw", CASES, ids=[c for (c, _) in CASES])
def test_random_reports_match_oracle(mastic_amd, circuit, kw):
    rng = random.Random(sum(map(ord, circuit)))
    kw = dict(kw)
    bits = kw.pop("bits")
    m = mastic_amd.Mastic(bits, circuit, **kw)
    o = _oracle_for(m)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 5)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    for (level, nprefix, wc) in [(0, 2, True), (bits - 1, 6, True), (bits // 2, 3, False)]:
        ap = _random_agg_param(m, rng, alphas, level, nprefix, wc)
        _check_against_oracle(m, o, CTX, vk, ap, alphas, weights, nonces, rands, check_shard=(level == 0))


def test_long_context_string(mastic_amd):
    """A ctx longer than one TurboSHAKE block moves every sponge prefix over a
    block boundary (prefix states with full blocks absorbed)."""
    rng = random.Random(7)
    m = mastic_amd.MasticSum(4, 5)
    o = _oracle_for(m)
    ctx = bytes(rng.getrandbits(8) for _ in range(301))
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 3)
    vk = bytes(range(32))
    ap = _random_agg_param(m, rng, alphas, 3, 4, True)
    _check_against_oracle(m, o, ctx, vk, ap, alphas, weights, nonces, rands)


@pytest.mark.parametrize("vk_len", [16, 17, 0, 255])
def test_verify_key_lengths(mastic_amd, vk_len):
    """The verify key is XofTurboShake128's length-prefixed seed
    (mastic.py:302-306,499-510): the reference driver passes 16 bytes
    (examples.py:38,176).  Eval proofs and query randomness (FLP verifier
    shares of a Sum circuit) must match the oracle for any length."""
    rng = random.Random(40 + vk_len)
    m = mastic_amd.MasticSum(5, 13)
    o = _oracle_for(m)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 3)
    vk = bytes(rng.getrandbits(8) for _ in range(vk_len))
    for (level, nprefix, wc) in [(0, 2, True), (4, 5, False)]:
        ap = _random_agg_param(m, rng, alphas, level, nprefix, wc)
        _check_against_oracle(m, o, CTX, vk, ap, alphas, weights, nonces, rands, check_shard=False)


def test_verify_key_too_long_rejected(mastic_amd):
    m = mastic_amd.MasticCount(3)
    ap = (0, ((False,), (True,)), True)
    with pytest.raises(ValueError):
        m.prep_init_batch(bytes(256), CTX, 0, ap, bytes(16), bytes(m.public_share_size()),
                          bytes(m.input_share_size(0)))


def test_empty_ctx_and_single_prefix(mastic_amd):
    rng = random.Random(8)
    m = mastic_amd.MasticCount(3)
    o = _oracle_for(m)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 2)
    ap = (2, (alphas[0],), True)
    _check_against_oracle(m, o, b"", bytes(32), ap, alphas, weights, nonces, rands)


@pytest.mark.parametrize("chunk_groups,n", [(1, 150), (4, 600)], ids=["64-report chunks", "pipelined halves"])
def test_chunked_batches_equal_unchunked(mastic_amd, chunk_groups, n):
    """Reports processed in several HBM-budget chunks give identical results
    (with >= 128-report chunks the chunks are pipelined through the two halves
    of the work arena, their tails on the sponge stream)."""
    rng = random.Random(9)
    m = mastic_amd.MasticCount(8)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, n)
    (pub, in0, _in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    ap = _random_agg_param(m, rng, alphas, 7, 20, True)
    vk = bytes(32)
    full = m.prep_init_batch(vk, CTX, 0, ap, nonces, pub, in0)
    agg_full = m.aggregate_device(0, ap)
    import ctypes
    from mastic_amd import _lib
    enc = m.encode_agg_param(ap)
    per = ctypes.c_uint64()
    assert _lib.lib().mastic_work_bytes(m._ctx, enc, len(enc), ctypes.byref(per)) == 0
    try:
        # -> 64-report chunks, or 256-report chunks pipelined as 128-report halves
        _lib.lib().mastic_set_memory_budget(m._ctx, (64 * chunk_groups + 64) * per.value + 1000)
        m2 = m.prep_init_batch(vk, CTX, 0, ap, nonces, pub, in0)
    finally:
        _lib.lib().mastic_set_memory_budget(m._ctx, 0)
    assert m2[0] == full[0] and m2[2] == full[2]
    assert m.aggregate_device(0, ap) == agg_full


def test_chunked_field128_large_rows_equal_unchunked_and_oracle(mastic_amd):
    """Field128 with rows of >= 16 KB to unpack per report (SumVec(64) to
    level 15: 16 x 1,088 B of correction words -- the coalesced row-tile
    unpack, k_rows_to_planes), a weight check (the FLP on its own stream beside
    the last sponges) and 256-report chunks pipelined as 128-report halves
    (their tails on the sponge streams): prep shares and out shares of both
    aggregators equal the unchunked call's, and sampled reports equal the
    oracle's."""
    import ctypes
    from mastic_amd import _lib
    rng = random.Random(21)
    m = mastic_amd.MasticSumVec(32, 64, 1, 8)
    o = _oracle_for(m)
    n = 600
    (alphas, weights, nonces, rands) = _random_reports(m, rng, n)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    ap = _random_agg_param(m, rng, alphas, 15, 24, True)
    vk = bytes(range(32))
    enc = m.encode_agg_param(ap)
    per = ctypes.c_uint64()
    assert _lib.lib().mastic_work_bytes(m._ctx, enc, len(enc), ctypes.byref(per)) == 0
    psz, isz = m.public_share_size(), [m.input_share_size(0), m.input_share_size(1)]
    for a in range(2):
        ins = in0 if a == 0 else in1
        full = m.prep_init_batch(vk, CTX, a, ap, nonces, pub, ins)
        try:
            _lib.lib().mastic_set_memory_budget(m._ctx, (64 * 4 + 64) * per.value + 1000)
            chunked = m.prep_init_batch(vk, CTX, a, ap, nonces, pub, ins)
        finally:
            _lib.lib().mastic_set_memory_budget(m._ctx, 0)
        assert chunked[0] == full[0] and chunked[2] == full[2], "agg %d" % a
        assert list(chunked[3]) == list(full[3])
        pss = m.prep_share_size(True)
        osz = len(full[2]) // n
        for i in (0, 301, n - 1):  # first chunk, second chunk (other arena half), last (partial) chunk
            cw = o.vidpf.decode_public_share(pub[psz * i:psz * (i + 1)])
            ish = o.decode_input_share(a, ins[isz[a] * i:isz[a] * (i + 1)])
            (ost, osh) = o.prep_init(vk, CTX, a, ap, nonces[16 * i:16 * (i + 1)], cw, ish)
            assert chunked[0][pss * i:pss * (i + 1)] == o.test_vec_encode_prep_share(osh), "agg %d report %d" % (a, i)
            assert chunked[2][osz * i:osz * (i + 1)] == o.field.encode_vec(ost[0]), "agg %d report %d" % (a, i)


def test_malformed_payload_correction_word_detected(mastic_amd):
    """poc/tests/test_mastic.py:126-175: tweak a payload CW -> eval proofs differ."""
    rng = random.Random(10)
    m = mastic_amd.MasticCount(5)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 4)
    alphas[0] = (True,) * 5
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    bad_level = 2
    cws = m.decode_public_share(pub[:m.public_share_size()])
    (s, c, w, p) = cws[bad_level]
    w = list(w)
    w[1] = w[1] + m.field(1)
    cws[bad_level] = (s, c, w, p)
    pub = m.encode_public_share(cws) + pub[m.public_share_size():]
    vk = bytes(32)
    for level in range(5):
        ap = (level, ((True,) * (level + 1),), False)
        sh = [m.prep_init_batch(vk, CTX, a, ap, nonces, pub, in0 if a == 0 else in1)[0] for a in range(2)]
        (_msgs, valid) = m.decide_batch(CTX, ap, sh[0], sh[1])
        assert valid[0] == (1 if level < bad_level else 0)
        assert list(valid[1:]) == [1, 1, 1]


def test_invalid_weight_rejected_by_flp(mastic_amd):
    """A client that encodes an out-of-range weight fails the FLP decide."""
    rng = random.Random(11)
    m = mastic_amd.MasticSum(3, 3)  # b = 2 bits
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 2)
    F = m.field
    bad = [F(1), F(1), F(0), F(1)]   # 3 with inconsistent offset bits
    ok = m.encode_measurement(2)
    ab = bytes([(sum(int(b) << (7 - i) for (i, b) in enumerate(a[:8]))) & 0xff for a in alphas])
    betas = F.encode_vec(bad) + F.encode_vec(ok)
    (pub, in0, in1) = m.shard_encoded(CTX, 2, ab, betas, nonces, rands)
    ap = (0, ((False,), (True,)), True)
    sh = [m.prep_init_batch(bytes(32), CTX, a, ap, nonces, pub, in0 if a == 0 else in1)[0] for a in range(2)]
    (_msgs, valid) = m.decide_batch(CTX, ap, sh[0], sh[1])
    assert list(valid) == [2, 1]


def test_errors_mirror_reference(mastic_amd):
    m = mastic_amd.MasticCount(4)
    with pytest.raises(ValueError):
        m.tree_stats(m.encode_agg_param((4, ((True,) * 5,), True)))          # level too deep
    with pytest.raises(ValueError):
        m.tree_stats(m.encode_agg_param((1, ((True, False), (True, False)), True)))  # non-unique


# ------------------------------------------------------------ full size
def test_c2_shape_properties_and_oracle_sample(mastic_amd):
    """BASELINE config C2 shape: Mastic(32, Sum 255), level 31, 2000 candidate
    prefixes (the bench uses 10k).  Size-independent checks over 128 reports:
    both aggregators' eval proofs agree, FLP decides every report valid, and
    the aggregate equals the plaintext functionality (talks/func.py:49-80).
    One report is replayed in the CPU oracle at full tree size."""
    rng = random.Random(12)
    m = mastic_amd.MasticSum(32, 255)
    attrs = [tuple(bool(rng.getrandbits(1)) for _ in range(32)) for _ in range(2000)]
    attrs = list(dict.fromkeys(attrs))
    n = 128
    alphas = [attrs[rng.randrange(len(attrs))] for _ in range(n)]
    weights = [rng.randrange(256) for _ in range(n)]
    nonces = bytes(rng.getrandbits(8) for _ in range(16 * n))
    rands = bytes(rng.getrandbits(8) for _ in range(m.RAND_SIZE * n))
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    ap = (31, tuple(sorted(attrs)), True)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    res = [m.prep_init_batch(vk, CTX, a, ap, nonces, pub, in0 if a == 0 else in1, want_out_shares=False)
           for a in range(2)]
    (_msgs, valid) = m.decide_batch(CTX, ap, res[0][0], res[1][0])
    assert list(valid) == [1] * n
    aggs = [m.aggregate_device(a, ap) for a in range(2)]
    result = m.unshard(ap, aggs, n)
    want = {}
    for (a, w) in zip(alphas, weights):
        want[a] = want.get(a, 0) + w
    assert result == [want.get(p, 0) for p in ap[1]]
    # reports of both 64-report groups through the oracle at full size (the
    # binder buffers are tiled per report group)
    o = _oracle_for(m)
    psz, isz = m.public_share_size(), m.input_share_size(1)
    for i in (0, 100):
        cws = o.vidpf.decode_public_share(pub[psz * i:psz * (i + 1)])
        isd = o.decode_input_share(1, in1[isz * i:isz * (i + 1)])
        (_st, sh) = o.prep_init(vk, CTX, 1, ap, nonces[16 * i:16 * (i + 1)], cws, isd)
        enc = o.test_vec_encode_prep_share(sh)
        assert res[1][0][len(enc) * i:len(enc) * (i + 1)] == enc, "report %d" % i


@pytest.mark.parametrize("blk", [0, 1, 4, 8])
def test_fast_path_handover_to_exact_stream(mastic_amd, blk):
    """The Field64 level kernel speculates that no next_vec candidate is
    rejected and hands over to the exact rejection-sampling stream when one
    might be (probability 2^-32 per candidate, never hit by random tests).
    Force the handover at block `blk` and check every output against the
    oracle: elements before the handover come from the fast path, the rest
    from the exact stream."""
    rng = random.Random(100 + blk)
    m = mastic_amd.MasticSum(6, 255)  # VALUE_LEN 17: 9 payload blocks per node
    m.set_test_hooks(force_slow_blk=blk)
    o = _oracle_for(m)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 4)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    ap = _random_agg_param(m, rng, alphas, 5, 5, True)
    _check_against_oracle(m, o, CTX, vk, ap, alphas, weights, nonces, rands, check_shard=False)


@pytest.mark.parametrize("blk", [0, 2, 6])
def test_fast_path_handover_field128(mastic_amd, blk):
    """Same handover for the Field128 fast path (one candidate per block; a
    candidate >= p has its top word 0xffffffff)."""
    rng = random.Random(200 + blk)
    m = mastic_amd.MasticHistogram(5, 7, 3)  # VALUE_LEN 8: 8 payload blocks per node
    m.set_test_hooks(force_slow_blk=blk)
    o = _oracle_for(m)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 4)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    ap = _random_agg_param(m, rng, alphas, 4, 5, True)
    _check_against_oracle(m, o, CTX, vk, ap, alphas, weights, nonces, rands, check_shard=False)


# ------------------------------------------------------------ edge cases
def test_empty_batch(mastic_amd):
    """Zero reports: empty outputs and an all-zero aggregate (agg_init)."""
    m = mastic_amd.MasticSum(6, 7)
    ap = (5, ((True,) * 6, (False,) * 6), True)
    (ps, js, out, st) = m.prep_init_batch(bytes(32), CTX, 0, ap, b"", b"", b"")
    assert ps == b"" and len(st) == 0
    agg = m.aggregate_device(0, ap)
    assert [x.int() for x in agg] == [0] * (2 * (1 + m.OUTPUT_LEN))


def test_empty_sharded_batch_and_view(mastic_amd):
    """A device batch sharded from zero reports (a rank of a split job that
    gets none) and a zero-report view of it run prep_init for both
    aggregators, decide and fold like any other batch."""
    m = mastic_amd.MasticSum(6, 7)
    ap = (5, ((True,) * 6, (False,) * 6), True)
    dev = m.reports_shard(CTX, b"", b"", b"", b"")
    assert dev.n == 0
    for batch in (dev, dev.view(0, 0)):
        for agg_id in range(2):
            m.prep_init_device(batch, bytes(16), CTX, agg_id, ap)
            (ps, _js, out, st) = m.prep_result(batch, agg_id, ap, want_out_shares=True)
            assert ps == b"" and out == b"" and len(st) == 0
        (acc, _codes) = m.decide_results(CTX, 0)
        assert len(acc) == 0
        agg = m.aggregate_device(1, ap)
        assert [x.int() for x in agg] == [0] * (2 * (1 + m.OUTPUT_LEN))


def test_empty_prefix_list_rejected(mastic_amd):
    """The poc cannot evaluate an empty candidate set (mastic.py:270 reads the
    root's unset children); the GPU path refuses it with ValueError."""
    rng = random.Random(21)
    m = mastic_amd.MasticCount(4)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 2)
    (pub, in0, _in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    for level in (0, 3):
        with pytest.raises(ValueError):
            m.prep_init_batch(bytes(32), CTX, 0, (level, (), True), nonces, pub, in0)


@pytest.mark.parametrize("n", [1, 63, 65])
def test_ragged_batch_sizes(mastic_amd, n):
    """Batches that do not fill whole 64-report groups: every report of the
    batch bit-exact against the oracle (padding lanes must not leak)."""
    rng = random.Random(300 + n)
    m = mastic_amd.MasticSum(5, 3)
    o = _oracle_for(m)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, n)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    ap = _random_agg_param(m, rng, alphas, 4, 6, True)
    _check_against_oracle(m, o, CTX, vk, ap, alphas, weights, nonces, rands, check_shard=(n == 1))


def test_max_bits_many_prefixes_properties(mastic_amd):
    """BITS 256 (the largest BASELINE config) at level 255 with 512 candidates:
    both aggregators agree (decide), and the aggregate equals the plaintext
    counts (talks/func.py:49-80)."""
    rng = random.Random(31)
    m = mastic_amd.MasticCount(256)
    n = 96
    pool = [tuple(bool(rng.getrandbits(1)) for _ in range(256)) for _ in range(24)]
    alphas = [pool[rng.randrange(len(pool))] for _ in range(n)]
    weights = [rng.randrange(2) for _ in range(n)]
    nonces = bytes(rng.getrandbits(8) for _ in range(16 * n))
    rands = bytes(rng.getrandbits(8) for _ in range(m.RAND_SIZE * n))
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    cand = set(pool)
    while len(cand) < 512:
        cand.add(tuple(bool(rng.getrandbits(1)) for _ in range(256)))
    ap = (255, tuple(sorted(cand)), True)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    res = [m.prep_init_batch(vk, CTX, a, ap, nonces, pub, in0 if a == 0 else in1, want_out_shares=False)
           for a in range(2)]
    (_msgs, valid) = m.decide_batch(CTX, ap, res[0][0], res[1][0])
    assert list(valid) == [1] * n
    aggs = [m.aggregate_device(a, ap) for a in range(2)]
    want = {}
    for (a, w) in zip(alphas, weights):
        want[a] = want.get(a, 0) + w
    assert m.unshard(ap, aggs, n) == [want.get(p, 0) for p in ap[1]]


def test_c2_full_prefix_count_oracle_report(mastic_amd):
    """BASELINE config C2 at its full size: Mastic(32, Sum 255), 10,000 random
    32-bit candidate prefixes at level 31 (376k tree nodes per report).  64
    reports through both aggregators: decide valid everywhere, aggregate equal
    to the plaintext per-attribute sums, and one report's prep share replayed
    in the CPU oracle at full tree size (about 25 s of CPU)."""
    rng = random.Random(13)
    m = mastic_amd.MasticSum(32, 255)
    attrs = set()
    while len(attrs) < 10000:
        attrs.add(tuple(bool(rng.getrandbits(1)) for _ in range(32)))
    attrs = sorted(attrs)
    n = 64
    alphas = [attrs[rng.randrange(len(attrs))] for _ in range(n)]
    weights = [rng.randrange(256) for _ in range(n)]
    nonces = bytes(rng.getrandbits(8) for _ in range(16 * n))
    rands = bytes(rng.getrandbits(8) for _ in range(m.RAND_SIZE * n))
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    ap = (31, tuple(attrs), True)
    assert m.tree_stats(ap)[0] > 370000
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    res = [m.prep_init_batch(vk, CTX, a, ap, nonces, pub, in0 if a == 0 else in1, want_out_shares=False)
           for a in range(2)]
    (_msgs, valid) = m.decide_batch(CTX, ap, res[0][0], res[1][0])
    assert list(valid) == [1] * n
    aggs = [m.aggregate_device(a, ap) for a in range(2)]
    want = {}
    for (a, w) in zip(alphas, weights):
        want[a] = want.get(a, 0) + w
    assert m.unshard(ap, aggs, n) == [want.get(p, 0) for p in ap[1]]
    o = _oracle_for(m)
    psz, isz = m.public_share_size(), m.input_share_size(0)
    i = 37
    cws = o.vidpf.decode_public_share(pub[psz * i:psz * (i + 1)])
    isd = o.decode_input_share(0, in0[isz * i:isz * (i + 1)])
    (_st, sh) = o.prep_init(vk, CTX, 0, ap, nonces[16 * i:16 * (i + 1)], cws, isd)
    enc = o.test_vec_encode_prep_share(sh)
    assert res[0][0][len(enc) * i:len(enc) * (i + 1)] == enc


@pytest.mark.parametrize("blk", [-1, 0, 150, 250])
def test_field128_long_payload_handover(mastic_amd, blk):
    """A long Field128 payload (VALUE_LEN 301: 301 convert blocks per child,
    the C5 shape at a smaller length).  Every output against the oracle, also
    with the exact-stream handover forced early, in the middle and near the
    end of the payload (the exact stream restarts from element 0 and emits
    from the handover element on)."""
    rng = random.Random(400 + blk)
    m = mastic_amd.MasticSumVec(4, 300, 1, 10)
    m.set_test_hooks(force_slow_blk=blk)
    assert m.VALUE_LEN == 301
    o = _oracle_for(m)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, 3)
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    for (level, nprefix, wc) in [(0, 2, True), (3, 4, False)]:
        ap = _random_agg_param(m, rng, alphas, level, nprefix, wc)
        _check_against_oracle(m, o, CTX, vk, ap, alphas, weights, nonces, rands, check_shard=(level == 0))
