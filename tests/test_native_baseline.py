"""The native multithreaded CPU baseline (oracle/native_prep.c through
oracle/native.py) computes exactly the reference's prep_init: every golden
vector's prep shares and out shares of both aggregators (test_vec/mastic,
byte copies in tests/golden/), and random reports of a Field64 and a
Field128 circuit against the Python oracle, on several threads.  bench.py
times it as cpu_baseline.native."""
import json
import random

import pytest

from conftest import golden_files


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.rsplit("/", 1)[-1])
def test_native_matches_golden_vectors(path):
    from oracle import mastic as om
    from oracle.native import prep_init_native
    tv = json.load(open(path))
    o = om.from_test_vec(tv)
    ctx = bytes.fromhex(tv["ctx"])
    vk = bytes.fromhex(tv["verify_key"])
    ap = o.decode_agg_param(bytes.fromhex(tv["agg_param"]))
    reps = tv["prep"]
    nonces = b"".join(bytes.fromhex(r["nonce"]) for r in reps)
    pubs = b"".join(bytes.fromhex(r["public_share"]) for r in reps)
    for agg_id in range(2):
        ins = b"".join(bytes.fromhex(r["input_shares"][agg_id]) for r in reps)
        (shares, outs) = prep_init_native(o, vk, ctx, agg_id, ap, nonces, pubs, ins, threads=2)
        assert [s.hex() for s in shares] == [r["prep_shares"][0][agg_id] for r in reps]
        want = b"".join(b"".join(bytes.fromhex(x) for x in r["out_shares"][agg_id]) for r in reps)
        assert outs == want


@pytest.mark.parametrize("kind", ["sum", "histogram"])
def test_native_matches_oracle_random(kind):
    from oracle import mastic as om
    from oracle.native import prep_init_native
    rng = random.Random(7 if kind == "sum" else 8)
    o = om.MasticSum(10, 255) if kind == "sum" else om.MasticHistogram(6, 9, 3)
    ctx = b"native baseline"
    n = 7
    reps = []
    for _ in range(n):
        alpha = tuple(bool(rng.getrandbits(1)) for _ in range(o.vidpf.BITS))
        w = rng.randrange(256) if kind == "sum" else rng.randrange(9)
        nonce = bytes(rng.getrandbits(8) for _ in range(16))
        rand = bytes(rng.getrandbits(8) for _ in range(o.RAND_SIZE))
        (cws, shares) = o.shard(ctx, (alpha, w), nonce, rand)
        reps.append((alpha, nonce, cws, shares))
    level = o.vidpf.BITS - 3
    prefixes = sorted(set(r[0][:level + 1] for r in reps) | {tuple([True] * (level + 1))})
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    for wc in (True, False):
        ap = (level, tuple(prefixes), wc)
        for agg_id in range(2):
            nonces = b"".join(r[1] for r in reps)
            pubs = b"".join(o.vidpf.encode_public_share(r[2]) for r in reps)
            ins = b"".join(o.test_vec_encode_input_share(r[3][agg_id]) for r in reps)
            (shares, outs) = prep_init_native(o, vk, ctx, agg_id, ap, nonces, pubs, ins, threads=3)
            for (i, r) in enumerate(reps):
                ((trunc, _jr), share) = o.prep_init(vk, ctx, agg_id, ap, r[1], r[2], r[3][agg_id])
                assert shares[i] == o.test_vec_encode_prep_share(share), (wc, agg_id, i)
                row = len(outs) // n
                assert outs[row * i:row * (i + 1)] == o.field.encode_vec(trunc), (wc, agg_id, i)
