"""Binder-sponge fill offsets against the oracle, frontier cache off and on.

The one-hot and payload checks are TurboSHAKE128 over
``le16(len(dst)) || dst || u8(0) || binder`` with ``dst = dst_alg(ctx, usage,
ID)`` (mastic.py:259-306, dst.py:35-42), so the binder message starts at byte
15 + len(ctx) of the sponge.  The GPU's 2-lane sponge has one absorb path for
a start that is a multiple of 4 bytes and a byte-shifted (DPP) path for the
other three residues; the 64-bit lanes see all eight residues mod 8.  Every
residue, a header that ends exactly on the 168-byte rate boundary (ctx 153)
and one that crosses it (ctx 160) are checked here: prep shares (eval proofs
and verifier shares) and out shares of every report equal the oracle's at
every level of a level-by-level walk, with the walk run once without the
frontier cache and once with it (levels >= 1 then resume the cached sponges).
"""
import random

import pytest

from test_gpu_parity import _oracle_for, _random_reports, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu

# 15 + len(ctx) mod 8 = 7, 0, 1, 2, 3, 4, 5, 6 for len 0..7; 19 = the bench's ctx
# (b"mastic-mi355x-bench"); 153: the header fills exactly one rate block; 160: it
# crosses into the second block
CTX_LENS = [0, 1, 2, 3, 4, 5, 6, 7, 19, 153, 160]


@pytest.mark.parametrize("ctx_len", CTX_LENS, ids=["ctx%d_off%d" % (n, (15 + n) % 8) for n in CTX_LENS])
def test_binder_fill_offsets_cache_off_and_on(mastic_amd, ctx_len):
    rng = random.Random(1000 + ctx_len)
    m = mastic_amd.MasticSum(5, 6)
    o = _oracle_for(m)
    ctx = bytes(rng.getrandbits(8) for _ in range(ctx_len))
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    n = 3
    (alphas, weights, nonces, rands) = _random_reports(m, rng, n)
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rands)
    psz, isz = m.public_share_size(), [m.input_share_size(0), m.input_share_size(1)]
    cws = [o.vidpf.decode_public_share(pub[psz * i:psz * (i + 1)]) for i in range(n)]
    ins = [[o.decode_input_share(a, (in0, in1)[a][isz[a] * i:isz[a] * (i + 1)]) for i in range(n)]
           for a in range(2)]
    # a walk whose every level keeps every prefix of the reports' alphas (no
    # pruning): with the cache on, levels >= 1 extend the cached tree
    aps = [(lv, tuple(sorted(set(a[:lv + 1] for a in alphas))), lv == 0) for lv in range(m.BITS)]
    want = {}
    for ap in aps:
        for a in range(2):
            ps, outs = b"", b""
            for i in range(n):
                (ost, osh) = o.prep_init(vk, ctx, a, ap, nonces[16 * i:16 * (i + 1)], cws[i], ins[a][i])
                ps += o.test_vec_encode_prep_share(osh)
                outs += o.field.encode_vec(ost[0])
            want[(ap[0], a)] = (ps, outs)
    for cache in (False, True):
        m.set_frontier_cache(cache)
        dev = m.reports_upload(nonces, pub, in0, in1)
        hits = 0
        for ap in aps:
            for a in range(2):
                m.prep_init_device(dev, vk, ctx, a, ap)
                hits += int(a == 0 and m.last_prep_was_cached())
                (ps, _js, outs, st) = m.prep_result(dev, a, ap, want_out_shares=True)
                assert list(st) == [0] * n
                assert ps == want[(ap[0], a)][0], "prep shares, level %d agg %d cache %s" % (ap[0], a, cache)
                assert outs == want[(ap[0], a)][1], "out shares, level %d agg %d cache %s" % (ap[0], a, cache)
        if cache:
            assert hits == m.BITS - 1, "levels 1.. should resume the cached sponges"
        del dev
    m.set_frontier_cache(False)
