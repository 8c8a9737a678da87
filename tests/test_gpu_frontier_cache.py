"""Frontier cache for level sweeps (Mastic.set_frontier_cache).

With the cache on, a prep_init whose tree is the previous call's tree plus one
level evaluates only that level and resumes both binder sponges from their
cached states.  The results must be bit-identical to a full evaluation: checked
level by level against a second context with the cache off, against the CPU
oracle for sampled reports, and end to end through the sweep driver."""
import random

import pytest

from test_gpu_parity import CTX, _oracle_for, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu


def _reports(m, rng, n, pool_size):
    pool = [tuple(bool(rng.getrandbits(1)) for _ in range(m.BITS)) for _ in range(pool_size)]
    alphas = [pool[min(int(rng.paretovariate(1.0)) - 1, pool_size - 1)] for _ in range(n)]
    weights = [rng.randrange(2) for _ in range(n)] if m.circuit == "Count" else \
        [rng.randrange(m.max_measurement + 1) for _ in range(n)]
    nonces = bytes(rng.getrandbits(8) for _ in range(16 * n))
    rands = bytes(rng.getrandbits(8) for _ in range(m.RAND_SIZE * n))
    return alphas, weights, nonces, rands


@pytest.mark.parametrize("circuit,kw", [("Count", dict(bits=10)), ("Sum", dict(bits=9, max_measurement=5))],
                         ids=["Count", "Sum"])
def test_cached_levels_bit_identical(mastic_amd, circuit, kw):
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    rng = random.Random(77)
    kw = dict(kw)
    bits = kw.pop("bits")
    m_off = mastic_amd.Mastic(bits, circuit, **kw)
    m_on = mastic_amd.Mastic(bits, circuit, **kw)
    o = _oracle_for(m_off)
    n = 150
    (alphas, weights, nonces, rands) = _reports(m_off, rng, n, 12)
    (pub, in0, in1) = m_off.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    # the per-level candidate lists of a real sweep (cache off)
    trace = []
    dev_off = m_off.reports_upload(nonces, pub, in0, in1)
    hh = compute_heavy_hitters(m_off, CTX, {"default": 4}, dev_off, verify_key=vk, trace=trace)
    assert trace[-1].prefixes, "the workload should keep candidates down to the last level"
    dev_on = m_on.reports_upload(nonces, pub, in0, in1)
    m_on.set_frontier_cache(True)
    hits = 0
    psz, isz = m_off.public_share_size(), m_off.input_share_size(1)
    for lv in trace:
        if not lv.prefixes:
            break
        ap = (lv.level, tuple(lv.prefixes), lv.level == 0)
        for agg_id in range(2):
            m_off.prep_init_device(dev_off, vk, CTX, agg_id, ap)
            m_on.prep_init_device(dev_on, vk, CTX, agg_id, ap)
            a = m_off.prep_result(dev_off, agg_id, ap, want_out_shares=True)
            b = m_on.prep_result(dev_on, agg_id, ap, want_out_shares=True)
            assert a[0] == b[0] and a[2] == b[2], "level %d agg %d" % (lv.level, agg_id)
            if m_on.last_prep_was_cached():
                hits += 1
                if agg_id == 1 and hits <= 8:
                    # sampled reports of a cached level through the oracle
                    for i in (0, n - 1):
                        cws = o.vidpf.decode_public_share(pub[psz * i:psz * (i + 1)])
                        isd = o.decode_input_share(1, in1[isz * i:isz * (i + 1)])
                        (_st, sh) = o.prep_init(vk, CTX, 1, ap, nonces[16 * i:16 * (i + 1)], cws, isd)
                        enc = o.test_vec_encode_prep_share(sh)
                        assert b[0][len(enc) * i:len(enc) * (i + 1)] == enc
    assert hits >= 2, hits  # levels whose tree extends the previous one take the cached path
    # the sweep driver with the cache gives the same heavy hitters
    cached = []
    assert compute_heavy_hitters(m_on, CTX, {"default": 4}, dev_on, verify_key=vk, frontier_cache=True,
                                 cached_levels=cached) == hh
    assert len(cached) >= 1
    m_on.set_frontier_cache(False)


def test_cache_not_used_across_different_inputs(mastic_amd):
    """A cached tree is only reused for the same reports, agg_id, verify key
    and ctx: changing any of them evaluates the whole tree."""
    rng = random.Random(78)
    m = mastic_amd.MasticCount(6)
    (alphas, weights, nonces, rands) = _reports(m, rng, 70, 4)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    dev = m.reports_upload(nonces, pub, in0, in1)
    m.set_frontier_cache(True)
    vk = bytes(32)
    p0 = tuple(sorted(set(a[:1] for a in alphas)))
    p1 = tuple(sorted(set(a[:2] for a in alphas) | set(p + (b,) for p in p0 for b in (False, True))))
    m.prep_init_device(dev, vk, CTX, 0, (0, ((False,), (True,)), False))
    m.prep_init_device(dev, vk, CTX, 0, (1, p1, False))
    assert m.last_prep_was_cached()
    m.prep_init_device(dev, vk, CTX, 0, (0, ((False,), (True,)), False))
    m.prep_init_device(dev, bytes([1]) * 32, CTX, 0, (1, p1, False))  # other verify key
    assert not m.last_prep_was_cached()
    m.prep_init_device(dev, vk, CTX, 0, (0, ((False,), (True,)), False))
    m.prep_init_device(dev, vk, CTX + b"x", 0, (1, p1, False))  # other ctx
    assert not m.last_prep_was_cached()
    m.prep_init_device(dev, vk, CTX, 0, (0, ((False,), (True,)), False))
    m.prep_init_device(dev, vk, CTX, 1, (1, p1, False))  # other aggregator
    assert not m.last_prep_was_cached()
    m.set_frontier_cache(False)


def test_cache_miss_when_counts_match_but_paths_differ(mastic_amd):
    """The hit rule compares level L-1's node paths, not just the per-level
    node counts: a level-2 call whose parents hang off the other level-0 node
    (same counts 1, 1, 1 as the cached level-1 tree) must evaluate the whole
    tree, and its results must equal a cache-off context's."""
    rng = random.Random(79)
    m = mastic_amd.MasticCount(5)
    ref = mastic_amd.MasticCount(5)
    (alphas, weights, nonces, rands) = _reports(m, rng, 70, 6)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    dev = m.reports_upload(nonces, pub, in0, in1)
    dev_ref = ref.reports_upload(nonces, pub, in0, in1)
    m.set_frontier_cache(True)
    vk = bytes(range(16))
    lvl1 = (1, ((False, False), (False, True)), False)              # tree under 0
    lvl2 = (2, ((True, False, False), (True, False, True)), False)  # tree under 1: counts 1, 1, 1
    assert m.tree_stats(lvl1)[0] == 4 and m.tree_stats(lvl2)[0] == 6
    m.prep_init_device(dev, vk, CTX, 0, (0, ((False,), (True,)), False))
    m.prep_init_device(dev, vk, CTX, 0, lvl1)
    assert m.last_prep_was_cached()
    m.prep_init_device(dev, vk, CTX, 0, lvl2)
    assert not m.last_prep_was_cached()
    got = m.prep_result(dev, 0, lvl2, want_out_shares=True)
    ref.prep_init_device(dev_ref, vk, CTX, 0, lvl2)
    want = ref.prep_result(dev_ref, 0, lvl2, want_out_shares=True)
    assert got[0] == want[0] and got[2] == want[2]
    m.set_frontier_cache(False)


def test_cache_across_hbm_chunks(mastic_amd):
    """The cache holds planes of all reports, independent of the HBM-budget
    chunks a call runs in: with 64- or 128-report chunks (changing from level
    to level) the cached levels still hit and every level is bit-identical to
    a cache-off context's."""
    import ctypes
    from mastic_amd import _lib
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    rng = random.Random(80)
    m_off = mastic_amd.MasticSum(9, 5)
    m_on = mastic_amd.MasticSum(9, 5)
    n = 150
    (alphas, weights, nonces, rands) = _reports(m_off, rng, n, 10)
    (pub, in0, in1) = m_off.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    trace = []
    dev_off = m_off.reports_upload(nonces, pub, in0, in1)
    compute_heavy_hitters(m_off, CTX, {"default": 3}, dev_off, verify_key=vk, trace=trace)
    dev_on = m_on.reports_upload(nonces, pub, in0, in1)
    m_on.set_frontier_cache(True)
    hits = 0
    try:
        for lv in trace:
            if not lv.prefixes:
                break
            ap = (lv.level, tuple(lv.prefixes), lv.level == 0)
            enc = m_on.encode_agg_param(ap)
            per = m_on.work_bytes(enc) + 64 * 1024  # + the cache's staging planes
            groups = 1 if lv.level % 2 else 2        # 64- or 128-report chunks
            _lib.lib().mastic_set_memory_budget(m_on._ctx, ctypes.c_uint64(per * 64 * groups + per * 64))
            for agg_id in range(2):
                m_off.prep_init_device(dev_off, vk, CTX, agg_id, ap)
                m_on.prep_init_device(dev_on, vk, CTX, agg_id, ap)
                hits += m_on.last_prep_was_cached()
                a = m_off.prep_result(dev_off, agg_id, ap, want_out_shares=True)
                b = m_on.prep_result(dev_on, agg_id, ap, want_out_shares=True)
                assert a[0] == b[0] and a[2] == b[2], "level %d agg %d" % (lv.level, agg_id)
    finally:
        _lib.lib().mastic_set_memory_budget(m_on._ctx, ctypes.c_uint64(0))
        m_on.set_frontier_cache(False)
    assert hits >= 4, hits


def test_cache_at_c3_parameters(mastic_amd):
    """BASELINE config C3's Mastic(256, Count) through a full 256-level
    threshold sweep with the cache on: every level bit-identical to a cache-off
    context, sampled reports of deep cached levels against the CPU oracle,
    and the heavy hitters equal to the plaintext counts."""
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    rng = random.Random(81)
    m_off = mastic_amd.MasticCount(256)
    m_on = mastic_amd.MasticCount(256)
    o = _oracle_for(m_off)
    n = 256
    (alphas, weights, nonces, rands) = _reports(m_off, rng, n, 6)
    (pub, in0, in1) = m_off.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    th = {"default": 12}
    trace = []
    dev_off = m_off.reports_upload(nonces, pub, in0, in1)
    hh = compute_heavy_hitters(m_off, CTX, th, dev_off, verify_key=vk, trace=trace)
    counts = {}
    for (a, w) in zip(alphas, weights):
        counts[a] = counts.get(a, 0) + w
    assert hh == sorted(a for (a, c) in counts.items() if c >= 12) and hh
    dev_on = m_on.reports_upload(nonces, pub, in0, in1)
    m_on.set_frontier_cache(True)
    psz, isz = m_off.public_share_size(), m_off.input_share_size(1)
    hits = 0
    targets = [40, 129, 250]  # oracle samples at the first cached level at or past each
    checked = []
    try:
        for lv in trace:
            if not lv.prefixes:
                break
            ap = (lv.level, tuple(lv.prefixes), lv.level == 0)
            for agg_id in range(2):
                m_off.prep_init_device(dev_off, vk, CTX, agg_id, ap)
                m_on.prep_init_device(dev_on, vk, CTX, agg_id, ap)
                cached = m_on.last_prep_was_cached()
                hits += cached
                a = m_off.prep_result(dev_off, agg_id, ap, want_out_shares=True)
                b = m_on.prep_result(dev_on, agg_id, ap, want_out_shares=True)
                assert a[0] == b[0] and a[2] == b[2], "level %d agg %d" % (lv.level, agg_id)
                if agg_id == 1 and cached and targets and lv.level >= targets[0]:
                    targets.pop(0)
                    checked.append(lv.level)
                    for i in (0, n - 1):
                        cws = o.vidpf.decode_public_share(pub[psz * i:psz * (i + 1)])
                        isd = o.decode_input_share(1, in1[isz * i:isz * (i + 1)])
                        (_st, sh) = o.prep_init(vk, CTX, 1, ap, nonces[16 * i:16 * (i + 1)], cws, isd)
                        enc = o.test_vec_encode_prep_share(sh)
                        assert b[0][len(enc) * i:len(enc) * (i + 1)] == enc, "level %d report %d" % (lv.level, i)
    finally:
        m_on.set_frontier_cache(False)
    assert hits >= 2 * 200, hits
    assert len(checked) == 3, checked


def test_cache_tracks_writes_through_views(mastic_amd):
    """A batch and its views share HBM and one contents generation: new
    reports uploaded through the parent batch invalidate a cache filled
    through a view (the next level evaluates its whole tree, equal to a
    cache-off context on the new data), and two views of equal size at
    different offsets never share cache entries."""
    rng = random.Random(81)
    m = mastic_amd.MasticCount(6)
    ref = mastic_amd.MasticCount(6)
    (alphas, weights, nonces, rands) = _reports(m, rng, 128, 4)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    (alphas2, weights2, nonces2, rands2) = _reports(m, rng, 128, 4)
    (pub2, in0_2, in1_2) = m.shard_batch(CTX, alphas2, weights2, nonces2, rands2)
    allr = m.reports_upload(nonces, pub, in0, in1)
    v0 = allr.view(0, 64)
    v1 = allr.view(64, 64)
    m.set_frontier_cache(True)
    vk = bytes(range(16))
    lvl0 = (0, ((False,), (True,)), False)
    lvl1 = (1, ((False, False), (False, True), (True, False), (True, True)), False)
    m.prep_init_device(v0, vk, CTX, 0, lvl0)
    m.prep_init_device(v0, vk, CTX, 0, lvl1)
    assert m.last_prep_was_cached()
    m.prep_init_device(v0, vk, CTX, 0, lvl0)
    m.prep_init_device(v1, vk, CTX, 0, lvl1)  # same size, other reports
    assert not m.last_prep_was_cached()
    m.prep_init_device(v0, vk, CTX, 0, lvl0)
    allr.upload(nonces2, pub2, in0_2, in1_2)  # new data through the parent
    m.prep_init_device(v0, vk, CTX, 0, lvl1)
    assert not m.last_prep_was_cached()
    got = m.prep_result(v0, 0, lvl1, want_out_shares=True)
    want = ref.prep_init_batch(vk, CTX, 0, lvl1, nonces2[:16 * 64], pub2[:len(pub2) // 2], in0_2[:len(in0_2) // 2])
    assert got[0] == want[0] and got[2] == want[2]
    m.set_frontier_cache(False)
