"""Both aggregators' prep_init queued before either result is fetched, with
the frontier cache on, in the orders a level sweep and its variants produce:
hit after hit, a hit beside a weight-check miss, a hit followed by a call with
another verify key (which rebuilds the prefix states), results fetched in
either order or folded straight from HBM.  A single-chunk cache-on call runs
its binder sponges in the cache's own planes and the level kernel writes the
out shares straight into the aggregator's result planes
(csrc/mastic_hip.hip run_chunk, "direct"), so the two aggregators' queued
calls share the work planes but not these.  Every result must equal a
cache-off context's."""
import random

import numpy as np
import pytest

from test_gpu_frontier_cache import _reports
from test_gpu_parity import CTX, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu


def _trace(m_off, dev_off, vk, threshold):
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    trace = []
    compute_heavy_hitters(m_off, CTX, {"default": threshold}, dev_off, verify_key=vk, trace=trace)
    return [lv for lv in trace if lv.prefixes]


def _pair(m, dev, vks, aps, order):
    """prep_init of both aggregators (vks[a], aps[a]), then both results."""
    for a in (0, 1):
        m.prep_init_device(dev, vks[a], CTX, a, aps[a])
    cached = m.last_prep_was_cached()
    res = {}
    for a in order:
        res[a] = m.prep_result(dev, a, aps[a], want_out_shares=True)
    return res, cached


@pytest.mark.parametrize("circuit,kw", [("Count", dict(bits=12)), ("Sum", dict(bits=10, max_measurement=7))],
                         ids=["Count", "Sum"])
def test_both_aggregators_queued(mastic_amd, circuit, kw):
    rng = random.Random(91)
    kw = dict(kw)
    bits = kw.pop("bits")
    m_off = mastic_amd.Mastic(bits, circuit, **kw)
    m_on = mastic_amd.Mastic(bits, circuit, **kw)
    n = 200
    (alphas, weights, nonces, rands) = _reports(m_off, rng, n, 10)
    (pub, in0, in1) = m_off.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    dev_off = m_off.reports_upload(nonces, pub, in0, in1)
    dev_on = m_on.reports_upload(nonces, pub, in0, in1)
    trace = _trace(m_off, dev_off, vk, 4)
    assert len(trace) >= 6
    m_on.set_frontier_cache(True)
    hits = 0
    try:
        for (i, lv) in enumerate(trace):
            ap = (lv.level, tuple(lv.prefixes), lv.level == 0)
            order = (0, 1) if i % 2 == 0 else (1, 0)
            (want, _) = _pair(m_off, dev_off, (vk, vk), (ap, ap), order)
            (got, cached) = _pair(m_on, dev_on, (vk, vk), (ap, ap), order)
            hits += cached
            for a in (0, 1):
                assert got[a][0] == want[a][0] and got[a][2] == want[a][2], "level %d agg %d" % (lv.level, a)
                assert (got[a][3] == want[a][3]).all()
            # the two aggregators' shares decide as the cache-off ones do
            assert (m_on.decide_results(CTX, n)[0] == m_off.decide_results(CTX, n)[0]).all()
    finally:
        m_on.set_frontier_cache(False)
    assert hits >= len(trace) - 2, (hits, len(trace))


def test_hit_beside_weight_check_miss(mastic_amd):
    """Every third level aggregator 1 runs with the weight check (never a hit),
    so aggregator 0's queued hit meets a miss and the next level's hit follows
    one."""
    rng = random.Random(92)
    m_off = mastic_amd.MasticSum(10, 7)
    m_on = mastic_amd.MasticSum(10, 7)
    n = 180
    (alphas, weights, nonces, rands) = _reports(m_off, rng, n, 8)
    (pub, in0, in1) = m_off.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    dev_off = m_off.reports_upload(nonces, pub, in0, in1)
    dev_on = m_on.reports_upload(nonces, pub, in0, in1)
    trace = _trace(m_off, dev_off, vk, 3)
    m_on.set_frontier_cache(True)
    try:
        for (i, lv) in enumerate(trace):
            ap0 = (lv.level, tuple(lv.prefixes), lv.level == 0)
            ap1 = (lv.level, tuple(lv.prefixes), lv.level == 0 or i % 3 == 2)
            (want, _) = _pair(m_off, dev_off, (vk, vk), (ap0, ap1), (1, 0))
            (got, _) = _pair(m_on, dev_on, (vk, vk), (ap0, ap1), (1, 0))
            for a in (0, 1):
                assert got[a][0] == want[a][0] and got[a][1] == want[a][1] and got[a][2] == want[a][2], \
                    "level %d agg %d" % (lv.level, a)
    finally:
        m_on.set_frontier_cache(False)


def test_hit_then_other_verify_key(mastic_amd):
    """Aggregator 0 hits, then aggregator 1 runs with another verify key (the
    prefix states are rebuilt while aggregator 0's call may still run).  Also
    folds aggregator 0's out shares straight from HBM (mastic_aggregate) while
    aggregator 1's call is queued."""
    rng = random.Random(93)
    m_off = mastic_amd.MasticCount(11)
    m_on = mastic_amd.MasticCount(11)
    n = 160
    (alphas, weights, nonces, rands) = _reports(m_off, rng, n, 6)
    (pub, in0, in1) = m_off.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    vk2 = bytes(rng.getrandbits(8) for _ in range(16))
    dev_off = m_off.reports_upload(nonces, pub, in0, in1)
    dev_on = m_on.reports_upload(nonces, pub, in0, in1)
    trace = _trace(m_off, dev_off, vk, 4)
    m_on.set_frontier_cache(True)
    try:
        for (i, lv) in enumerate(trace):
            ap = (lv.level, tuple(lv.prefixes), lv.level == 0)
            vks = (vk, vk2 if i % 2 else vk)
            (want, _) = _pair(m_off, dev_off, vks, (ap, ap), (0, 1))
            want_agg = m_off.aggregate_device(0, ap, raw=True)
            for a in (0, 1):
                m_on.prep_init_device(dev_on, vks[a], CTX, a, ap)
            got_agg = m_on.aggregate_device(0, ap, raw=True)
            got = {a: m_on.prep_result(dev_on, a, ap, want_out_shares=True) for a in (1, 0)}
            assert got_agg == want_agg, "level %d" % lv.level
            for a in (0, 1):
                assert got[a][0] == want[a][0] and got[a][2] == want[a][2], "level %d agg %d" % (lv.level, a)
    finally:
        m_on.set_frontier_cache(False)


def test_queued_hits_timing_and_sync(mastic_amd):
    """last_timing of a queued hit and synchronize with both aggregators'
    hits queued."""
    rng = random.Random(94)
    m = mastic_amd.MasticCount(8)
    n = 128
    (alphas, weights, nonces, rands) = _reports(m, rng, n, 5)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    dev = m.reports_upload(nonces, pub, in0, in1)
    vk = bytes(16)
    m.set_frontier_cache(True)
    try:
        lvl0 = (0, ((False,), (True,)), False)
        lvl1 = (1, ((False, False), (False, True), (True, False), (True, True)), False)
        for a in (0, 1):
            m.prep_init_device(dev, vk, CTX, a, lvl0)
        for a in (0, 1):
            m.prep_init_device(dev, vk, CTX, a, lvl1)
            assert m.last_prep_was_cached()
        m.synchronize()
        m.select_timing(0)
        t = m.last_timing()
        assert t[-1] > 0 and np.isfinite(t[-1])
    finally:
        m.set_frontier_cache(False)


def test_hit_timing_with_busy_sponge_stream(mastic_amd):
    """A single-chunk frontier-cache hit records empty timing marks on the
    binder-sponge stream while its sponges run on the main stream, so the main
    stream never waits for them.  With that stream held busy (the sponge-delay
    test hook: a 400 ms idle kernel queued there first), mastic_last_timing3
    right after the call -- no synchronize -- must wait for the marks
    themselves and return finite times (round 5's "device not ready" failure
    in a 4-rank run sharing one GPU; fixed in 47221e6).  The knob build's
    MASTIC_DBG_TIMING_NOWAIT=1 restores the old behaviour: tools/timing_fix_ab.py."""
    rng = random.Random(95)
    m = mastic_amd.MasticCount(8)
    n = 128
    (alphas, weights, nonces, rands) = _reports(m, rng, n, 5)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    dev = m.reports_upload(nonces, pub, in0, in1)
    vk = bytes(16)
    m.set_frontier_cache(True)
    try:
        lvl0 = (0, ((False,), (True,)), False)
        lvl1 = (1, ((False, False), (False, True), (True, False), (True, True)), False)
        m.prep_init_device(dev, vk, CTX, 0, lvl0)
        m.synchronize()
        m.set_test_sponge_delay(400000)
        m.prep_init_device(dev, vk, CTX, 0, lvl1)
        assert m.last_prep_was_cached()
        t = m.last_timing3()
        assert all(np.isfinite(x) and x >= 0 for x in t)
        assert t[-1] > 0
    finally:
        m.set_frontier_cache(False)
