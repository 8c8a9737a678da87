"""The out-of-memory recovery path of prep_init.

A result buffer or frontier-cache slot that cannot be allocated makes
prep_init wait for everything queued on the ctx's three streams, free the
retired buffers and the work arena, and retry (mastic_hip.hip ``rgrow`` and
the cache ``alloc``).  At full scale only C3's 2M-report sweep reaches it, so
the result-preserving ``fail_allocs`` test hook (``mastic_set_test_hooks``)
forces those allocations to fail: the outputs must be bit-identical to an
unconstrained context, and every injected failure must have been consumed
(i.e. the recovery ran).  The first case queues aggregator 0's prep_init and
then forces the recovery inside aggregator 1's, so the arena it frees is
still being read by queued kernels when the recovery starts."""
import random

import pytest

from test_gpu_frontier_cache import _reports
from test_gpu_parity import CTX, _oracle_for, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu


def test_result_alloc_failure_recovers_bit_identical(mastic_amd):
    rng = random.Random(91)
    m = mastic_amd.MasticSum(8, 255)
    ref = mastic_amd.MasticSum(8, 255)
    o = _oracle_for(m)
    n = 200
    (alphas, weights, nonces, rands) = _reports(m, rng, n, 10)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(16))
    ap = (7, tuple(sorted(set(alphas))), True)
    dev = m.reports_upload(nonces, pub, in0, in1)
    dev_ref = ref.reports_upload(nonces, pub, in0, in1)
    # aggregator 0 queued (uses the work arena), then aggregator 1 with its
    # first two result allocations failing: the recovery waits for agg 0's
    # kernels, frees the arena and re-allocates it
    m.prep_init_device(dev, vk, CTX, 0, ap)
    m.set_test_hooks(fail_allocs=2)
    m.prep_init_device(dev, vk, CTX, 1, ap)
    assert m.set_test_hooks() == 0, "the injected allocation failures were not all reached"
    for agg_id in range(2):
        ref.prep_init_device(dev_ref, vk, CTX, agg_id, ap)
        a = m.prep_result(dev, agg_id, ap, want_out_shares=True)
        b = ref.prep_result(dev_ref, agg_id, ap, want_out_shares=True)
        assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2], agg_id
        assert list(a[3]) == [0] * n
    # and against the oracle for two reports of the recovered aggregator
    psz, isz = m.public_share_size(), m.input_share_size(1)
    a1 = m.prep_result(dev, 1, ap)
    for i in (0, n - 1):
        cws = o.vidpf.decode_public_share(pub[psz * i:psz * (i + 1)])
        isd = o.decode_input_share(1, in1[isz * i:isz * (i + 1)])
        (_st, sh) = o.prep_init(vk, CTX, 1, ap, nonces[16 * i:16 * (i + 1)], cws, isd)
        enc = o.test_vec_encode_prep_share(sh)
        assert a1[0][len(enc) * i:len(enc) * (i + 1)] == enc
    # the aggregate after the recovery equals the reference context's
    assert m.aggregate_device(1, ap, raw=True) == ref.aggregate_device(1, ap, raw=True)


def test_cache_slot_alloc_failure_recovers_bit_identical(mastic_amd):
    """A frontier-cache sweep whose slot allocations fail at every level: each
    level's results equal a cache-off context's, and the cached levels still
    take the cached path after the recovery."""
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    rng = random.Random(92)
    m_off = mastic_amd.MasticCount(9)
    m_on = mastic_amd.MasticCount(9)
    n = 180
    (alphas, weights, nonces, rands) = _reports(m_off, rng, n, 10)
    (pub, in0, in1) = m_off.shard_batch(CTX, alphas, weights, nonces, rands)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    trace = []
    dev_off = m_off.reports_upload(nonces, pub, in0, in1)
    compute_heavy_hitters(m_off, CTX, {"default": 4}, dev_off, verify_key=vk, trace=trace)
    dev_on = m_on.reports_upload(nonces, pub, in0, in1)
    m_on.set_frontier_cache(True)
    hits = recovered = 0
    for lv in trace:
        if not lv.prefixes:
            break
        ap = (lv.level, tuple(lv.prefixes), lv.level == 0)
        for agg_id in range(2):
            # a cache call allocates its sponge-state slot, its root-sum slot
            # and (when the frontier widens) new seed / convert-seed slots
            m_on.set_test_hooks(fail_allocs=3)
            m_off.prep_init_device(dev_off, vk, CTX, agg_id, ap)
            m_on.prep_init_device(dev_on, vk, CTX, agg_id, ap)
            pending = m_on.set_test_hooks()
            recovered += 3 - pending
            a = m_off.prep_result(dev_off, agg_id, ap, want_out_shares=True)
            b = m_on.prep_result(dev_on, agg_id, ap, want_out_shares=True)
            assert a[0] == b[0] and a[2] == b[2], "level %d agg %d" % (lv.level, agg_id)
            hits += m_on.last_prep_was_cached()
    assert recovered >= 2 * len([lv for lv in trace if lv.prefixes]), recovered
    assert hits >= 2, hits
    m_on.set_frontier_cache(False)
