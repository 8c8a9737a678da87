"""Heavy-hitters sweep and attribute metrics on the GPU.

The three end-to-end drivers of the reference (poc/examples.py:94-260) run
unchanged against mastic_amd, with the reference's own asserted outputs; a
larger random sweep is checked level by level against the plaintext
functionality (talks/func.py:49-80, restated in test_sweep.py).
"""
import hashlib
import os
import random

import numpy as np
import pytest

from conftest import PKG_ROOT  # noqa: F401
from test_sweep import index, plain_heavy_hitters, plain_sums

pytestmark = pytest.mark.gpu


def _reports(mastic, ctx, measurements, rng):
    out = []
    for m in measurements:
        nonce = rng.randbytes(16)
        rand = rng.randbytes(mastic.RAND_SIZE)
        (pub, ins) = mastic.shard(ctx, m, nonce, rand)
        out.append((nonce, pub, ins))
    return out


def test_example_weighted_heavy_hitters_mode():
    """poc/examples.py:94-128"""
    from mastic_amd import MasticCount
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    bits = 4
    ctx = b'example_weighted_heavy_hitters_mode'
    mastic = MasticCount(bits)
    ix = mastic.vidpf.test_index_from_int
    measurements = [(ix(v, bits), w) for (v, w) in [
        (0b1001, 1), (0b0000, 1), (0b0000, 0), (0b0000, 1), (0b1001, 1), (0b0000, 1),
        (0b1100, 1), (0b0011, 1), (0b1111, 0), (0b1111, 0), (0b1111, 1)]]
    reports = _reports(mastic, ctx, measurements, random.Random(5))
    hh = compute_heavy_hitters(mastic, ctx, {'default': 2}, reports)
    assert hh == [ix(0b0000, bits), ix(0b1001, bits)]


def test_example_weighted_heavy_hitters_mode_with_different_thresholds():
    """poc/examples.py:131-169"""
    from mastic_amd import MasticCount
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    bits = 4
    ctx = b'example_weighted_heavy_hitters_mode_with_different_thresholds'
    mastic = MasticCount(bits)
    ix = mastic.vidpf.test_index_from_int
    measurements = [(ix(v, bits), 1) for v in
                    [0b0000, 0b0001, 0b1001, 0b1001, 0b1010, 0b1010, 0b1111, 0b1111, 0b1111, 0b1111, 0b1111]]
    reports = _reports(mastic, ctx, measurements, random.Random(6))
    thresholds = {'default': 2, ix(0b00, 2): 1, ix(0b10, 2): 3, ix(0b11, 2): 5}
    hh = compute_heavy_hitters(mastic, ctx, thresholds, reports)
    assert hh == [ix(0b0000, bits), ix(0b0001, bits), ix(0b1111, bits)]


def test_example_attribute_based_metrics_mode():
    """poc/examples.py:172-260, through the reference's per-report API."""
    from mastic_amd import MasticSum
    bits = 8
    ctx = b'example_attribute_based_metrics_mode'
    mastic = MasticSum(bits, 3)
    verify_key = os.urandom(16)  # gen_rand(16), as examples.py:176

    def h(attr):
        return mastic.vidpf.test_index_from_int(hashlib.sha3_256(attr.encode('ascii')).digest()[0], bits)

    measurements = [('United States', 1), ('Greece', 1), ('United States', 2), ('Greece', 0),
                    ('United States', 0), ('India', 1), ('Greece', 0), ('United States', 1),
                    ('Greece', 1), ('Greece', 3), ('Greece', 1)]
    rng = random.Random(7)
    reports = _reports(mastic, ctx, [(h(a), v) for (a, v) in measurements], rng)
    attrs = ['Greece', 'Mexico', 'United States']
    agg_param = (bits - 1, list(map(h, attrs)), True)
    assert mastic.is_valid(agg_param, [])
    agg_shares = [mastic.agg_init(agg_param) for _ in range(2)]
    for (nonce, public_share, input_shares) in reports:
        (prep_state, prep_shares) = zip(*[
            mastic.prep_init(verify_key, ctx, agg_id, agg_param, nonce, public_share, input_shares[agg_id])
            for agg_id in range(2)])
        prep_msg = mastic.prep_shares_to_prep(ctx, agg_param, prep_shares)
        for agg_id in range(2):
            out_share = mastic.prep_next(ctx, prep_state[agg_id], prep_msg)
            agg_shares[agg_id] = mastic.agg_update(agg_param, agg_shares[agg_id], out_share)
    assert mastic.unshard(agg_param, agg_shares, len(measurements)) == [6, 0, 4]


def test_random_sweep_matches_plaintext_per_level():
    """A 12-bit Count sweep over 2000 GPU-sharded reports: every level's
    aggregate equals the plaintext per-prefix sums, and the heavy hitters equal
    the plaintext driver's."""
    from mastic_amd import MasticCount
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    bits, n = 12, 2000
    rng = random.Random(11)
    heavy = [rng.randrange(2 ** bits) for _ in range(6)]
    vals = [rng.choice(heavy) if rng.random() < 0.5 else rng.randrange(2 ** bits) for _ in range(n)]
    weights = [int(rng.random() < 0.9) for _ in range(n)]
    meas = [(index(v, bits), w) for (v, w) in zip(vals, weights)]
    mastic = MasticCount(bits)
    ctx = b'sweep'
    ab = (bits + 7) // 8
    alphas = b"".join(v.to_bytes(ab, "big") if bits % 8 == 0 else (v << (8 * ab - bits)).to_bytes(ab, "big")
                      for v in vals)
    betas = b"".join(mastic.field.encode_vec(mastic.encode_measurement(w)) for w in weights)
    dev = mastic.reports_shard(ctx, alphas, betas, rng.randbytes(16 * n), rng.randbytes(mastic.RAND_SIZE * n))
    th = {'default': 40, index(0b1, 1): 60}
    trace = []
    hh = compute_heavy_hitters(mastic, ctx, th, dev, verify_key=rng.randbytes(32), trace=trace)
    for t in trace:
        assert t.n_valid == n
        assert t.agg_result == plain_sums(meas, t.prefixes), t.level
    assert hh == plain_heavy_hitters(meas, th, bits)
    assert hh


def test_sweep_drops_tampered_report():
    """A report whose correction word for level 2 is corrupted passes levels
    0-1 and is rejected (dropped) from level 2 on; the reference driver would
    raise there instead."""
    from mastic_amd import MasticCount
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    bits = 6
    mastic = MasticCount(bits)
    ctx = b'tamper'
    rng = random.Random(12)
    meas = [(index(0b101101, bits), 1)] * 4 + [(index(0b010011, bits), 1)] * 3
    reports = _reports(mastic, ctx, meas, rng)
    (nonce, pub, ins) = reports[0]
    pub = list(pub)
    (seed, ctrl, w, proof) = pub[2]
    pub[2] = (bytes([seed[0] ^ 1]) + bytes(seed[1:]), ctrl, w, proof)
    reports[0] = (nonce, pub, ins)
    trace = []
    hh = compute_heavy_hitters(mastic, ctx, {'default': 4}, reports, verify_key=rng.randbytes(32), trace=trace)
    assert [t.n_valid for t in trace[:2]] == [7, 7]
    assert all(t.n_valid == 6 for t in trace[2:] if t.prefixes)
    assert hh == []  # 101101 falls to 3 copies
    assert np.all(np.array([t.n_valid for t in trace]) <= 7)


class _TotalAtLeast:
    """Threshold on a vector-valued aggregate (Histogram): its total."""

    def __init__(self, t):
        self.t = t

    def __le__(self, other):  # `count >= threshold` with count a list
        return sum(other) >= self.t


def test_sweep_joint_rand_confirmation_drops_report():
    """prep_next's joint-rand confirmation (mastic.py:364-377, examples.py:67):
    a report whose leader input share carries a corrupted peer joint-rand part
    (mastic.py:516-529) derives a joint-rand seed that differs from the prep
    message; the batched check flags exactly that report and the sweep drops
    it from every level."""
    from mastic_amd import MasticHistogram
    from mastic_amd.heavy_hitters import compute_heavy_hitters, joint_rand_confirmed
    bits = 4
    mastic = MasticHistogram(bits, 4, 2)
    assert mastic.JOINT_RAND_LEN > 0
    ctx = b'jr'
    rng = random.Random(13)
    meas = [(index(0b1011, bits), 2)] * 5 + [(index(0b0100, bits), 1)] * 4
    reports = _reports(mastic, ctx, meas, rng)
    (nonce, pub, ins) = reports[0]
    (key, proof_share, seed, peer) = ins[0]
    ins = [(key, proof_share, seed, bytes([peer[0] ^ 0x80]) + peer[1:]), ins[1]]
    reports[0] = (nonce, pub, ins)
    # the batched pieces directly: the confirmation fails for report 0 only
    from mastic_amd.heavy_hitters import _encode_reports
    dev = mastic.reports_upload(*_encode_reports(mastic, reports))
    vk = rng.randbytes(16)
    ap = (0, ((False,), (True,)), True)
    enc = mastic.encode_agg_param(ap)
    sh = []
    for a in range(2):
        mastic.prep_init_device(dev, vk, ctx, a, enc)
        sh.append(mastic.prep_result(dev, a, enc))
    (msgs, _valid) = mastic.decide_batch(ctx, enc, sh[0][0], sh[1][0])
    ok = joint_rand_confirmed(msgs, sh[0][1], sh[1][1], len(meas))
    assert list(ok) == [False] + [True] * (len(meas) - 1)
    trace = []
    hh = compute_heavy_hitters(mastic, ctx, {'default': _TotalAtLeast(4)}, dev, verify_key=vk, trace=trace)
    assert all(t.n_valid == len(meas) - 1 for t in trace if t.prefixes)
    assert hh == [index(0b0100, bits), index(0b1011, bits)]


@pytest.mark.parametrize("circuit", ["Count", "Histogram"])
def test_sweep_without_reports_keeps_every_candidate_at_threshold_zero(circuit):
    """No reports and threshold 0: every candidate's aggregate is agg_init's
    zero, which reaches the threshold, so every prefix survives every level
    (examples.py:80-90).  The lazy path (packed candidates, no trace) and the
    tuple path (with a trace) agree."""
    from mastic_amd import MasticCount, MasticHistogram
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    bits = 3
    mastic = MasticCount(bits) if circuit == "Count" else MasticHistogram(bits, 3, 2)
    th = {'default': 0} if circuit == "Count" else {'default': _TotalAtLeast(0)}
    lazy = compute_heavy_hitters(mastic, b'none', th, [], verify_key=bytes(16))
    trace = []
    full = compute_heavy_hitters(mastic, b'none', th, [], verify_key=bytes(16), trace=trace)
    want = [index(v, bits) for v in range(2 ** bits)]
    assert lazy == full == want
    assert [len(t.prefixes) for t in trace] == [2, 4, 8]
