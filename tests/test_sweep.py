"""Heavy-hitters sweep driver: host logic on CPU.

The sweep loop is checked with a stand-in aggregator that returns plaintext
per-prefix sums, against the plaintext functionality of the reference's
``talks/func.py:49-80`` (``mastic_func`` / ``weighted_heavy_hitters``),
restated below.  The GPU run of the same driver is in test_gpu_sweep.py.
"""
import random

import numpy as np
import pytest

from conftest import PKG_ROOT  # noqa: F401  (puts the package on sys.path)
from mastic_amd.heavy_hitters import compute_heavy_hitters, get_threshold


def index(value, length):
    return tuple((value >> (length - 1 - i)) & 1 != 0 for i in range(length))


def plain_sums(measurements, prefixes):
    """talks/func.py:49-60: total weight per prefix."""
    return [sum(w for (a, w) in measurements if a[:len(p)] == p) for p in prefixes]


def plain_heavy_hitters(measurements, thresholds, bits):
    """poc/examples.py:37-91 on plaintext (talks/func.py:62-80 with per-prefix thresholds)."""
    prefixes = [(False,), (True,)]
    out = []
    for level in range(bits):
        sums = plain_sums(measurements, prefixes)
        nxt = []
        for (p, s) in zip(prefixes, sums):
            if s >= get_threshold(thresholds, p):
                if level < bits - 1:
                    nxt += [p + (False,), p + (True,)]
                else:
                    out.append(p)
        prefixes = nxt
    return out


class _StubReports:
    def __init__(self, meas):
        self.meas = meas
        self.n = len(meas)


class _StubMastic:
    """Stands in for mastic_amd.Mastic: 'shares' are the plaintext sums for
    aggregator 0 and zeros for aggregator 1; ``bad`` reports fail decide from
    level ``bad_level`` on."""
    VERIFY_KEY_SIZE = 32
    OUTPUT_LEN = 0
    JOINT_RAND_LEN = 0

    def __init__(self, bits, bad=(), bad_level=0):
        class V:
            BITS = bits
        self.vidpf = V()
        self.bad = set(bad)
        self.bad_level = bad_level
        self.calls = []

    def is_valid(self, agg_param, prev):
        wc = (agg_param[2] and not prev) or (not agg_param[2] and any(p[2] for p in prev))
        return wc and (not prev or agg_param[0] > prev[-1][0])

    def encode_agg_param(self, agg_param):
        return agg_param  # the stub's batch calls take the tuple itself

    def prep_init_device(self, dev, vk, ctx, agg_id, agg_param):
        self.calls.append((agg_id, agg_param[0], len(agg_param[1])))
        self._dev, self._ap = dev, agg_param

    def prep_result(self, dev, agg_id, agg_param):
        return (agg_id, None, None, np.zeros(dev.n, np.int32))

    def decide_batch(self, ctx, agg_param, ps0, ps1):
        lvl = agg_param[0]
        v = np.array([0 if (i in self.bad and lvl >= self.bad_level) else 1 for i in range(self._dev.n)], np.uint8)
        return (b"", v)

    def aggregate_device(self, agg_id, agg_param, mask):
        if agg_id == 1:
            return [0] * len(agg_param[1])
        meas = [m for (m, k) in zip(self._dev.meas, mask) if k]
        return plain_sums(meas, agg_param[1])

    def agg_init(self, agg_param):
        return [0] * len(agg_param[1])

    def unshard(self, agg_param, agg_shares, n):
        return [a + b for (a, b) in zip(*agg_shares)]


def test_get_threshold_semantics():
    """poc/examples.py:26-34: the prefix itself is never looked up; the longest
    listed proper prefix wins; else the default."""
    th = {'default': 2, index(0b00, 2): 1, index(0b10, 2): 3, index(0b11, 2): 5}
    assert get_threshold(th, index(0b0, 1)) == 2
    assert get_threshold(th, index(0b00, 2)) == 2          # itself excluded
    assert get_threshold(th, index(0b001, 3)) == 1
    assert get_threshold(th, index(0b1011, 4)) == 3
    assert get_threshold(th, index(0b1111, 4)) == 5
    assert get_threshold(th, index(0b0111, 4)) == 2


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sweep_logic_matches_plaintext(seed):
    rng = random.Random(seed)
    bits = 8
    heavy = [rng.randrange(2 ** bits) for _ in range(4)]
    meas = []
    for _ in range(300):
        v = rng.choice(heavy) if rng.random() < 0.6 else rng.randrange(2 ** bits)
        meas.append((index(v, bits), rng.randrange(0, 3)))
    th = {'default': 12, index(0b1, 1): 20}
    m = _StubMastic(bits)
    got = compute_heavy_hitters(m, b"ctx", th, _StubReports(meas), verify_key=bytes(32))
    assert got == plain_heavy_hitters(meas, th, bits)
    assert got, "workload should have heavy hitters"
    # one prep_init per aggregator per level, weight check only at level 0
    assert [c[1] for c in m.calls] == [l for l in range(bits) for _ in range(2)]


def test_sweep_drops_reports_failing_later_levels():
    bits = 6
    meas = [(index(0b101010, bits), 1)] * 5 + [(index(0b000111, bits), 1)] * 3
    trace = []
    m = _StubMastic(bits, bad=(0, 1, 2), bad_level=3)
    got = compute_heavy_hitters(m, b"ctx", {'default': 3}, _StubReports(meas), verify_key=bytes(32),
                                trace=trace)
    # after level 3 only two copies of 101010 remain valid: below threshold
    assert got == [index(0b000111, bits)]
    assert [t.n_valid for t in trace] == [8, 8, 8, 5, 5, 5]


def test_sweep_empty_frontier():
    bits = 5
    meas = [(index(i, bits), 1) for i in range(8)]
    trace = []
    m = _StubMastic(bits)
    assert compute_heavy_hitters(m, b"ctx", {'default': 100}, _StubReports(meas), verify_key=bytes(32),
                                 trace=trace) == []
    assert len(trace) == bits and trace[1].prefixes == []
    assert len(m.calls) == 2  # nothing is prepared once the frontier is empty


def test_child_packing_matches_pack_path():
    """The sweep driver's incremental prefix packing equals the MSB-first
    packing of the whole prefix (PrefixTreeIndex.encode, vidpf.py:33-39)."""
    from mastic_amd.heavy_hitters import _child_packed
    from mastic_amd.vdaf import _pack_path
    rng = random.Random(5)
    for length in range(1, 260):
        prefix = tuple(bool(rng.getrandbits(1)) for _ in range(length))
        for bit in (False, True):
            assert _child_packed(_pack_path(prefix), length, bit) == _pack_path(prefix + (bit,))


def test_joint_rand_confirmation_mask():
    """prep_next's check (mastic.py:369-375) for both aggregators, batched."""
    from mastic_amd.heavy_hitters import joint_rand_confirmed
    rng = random.Random(9)
    n = 5
    msgs = bytes(rng.getrandbits(8) for _ in range(32 * n))
    j0 = bytearray(msgs)
    j1 = bytearray(msgs)
    j0[32 * 1 + 7] ^= 1      # report 1: leader's seed differs
    j1[32 * 3 + 31] ^= 0x40  # report 3: helper's seed differs
    assert list(joint_rand_confirmed(msgs, bytes(j0), bytes(j1), n)) == [True, False, True, False, True]
    assert len(joint_rand_confirmed(b"", b"", b"", 0)) == 0
