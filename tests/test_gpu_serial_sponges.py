"""The measurement schedule (Mastic.set_serial_sponges, mastic_set_serial_sponges):
every binder-sponge launch runs alone on the GPU so bench.py can time the
sponge kernels and the level kernel each by itself.  It must change timing
only: a frontier-cached Sum sweep (hits and misses, both aggregators) and a
Field128 weight-check call give byte-identical traces, prep shares and out
shares with it on and off, and last_timing3 reports the sponge launches."""
import random

import numpy as np
import pytest

from test_gpu_frontier_cache import _reports
from test_gpu_parity import CTX, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu


def test_serial_sponges_sweep_identical(mastic_amd):
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    rng = random.Random(606)
    m = mastic_amd.MasticSum(10, 7)
    n = 300
    (alphas, weights, nonces, rands) = _reports(m, rng, n, 7)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    dev = m.reports_upload(nonces, pub, in0, in1)
    vk = bytes(16)
    traces = []
    for serial in (False, True, False):
        assert m.set_serial_sponges(serial) in (True, False)
        tr = []
        hh = compute_heavy_hitters(m, CTX, {"default": 40}, dev, verify_key=vk, trace=tr, frontier_cache=True)
        traces.append(([(lv.level, lv.prefixes, lv.agg_result) for lv in tr], hh))
    assert m.set_serial_sponges(None) is False
    assert traces[0] == traces[1] == traces[2]
    assert traces[0][1]


def test_serial_sponges_field128_call_identical(mastic_amd):
    rng = random.Random(607)
    m = mastic_amd.MasticHistogram(8, 5, 2)
    n = 130
    alphas = [tuple(bool(rng.getrandbits(1)) for _ in range(8)) for _ in range(n)]
    weights = [rng.randrange(5) for _ in range(n)]
    nonces = rng.randbytes(16 * n)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rng.randbytes(m.RAND_SIZE * n))
    ap = (5, tuple(sorted(set(a[:6] for a in alphas))), True)
    vk = rng.randbytes(32)
    res = []
    for serial in (False, True):
        m.set_serial_sponges(serial)
        res.append([m.prep_init_batch(vk, CTX, a, ap, nonces, pub, in0 if a == 0 else in1) for a in range(2)])
        t = m.last_timing3()
        assert t[5] > 0 and all(np.isfinite(x) for x in t)
    m.set_serial_sponges(False)
    for a in range(2):
        assert res[0][a][0] == res[1][a][0] and res[0][a][2] == res[1][a][2]
        assert list(res[0][a][3]) == list(res[1][a][3]) == [0] * n
