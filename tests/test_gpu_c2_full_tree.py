"""BASELINE config C2 at its exact tree size under the oracle: Mastic(32, Sum
255), level 31 with 10,000 candidate prefixes and the weight check (the
bench's C2 agg param shape), 128 reports (both 64-report groups of the tiled
binder buffers), both aggregators.  Every prep share and every truncated out
share of the GPU path equals the native CPU restatement of prep_init
(oracle/native_prep.c: bit-exact against all nine golden vectors and the
Python oracle, tests/test_native_baseline.py), and the two aggregators'
results decide and unshard to the plaintext sums (talks/func.py:49-80).
Reference: poc/mastic.py:205-318 (prep_init), :320-362 (decide)."""
import os
import random

import numpy as np
import pytest

from test_gpu_parity import CTX, _oracle_for, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu


def _threads():
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 16))


def test_c2_full_10k_prefix_tree_equals_native_oracle(mastic_amd):
    from oracle.native import prep_init_native
    rng = random.Random(2026)
    nrng = np.random.default_rng(2026)
    m = mastic_amd.MasticSum(32, 255)
    vals = np.unique(nrng.integers(0, 2 ** 32, size=12000, dtype=np.uint64))[:10000]
    assert len(vals) == 10000
    attrs = [tuple(bool((int(v) >> (31 - b)) & 1) for b in range(32)) for v in vals]
    n = 128
    alphas = [attrs[rng.randrange(len(attrs))] if i % 8 else tuple(bool(rng.getrandbits(1)) for _ in range(32))
              for i in range(n)]  # every 8th report off the candidate list
    weights = [rng.randrange(256) for _ in range(n)]
    nonces = rng.randbytes(16 * n)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rng.randbytes(m.RAND_SIZE * n))
    ap = (31, tuple(attrs), True)
    assert m.tree_stats(ap)[0] > 100000  # nodes per report: the full C2-sized tree
    vk = rng.randbytes(16)
    o = _oracle_for(m)
    ins = (in0, in1)
    res = []
    for a in range(2):
        (gps, _jr, gout, st) = m.prep_init_batch(vk, CTX, a, ap, nonces, pub, ins[a], want_out_shares=True)
        assert list(st) == [0] * n
        (shares, outs) = prep_init_native(o, vk, CTX, a, ap, nonces, pub, ins[a], threads=_threads())
        psz = len(shares[0])
        for i in range(n):
            assert gps[psz * i:psz * (i + 1)] == shares[i], "agg %d report %d prep share" % (a, i)
        assert gout == outs, "agg %d out shares" % a
        res.append(gps)
    (_msgs, valid) = m.decide_batch(CTX, ap, res[0], res[1])
    assert list(valid) == [1] * n
    aggs = [m.aggregate_device(a, ap) for a in range(2)]
    want = {}
    for (al, w) in zip(alphas, weights):
        want[al] = want.get(al, 0) + w
    assert m.unshard(ap, aggs, n) == [want.get(p, 0) for p in ap[1]]
