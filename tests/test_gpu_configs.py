"""GPU parity at the exact Mastic parameters of every BASELINE.json config
(SURVEY.md §8 table C1-C5), at report counts the CPU oracle finishes in
seconds.  Each case shards on the GPU, checks the public/input shares, both
aggregators' prep shares, out shares and joint-rand seeds against the oracle
bit for bit, runs the batched decide, and checks the GPU fold (agg_update)
against the oracle's agg shares and the plaintext functionality
(talks/func.py:49-80).

C1 Mastic(16, Count); C2 Mastic(32, Sum 255); C3 Mastic(256, Count);
C4 Mastic(64, Histogram 64, chunk 8) over Field128; C5 Mastic(32, SumVec 1024,
bits 1, chunk 32) over Field128.  C2 at the bench's full prefix count is
covered by test_gpu_parity.test_c2_shape_properties_and_oracle_sample.
"""
import random

import pytest

from test_gpu_parity import CTX, _check_against_oracle, _oracle_for, _random_reports, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu

CONFIGS = [
    # id, constructor kwargs, reports, [(level, prefixes, weight_check)]
    ("C1", ("Count", dict(bits=16)), 6, [(0, 2, True), (7, 12, False), (15, 40, True)]),
    ("C2", ("Sum", dict(bits=32, max_measurement=255)), 6, [(31, 64, True), (12, 9, False)]),
    ("C3", ("Count", dict(bits=256)), 4, [(255, 16, True), (100, 5, False)]),
    ("C4", ("Histogram", dict(bits=64, length=64, chunk_length=8)), 4, [(63, 8, True), (20, 3, False)]),
    ("C5", ("SumVec", dict(bits=32, length=1024, sum_vec_bits=1, chunk_length=32)), 3, [(31, 3, True)]),
]


def _agg_param(rng, alphas, bits, level, nprefix, wc):
    pre = list(dict.fromkeys(tuple(a[:level + 1]) for a in alphas))[:nprefix]
    seen = set(pre)
    while len(pre) < nprefix:
        p = tuple(bool(rng.getrandbits(1)) for _ in range(level + 1))
        if p not in seen:
            seen.add(p)
            pre.append(p)
    rng.shuffle(pre)
    return (level, tuple(pre), wc)


def _plaintext(m, alphas, weights, prefixes):
    """talks/func.py:49-80: per prefix, the sum of the (truncated) weights of
    the reports whose alpha starts with it."""
    c = m.circuit
    out = []
    for p in prefixes:
        hit = [w for (a, w) in zip(alphas, weights) if tuple(a[:len(p)]) == p]
        if c in ("Count", "Sum"):
            out.append(sum(int(w) for w in hit))
        elif c == "Histogram":
            out.append([sum(1 for w in hit if w == j) for j in range(m.length)])
        else:  # SumVec
            out.append([sum(w[j] for w in hit) for j in range(m.length)])
    return out


@pytest.mark.parametrize("cid,spec,n,params", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_config_shape_matches_oracle(mastic_amd, cid, spec, n, params):
    (circuit, kw) = spec
    kw = dict(kw)
    bits = kw.pop("bits")
    m = mastic_amd.Mastic(bits, circuit, **kw)
    o = _oracle_for(m)
    rng = random.Random(0x4D41 + int(cid[1]))
    (alphas, weights, nonces, rands) = _random_reports(m, rng, n)
    # two reports share an alpha so some prefix aggregates more than one report
    alphas[1] = alphas[0]
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    for (i, (level, nprefix, wc)) in enumerate(params):
        ap = _agg_param(rng, alphas, bits, level, nprefix, wc)
        gpu = _check_against_oracle(m, o, CTX, vk, ap, alphas, weights, nonces, rands, check_shard=(i == 0))
        # GPU fold == oracle agg_update over the oracle-checked out shares
        k = 1 + m.OUTPUT_LEN
        aggs = []
        for a in range(2):
            agg = m.aggregate_device(a, ap)
            out = gpu[a][2]
            ow = len(out) // n
            want = o.agg_init(ap)
            for r in range(n):
                want = o.agg_update(ap, want, o.field.decode_vec(out[ow * r:ow * (r + 1)]))
            assert m.field.encode_vec(agg) == o.field.encode_vec(want), "%s agg %d level %d" % (cid, a, level)
            assert len(agg) == len(ap[1]) * k
            aggs.append(agg)
        assert m.unshard(ap, aggs, n) == _plaintext(m, alphas, weights, ap[1])
