"""VIDPF-proof aggregation mode (mastic_amd.proof_agg; draft "Plain
Heavy-Hitters with VIDPF-Proof Aggregation").  The reference has no code or
wire format for it, so parity is unpinned against the reference: the GPU
Merkle tree is checked against a CPU construction with the oracle's
XofTurboShake128 (vdaf_poc restatement) and poc/dst.py's dst layout, and the
isolation result against the per-report decide of the GPU path."""
import random

import pytest

from test_gpu_parity import CTX, _oracle_for, _random_reports, _random_agg_param, mastic_amd  # noqa: F401

pytestmark = pytest.mark.gpu


def _cpu_tree(leaves, ctx):
    from oracle.dst import VERSION
    from oracle.xof import XofTurboShake128
    dst = b"mastic" + bytes([VERSION, 12]) + ctx
    levels = [list(leaves)]
    while len(levels[-1]) > 1:
        cur = levels[-1]
        nxt = []
        for i in range(0, len(cur), 2):
            if i + 1 < len(cur):
                nxt.append(XofTurboShake128(b"", dst, cur[i] + cur[i + 1]).next(32))
            else:
                nxt.append(cur[i])
        levels.append(nxt)
    return levels if leaves else []


@pytest.mark.parametrize("n", [1, 2, 77])
def test_proof_tree_matches_cpu_and_isolates_invalid(mastic_amd, n):
    from mastic_amd.proof_agg import isolate_invalid
    rng = random.Random(400 + n)
    m = mastic_amd.MasticCount(6)
    (alphas, weights, nonces, rands) = _random_reports(m, rng, n)
    (pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
    # corrupt the helper's VIDPF key of some reports: their eval proofs then
    # differ between the aggregators
    isz = m.input_share_size(1)
    bad = sorted(rng.sample(range(n), min(3, n - 1))) if n > 1 else []
    in1b = bytearray(in1)
    for i in bad:
        in1b[isz * i] ^= 0x01  # first byte of the helper's key
    ap = _random_agg_param(m, rng, alphas, 5, 4, True)
    vk = bytes(rng.getrandbits(8) for _ in range(32))
    r0 = m.prep_init_batch(vk, CTX, 0, ap, nonces, pub, in0)
    t0 = m.proof_tree(0, CTX, n)
    r1 = m.prep_init_batch(vk, CTX, 1, ap, nonces, pub, bytes(in1b))
    t1 = m.proof_tree(1, CTX, n)
    ppsz = m.prep_share_size(True)
    for (r, t) in ((r0, t0), (r1, t1)):
        leaves = [r[0][ppsz * i:ppsz * i + 32] for i in range(n)]
        assert t == _cpu_tree(leaves, CTX)
    (_msgs, valid) = m.decide_batch(CTX, ap, r0[0], r1[0])
    want = [i for i in range(n) if valid[i] != 1]
    assert want == bad
    (found, sent, rounds) = isolate_invalid(t0, t1)
    assert found == bad
    assert rounds == len(t0) or not bad
    if not bad:
        assert sent == 1 and t0[-1] == t1[-1]  # one root per batch when every report is valid
