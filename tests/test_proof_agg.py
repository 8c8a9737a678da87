"""Host logic of the proof-aggregation traversal (mastic_amd.proof_agg) on
CPU, over trees built with the oracle's XofTurboShake128 (the GPU tree is
checked against the same construction in test_gpu_proof_agg.py)."""
import random

import pytest

from conftest import PKG_ROOT  # noqa: F401  (puts the package on sys.path)
from mastic_amd.proof_agg import isolate_invalid, level_sizes


def _tree(leaves, ctx=b"ctx"):
    from oracle.xof import XofTurboShake128
    dst = b"mastic" + bytes([0, 12]) + ctx
    levels = [list(leaves)]
    while len(levels[-1]) > 1:
        cur = levels[-1]
        levels.append([XofTurboShake128(b"", dst, cur[i] + cur[i + 1]).next(32) if i + 1 < len(cur) else cur[i]
                       for i in range(0, len(cur), 2)])
    return levels if leaves else []


def test_level_sizes():
    assert level_sizes(0) == []
    assert level_sizes(1) == [1]
    assert level_sizes(5) == [5, 3, 2, 1]
    assert level_sizes(8) == [8, 4, 2, 1]
    for n in range(1, 70):
        assert [len(x) for x in _tree([bytes(32)] * n)] == level_sizes(n)


@pytest.mark.parametrize("n,k", [(1, 0), (1, 1), (2, 1), (13, 0), (13, 2), (64, 5), (100, 100)])
def test_isolate_finds_exactly_the_differing_leaves(n, k):
    rng = random.Random(n * 131 + k)
    a = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]
    bad = sorted(rng.sample(range(n), k))
    b = [bytes(x ^ 0xFF for x in a[i]) if i in bad else a[i] for i in range(n)]
    (found, sent, rounds) = isolate_invalid(_tree(a), _tree(b))
    assert found == bad
    if not bad:
        assert sent == 1 and rounds == 1
    else:
        assert rounds == len(level_sizes(n))
        assert sent <= 1 + 2 * len(bad) * len(level_sizes(n))


def test_isolate_rejects_shape_mismatch():
    with pytest.raises(ValueError):
        isolate_invalid(_tree([bytes(32)] * 3), _tree([bytes(32)] * 4))
