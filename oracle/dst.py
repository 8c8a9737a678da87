"""Domain-separation tags (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates ``poc/dst.py:11-42``: ``dst(ctx, usage) = b'mastic' || VERSION ||
usage || ctx`` and ``dst_alg`` additionally carries ``be32(algorithm_id)``
before ``ctx``.
"""
from .common import byte, to_be_bytes

VERSION = 0                      # poc/dst.py:11

USAGE_PROVE_RAND = 0             # poc/dst.py:14-27
USAGE_PROOF_SHARE = 1
USAGE_QUERY_RAND = 2
USAGE_JOINT_RAND_SEED = 3
USAGE_JOINT_RAND_PART = 4
USAGE_JOINT_RAND = 5
USAGE_ONEHOT_CHECK = 6
USAGE_PAYLOAD_CHECK = 7
USAGE_EVAL_PROOF = 8
USAGE_NODE_PROOF = 9
USAGE_EXTEND = 10
USAGE_CONVERT = 11


def dst(ctx: bytes, usage: int) -> bytes:
    """poc/dst.py:30-32"""
    assert 0 <= usage < 12
    return b"mastic" + byte(VERSION) + byte(usage) + ctx


def dst_alg(ctx: bytes, usage: int, algorithm_id: int) -> bytes:
    """poc/dst.py:35-42"""
    assert 0 <= usage < 12
    assert 0 <= algorithm_id < 2 ** 32 - 1
    return b"mastic" + byte(VERSION) + byte(usage) + to_be_bytes(algorithm_id, 4) + ctx
