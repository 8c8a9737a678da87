"""Byte / vector helpers (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates the helpers the reference imports from ``vdaf_poc.common``
(``poc/vidpf.py:7``, ``poc/mastic.py:6-7``, ``poc/dst.py:6``) and
``vdaf_poc.idpf_bbcggi21.pack_bits`` (``poc/vidpf.py:9,387``).
"""


def byte(x: int) -> bytes:
    return bytes([x])


def to_le_bytes(x: int, n: int) -> bytes:
    return int(x).to_bytes(n, "little")


def to_be_bytes(x: int, n: int) -> bytes:
    return int(x).to_bytes(n, "big")


def from_le_bytes(b: bytes) -> int:
    return int.from_bytes(b, "little")


def from_be_bytes(b: bytes) -> int:
    return int.from_bytes(b, "big")


def xor(a: bytes, b: bytes) -> bytes:
    assert len(a) == len(b)
    return bytes(x ^ y for (x, y) in zip(a, b))


def front(n, v):
    return (v[:n], v[n:])


def concat(parts) -> bytes:
    return b"".join(parts)


def vec_add(a, b):
    assert len(a) == len(b)
    return [x + y for (x, y) in zip(a, b)]


def vec_sub(a, b):
    assert len(a) == len(b)
    return [x - y for (x, y) in zip(a, b)]


def vec_neg(a):
    return [-x for x in a]


def next_power_of_2(n: int) -> int:
    assert n > 0
    return 1 << (n - 1).bit_length()


def pack_bits(bits) -> bytes:
    """LSB-first packing of control bits (idpf_bbcggi21.pack_bits)."""
    out = bytearray((len(bits) + 7) // 8)
    for (i, bit) in enumerate(bits):
        out[i // 8] |= int(bool(bit)) << (i % 8)
    return bytes(out)


def unpack_bits(data: bytes, n: int) -> list:
    return [bool((data[i // 8] >> (i % 8)) & 1) for i in range(n)]


def encode_path_msb_first(path) -> bytes:
    """MSB-first bit packing used by PrefixTreeIndex.encode (poc/vidpf.py:33-39)
    and Mastic.encode_agg_param (poc/mastic.py:424-429)."""
    out = bytearray((len(path) + 7) // 8)
    for (i, bit) in enumerate(path):
        out[i // 8] |= int(bool(bit)) << (7 - (i % 8))
    return bytes(out)


def decode_path_msb_first(data: bytes, nbits: int) -> tuple:
    return tuple(bool((data[i // 8] >> (7 - (i % 8))) & 1) for i in range(nbits))
