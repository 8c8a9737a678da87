"""Known-answer tests for the oracle's C primitives and XOF edge cases
(the rejection-sampling branch that no reference vector reaches)."""
from oracle import _prims
from oracle.field import Field64, Field128
from oracle.xof import XofFixedKeyAes128, XofTurboShake128


def test_aes128_fips197_c1():
    rk = _prims.aes128_expand(bytes(range(16)))
    ct = _prims.aes128_encrypt(rk, bytes.fromhex("00112233445566778899aabbccddeeff"))
    assert ct.hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_turboshake128_rfc9861_empty():
    out = _prims.turboshake128(b"", 0x1F, 64)
    assert out.hex() == ("1e415f1c5983aff2169217277d17bb538cd945a397ddec541f1ce41af2c1b74c"
                         "3e8ccae2a4dae56c84a04c2385c03c15e8193bdf58737363321691c05462c8df")


def test_turboshake_stream_is_prefix_stable():
    x = XofTurboShake128(b"k" * 32, b"dst", b"binder")
    a = x.next(100) + x.next(300)
    assert a == _prims.turboshake128(b"\x03\x00dst\x20" + b"k" * 32 + b"binder", 1, 400)


def test_fixed_key_aes_stream_offsets():
    x = XofFixedKeyAes128(bytes(16), b"d", bytes(16))
    y = XofFixedKeyAes128(bytes(16), b"d", bytes(16))
    assert x.next(5) + x.next(40) + x.next(3) == y.next(48)


class _Stream:
    def __init__(self, data):
        self.data = data
        self.pos = 0

    def next(self, n):
        out = self.data[self.pos:self.pos + n]
        self.pos += n
        return out

    next_vec = XofTurboShake128.next_vec


def test_next_vec_rejects_out_of_range_field64():
    p = Field64.MODULUS
    data = (p).to_bytes(8, "little") + (p - 1).to_bytes(8, "little") + (2 ** 64 - 1).to_bytes(8, "little") \
        + (5).to_bytes(8, "little")
    assert _Stream(data).next_vec(Field64, 2) == [Field64(p - 1), Field64(5)]


def test_next_vec_rejects_out_of_range_field128():
    p = Field128.MODULUS
    data = (p + 3).to_bytes(16, "little") + (7).to_bytes(16, "little")
    assert _Stream(data).next_vec(Field128, 1) == [Field128(7)]
