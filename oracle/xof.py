"""XOFs (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates ``vdaf_poc.xof`` at draft-irtf-cfrg-vdaf-13, as called by the
reference at ``poc/vidpf.py:339,361,377`` and ``poc/mastic.py:70,277-306,452-510``
(SURVEY.md §8a rows a18, a19):

* ``XofTurboShake128(seed, dst, binder)``: message
  ``le16(len(dst)) || dst || u8(len(seed)) || seed || binder``, stream =
  TurboSHAKE128(message, D=0x01); SEED_SIZE 32.
* ``XofFixedKeyAes128(seed, dst, binder)``: fixed key
  ``TurboSHAKE128(le16(len(dst)) || dst || binder, D=0x02, 16)``; block i is
  ``AES_k(sigma(x)) XOR sigma(x)`` with ``x = seed XOR le128(i)`` and
  ``sigma(x) = x[8:16] || (x[8:16] XOR x[0:8])``; SEED_SIZE 16.
* ``next_vec`` reads ENCODED_SIZE little-endian bytes at a time and rejects
  values >= p (the power-of-two mask is a no-op for both fields).
"""
from . import _prims
from .common import from_le_bytes, to_le_bytes


class _XofBase:
    SEED_SIZE = 0

    def next(self, length: int) -> bytes:
        raise NotImplementedError

    def next_vec(self, field, length: int):
        mask = (1 << (field.MODULUS - 1).bit_length()) - 1
        out = []
        while len(out) < length:
            x = from_le_bytes(self.next(field.ENCODED_SIZE)) & mask
            if x < field.MODULUS:
                out.append(field(x))
        return out

    @classmethod
    def derive_seed(cls, seed: bytes, dst: bytes, binder: bytes) -> bytes:
        return cls(seed, dst, binder).next(cls.SEED_SIZE)

    @classmethod
    def expand_into_vec(cls, field, seed: bytes, dst: bytes, binder: bytes, length: int):
        return cls(seed, dst, binder).next_vec(field, length)


class XofTurboShake128(_XofBase):
    SEED_SIZE = 32

    def __init__(self, seed: bytes, dst: bytes, binder: bytes):
        self._msg = to_le_bytes(len(dst), 2) + dst + to_le_bytes(len(seed), 1) + seed + binder
        self._stream = b""
        self._pos = 0

    def next(self, length: int) -> bytes:
        need = self._pos + length
        if need > len(self._stream):
            # Squeeze generously; TurboSHAKE output is a prefix-stable stream.
            n = max(need, 2 * len(self._stream), 168)
            self._stream = _prims.turboshake128(self._msg, 1, n)
        out = self._stream[self._pos:need]
        self._pos = need
        return out


class XofFixedKeyAes128(_XofBase):
    SEED_SIZE = 16
    _key_cache: dict = {}

    def __init__(self, seed: bytes, dst: bytes, binder: bytes):
        if len(seed) != self.SEED_SIZE:
            raise ValueError("incorrect seed size")
        key_msg = to_le_bytes(len(dst), 2) + dst + binder
        rk = self._key_cache.get(key_msg)
        if rk is None:
            rk = _prims.aes128_expand(_prims.turboshake128(key_msg, 2, 16))
            if len(self._key_cache) > 4096:
                self._key_cache.clear()
            self._key_cache[key_msg] = rk
        self._rk = rk
        self._seed = seed
        self._consumed = 0

    def next(self, length: int) -> bytes:
        start = self._consumed
        end = start + length
        first_block = start // 16
        last_block = (end + 15) // 16
        data = _prims.fixed_key_aes_blocks(self._rk, self._seed, first_block,
                                           last_block - first_block)
        self._consumed = end
        off = start - 16 * first_block
        return data[off:off + length]
