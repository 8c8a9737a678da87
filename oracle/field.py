"""Prime fields Field64 / Field128 (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates ``vdaf_poc.field`` (draft-irtf-cfrg-vdaf-13) as used by the
reference at ``poc/vidpf.py:8,363,391`` and ``poc/mastic.py:8,270,296,381,540``:

* Field64:  p = 2^32 * (2^32 - 1) + 1 = 2^64 - 2^32 + 1, ENCODED_SIZE 8,
            GEN_ORDER 2^32, generator 7^(2^32 - 1).
* Field128: p = 2^66 * (2^62 - 7) + 1 = 2^128 - 28 * 2^64 + 1, ENCODED_SIZE 16,
            GEN_ORDER 2^66, generator 7^(2^62 - 7).

Elements encode little-endian (``encode_vec``).  ``encode_into_bit_vector`` /
``decode_from_bit_vector`` are LSB-first.
"""
from .common import from_le_bytes, to_le_bytes


class _Field:
    MODULUS: int = 0
    ENCODED_SIZE: int = 0
    GEN_ORDER: int = 0
    _GEN_BASE_EXP: int = 0
    __slots__ = ("val",)

    def __init__(self, val):
        self.val = int(val) % self.MODULUS

    # --- arithmetic -------------------------------------------------
    def __add__(self, other):
        return self.__class__(self.val + other.val)

    def __sub__(self, other):
        return self.__class__(self.val - other.val)

    def __mul__(self, other):
        return self.__class__(self.val * other.val)

    def __neg__(self):
        return self.__class__(-self.val)

    def __pow__(self, e: int):
        return self.__class__(pow(self.val, e, self.MODULUS))

    def inv(self):
        return self.__class__(pow(self.val, self.MODULUS - 2, self.MODULUS))

    def __eq__(self, other):
        return isinstance(other, _Field) and self.MODULUS == other.MODULUS and self.val == other.val

    def __hash__(self):
        return hash((self.MODULUS, self.val))

    def __repr__(self):
        return "%s(%d)" % (self.__class__.__name__, self.val)

    def int(self) -> int:
        return self.val

    # --- class helpers ----------------------------------------------
    @classmethod
    def zeros(cls, n: int):
        return [cls(0) for _ in range(n)]

    @classmethod
    def gen(cls):
        return cls(7) ** cls._GEN_BASE_EXP

    @classmethod
    def encode_vec(cls, vec) -> bytes:
        return b"".join(to_le_bytes(x.val, cls.ENCODED_SIZE) for x in vec)

    @classmethod
    def decode_vec(cls, data: bytes):
        n = cls.ENCODED_SIZE
        if len(data) % n != 0:
            raise ValueError("input length must be a multiple of the encoded size")
        out = []
        for i in range(0, len(data), n):
            x = from_le_bytes(data[i:i + n])
            if x >= cls.MODULUS:
                raise ValueError("encoded element out of range")
            out.append(cls(x))
        return out

    @classmethod
    def encode_into_bit_vector(cls, val: int, bits: int):
        if val >= 2 ** bits or val < 0:
            raise ValueError("value out of range for bit vector")
        return [cls((val >> l) & 1) for l in range(bits)]

    @classmethod
    def decode_from_bit_vector(cls, vec):
        acc = cls(0)
        for (l, bit) in enumerate(vec):
            acc += cls(1 << l) * bit
        return acc


class Field64(_Field):
    MODULUS = 2 ** 32 * 4294967295 + 1
    ENCODED_SIZE = 8
    GEN_ORDER = 2 ** 32
    _GEN_BASE_EXP = 4294967295
    __slots__ = ()


class Field128(_Field):
    MODULUS = 2 ** 66 * 4611686018427387897 + 1
    ENCODED_SIZE = 16
    GEN_ORDER = 2 ** 66
    _GEN_BASE_EXP = 4611686018427387897
    __slots__ = ()


# --- polynomial helpers used by the FLP (restating vdaf_poc.polynomial) ---

def poly_eval(field, poly, x):
    acc = field(0)
    for c in reversed(poly):
        acc = acc * x + c
    return acc


def poly_mul(field, a, b):
    out = [field(0) for _ in range(len(a) + len(b) - 1)]
    for (i, ai) in enumerate(a):
        if ai.val == 0:
            continue
        for (j, bj) in enumerate(b):
            out[i + j] += ai * bj
    return out


def poly_interp_roots_of_unity(field, alpha, ys):
    """Coefficients of the unique poly of degree < n with p(alpha^k) = ys[k],
    n = len(ys), alpha a primitive n-th root of unity (inverse DFT)."""
    n = len(ys)
    n_inv = field(n).inv()
    alpha_inv = alpha.inv()
    coeffs = []
    for i in range(n):
        w = alpha_inv ** i
        acc = field(0)
        wk = field(1)
        for k in range(n):
            acc += ys[k] * wk
            wk = wk * w
        coeffs.append(acc * n_inv)
    return coeffs
