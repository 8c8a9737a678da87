"""Host-side field element types of the drop-in API (Field64 / Field128 of
vdaf_poc.field, vdaf-13).  Pure bookkeeping for values crossing the API; all
bulk arithmetic on the prep path happens in the HIP kernels."""


class FieldElement:
    MODULUS = 0
    ENCODED_SIZE = 0
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = int(v) % self.MODULUS

    def int(self) -> int:
        return self.v

    def __add__(self, o):
        return type(self)(self.v + o.v)

    def __sub__(self, o):
        return type(self)(self.v - o.v)

    def __mul__(self, o):
        return type(self)(self.v * o.v)

    def __neg__(self):
        return type(self)(-self.v)

    def __eq__(self, o):
        return isinstance(o, FieldElement) and o.MODULUS == self.MODULUS and o.v == self.v

    def __hash__(self):
        return hash((self.MODULUS, self.v))

    def __repr__(self):
        return "%s(%d)" % (type(self).__name__, self.v)

    @classmethod
    def zeros(cls, n):
        return [cls(0) for _ in range(n)]

    @classmethod
    def encode_vec(cls, vec) -> bytes:
        return b"".join(x.v.to_bytes(cls.ENCODED_SIZE, "little") for x in vec)

    @classmethod
    def decode_vec(cls, data: bytes):
        n = cls.ENCODED_SIZE
        if len(data) % n:
            raise ValueError("input length must be a multiple of the encoded size")
        out = []
        for i in range(0, len(data), n):
            x = int.from_bytes(data[i:i + n], "little")
            if x >= cls.MODULUS:
                raise ValueError("encoded element out of range")
            out.append(cls(x))
        return out

    @classmethod
    def encode_into_bit_vector(cls, val: int, bits: int):
        if not 0 <= val < 2 ** bits:
            raise ValueError("value out of range for bit vector")
        return [cls((val >> i) & 1) for i in range(bits)]

    @classmethod
    def decode_from_bit_vector(cls, vec):
        return cls(sum(x.v << i for (i, x) in enumerate(vec)))


class Field64(FieldElement):
    MODULUS = 2 ** 64 - 2 ** 32 + 1
    ENCODED_SIZE = 8
    __slots__ = ()


class Field128(FieldElement):
    MODULUS = 2 ** 128 - 28 * 2 ** 64 + 1
    ENCODED_SIZE = 16
    __slots__ = ()
