"""FLP of [BBCGGI19] (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates ``vdaf_poc.flp_bbcggi19`` at draft-irtf-cfrg-vdaf-13 as used by the
reference (``poc/mastic.py:9-10,85,118,126,250-256,314,349,410,574-614``).
Conventions (SURVEY.md §8a "FLP conventions [V]"):

* proof = per gadget ``wire_seeds[ARITY] || gadget_poly[DEGREE*(P-1)+1]``,
  ``P = next_pow2(1 + CALLS)``, ``alpha = gen^(GEN_ORDER / P)``;
* wire j of a gadget holds ``seed_j`` at alpha^0 and the j-th input of call k at
  alpha^k (k = 1..CALLS), zero elsewhere;
* query: call k of a gadget returns ``gadget_poly(alpha^k)``; the circuit
  output is reduced by the first EVAL_OUTPUT_LEN query rands when
  EVAL_OUTPUT_LEN > 1; the next query rand per gadget is the test point t
  (abort if ``t^P == 1``); verifier = ``[v] + per gadget [wire_j(t)..., gadget_poly(t)]``;
* constants inside the circuits are scaled by ``1/num_shares``.
"""
from .common import front, next_power_of_2
from .field import poly_eval, poly_interp_roots_of_unity, poly_mul


# ---------------------------------------------------------------- gadgets

class Mul:
    ARITY = 2
    DEGREE = 2

    def eval(self, field, inp):
        return inp[0] * inp[1]

    def eval_poly(self, field, polys):
        return poly_mul(field, polys[0], polys[1])


class Range2:
    """x^2 - x"""
    ARITY = 1
    DEGREE = 2

    def eval(self, field, inp):
        return inp[0] * inp[0] - inp[0]

    def eval_poly(self, field, polys):
        sq = poly_mul(field, polys[0], polys[0])
        for (i, c) in enumerate(polys[0]):
            sq[i] = sq[i] - c
        return sq


class ParallelSum:
    def __init__(self, inner, count):
        self.inner = inner
        self.count = count
        self.ARITY = inner.ARITY * count
        self.DEGREE = inner.DEGREE

    def eval(self, field, inp):
        a = self.inner.ARITY
        acc = field(0)
        for i in range(self.count):
            acc += self.inner.eval(field, inp[i * a:(i + 1) * a])
        return acc

    def eval_poly(self, field, polys):
        a = self.inner.ARITY
        acc = None
        for i in range(self.count):
            p = self.inner.eval_poly(field, polys[i * a:(i + 1) * a])
            if acc is None:
                acc = p
            else:
                for (j, c) in enumerate(p):
                    acc[j] += c
        return acc


# --------------------------------------------------------------- circuits

class Valid:
    field = None
    GADGETS: list = []
    GADGET_CALLS: list = []
    MEAS_LEN = 0
    JOINT_RAND_LEN = 0
    OUTPUT_LEN = 0
    EVAL_OUTPUT_LEN = 0

    def prove_rand_len(self):
        return sum(g.ARITY for g in self.GADGETS)

    def query_rand_len(self):
        n = len(self.GADGETS)
        if self.EVAL_OUTPUT_LEN > 1:
            n += self.EVAL_OUTPUT_LEN
        return n

    def proof_len(self):
        n = 0
        for (g, calls) in zip(self.GADGETS, self.GADGET_CALLS):
            p = next_power_of_2(1 + calls)
            n += g.ARITY + g.DEGREE * (p - 1) + 1
        return n

    def verifier_len(self):
        return 1 + sum(g.ARITY + 1 for g in self.GADGETS)

    def test_vec_set_type_param(self, test_vec):
        return []


def _range_check_chunks(valid, gadget, meas, joint_rand, shares_inv, calls, chunk):
    """sum_i G(r_i^1 m_{i,0}, m_{i,0} - 1/s, r_i^2 m_{i,1}, ...) (SumVec/Histogram/Multihot)."""
    field = valid.field
    acc = field(0)
    for i in range(calls):
        r = joint_rand[i]
        rp = r
        inp = []
        for j in range(chunk):
            idx = i * chunk + j
            m = meas[idx] if idx < len(meas) else field(0)
            inp.append(rp * m)
            inp.append(m - shares_inv)
            rp = rp * r
        acc += gadget.eval(field, inp)
    return acc


class Count(Valid):
    def __init__(self, field):
        self.field = field
        self.GADGETS = [Mul()]
        self.GADGET_CALLS = [1]
        self.MEAS_LEN = 1
        self.JOINT_RAND_LEN = 0
        self.OUTPUT_LEN = 1
        self.EVAL_OUTPUT_LEN = 1

    def eval(self, meas, joint_rand, num_shares):
        return [self.GADGETS[0].eval(self.field, [meas[0], meas[0]]) - meas[0]]

    def encode(self, measurement):
        return [self.field(int(measurement))]

    def truncate(self, meas):
        return meas

    def decode(self, output, num_measurements):
        return output[0].int()


class Sum(Valid):
    def __init__(self, field, max_measurement):
        self.field = field
        self.max_measurement = max_measurement
        self.bits = max_measurement.bit_length()
        self.offset = field(2 ** self.bits - 1 - max_measurement)
        self.GADGETS = [Range2()]
        self.GADGET_CALLS = [2 * self.bits]
        self.MEAS_LEN = 2 * self.bits
        self.JOINT_RAND_LEN = 0
        self.OUTPUT_LEN = 1
        self.EVAL_OUTPUT_LEN = 2 * self.bits + 1

    def eval(self, meas, joint_rand, num_shares):
        f = self.field
        shares_inv = f(num_shares).inv()
        out = [self.GADGETS[0].eval(f, [b]) for b in meas]
        out.append(self.offset * shares_inv
                   + f.decode_from_bit_vector(meas[:self.bits])
                   - f.decode_from_bit_vector(meas[self.bits:]))
        return out

    def encode(self, measurement):
        if measurement < 0 or measurement > self.max_measurement:
            raise ValueError("measurement out of range")
        return (self.field.encode_into_bit_vector(measurement, self.bits)
                + self.field.encode_into_bit_vector(measurement + self.offset.int(), self.bits))

    def truncate(self, meas):
        return [self.field.decode_from_bit_vector(meas[:self.bits])]

    def decode(self, output, num_measurements):
        return output[0].int()

    def test_vec_set_type_param(self, test_vec):
        test_vec["max_measurement"] = int(self.max_measurement)
        return ["max_measurement"]


class SumVec(Valid):
    def __init__(self, field, length, bits, chunk_length):
        self.field = field
        self.length = length
        self.bits = bits
        self.chunk_length = chunk_length
        self.GADGETS = [ParallelSum(Mul(), chunk_length)]
        self.GADGET_CALLS = [(length * bits + chunk_length - 1) // chunk_length]
        self.MEAS_LEN = length * bits
        self.JOINT_RAND_LEN = self.GADGET_CALLS[0]
        self.OUTPUT_LEN = length
        self.EVAL_OUTPUT_LEN = 1

    def eval(self, meas, joint_rand, num_shares):
        shares_inv = self.field(num_shares).inv()
        return [_range_check_chunks(self, self.GADGETS[0], meas, joint_rand, shares_inv,
                                    self.GADGET_CALLS[0], self.chunk_length)]

    def encode(self, measurement):
        if len(measurement) != self.length:
            raise ValueError("incorrect measurement length")
        out = []
        for v in measurement:
            out += self.field.encode_into_bit_vector(int(v), self.bits)
        return out

    def truncate(self, meas):
        return [self.field.decode_from_bit_vector(meas[i * self.bits:(i + 1) * self.bits])
                for i in range(self.length)]

    def decode(self, output, num_measurements):
        return [x.int() for x in output]

    def test_vec_set_type_param(self, test_vec):
        test_vec["length"] = int(self.length)
        test_vec["bits"] = int(self.bits)
        test_vec["chunk_length"] = int(self.chunk_length)
        return ["length", "bits", "chunk_length"]


class Histogram(Valid):
    def __init__(self, field, length, chunk_length):
        self.field = field
        self.length = length
        self.chunk_length = chunk_length
        self.GADGETS = [ParallelSum(Mul(), chunk_length)]
        self.GADGET_CALLS = [(length + chunk_length - 1) // chunk_length]
        self.MEAS_LEN = length
        self.JOINT_RAND_LEN = self.GADGET_CALLS[0]
        self.OUTPUT_LEN = length
        self.EVAL_OUTPUT_LEN = 2

    def eval(self, meas, joint_rand, num_shares):
        shares_inv = self.field(num_shares).inv()
        range_check = _range_check_chunks(self, self.GADGETS[0], meas, joint_rand, shares_inv,
                                          self.GADGET_CALLS[0], self.chunk_length)
        sum_check = -shares_inv
        for b in meas:
            sum_check += b
        return [range_check, sum_check]

    def encode(self, measurement):
        if measurement < 0 or measurement >= self.length:
            raise ValueError("bucket out of range")
        out = self.field.zeros(self.length)
        out[measurement] = self.field(1)
        return out

    def truncate(self, meas):
        return meas

    def decode(self, output, num_measurements):
        return [x.int() for x in output]

    def test_vec_set_type_param(self, test_vec):
        test_vec["length"] = int(self.length)
        test_vec["chunk_length"] = int(self.chunk_length)
        return ["length", "chunk_length"]


class MultihotCountVec(Valid):
    def __init__(self, field, length, max_weight, chunk_length):
        self.field = field
        self.length = length
        self.max_weight = max_weight
        self.chunk_length = chunk_length
        self.bits_for_weight = max_weight.bit_length()
        self.offset = field(2 ** self.bits_for_weight - 1 - max_weight)
        self.GADGETS = [ParallelSum(Mul(), chunk_length)]
        self.GADGET_CALLS = [(length + self.bits_for_weight + chunk_length - 1) // chunk_length]
        self.MEAS_LEN = length + self.bits_for_weight
        self.JOINT_RAND_LEN = self.GADGET_CALLS[0]
        self.OUTPUT_LEN = length
        self.EVAL_OUTPUT_LEN = 2

    def eval(self, meas, joint_rand, num_shares):
        f = self.field
        shares_inv = f(num_shares).inv()
        range_check = _range_check_chunks(self, self.GADGETS[0], meas, joint_rand, shares_inv,
                                          self.GADGET_CALLS[0], self.chunk_length)
        weight = f(0)
        for b in meas[:self.length]:
            weight += b
        reported = f.decode_from_bit_vector(meas[self.length:])
        return [range_check, self.offset * shares_inv + weight - reported]

    def encode(self, measurement):
        if len(measurement) != self.length:
            raise ValueError("incorrect measurement length")
        total = sum(int(bool(x)) for x in measurement)
        if total > self.max_weight:
            raise ValueError("measurement weight too large")
        return ([self.field(int(bool(x))) for x in measurement]
                + self.field.encode_into_bit_vector(self.offset.int() + total, self.bits_for_weight))

    def truncate(self, meas):
        return meas[:self.length]

    def decode(self, output, num_measurements):
        return [x.int() for x in output]

    def test_vec_set_type_param(self, test_vec):
        test_vec["length"] = int(self.length)
        test_vec["max_weight"] = int(self.max_weight)
        test_vec["chunk_length"] = int(self.chunk_length)
        return ["length", "max_weight", "chunk_length"]


# ---------------------------------------------------------------- the FLP

class _RecordingGadget:
    """Wraps a gadget for prove (records inputs) or query (also answers from
    the gadget polynomial)."""

    def __init__(self, field, inner, calls, seeds, poly=None):
        self.inner = inner
        self.ARITY = inner.ARITY
        self.DEGREE = inner.DEGREE
        self.p = next_power_of_2(1 + calls)
        self.alpha = field.gen() ** (field.GEN_ORDER // self.p)
        self.wires = []
        for s in seeds:
            w = field.zeros(self.p)
            w[0] = s
            self.wires.append(w)
        self.poly = poly
        self.k = 0

    def eval(self, field, inp):
        self.k += 1
        for (j, x) in enumerate(inp):
            self.wires[j][self.k] = x
        if self.poly is None:
            return self.inner.eval(field, inp)
        return poly_eval(field, self.poly, self.alpha ** self.k)


class FlpBBCGGI19:
    def __init__(self, valid):
        self.valid = valid
        self.field = valid.field
        self.MEAS_LEN = valid.MEAS_LEN
        self.OUTPUT_LEN = valid.OUTPUT_LEN
        self.JOINT_RAND_LEN = valid.JOINT_RAND_LEN
        self.PROVE_RAND_LEN = valid.prove_rand_len()
        self.QUERY_RAND_LEN = valid.query_rand_len()
        self.PROOF_LEN = valid.proof_len()
        self.VERIFIER_LEN = valid.verifier_len()

    def _run(self, meas, joint_rand, num_shares, gadgets):
        saved = self.valid.GADGETS
        self.valid.GADGETS = gadgets
        try:
            return self.valid.eval(meas, joint_rand, num_shares)
        finally:
            self.valid.GADGETS = saved

    def prove(self, meas, prove_rand, joint_rand):
        f = self.field
        wrapped = []
        i = 0
        for (g, calls) in zip(self.valid.GADGETS, self.valid.GADGET_CALLS):
            wrapped.append(_RecordingGadget(f, g, calls, prove_rand[i:i + g.ARITY]))
            i += g.ARITY
        self._run(meas, joint_rand, 1, wrapped)
        proof = []
        for w in wrapped:
            wire_polys = [poly_interp_roots_of_unity(f, w.alpha, wire) for wire in w.wires]
            gpoly = w.inner.eval_poly(f, wire_polys)
            glen = w.DEGREE * (w.p - 1) + 1
            gpoly = (gpoly + f.zeros(glen))[:glen]
            proof += [wire[0] for wire in w.wires]
            proof += gpoly
        return proof

    def query(self, meas, proof, query_rand, joint_rand, num_shares):
        f = self.field
        wrapped = []
        rest = proof
        for (g, calls) in zip(self.valid.GADGETS, self.valid.GADGET_CALLS):
            p = next_power_of_2(1 + calls)
            (seeds, rest) = front(g.ARITY, rest)
            (poly, rest) = front(g.DEGREE * (p - 1) + 1, rest)
            wrapped.append(_RecordingGadget(f, g, calls, seeds, poly))
        out = self._run(meas, joint_rand, num_shares, wrapped)
        if len(out) != self.valid.EVAL_OUTPUT_LEN:
            raise ValueError("circuit output length mismatch")
        if self.valid.EVAL_OUTPUT_LEN > 1:
            (rand, query_rand) = front(self.valid.EVAL_OUTPUT_LEN, query_rand)
            v = f(0)
            for (r, o) in zip(rand, out):
                v += r * o
        else:
            v = out[0]
        verifier = [v]
        for (w, t) in zip(wrapped, query_rand):
            if t ** w.p == f(1):
                raise ValueError("test point is a root of unity")
            for wire in w.wires:
                verifier.append(poly_eval(f, poly_interp_roots_of_unity(f, w.alpha, wire), t))
            verifier.append(poly_eval(f, w.poly, t))
        return verifier

    def decide(self, verifier):
        f = self.field
        ([v], rest) = front(1, verifier)
        if v != f(0):
            return False
        for g in self.valid.GADGETS:
            (x, rest) = front(g.ARITY, rest)
            ([y], rest) = front(1, rest)
            if g.eval(f, x) != y:
                return False
        return True

    def encode(self, measurement):
        return self.valid.encode(measurement)

    def truncate(self, meas):
        return self.valid.truncate(meas)

    def decode(self, output, num_measurements):
        return self.valid.decode(output, num_measurements)

    def test_vec_set_type_param(self, test_vec):
        return self.valid.test_vec_set_type_param(test_vec)
