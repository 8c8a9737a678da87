// Mastic instantiation parameters (poc/mastic.py:81-89, :567-614) and the
// FLP shape of each validity circuit (vdaf_poc.flp_bbcggi19, vdaf-13).
#pragma once
#ifdef __HIP__
#include "common.hpp"
#else
// host-only build of the parameter logic (tests/host/fuzz_host.cpp, sanitizers)
#include <stdint.h>
#define MH_HD inline
#endif

enum McCircuit : int {
    MC_COUNT = 1,
    MC_SUM = 2,
    MC_SUMVEC = 3,
    MC_HISTOGRAM = 4,
    MC_MULTIHOT = 5,
};

enum McGadget : int {
    G_MUL = 1,      // Mul: x*y                      (arity 2, degree 2)
    G_RANGE2 = 2,   // Range2: x^2 - x               (arity 1, degree 2)
    G_PSUM_MUL = 3, // ParallelSum(Mul, chunk)       (arity 2*chunk, degree 2)
};

struct McParams {
    int circuit;
    int bits;           // VIDPF BITS
    int field;          // 64 or 128
    int enc;            // ENCODED_SIZE
    int w32;            // 32-bit words per element
    int value_len;      // VALUE_LEN = 1 + MEAS_LEN
    int meas_len;
    int output_len;
    int eval_output_len;
    int joint_rand_len;
    int query_rand_len;
    int prove_rand_len;
    int proof_len;
    int verifier_len;
    int gadget;
    int arity;
    int degree;
    int calls;
    int P;              // next_pow2(1 + calls)
    int chunk;          // ParallelSum count
    int length;         // SumVec / Histogram / Multihot length
    int sv_bits;        // SumVec bits
    int wbits;          // Sum: max.bit_length(); Multihot: max_weight.bit_length()
    uint64_t max_measurement;
    uint64_t offset;    // Sum / Multihot offset = 2^wbits - 1 - max
    // truncation: out[1 + m / tgroup] += 2^(m % tgroup) * meas[m] for m < tlimit
    int tgroup;
    int tlimit;
    uint32_t alg_id;
};

MH_HD int mc_next_pow2(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}
MH_HD int mc_bit_length(uint64_t x) {
    int b = 0;
    while (x) { b++; x >>= 1; }
    return b;
}

// Largest SumVec / Histogram / MultihotCountVec length and chunk length
// accepted (the reference has no limit; these keep every size in int range).
#define MC_MAX_LENGTH (1 << 22)

// Returns 0 on success, -1 on invalid parameters.
inline int mc_derive(int circuit, int bits, int length, int sv_bits, uint64_t max_measurement,
                     int chunk, McParams* out) {
    McParams p = {};
    p.circuit = circuit;
    p.bits = bits;
    p.length = length;
    p.sv_bits = sv_bits;
    p.chunk = chunk;
    p.max_measurement = max_measurement;
    if (bits < 1 || bits > 65535) return -1;
    switch (circuit) {
    case MC_COUNT:
        p.field = 64; p.gadget = G_MUL; p.arity = 2; p.calls = 1;
        p.meas_len = 1; p.output_len = 1; p.eval_output_len = 1; p.joint_rand_len = 0;
        p.tgroup = 1; p.tlimit = 1; p.alg_id = 0xFFFF0001u;
        break;
    case MC_SUM:
        if (max_measurement == 0) return -1;
        p.field = 64; p.gadget = G_RANGE2; p.arity = 1;
        p.wbits = mc_bit_length(max_measurement);
        if (p.wbits > 63) return -1;
        p.offset = ((1ull << p.wbits) - 1) - max_measurement;
        p.calls = 2 * p.wbits; p.meas_len = 2 * p.wbits; p.output_len = 1;
        p.eval_output_len = 2 * p.wbits + 1; p.joint_rand_len = 0;
        p.tgroup = p.wbits; p.tlimit = p.wbits; p.alg_id = 0xFFFF0002u;
        break;
    case MC_SUMVEC:
        if (length < 1 || length > MC_MAX_LENGTH || sv_bits < 1 || sv_bits > 63 || chunk < 1 || chunk > MC_MAX_LENGTH)
            return -1;
        p.field = 128; p.gadget = G_PSUM_MUL; p.arity = 2 * chunk;
        p.calls = (length * sv_bits + chunk - 1) / chunk;
        p.meas_len = length * sv_bits; p.output_len = length; p.eval_output_len = 1;
        p.joint_rand_len = p.calls;
        p.tgroup = sv_bits; p.tlimit = length * sv_bits; p.alg_id = 0xFFFF0003u;
        break;
    case MC_HISTOGRAM:
        if (length < 1 || length > MC_MAX_LENGTH || chunk < 1 || chunk > MC_MAX_LENGTH) return -1;
        p.field = 128; p.gadget = G_PSUM_MUL; p.arity = 2 * chunk;
        p.calls = (length + chunk - 1) / chunk;
        p.meas_len = length; p.output_len = length; p.eval_output_len = 2;
        p.joint_rand_len = p.calls;
        p.tgroup = 1; p.tlimit = length; p.alg_id = 0xFFFF0004u;
        break;
    case MC_MULTIHOT:
        if (length < 1 || length > MC_MAX_LENGTH || chunk < 1 || chunk > MC_MAX_LENGTH || max_measurement == 0)
            return -1;
        p.field = 128; p.gadget = G_PSUM_MUL; p.arity = 2 * chunk;
        p.wbits = mc_bit_length(max_measurement);
        if (p.wbits > 63) return -1;
        p.offset = ((1ull << p.wbits) - 1) - max_measurement;
        p.calls = (length + p.wbits + chunk - 1) / chunk;
        p.meas_len = length + p.wbits; p.output_len = length; p.eval_output_len = 2;
        p.joint_rand_len = p.calls;
        p.tgroup = 1; p.tlimit = length; p.alg_id = 0xFFFF0005u;
        break;
    default:
        return -1;
    }
    p.degree = 2;
    p.enc = p.field / 8;
    p.w32 = p.enc / 4;
    p.value_len = 1 + p.meas_len;
    p.P = mc_next_pow2(1 + p.calls);
    p.prove_rand_len = p.arity;
    p.query_rand_len = 1 + (p.eval_output_len > 1 ? p.eval_output_len : 0);
    p.proof_len = p.arity + p.degree * (p.P - 1) + 1;
    p.verifier_len = 1 + p.arity + 1;
    // every wire size must fit the int arithmetic of the size helpers below
    const uint64_t pub = (uint64_t)(2 * bits + 7) / 8 + 48ull * (uint64_t)bits + (uint64_t)bits * p.value_len * p.enc;
    if (pub > (uint64_t)INT32_MAX / 2 || (uint64_t)p.proof_len * p.enc > (uint64_t)INT32_MAX / 4) return -1;
    *out = p;
    return 0;
}

// Wire sizes (poc/vidpf.py:382-394, poc/mastic.py:516-559)
MH_HD int mc_public_share_size(const McParams& p) {
    return (2 * p.bits + 7) / 8 + p.bits * 16 + p.bits * p.value_len * p.enc + p.bits * 32;
}
MH_HD int mc_input_share_size(const McParams& p, int agg_id) {
    int n = 16;
    if (agg_id == 0) {
        n += p.proof_len * p.enc;
        if (p.joint_rand_len > 0) n += 64;
    } else {
        n += 32;
        if (p.joint_rand_len > 0) n += 32;
    }
    return n;
}
MH_HD int mc_prep_share_size(const McParams& p, bool weight_check) {
    int n = 32;
    if (weight_check) {
        n += p.verifier_len * p.enc;
        if (p.joint_rand_len > 0) n += 32;
    }
    return n;
}
MH_HD int mc_rand_size(const McParams& p) { return 32 + 64 + (p.joint_rand_len > 0 ? 32 : 0); }
