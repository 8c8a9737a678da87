// GF(p) arithmetic for the two Mastic fields, usable on host and device.
//
// Field64:  p = 2^64 - 2^32 + 1          (vdaf_poc.field.Field64,  vdaf-13)
// Field128: p = 2^128 - 28 * 2^64 + 1    (vdaf_poc.field.Field128, vdaf-13)
//
// Elements are kept canonical (< p).  Their little-endian byte image is the
// wire encoding (Field.encode_vec), so an element is also its own storage
// format: F64 = one uint64, F128 = {lo, hi} uint64 pair.
#pragma once
#include "common.hpp"

typedef unsigned __int128 mh_u128;
typedef __int128 mh_i128;

struct F64 {
    typedef uint64_t E;
    static constexpr int ENC = 8;    // ENCODED_SIZE
    static constexpr int W32 = 2;    // 32-bit words per element
    static constexpr uint64_t P = 0xFFFFFFFF00000001ull;
    static constexpr uint64_t EPS = 0xFFFFFFFFull;  // 2^64 mod p

    MH_HD static E zero() { return 0; }
    MH_HD static E from_u64(uint64_t x) { return x >= P ? x - P : x; }
    MH_HD static bool is_zero(E a) { return a == 0; }
    MH_HD static bool eq(E a, E b) { return a == b; }
    // next_vec acceptance test on a raw little-endian candidate.
    MH_HD static bool valid(E x) { return x < P; }

    MH_HD static E add(E a, E b) {
        uint64_t s = a + b;
        if (s < a || s >= P) s -= P;
        return s;
    }
    MH_HD static E sub(E a, E b) {
        uint64_t d = a - b;
        if (a < b) d += P;
        return d;
    }
    MH_HD static E neg(E a) { return a == 0 ? 0 : P - a; }
    MH_HD static E reduce128(uint64_t lo, uint64_t hi) {
        uint64_t hh = hi >> 32, hl = hi & EPS;
        uint64_t t0 = lo - hh;
        if (lo < hh) t0 -= EPS;
        uint64_t t1 = hl * EPS;
        uint64_t t2 = t0 + t1;
        if (t2 < t0) t2 += EPS;
        if (t2 >= P) t2 -= P;
        return t2;
    }
    MH_HD static E mul(E a, E b) {
        mh_u128 x = (mh_u128)a * b;
        return reduce128((uint64_t)x, (uint64_t)(x >> 64));
    }

    // word access (little-endian 32-bit halves)
    MH_HD static uint32_t word(E a, int i) { return (uint32_t)(a >> (32 * i)); }
    MH_HD static E from_words(const uint32_t* w) { return (uint64_t)w[0] | ((uint64_t)w[1] << 32); }
};

struct F128 {
    struct E {
        uint64_t lo, hi;
    };
    static constexpr int ENC = 16;
    static constexpr int W32 = 4;
    static constexpr uint64_t P_LO = 1ull;
    static constexpr uint64_t P_HI = 0xFFFFFFFFFFFFFFE4ull;  // 2^64 - 28

    MH_HD static E zero() { return E{0, 0}; }
    MH_HD static E from_u64(uint64_t x) { return E{x, 0}; }
    MH_HD static bool is_zero(E a) { return (a.lo | a.hi) == 0; }
    MH_HD static bool eq(E a, E b) { return a.lo == b.lo && a.hi == b.hi; }
    MH_HD static bool ge_p(uint64_t lo, uint64_t hi) {
        return hi > P_HI || (hi == P_HI && lo >= P_LO);
    }
    MH_HD static bool valid(E x) { return !ge_p(x.lo, x.hi); }

    MH_HD static E sub_p(E a) {
        uint64_t lo = a.lo - P_LO;
        uint64_t br = a.lo < P_LO;
        return E{lo, a.hi - P_HI - br};
    }
    MH_HD static E add(E a, E b) {
        uint64_t lo = a.lo + b.lo;
        uint64_t c = lo < a.lo;
        uint64_t hi1 = a.hi + b.hi;
        uint64_t c1 = hi1 < a.hi;
        uint64_t hi = hi1 + c;
        c1 |= hi < hi1;
        E s{lo, hi};
        if (c1 || ge_p(lo, hi)) s = sub_p(s);  // wraps correctly when c1 set
        return s;
    }
    MH_HD static E sub(E a, E b) {
        uint64_t lo = a.lo - b.lo;
        uint64_t br = a.lo < b.lo;
        uint64_t hi = a.hi - b.hi - br;
        bool under = (a.hi < b.hi) || (a.hi == b.hi && a.lo < b.lo);
        E d{lo, hi};
        if (under) {
            uint64_t l2 = d.lo + P_LO;
            uint64_t c = l2 < d.lo;
            d = E{l2, d.hi + P_HI + c};
        }
        return d;
    }
    MH_HD static E neg(E a) { return sub(zero(), a); }

    // value = L + c * H with c = 28 * 2^64 - 1 = 2^128 mod p.
    MH_HD static void fold(uint64_t l0, uint64_t l1, uint64_t h0, uint64_t h1,
                           uint64_t& z0, uint64_t& z1, uint64_t& z2, uint64_t& z3) {
        mh_u128 t = (mh_u128)h0 * 28u;
        uint64_t a0 = (uint64_t)t;
        mh_u128 t2 = (mh_u128)h1 * 28u + (uint64_t)(t >> 64);
        uint64_t a1 = (uint64_t)t2;
        uint64_t a2 = (uint64_t)(t2 >> 64);
        // [l0, l1] + [0, a0, a1, a2] - [h0, h1]
        z0 = l0 - h0;
        uint64_t b0 = l0 < h0;
        mh_i128 acc = (mh_i128)l1 + (mh_i128)a0 - (mh_i128)h1 - (mh_i128)b0;
        z1 = (uint64_t)acc;
        mh_i128 cy = acc >> 64;
        mh_i128 acc2 = (mh_i128)a1 + cy;
        z2 = (uint64_t)acc2;
        cy = acc2 >> 64;
        z3 = a2 + (uint64_t)cy;
    }
    MH_HD static E mul(E a, E b) {
        mh_u128 p00 = (mh_u128)a.lo * b.lo;
        mh_u128 p01 = (mh_u128)a.lo * b.hi;
        mh_u128 p10 = (mh_u128)a.hi * b.lo;
        mh_u128 p11 = (mh_u128)a.hi * b.hi;
        uint64_t r0 = (uint64_t)p00;
        mh_u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
        uint64_t r1 = (uint64_t)mid;
        mh_u128 mid2 = (mid >> 64) + (p01 >> 64) + (p10 >> 64) + (uint64_t)p11;
        uint64_t r2 = (uint64_t)mid2;
        uint64_t r3 = (uint64_t)((mid2 >> 64) + (p11 >> 64));
#pragma unroll
        for (int i = 0; i < 5; i++) {
            if ((r2 | r3) == 0) break;
            uint64_t z0, z1, z2, z3;
            fold(r0, r1, r2, r3, z0, z1, z2, z3);
            r0 = z0; r1 = z1; r2 = z2; r3 = z3;
        }
        E out{r0, r1};
        if (ge_p(out.lo, out.hi)) out = sub_p(out);
        return out;
    }

    MH_HD static uint32_t word(E a, int i) {
        return i < 2 ? (uint32_t)(a.lo >> (32 * i)) : (uint32_t)(a.hi >> (32 * (i - 2)));
    }
    MH_HD static E from_words(const uint32_t* w) {
        return E{(uint64_t)w[0] | ((uint64_t)w[1] << 32), (uint64_t)w[2] | ((uint64_t)w[3] << 32)};
    }
};

// Generic helpers -------------------------------------------------------
template <class F>
MH_HD typename F::E fpow(typename F::E base, const uint64_t* exp_le, int exp_words) {
    typename F::E acc = F::from_u64(1);
    for (int w = exp_words - 1; w >= 0; w--) {
        for (int b = 63; b >= 0; b--) {
            acc = F::mul(acc, acc);
            if ((exp_le[w] >> b) & 1) acc = F::mul(acc, base);
        }
    }
    return acc;
}

template <class F> struct FieldConsts;
template <> struct FieldConsts<F64> {
    // p - 2 for Fermat inversion
    MH_HD static void pm2(uint64_t* e) { e[0] = F64::P - 2; e[1] = 0; }
    static constexpr int GEN_ORDER_LOG2 = 32;
};
template <> struct FieldConsts<F128> {
    MH_HD static void pm2(uint64_t* e) { e[0] = F128::P_LO - 2; e[1] = F128::P_HI - 1; }
    static constexpr int GEN_ORDER_LOG2 = 66;
};

template <class F>
MH_HD typename F::E finv(typename F::E a) {
    uint64_t e[2];
    FieldConsts<F>::pm2(e);
    return fpow<F>(a, e, 2);
}

template <class F>
MH_HD typename F::E fpow_u64(typename F::E base, uint64_t e) {
    uint64_t ex[1] = {e};
    return fpow<F>(base, ex, 1);
}
