// Keccak-p[1600, 12] and TurboSHAKE128 sponge plumbing for gfx950.
//
// One sponge per lane.  The 1600-bit state lives in 50 VGPRs as 25 {lo, hi}
// pairs; 64-bit rotations are two v_alignbit_b32, chi is one v_bitop3_b32 per
// half, theta's 5-way parities are two 3-input XORs per half.
//
// Every sponge in Mastic absorbs   prefix || body   where the prefix
// (le16(len(dst)) || dst || u8(len(seed)) || seed) is identical for all
// reports of a batch.  A one-thread setup kernel absorbs the prefix once
// (PrefixState); lanes start from that state at byte position `f`, which is
// uniform across the grid, and absorb word-aligned body words whose byte image
// is shifted by f % 4 with v_alignbit_b32.  No per-lane dynamic indexing of
// the state is ever needed: positions are uniform, loads are per-lane.
#pragma once
#include "common.hpp"

#define KECCAK_RATE 168
#define KECCAK_RATE_WORDS 42

struct KState {
    u32x2 a[25];
};

// rotation offsets r[x + 5y]
#define KR(x, y) KECCAK_ROTC[(x) + 5 * (y)]
static constexpr int KECCAK_ROTC[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                        25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

MH_D u32x2 chi1(u32x2 a, u32x2 b, u32x2 c) {
    // a ^ (~b & c)  == bitop3 LUT 0xD2 with (a,b,c) = (src0,src1,src2)
    return u32x2{(uint32_t)__builtin_amdgcn_bitop3_b32(a.lo, b.lo, c.lo, 0xD2),
                 (uint32_t)__builtin_amdgcn_bitop3_b32(a.hi, b.hi, c.hi, 0xD2)};
}

// Round constants are read as literal constants (the loop is fully unrolled).
// U = rounds per loop iteration (12 = fully unrolled).  Measured on MI355X:
// rolling the rounds (U = 2) made the binder sponge chain 25 % slower and did
// not speed up the level kernels beside it, so every caller unrolls fully.
// FUSE_D: theta's D[x] = C[x-1] ^ rotl(C[x+1], 1) is never formed, each word
// takes both terms in one 3-input XOR per half (10 fewer XORs per round); it
// keeps C live through rho, so the 96-VGPR plain level kernel (whose proof
// waves run this permutation) uses the unfused form: there it doubled the
// spills and cost C2 1.6 % (profiles/r04_v17_ab_theta_fusion.txt).
template <int U = 12, bool FUSE_D = true>
MH_D void keccak_p12(KState& s) {
    static constexpr uint32_t RCL[12] = {0x8000808bu, 0x0000008bu, 0x00008089u, 0x00008003u,
                                         0x00008002u, 0x00000080u, 0x0000800au, 0x8000000au,
                                         0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
    static constexpr uint32_t RCH[12] = {0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u,
                                         0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u,
                                         0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};
    u32x2* A = s.a;
#pragma unroll U
    for (int round = 0; round < 12; round++) {
        u32x2 C[5], D[5];
#pragma unroll
        for (int x = 0; x < 5; x++) {
            u32x2 t = xor3_64(A[x], A[x + 5], A[x + 10]);
            C[x] = xor3_64(t, A[x + 15], A[x + 20]);
        }
        u32x2 B[25];
        if constexpr (FUSE_D) {
#pragma unroll
            for (int x = 0; x < 5; x++) D[x] = rotl64(C[(x + 1) % 5], 1);
#pragma unroll
            for (int x = 0; x < 5; x++)
#pragma unroll
                for (int y = 0; y < 5; y++)
                    B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(xor3_64(A[x + 5 * y], C[(x + 4) % 5], D[x]), KR(x, y));
        } else {
#pragma unroll
            for (int x = 0; x < 5; x++) D[x] = xor64(C[(x + 4) % 5], rotl64(C[(x + 1) % 5], 1));
#pragma unroll
            for (int x = 0; x < 5; x++)
#pragma unroll
                for (int y = 0; y < 5; y++)
                    B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(xor64(A[x + 5 * y], D[x]), KR(x, y));
        }
#pragma unroll
        for (int y = 0; y < 5; y++)
#pragma unroll
            for (int x = 0; x < 5; x++)
                A[x + 5 * y] = chi1(B[x + 5 * y], B[(x + 1) % 5 + 5 * y], B[(x + 2) % 5 + 5 * y]);
        A[0].lo ^= RCL[round];
        A[0].hi ^= RCH[round];
    }
}

// ---- two lanes per sponge ------------------------------------------------
// Lane pair (2k, 2k+1) holds one state: the even lane the low 32-bit halves of
// the 25 words, the odd lane the high halves.  A 64-bit rotation needs the
// partner's half, fetched with one DPP quad_perm [1,0,3,2] (v_mov_b32_dpp);
// the rotation is then one v_alignbit_b32 with the same operands on both lanes
// (rotl by r < 32: alignbit(own, partner, 32 - r); by r > 32:
// alignbit(partner, own, 64 - r)).  Per round and lane: 10 (theta parities)
// + 15 (D) + 25 (A ^ D) + 48 (rho) + 25 (chi) + 2 (iota) ≈ 125 instructions
// against ≈ 190 for one lane holding both halves, so the serial sponge chain
// runs ≈ 1.5x shorter.  Both lanes of a pair must be active at every call.
struct KHalf {
    uint32_t a[25];
};

MH_D uint32_t pair_swap(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

MH_D uint32_t pair_rotl(uint32_t v, int r) {  // r compile-time, r != 32
    if (r == 0) return v;
    const uint32_t p = pair_swap(v);
    return r < 32 ? __builtin_amdgcn_alignbit(v, p, 32 - r) : __builtin_amdgcn_alignbit(p, v, 64 - r);
}

template <int U = 12>
MH_D void keccak_p12_pair(KHalf& s, bool hi) {
    static constexpr uint32_t RCL[12] = {0x8000808bu, 0x0000008bu, 0x00008089u, 0x00008003u,
                                         0x00008002u, 0x00000080u, 0x0000800au, 0x8000000au,
                                         0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
    static constexpr uint32_t RCH[12] = {0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u,
                                         0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u,
                                         0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};
    uint32_t* A = s.a;
#pragma unroll U
    for (int round = 0; round < 12; round++) {
        uint32_t C[5], D[5];
#pragma unroll
        for (int x = 0; x < 5; x++) C[x] = xor3_u32(xor3_u32(A[x], A[x + 5], A[x + 10]), A[x + 15], A[x + 20]);
#pragma unroll
        for (int x = 0; x < 5; x++) D[x] = pair_rotl(C[(x + 1) % 5], 1);  // (C[x-1] folded in below)
        uint32_t B[25];
#pragma unroll
        for (int x = 0; x < 5; x++)
#pragma unroll
            for (int y = 0; y < 5; y++)
                B[y + 5 * ((2 * x + 3 * y) % 5)] = pair_rotl(xor3_u32(A[x + 5 * y], C[(x + 4) % 5], D[x]), KR(x, y));
#pragma unroll
        for (int y = 0; y < 5; y++)
#pragma unroll
            for (int x = 0; x < 5; x++)
                A[x + 5 * y] = (uint32_t)__builtin_amdgcn_bitop3_b32(B[x + 5 * y], B[(x + 1) % 5 + 5 * y],
                                                                    B[(x + 2) % 5 + 5 * y], 0xD2);
        A[0] ^= hi ? RCH[round] : RCL[round];
    }
}

MH_D uint32_t kword(const KState& s, int j) {  // j must be a compile-time constant
    return (j & 1) ? s.a[j >> 1].hi : s.a[j >> 1].lo;
}
MH_D void kxor_word(KState& s, int j, uint32_t v) {  // j compile-time constant
    if (j & 1) s.a[j >> 1].hi ^= v; else s.a[j >> 1].lo ^= v;
}

// Absorb `nbytes` body bytes given as little-endian 32-bit words ld(m),
// m in [0, ceil(nbytes/4)), into a sponge currently filled up to byte f of its
// block.  f is uniform.  Bytes of the last word past nbytes must be zero.
// Returns the new fill position.  Branch-free: out-of-range words are loaded
// from a clamped index and replaced by zero with a uniform select, so the
// state never sits live across dozens of tiny basic blocks.
template <class Loader>
MH_D int sponge_absorb_words(KState& s, int f, int nbytes, Loader ld) {
    if (nbytes <= 0) return f;
    const int q = f >> 2;
    const int sh = f & 3;
    const int off = sh ? 1 : 0;
    const int amt = (32 - 8 * sh) & 31;
    const int nw = (nbytes + 3) >> 2;
    const int end = f + nbytes;
    for (int b = 0;; b++) {
        const int base = KECCAK_RATE_WORDS * b - q - off;
        uint32_t w[KECCAK_RATE_WORDS + 1];
        // all loads first (clamped index), then the uniform zero-selects
#pragma unroll
        for (int j = 0; j < KECCAK_RATE_WORDS + 1; j++) {
            const int m = base + j;
            w[j] = ld(m < 0 ? 0 : (m >= nw ? nw - 1 : m));
        }
#pragma unroll
        for (int j = 0; j < KECCAK_RATE_WORDS + 1; j++) {
            const int m = base + j;
            w[j] = (m >= 0 && m < nw) ? w[j] : 0u;
        }
#pragma unroll
        for (int j = 0; j < KECCAK_RATE_WORDS; j++) kxor_word(s, j, __builtin_amdgcn_alignbit(w[j + 1], w[j], amt));
        if (end >= KECCAK_RATE * (b + 1)) {
            keccak_p12(s);
            if (end == KECCAK_RATE * (b + 1)) return 0;
        } else {
            return end - KECCAK_RATE * b;
        }
    }
}

// TurboSHAKE padding: domain byte at position f, 0x80 into byte 167, permute.
MH_D void sponge_pad(KState& s, int f, uint32_t domain) {
    const int q = f >> 2;
    const uint32_t dw = domain << (8 * (f & 3));
#pragma unroll
    for (int j = 0; j < KECCAK_RATE_WORDS; j++) kxor_word(s, j, j == q ? dw : 0u);
    s.a[20].hi ^= 0x80000000u;
    keccak_p12(s);
}

// Squeeze next_vec(field, count) from a padded sponge: stream words are read in
// order, every W32 of them form a little-endian candidate, candidates >= p
// are skipped (vdaf_poc.xof.Xof.next_vec).  `put(e, words)` stores element e.
// Lanes may consume different numbers of candidates (rejection), so the loop
// runs until every lane of the wave is done.
template <int W32, class Valid, class Put>
MH_D void sponge_squeeze_vec(KState& s, int count, Valid valid, Put put) {
    uint32_t cand[W32];
#pragma unroll
    for (int i = 0; i < W32; i++) cand[i] = 0;
    int e = 0;
    int t = 0;  // stream word index (uniform)
    for (;;) {
#pragma unroll
        for (int j = 0; j < KECCAK_RATE_WORDS; j++) {
#pragma unroll
            for (int i = 0; i < W32 - 1; i++) cand[i] = cand[i + 1];
            cand[W32 - 1] = kword(s, j);
            if (((t + j) % W32) == W32 - 1) {
                if (e < count && valid(cand)) {
                    put(e, cand);
                    e++;
                }
            }
        }
        t += KECCAK_RATE_WORDS;
        if (!__any(e < count)) break;
        keccak_p12(s);
    }
}

// Squeeze raw bytes (derive_seed / XOF.next(n)), n a multiple of 4 <= 168.
template <class Put>
MH_D void sponge_squeeze_words(const KState& s, int nwords, Put put) {
#pragma unroll
    for (int j = 0; j < KECCAK_RATE_WORDS; j++)
        if (j < nwords) put(j, kword(s, j));
}

// Generic byte absorb with dynamic positions, for one-thread setup kernels.
MH_D int sponge_absorb_bytes_slow(KState& s, int f, const uint8_t* p, int n) {
    for (int i = 0; i < n; i++) {
        int w = f >> 2;
        uint32_t v = (uint32_t)p[i] << (8 * (f & 3));
        if (w & 1) s.a[w >> 1].hi ^= v; else s.a[w >> 1].lo ^= v;
        f++;
        if (f == KECCAK_RATE) {
            keccak_p12(s);
            f = 0;
        }
    }
    return f;
}

MH_D void kstate_zero(KState& s) {
#pragma unroll
    for (int i = 0; i < 25; i++) s.a[i] = u32x2{0, 0};
}
