// AES-128 for XofFixedKeyAes128 (vdaf_poc.xof, vdaf-13) on gfx950.
//
// T-table AES with ONE table T0 in LDS, replicated 32 times so that lane l
// always reads bank (l mod 32): random-index lookups are bank-conflict free
// (ds_read_b32 services lanes in two groups of 32, one bank each).  The other
// three tables are byte rotations of T0 (v_alignbit_b32).  32 KiB of LDS.
//
// State bytes are kept as four little-endian column words
// (column c = bytes 4c..4c+3), matching the wire byte order of the block.
#pragma once
#include "common.hpp"

#define AES_LDS_WORDS (256 * 32)

static constexpr uint8_t AES_SBOX[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

MH_HD uint32_t aes_xtime(uint32_t b) { return ((b << 1) ^ ((b & 0x80) ? 0x1b : 0)) & 0xff; }

// T0[x] little-endian word = (2S, S, S, 3S)
MH_HD uint32_t aes_t0(int x) {
    uint32_t s = AES_SBOX[x];
    uint32_t s2 = aes_xtime(s);
    uint32_t s3 = s2 ^ s;
    return s2 | (s << 8) | (s << 16) | (s3 << 24);
}

// T0 words of all 256 S-box entries, built at compile time.  The table
// fills below write runs of 64 words whose entries are wave-uniform, so each
// run costs one scalar load of this table instead of a per-lane S-box byte
// load whose latency the fill loop waited out 32 times per thread (~10 us per
// level-kernel workgroup; profiles/r06_v12_*).
struct AesT0Words {
    uint32_t w[256];
};
constexpr AesT0Words aes_t0_words() {
    AesT0Words t{};
    for (int x = 0; x < 256; x++) {
        const uint32_t s = AES_SBOX[x];
        const uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x1bu : 0u)) & 0xffu;
        t.w[x] = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
    }
    return t;
}
static constexpr AesT0Words AES_T0W = aes_t0_words();

// Cooperative fill of the replicated table: T[(x << 5) | r] = T0[x].
// nthreads: whole waves (tid = threadIdx.x).
MH_D void aes_lds_fill(uint32_t* T, int tid, int nthreads) {
    const uint32_t lane = (uint32_t)tid & 63u;
    const int w0 = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nthreads >> 6;
#pragma unroll 8
    for (int run = w0; run < AES_LDS_WORDS / 64; run += nw) {
        // words [64 run, 64 run + 64): entries 2 run (lanes 0-31) and 2 run + 1
        const uint32_t a = AES_T0W.w[2 * run], b = AES_T0W.w[2 * run + 1];
        T[run * 64 + lane] = (lane & 32u) ? b : a;
    }
}

struct AesLds {
    const uint32_t* base;  // &T[lane & 31]
    MH_D uint32_t t0(uint32_t byte_idx) const { return base[byte_idx << 5]; }
};

MH_D uint32_t rot8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
MH_D uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
MH_D uint32_t rot24(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }

MH_D uint32_t b0(uint32_t x) { return x & 0xffu; }
MH_D uint32_t b1(uint32_t x) { return __builtin_amdgcn_ubfe(x, 8, 8); }
MH_D uint32_t b2(uint32_t x) { return __builtin_amdgcn_ubfe(x, 16, 8); }
MH_D uint32_t b3(uint32_t x) { return x >> 24; }

// Round-key sources: 44 words in registers, or a per-lane 176-byte row in LDS
// read as one ds_read_b128 per round (rows of consecutive lanes are 176 B
// apart: conflict-free for the b128 lane groups).
struct RkRegs {
    const uint32_t* k;
    MH_D uint4 operator()(int round) const {
        return uint4{k[4 * round], k[4 * round + 1], k[4 * round + 2], k[4 * round + 3]};
    }
};
struct RkLds {
    const uint4* row;
    MH_D uint4 operator()(int round) const { return row[round]; }
};

// Encrypt one block.
template <class RK>
MH_D void aes128_encrypt(const AesLds& T, const RK& rk, uint32_t s[4]) {
    uint4 k = rk(0);
    uint32_t s0 = s[0] ^ k.x, s1 = s[1] ^ k.y, s2 = s[2] ^ k.z, s3 = s[3] ^ k.w;
#pragma unroll
    for (int r = 1; r < 10; r++) {
        k = rk(r);
        uint32_t t0 = xor3_u32(T.t0(b0(s0)), rot8(T.t0(b1(s1))), rot16(T.t0(b2(s2))));
        uint32_t t1 = xor3_u32(T.t0(b0(s1)), rot8(T.t0(b1(s2))), rot16(T.t0(b2(s3))));
        uint32_t t2 = xor3_u32(T.t0(b0(s2)), rot8(T.t0(b1(s3))), rot16(T.t0(b2(s0))));
        uint32_t t3 = xor3_u32(T.t0(b0(s3)), rot8(T.t0(b1(s0))), rot16(T.t0(b2(s1))));
        t0 = xor3_u32(t0, rot24(T.t0(b3(s3))), k.x);
        t1 = xor3_u32(t1, rot24(T.t0(b3(s0))), k.y);
        t2 = xor3_u32(t2, rot24(T.t0(b3(s1))), k.z);
        t3 = xor3_u32(t3, rot24(T.t0(b3(s2))), k.w);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // Final round: S-box byte = byte 1 of the T0 entry.
    k = rk(10);
    auto sb = [&](uint32_t x) { return b1(T.t0(x)); };
    uint32_t o0 = sb(b0(s0)) | (sb(b1(s1)) << 8) | (sb(b2(s2)) << 16) | (sb(b3(s3)) << 24);
    uint32_t o1 = sb(b0(s1)) | (sb(b1(s2)) << 8) | (sb(b2(s3)) << 16) | (sb(b3(s0)) << 24);
    uint32_t o2 = sb(b0(s2)) | (sb(b1(s3)) << 8) | (sb(b2(s0)) << 16) | (sb(b3(s1)) << 24);
    uint32_t o3 = sb(b0(s3)) | (sb(b1(s0)) << 8) | (sb(b2(s1)) << 16) | (sb(b3(s2)) << 24);
    s[0] = o0 ^ k.x;
    s[1] = o1 ^ k.y;
    s[2] = o2 ^ k.z;
    s[3] = o3 ^ k.w;
}

// AES-128 key expansion (FIPS-197 §5.2) with the S-box from the LDS table.
MH_D void aes128_expand(const AesLds& T, const uint32_t key[4], uint32_t rk[44]) {
    rk[0] = key[0]; rk[1] = key[1]; rk[2] = key[2]; rk[3] = key[3];
    uint32_t rcon = 1;
#pragma unroll
    for (int i = 4; i < 44; i++) {
        uint32_t t = rk[i - 1];
        if ((i & 3) == 0) {
            // RotWord then SubWord on little-endian words: bytes (t1, t2, t3, t0)
            uint32_t r = b1(T.t0(b1(t))) | (b1(T.t0(b2(t))) << 8) | (b1(T.t0(b3(t))) << 16) |
                         (b1(T.t0(b0(t))) << 24);
            t = r ^ rcon;
            rcon = aes_xtime(rcon);
        }
        rk[i] = rk[i - 4] ^ t;
    }
}

// XofFixedKeyAes128.hash_block for counter `ctr` (< 2^32 here):
//   x = seed ^ le128(ctr); sigma(x) = x_hi || (x_hi ^ x_lo); out = AES(sigma) ^ sigma
template <class TT, class RK>
MH_D void fixed_key_block(const TT& T, const RK& rk, const uint32_t seed[4], uint32_t ctr, uint32_t out[4]) {
    uint32_t x0 = seed[0] ^ ctr, x1 = seed[1], x2 = seed[2], x3 = seed[3];
    uint32_t sg[4] = {x2, x3, x2 ^ x0, x3 ^ x1};
    uint32_t c[4] = {sg[0], sg[1], sg[2], sg[3]};
    aes128_encrypt(T, rk, c);
    out[0] = c[0] ^ sg[0];
    out[1] = c[1] ^ sg[1];
    out[2] = c[2] ^ sg[2];
    out[3] = c[3] ^ sg[3];
}
MH_D void fixed_key_block(const AesLds& T, const uint32_t* rk, const uint32_t seed[4], uint32_t ctr,
                          uint32_t out[4]) {
    fixed_key_block(T, RkRegs{rk}, seed, ctr, out);
}

// Two independent blocks in lockstep, round by round: one wave then always has
// 32 independent T-table lookups in flight instead of 16, which hides the LDS
// latency of one chain behind the other (both use the same key schedule).
template <class RK>
MH_D void aes128_encrypt2(const AesLds& T, const RK& rk, uint32_t a[4], uint32_t b[4]) {
    uint4 k = rk(0);
    uint32_t a0 = a[0] ^ k.x, a1 = a[1] ^ k.y, a2 = a[2] ^ k.z, a3 = a[3] ^ k.w;
    uint32_t c0 = b[0] ^ k.x, c1 = b[1] ^ k.y, c2 = b[2] ^ k.z, c3 = b[3] ^ k.w;
#pragma unroll
    for (int r = 1; r < 10; r++) {
        k = rk(r);
        uint32_t t0 = xor3_u32(T.t0(b0(a0)), rot8(T.t0(b1(a1))), rot16(T.t0(b2(a2))));
        uint32_t u0 = xor3_u32(T.t0(b0(c0)), rot8(T.t0(b1(c1))), rot16(T.t0(b2(c2))));
        uint32_t t1 = xor3_u32(T.t0(b0(a1)), rot8(T.t0(b1(a2))), rot16(T.t0(b2(a3))));
        uint32_t u1 = xor3_u32(T.t0(b0(c1)), rot8(T.t0(b1(c2))), rot16(T.t0(b2(c3))));
        uint32_t t2 = xor3_u32(T.t0(b0(a2)), rot8(T.t0(b1(a3))), rot16(T.t0(b2(a0))));
        uint32_t u2 = xor3_u32(T.t0(b0(c2)), rot8(T.t0(b1(c3))), rot16(T.t0(b2(c0))));
        uint32_t t3 = xor3_u32(T.t0(b0(a3)), rot8(T.t0(b1(a0))), rot16(T.t0(b2(a1))));
        uint32_t u3 = xor3_u32(T.t0(b0(c3)), rot8(T.t0(b1(c0))), rot16(T.t0(b2(c1))));
        t0 = xor3_u32(t0, rot24(T.t0(b3(a3))), k.x);
        u0 = xor3_u32(u0, rot24(T.t0(b3(c3))), k.x);
        t1 = xor3_u32(t1, rot24(T.t0(b3(a0))), k.y);
        u1 = xor3_u32(u1, rot24(T.t0(b3(c0))), k.y);
        t2 = xor3_u32(t2, rot24(T.t0(b3(a1))), k.z);
        u2 = xor3_u32(u2, rot24(T.t0(b3(c1))), k.z);
        t3 = xor3_u32(t3, rot24(T.t0(b3(a2))), k.w);
        u3 = xor3_u32(u3, rot24(T.t0(b3(c2))), k.w);
        a0 = t0; a1 = t1; a2 = t2; a3 = t3;
        c0 = u0; c1 = u1; c2 = u2; c3 = u3;
    }
    k = rk(10);
    auto sb = [&](uint32_t x) { return b1(T.t0(x)); };
    a[0] = (sb(b0(a0)) | (sb(b1(a1)) << 8) | (sb(b2(a2)) << 16) | (sb(b3(a3)) << 24)) ^ k.x;
    b[0] = (sb(b0(c0)) | (sb(b1(c1)) << 8) | (sb(b2(c2)) << 16) | (sb(b3(c3)) << 24)) ^ k.x;
    a[1] = (sb(b0(a1)) | (sb(b1(a2)) << 8) | (sb(b2(a3)) << 16) | (sb(b3(a0)) << 24)) ^ k.y;
    b[1] = (sb(b0(c1)) | (sb(b1(c2)) << 8) | (sb(b2(c3)) << 16) | (sb(b3(c0)) << 24)) ^ k.y;
    a[2] = (sb(b0(a2)) | (sb(b1(a3)) << 8) | (sb(b2(a0)) << 16) | (sb(b3(a1)) << 24)) ^ k.z;
    b[2] = (sb(b0(c2)) | (sb(b1(c3)) << 8) | (sb(b2(c0)) << 16) | (sb(b3(c1)) << 24)) ^ k.z;
    a[3] = (sb(b0(a3)) | (sb(b1(a0)) << 8) | (sb(b2(a1)) << 16) | (sb(b3(a2)) << 24)) ^ k.w;
    b[3] = (sb(b0(c3)) | (sb(b1(c0)) << 8) | (sb(b2(c1)) << 16) | (sb(b3(c2)) << 24)) ^ k.w;
}

// Two fixed-key blocks (seed_a, ctr_a) and (seed_b, ctr_b) in lockstep.
template <class TT, class RK>
MH_D void fixed_key_block2(const TT& T, const RK& rk, const uint32_t sa[4], uint32_t ca, const uint32_t sb_[4],
                           uint32_t cb, uint32_t oa[4], uint32_t ob[4]) {
    uint32_t ga[4] = {sa[2], sa[3], sa[2] ^ sa[0] ^ ca, sa[3] ^ sa[1]};
    uint32_t gb[4] = {sb_[2], sb_[3], sb_[2] ^ sb_[0] ^ cb, sb_[3] ^ sb_[1]};
    uint32_t xa[4] = {ga[0], ga[1], ga[2], ga[3]};
    uint32_t xb[4] = {gb[0], gb[1], gb[2], gb[3]};
    aes128_encrypt2(T, rk, xa, xb);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        oa[i] = xa[i] ^ ga[i];
        ob[i] = xb[i] ^ gb[i];
    }
}

// ---- T0/T2 table addressed by v_perm_b32 (level-eval kernel) ---------------
// Layout (64 KiB): row x (256 B) holds T0[x] replicated at bytes 4l (lane
// l < 32) and T2[x] = rot16(T0[x]) replicated at bytes 128 + 4l.  The LDS
// byte address of a lookup is then  (x << 8) | lane_byte,  built from the
// state word by ONE v_perm_b32 (byte k of the state word into bits 8..15, the
// lane's byte into bits 0..7) instead of a bit-field extract plus a
// shift-add.  Banks stay conflict-free: lane l always reads bank l mod 32.
// With T2 stored, a column needs one rotation instead of three:
//   T0[a] ^ T1[b] ^ T2[c] ^ T3[d] = T0[a] ^ T2[c] ^ rot8(T0[b] ^ T2[d]).
// A round costs 16 v_perm + 4 x (xor3, rot, xor3) = 28 VALU against
// 52 with one rotated table and two-instruction addressing.
//
// AES_T4 (default): all four tables.  A second 64 KiB block at LDS address
// 64 KiB holds T1 = rot8(T0) and T3 = rot24(T0) in the same layout; its lane
// byte register carries 0x01 in byte 2, which the v_perm selector copies into
// address bits 16..23, so every lookup is still ONE v_perm.  A column is then
// two xor3 (T0 ^ T1 ^ T2, then ^ T3 ^ k): 16 v_perm + 8 VALU per round (24
// instead of 28), plain round keys, 128 KiB of LDS.
#ifndef AES_T4
#define AES_T4 1
#endif
#define AES_PERM_LDS_WORDS (AES_T4 ? 256 * 128 : 256 * 64)

// nthreads: whole waves (tid = threadIdx.x).  Word i = 64 run + lane holds
// entry run & 255 (wave-uniform: one scalar load per run, AES_T0W) as T0 or
// T2 (lanes 0-31 / 32-63), or T1 / T3 in the second block (run >= 256).
MH_D void aes_perm_fill(uint32_t* T, int tid, int nthreads) {
    const uint32_t lane = (uint32_t)tid & 63u;
    const int w0 = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nthreads >> 6;
#pragma unroll 8
    for (int run = w0; run < AES_PERM_LDS_WORDS / 64; run += nw) {
        const uint32_t t0 = AES_T0W.w[run & 255];
        const bool hi = run >= 256;  // T1 / T3 block
        T[run * 64 + lane] = (lane & 32u) ? (hi ? rot24(t0) : rot16(t0)) : (hi ? rot8(t0) : t0);
    }
}

struct AesPerm {
    const uint32_t* T;  // the table; must sit at LDS address 0 (see lds_read_asm)
    uint32_t lb0;       // 4 * (lane & 31)
    uint32_t lb2;       // 128 + 4 * (lane & 31)
    // v_perm_b32 issues at half rate (4 cycles per wave64 instruction on a
    // SIMD, tools/valu_peak.hip); byte 1 already sits at address bits 8..15,
    // so its address is a bitwise select (x & 0xff00) | (lane & ~0xff00): ONE
    // full-rate v_bitop3_b32 (LUT 0xE4 = src2 ? src0 : src1).
    template <int K>
    MH_D static uint32_t addr(uint32_t x, uint32_t lane, uint32_t sel_hi) {
        if constexpr (K == 1) return __builtin_amdgcn_bitop3_b32(x, lane, 0xff00u, 0xE4);
        return __builtin_amdgcn_perm(x, lane, sel_hi | ((4u + K) << 8));
    }
    template <int K>
    MH_D uint32_t a0(uint32_t x) const { return addr<K>(x, lb0, 0x0c0c0000u); }
    template <int K>
    MH_D uint32_t a2(uint32_t x) const { return addr<K>(x, lb2, 0x0c0c0000u); }
    // T1 / T3 (AES_T4): same lane bytes plus 0x01 in byte 2 -> +64 KiB
    template <int K>
    MH_D uint32_t a1(uint32_t x) const { return addr<K>(x, lb0 | 0x10000u, 0x0c020000u); }
    template <int K>
    MH_D uint32_t a3(uint32_t x) const { return addr<K>(x, lb2 | 0x10000u, 0x0c020000u); }
    template <int K>
    MH_D uint32_t t0(uint32_t x) const { return *(const uint32_t*)((const char*)T + a0<K>(x)); }
    template <int K>
    MH_D uint32_t t2(uint32_t x) const { return *(const uint32_t*)((const char*)T + a2<K>(x)); }
};

// LDS read of a table word at byte address a, issued as inline asm: the
// v_perm result IS the LDS address (the table is the kernel's only LDS
// block, at address 0), so no base add per lookup.  The compiler does not
// track these reads; aes_pin<> waits for them (s_waitcnt lgkmcnt(0)) before
// any result is used.
MH_D uint32_t lds_read_asm(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a));
    return v;
}

// Word i (< 44) of a key schedule as stored for AesPerm: plain with AES_T4;
// with two tables a column is T0[.] ^ T2[.] ^ rot8(T0[.] ^ T2[.] ^ rotr8(k)),
// so rounds 1..9 are stored rotated right by 8.
MH_HD uint32_t aes_perm_key_word(int i, uint32_t w) {
    if (AES_T4) return w;
    return (i >= 4 && i < 40) ? ((w >> 8) | (w << 24)) : w;
}
// Middle rounds.  All 16 N table lookups of a round are issued before any is
// consumed: an empty asm statement takes every lookup result as an operand,
// so the compiler cannot interleave "two reads, wait, xor" (which it does
// inside the level kernel when left alone, leaving 2 of the LDS pipe's reads
// in flight per wave instead of 16 N).  One wait per round, then the XORs.
#define MH_PIN16(L, o)                                                                                        \
    "+v"(L[o + 0]), "+v"(L[o + 1]), "+v"(L[o + 2]), "+v"(L[o + 3]), "+v"(L[o + 4]), "+v"(L[o + 5]),           \
        "+v"(L[o + 6]), "+v"(L[o + 7]), "+v"(L[o + 8]), "+v"(L[o + 9]), "+v"(L[o + 10]), "+v"(L[o + 11]),     \
        "+v"(L[o + 12]), "+v"(L[o + 13]), "+v"(L[o + 14]), "+v"(L[o + 15])
template <int N>
MH_D void aes_pin(uint32_t (&L)[16 * N]) {
    if constexpr (N == 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" : MH_PIN16(L, 0));
    } else if constexpr (N == 2) {
        asm volatile("s_waitcnt lgkmcnt(0)" : MH_PIN16(L, 0), MH_PIN16(L, 16));
    } else {
        static_assert(N % 2 == 0, "N = 1, 2 or even");
#pragma unroll
        for (int j = 0; j + 1 < N; j += 2)
            asm volatile("s_waitcnt lgkmcnt(0)" : MH_PIN16(L, 16 * j), MH_PIN16(L, 16 * j + 16));
    }
}

// One middle round of N blocks; k holds the round key as stored for AesPerm
// (rotated right by 8, see aes_perm_key_word).
template <int N>
MH_D void aes_round_n(const AesPerm& T, uint32_t (&s)[N][4], uint4 k) {
    uint32_t L[16 * N];
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            L[16 * j + 4 * c + 0] = lds_read_asm(T.a0<0>(s[j][c]));
            L[16 * j + 4 * c + 1] = lds_read_asm(AES_T4 ? T.a1<1>(s[j][(c + 1) & 3]) : T.a0<1>(s[j][(c + 1) & 3]));
            L[16 * j + 4 * c + 2] = lds_read_asm(T.a2<2>(s[j][(c + 2) & 3]));
            L[16 * j + 4 * c + 3] = lds_read_asm(AES_T4 ? T.a3<3>(s[j][(c + 3) & 3]) : T.a2<3>(s[j][(c + 3) & 3]));
        }
    aes_pin<N>(L);
    const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t* q = L + 16 * j + 4 * c;
            if (AES_T4)
                s[j][c] = xor3_u32(xor3_u32(q[0], q[1], q[2]), q[3], kk[c]);
            else
                s[j][c] = xor3_u32(q[0], q[2], rot8(xor3_u32(q[1], q[3], kk[c])));
        }
}

// Final round of N blocks: S-box bytes (byte 1 of the T0 entries) packed with
// two v_perm_b32 and merged with the round key by one xor3.
template <int N>
MH_D void aes_last_n(const AesPerm& T, uint32_t (&s)[N][4], uint4 k) {
    uint32_t L[16 * N];
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            L[16 * j + 4 * c + 0] = lds_read_asm(T.a0<0>(s[j][c]));
            L[16 * j + 4 * c + 1] = lds_read_asm(T.a0<1>(s[j][(c + 1) & 3]));
            L[16 * j + 4 * c + 2] = lds_read_asm(T.a0<2>(s[j][(c + 2) & 3]));
            L[16 * j + 4 * c + 3] = lds_read_asm(T.a0<3>(s[j][(c + 3) & 3]));
        }
    aes_pin<N>(L);
    const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t* q = L + 16 * j + 4 * c;
            const uint32_t lo = __builtin_amdgcn_perm(q[1], q[0], 0x0c0c0501u);
            const uint32_t hi = __builtin_amdgcn_perm(q[3], q[2], 0x05010c0cu);
            s[j][c] = xor3_u32(lo, hi, kk[c]);
        }
}

// N blocks in lockstep (N = 2: the two children of a parent; N = 4: two
// payload blocks per sibling): a round issues 16 N independent lookups per
// wave, which keeps the LDS pipe fed at 4 waves/SIMD.
template <int N, class RK>
MH_D void aes128_encrypt_n(const AesPerm& T, const RK& rk, uint32_t (&x)[N][4]) {
    uint4 k = rk(0);
#pragma unroll
    for (int j = 0; j < N; j++) {
        x[j][0] ^= k.x;
        x[j][1] ^= k.y;
        x[j][2] ^= k.z;
        x[j][3] ^= k.w;
    }
#pragma unroll
    for (int r = 1; r < 10; r++) aes_round_n<N>(T, x, rk(r));
    aes_last_n<N>(T, x, rk(10));
}

template <class RK>
MH_D void aes128_encrypt2(const AesPerm& T, const RK& rk, uint32_t a[4], uint32_t b[4]) {
    uint32_t x[2][4] = {{a[0], a[1], a[2], a[3]}, {b[0], b[1], b[2], b[3]}};
    aes128_encrypt_n<2>(T, rk, x);
#pragma unroll
    for (int c = 0; c < 4; c++) {
        a[c] = x[0][c];
        b[c] = x[1][c];
    }
}

template <class RK>
MH_D void aes128_encrypt(const AesPerm& T, const RK& rk, uint32_t s[4]) {
    uint32_t x[1][4] = {{s[0], s[1], s[2], s[3]}};
    aes128_encrypt_n<1>(T, rk, x);
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = x[0][c];
}

// ---- counter groups: rounds 1 and 2 shared by the blocks of one seed -----
// The blocks of one XofFixedKeyAes128 stream differ only in the counter, and
// the counter enters sigma(seed ^ le128(ctr)) = (s2, s3, s2 ^ s0 ^ ctr, s3 ^ s1)
// in word 2 alone.  Blocks whose counters agree above bit 7 therefore share 15
// of the 16 round-1 S-box inputs (all but byte 8), so 3 of the 4 round-1
// output columns and, in round 2, 3 of the 4 lookups of every column: per
// block, rounds 1 and 2 need 1 + 4 table lookups instead of 32 (27 of the 160
// lookups of a block, and their address / XOR work).  The shared part is
// computed once per (seed, ctr >> 8) by ctr_group_init; ctr_blocks_n finishes
// N blocks from their groups in lockstep.  (The well-known first-rounds
// precomputation of AES counter mode, applied per seed.)
static_assert(AES_T4, "counter groups assume the four-table layout");
struct AesCtrGroup {
    uint32_t a;     // LDS address of T0[round-0 byte 8] for counter low byte 0
    uint32_t p2;    // round-1 column 2 without its T0 lookup
    uint32_t q[4];  // round-2 columns without their lookup of round-1 column 2
};

// The shared part of N groups (seeds seed[j], counters ctr_hi[j] & ~0xff) in
// lockstep: 15 round-1 and 12 round-2 lookups per group.
template <int N, class RK>
MH_D void ctr_group_init(const AesPerm& T, const RK& rk, const uint32_t* const (&seed)[N], const uint32_t (&ctr_hi)[N],
                         AesCtrGroup* const (&g)[N]) {
    static_assert(N == 1 || N == 2, "N = 1 or 2");
    const uint4 k0 = rk(0), k1 = rk(1), k2 = rk(2);
    uint32_t L[16 * N];  // 15 used per group
    uint32_t a2v[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t* sd = seed[j];
        const uint32_t a0 = sd[2] ^ k0.x, a1 = sd[3] ^ k0.y;
        const uint32_t a2 = sd[2] ^ sd[0] ^ (ctr_hi[j] & ~0xffu) ^ k0.z, a3 = sd[3] ^ sd[1] ^ k0.w;
        a2v[j] = a2;
        uint32_t* l = L + 16 * j;
        // round 1: columns 0, 1, 3 complete, column 2 without T0[a2.b0]
        l[0] = lds_read_asm(T.a0<0>(a0));
        l[1] = lds_read_asm(T.a1<1>(a1));
        l[2] = lds_read_asm(T.a2<2>(a2));
        l[3] = lds_read_asm(T.a3<3>(a3));
        l[4] = lds_read_asm(T.a0<0>(a1));
        l[5] = lds_read_asm(T.a1<1>(a2));
        l[6] = lds_read_asm(T.a2<2>(a3));
        l[7] = lds_read_asm(T.a3<3>(a0));
        l[8] = lds_read_asm(T.a1<1>(a3));
        l[9] = lds_read_asm(T.a2<2>(a0));
        l[10] = lds_read_asm(T.a3<3>(a1));
        l[11] = lds_read_asm(T.a0<0>(a3));
        l[12] = lds_read_asm(T.a1<1>(a0));
        l[13] = lds_read_asm(T.a2<2>(a1));
        l[14] = lds_read_asm(T.a3<3>(a2));
        l[15] = 0u;
    }
    aes_pin<N>(L);
    uint32_t t[N][4];
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t* l = L + 16 * j;
        t[j][0] = xor3_u32(xor3_u32(l[0], l[1], l[2]), l[3], k1.x);
        t[j][1] = xor3_u32(xor3_u32(l[4], l[5], l[6]), l[7], k1.y);
        t[j][3] = xor3_u32(xor3_u32(l[11], l[12], l[13]), l[14], k1.w);
        g[j]->p2 = xor3_u32(l[8], l[9], l[10]) ^ k1.z;
        g[j]->a = T.a0<0>(a2v[j]);
    }
    // round 2: column c reads one byte of round-1 column 2 (c = 0: byte 2,
    // 1: byte 1, 2: byte 0, 3: byte 3); the other three lookups are shared
    uint32_t M[16 * N];  // 12 used per group
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t t0 = t[j][0], t1 = t[j][1], t3 = t[j][3];
        uint32_t* m = M + 16 * j;
        m[0] = lds_read_asm(T.a0<0>(t0));
        m[1] = lds_read_asm(T.a1<1>(t1));
        m[2] = lds_read_asm(T.a3<3>(t3));
        m[3] = lds_read_asm(T.a0<0>(t1));
        m[4] = lds_read_asm(T.a2<2>(t3));
        m[5] = lds_read_asm(T.a3<3>(t0));
        m[6] = lds_read_asm(T.a1<1>(t3));
        m[7] = lds_read_asm(T.a2<2>(t0));
        m[8] = lds_read_asm(T.a3<3>(t1));
        m[9] = lds_read_asm(T.a0<0>(t3));
        m[10] = lds_read_asm(T.a1<1>(t0));
        m[11] = lds_read_asm(T.a2<2>(t1));
#pragma unroll
        for (int i = 12; i < 16; i++) m[i] = 0u;
    }
    aes_pin<N>(M);
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t* m = M + 16 * j;
        g[j]->q[0] = xor3_u32(m[0], m[1], m[2]) ^ k2.x;
        g[j]->q[1] = xor3_u32(m[3], m[4], m[5]) ^ k2.y;
        g[j]->q[2] = xor3_u32(m[6], m[7], m[8]) ^ k2.z;
        g[j]->q[3] = xor3_u32(m[9], m[10], m[11]) ^ k2.w;
    }
}

// XofFixedKeyAes128 blocks j < N: counter ctr[j] of the seed of group g[j]
// (ctr[j] >> 8 must be the group's ctr_hi >> 8), in lockstep.
template <int N, class RK>
MH_D void ctr_blocks_n(const AesPerm& T, const RK& rk, const AesCtrGroup* const (&g)[N],
                       const uint32_t* const (&seed)[N], const uint32_t (&ctr)[N], uint32_t* const (&out)[N]) {
    // round 1: the one varying lookup per block
    uint32_t L1[N];
#pragma unroll
    for (int j = 0; j < N; j++) L1[j] = lds_read_asm(g[j]->a ^ ((ctr[j] & 0xffu) << 8));
    if constexpr (N == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(L1[0]));
    else if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(L1[0]), "+v"(L1[1]));
    else {
        static_assert(N == 4, "N = 1, 2 or 4");
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(L1[0]), "+v"(L1[1]), "+v"(L1[2]), "+v"(L1[3]));
    }
    // round 2: four lookups of round-1 column 2 per block
    uint32_t L2[4 * N];
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t u2 = g[j]->p2 ^ L1[j];
        L2[4 * j + 0] = lds_read_asm(T.a2<2>(u2));
        L2[4 * j + 1] = lds_read_asm(T.a1<1>(u2));
        L2[4 * j + 2] = lds_read_asm(T.a0<0>(u2));
        L2[4 * j + 3] = lds_read_asm(T.a3<3>(u2));
    }
    if constexpr (N == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(L2[0]), "+v"(L2[1]), "+v"(L2[2]), "+v"(L2[3]));
    else if constexpr (N == 2)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(L2[0]), "+v"(L2[1]), "+v"(L2[2]), "+v"(L2[3]), "+v"(L2[4]), "+v"(L2[5]), "+v"(L2[6]),
                       "+v"(L2[7]));
    else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(L2[0]), "+v"(L2[1]), "+v"(L2[2]), "+v"(L2[3]), "+v"(L2[4]), "+v"(L2[5]), "+v"(L2[6]),
                       "+v"(L2[7]), "+v"(L2[8]), "+v"(L2[9]), "+v"(L2[10]), "+v"(L2[11]), "+v"(L2[12]),
                       "+v"(L2[13]), "+v"(L2[14]), "+v"(L2[15]));
    uint32_t x[N][4];
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[j][c] = g[j]->q[c] ^ L2[4 * j + c];
#pragma unroll
    for (int r = 3; r < 10; r++) aes_round_n<N>(T, x, rk(r));
    aes_last_n<N>(T, x, rk(10));
    // output: AES(sigma) ^ sigma
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t* sd = seed[j];
        out[j][0] = x[j][0] ^ sd[2];
        out[j][1] = x[j][1] ^ sd[3];
        out[j][2] = xor3_u32(x[j][2], sd[2] ^ sd[0], ctr[j]);
        out[j][3] = xor3_u32(x[j][3], sd[3], sd[1]);
    }
}

// XofFixedKeyAes128 blocks (seed[j], ctr[j]) for j < N, in lockstep.
template <int N, class RK>
MH_D void fixed_key_block_n(const AesPerm& T, const RK& rk, const uint32_t* const (&seed)[N],
                            const uint32_t (&ctr)[N], uint32_t* const (&out)[N]) {
    uint32_t g[N][4], x[N][4];
#pragma unroll
    for (int j = 0; j < N; j++) {
        const uint32_t* sd = seed[j];
        g[j][0] = sd[2];
        g[j][1] = sd[3];
        g[j][2] = sd[2] ^ sd[0] ^ ctr[j];
        g[j][3] = sd[3] ^ sd[1];
#pragma unroll
        for (int c = 0; c < 4; c++) x[j][c] = g[j][c];
    }
    aes128_encrypt_n<N>(T, rk, x);
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) out[j][c] = x[j][c] ^ g[j][c];
}
