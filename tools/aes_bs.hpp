// Bitsliced AES-128 for the XofFixedKeyAes128 counter stream (VERDICT r3 item
// 1: the measured alternative to the LDS T-table AES of the Field128 payload
// loop).  32-way bitslice: one 32-bit word per state bit, bit j of every word
// belongs to block j, so one lane encrypts 32 blocks under ITS OWN key (the
// level kernel's layout: lane = report, per-report key).  Generic over the
// word type so the host test (tests/host/aes_bs_check.cpp) checks it against
// FIPS-197 and a byte-wise AES; tools/aes_bs_mb.hip times it on gfx950.
//
// Layout: s[i][b] = bit b (0 = LSB) of state byte i (FIPS-197 byte order,
// byte i = row i % 4, column i / 4).  Round keys enter as masks through a
// functor km(round, word, bit) -> W (all ones where that key bit is set); the
// S-box's affine constant 0x63 is folded into the round keys of rounds 1..10
// (MixColumns maps the constant column (c, c, c, c) to itself), so the S-box
// circuit below has no NOT gates.
//
// Counter stream (vdaf-13 XofFixedKeyAes128.hash_block): block j of a batch
// encrypts sigma(seed ^ le128(base + j)) = (s2, s3, s2 ^ s0 ^ ctr, s3 ^ s1);
// with base % 32 == 0 the 32 blocks differ only in bits 0..4 of state byte 8,
// so the input "transposition" is 128 broadcast masks plus 5 constant
// patterns, and round 1 shares all but one S-box input.  Not part of the
// product (DESIGN.md §5 "Bitsliced AES").
#pragma once
#include <stdint.h>

#ifndef MH_HD
#define MH_HD inline
#endif

template <class W>
MH_HD W bs_x3(W a, W b, W c) {
    return a ^ b ^ c;
}

// bit j of BS_PAT[b] = bit b of j: the counter's low five bits across a batch
static constexpr uint32_t BS_PAT[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};

// AES S-box (without its affine constant 0x63) on eight bit-slices, in place:
// the depth-16, 113-gate circuit of Boyar and Peralta ("A depth-16 circuit for
// the AES S-box", 2011): a linear top layer, a shared nonlinear middle (GF(2^4)
// inversion) and a linear bottom layer.  u0 is the most significant bit.
template <class W>
MH_HD void bs_sbox(W (&q)[8]) {
    const W u0 = q[7], u1 = q[6], u2 = q[5], u3 = q[4], u4 = q[3], u5 = q[2], u6 = q[1], u7 = q[0];
    // top linear layer
    const W y14 = u3 ^ u5, y13 = u0 ^ u6, y9 = u0 ^ u3, y8 = u0 ^ u5;
    const W t0 = u1 ^ u2;
    const W y1 = t0 ^ u7, y4 = y1 ^ u3, y12 = y13 ^ y14, y2 = y1 ^ u0, y5 = y1 ^ u6;
    const W y3 = y5 ^ y8;
    const W t1 = u4 ^ y12;
    const W y15 = t1 ^ u5, y20 = t1 ^ u1;
    const W y6 = y15 ^ u7, y10 = y15 ^ t0, y11 = y20 ^ y9;
    const W y7 = u7 ^ y11, y17 = y10 ^ y11, y19 = y10 ^ y8, y16 = t0 ^ y11;
    const W y21 = y13 ^ y16, y18 = u0 ^ y16;
    // nonlinear middle
    const W t2 = y12 & y15, t3 = y3 & y6, t4 = t3 ^ t2, t5 = y4 & u7, t6 = t5 ^ t2;
    const W t7 = y13 & y16, t8 = y5 & y1, t9 = t8 ^ t7, t10 = y2 & y7, t11 = t10 ^ t7;
    const W t12 = y9 & y11, t13 = y14 & y17, t14 = t13 ^ t12, t15 = y8 & y10, t16 = t15 ^ t12;
    const W t17 = t4 ^ t14, t18 = t6 ^ t16, t19 = t9 ^ t14, t20 = t11 ^ t16;
    const W t21 = t17 ^ y20, t22 = t18 ^ y19, t23 = t19 ^ y21, t24 = t20 ^ y18;
    const W t25 = t21 ^ t22, t26 = t21 & t23, t27 = t24 ^ t26, t28 = t25 & t27, t29 = t28 ^ t22;
    const W t30 = t23 ^ t24, t31 = t22 ^ t26, t32 = t31 & t30, t33 = t32 ^ t24, t34 = t23 ^ t33;
    const W t35 = t27 ^ t33, t36 = t24 & t35, t37 = t36 ^ t34, t38 = t27 ^ t36, t39 = t29 & t38;
    const W t40 = t25 ^ t39;
    const W t41 = t40 ^ t37, t42 = t29 ^ t33, t43 = t29 ^ t40, t44 = t33 ^ t37, t45 = t42 ^ t41;
    const W z0 = t44 & y15, z1 = t37 & y6, z2 = t33 & u7, z3 = t43 & y16, z4 = t40 & y1, z5 = t29 & y7;
    const W z6 = t42 & y11, z7 = t45 & y17, z8 = t41 & y10, z9 = t44 & y12, z10 = t37 & y3, z11 = t33 & y4;
    const W z12 = t43 & y13, z13 = t40 & y5, z14 = t29 & y2, z15 = t42 & y9, z16 = t45 & y14, z17 = t41 & y8;
    // bottom linear layer
    const W t46 = z15 ^ z16, t47 = z10 ^ z11, t48 = z5 ^ z13, t49 = z9 ^ z10, t50 = z2 ^ z12;
    const W t51 = z2 ^ z5, t52 = z7 ^ z8, t53 = z0 ^ z3, t54 = z6 ^ z7, t55 = z16 ^ z17;
    const W t56 = z12 ^ t48, t57 = t50 ^ t53, t58 = z4 ^ t46, t59 = z3 ^ t54, t60 = t46 ^ t57;
    const W t61 = z14 ^ t57, t62 = t52 ^ t58, t63 = t49 ^ t58, t64 = z4 ^ t59, t65 = t61 ^ t62;
    const W t66 = z1 ^ t63;
    const W s0 = t59 ^ t63, s6 = t56 ^ t62, s7 = t48 ^ t60;
    const W t67 = t64 ^ t65;
    const W s3 = t53 ^ t66, s4 = t51 ^ t66, s5 = t47 ^ t65;
    const W s1 = t64 ^ s3, s2 = t55 ^ t67;
    q[7] = s0; q[6] = s1; q[5] = s2; q[4] = s3;
    q[3] = s4; q[2] = s5; q[1] = s6; q[0] = s7;
}

// ShiftRows as a source index: output byte i (row r, column c) takes input
// byte (row r, column c + r mod 4)
constexpr int bs_sr(int i) { return (i & 3) + 4 * (((i >> 2) + (i & 3)) & 3); }

// One middle round on s: SubBytes, ShiftRows, MixColumns, AddRoundKey (round r).
template <class W, class KM>
MH_HD void bs_round(W (&s)[16][8], const KM& km, int r) {
#pragma unroll
    for (int i = 0; i < 16; i++) bs_sbox(s[i]);
    W o[16][8];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        // column c after ShiftRows: a[row] = s[bs_sr(4c + row)]
        const W(&a0)[8] = s[bs_sr(4 * c + 0)];
        const W(&a1)[8] = s[bs_sr(4 * c + 1)];
        const W(&a2)[8] = s[bs_sr(4 * c + 2)];
        const W(&a3)[8] = s[bs_sr(4 * c + 3)];
        const W* a[4] = {a0, a1, a2, a3};
        W t[4][8], u[8];
#pragma unroll
        for (int b = 0; b < 8; b++) {
            t[0][b] = a0[b] ^ a1[b];
            t[1][b] = a1[b] ^ a2[b];
            t[2][b] = a2[b] ^ a3[b];
            t[3][b] = a3[b] ^ a0[b];
            u[b] = t[0][b] ^ t[2][b];
        }
        // out_row = xtime(a_row ^ a_row+1) ^ (a_row+1 ^ a_row+2 ^ a_row+3) ^ k
#pragma unroll
        for (int row = 0; row < 4; row++) {
            const W* tt = t[row];
            const W* ar = a[row];
            W* out = o[4 * c + row];
            const int w = c, sh = 8 * row;  // key word / bit offset of byte 4c + row
            out[0] = bs_x3(tt[7], u[0], ar[0]) ^ km(r, w, sh + 0);
            out[1] = bs_x3(bs_x3(tt[0], tt[7], u[1]), ar[1], km(r, w, sh + 1));
            out[2] = bs_x3(tt[1], u[2], ar[2]) ^ km(r, w, sh + 2);
            out[3] = bs_x3(bs_x3(tt[2], tt[7], u[3]), ar[3], km(r, w, sh + 3));
            out[4] = bs_x3(bs_x3(tt[3], tt[7], u[4]), ar[4], km(r, w, sh + 4));
            out[5] = bs_x3(tt[4], u[5], ar[5]) ^ km(r, w, sh + 5);
            out[6] = bs_x3(tt[5], u[6], ar[6]) ^ km(r, w, sh + 6);
            out[7] = bs_x3(tt[6], u[7], ar[7]) ^ km(r, w, sh + 7);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; i++)
#pragma unroll
        for (int b = 0; b < 8; b++) s[i][b] = o[i][b];
}

// Last round: SubBytes, ShiftRows, AddRoundKey (round 10).
template <class W, class KM>
MH_HD void bs_last(W (&s)[16][8], const KM& km) {
#pragma unroll
    for (int i = 0; i < 16; i++) bs_sbox(s[i]);
    W o[16][8];
#pragma unroll
    for (int i = 0; i < 16; i++)
#pragma unroll
        for (int b = 0; b < 8; b++) o[i][b] = s[bs_sr(i)][b] ^ km(10, i >> 2, 8 * (i & 3) + b);
#pragma unroll
    for (int i = 0; i < 16; i++)
#pragma unroll
        for (int b = 0; b < 8; b++) s[i][b] = o[i][b];
}

// In-place 32 x 32 bit-matrix transpose: afterwards bit k of r[j] is the
// former bit j of r[k].
template <class W>
MH_HD void bs_transpose32(W (&r)[32]) {
    const W m[5] = {(W)0x55555555u, (W)0x33333333u, (W)0x0F0F0F0Fu, (W)0x00FF00FFu, (W)0x0000FFFFu};
#pragma unroll
    for (int st = 4; st >= 0; st--) {
        const int w = 1 << st;
#pragma unroll
        for (int i = 0; i < 32; i++) {
            if (i & w) continue;
            // swap the high w-bit groups of r[i] with the low ones of r[i + w]
            const W t = ((r[i] >> w) ^ r[i + w]) & m[st];
            r[i + w] ^= t;
            r[i] ^= t << w;
        }
    }
}

// 32 XofFixedKeyAes128 blocks (ctr = base + j, base % 32 == 0) of one seed.
// bm(v, bit) -> W: the broadcast mask of bit `bit` of the lane's word v.
// km(round, word, bit): round-key masks (rounds 1..10 with 0x63 folded in).
// rk0: round key 0 as plain words.  out[j][w]: word w of block j.
template <class W, class BM, class KM>
MH_HD void bs_ctr32(const uint32_t seed[4], uint32_t base, const uint32_t rk0[4], const BM& bm, const KM& km,
                    W (&out)[32][4]) {
    const uint32_t sg[4] = {seed[2], seed[3], seed[2] ^ seed[0] ^ base, seed[3] ^ seed[1]};
    W s[16][8];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t v = sg[i >> 2] ^ rk0[i >> 2];
#pragma unroll
        for (int b = 0; b < 8; b++) s[i][b] = bm(v, 8 * (i & 3) + b);
    }
#pragma unroll
    for (int b = 0; b < 5; b++) s[8][b] ^= (W)BS_PAT[b];
#pragma unroll
    for (int r = 1; r < 10; r++) bs_round(s, km, r);
    bs_last(s, km);
    // output = AES(sigma) ^ sigma, in the sliced domain, then back to blocks
#pragma unroll
    for (int w = 0; w < 4; w++) {
        W R[32];
#pragma unroll
        for (int k = 0; k < 32; k++) R[k] = s[4 * w + (k >> 3)][k & 7] ^ bm(sg[w], k);
        if (w == 2) {
#pragma unroll
            for (int b = 0; b < 5; b++) R[b] ^= (W)BS_PAT[b];
        }
        bs_transpose32(R);
#pragma unroll
        for (int j = 0; j < 32; j++) out[j][w] = R[j];
    }
}
