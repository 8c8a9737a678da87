// Host check of the bitsliced AES-128 counter stream (tools/aes_bs.hpp)
// against a byte-wise FIPS-197 AES: the FIPS-197 C.1 known answer, then random
// seeds / keys / counter bases, 32 blocks each (XofFixedKeyAes128.hash_block,
// vdaf-13).  Prints "ok" and exits 0 on success.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../tools/aes_bs.hpp"

static uint8_t SBOX[256];

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) p ^= a;
        const uint8_t hi = a & 0x80;
        a <<= 1;
        if (hi) a ^= 0x1b;
        b >>= 1;
    }
    return p;
}

static void make_sbox() {
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        for (int y = 1; y < 256 && x; y++)
            if (gmul((uint8_t)x, (uint8_t)y) == 1) inv = (uint8_t)y;
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; i++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        SBOX[x] = s ^ 0x63;
    }
}

// key schedule as 44 little-endian words (byte 4w + k of the round-key block = byte k of word w)
static void expand(const uint8_t key[16], uint32_t rk[44]) {
    memcpy(rk, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint32_t t = rk[i - 1];
        if (i % 4 == 0) {
            const uint8_t b[4] = {(uint8_t)(t >> 8), (uint8_t)(t >> 16), (uint8_t)(t >> 24), (uint8_t)t};
            t = (uint32_t)(SBOX[b[0]] ^ rcon) | (uint32_t)SBOX[b[1]] << 8 | (uint32_t)SBOX[b[2]] << 16 |
                (uint32_t)SBOX[b[3]] << 24;
            rcon = gmul(rcon, 2);
        }
        rk[i] = rk[i - 4] ^ t;
    }
}

static void aes_ref(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    const uint8_t* k = (const uint8_t*)rk;
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ k[i];
    for (int r = 1; r <= 10; r++) {
        uint8_t t[16];
        for (int i = 0; i < 16; i++) t[i] = SBOX[s[bs_sr(i)]];
        if (r < 10) {
            for (int c = 0; c < 4; c++) {
                const uint8_t* a = t + 4 * c;
                uint8_t m[4];
                for (int row = 0; row < 4; row++)
                    m[row] = gmul(a[row], 2) ^ gmul(a[(row + 1) & 3], 3) ^ a[(row + 2) & 3] ^ a[(row + 3) & 3];
                memcpy(s + 4 * c, m, 4);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= k[16 * r + i];
    }
    memcpy(out, s, 16);
}

static bool run_batch(const uint32_t rk[44], const uint32_t seed[4], uint32_t base) {
    auto bm = [](uint32_t v, int bit) -> uint32_t { return 0u - ((v >> bit) & 1u); };
    auto km = [&](int r, int w, int bit) -> uint32_t {
        const uint32_t kw = rk[4 * r + w] ^ (r >= 1 ? 0x63636363u : 0u);
        return 0u - ((kw >> bit) & 1u);
    };
    uint32_t out[32][4];
    bs_ctr32<uint32_t>(seed, base, rk, bm, km, out);
    for (int j = 0; j < 32; j++) {
        const uint32_t ctr = base + (uint32_t)j;
        const uint32_t sg[4] = {seed[2], seed[3], seed[2] ^ seed[0] ^ ctr, seed[3] ^ seed[1]};
        uint8_t in[16], enc[16];
        memcpy(in, sg, 16);
        aes_ref(rk, in, enc);
        uint32_t want[4];
        memcpy(want, enc, 16);
        for (int w = 0; w < 4; w++)
            if ((want[w] ^ sg[w]) != out[j][w]) {
                printf("mismatch block %d word %d: %08x vs %08x\n", j, w, want[w] ^ sg[w], out[j][w]);
                return false;
            }
    }
    return true;
}

int main() {
    make_sbox();
    if (SBOX[0] != 0x63 || SBOX[0x53] != 0xed) {
        printf("sbox construction wrong\n");
        return 1;
    }
    // the bitsliced S-box alone, exhaustively (bit j of slice b = bit b of input j + 32 * g)
    for (int g = 0; g < 8; g++) {
        uint32_t q[8] = {0};
        for (int j = 0; j < 32; j++)
            for (int b = 0; b < 8; b++) q[b] |= (uint32_t)(((32 * g + j) >> b) & 1) << j;
        bs_sbox(q);
        for (int j = 0; j < 32; j++) {
            int v = 0;
            for (int b = 0; b < 8; b++) v |= (int)((q[b] >> j) & 1) << b;
            if ((v ^ 0x63) != SBOX[32 * g + j]) {
                printf("bs_sbox(%02x) = %02x, want %02x\n", 32 * g + j, v ^ 0x63, SBOX[32 * g + j]);
                return 1;
            }
        }
    }
    // FIPS-197 C.1: key 000102..0f, plaintext 00112233..ff -> 69c4e0d86a7b0430d8cdb78070b4c55a
    uint8_t key[16], pt[16];
    for (int i = 0; i < 16; i++) {
        key[i] = (uint8_t)i;
        pt[i] = (uint8_t)(0x11 * i);
    }
    uint32_t rk[44];
    expand(key, rk);
    static const uint8_t want_c1[16] = {0x69, 0xc4, 0xe0, 0xd8, 0x6a, 0x7b, 0x04, 0x30,
                                        0xd8, 0xcd, 0xb7, 0x80, 0x70, 0xb4, 0xc5, 0x5a};
    uint8_t ref[16];
    aes_ref(rk, pt, ref);
    if (memcmp(ref, want_c1, 16) != 0) {
        printf("reference AES fails FIPS-197 C.1\n");
        return 1;
    }
    // a seed whose block 0 input sigma(seed ^ base) is the C.1 plaintext
    uint32_t p[4];
    memcpy(p, pt, 16);
    const uint32_t base = 0x40u;
    const uint32_t seed[4] = {p[2] ^ p[0] ^ base, p[3] ^ p[1], p[0], p[1]};
    {
        auto bm = [](uint32_t v, int bit) -> uint32_t { return 0u - ((v >> bit) & 1u); };
        auto km = [&](int r, int w, int bit) -> uint32_t {
            const uint32_t kw = rk[4 * r + w] ^ (r >= 1 ? 0x63636363u : 0u);
            return 0u - ((kw >> bit) & 1u);
        };
        uint32_t out[32][4];
        bs_ctr32<uint32_t>(seed, base, rk, bm, km, out);
        uint32_t c[4];
        for (int w = 0; w < 4; w++) c[w] = out[0][w] ^ p[w];
        if (memcmp(c, want_c1, 16) != 0) {
            printf("bitsliced AES fails FIPS-197 C.1\n");
            return 1;
        }
    }
    // random keys, seeds and counter bases
    srand(12345);
    for (int t = 0; t < 200; t++) {
        for (int i = 0; i < 16; i++) key[i] = (uint8_t)rand();
        expand(key, rk);
        uint32_t sd[4];
        for (int w = 0; w < 4; w++) sd[w] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
        const uint32_t b = ((uint32_t)rand() % 2048u) * 32u;
        if (!run_batch(rk, sd, b)) return 1;
    }
    printf("ok\n");
    return 0;
}
