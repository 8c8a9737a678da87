/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into or called by the
 * product path (draft-mouris-cfrg-mastic_amd/).  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load this library, and only
 * as the checker / CPU baseline.
 *
 * Plain-C restatement of the two symmetric primitives the reference reaches
 * through the un-vendored dependency `vdaf_poc.xof` (pinned by
 * poc/requirements.txt:4, draft-irtf-cfrg-vdaf-13), which in turn calls
 * pycryptodomex 3.21.0 (poc/requirements.txt:3):
 *
 *   - TurboSHAKE128(M, D, L): Keccak-p[1600, 12] sponge, rate 168 B, domain
 *     byte D, pad10*1 (RFC 9861).  Used by XofTurboShake128 (node proofs
 *     poc/vidpf.py:377, checks poc/mastic.py:277-306, FLP randomness
 *     poc/mastic.py:452-510) and by the XofFixedKeyAes128 key derivation.
 *   - AES-128 block encryption (FIPS-197), used by XofFixedKeyAes128 for
 *     Vidpf.extend / Vidpf.convert (poc/vidpf.py:339,361).
 *
 * Straightforward byte-oriented code: correctness over speed.  It is pinned
 * by FIPS-197 / RFC 9861 known answers (tests/test_oracle_prims.py) and,
 * transitively, by every field of the reference's test_vec/mastic vectors.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

/* ------------------------------------------------------------------ */
/* Keccak-p[1600, 12]                                                   */
/* ------------------------------------------------------------------ */

static const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL,
    0x8000000080008000ULL, 0x000000000000808bULL, 0x0000000080000001ULL,
    0x8000000080008081ULL, 0x8000000000008009ULL, 0x000000000000008aULL,
    0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL,
    0x8000000000008003ULL, 0x8000000000008002ULL, 0x8000000000000080ULL,
    0x000000000000800aULL, 0x800000008000000aULL, 0x8000000080008081ULL,
    0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL,
};

static const int KECCAK_ROT[25] = {
    /* r[x + 5y] */
    0, 1, 62, 28, 27,
    36, 44, 6, 55, 20,
    3, 10, 43, 25, 39,
    41, 45, 15, 21, 8,
    18, 2, 61, 56, 14,
};

static inline uint64_t rotl64(uint64_t v, int r) {
    return r == 0 ? v : (v << r) | (v >> (64 - r));
}

/* The 12-round Keccak-p permutation uses round indices 12..23. */
void oracle_keccak_p1600_12(uint64_t a[25]) {
    for (int round = 12; round < 24; round++) {
        uint64_t c[5], d[5], b[25];
        for (int x = 0; x < 5; x++)
            c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; x++)
            d[x] = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
        for (int i = 0; i < 25; i++) a[i] ^= d[i % 5];
        /* rho + pi: B[y, 2x+3y] = rot(A[x, y], r[x, y]) */
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++)
                b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(a[x + 5 * y], KECCAK_ROT[x + 5 * y]);
        /* chi */
        for (int y = 0; y < 5; y++)
            for (int x = 0; x < 5; x++)
                a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= KECCAK_RC[round];
    }
}

static void xor_bytes_into_state(uint64_t st[25], const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) st[i / 8] ^= (uint64_t)p[i] << (8 * (i % 8));
}

/*
 * TurboSHAKE128(M, D, L) -> out[0..L).  The message is given as up to
 * `nparts` pieces that are concatenated (so callers need not allocate).
 */
void oracle_turboshake128_parts(const uint8_t *const *parts, const size_t *lens, int nparts,
                                uint8_t domain, uint8_t *out, size_t out_len) {
    uint64_t st[25];
    uint8_t block[168];
    size_t fill = 0;
    memset(st, 0, sizeof(st));
    for (int k = 0; k < nparts; k++) {
        const uint8_t *p = parts[k];
        size_t n = lens[k];
        while (n > 0) {
            size_t take = 168 - fill;
            if (take > n) take = n;
            memcpy(block + fill, p, take);
            fill += take; p += take; n -= take;
            if (fill == 168) {
                xor_bytes_into_state(st, block, 168);
                oracle_keccak_p1600_12(st);
                fill = 0;
            }
        }
    }
    memset(block + fill, 0, 168 - fill);
    block[fill] ^= domain;
    block[167] ^= 0x80;
    xor_bytes_into_state(st, block, 168);
    oracle_keccak_p1600_12(st);
    size_t done = 0;
    for (;;) {
        for (size_t i = 0; i < 168 && done < out_len; i++, done++)
            out[done] = (uint8_t)(st[i / 8] >> (8 * (i % 8)));
        if (done >= out_len) break;
        oracle_keccak_p1600_12(st);
    }
}

void oracle_turboshake128(const uint8_t *msg, size_t msg_len, uint8_t domain,
                          uint8_t *out, size_t out_len) {
    const uint8_t *parts[1] = {msg};
    size_t lens[1] = {msg_len};
    oracle_turboshake128_parts(parts, lens, 1, domain, out, out_len);
}

/* ------------------------------------------------------------------ */
/* AES-128 (FIPS-197), plain byte-oriented implementation               */
/* ------------------------------------------------------------------ */

static uint8_t SBOX[256];
static int sbox_ready = 0;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

static void build_sbox(void) {
    /* S(x) = affine(x^-1), derived rather than tabulated. */
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; y++)
                if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        }
        uint8_t s = inv;
        uint8_t r = inv;
        for (int i = 0; i < 4; i++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        SBOX[x] = s ^ 0x63;
    }
    sbox_ready = 1;
}

void oracle_aes128_expand(const uint8_t key[16], uint8_t rk[176]) {
    if (!sbox_ready) build_sbox();
    memcpy(rk, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t t0 = t[0];
            t[0] = SBOX[t[1]] ^ rcon;
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[t0];
            rcon = gf_mul(rcon, 2);
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = rk[4 * (i - 4) + j] ^ t[j];
    }
}

void oracle_aes128_encrypt(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
    if (!sbox_ready) build_sbox();
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int round = 1; round <= 10; round++) {
        uint8_t t[16];
        /* SubBytes + ShiftRows (state is column-major: s[r + 4c]) */
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++)
                t[r + 4 * c] = SBOX[s[r + 4 * ((c + r) % 4)]];
        if (round != 10) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = gf_mul(a0, 2) ^ gf_mul(a1, 3) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ gf_mul(a1, 2) ^ gf_mul(a2, 3) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ gf_mul(a2, 2) ^ gf_mul(a3, 3);
                s[4 * c + 3] = gf_mul(a0, 3) ^ a1 ^ a2 ^ gf_mul(a3, 2);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

/*
 * XofFixedKeyAes128.hash_block over `nblocks` consecutive counters:
 *   x = seed XOR le128(ctr), sigma(x) = x[8:16] || (x[8:16] XOR x[0:8]),
 *   out = AES_k(sigma(x)) XOR sigma(x)      (vdaf_poc.xof)
 */
void oracle_fixed_key_aes_blocks(const uint8_t rk[176], const uint8_t seed[16],
                                 uint64_t first_ctr, size_t nblocks, uint8_t *out) {
    for (size_t b = 0; b < nblocks; b++) {
        uint8_t x[16], sig[16], enc[16];
        memcpy(x, seed, 16);
        uint64_t ctr = first_ctr + b;
        for (int i = 0; i < 8; i++) x[i] ^= (uint8_t)(ctr >> (8 * i));
        for (int i = 0; i < 8; i++) {
            sig[i] = x[8 + i];
            sig[8 + i] = x[8 + i] ^ x[i];
        }
        oracle_aes128_encrypt(rk, sig, enc);
        for (int i = 0; i < 16; i++) out[16 * b + i] = enc[i] ^ sig[i];
    }
}
