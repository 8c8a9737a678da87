/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Never linked into or called by the
 * product path (draft-mouris-cfrg-mastic_amd/).  bench.py's cpu_baseline leg
 * times it as the NATIVE multithreaded CPU baseline, and tests/ check it
 * against the Python oracle and the reference's golden vectors.
 *
 * A competent CPU implementation of the VIDPF part of Mastic.prep_init
 * (poc/mastic.py:205-318; the FLP query of the weight check stays in the
 * Python oracle, under 1 % of the work at C2): eval_with_siblings
 * (poc/vidpf.py:213-261) with eval_next / extend / convert / node_proof
 * (:281-380), the BFS one-hot and payload binders and their checks, the
 * counter check and the eval proof (mastic.py:259-306), the beta share
 * (vidpf.py:263-279) and the truncated out shares (mastic.py:308-316).
 * AES-128 through AES-NI when the CPU has it (a byte-wise FIPS-197 fallback
 * otherwise), a 64-bit Keccak-p[1600,12], one thread per report range
 * (pthreads).  The tree walk is the reference's: per report, each candidate
 * prefix descends from the root and evaluates both children of every node on
 * its path once.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

typedef unsigned __int128 u128;

/* ------------------------------------------------------------ Keccak */
static const uint64_t RC12[12] = {
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL,
};
#define ROL(v, r) (((v) << (r)) | ((v) >> (64 - (r))))

static void keccak12(uint64_t A[25]) {
    for (int rd = 0; rd < 12; rd++) {
        uint64_t C0 = A[0] ^ A[5] ^ A[10] ^ A[15] ^ A[20], C1 = A[1] ^ A[6] ^ A[11] ^ A[16] ^ A[21];
        uint64_t C2 = A[2] ^ A[7] ^ A[12] ^ A[17] ^ A[22], C3 = A[3] ^ A[8] ^ A[13] ^ A[18] ^ A[23];
        uint64_t C4 = A[4] ^ A[9] ^ A[14] ^ A[19] ^ A[24];
        uint64_t D0 = C4 ^ ROL(C1, 1), D1 = C0 ^ ROL(C2, 1), D2 = C1 ^ ROL(C3, 1), D3 = C2 ^ ROL(C4, 1),
                 D4 = C3 ^ ROL(C0, 1);
        uint64_t B[25];
        /* B[y, 2x+3y] = rot(A[x, y] ^ D[x], r[x, y]) */
        B[0] = A[0] ^ D0;
        B[10] = ROL(A[1] ^ D1, 1);
        B[20] = ROL(A[2] ^ D2, 62);
        B[5] = ROL(A[3] ^ D3, 28);
        B[15] = ROL(A[4] ^ D4, 27);
        B[16] = ROL(A[5] ^ D0, 36);
        B[1] = ROL(A[6] ^ D1, 44);
        B[11] = ROL(A[7] ^ D2, 6);
        B[21] = ROL(A[8] ^ D3, 55);
        B[6] = ROL(A[9] ^ D4, 20);
        B[7] = ROL(A[10] ^ D0, 3);
        B[17] = ROL(A[11] ^ D1, 10);
        B[2] = ROL(A[12] ^ D2, 43);
        B[12] = ROL(A[13] ^ D3, 25);
        B[22] = ROL(A[14] ^ D4, 39);
        B[23] = ROL(A[15] ^ D0, 41);
        B[8] = ROL(A[16] ^ D1, 45);
        B[18] = ROL(A[17] ^ D2, 15);
        B[3] = ROL(A[18] ^ D3, 21);
        B[13] = ROL(A[19] ^ D4, 8);
        B[14] = ROL(A[20] ^ D0, 18);
        B[24] = ROL(A[21] ^ D1, 2);
        B[9] = ROL(A[22] ^ D2, 61);
        B[19] = ROL(A[23] ^ D3, 56);
        B[4] = ROL(A[24] ^ D4, 14);
        for (int y = 0; y < 25; y += 5) {
            const uint64_t b0 = B[y], b1 = B[y + 1], b2 = B[y + 2], b3 = B[y + 3], b4 = B[y + 4];
            A[y] = b0 ^ (~b1 & b2);
            A[y + 1] = b1 ^ (~b2 & b3);
            A[y + 2] = b2 ^ (~b3 & b4);
            A[y + 3] = b3 ^ (~b4 & b0);
            A[y + 4] = b4 ^ (~b0 & b1);
        }
        A[0] ^= RC12[rd];
    }
}

/* TurboSHAKE128 with incremental absorb (little-endian host) */
typedef struct {
    uint64_t st[25];
    size_t fill; /* bytes absorbed into the current block */
} ts_t;

static void ts_init(ts_t* t) {
    memset(t->st, 0, sizeof t->st);
    t->fill = 0;
}
static void ts_absorb(ts_t* t, const uint8_t* p, size_t n) {
    uint8_t* s = (uint8_t*)t->st;
    while (n) {
        if (t->fill == 0 && n >= 168) {
            const uint64_t* w = (const uint64_t*)p;
            for (int i = 0; i < 21; i++) {
                uint64_t v;
                memcpy(&v, w + i, 8);
                t->st[i] ^= v;
            }
            keccak12(t->st);
            p += 168;
            n -= 168;
            continue;
        }
        size_t k = 168 - t->fill;
        if (k > n) k = n;
        for (size_t i = 0; i < k; i++) s[t->fill + i] ^= p[i];
        t->fill += k;
        p += k;
        n -= k;
        if (t->fill == 168) {
            keccak12(t->st);
            t->fill = 0;
        }
    }
}
static void ts_final(ts_t* t, uint8_t domain, uint8_t* out, size_t outlen) {
    uint8_t* s = (uint8_t*)t->st;
    s[t->fill] ^= domain;
    s[167] ^= 0x80;
    keccak12(t->st);
    size_t done = 0;
    for (;;) {
        size_t k = outlen - done < 168 ? outlen - done : 168;
        memcpy(out + done, s, k);
        done += k;
        if (done == outlen) break;
        keccak12(t->st);
    }
}
static void put_le16(uint8_t* p, unsigned v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}
/* XofTurboShake128(seed, dst, binder) prefix: le16(len(dst)) || dst || u8(len(seed)) || seed */
static void xts_begin(ts_t* t, const uint8_t* dst, size_t dlen, const uint8_t* seed, size_t slen) {
    uint8_t h[2];
    ts_init(t);
    put_le16(h, (unsigned)dlen);
    ts_absorb(t, h, 2);
    ts_absorb(t, dst, dlen);
    uint8_t sl = (uint8_t)slen;
    ts_absorb(t, &sl, 1);
    if (slen) ts_absorb(t, seed, slen);
}

/* ------------------------------------------------------------ AES-128 */
static uint8_t SB[256];
static int sb_ready = 0;
static pthread_once_t sb_once = PTHREAD_ONCE_INIT;
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) p ^= a;
        uint8_t hi = a & 0x80;
        a <<= 1;
        if (hi) a ^= 0x1b;
        b >>= 1;
    }
    return p;
}
static void sb_init(void) {
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        for (int y = 1; y < 256 && x; y++)
            if (gmul((uint8_t)x, (uint8_t)y) == 1) inv = (uint8_t)y;
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; i++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        SB[x] = s ^ 0x63;
    }
    sb_ready = 1;
}
static void aes_expand(const uint8_t key[16], uint8_t rk[176]) {
    pthread_once(&sb_once, sb_init);
    memcpy(rk, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t u = t[0];
            t[0] = SB[t[1]] ^ rcon;
            t[1] = SB[t[2]];
            t[2] = SB[t[3]];
            t[3] = SB[u];
            rcon = gmul(rcon, 2);
        }
        for (int k = 0; k < 4; k++) rk[4 * i + k] = rk[4 * (i - 4) + k] ^ t[k];
    }
}
static void aes_enc_soft(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= 10; r++) {
        for (int i = 0; i < 16; i++) t[i] = SB[s[(i & 3) + 4 * (((i >> 2) + (i & 3)) & 3)]];
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
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

static int use_aesni = 0;

/* XofFixedKeyAes128 blocks [ctr0, ctr0 + n) of seed: AES(sigma(x)) ^ sigma(x), x = seed ^ le128(ctr) */
#if defined(__x86_64__)
__attribute__((target("aes,sse4.1"))) static void fk_blocks_ni(const uint8_t rk[176], const uint8_t seed[16],
                                                               uint64_t ctr0, int n, uint8_t* out) {
    __m128i k[11];
    for (int i = 0; i < 11; i++) k[i] = _mm_loadu_si128((const __m128i*)(rk + 16 * i));
    const __m128i sd = _mm_loadu_si128((const __m128i*)seed);
    int j = 0;
    for (; j + 4 <= n; j += 4) {
        __m128i sg[4], x[4];
        for (int q = 0; q < 4; q++) {
            const __m128i xs = _mm_xor_si128(sd, _mm_set_epi64x(0, (long long)(ctr0 + j + q)));
            const __m128i hi = _mm_unpackhi_epi64(xs, xs);              /* x[8:16] twice */
            sg[q] = _mm_xor_si128(hi, _mm_slli_si128(xs, 8));           /* (x_hi, x_hi ^ x_lo) */
            x[q] = _mm_xor_si128(sg[q], k[0]);
        }
        for (int r = 1; r < 10; r++)
            for (int q = 0; q < 4; q++) x[q] = _mm_aesenc_si128(x[q], k[r]);
        for (int q = 0; q < 4; q++)
            _mm_storeu_si128((__m128i*)(out + 16 * (j + q)),
                             _mm_xor_si128(_mm_aesenclast_si128(x[q], k[10]), sg[q]));
    }
    for (; j < n; j++) {
        const __m128i xs = _mm_xor_si128(sd, _mm_set_epi64x(0, (long long)(ctr0 + j)));
        const __m128i sg = _mm_xor_si128(_mm_unpackhi_epi64(xs, xs), _mm_slli_si128(xs, 8));
        __m128i x = _mm_xor_si128(sg, k[0]);
        for (int r = 1; r < 10; r++) x = _mm_aesenc_si128(x, k[r]);
        _mm_storeu_si128((__m128i*)(out + 16 * j), _mm_xor_si128(_mm_aesenclast_si128(x, k[10]), sg));
    }
}
#endif
static void fk_blocks(const uint8_t rk[176], const uint8_t seed[16], uint64_t ctr0, int n, uint8_t* out) {
#if defined(__x86_64__)
    if (use_aesni) {
        fk_blocks_ni(rk, seed, ctr0, n, out);
        return;
    }
#endif
    for (int j = 0; j < n; j++) {
        uint8_t x[16], sg[16], c[16];
        memcpy(x, seed, 16);
        uint64_t ctr = ctr0 + (uint64_t)j;
        for (int i = 0; i < 8; i++) x[i] ^= (uint8_t)(ctr >> (8 * i));
        for (int i = 0; i < 8; i++) {
            sg[i] = x[8 + i];
            sg[8 + i] = x[8 + i] ^ x[i];
        }
        aes_enc_soft(rk, sg, c);
        for (int i = 0; i < 16; i++) out[16 * j + i] = c[i] ^ sg[i];
    }
}

/* ------------------------------------------------------------ fields */
static const uint64_t P64 = 0xFFFFFFFF00000001ULL;
#define P128 (((u128)0xFFFFFFFFFFFFFFE4ULL << 64) | 1u) /* 2^128 - 28 * 2^64 + 1 */

typedef struct {
    int fbits, enc, vl;
} fld_t;

static u128 f_add(const fld_t* f, u128 a, u128 b) {
    if (f->fbits == 64) {
        const uint64_t x = (uint64_t)a, y = (uint64_t)b;
        uint64_t s = x + y;
        if (s < x || s >= P64) s -= P64; /* a carry out: x + y - 2^64 + (2^64 - P64) */
        return s;
    }
    u128 s = a + b;
    if (s < a || s >= P128) s -= P128; /* wrap: a + b - 2^128 + (2^128 - P) */
    return s;
}
static u128 f_neg(const fld_t* f, u128 a) { return a == 0 ? 0 : (f->fbits == 64 ? (u128)P64 - a : P128 - a); }
static u128 f_sub(const fld_t* f, u128 a, u128 b) { return f_add(f, a, f_neg(f, b)); }
/* little-endian encode_vec elements (x86 host) */
static u128 f_get(const fld_t* f, const uint8_t* p) {
    uint64_t lo, hi = 0;
    memcpy(&lo, p, 8);
    if (f->enc == 16) memcpy(&hi, p + 8, 8);
    return ((u128)hi << 64) | lo;
}
static void f_put(const fld_t* f, uint8_t* p, u128 v) {
    const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    memcpy(p, &lo, 8);
    if (f->enc == 16) memcpy(p + 8, &hi, 8);
}

/* ------------------------------------------------------------ job */
typedef struct {
    fld_t f;
    int bits, agg_id, level, n_prefixes, tgroup, tlimit;
    const uint8_t* prefixes; /* n_prefixes x pbytes, MSB-first */
    int pbytes;
    const uint8_t *dst_ext, *dst_conv, *dst_node, *dst_onehot, *dst_payload, *dst_eval;
    size_t l_ext, l_conv, l_node, l_onehot, l_payload, l_eval;
    const uint8_t* vk;
    size_t vk_len;
    int ps_size, is_size;
    const uint8_t *nonces, *pubs, *ins;
    uint8_t *eval_proofs, *beta_shares, *out_shares;
    int out_row; /* bytes of one report's truncated out shares */
} job_t;

typedef struct {
    uint8_t seed[16];
    uint8_t ctrl;
    int32_t left, right;
    uint8_t proof[32];
} node_t;

typedef struct {
    const job_t* J;
    size_t lo, hi;
    int rc;
} part_t;

static int path_bit(const uint8_t* pfx, int i) { return (pfx[i >> 3] >> (7 - (i & 7))) & 1; }

static void prep_one(const job_t* J, size_t r, node_t** pool_p, u128** w_p, size_t* cap_p) {
    const fld_t* f = &J->f;
    const int B = J->bits, VL = f->vl;
    const uint8_t* nonce = J->nonces + 16 * r;
    const uint8_t* ps = J->pubs + (size_t)J->ps_size * r;
    const uint8_t* key = J->ins + (size_t)J->is_size * r; /* the VIDPF key leads the input share */
    const int nb = (2 * B + 7) / 8;
    const uint8_t* seed_cw = ps + nb;
    const uint8_t* w_cw = seed_cw + 16 * B;
    const uint8_t* proof_cw = w_cw + (size_t)B * VL * f->enc;
    /* XofFixedKeyAes128 keys: TurboSHAKE128(le16(len(dst)) || dst || nonce, D=2, 16) */
    uint8_t rk_ext[176], rk_conv[176];
    {
        ts_t t;
        uint8_t h[2], k[16];
        ts_init(&t);
        put_le16(h, (unsigned)J->l_ext);
        ts_absorb(&t, h, 2);
        ts_absorb(&t, J->dst_ext, J->l_ext);
        ts_absorb(&t, nonce, 16);
        ts_final(&t, 2, k, 16);
        aes_expand(k, rk_ext);
        ts_init(&t);
        put_le16(h, (unsigned)J->l_conv);
        ts_absorb(&t, h, 2);
        ts_absorb(&t, J->dst_conv, J->l_conv);
        ts_absorb(&t, nonce, 16);
        ts_final(&t, 2, k, 16);
        aes_expand(k, rk_conv);
    }
    /* node pool: root = 0 */
    size_t n_nodes = 1;
    node_t* pool = *pool_p;
    u128* W = *w_p;
    memcpy(pool[0].seed, key, 16);
    pool[0].ctrl = (uint8_t)J->agg_id;
    pool[0].left = pool[0].right = -1;
    const int nwords = (B > 0 ? (B + 7) / 8 : 1);
    uint8_t pathbuf[64];
    int blk_cap = 2 + VL + 8;
    uint8_t* blocks = (uint8_t*)malloc(16 * (size_t)blk_cap);
    /* eval_with_siblings: each prefix walks down from the root */
    for (int pi = 0; pi < J->n_prefixes; pi++) {
        const uint8_t* pfx = J->prefixes + (size_t)J->pbytes * pi;
        int32_t cur = 0;
        for (int i = 0; i <= J->level; i++) {
            node_t* n = &pool[cur];
            if (n->left < 0) {
                if (n_nodes + 2 > *cap_p) {
                    *cap_p *= 2;
                    pool = *pool_p = (node_t*)realloc(pool, *cap_p * sizeof(node_t));
                    W = *w_p = (u128*)realloc(W, *cap_p * (size_t)VL * sizeof(u128));
                    n = &pool[cur];
                }
                /* extend once (both children read it), vidpf.py:330-350 */
                uint8_t s[32];
                fk_blocks(rk_ext, n->seed, 0, 2, s);
                uint8_t t[2] = {(uint8_t)(s[0] & 1), (uint8_t)(s[16] & 1)};
                s[0] &= 0xFE;
                s[16] &= 0xFE;
                const uint8_t* cwd = seed_cw + 16 * i;
                const uint8_t cc[2] = {(uint8_t)((ps[(2 * i) >> 3] >> ((2 * i) & 7)) & 1),
                                       (uint8_t)((ps[(2 * i + 1) >> 3] >> ((2 * i + 1) & 7)) & 1)};
                for (int keep = 0; keep < 2; keep++) {
                    uint8_t* sk = s + 16 * keep;
                    uint8_t tk = t[keep];
                    if (n->ctrl) {
                        for (int b = 0; b < 16; b++) sk[b] ^= cwd[b];
                        tk ^= cc[keep];
                    }
                    /* convert, vidpf.py:352-364: next(16) then next_vec(VL) with rejection */
                    const int32_t ci = (int32_t)n_nodes++;
                    node_t* c = &pool[ci];
                    u128* w = W + (size_t)ci * VL;
                    const int epb = 16 / f->enc;
                    int nblk = 1 + (VL + epb - 1) / epb;
                    fk_blocks(rk_conv, sk, 0, nblk, blocks);
                    memcpy(c->seed, blocks, 16);
                    int got = 0, bi = 1, off = 0;
                    while (got < VL) {
                        if (bi == nblk) { /* a rejection: one more block */
                            if (nblk == blk_cap) {
                                blk_cap *= 2;
                                blocks = (uint8_t*)realloc(blocks, 16 * (size_t)blk_cap);
                            }
                            fk_blocks(rk_conv, sk, (uint64_t)nblk, 1, blocks + 16 * nblk);
                            nblk++;
                        }
                        const u128 x = f_get(f, blocks + 16 * bi + off);
                        off += f->enc;
                        if (off == 16) {
                            off = 0;
                            bi++;
                        }
                        if (f->fbits == 64 ? x < P64 : x < P128) w[got++] = x;
                    }
                    c->ctrl = tk;
                    if (tk)
                        for (int e = 0; e < VL; e++) w[e] = f_add(f, w[e], f_get(f, w_cw + ((size_t)i * VL + e) * f->enc));
                    /* node proof, vidpf.py:366-380 */
                    {
                        ts_t ts;
                        xts_begin(&ts, J->dst_node, J->l_node, c->seed, 16);
                        uint8_t h[4];
                        put_le16(h, (unsigned)B);
                        put_le16(h + 2, (unsigned)i);
                        ts_absorb(&ts, h, 4);
                        const int plen = (i + 1 + 7) / 8;
                        memset(pathbuf, 0, (size_t)plen);
                        for (int b = 0; b < i; b++)
                            if (path_bit(pfx, b)) pathbuf[b >> 3] |= (uint8_t)(0x80 >> (b & 7));
                        if (keep) pathbuf[i >> 3] |= (uint8_t)(0x80 >> (i & 7));
                        ts_absorb(&ts, pathbuf, (size_t)plen);
                        ts_final(&ts, 1, c->proof, 32);
                        if (tk)
                            for (int b = 0; b < 32; b++) c->proof[b] ^= proof_cw[32 * i + b];
                    }
                    c->left = c->right = -1;
                    if (keep == 0) n->left = ci;
                    else n->right = ci;
                }
            }
            cur = path_bit(pfx, i) ? pool[cur].right : pool[cur].left;
        }
        /* the level-L node's payload: truncated out share (mastic.py:308-316) */
        const u128* w = W + (size_t)cur * VL;
        uint8_t* o = J->out_shares + (size_t)J->out_row * r + (size_t)pi * (1 + (J->tlimit + J->tgroup - 1) / J->tgroup) * f->enc;
        f_put(f, o, J->agg_id ? f_neg(f, w[0]) : w[0]);
        int k = 1;
        for (int m = 0; m < J->tlimit; m += J->tgroup, k++) {
            /* decode_from_bit_vector: sum_g 2^g x_g, by Horner from the top bit */
            u128 acc = 0;
            for (int g = J->tgroup - 1; g >= 0; g--) acc = f_add(f, f_add(f, acc, acc), w[1 + m + g]);
            f_put(f, o + (size_t)k * f->enc, J->agg_id ? f_neg(f, acc) : acc);
        }
    }
    (void)nwords;
    free(blocks);
    /* BFS over the evaluated nodes (root's children first): binders (mastic.py:259-287) */
    int32_t* q = (int32_t*)malloc(n_nodes * sizeof(int32_t));
    size_t qh = 0, qt = 0;
    const node_t* root = &pool[0];
    if (root->left >= 0) q[qt++] = root->left;
    if (root->right >= 0) q[qt++] = root->right;
    ts_t oh, pl;
    xts_begin(&oh, J->dst_onehot, J->l_onehot, NULL, 0);
    xts_begin(&pl, J->dst_payload, J->l_payload, NULL, 0);
    uint8_t* enc = (uint8_t*)alloca((size_t)VL * f->enc);
    while (qh < qt) {
        const node_t* n = &pool[q[qh++]];
        if (n->left >= 0 && n->right >= 0) {
            const u128* w = W + (size_t)(n - pool) * VL;
            const u128* wl = W + (size_t)n->left * VL;
            const u128* wr = W + (size_t)n->right * VL;
            for (int e = 0; e < VL; e++) f_put(f, enc + (size_t)e * f->enc, f_sub(f, w[e], f_add(f, wl[e], wr[e])));
            ts_absorb(&pl, enc, (size_t)VL * f->enc);
        }
        ts_absorb(&oh, n->proof, 32);
        if (n->left >= 0) q[qt++] = n->left;
        if (n->right >= 0) q[qt++] = n->right;
    }
    free(q);
    uint8_t checks[32 + 16 + 32];
    ts_final(&oh, 1, checks, 32);
    const u128* w0 = W + (size_t)root->left * VL;
    const u128* w1 = W + (size_t)root->right * VL;
    f_put(f, checks + 32, f_add(f, f_add(f, w0[0], w1[0]), (u128)J->agg_id));
    ts_final(&pl, 1, checks + 32 + f->enc, 32);
    ts_t ev;
    xts_begin(&ev, J->dst_eval, J->l_eval, J->vk, J->vk_len);
    ts_absorb(&ev, checks, (size_t)(64 + f->enc));
    ts_final(&ev, 1, J->eval_proofs + 32 * r, 32);
    /* beta share (vidpf.py:263-279): the root's children's payloads */
    uint8_t* bs = J->beta_shares + (size_t)VL * f->enc * r;
    for (int e = 0; e < VL; e++) {
        const u128 s = f_add(f, w0[e], w1[e]);
        f_put(f, bs + (size_t)e * f->enc, J->agg_id ? f_neg(f, s) : s);
    }
}

static void* worker(void* arg) {
    part_t* P = (part_t*)arg;
    size_t cap = 1024;
    node_t* pool = (node_t*)malloc(cap * sizeof(node_t));
    u128* W = (u128*)malloc(cap * (size_t)P->J->f.vl * sizeof(u128));
    for (size_t r = P->lo; r < P->hi; r++) prep_one(P->J, r, &pool, &W, &cap);
    free(pool);
    free(W);
    P->rc = 0;
    return NULL;
}

/* prep_init's VIDPF part for n reports on `threads` threads.  dsts: the six
 * dst strings (extend, convert, node proof, one-hot check, payload check,
 * eval proof) and their lengths.  Outputs: eval proofs n x 32, beta shares
 * n x VL x enc, truncated out shares n x n_prefixes x (1 + ceil(tlimit /
 * tgroup)) x enc.  Returns 0, or -1 on a bad argument. */
int native_prep_vidpf(int fbits, int bits, int value_len, int agg_id, int level, int n_prefixes,
                      const uint8_t* prefixes, int tgroup, int tlimit, const uint8_t* const* dsts,
                      const size_t* dst_lens, const uint8_t* vk, size_t vk_len, size_t n, const uint8_t* nonces,
                      const uint8_t* pubs, int ps_size, const uint8_t* ins, int is_size, int threads,
                      uint8_t* eval_proofs, uint8_t* beta_shares, uint8_t* out_shares) {
    if ((fbits != 64 && fbits != 128) || level < 0 || level >= bits || n_prefixes < 1 || tgroup < 1 || threads < 1)
        return -1;
#if defined(__x86_64__)
    use_aesni = __builtin_cpu_supports("aes");
#endif
    pthread_once(&sb_once, sb_init);
    job_t J;
    memset(&J, 0, sizeof J);
    J.f.fbits = fbits;
    J.f.enc = fbits / 8;
    J.f.vl = value_len;
    J.bits = bits;
    J.agg_id = agg_id;
    J.level = level;
    J.n_prefixes = n_prefixes;
    J.prefixes = prefixes;
    J.pbytes = (level + 1 + 7) / 8;
    J.tgroup = tgroup;
    J.tlimit = tlimit;
    J.dst_ext = dsts[0];
    J.l_ext = dst_lens[0];
    J.dst_conv = dsts[1];
    J.l_conv = dst_lens[1];
    J.dst_node = dsts[2];
    J.l_node = dst_lens[2];
    J.dst_onehot = dsts[3];
    J.l_onehot = dst_lens[3];
    J.dst_payload = dsts[4];
    J.l_payload = dst_lens[4];
    J.dst_eval = dsts[5];
    J.l_eval = dst_lens[5];
    J.vk = vk;
    J.vk_len = vk_len;
    J.ps_size = ps_size;
    J.is_size = is_size;
    J.nonces = nonces;
    J.pubs = pubs;
    J.ins = ins;
    J.eval_proofs = eval_proofs;
    J.beta_shares = beta_shares;
    J.out_shares = out_shares;
    J.out_row = n_prefixes * (1 + (tlimit + tgroup - 1) / tgroup) * J.f.enc;
    if ((size_t)threads > n) threads = n ? (int)n : 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    part_t* parts = (part_t*)malloc(sizeof(part_t) * (size_t)threads);
    for (int i = 0; i < threads; i++) {
        parts[i].J = &J;
        parts[i].lo = n * (size_t)i / (size_t)threads;
        parts[i].hi = n * (size_t)(i + 1) / (size_t)threads;
        parts[i].rc = -1;
        pthread_create(&th[i], NULL, worker, &parts[i]);
    }
    int rc = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        rc |= parts[i].rc;
    }
    free(th);
    free(parts);
    return rc;
}

int native_has_aesni(void) {
#if defined(__x86_64__)
    return __builtin_cpu_supports("aes");
#else
    return 0;
#endif
}
