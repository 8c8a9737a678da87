/*
 * TEST INFRASTRUCTURE — fixture generator only (tests/rejection/make_fixture.py
 * runs it once; its output is committed as tests/golden/rejection_*.json).
 * Never built into or called by the product path.
 *
 * Brute-forces a 16-byte VIDPF key k (the client's key0, Vidpf.gen
 * poc/vidpf.py:103-211) whose level-0 children, after Vidpf.extend
 * (vidpf.py:330-350), have a Vidpf.convert stream (vidpf.py:352-364: next(16)
 * then next_vec(field, VALUE_LEN)) holding a candidate whose top 32-bit word is
 * 0xffffffff among the VALUE_LEN elements next_vec reads.  For Field64 that is
 * a candidate >= p = 2^64 - 2^32 + 1 (rejected) unless its low word is 0; for
 * Field128 it is the trigger of the GPU fast path's handover to the exact
 * stream (a real Field128 rejection, probability ~2^-59 per candidate, is out
 * of reach).  The AES keys are fixed by (ctx, nonce), so they are derived once
 * by the oracle and passed in as expanded round keys.
 *
 * XofFixedKeyAes128 block i (vdaf-13): x = seed ^ le128(i),
 * sigma(x) = x[8:16] || (x[8:16] ^ x[0:8]), out = AES_k(sigma(x)) ^ sigma(x).
 * AES-128 via AES-NI (same FIPS-197 block order as oracle/prims.c).
 *
 *   find_rejection <rk_ext hex 352> <rk_conv hex 352> <64|128> <value_len> <salt hex 16> <threads>
 * prints: <counter> <child 0|1> <candidate index> <rejected 0|1>
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <wmmintrin.h>

static __m128i RK_EXT[11], RK_CONV[11];
static int FIELD, VL, THREADS;
static uint8_t SALT[8];
static volatile int found = 0;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static uint64_t best_ctr = UINT64_MAX;
static int best_child, best_cand, best_rej;

static void hex_in(const char* h, uint8_t* out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        unsigned v;
        sscanf(h + 2 * i, "%2x", &v);
        out[i] = (uint8_t)v;
    }
}

static inline __m128i aes(const __m128i* rk, __m128i x) {
    x = _mm_xor_si128(x, rk[0]);
    for (int r = 1; r < 10; r++) x = _mm_aesenc_si128(x, rk[r]);
    return _mm_aesenclast_si128(x, rk[10]);
}

static inline void fixed_key_block(const __m128i* rk, const uint8_t seed[16], uint64_t ctr, uint8_t out[16]) {
    uint8_t x[16], sig[16];
    memcpy(x, seed, 16);
    for (int i = 0; i < 8; i++) x[i] ^= (uint8_t)(ctr >> (8 * i));
    for (int i = 0; i < 8; i++) {
        sig[i] = x[8 + i];
        sig[8 + i] = x[8 + i] ^ x[i];
    }
    __m128i s = _mm_loadu_si128((const __m128i*)sig);
    _mm_storeu_si128((__m128i*)out, _mm_xor_si128(aes(rk, s), s));
}

static void* worker(void* arg) {
    const uint64_t tid = (uint64_t)(uintptr_t)arg;
    const int enc = FIELD / 8;
    const int nblk = (VL * enc + 15) / 16;
    uint8_t key[16], child[16], blk[16];
    memcpy(key + 8, SALT, 8);
    for (uint64_t ctr = tid; !found; ctr += (uint64_t)THREADS) {
        for (int i = 0; i < 8; i++) key[i] = (uint8_t)(ctr >> (8 * i));
        for (int c = 0; c < 2; c++) {
            fixed_key_block(RK_EXT, key, (uint64_t)c, child);
            child[0] &= 0xFE;  // the control bit is taken out of byte 0
            for (int b = 1; b <= nblk; b++) {
                fixed_key_block(RK_CONV, child, (uint64_t)b, blk);
                // candidates in this block: bytes [16(b-1), 16b) of the payload stream
                for (int off = 0; off < 16; off += enc) {
                    const int j = (16 * (b - 1) + off) / enc;
                    if (j >= VL) break;
                    uint32_t top;
                    memcpy(&top, blk + off + enc - 4, 4);
                    if (top != 0xffffffffu) continue;
                    uint32_t lo;
                    memcpy(&lo, blk + off, 4);
                    int rej = FIELD == 64 ? lo != 0 : 0;
                    pthread_mutex_lock(&mu);
                    if (ctr < best_ctr) {
                        best_ctr = ctr;
                        best_child = c;
                        best_cand = j;
                        best_rej = rej;
                    }
                    found = 1;
                    pthread_mutex_unlock(&mu);
                }
            }
        }
    }
    return NULL;
}

int main(int argc, char** argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: find_rejection rk_ext rk_conv field value_len salt threads\n");
        return 2;
    }
    uint8_t rk[176];
    hex_in(argv[1], rk, 176);
    for (int i = 0; i < 11; i++) RK_EXT[i] = _mm_loadu_si128((const __m128i*)(rk + 16 * i));
    hex_in(argv[2], rk, 176);
    for (int i = 0; i < 11; i++) RK_CONV[i] = _mm_loadu_si128((const __m128i*)(rk + 16 * i));
    FIELD = atoi(argv[3]);
    VL = atoi(argv[4]);
    hex_in(argv[5], SALT, 8);
    THREADS = atoi(argv[6]);
    pthread_t th[256];
    for (int t = 0; t < THREADS; t++) pthread_create(&th[t], NULL, worker, (void*)(uintptr_t)t);
    for (int t = 0; t < THREADS; t++) pthread_join(th[t], NULL);
    printf("%llu %d %d %d\n", (unsigned long long)best_ctr, best_child, best_cand, best_rej);
    return 0;
}
