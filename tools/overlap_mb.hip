// Microbenchmark: how well the level kernel's two pipes overlap on one CU.
// A "unit" is the C2 level kernel's work per report-node in miniature: 5 AES
// block pairs (T-table lookups in LDS, AesPerm exactly as k_eval_aes) and one
// Keccak-p[1600,12] (VALU only, the node proof).  One workgroup of 16 waves
// per CU (the table + key schedule LDS footprint of k_eval_aes), 64 lanes =
// 64 independent reports.  Modes:
//   aes      every wave does only the AES of its units
//   keccak   every wave does only the Keccak of its units
//   split:A  A waves do the AES of all units, 16 - A waves the Keccak
//   seq      every wave: 5 pairs, then one Keccak-p
//   fill     every wave: 5 pairs whose middle rounds carry one Keccak round
//            between issuing a round's 32 lookups and waiting for them
//   fill2    as fill, the Keccak round between the two blocks' 16 lookups
// t(aes) + t(keccak) = no overlap; max(t(aes), t(keccak)) = perfect overlap.
// Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -o overlap_mb overlap_mb.hip
#include "../draft-mouris-cfrg-mastic_amd/csrc/aes.hpp"
#include "../draft-mouris-cfrg-mastic_amd/csrc/keccak.hpp"
#include <stdio.h>
#include <stdlib.h>

#define WAVES 16
#define LDS_BYTES (AES_PERM_LDS_WORDS * 4 + 64 * 11 * 16)

__constant__ uint32_t RC_LO[12] = {0x8000808bu, 0x0000008bu, 0x00008089u, 0x00008003u, 0x00008002u, 0x00000080u,
                                   0x0000800au, 0x8000000au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__constant__ uint32_t RC_HI[12] = {0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u,
                                   0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

// one Keccak round with a run-time (uniform) round index
MH_D void keccak_round(KState& s, int round) {
    u32x2* A = s.a;
    u32x2 C[5], D[5];
#pragma unroll
    for (int x = 0; x < 5; x++) C[x] = xor3_64(xor3_64(A[x], A[x + 5], A[x + 10]), A[x + 15], A[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; x++) D[x] = xor64(C[(x + 4) % 5], rotl64(C[(x + 1) % 5], 1));
    u32x2 B[25];
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
        for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(xor64(A[x + 5 * y], D[x]), KR(x, y));
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
        for (int x = 0; x < 5; x++) A[x + 5 * y] = chi1(B[x + 5 * y], B[(x + 1) % 5 + 5 * y], B[(x + 2) % 5 + 5 * y]);
    A[0].lo ^= RC_LO[round];
    A[0].hi ^= RC_HI[round];
}

// the Keccak state is "produced" after the lookups were issued (so its round
// cannot be hoisted above them) and "consumed" before the wait (so it cannot
// sink below it); volatile asm statements keep their order
MH_D void ks_def(KState& s) {
#pragma unroll
    for (int i = 0; i < 25; i += 5)
        asm volatile("" : "+v"(s.a[i].lo), "+v"(s.a[i].hi), "+v"(s.a[i + 1].lo), "+v"(s.a[i + 1].hi),
                     "+v"(s.a[i + 2].lo), "+v"(s.a[i + 2].hi), "+v"(s.a[i + 3].lo), "+v"(s.a[i + 3].hi),
                     "+v"(s.a[i + 4].lo), "+v"(s.a[i + 4].hi));
}
MH_D void ks_use(const KState& s) {
#pragma unroll
    for (int i = 0; i < 25; i += 5)
        asm volatile("" ::"v"(s.a[i].lo), "v"(s.a[i].hi), "v"(s.a[i + 1].lo), "v"(s.a[i + 1].hi), "v"(s.a[i + 2].lo),
                     "v"(s.a[i + 2].hi), "v"(s.a[i + 3].lo), "v"(s.a[i + 3].hi), "v"(s.a[i + 4].lo),
                     "v"(s.a[i + 4].hi));
}

// a middle round of two blocks with an optional Keccak round as filler
// FILL 1: after all 32 lookups; FILL 2: after block 0's 16 lookups
template <int FILL>
MH_D void round2_fill(const AesPerm& T, uint32_t (&s)[2][4], uint4 k, KState& ks, int& kr, bool fill) {
    uint32_t L[32];
#pragma unroll
    for (int j = 0; j < 2; j++) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            L[16 * j + 4 * c + 0] = lds_read_asm(T.a0<0>(s[j][c]));
            L[16 * j + 4 * c + 1] = lds_read_asm(T.a1<1>(s[j][(c + 1) & 3]));
            L[16 * j + 4 * c + 2] = lds_read_asm(T.a2<2>(s[j][(c + 2) & 3]));
            L[16 * j + 4 * c + 3] = lds_read_asm(T.a3<3>(s[j][(c + 3) & 3]));
        }
        if ((FILL == 2 && j == 0) || (FILL == 1 && j == 1)) {
            if (fill) {
                ks_def(ks);
                keccak_round(ks, kr);
                ks_use(ks);
                kr++;
            }
        }
    }
    aes_pin<2>(L);
    const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t* q = L + 16 * j + 4 * c;
            s[j][c] = xor3_u32(xor3_u32(q[0], q[1], q[2]), q[3], kk[c]);
        }
}

template <int FILL>
MH_D void pair_fill(const AesPerm& T, const RkLds& rk, uint32_t (&x)[2][4], KState& ks, int& kr, int pair) {
    uint4 k = rk(0);
#pragma unroll
    for (int j = 0; j < 2; j++) {
        x[j][0] ^= k.x; x[j][1] ^= k.y; x[j][2] ^= k.z; x[j][3] ^= k.w;
    }
    // 45 middle rounds per unit carry the 12 Keccak rounds: rounds 1..9 of
    // pair p fill when (9p + r - 1) * 12 / 45 steps
#pragma unroll
    for (int r = 1; r < 10; r++) {
        const int ph = 9 * pair + r - 1;
        const bool fill = (ph * 12) / 45 != ((ph + 1) * 12) / 45;
        round2_fill<FILL>(T, x, rk(r), ks, kr, fill);
    }
    aes_last_n<2>(T, x, rk(10));
}

template <int MODE, int FILL>
__global__ __launch_bounds__(64 * WAVES) void k_ov(uint32_t* out, int units, int aes_waves) {
    extern __shared__ uint4 lds[];
    uint32_t* T = (uint32_t*)lds;
    uint4* RK = lds + AES_PERM_LDS_WORDS / 4;
    if ((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint4*)lds != 0u) __builtin_trap();
    aes_perm_fill(T, threadIdx.x, 64 * WAVES);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < 64 * 44; i += 64 * WAVES) {
        const uint32_t v = 0x9e3779b9u * (uint32_t)(i + 1) ^ (blockIdx.x << 7);
        ((uint32_t*)RK)[i] = aes_perm_key_word(i % 44, v);
    }
    __syncthreads();
    const AesPerm TL{T, 4u * (uint32_t)(lane & 31), 128u + 4u * (uint32_t)(lane & 31)};
    const RkLds rk{RK + lane * 11};
    uint32_t x[2][4];
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[j][c] = threadIdx.x * 7919u + blockIdx.x * 131u + j * 17u + c;
    KState ks;
#pragma unroll
    for (int i = 0; i < 25; i++) ks.a[i] = u32x2{threadIdx.x + i, blockIdx.x ^ (uint32_t)i};
    // units of this wave (MODE 2 gives each side all the workgroup's units)
    int n_aes = 0, n_kec = 0;
    if (MODE == 0) n_aes = units;
    if (MODE == 1) n_kec = units;
    if (MODE == 2) {
        if (wave < aes_waves) n_aes = units * WAVES / aes_waves;
        else n_kec = units * WAVES / (WAVES - aes_waves);
    }
    if (MODE >= 3) n_aes = n_kec = units;
    if (MODE <= 3) {
        for (int u = 0; u < max(n_aes, n_kec); u++) {
            if (u < n_aes) {
                for (int p = 0; p < 5; p++) {
                    asm volatile("" ::: "memory");
                    aes128_encrypt_n<2>(TL, rk, x);
                }
            }
            if (u < n_kec) {
                asm volatile("" ::: "memory");
                keccak_p12(ks);
            }
        }
    } else {
        for (int u = 0; u < units; u++) {
            int kr = 0;
            for (int p = 0; p < 5; p++) {
                asm volatile("" ::: "memory");
                pair_fill<FILL>(TL, rk, x, ks, kr, p);
            }
        }
    }
    uint32_t acc = x[0][0] ^ x[1][1] ^ x[0][2] ^ x[1][3];
#pragma unroll
    for (int i = 0; i < 25; i++) acc ^= ks.a[i].lo ^ ks.a[i].hi;
    out[blockIdx.x * 64 * WAVES + threadIdx.x] = acc;
}

static double run(int mode, int aes_waves, int fill, uint32_t* out, int grid, int units) {
    auto launch = [&](int u) {
        switch (mode * 10 + fill) {
            case 0: hipLaunchKernelGGL((k_ov<0, 0>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, 0, out, u, aes_waves); break;
            case 10: hipLaunchKernelGGL((k_ov<1, 0>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, 0, out, u, aes_waves); break;
            case 20: hipLaunchKernelGGL((k_ov<2, 0>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, 0, out, u, aes_waves); break;
            case 30: hipLaunchKernelGGL((k_ov<3, 0>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, 0, out, u, aes_waves); break;
            case 41: hipLaunchKernelGGL((k_ov<4, 1>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, 0, out, u, aes_waves); break;
            case 42: hipLaunchKernelGGL((k_ov<4, 2>), dim3(grid), dim3(64 * WAVES), LDS_BYTES, 0, out, u, aes_waves); break;
        }
    };
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch(2);
    hipDeviceSynchronize();
    hipEventRecord(a);
    launch(units);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main(int argc, char** argv) {
    const int units = argc > 1 ? atoi(argv[1]) : 64;
    const int grid = 256 * 2;  // two workgroups per CU in sequence (one resident at a time)
    uint32_t* out;
    hipMalloc(&out, (size_t)grid * 64 * WAVES * 4);
    hipFuncSetAttribute((const void*)k_ov<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute((const void*)k_ov<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute((const void*)k_ov<2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute((const void*)k_ov<3, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute((const void*)k_ov<4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute((const void*)k_ov<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    struct V { const char* name; int mode, aw, fill; };
    const V vs[] = {{"aes", 0, 16, 0},     {"keccak", 1, 0, 0},  {"split:8", 2, 8, 0}, {"split:12", 2, 12, 0},
                    {"split:4", 2, 4, 0},  {"seq", 3, 16, 0},    {"fill", 4, 16, 1},   {"fill2", 4, 16, 2}};
    // units per CU-second: grid * 64 lanes * 16 waves * units
    const double work = (double)grid * 64 * WAVES * units;
    double t_aes = 0, t_kec = 0;
    for (const V& v : vs) {
        const double ms = run(v.mode, v.aw, v.fill, out, grid, units);
        if (v.mode == 0) t_aes = ms;
        if (v.mode == 1) t_kec = ms;
        // LDS-array cycles per unit per 64 lanes: 10 blocks x 160 lookups x 2 / 64
        const double cu_cycles = ms * 1e-3 * 2.4e9 * 256;
        const double lds_busy = v.mode == 1 ? 0.0 : (work / 64) * 10 * 160 * 2 / cu_cycles;
        printf("{\"variant\": \"%s\", \"ms\": %.3f, \"units_per_s\": %.4g, \"lds_busy_at_2.4GHz\": %.3f", v.name, ms,
               work / (ms * 1e-3), lds_busy);
        if (t_aes > 0 && t_kec > 0 && v.mode >= 2)
            printf(", \"vs_serial\": %.3f, \"vs_perfect\": %.3f", ms / (t_aes + t_kec), ms / (t_aes > t_kec ? t_aes : t_kec));
        printf("}\n");
        fflush(stdout);
    }
    hipFree(out);
    return 0;
}
