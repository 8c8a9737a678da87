// Microbenchmark: T-table AES-128 throughput on gfx950 in isolation (no HBM
// traffic), to choose the level kernel's LDS table layout, blocks in lockstep
// and occupancy.  Build: hipcc --offload-arch=gfx950 -O3 -o aes_mb aes_mb.hip
// Not part of the product; prints one line per variant.
#include "../draft-mouris-cfrg-mastic_amd/csrc/aes.hpp"
#include <stdio.h>
#include <vector>

// T0-only table, 32 replicas (32 KiB): address (x << 7) | 4 * (lane & 31)
struct AesT0 {
    const uint32_t* T;
    uint32_t lb;
    template <int K>
    MH_D uint32_t t0(uint32_t x) const {
        const uint32_t b = K == 0 ? (x & 0xffu) : K == 3 ? (x >> 24) : __builtin_amdgcn_ubfe(x, 8 * K, 8);
        return *(const uint32_t*)((const char*)T + ((b << 7) | lb));
    }
};
MH_D uint32_t col_t0(const AesT0& T, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t k) {
    // T0[a] ^ rot8(T0[b]) ^ rot16(T0[c]) ^ rot24(T0[d]) ^ k
    //  = T0[a] ^ k ^ rot8(T0[b] ^ rot8(T0[c] ^ rot8(T0[d])))
    const uint32_t d = rot8(T.t0<3>(w3));
    const uint32_t c = rot8(T.t0<2>(w2) ^ d);
    const uint32_t b = rot8(T.t0<1>(w1) ^ c);
    return xor3_u32(T.t0<0>(w0), b, k);
}
MH_D uint32_t col_t0_last(const AesT0& T, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t k) {
    const uint32_t lo = __builtin_amdgcn_perm(T.t0<1>(w1), T.t0<0>(w0), 0x0c0c0501u);
    const uint32_t hi = __builtin_amdgcn_perm(T.t0<3>(w3), T.t0<2>(w2), 0x05010c0cu);
    return xor3_u32(lo, hi, k);
}

template <int N, class RK>
MH_D void enc_t0(const AesT0& T, const RK& rk, uint32_t (&s)[N][4]) {
    uint4 k = rk(0);
#pragma unroll
    for (int j = 0; j < N; j++) {
        s[j][0] ^= k.x; s[j][1] ^= k.y; s[j][2] ^= k.z; s[j][3] ^= k.w;
    }
#pragma unroll
    for (int r = 1; r < 10; r++) {
        k = rk(r);
        uint32_t t[N][4];
#pragma unroll
        for (int j = 0; j < N; j++) {
            t[j][0] = col_t0(T, s[j][0], s[j][1], s[j][2], s[j][3], k.x);
            t[j][1] = col_t0(T, s[j][1], s[j][2], s[j][3], s[j][0], k.y);
            t[j][2] = col_t0(T, s[j][2], s[j][3], s[j][0], s[j][1], k.z);
            t[j][3] = col_t0(T, s[j][3], s[j][0], s[j][1], s[j][2], k.w);
        }
#pragma unroll
        for (int j = 0; j < N; j++)
#pragma unroll
            for (int c = 0; c < 4; c++) s[j][c] = t[j][c];
    }
    k = rk(10);
#pragma unroll
    for (int j = 0; j < N; j++) {
        uint32_t a0 = s[j][0], a1 = s[j][1], a2 = s[j][2], a3 = s[j][3];
        s[j][0] = col_t0_last(T, a0, a1, a2, a3, k.x);
        s[j][1] = col_t0_last(T, a1, a2, a3, a0, k.y);
        s[j][2] = col_t0_last(T, a2, a3, a0, a1, k.z);
        s[j][3] = col_t0_last(T, a3, a0, a1, a2, k.w);
    }
}

// MODE 0: AesPerm (T0/T2, 64 KiB) ; MODE 1: AesT0 (32 KiB)
template <int MODE, int NB, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_mb(uint32_t* out, int iters) {
    constexpr int TW = MODE == 0 ? AES_PERM_LDS_WORDS : 256 * 32;
    __shared__ uint32_t T[TW];
    __shared__ uint4 RK[64 * 11];
    if (MODE == 0) {
        aes_perm_fill(T, threadIdx.x, 64 * WAVES);
    } else {
        for (int i = threadIdx.x; i < TW; i += 64 * WAVES) T[i] = aes_t0(i >> 5);
    }
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 64 * 44; i += 64 * WAVES) {
        const int ln = i / 44, w = i % 44;
        const uint32_t v = 0x9e3779b9u * (uint32_t)(i + 1) ^ (blockIdx.x << 7);
        ((uint32_t*)RK)[ln * 44 + w] = MODE == 0 ? aes_perm_key_word(w, v) : v;
    }
    __syncthreads();
    const RkLds rk{RK + lane * 11};
    uint32_t s[NB][4];
#pragma unroll
    for (int j = 0; j < NB; j++)
#pragma unroll
        for (int c = 0; c < 4; c++) s[j][c] = threadIdx.x * 7919u + blockIdx.x * 131u + j * 17u + c;
    for (int it = 0; it < iters; it++) {
        asm volatile("" ::: "memory");
        if (MODE == 0) {
            const AesPerm TL{T, 4u * (uint32_t)(lane & 31), 128u + 4u * (uint32_t)(lane & 31)};
            aes128_encrypt_n<NB>(TL, rk, s);
        } else {
            const AesT0 TL{T, 4u * (uint32_t)(lane & 31)};
            enc_t0<NB>(TL, rk, s);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < NB; j++) acc ^= s[j][0] ^ s[j][1] ^ s[j][2] ^ s[j][3];
    out[blockIdx.x * 64 * WAVES + threadIdx.x] = acc;
}

template <int MODE, int NB, int WAVES>
void run(uint32_t* out, int wg_per_cu, const char* name) {
    const int grid = 256 * wg_per_cu * 4;  // 4 rounds of residency
    const int iters = 400 / NB;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_mb<MODE, NB, WAVES>), dim3(grid), dim3(64 * WAVES), 0, 0, out, 8);
    hipDeviceSynchronize();
    hipEventRecord(a);
    hipLaunchKernelGGL((k_mb<MODE, NB, WAVES>), dim3(grid), dim3(64 * WAVES), 0, 0, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double blocks = (double)grid * 64 * WAVES * NB * iters;
    const double bps = blocks / (ms / 1e3);
    // lookups: 160 per block; LDS peak 32 lookups/clk/CU
    const double lk_per_clk_cu = bps * 160 / (256 * 2.1e9);
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"blocks_per_s\": %.4g, \"lookups_per_clk_cu_at_2.1GHz\": %.2f}\n",
           name, ms, bps, lk_per_clk_cu);
    fflush(stdout);
}

int main_ladder();
int main() {
    if (main_ladder()) return 1;
    uint32_t* out;
    hipMalloc(&out, 256 * 16 * 1024 * 4 * sizeof(uint32_t));
    run<0, 1, 16>(out, 1, "perm64K nb1 w16");
    run<0, 2, 16>(out, 1, "perm64K nb2 w16");
    run<0, 4, 16>(out, 1, "perm64K nb4 w16");
    run<0, 8, 16>(out, 1, "perm64K nb8 w16");
    run<0, 2, 8>(out, 1, "perm64K nb2 w8");
    run<0, 4, 8>(out, 1, "perm64K nb4 w8");
    run<1, 2, 16>(out, 1, "t0_32K nb2 w16 (1 wg/cu)");
    run<1, 4, 16>(out, 1, "t0_32K nb4 w16 (1 wg/cu)");
    run<1, 2, 8>(out, 3, "t0_32K nb2 w8 (3 wg/cu)");
    run<1, 4, 8>(out, 3, "t0_32K nb4 w8 (3 wg/cu)");
    run<1, 2, 16>(out, 2, "t0_32K nb2 w16 (2 wg/cu)");
    run<1, 4, 16>(out, 2, "t0_32K nb4 w16 (2 wg/cu)");
    hipFree(out);
    return 0;
}

// ---------------------------------------------------------------------------
// Level-kernel ladder: the real kernel's per-parent structure (extend pair ->
// seed pair -> 9 payload pairs), 16 waves per workgroup, 64 reports per
// workgroup, planes [word][stride] in HBM like the product.
//   FLAGS & 1: store child seeds (10 words) + payload diff (34) + frontier (68)
//   FLAGS & 2: load parent seed (5 words) + parent payload (34)
template <int FLAGS>
__global__ __launch_bounds__(1024) void k_ladder(uint32_t* planes, int stride, int parents_per_wave, uint32_t* out) {
    __shared__ uint32_t T[AES_PERM_LDS_WORDS];
    __shared__ uint4 RKE[64 * 11];
    __shared__ uint4 RKC[64 * 11];
    aes_perm_fill(T, threadIdx.x, 1024);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < 64 * 44; i += 1024) {
        const uint32_t v = 0x9e3779b9u * (uint32_t)(i + 1) ^ (blockIdx.x << 7);
        ((uint32_t*)RKE)[i] = aes_perm_key_word(i % 44, v);
        ((uint32_t*)RKC)[i] = aes_perm_key_word(i % 44, v * 3u);
    }
    __syncthreads();
    const AesPerm TL{T, 4u * (uint32_t)(lane & 31), 128u + 4u * (uint32_t)(lane & 31)};
    const RkLds rke{RKE + lane * 11};
    const RkLds rkc{RKC + lane * 11};
    const int r = blockIdx.x * 64 + lane;
    const uint32_t lb = (uint32_t)r * 4u;
    const int S = stride;
    uint32_t acc = 0;
    const int p0 = (blockIdx.y * 16 + wave) * parents_per_wave;
    for (int pi = p0; pi < p0 + parents_per_wave; pi++) {
        asm volatile("" ::: "memory");
        uint32_t ps[4];
        if (FLAGS & 2) {
#pragma unroll
            for (int i = 0; i < 4; i++) ps[i] = pld(planes + ((size_t)pi * 5 + i) * S, lb);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) ps[i] = pi * 4 + i + lane;
        }
        uint32_t cs0[4], cs1[4], ns0[4], ns1[4];
        fixed_key_block2(TL, rke, ps, 0u, ps, 1u, cs0, cs1);
        cs0[0] &= ~1u;
        cs1[0] &= ~1u;
        fixed_key_block2(TL, rkc, cs0, 0u, cs1, 0u, ns0, ns1);
        if (FLAGS & 1) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                pst(planes + ((size_t)(2 * pi) * 5 + i) * S, lb, ns0[i]);
                pst(planes + ((size_t)(2 * pi + 1) * 5 + i) * S, lb, ns1[i]);
            }
        } else {
            acc ^= ns0[0] ^ ns1[1];
        }
        for (int b = 0; b < 9; b++) {
            asm volatile("" ::: "memory");
            uint32_t wp[4];
            if (FLAGS & 2) {
#pragma unroll
                for (int i = 0; i < 4; i++) wp[i] = pld(planes + ((size_t)pi * 36 + 4 * b + i) * S, lb);
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++) wp[i] = b + i;
            }
            uint32_t o0[4], o1[4];
            fixed_key_block2(TL, rkc, cs0, (uint32_t)(b + 1), cs1, (uint32_t)(b + 1), o0, o1);
            if (FLAGS & 1) {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    pst(planes + ((size_t)(2 * pi) * 36 + 4 * b + i) * S, lb, o0[i]);
                    pst(planes + ((size_t)(2 * pi + 1) * 36 + 4 * b + i) * S, lb, o1[i]);
                    pst(planes + ((size_t)pi * 36 + 4 * b + i + 7) * S, lb, wp[i] - o0[i] - o1[i]);
                }
            } else {
                acc ^= o0[0] ^ o1[1] ^ o0[2] ^ o1[3] ^ wp[0];
            }
        }
    }
    out[blockIdx.y * gridDim.x * 1024 + blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <int FLAGS>
void run_ladder(uint32_t* planes, int stride, uint32_t* out, const char* name) {
    const int groups = stride / 64, ppw = 32, ychunks = 10;  // 10 * 16 * 32 = 5120 parents
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_ladder<FLAGS>), dim3(groups, 1), dim3(1024), 0, 0, planes, stride, 1, out);
    hipDeviceSynchronize();
    hipEventRecord(a);
    hipLaunchKernelGGL((k_ladder<FLAGS>), dim3(groups, ychunks), dim3(1024), 0, 0, planes, stride, ppw, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double blocks = (double)stride * ychunks * 16 * ppw * 22;
    printf("{\"variant\": \"ladder %s\", \"ms\": %.3f, \"blocks_per_s\": %.4g}\n", name, ms, blocks / (ms / 1e3));
    fflush(stdout);
}

int main_ladder() {
    const int stride = 4096;
    uint32_t *planes, *out;
    const size_t words = (size_t)5120 * 2 * 36 + 64;
    if (hipMalloc(&planes, words * stride * 4) != hipSuccess) return 1;
    hipMemset(planes, 0, words * stride * 4);
    hipMalloc(&out, (size_t)10 * (stride / 64) * 1024 * 4);
    run_ladder<0>(planes, stride, out, "compute only");
    run_ladder<1>(planes, stride, out, "+stores");
    run_ladder<2>(planes, stride, out, "+loads");
    run_ladder<3>(planes, stride, out, "+loads+stores");
    hipFree(planes);
    hipFree(out);
    return 0;
}
