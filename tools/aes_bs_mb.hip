// Microbenchmark: 32-way bitsliced AES-128 over the
// XofFixedKeyAes128 counter stream (tools/aes_bs.hpp) against the LDS T-table
// AES of the level kernel (tools/aes_mb.hip, profiles/r02_v16_aes_mb.txt), in
// isolation: no HBM traffic, every lane one report with its own key schedule
// (in LDS, as the level kernel keeps it), 32 consecutive counters per batch.
// Variants:
//   bs            per-lane keys: round-key masks by v_bfe_i32 from the LDS words
//   bs_ukey       a wave-uniform key (what one-report-per-wave would allow):
//                 masks from SGPRs, no per-lane extraction
//   bs_notr       per-lane keys, output left sliced (no transpose back):
//                 the transposes' share
//   tt_ctr        the T-table with counter groups (aes.hpp ctr_blocks_n, N = 2),
//                 the level kernel's payload loop, same per-lane keys
//   tt_ctr_ukey   the same T-table loop with ONE wave-uniform key schedule
//                 (round 6): the 44 key words read once into
//                 SGPRs (readfirstlane), so a round's key costs no LDS read --
//                 what one report's convert stream spread over a wave's lanes
//                 (consecutive counter blocks per lane) would allow
// Blocks per second over the chip and per CU-clock.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/aes_bs_mb tools/aes_bs_mb.hip
// Not part of the product.
#include "../draft-mouris-cfrg-mastic_amd/csrc/aes.hpp"
// three-input XOR as one full-rate v_bitop3_b32 (declared before aes_bs.hpp's
// generic template, so overload resolution prefers it on the device)
MH_D uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
#include "aes_bs.hpp"
#include <stdio.h>
#include <stdlib.h>

struct BmBfe {  // broadcast mask of a lane's data bit
    MH_D uint32_t operator()(uint32_t v, int bit) const { return (uint32_t)__builtin_amdgcn_sbfe((int)v, bit, 1); }
};
struct KmLds {  // per-lane round keys (uint4 per round in LDS), 0x63 folded in for rounds >= 1
    const uint4* row;
    MH_D uint32_t operator()(int r, int w, int bit) const {
        const uint4 k = row[r];
        uint32_t kw = w == 0 ? k.x : w == 1 ? k.y : w == 2 ? k.z : k.w;
        if (r >= 1) kw ^= 0x63636363u;
        return (uint32_t)__builtin_amdgcn_sbfe((int)kw, bit, 1);
    }
};
struct KmUniform {  // wave-uniform key words (SGPRs)
    const uint32_t* k;  // 44 words, kernel argument memory
    MH_D uint32_t operator()(int r, int w, int bit) const {
        uint32_t kw = __builtin_amdgcn_readfirstlane(k[4 * r + w]);
        if (r >= 1) kw ^= 0x63636363u;
        return (uint32_t)(-(int)((kw >> bit) & 1u));  // scalar ops on a uniform value
    }
};

// MODE 0 bs, 1 bs_ukey, 2 bs_notr, 3 tt_ctr, 4 tt_ctr_ukey
template <int MODE, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_mb(uint32_t* out, const uint32_t* ukey, int iters) {
    constexpr bool TT = MODE == 3 || MODE == 4;
    extern __shared__ uint32_t lds[];
    uint32_t* T = lds;  // T-table (AesPerm layout, must sit at LDS address 0) for MODE 3
    uint4* RK = (uint4*)(lds + (TT ? AES_PERM_LDS_WORDS : 0));
    if (TT) aes_perm_fill(T, threadIdx.x, 64 * WAVES);
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 64 * 44; i += 64 * WAVES) {
        const uint32_t v = 0x9e3779b9u * (uint32_t)(i + 1) ^ (blockIdx.x << 7);
        ((uint32_t*)RK)[i] = v;
    }
    __syncthreads();
    const uint4* row = RK + lane * 11;
    uint32_t seed[4] = {threadIdx.x * 7919u + blockIdx.x * 131u, 0x1234567u ^ threadIdx.x, 0x89abcdefu + blockIdx.x,
                        0x0f1e2d3cu};
    uint32_t acc = 0;
    uint32_t base = 0;
    for (int it = 0; it < iters; it++, base += 32) {
        asm volatile("" ::: "memory");
        if constexpr (TT) {
            const AesPerm TL{T, 4u * (uint32_t)(lane & 31), 128u + 4u * (uint32_t)(lane & 31)};
            uint32_t kw[44];
            if constexpr (MODE == 4) {
#pragma unroll
                for (int i = 0; i < 44; i++) kw[i] = __builtin_amdgcn_readfirstlane(ukey[i]);
            }
            const RkLds rkl{row};
            const RkRegs rkr{kw};
            const auto& rk = [&]() -> const auto& {
                if constexpr (MODE == 4) return rkr; else return rkl;
            }();
            // 32 blocks of one seed as the payload loop does them: one counter
            // group per 256 counters, pairs in lockstep
            AesCtrGroup g;
            const uint32_t* sp[1] = {seed};
            const uint32_t chi[1] = {base};
            AesCtrGroup* gp[1] = {&g};
            ctr_group_init<1>(TL, rk, sp, chi, gp);
#pragma unroll 1
            for (int j = 0; j < 32; j += 2) {
                uint32_t o0[4], o1[4];
                const AesCtrGroup* gg[2] = {&g, &g};
                const uint32_t* ss[2] = {seed, seed};
                const uint32_t cc[2] = {base + j, base + j + 1};
                uint32_t* oo[2] = {o0, o1};
                ctr_blocks_n<2>(TL, rk, gg, ss, cc, oo);
                acc ^= o0[0] ^ o0[1] ^ o0[2] ^ o0[3] ^ o1[0] ^ o1[1] ^ o1[2] ^ o1[3];
            }
        } else {
            const uint4 k0 = row[0];
            const uint32_t rk0[4] = {k0.x, k0.y, k0.z, k0.w};
            uint32_t o[32][4];
            if constexpr (MODE == 1) {
                bs_ctr32<uint32_t>(seed, base, rk0, BmBfe{}, KmUniform{ukey}, o);
            } else if constexpr (MODE == 2) {
                // as bs_ctr32 without the transposes: rounds only, sliced output folded
                const uint32_t sg[4] = {seed[2], seed[3], seed[2] ^ seed[0] ^ base, seed[3] ^ seed[1]};
                uint32_t s[16][8];
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    const uint32_t v = sg[i >> 2] ^ rk0[i >> 2];
#pragma unroll
                    for (int b = 0; b < 8; b++) s[i][b] = BmBfe{}(v, 8 * (i & 3) + b);
                }
#pragma unroll
                for (int b = 0; b < 5; b++) s[8][b] ^= BS_PAT[b];
#pragma unroll
                for (int r = 1; r < 10; r++) bs_round(s, KmLds{row}, r);
                bs_last(s, KmLds{row});
#pragma unroll
                for (int i = 0; i < 16; i++)
#pragma unroll
                    for (int b = 0; b < 8; b++) o[(8 * i + b) >> 2][b & 3] = s[i][b];
            } else {
                bs_ctr32<uint32_t>(seed, base, rk0, BmBfe{}, KmLds{row}, o);
            }
#pragma unroll
            for (int j = 0; j < 32; j++) acc ^= o[j][0] ^ o[j][1] ^ o[j][2] ^ o[j][3];
        }
    }
    out[blockIdx.x * 64 * WAVES + threadIdx.x] = acc;
}

template <int MODE, int WAVES>
void run(uint32_t* out, const uint32_t* ukey, int grid, const char* name) {
    const size_t lds = (MODE == 3 || MODE == 4 ? AES_PERM_LDS_WORDS * 4 : 0) + 64 * 11 * 16;
    hipFuncSetAttribute((const void*)k_mb<MODE, WAVES>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncAttributes fa;
    hipFuncGetAttributes(&fa, (const void*)k_mb<MODE, WAVES>);
    const int iters = 64;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_mb<MODE, WAVES>), dim3(grid), dim3(64 * WAVES), lds, 0, out, ukey, 4);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("{\"variant\": \"%s\", \"error\": \"launch failed\"}\n", name);
        return;
    }
    hipEventRecord(a);
    hipLaunchKernelGGL((k_mb<MODE, WAVES>), dim3(grid), dim3(64 * WAVES), lds, 0, out, ukey, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double blocks = (double)grid * 64 * WAVES * 32 * iters;
    const double bps = blocks / (ms / 1e3);
    printf("{\"variant\": \"%s\", \"waves_per_wg\": %d, \"grid\": %d, \"vgprs\": %d, \"spill_bytes\": %d, "
           "\"lds_bytes\": %zu, \"ms\": %.3f, \"blocks_per_s\": %.4g, \"blocks_per_clk_cu_at_2.4GHz\": %.4f}\n",
           name, WAVES, grid, fa.numRegs, (int)fa.localSizeBytes, lds, ms, bps, bps / (256 * 2.4e9));
    fflush(stdout);
}

int main() {
    uint32_t *out, *ukey;
    hipMalloc(&out, (size_t)256 * 64 * 1024 * 16 * sizeof(uint32_t));
    hipMalloc(&ukey, 64 * sizeof(uint32_t));
    hipMemset(ukey, 0x5a, 64 * sizeof(uint32_t));
    for (int rep = 0; rep < 2; rep++) {
        run<3, 16>(out, ukey, 256 * 4, "tt_ctr (T-table, counter groups, pairs) w16");
        run<4, 16>(out, ukey, 256 * 4, "tt_ctr_ukey (same, one wave-uniform key in SGPRs) w16");
        if (getenv("AES_MB_TT_ONLY")) continue;
        run<0, 4>(out, ukey, 256 * 16, "bs w4");
        run<0, 8>(out, ukey, 256 * 8, "bs w8");
        run<1, 4>(out, ukey, 256 * 16, "bs_ukey w4");
        run<2, 4>(out, ukey, 256 * 16, "bs_notr w4");
    }
    hipFree(out);
    hipFree(ukey);
    return 0;
}
