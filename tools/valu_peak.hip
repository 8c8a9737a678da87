// VALU throughput microbenchmark (gfx950): wave64 instructions per cycle per
// SIMD for the integer ops the hot path uses (v_xor_b32, v_bitop3_b32,
// v_perm_b32, v_alignbit_b32, v_add_u32), v_fma_f32 for comparison, and the
// candidates for cheaper AES addresses / Keccak rotations (64-bit shifts,
// v_lshl_add_u64, packed 16-bit ops, 24-bit multiply-adds).
// Every thread runs 8 independent dependency chains of one instruction kind
// (inline asm, so nothing is folded), full occupancy, many workgroups.
// Prints one JSON object: per op, wave-instructions/s, cycles per
// wave-instruction per SIMD at the measured clock assumption (2.4 GHz), and
// the implied chip peak in lane-ops/s.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_peak tools/valu_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096

#define CHAIN8(OP)                                                                         \
    for (int i = 0; i < ITERS; i++) {                                                    \
        OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)                          \
    }

#define XOR(r) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(k));
#define BOP3(r) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r) : "v"(k), "v"(k2));
#define PERM(r) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r) : "v"(k), "v"(k2));
#define ALIGN(r) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(r) : "v"(k));
#define ADD(r) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(k));
#define SDWA(r) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(r) : "v"(k));
#define ANDOR(r) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(r) : "v"(k), "v"(k2));
#define LSHLOR(r) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(r) : "v"(k));
#define BFE(r) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(r));
#define BFI(r) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(r) : "v"(k), "v"(k2));
#define LSHR(r) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(r));
#define FMA(r) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r) : "v"(k), "v"(k2));

#define LSHL64(r) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(r));
#define LSHR64(r) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(r));
#define LSHLADD64(r) asm volatile("v_lshl_add_u64 %0, %0, 3, %1" : "+v"(r) : "v"(kk));
#define MOV64(r) asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "v"(r ^ kk));
#define PKMOV(r) asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(r) : "v"(kk));
#define ADD64(r) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(r) : "v"(kk));
#define ALIGNBYTE(r) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(r) : "v"(k));
#define PKMAD16(r) asm volatile("v_pk_mad_u16 %0, %0, %1, %2" : "+v"(r) : "v"(k), "v"(k2));
#define PKLSHL16(r) asm volatile("v_pk_lshlrev_b16 %0, 8, %0" : "+v"(r));
#define MAD24(r) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(r) : "v"(k), "v"(k2));
#define MUL24(r) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r) : "v"(k));
#define XOR3(r) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(r) : "v"(k), "v"(k2));
#define LSHLADD(r) asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(r) : "v"(k));
#define ADD3(r) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r) : "v"(k), "v"(k2));
#define LSHL(r) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(r));
#define XORDPP(r) asm volatile("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(k));
#define CND(r) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r) : "v"(k));
#define MOVDPP(r) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r));
// lane i <-> i+32 / i+16 half exchanges (gfx950): one instruction writes both registers of a pair;
// counted below as one wave-instruction per swap (4 swaps per 8 registers per iteration, so the
// kernel runs twice the iterations to issue as many instructions as the others)
#define PL32(x, y) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
#define PL16(x, y) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
#define PAIRS(OP) OP(a0, a1) OP(a2, a3) OP(a4, a5) OP(a6, a7)
#define KERNELPAIR(NAME, OP)                                                             \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {          \
        uint32_t k = seed ^ threadIdx.x;                                                  \
        uint32_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5,     \
                 a6 = k + 6, a7 = k + 7;                                                  \
        for (int i = 0; i < 2 * ITERS; i++) { PAIRS(OP) }                                \
        uint32_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                               \
        if (s == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = s;                    \
    }

#define KERNEL(NAME, OP)                                                                 \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {          \
        uint32_t k = seed ^ threadIdx.x, k2 = seed * 3u + blockIdx.x;                     \
        uint32_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5,     \
                 a6 = k + 6, a7 = k + 7;                                                  \
        CHAIN8(OP)                                                                       \
        uint32_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                               \
        if (s == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = s;                    \
    }

#define KERNEL64(NAME, OP)                                                               \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {          \
        uint64_t kk = ((uint64_t)(seed ^ threadIdx.x) << 32) | (seed * 3u + blockIdx.x); \
        uint64_t a0 = kk, a1 = kk + 1, a2 = kk + 2, a3 = kk + 3, a4 = kk + 4, a5 = kk + 5, \
                 a6 = kk + 6, a7 = kk + 7;                                                \
        CHAIN8(OP)                                                                       \
        uint64_t s = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                               \
        if ((uint32_t)s == 0x12345678u) out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(s >> 32); \
    }

KERNEL(k_xor, XOR)
KERNEL(k_bitop3, BOP3)
KERNEL(k_perm, PERM)
KERNEL(k_alignbit, ALIGN)
KERNEL(k_add, ADD)
KERNEL(k_fma, FMA)
KERNEL(k_sdwa, SDWA)
KERNEL(k_andor, ANDOR)
KERNEL(k_lshlor, LSHLOR)
KERNEL(k_bfe, BFE)
KERNEL(k_bfi, BFI)
KERNEL(k_lshr, LSHR)
KERNEL64(k_lshl64, LSHL64)
KERNEL64(k_lshr64, LSHR64)
KERNEL64(k_lshladd64, LSHLADD64)
KERNEL64(k_mov64, MOV64)
KERNEL64(k_pkmov, PKMOV)
KERNEL(k_alignbyte, ALIGNBYTE)
KERNEL(k_pkmad16, PKMAD16)
KERNEL(k_pklshl16, PKLSHL16)
KERNEL(k_mad24, MAD24)
KERNEL(k_mul24, MUL24)
KERNEL(k_xor3, XOR3)
KERNEL(k_lshladd, LSHLADD)
KERNEL(k_add3, ADD3)
KERNEL(k_lshl, LSHL)
KERNEL(k_xordpp, XORDPP)
KERNEL(k_cnd, CND)
KERNEL(k_movdpp, MOVDPP)
KERNELPAIR(k_pl32, PL32)
KERNELPAIR(k_pl16, PL16)

int main() {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    const int cus = prop.multiProcessorCount;
    const double clk = 2.4e9;
    uint32_t* out;
    if (hipMalloc(&out, sizeof(uint32_t) * 256 * 8192) != hipSuccess) return 1;
    const int blocks = cus * 32;  // 8 waves per SIMD worth of 256-thread workgroups, many rounds
    struct K {
        const char* name;
        void (*fn)(uint32_t*, uint32_t);
    } ks[] = {{"v_xor_b32", k_xor},     {"v_bitop3_b32", k_bitop3}, {"v_perm_b32", k_perm},
              {"v_alignbit_b32", k_alignbit}, {"v_add_u32", k_add},       {"v_fma_f32", k_fma},
              {"v_mov_b32_sdwa(byte1<-byte2,preserve)", k_sdwa}, {"v_and_or_b32", k_andor},
              {"v_lshl_or_b32", k_lshlor}, {"v_bfe_u32", k_bfe}, {"v_bfi_b32", k_bfi}, {"v_lshrrev_b32", k_lshr},
              {"v_lshlrev_b64", k_lshl64}, {"v_lshrrev_b64", k_lshr64}, {"v_lshl_add_u64", k_lshladd64},
              {"v_mov_b64", k_mov64}, {"v_pk_mov_b32", k_pkmov}, {"v_alignbyte_b32", k_alignbyte},
              {"v_pk_mad_u16", k_pkmad16}, {"v_pk_lshlrev_b16", k_pklshl16}, {"v_mad_u32_u24", k_mad24},
              {"v_mul_u32_u24", k_mul24}, {"v_or3_b32", k_xor3}, {"v_lshl_add_u32", k_lshladd},
              {"v_add3_u32", k_add3}, {"v_lshlrev_b32", k_lshl}, {"v_xor_b32_dpp", k_xordpp},
              {"v_cndmask_b32", k_cnd}, {"v_mov_b32_dpp(quad_perm swap)", k_movdpp},
              {"v_permlane32_swap_b32", k_pl32}, {"v_permlane16_swap_b32", k_pl16}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d, \"clock_assumed_hz\": %.3g, \"blocks\": %d, \"threads\": 256, \"runs\": [", cus, clk,
           blocks);
    const int nk = (int)(sizeof(ks) / sizeof(ks[0]));
    for (int ii = 0; ii < 2 * nk; ii++) {  // two passes, the second in reverse order (clock drift check)
        const int i = ii < nk ? ii : 2 * nk - 1 - ii;
        hipLaunchKernelGGL(ks[i].fn, dim3(blocks), dim3(256), 0, 0, out, 1u);  // warm-up
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 5;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(ks[i].fn, dim3(blocks), dim3(256), 0, 0, out, 2u + r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double wave_instr = (double)reps * blocks * 4 /*waves*/ * ITERS * 8;
        const double wips = wave_instr / (ms / 1e3);
        const double cyc_per_wi_simd = (double)cus * 4 * clk / wips;
        printf("%s{\"op\": \"%s\", \"ms\": %.3f, \"wave_instr_per_s\": %.4g, \"cycles_per_wave_instr_per_simd\": %.3f, "
               "\"lane_ops_per_s\": %.4g}",
               ii ? ", " : "", ks[i].name, ms, wips, cyc_per_wi_simd, wips * 64);
    }
    printf("]}\n");
    return 0;
}
