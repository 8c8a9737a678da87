// Shared definitions for the MI355X Mastic aggregator (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#define MH_HD __host__ __device__ __forceinline__
#define MH_D __device__ __forceinline__

// Three-input XOR.  On gfx950 this is one v_bitop3_b32 (LUT 0x96); hipcc does
// not fuse a ^ b ^ c on its own.
MH_D uint32_t xor3_u32(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct u32x2 {
    uint32_t lo, hi;
};

// 64-bit lane helpers on 32-bit halves (CDNA has no 64-bit bitwise ALU).
MH_D u32x2 rotl64(u32x2 v, int r) {
    // r is a compile-time constant at every call site; the branches fold away.
    if (r == 0) return v;
    if (r == 32) return u32x2{v.hi, v.lo};
    if (r < 32)
        return u32x2{__builtin_amdgcn_alignbit(v.lo, v.hi, 32 - r),
                     __builtin_amdgcn_alignbit(v.hi, v.lo, 32 - r)};
    return u32x2{__builtin_amdgcn_alignbit(v.hi, v.lo, 64 - r),
                 __builtin_amdgcn_alignbit(v.lo, v.hi, 64 - r)};
}

MH_D u32x2 xor64(u32x2 a, u32x2 b) { return u32x2{a.lo ^ b.lo, a.hi ^ b.hi}; }
MH_D u32x2 xor3_64(u32x2 a, u32x2 b, u32x2 c) {
    return u32x2{xor3_u32(a.lo, b.lo, c.lo), xor3_u32(a.hi, b.hi, c.hi)};
}

// Plane access through buffer resources: the base address is wave-uniform
// (kernel arguments + uniform indices) and lives in an SGPR descriptor; the
// only per-lane part is the 32-bit byte offset of the lane's report.  One VGPR
// serves every plane access instead of a 64-bit pointer per access stream
// (cdna_hip_programming.md T8/T20: readfirstlane makes uniformity provable).
MH_D __amdgpu_buffer_rsrc_t mh_rsrc(const void* p) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff, 0x00020000);
}
// load / store word `lane_bytes / 4` of the plane starting at uniform address p
MH_D uint32_t pld(const uint32_t* p, uint32_t lane_bytes) {
    return __builtin_amdgcn_raw_buffer_load_b32(mh_rsrc(p), lane_bytes, 0, 0);
}
MH_D void pst(uint32_t* p, uint32_t lane_bytes, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b32(v, mh_rsrc(p), lane_bytes, 0, 0);
}
// Word `soff / 4` of a block of planes: one descriptor per block (rs, uniform)
// and the uniform plane offset in soffset, so a 43-plane block costs 4 SGPRs
// for the descriptor instead of one descriptor per plane.
// (the binder sponges' block loads: a stream read once; MASTIC_SPONGE_LOAD_AUX
// sets their cache policy bits -- gfx950: 1 = sc0, 2 = nt, 16 = sc1)
#ifndef MASTIC_SPONGE_LOAD_AUX
#define MASTIC_SPONGE_LOAD_AUX 0
#endif
MH_D uint32_t pld_so(__amdgpu_buffer_rsrc_t rs, uint32_t lane_bytes, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, lane_bytes, soff, MASTIC_SPONGE_LOAD_AUX);
}
MH_D void pst_so(__amdgpu_buffer_rsrc_t rs, uint32_t lane_bytes, uint32_t soff, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b32(v, rs, lane_bytes, soff, 0);
}
