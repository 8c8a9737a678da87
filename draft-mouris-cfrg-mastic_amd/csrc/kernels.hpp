// HIP kernels of the batched Mastic aggregator (gfx950).
//
// Data layout in HBM: every per-report vector is stored as word PLANES,
// plane[w][stride] with stride = reports padded to a multiple of 64, so lane
// r of a wave always touches word r of a plane: all loads/stores coalesce.
// The tree shape (agg_param) is shared by every report of a batch, so all
// control flow below is wave-uniform; only data differs per lane.
//
// Reference mapping (poc/):
//   k_eval_aes     Vidpf.eval_with_siblings / eval_next / extend / convert
//                  (vidpf.py:213-364) for one tree level, plus the per-parent
//                  payload difference of Mastic.prep_init (mastic.py:267-271)
//                  and the truncated out shares (:311-314)
//   k_node_proof   Vidpf.node_proof (vidpf.py:366-380) for one tree level
//   k_absorb       the one-hot / payload binders' TurboSHAKE absorption
//                  (mastic.py:259-287), streamed level by level
//   k_finalize     payload/onehot checks, counter check, eval proof (:277-306)
//   k_flp_rand     query rand, helper proof share, joint rand (:437-510)
//   k_flp_query    FlpBBCGGI19.query (:250-256)
//   k_fold         agg_update / merge over reports (:379-397)
//   k_decide       prep_shares_to_prep (:320-362)
//   k_shard        client Mastic.shard (:91-185) incl. Vidpf.gen (vidpf.py:103-211)
#pragma once
#include "aes.hpp"
#include "flp.hpp"
#include "keccak.hpp"

// ------------------------------------------------------------- prefix states
enum PfxId {
    PFX_EXT = 0,        // XofFixedKeyAes128 key, usage EXTEND  (D = 2)
    PFX_CONV,           // XofFixedKeyAes128 key, usage CONVERT (D = 2)
    PFX_NODE,           // node proof, seed length 16
    PFX_ONEHOT,         // onehot check, empty seed
    PFX_PAYLOAD,        // payload check, empty seed
    PFX_EVAL,           // eval proof, verify key as seed
    PFX_QUERY,          // query rand, verify key as seed
    PFX_PROOF_SHARE,    // helper proof share, 32-byte seed follows
    PFX_JR_PART,        // joint rand part, 32-byte seed follows
    PFX_JR_SEED,        // joint rand seed, empty seed
    PFX_JR,             // joint rand, 32-byte seed follows
    PFX_PROVE_RAND,     // prove rand (client), 32-byte seed follows
    PFX_TREE,           // eval-proof Merkle tree node hash (proof-aggregation mode), empty seed
    PFX_COUNT
};

struct PrefixState {
    KState st;
    int f;
    int pad[3];
};

__global__ void k_prefix_states(const uint8_t* bytes, const int* offs, const int* lens, int count,
                                PrefixState* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int i = 0; i < count; i++) {
        KState s;
        kstate_zero(s);
        int f = sponge_absorb_bytes_slow(s, 0, bytes + offs[i], lens[i]);
        out[i].st = s;
        out[i].f = f;
    }
}

MH_D void load_prefix(const PrefixState* ps, int id, KState& s, int& f) {
    s = ps[id].st;
    f = ps[id].f;
}

MH_D uint32_t ld_u32_bytes(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// ------------------------------------------------------------- planes
struct Planes {
    int n, stride;
    // report inputs (unpacked)
    uint32_t* key;       // [4]
    uint32_t* nonce;     // [4]
    uint32_t* cw_seed;   // [bits][4]
    uint32_t* cw_ctrl;   // [bits]
    uint32_t* cw_w;      // [bits][vl*w32]
    uint32_t* cw_proof;  // [bits][8]
    uint32_t* lps;       // [proof_len*w32] leader proof share (agg 0)
    uint32_t* seed;      // [8]  FLP seed (agg 1: helper seed, agg 0: leader seed)
    uint32_t* peer;      // [8]  peer joint rand part
    uint32_t* rk_ext;    // [44]
    uint32_t* rk_conv;   // [44]
    // sponges
    uint32_t* sp_onehot;   // [50]
    uint32_t* sp_payload;  // [50]
    // results
    uint32_t* rootsum;     // [vl*w32]   w_L0 + w_R0 (raw)
    uint32_t* beta;        // [vl*w32]   beta share (negated for agg 1)
    uint32_t* eval_proof;  // [8]
    uint32_t* proof;       // [proof_len*w32]
    uint32_t* qr;          // [qrl*w32]
    uint32_t* jr;          // [jrl*w32]
    uint32_t* jr_part;     // [8]
    uint32_t* jr_seed;     // [8]
    uint32_t* verifier;    // [verifier_len*w32]
    int32_t* status;       // [1]
};

// ------------------------------------------------------------- unpack
// nw little-endian words of one report's wire row into plane rows dst[k * step].
// A == 8: the row, the segment and every report's row start are 8-byte aligned
// (the common case: BITS a multiple of 32), so a lane reads two words per load
// instead of eight byte loads (each lane reads its own row: every load of the
// wave touches 64 cache lines, so the instruction count is what costs).
template <int A>
MH_D void unpack_words(const uint8_t* src, int nw, uint32_t* dst, size_t step) {
    if constexpr (A == 8) {
        const uint2* s2 = (const uint2*)src;
        int k = 0;
        for (; k + 1 < nw; k += 2) {
            const uint2 v = s2[k >> 1];
            dst[(size_t)k * step] = v.x;
            dst[(size_t)(k + 1) * step] = v.y;
        }
        if (k < nw) dst[(size_t)k * step] = ((const uint32_t*)src)[k];
    } else {
        for (int k = 0; k < nw; k++) dst[(size_t)k * step] = ld_u32_bytes(src + 4 * k);
    }
}

// Wire public share: pack_bits(ctrl) || seed_cw[B] || w_cw[B] || proof_cw[B]
// (poc/vidpf.py:382-394).  Input share: key || [leader proof share] || [seed]
// || [peer jr part] (poc/mastic.py:516-529).
// big = false: every segment; big = true: the correction words and the
// leader proof share are left to k_rows_to_planes (coalesced row tiles).
template <int A>
MH_D void unpack_report(const McParams& p, const Planes& pl, int agg_id, int r, const uint8_t* ps, const uint8_t* is,
                        const uint8_t* nc, int l_lo, int l_hi, bool big = false) {
    const size_t S = (size_t)pl.stride;
    const int nctrl = (2 * p.bits + 7) / 8;
    const int wl = p.value_len * p.w32;
    unpack_words<A>(nc, 4, pl.nonce + r, S);
    unpack_words<A>(is, 4, pl.key + r, S);
    for (int l = l_lo; l < l_hi; l++) {
        uint32_t c0 = (ps[(2 * l) >> 3] >> ((2 * l) & 7)) & 1;
        uint32_t c1 = (ps[(2 * l + 1) >> 3] >> ((2 * l + 1) & 7)) & 1;
        pl.cw_ctrl[(size_t)l * S + r] = c0 | (c1 << 1);
        if (big) continue;
        unpack_words<A>(ps + nctrl + 16 * l, 4, pl.cw_seed + (size_t)l * 4 * S + r, S);
        unpack_words<A>(ps + nctrl + 16 * p.bits + (size_t)l * p.value_len * p.enc, wl,
                        pl.cw_w + (size_t)l * wl * S + r, S);
        unpack_words<A>(ps + nctrl + 16 * p.bits + (size_t)p.bits * p.value_len * p.enc + 32 * l, 8,
                        pl.cw_proof + (size_t)l * 8 * S + r, S);
    }
    const uint8_t* q = is + 16;
    if (agg_id == 0) {
        if (!big) unpack_words<A>(q, p.proof_len * p.w32, pl.lps + r, S);
        q += (size_t)p.proof_len * p.enc;
    }
    if (agg_id == 1 || p.joint_rand_len > 0) {
        unpack_words<A>(q, 8, pl.seed + r, S);
        q += 32;
    }
    if (p.joint_rand_len > 0) unpack_words<A>(q, 8, pl.peer + r, S);
}

__global__ __launch_bounds__(256) void k_unpack(McParams p, Planes pl, int agg_id, const uint8_t* nonces,
                                                const uint8_t* pub, const uint8_t* ins, int l_lo, int l_hi,
                                                int big) {
    // correction words of levels l_lo .. l_hi-1 only: a call at level L never
    // reads deeper ones, and a frontier-cache hit only reads level L's
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= pl.n) return;
    const size_t ps_size = mc_public_share_size(p);
    const size_t is_size = mc_input_share_size(p, agg_id);
    const uint8_t* ps = pub + ps_size * r;
    const uint8_t* is = ins + is_size * r;
    const uint8_t* nc = nonces + 16 * (size_t)r;
    const size_t nctrl = (2 * p.bits + 7) / 8;
    // every segment offset is nctrl plus multiples of 8 bytes (enc is 8 or 16)
    const bool a8 = (((uintptr_t)pub | (uintptr_t)ins | (uintptr_t)nonces | ps_size | is_size | nctrl) & 7) == 0;
    if (a8)
        unpack_report<8>(p, pl, agg_id, r, ps, is, nc, l_lo, l_hi, big != 0);
    else
        unpack_report<1>(p, pl, agg_id, r, ps, is, nc, l_lo, l_hi);
}

// Words [0, nwords) of every report's wire row (row r at src + r * row_bytes,
// 8-byte aligned) into plane rows: dst[j * S + r] = word j of row r.  With one
// lane per report (k_unpack) every load of a wave touches 64 rows, i.e. 64
// cache lines for 8 bytes each (C5: 32 ms for its 526 KB public shares at
// 16,384 reports, ~0.5 TB/s); here a workgroup moves a tile of 64 reports x
// 64 words through LDS: each half-wave reads 256 contiguous bytes of one row,
// each wave writes 256 contiguous bytes of one plane row.
__global__ __launch_bounds__(256) void k_rows_to_planes(const uint8_t* src, size_t row_bytes, int n, int nwords,
                                                        uint32_t* dst, int S) {
    __shared__ uint32_t tile[64 * 65];  // [report][word], pitch 65: the transposed reads hit 64 banks
    const int r0 = blockIdx.x * 64, j0 = blockIdx.y * 64;
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int q = k * 256 + t;
        const int rr = q >> 5, wp = q & 31;  // report of the tile, word pair
        const int j = j0 + 2 * wp;
        uint2 v = make_uint2(0u, 0u);
        if (r0 + rr < n) {
            const uint8_t* row = src + (size_t)(r0 + rr) * row_bytes;
            if (j + 1 < nwords)
                v = *(const uint2*)(row + 4 * (size_t)j);
            else if (j < nwords)
                v.x = *(const uint32_t*)(row + 4 * (size_t)j);
        }
        tile[rr * 65 + 2 * wp] = v.x;
        tile[rr * 65 + 2 * wp + 1] = v.y;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int q = k * 256 + t;
        const int jj = q >> 6, rr = q & 63;
        if (r0 + rr < n && j0 + jj < nwords) dst[(size_t)(j0 + jj) * S + r0 + rr] = tile[rr * 65 + jj];
    }
}

// ------------------------------------------------------------- key setup
// The two fixed AES keys of a report depend only on (ctx, usage, nonce)
// (vdaf_poc XofFixedKeyAes128): derive them once, expand once.  sponges:
// also start both binder sponges (not on a frontier-cache hit, which resumes
// them from the cache's planes).
__global__ __launch_bounds__(256) void k_setup(Planes pl, const PrefixState* pfx, int sponges) {
    __shared__ uint32_t T[AES_LDS_WORDS];
    aes_lds_fill(T, threadIdx.x, 256);
    __syncthreads();
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= pl.stride) return;
    const int S = pl.stride;
    AesLds TL{T + (threadIdx.x & 31)};
    for (int which = 0; which < 2; which++) {
        KState s;
        int f;
        load_prefix(pfx, which == 0 ? PFX_EXT : PFX_CONV, s, f);
        f = sponge_absorb_words(s, f, 16, [&](int m) { return pl.nonce[m * S + r]; });
        sponge_pad(s, f, 0x02);
        uint32_t key[4] = {s.a[0].lo, s.a[0].hi, s.a[1].lo, s.a[1].hi};
        uint32_t rk[44];
        aes128_expand(TL, key, rk);
        uint32_t* dst = which == 0 ? pl.rk_ext : pl.rk_conv;
#pragma unroll
        for (int i = 0; i < 44; i++) dst[i * S + r] = rk[i];
    }
    if (!sponges) return;
    KState s;
    int f;
    load_prefix(pfx, PFX_ONEHOT, s, f);
#pragma unroll
    for (int i = 0; i < 25; i++) {
        pl.sp_onehot[(2 * i) * S + r] = s.a[i].lo;
        pl.sp_onehot[(2 * i + 1) * S + r] = s.a[i].hi;
    }
    load_prefix(pfx, PFX_PAYLOAD, s, f);
#pragma unroll
    for (int i = 0; i < 25; i++) {
        pl.sp_payload[(2 * i) * S + r] = s.a[i].lo;
        pl.sp_payload[(2 * i + 1) * S + r] = s.a[i].hi;
    }
}

// ------------------------------------------------------------- convert stream
// XofFixedKeyAes128(seed, dst(ctx, CONVERT), nonce) after next(16):
// next_vec(field, VALUE_LEN) with rejection of candidates >= p.
template <class F> struct ConvStream;

template <> struct ConvStream<F64> {
    uint32_t seed[4];
    uint32_t blk[4];
    uint32_t ctr;
    uint32_t half;
    MH_D void init(const uint32_t s[4]) {
        seed[0] = s[0]; seed[1] = s[1]; seed[2] = s[2]; seed[3] = s[3];
        ctr = 1;
        half = 2;
    }
    // Common case: both children's streams need their next block at the same
    // element (no rejection so far): produce both in one paired AES call.
    template <class TT, class RK>
    MH_D void refill_pair(ConvStream& o, const TT& T, const RK& rk) {
        if (half == 2 && o.half == 2) {
            fixed_key_block2(T, rk, seed, ctr, o.seed, o.ctr, blk, o.blk);
            ctr++;
            o.ctr++;
            half = 0;
            o.half = 0;
        }
    }
    template <class TT, class RK>
    MH_D uint64_t next(const TT& T, const RK& rk) {
        uint64_t v;
        do {
            if (half == 2) {
                fixed_key_block(T, rk, seed, ctr, blk);
                ctr++;
                half = 0;
            }
            v = half ? (((uint64_t)blk[3] << 32) | blk[2]) : (((uint64_t)blk[1] << 32) | blk[0]);
            half++;
        } while (!F64::valid(v));
        return v;
    }
};

// Field64 stream of the level kernel: up to four candidates (two blocks)
// buffered per node, so two sibling streams refill with ONE 4-block lockstep
// AES call (fixed_key_block_n<4>); the last refill of a node (at most two
// elements still needed) is a paired call of one block per sibling.  A stream
// that rejected a candidate (probability ~2^-32) falls out of step with its
// sibling and refills alone, block by block, exactly as the reference's
// next_vec does.
template <bool QUAD>
struct ConvQuad {
    static constexpr int GROUP = QUAD ? 4 : 2;  // candidates per refill
    uint32_t seed[4];
    uint32_t blk[8];  // candidate i = blk[2i] | blk[2i+1] << 32
    uint32_t ctr;
    uint32_t pos;     // next candidate slot, 4 = empty
    MH_D void init(const uint32_t s[4]) {
        seed[0] = s[0]; seed[1] = s[1]; seed[2] = s[2]; seed[3] = s[3];
        ctr = 1;
        pos = 4;
    }
    template <class RK>
    MH_D void refill(ConvQuad& o, int remaining, const AesPerm& T, const RK& rk) {
        if (pos == 4 && o.pos == 4) {
            if (QUAD && remaining > 2) {
                const uint32_t* const sd[4] = {seed, seed, o.seed, o.seed};
                const uint32_t cv[4] = {ctr, ctr + 1, o.ctr, o.ctr + 1};
                uint32_t* const ov[4] = {blk, blk + 4, o.blk, o.blk + 4};
                fixed_key_block_n<4>(T, rk, sd, cv, ov);
                ctr += 2;
                o.ctr += 2;
                pos = 0;
                o.pos = 0;
            } else {
                const uint32_t* const sd[2] = {seed, o.seed};
                const uint32_t cv[2] = {ctr, o.ctr};
                uint32_t* const ov[2] = {blk + 4, o.blk + 4};
                fixed_key_block_n<2>(T, rk, sd, cv, ov);
                ctr++;
                o.ctr++;
                pos = 2;
                o.pos = 2;
            }
        }
    }
    template <class RK>
    MH_D uint64_t next(const AesPerm& T, const RK& rk) {
        uint64_t v;
        do {
            if (pos == 4) {
                const uint32_t* const sd[1] = {seed};
                const uint32_t cv[1] = {ctr};
                uint32_t* const ov[1] = {blk + 4};
                fixed_key_block_n<1>(T, rk, sd, cv, ov);
                ctr++;
                pos = 2;
            }
            const uint32_t lo = pos == 0 ? blk[0] : pos == 1 ? blk[2] : pos == 2 ? blk[4] : blk[6];
            const uint32_t hi = pos == 0 ? blk[1] : pos == 1 ? blk[3] : pos == 2 ? blk[5] : blk[7];
            v = ((uint64_t)hi << 32) | lo;
            pos++;
        } while (!F64::valid(v));
        return v;
    }
};

// Field128 counterpart: one candidate per block, two buffered per node.
template <bool QUAD>
struct ConvQuad128 {
    static constexpr int GROUP = QUAD ? 2 : 1;
    uint32_t seed[4];
    uint32_t blk[8];  // candidate i = blk[4i .. 4i+3]
    uint32_t ctr;
    uint32_t pos;     // next candidate slot, 2 = empty
    MH_D void init(const uint32_t s[4]) {
        seed[0] = s[0]; seed[1] = s[1]; seed[2] = s[2]; seed[3] = s[3];
        ctr = 1;
        pos = 2;
    }
    template <class RK>
    MH_D void refill(ConvQuad128& o, int remaining, const AesPerm& T, const RK& rk) {
        if (pos == 2 && o.pos == 2) {
            if (QUAD && remaining > 1) {
                const uint32_t* const sd[4] = {seed, seed, o.seed, o.seed};
                const uint32_t cv[4] = {ctr, ctr + 1, o.ctr, o.ctr + 1};
                uint32_t* const ov[4] = {blk, blk + 4, o.blk, o.blk + 4};
                fixed_key_block_n<4>(T, rk, sd, cv, ov);
                ctr += 2;
                o.ctr += 2;
                pos = 0;
                o.pos = 0;
            } else {
                const uint32_t* const sd[2] = {seed, o.seed};
                const uint32_t cv[2] = {ctr, o.ctr};
                uint32_t* const ov[2] = {blk + 4, o.blk + 4};
                fixed_key_block_n<2>(T, rk, sd, cv, ov);
                ctr++;
                o.ctr++;
                pos = 1;
                o.pos = 1;
            }
        }
    }
    template <class RK>
    MH_D F128::E next(const AesPerm& T, const RK& rk) {
        F128::E v;
        do {
            if (pos == 2) {
                const uint32_t* const sd[1] = {seed};
                const uint32_t cv[1] = {ctr};
                uint32_t* const ov[1] = {blk + 4};
                fixed_key_block_n<1>(T, rk, sd, cv, ov);
                ctr++;
                pos = 1;
            }
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; i++) w[i] = pos == 0 ? blk[i] : blk[4 + i];
            v = F128::from_words(w);
            pos++;
        } while (!F128::valid(v));
        return v;
    }
};

template <> struct ConvStream<F128> {
    uint32_t seed[4];
    uint32_t blk[4];
    uint32_t ctr;
    uint32_t have;  // blk holds an unconsumed candidate
    MH_D void init(const uint32_t s[4]) {
        seed[0] = s[0]; seed[1] = s[1]; seed[2] = s[2]; seed[3] = s[3];
        ctr = 1;
        have = 0;
    }
    template <class TT, class RK>
    MH_D void refill(ConvStream& o, int, const TT& T, const RK& rk) {
        refill_pair(o, T, rk);
    }
    template <class TT, class RK>
    MH_D void refill_pair(ConvStream& o, const TT& T, const RK& rk) {
        if (!have && !o.have) {
            fixed_key_block2(T, rk, seed, ctr, o.seed, o.ctr, blk, o.blk);
            ctr++;
            o.ctr++;
            have = 1;
            o.have = 1;
        }
    }
    template <class TT, class RK>
    MH_D F128::E next(const TT& T, const RK& rk) {
        F128::E v;
        do {
            if (!have) {
                fixed_key_block(T, rk, seed, ctr, blk);
                ctr++;
            }
            have = 0;
            v = F128::from_words(blk);
        } while (!F128::valid(v));
        return v;
    }
};

template <class F, bool QUAD> struct EvalStream;
template <bool Q> struct EvalStream<F64, Q> { typedef ConvQuad<Q> type; };
template <bool Q> struct EvalStream<F128, Q> { typedef ConvQuad128<Q> type; };

// ------------------------------------------------------------- node proof body
#define NP_WIN 14
template <int Q>
MH_D void np_xor_window(KState& s, const uint32_t* x) {
#pragma unroll
    for (int k = 0; k < NP_WIN; k++)
        if (Q + k < KECCAK_RATE_WORDS) kxor_word(s, Q + k, x[k]);
}
template <int Q>
MH_D void np_xor_overflow(KState& s, const uint32_t* x) {
#pragma unroll
    for (int k = 0; k < NP_WIN; k++)
        if (Q + k >= KECCAK_RATE_WORDS) kxor_word(s, Q + k - KECCAK_RATE_WORDS, x[k]);
}
#define NP_CASES(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) \
    M(15) M(16) M(17) M(18) M(19) M(20) M(21) M(22) M(23) M(24) M(25) M(26) M(27) M(28) M(29) M(30) \
    M(31) M(32) M(33) M(34) M(35) M(36) M(37) M(38) M(39) M(40) M(41)

// One node proof: TurboSHAKE128 over the pre-absorbed prefix state np (fill
// position f) and the body  seed || le16(BITS) || le16(level) || path,
// XORed with the level's proof correction word when the node's control bit
// t is set.  Writes 8 words through `put(j, w)`.  All positions uniform.
template <bool FUSE_D = true, class Put>
MH_D void node_proof_one(const PrefixState* np, int f, int bits, int level, int path_bytes, const uint32_t seed[4],
                         const uint32_t* path, uint32_t t, const uint32_t pcw[8], Put put) {
    const int q = f >> 2;
    const int sh = f & 3;
    const int nbytes = 20 + path_bytes;  // body; the domain byte 0x01 follows
    const bool cross = f + nbytes >= KECCAK_RATE;
    const uint32_t amt = (32 - 8 * sh) & 31;
    const int dw = nbytes >> 2;
    const uint32_t dbit = 1u << (8 * (nbytes & 3));
    uint32_t B[NP_WIN];
#pragma unroll
    for (int i = 0; i < 4; i++) B[i] = seed[i];
    B[4] = (uint32_t)bits | ((uint32_t)level << 16);
#pragma unroll
    for (int k = 5; k < NP_WIN; k++) B[k] = k - 5 < 8 ? path[k - 5] : 0u;
#pragma unroll
    for (int k = 4; k < NP_WIN; k++) B[k] |= (k == dw) ? dbit : 0u;
    uint32_t x[NP_WIN];
#pragma unroll
    for (int k = 0; k < NP_WIN; k++) {
        const uint32_t hi = B[k];
        const uint32_t lo = k ? B[k - 1] : 0u;
        x[k] = sh ? __builtin_amdgcn_alignbit(hi, lo, amt) : hi;
    }
    asm volatile("" ::: "memory");  // re-read the uniform prefix state, do not pin 50 registers
    KState s = np->st;
    switch (q) {
#define NP_W(Q) case Q: np_xor_window<Q>(s, x); break;
        NP_CASES(NP_W)
#undef NP_W
    }
    if (cross) {
        keccak_p12<12, FUSE_D>(s);
        switch (q) {
#define NP_O(Q) case Q: np_xor_overflow<Q>(s, x); break;
            NP_CASES(NP_O)
#undef NP_O
        }
    }
    s.a[20].hi ^= 0x80000000u;
    keccak_p12<12, FUSE_D>(s);
#pragma unroll
    for (int j = 0; j < 8; j++) put(j, kword(s, j) ^ (t ? pcw[j] : 0u));
}

// ------------------------------------------------------------- eval level
// A tree level is evaluated by two kernels:
//   k_eval_aes    extend + correct + convert of both children of every parent
//                 (all the AES: 2 + 2 * (1 + ceil(VL*ENC/16)) blocks per
//                 parent), payload corrections, the parent payload difference
//                 and the truncated out shares;
//   k_node_proof  the children's node proofs (one Keccak-p each).
// The next seeds and control bits of all children go through a per-level
// plane buffer ("child seeds", 5 words per node) from the first to the second
// kernel and to the next level's k_eval_aes.  Splitting lets the LDS-bound AES
// run at 4 waves/SIMD and the VALU-only Keccak overlap it on another stream.
struct AesArgs {
    int level;
    int agg_id;
    int n_parents;       // parents at this level (1 = the root at level 0)
    int ppw;             // items per wave (an item is a parent, or one block range of one)
    // Small levels (few parents: the top of every tree) leave most waves of a
    // workgroup idle and each parent's ~2 + 2 nblk AES blocks a serial chain
    // of one wave.  There a parent is split into `split` items: item k
    // recomputes the parent's extend pair (2 blocks) and evaluates blocks
    // [k * split_blocks, (k + 1) * split_blocks) of both children's convert
    // streams (counter mode: the blocks are independent); item 0 also the
    // next seeds.  Never at a level that emits out shares (the truncation
    // accumulates across elements) or on a frontier-cache hit.
    int split;
    int split_blocks;
    const int32_t* parent_node;  // [n_parents] node index of each parent in level-1 (level >= 1)
    const int32_t* child_exp;    // [2 * n_parents] index into this level's frontier, -1 = leaf
    const int32_t* child_pfx;    // [2 * n_parents] index into the prefix list (level L), -1 = none
    const uint32_t* cs_in;       // child seeds of level-1: [node][5]
    uint32_t* cs_out;            // child seeds of this level: [node][5] (seed words, ctrl)
    const uint32_t* fr_w_in;     // payloads of level-1's expanded nodes [e][vl*w32]
    uint32_t* fr_w_out;
    uint32_t* payload;   // [n_parents * vl*w32]  w_p - w_L - w_R of the parents (BFS order)
    uint32_t* out;       // [n_prefixes * (1 + out_len) * w32] planes of the result buffer (row stride out_stride)
    int out_stride;
    int force_slow_blk;  // test hook: the Field64 fast path hands over to the exact stream at this block (-1 = never)
    // frontier cache (mastic_set_frontier_cache).  A cached node is 5 words: its convert seed (the
    // extend output after correction, the seed of convert) and its control bit.  Last level of a
    // prep_init: every child's node is written straight into the cache's spare slot (cache_out,
    // plane stride cache_stride).  Cache hit: the parents come from the cache (cs_in, stride
    // in_stride), and each parent's seed (block 0 of its convert stream) and payload (the rest of
    // the stream, corrected) are recomputed, the payload into wp_buf by parent ordinal.
    uint32_t* cache_out;
    int cache_stride;
    uint32_t* wp_buf;
    int recompute_wp;
    int in_stride;  // plane stride of cs_in (the cache's, on a hit; else the work buffer's)
    // frontier-cache hit (FC only): the AES waves also compute THIS level's
    // node proofs right after each parent's payloads (no k_node_proof launch)
    int fuse_proofs;
    int cur_path_bytes;              // ceil((level + 1) / 8)
    const uint32_t* cur_child_path;  // [2 * n_parents][8]
    uint32_t* cur_onehot;            // this level's proof tiles
    // node proofs of the PREVIOUS level (vidpf.py:366-380, :321-323), computed
    // by the workgroup's EVAL_PROOF_WAVES proof waves beside the AES waves
    int pv_level;                   // level - 1
    int pv_nodes;                   // its node count (0 at level 0)
    int pv_npw;                     // nodes per proof wave
    int pv_path_bytes;              // ceil(level / 8)
    const uint32_t* pv_child_path;  // [pv_nodes][8]
    uint32_t* pv_onehot;            // [pv_nodes * 8] proofs of level - 1 (tiled, see AbsorbArgs)
    int oh_gstride;                 // words per report group of the proof buffers
    int bin_rstride;                // words between consecutive words of a report in them
    int pay_gstride;                // ... of the payload-difference buffers
    const PrefixState* np;          // node-proof prefix state
    int np_f;                       // its fill position
    int aes_waves;                  // waves [0, aes_waves) walk parents, the rest are proof waves
    int par_waves;                  // parents per workgroup = par_waves * ppw (aes_waves, or all 16 waves)
    int proof_prio;                 // s_setprio of the proof waves
    int aes_prio;                   // s_setprio of the AES waves
    int dbg_skip;                   // timing experiments only (results wrong): 1 = no proof work, 2 = no AES work
};

// Frontier-cache hit: the payload w_p of a parent (a node of the cached
// level), elements [e_lo, e_hi), recomputed from its convert seed cv and
// control bit t exactly as its own evaluation produced it (vidpf.py:352-364
// then the payload correction of eval_next, vidpf.py:317-319) and stored as
// element row0 + e of the planes `out`.  Fast path: consecutive blocks of the
// one stream in pairs (counters c, c+1 share their rounds 1-2 when c >> 8
// agrees), speculating that no candidate is rejected; if a lane of the wave
// meets a candidate >= p among the elements it uses, the exact next_vec
// stream takes over from that element.
template <class F>
MH_D void parent_payload(const AesPerm& TL, const RkLds& rkc, const uint32_t cv[4], uint32_t t, const uint32_t* cw,
                         int S, int r, int e_lo, int e_hi, uint32_t* out, int row0, int force_slow_blk,
                         uint32_t seed_out[4]) {
    typedef typename F::E E;
    constexpr int EPB = F::W32 == 2 ? 2 : 1;  // elements per block
    const int nblk = (e_hi + EPB - 1) / EPB;
    AesCtrGroup g;
    uint32_t g_hi = 0u;
    {
        // the parent's seed: block 0 of the same stream (next(16), vidpf.py:352-364), in the
        // counter group of the payload's first blocks
        const uint32_t* const sd[1] = {cv};
        const uint32_t hv[1] = {0u};
        AesCtrGroup* const gi[1] = {&g};
        ctr_group_init<1>(TL, rkc, sd, hv, gi);
        const AesCtrGroup* const gg[1] = {&g};
        const uint32_t c0v[1] = {0u};
        uint32_t* const ov[1] = {seed_out};
        ctr_blocks_n<1>(TL, rkc, gg, sd, c0v, ov);
    }
    int e_fast = e_lo;
    auto put = [&](int e, E x) {
        if (t) x = F::add(x, pl_load<F>(cw, e, S, r));
        pl_store<F>(out, row0 + e, S, r, x);
    };
    for (int b = e_lo / EPB; b < nblk; b += 2) {
        asm volatile("" ::: "memory");
        const uint32_t c0 = (uint32_t)(b + 1), c1 = c0 + 1;
        const bool two = b + 1 < nblk;
        // this pair's payload correction words, loaded before its AES (after
        // the previous pair's stores they would wait for those stores)
        E cwv[2 * EPB];
#pragma unroll
        for (int k = 0; k < 2 * EPB; k++) cwv[k] = pl_load<F>(cw, min(EPB * b + k, e_hi - 1), S, r);
        uint32_t o[2][4];
        if ((c0 & ~0xffu) == (c1 & ~0xffu)) {
            if ((c0 & ~0xffu) != g_hi) {
                const uint32_t* const sd[1] = {cv};
                const uint32_t hv[1] = {c0 & ~0xffu};
                AesCtrGroup* const gi[1] = {&g};
                ctr_group_init<1>(TL, rkc, sd, hv, gi);
                g_hi = c0 & ~0xffu;
            }
            const AesCtrGroup* const gg[2] = {&g, &g};
            const uint32_t* const sd2[2] = {cv, cv};
            const uint32_t cvv[2] = {c0, c1};
            uint32_t* const ov[2] = {o[0], o[1]};
            ctr_blocks_n<2>(TL, rkc, gg, sd2, cvv, ov);
        } else {  // the pair straddles a counter group (C5's long streams)
            const uint32_t* const sd2[2] = {cv, cv};
            const uint32_t cvv[2] = {c0, c1};
            uint32_t* const ov[2] = {o[0], o[1]};
            fixed_key_block_n<2>(TL, rkc, sd2, cvv, ov);
        }
        // candidates of these blocks that the parent uses: elements EPB*b ..
        bool sus = false;
        const int e0 = EPB * b;
#pragma unroll
        for (int k = 0; k < 2 * EPB; k++) {
            const int e = e0 + k;
            const uint32_t top = EPB == 2 ? o[k >> 1][2 * (k & 1) + 1] : o[k][3];
            if (e < e_hi && (k < EPB || two)) sus |= top == ~0u;
        }
        if (__builtin_expect(__any(sus), 0) || b == force_slow_blk || b + 1 == force_slow_blk) break;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the loads above and the previous stores are done
#pragma unroll
        for (int k = 0; k < 2 * EPB; k++) {
            const int e = e0 + k;
            if (e < e_hi && (k < EPB || two)) {
                E x = F::from_words(&o[k / EPB][(k % EPB) * F::W32]);
                if (t) x = F::add(x, cwv[k]);
                pl_store<F>(out, row0 + e, S, r, x);
            }
        }
        e_fast = min(e_hi, e0 + 2 * EPB);
    }
    if (e_fast < e_hi) {
        // exact next_vec stream from the stream's start, emitting from e_fast on
        typename EvalStream<F, false>::type st;
        st.init(cv);
        for (int e = 0; e < e_hi; e++) {
            asm volatile("" ::: "memory");
            const E x = st.next(TL, rkc);
            if (e >= e_fast) put(e, x);
        }
    }
}

// One workgroup = 64 reports (one per lane) x 16 waves: 8 AES waves walk
// this level's parents and 8 proof waves first compute the node proofs of the
// previous level's children (a Keccak-p per node, VALU only), then join the
// AES waves; parents are claimed in runs through an LDS counter.  LDS-bound
// AES and VALU-bound Keccak share every CU inside one launch instead of two
// kernels competing for CU slots.  LDS: the v_perm-addressed T0/T2 table (64 KiB,
// aes.hpp AesPerm) and the 64 reports' two AES key schedules (22 KiB, one
// ds_read_b128 per round) are shared by all 16 waves: 86 KiB per workgroup,
// one workgroup = 4 waves per SIMD per CU.
#define EVAL_WAVES 16
// Counter groups (aes.hpp): rounds 1-2 shared by the blocks of one seed in
// the extend pair, the convert seeds and the payload fast path.
#ifndef MASTIC_EMIT_WAIT
#define MASTIC_EMIT_WAIT 1
#endif
#ifndef MASTIC_CTR_GROUPS
#define MASTIC_CTR_GROUPS 1
#endif
#define EVAL_PROOF_WAVES 8  // default split (mastic_ctx::proof_waves); measured best of 2..12
// VGPR cap of the level kernel: 4 waves x 96 per SIMD leave 128 of the 512
// for one binder-sponge wave (k_absorb_pair), so the two kernels can share a
// CU instead of taking turns.
// (expressed as a minimum occupancy: 5 waves/SIMD <=> at most 96 VGPRs)
#ifndef EVAL_MIN_WAVES
#define EVAL_MIN_WAVES 5
#endif
// The frontier-cache instantiation (FC: a cache hit's one level, a cache-on
// call's last level) runs with no binder-sponge waves beside it on a hit, so
// it may take all 128 VGPRs of its 4 waves per SIMD (the LDS-resident tables
// allow one workgroup per CU): no spills of the recompute / fused-proof state.
#ifndef EVAL_FC_MIN_WAVES
#define EVAL_FC_MIN_WAVES 4
#endif
#define EVAL_VGPR_ATTR __attribute__((amdgpu_waves_per_eu(FC ? EVAL_FC_MIN_WAVES : EVAL_MIN_WAVES)))
// workgroup sync words after the key schedules: [0] parent-run counter, [1]
// node-proof counter (frontier-cache hits), [8, 40) "child seeds stored" bitmap
// of the workgroup's parents (<= 16 waves x 64 parents per wave)
#define EVAL_SYNC_WORDS 40
#define EVAL_LDS_BYTES (AES_PERM_LDS_WORDS * 4 + 2 * 64 * 11 * 16 + 4 * EVAL_SYNC_WORDS)
// GEN: the general level (the root level, which writes the root sum instead
// of parent payload differences, and the last level, which emits the
// truncated out shares, with their field multiplications for grouped
// truncations); the interior levels (all others: 30 of C2's 32, 31 of C5's)
// run an instantiation without that code, whose block loop then needs fewer
// scalar registers (no spills of uniform flags into VGPR lanes).  FC: the
// frontier cache's convert-seed staging, parent-payload recompute and fused
// proofs are compiled in (only at a call's last level, so always with GEN);
// the plain instantiation carries none of it (the uniform branches cost 2.5 %
// at C2).
// SPLIT: a small level's parents split into block-range items (AesArgs::split;
// never with FC); a separate instantiation so the other levels' kernels carry
// none of its bookkeeping (in the plain kernel it quadrupled the SGPR spills).
template <class F, bool GEN, bool FC, bool SPLIT = false>
__global__ __launch_bounds__(64 * EVAL_WAVES) EVAL_VGPR_ATTR
void k_eval_aes(McParams p, Planes pl, AesArgs a) {
    typedef typename F::E E;
    // dynamic LDS (EVAL_LDS_BYTES): with a static size the compiler derives
    // the occupancy from it and ignores the VGPR cap of EVAL_VGPR_ATTR
    extern __shared__ uint4 eval_lds[];
    uint32_t* T = (uint32_t*)eval_lds;
    uint4* RKE = eval_lds + AES_PERM_LDS_WORDS / 4;
    uint4* RKC = RKE + 64 * 11;
    uint32_t* next_parent = (uint32_t*)(RKC + 64 * 11);  // the workgroup's parent-run counter
    uint32_t* next_proof = next_parent + 1;               // fused proofs: next node (workgroup ordinal)
    uint32_t* parent_done = next_parent + 8;              // fused proofs: parents whose child seeds are stored
    // the T-table lookups use the v_perm result as the absolute LDS address
    // (aes.hpp lds_read_asm): the table must start at LDS address 0
    if ((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint4*)eval_lds != 0u) __builtin_trap();

    const int S = pl.stride;
    const int S_in = FC ? a.in_stride : S;  // cs_in / fr_w_in
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = blockIdx.x * 64 + lane;
    const uint32_t lb = (uint32_t)r * 4u;
    {
        // the two key schedules' 44 words per report: every wave's loads issued
        // first (one HBM round trip per workgroup, not three), the table filled
        // while they are in flight, then the words stored
        uint32_t* ke = (uint32_t*)RKE;
        uint32_t* kc = (uint32_t*)RKC;
        constexpr int KR = (44 + EVAL_WAVES - 1) / EVAL_WAVES;
        uint32_t xe[KR], xc[KR];
#pragma unroll
        for (int j = 0; j < KR; j++) {
            const int i = wave + j * EVAL_WAVES;
            if (i < 44) {
                xe[j] = pld(pl.rk_ext + (size_t)i * S, lb);
                xc[j] = pld(pl.rk_conv + (size_t)i * S, lb);
            }
        }
        aes_perm_fill(T, threadIdx.x, 64 * EVAL_WAVES);
#pragma unroll
        for (int j = 0; j < KR; j++) {
            const int i = wave + j * EVAL_WAVES;
            if (i < 44) {
                ke[lane * 44 + i] = aes_perm_key_word(i, xe[j]);
                kc[lane * 44 + i] = aes_perm_key_word(i, xc[j]);
            }
        }
    }
    // words [8, 40): the fused-proof bitmap (FC) or, with split parents, each
    // parent's first element whose block a lane flagged (split_first below)
    if (threadIdx.x < EVAL_SYNC_WORDS) next_parent[threadIdx.x] = (SPLIT && threadIdx.x >= 8) ? ~0u : 0u;
    __syncthreads();
    const int aes_waves = a.aes_waves;
    // Proof waves: node proofs of level - 1 (children seeds from cs_in), then
    // they help with the parents; with no proofs to do (level 0, a frontier-
    // cache hit) they walk parents from the start.  No wave returns early: a
    // cache hit's fused proofs below take nodes from every wave (and the A/B
    // barrier schedule ends with a workgroup barrier).
    if (wave >= aes_waves && a.pv_nodes > 0 && !(a.dbg_skip & 1)) {
        if (a.proof_prio == 1) __builtin_amdgcn_s_setprio(1);
        if (a.proof_prio == 2) __builtin_amdgcn_s_setprio(2);
        const int nbeg = (blockIdx.y * (EVAL_WAVES - aes_waves) + (wave - aes_waves)) * a.pv_npw;
        const int nend = min(nbeg + a.pv_npw, a.pv_nodes);
        const int pl_ = a.pv_level;
        uint32_t* ohg = a.pv_onehot + (size_t)blockIdx.x * a.oh_gstride;  // tile group of these 64 reports
        const uint32_t lt = (uint32_t)lane * 4u;
        uint32_t pcw[8];
#pragma unroll
        for (int j = 0; j < 8; j++) pcw[j] = pld(pl.cw_proof + ((size_t)pl_ * 8 + j) * S, lb);
        for (int node = nbeg; node < nend; node++) {
            uint32_t sd[4];
#pragma unroll
            for (int i = 0; i < 4; i++) sd[i] = pld(a.cs_in + ((size_t)node * 5 + i) * S_in, lb);
            const uint32_t t = pld(a.cs_in + ((size_t)node * 5 + 4) * S_in, lb);
            node_proof_one<FC>(a.np, a.np_f, p.bits, pl_, a.pv_path_bytes, sd, a.pv_child_path + node * 8, t, pcw,
                           [&](int j, uint32_t w) { pst(ohg + ((size_t)node * 8 + j) * a.bin_rstride, lt, w); });
        }
        if (a.proof_prio) __builtin_amdgcn_s_setprio(0);
        // then help with this workgroup's parents (below)
    }
    // Parents of this workgroup: [wp0, wp1), claimed in runs of `run` by
    // every wave through an LDS counter: the proof waves join once their
    // proofs are done, so no wave idles while another still has parents.
    const int wp0 = blockIdx.y * a.par_waves * a.ppw;
    const int wp1 = min(wp0 + a.par_waves * a.ppw, SPLIT ? a.n_parents * a.split : a.n_parents);  // items
    // Frontier-cache hit (FC, fuse_proofs == 1): THIS level's node proofs
    // (vidpf.py:366-380, :321-323) of the workgroup's children, overlapped with
    // its parents' AES.  The AES waves [0, aes_waves) walk the parents; a wave
    // that has stored a parent's child seeds and control bits marks the parent
    // in parent_done (release, workgroup scope).  The proof waves take the
    // children in order through next_proof and wait (acquire) for their
    // parent's mark; AES waves that run out of parents join them.  So some
    // waves run the LDS-bound AES while others run the VALU-bound Keccak: with
    // one workgroup per CU (150 KiB of LDS) the two pipes otherwise take turns
    // (AES of every parent, barrier, proofs).  The host sizes the split by the
    // two kinds' work per parent.  fuse_proofs == 3 (A/B only): the barrier
    // schedule.  (Taking ready nodes inside the parent loop instead keeps the
    // loop's state live across the Keccak: 74 spilled VGPRs, 769 scratch loads.)
    const int pn_beg = 2 * wp0, pn_end = 2 * wp1;  // this workgroup's child nodes
    const bool fuse_ovl = FC && a.fuse_proofs == 1;
    auto parent_marked = [&](int q) -> bool {
        const uint32_t w = __hip_atomic_load(parent_done + (q >> 5), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        return (__builtin_amdgcn_readfirstlane(w) >> (q & 31)) & 1u;
    };
    auto claim_node = [&]() -> int {
        uint32_t o = 0;
        if (lane == 0) o = atomicAdd(next_proof, 1u);
        return pn_beg + (int)__builtin_amdgcn_readfirstlane(o);
    };
    auto node_proof_at = [&](int node) {
        if (a.dbg_skip & 2) return;  // timing knob: no parents were evaluated
        if (fuse_ovl)
            while (!parent_marked((node - pn_beg) >> 1)) __builtin_amdgcn_s_sleep(2);
        const int l = a.level;
        uint32_t* ohg = a.cur_onehot + (size_t)blockIdx.x * a.oh_gstride;
        const uint32_t lt = (uint32_t)lane * 4u;
        uint32_t pcw[8];
#pragma unroll
        for (int j = 0; j < 8; j++) pcw[j] = pld(pl.cw_proof + ((size_t)l * 8 + j) * S, lb);
        uint32_t sd[4];
#pragma unroll
        for (int i = 0; i < 4; i++) sd[i] = pld(a.cs_out + ((size_t)node * 5 + i) * S, lb);
        const uint32_t t = pld(a.cs_out + ((size_t)node * 5 + 4) * S, lb);
        node_proof_one<FC>(a.np, a.np_f, p.bits, l, a.cur_path_bytes, sd, a.cur_child_path + node * 8, t, pcw,
                       [&](int j, uint32_t w) { pst(ohg + ((size_t)node * 8 + j) * a.bin_rstride, lt, w); });
    };
    if (a.dbg_skip & 2) goto aes_done;
    if (fuse_ovl && wave >= aes_waves) goto aes_done;  // proof waves of a hit
    {
    if (a.aes_prio == 1) __builtin_amdgcn_s_setprio(1);
    if (a.aes_prio == 2) __builtin_amdgcn_s_setprio(2);
    const int l = a.level;
    const int vl = p.value_len;
    const int wl = vl * F::W32;
    const AesPerm TL{T, 4u * (uint32_t)(lane & 31), 128u + 4u * (uint32_t)(lane & 31)};
    const RkLds rke{RKE + lane * 11};
    const RkLds rkc{RKC + lane * 11};

    uint32_t scw[4];
#pragma unroll
    for (int i = 0; i < 4; i++) scw[i] = pld(pl.cw_seed + ((size_t)l * 4 + i) * S, lb);
    const uint32_t ccw = pld(pl.cw_ctrl + (size_t)l * S, lb);
    const uint32_t* wcw = pl.cw_w + (size_t)l * wl * S;

    // Split parents (AesArgs::split, small levels; never FC): pass 0 runs the
    // items.  A block range that meets a candidate >= p (or the test hook's
    // block) does not run the exact stream itself -- a rejection shifts every
    // later element, including other items' ranges, which may already be
    // stored -- but records its first element in split_first; after a
    // workgroup barrier, pass 1 re-evaluates each flagged parent with the
    // exact next_vec stream from that element to the end, overwriting.
    // (Both children of a parent and all its items are in this workgroup: the
    // host gives a split level one workgroup per report group.)
    const int K = SPLIT ? a.split : 1;
    constexpr int npass = SPLIT ? 2 : 1;
    const int pb = wp0 / K, pe = (wp1 + K - 1) / K;  // parents of this workgroup
    uint32_t* const split_first = parent_done;
    for (int pass = 0; pass < npass; pass++) {
    if (pass == 1) __syncthreads();  // every item of pass 0 is stored (workgroup fence + barrier)
    const int run = pass ? 1 : max(1, a.ppw / 8);
    const int pend = pass ? pe : wp1;
    auto claim = [&]() -> int {
        uint32_t o = 0;
        if (pass == 0) {
            if (lane == 0) o = atomicAdd(next_parent, (uint32_t)run);
            return wp0 + (int)__builtin_amdgcn_readfirstlane(o);
        }
        for (;;) {  // pass 1: the next flagged parent
            if (lane == 0) o = atomicAdd(next_parent + 1, 1u);
            const int q = pb + (int)__builtin_amdgcn_readfirstlane(o);
            if (q >= pe || __builtin_amdgcn_readfirstlane(split_first[q - pb]) < (uint32_t)p.value_len) return q;
        }
    };
    int rbeg = claim();
    if (rbeg >= pend) continue;
    int rend = min(rbeg + run, pend);
    // Parent seed / control bit, software-pipelined one parent ahead so the
    // HBM latency of the child-seed planes hides under the previous parent's
    // AES work.
    auto load_parent = [&](int item, uint32_t* ps, uint32_t& pctrl) {
        const int pi = (K > 1 && !pass) ? item / K : item;
        if (l == 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) ps[i] = pld(pl.key + (size_t)i * S, lb);
            pctrl = a.agg_id;
        } else {
            const int pn = a.parent_node[pi];
#pragma unroll
            for (int i = 0; i < 4; i++) ps[i] = pld(a.cs_in + ((size_t)pn * 5 + i) * S_in, lb);
            pctrl = pld(a.cs_in + ((size_t)pn * 5 + 4) * S_in, lb);
        }
    };
    uint32_t nps[4], npctrl;
    load_parent(rbeg, nps, npctrl);
    for (int item = rbeg; item >= 0;) {
        const int pi = (K > 1 && !pass) ? item / K : item;  // parent
        const int kp = pass ? 1 : (K > 1 ? item - pi * K : 0);  // its block range (pass 1: no next seeds)
        constexpr int EPB_ = F::W32 == 2 ? 2 : 1;  // elements per block
        const int e_lo = pass ? (int)__builtin_amdgcn_readfirstlane(split_first[pi - pb]) : kp * a.split_blocks * EPB_;
        const int e_hi = (K > 1 && !pass) ? min(vl, e_lo + a.split_blocks * EPB_) : vl;
        bool deferred = false;  // pass 0 of a split parent met a suspicious block: pass 1 redoes it
        // The key schedules are re-read from LDS (one ds_read_b128 per round):
        // without the barrier the compiler hoists all 22 reads out of the loop
        // and pins 88 VGPRs.
        asm volatile("" ::: "memory");
        uint32_t ps[4] = {nps[0], nps[1], nps[2], nps[3]};
        const uint32_t pctrl = npctrl;
        // next item: the rest of this run, else a new run
        int nxt = item + 1;
        if (nxt == rend) {
            rbeg = claim();
            rend = min(rbeg + run, pend);
            nxt = rbeg < pend ? rbeg : -1;
        }
        if (nxt >= 0) load_parent(nxt, nps, npctrl);
        if constexpr (FC) {
            if (a.recompute_wp) {
                // frontier-cache hit: ps holds this parent's cached convert seed; its payload
                // and its seed (into ps) from the convert stream
                const uint32_t pcv[4] = {ps[0], ps[1], ps[2], ps[3]};
                parent_payload<F>(TL, rkc, pcv, pctrl, pl.cw_w + (size_t)(l - 1) * wl * S, S, r, e_lo, e_hi, a.wp_buf,
                                  pi * vl, a.force_slow_blk, ps);
                // the children's loop below reads these elements back (same lanes)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        // extend: block 0 -> left child, block 1 -> right child (one paired
        // AES call), correct, then both children's convert seed blocks.
        uint32_t cs0[4], cs1[4], ns0[4], ns1[4];
#if MASTIC_CTR_GROUPS
        {
            // both extend blocks share the parent seed (aes.hpp counter groups)
            AesCtrGroup gp;
            const uint32_t* const sd[1] = {ps};
            const uint32_t ch[1] = {0u};
            AesCtrGroup* const gi[1] = {&gp};
            ctr_group_init<1>(TL, rke, sd, ch, gi);
            const AesCtrGroup* const gg[2] = {&gp, &gp};
            const uint32_t* const sd2[2] = {ps, ps};
            const uint32_t cv[2] = {0u, 1u};
            uint32_t* const ov[2] = {cs0, cs1};
            ctr_blocks_n<2>(TL, rke, gg, sd2, cv, ov);
        }
#else
        fixed_key_block2(TL, rke, ps, 0u, ps, 1u, cs0, cs1);
#endif
        uint32_t tc0 = cs0[0] & 1u, tc1 = cs1[0] & 1u;
        cs0[0] &= ~1u;
        cs1[0] &= ~1u;
        if (pctrl) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                cs0[i] ^= scw[i];
                cs1[i] ^= scw[i];
            }
            tc0 ^= ccw & 1u;
            tc1 ^= (ccw >> 1) & 1u;
        }
#if MASTIC_CTR_GROUPS
        // each child's convert stream (next seed: counter 0, payload blocks:
        // counters 1, 2, ...) is one counter group per 256 counters
        AesCtrGroup g0, g1;
        uint32_t g_hi = 0;  // counter bits above 7 of the groups (uniform)
        const uint32_t* const csd[2] = {cs0, cs1};
        auto init_groups = [&](uint32_t hi) {
            const uint32_t ch2[2] = {hi, hi};
            AesCtrGroup* const gi[2] = {&g0, &g1};
            ctr_group_init<2>(TL, rkc, csd, ch2, gi);
            g_hi = hi;
        };
        const AesCtrGroup* const gg[2] = {&g0, &g1};
        init_groups(0u);
        if (kp == 0) {
            const uint32_t cv[2] = {0u, 0u};
            uint32_t* const ov[2] = {ns0, ns1};
            ctr_blocks_n<2>(TL, rkc, gg, csd, cv, ov);
        }
#else
        if (kp == 0) fixed_key_block2(TL, rkc, cs0, 0u, cs1, 0u, ns0, ns1);
#endif
        if constexpr (FC) {
            if (a.cache_out) {
                // the last level's children as frontier-cache nodes: convert seed, control bit
                const int CS = a.cache_stride;
                const size_t n0 = (size_t)(2 * pi) * 5, n1 = n0 + 5;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    pst(a.cache_out + (n0 + i) * CS, lb, cs0[i]);
                    pst(a.cache_out + (n1 + i) * CS, lb, cs1[i]);
                }
                pst(a.cache_out + (n0 + 4) * CS, lb, tc0);
                pst(a.cache_out + (n1 + 4) * CS, lb, tc1);
            }
        }
        if (kp == 0) {
            const size_t n0 = (size_t)(2 * pi) * 5, n1 = n0 + 5;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                pst(a.cs_out + (n0 + i) * S, lb, ns0[i]);
                pst(a.cs_out + (n1 + i) * S, lb, ns1[i]);
            }
            pst(a.cs_out + (n0 + 4) * S, lb, tc0);
            pst(a.cs_out + (n1 + 4) * S, lb, tc1);
        }
        const int ce0 = a.child_exp[2 * pi], ce1 = a.child_exp[2 * pi + 1];
        const int pf0 = GEN ? a.child_pfx[2 * pi] : -1, pf1 = GEN ? a.child_pfx[2 * pi + 1] : -1;
        const int row = 1 + p.output_len;
        E acc0 = F::zero(), acc1 = F::zero(), coef = F::from_u64(1);
        // Element e of both children: payload correction, frontier payloads,
        // the parent's payload difference (or the root sum), out shares.
        uint32_t* const payg = a.payload + (size_t)blockIdx.x * a.pay_gstride;  // tiled group
#ifdef MASTIC_EXPERIMENT_KNOBS
        // timing experiments (results wrong): 8 = no frontier-payload stores,
        // 16 = no parent-payload loads, 32 = no payload-difference stores
        const bool x_fr = !(a.dbg_skip & 8), x_diff = !(a.dbg_skip & 32);
#else
        constexpr bool x_fr = true, x_diff = true;
#endif
        auto emit = [&](int e, E x0, E x1, E cw, E wp) {
            if (tc0) x0 = F::add(x0, cw);
            if (tc1) x1 = F::add(x1, cw);
            if (x_fr && ce0 >= 0) pl_store<F>(a.fr_w_out, ce0 * vl + e, S, r, x0);
            if (x_fr && ce1 >= 0) pl_store<F>(a.fr_w_out, ce1 * vl + e, S, r, x1);
            if (GEN && l == 0) {
                pl_store<F>(pl.rootsum, e, S, r, F::add(x0, x1));
            } else if (!x_diff) {
                if (F::is_zero(F::sub(F::sub(wp, x0), x1))) a.out[0] = 0u;  // keep the work, drop the store
            } else {
                // tiled (AbsorbArgs): word m of this group's 64 reports = one row
                pl_store_rows<F>(payg, pi * vl + e, a.bin_rstride, (uint32_t)lane * 4u, F::sub(F::sub(wp, x0), x1));
            }
            if (GEN && (pf0 >= 0 || pf1 >= 0)) {
                // truncated out share, negated for the helper (vidpf.py:259, mastic.py:311-314)
                if (e == 0) {
                    if (pf0 >= 0) pl_store<F>(a.out, pf0 * row, a.out_stride, r, a.agg_id ? F::neg(x0) : x0);
                    if (pf1 >= 0) pl_store<F>(a.out, pf1 * row, a.out_stride, r, a.agg_id ? F::neg(x1) : x1);
                } else if (e - 1 < p.tlimit) {
                    const int m = e - 1;
                    const int g = m % p.tgroup;
                    if (p.tgroup == 1) {
                        acc0 = x0;
                        acc1 = x1;
                    } else {
                        coef = g == 0 ? F::from_u64(1) : F::add(coef, coef);
                        acc0 = F::add(g == 0 ? F::zero() : acc0, F::mul(coef, x0));
                        acc1 = F::add(g == 0 ? F::zero() : acc1, F::mul(coef, x1));
                    }
                    if (g == p.tgroup - 1) {
                        const int o = 1 + m / p.tgroup;
                        if (pf0 >= 0) pl_store<F>(a.out, pf0 * row + o, a.out_stride, r, a.agg_id ? F::neg(acc0) : acc0);
                        if (pf1 >= 0) pl_store<F>(a.out, pf1 * row + o, a.out_stride, r, a.agg_id ? F::neg(acc1) : acc1);
                    }
                }
            }
        };
        auto load_cw = [&](int e) { return pl_load<F>(wcw, e, S, r); };
        const uint32_t* wpb = a.fr_w_in;
        if constexpr (FC) wpb = a.recompute_wp ? a.wp_buf : a.fr_w_in;
        // level 0: the root's "parent payload" planes are zeroed by the host
        // (no branch, no zero-initialised registers in the block loop)
#ifdef MASTIC_EXPERIMENT_KNOBS
        const bool x_wp = !(a.dbg_skip & 16);
        auto load_wp = [&](int e) { return x_wp ? pl_load<F>(wpb, pi * vl + e, S, r) : F::from_u64((uint64_t)e); };
#else
        auto load_wp = [&](int e) { return pl_load<F>(wpb, pi * vl + e, S, r); };
#endif
        int e_fast = e_lo;  // elements completed by the fast path
#if MASTIC_EMIT_WAIT
        // the same before the block loop: the next parent's prefetched seed
        // and this parent's child-seed stores are long done; without it the
        // waitcnt pass keeps a vmcnt wait in the loop header (every block)
        __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
        if constexpr (FC) {
            if (fuse_ovl && lane == 0) {
                // the child seeds / control bits above are stored: their proofs may start
                const int q = pi - wp0;
                __hip_atomic_fetch_or(parent_done + (q >> 5), 1u << (q & 31), __ATOMIC_RELEASE,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        {
            // Fast path: block b (counter b + 1) of each child's convert stream
            // holds Field64 candidates 2b and 2b + 1, or Field128 candidate b
            // (vdaf_poc next_vec after next(16)).  Speculate that no candidate
            // is rejected: one paired AES call per block index, straight-line.
            // A candidate >= p has its top word 0xffffffff (probability 2^-32
            // for Field64, ~2^-59 for Field128); if any lane of the wave sees
            // such a word among the elements it is about to use, the exact
            // stream below redoes this parent from that element on (elements
            // before it are unaffected by the rejection).
            constexpr int EPB = F::W32 == 2 ? 2 : 1;  // elements per block
            const int nblk = pass ? 0 : (e_hi + EPB - 1) / EPB;  // pass 1: the exact stream only
            for (int b = e_lo / EPB; b < nblk; b++) {
                asm volatile("" ::: "memory");
                const int e = EPB * b;
                const bool two = EPB == 2 && e + 1 < e_hi;
                const int e1 = two ? e + 1 : e;  // uniform clamp
                const E cwa = load_cw(e), wpa = load_wp(e);
                E cwb = cwa, wpb = wpa;
                if constexpr (EPB == 2) {
                    cwb = load_cw(e1);
                    wpb = load_wp(e1);
                }
                uint32_t o0[4], o1[4];
#if MASTIC_CTR_GROUPS
                {
                    const uint32_t c = (uint32_t)(b + 1);
                    if ((c & ~0xffu) != g_hi) init_groups(c & ~0xffu);
                    const uint32_t cv[2] = {c, c};
                    uint32_t* const ov[2] = {o0, o1};
                    ctr_blocks_n<2>(TL, rkc, gg, csd, cv, ov);
                }
#else
                fixed_key_block2(TL, rkc, cs0, (uint32_t)(b + 1), cs1, (uint32_t)(b + 1), o0, o1);
#endif
                bool sus;
                if constexpr (EPB == 2)
                    sus = (o0[1] == ~0u) | (o1[1] == ~0u) | (two & ((o0[3] == ~0u) | (o1[3] == ~0u)));
                else
                    sus = (o0[3] == ~0u) | (o1[3] == ~0u);
                if (__builtin_expect(__any(sus), 0) || b == a.force_slow_blk) {
                    if (K > 1) {
                        if (lane == 0) atomicMin(split_first + (pi - pb), (uint32_t)e);
                        deferred = true;
                    }
                    break;
                }
                // All of this block's loads (issued before its AES) and the
                // previous block's stores have long completed: say so with one
                // explicit wait.  Otherwise the waitcnt pass, which loses track
                // of the conditionally issued loads, waits for vmcnt(2..3)
                // between the stores below, i.e. for the stores themselves to
                // be acknowledged, several times per block.
#if MASTIC_EMIT_WAIT
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt / lgkmcnt untouched
#endif
                emit(e, F::from_words(o0), F::from_words(o1), cwa, wpa);
                if constexpr (EPB == 2) {
                    if (two) emit(e + 1, F::from_words(o0 + 2), F::from_words(o1 + 2), cwb, wpb);
                }
                e_fast = e + 1 + (two ? 1 : 0);
            }
        }
        if (e_fast < e_hi && !deferred) {
            // exact next_vec streams (rejection sampling), element by element
            // from the stream's start (a rejection shifts every later element)
            // up to e_hi, emitting from e_fast on; elements before it were
            // emitted by the fast path
            typename EvalStream<F, false>::type st0, st1;
            st0.init(cs0);
            st1.init(cs1);
            constexpr int G = EvalStream<F, false>::type::GROUP;
            for (int e0 = 0; e0 < e_hi; e0 += G) {
                asm volatile("" ::: "memory");
                st0.refill(st1, e_hi - e0, TL, rkc);
#pragma unroll
                for (int i = 0; i < G; i++) {
                    const int e = e0 + i;
                    if (e >= e_hi) break;
                    const E x0 = st0.next(TL, rkc);
                    const E x1 = st1.next(TL, rkc);
                    if (e >= e_fast) emit(e, x0, x1, load_cw(e), load_wp(e));
                }
            }
        }
        item = nxt;
    }
    }  // pass
    }
aes_done:
    if constexpr (FC) {
        if (a.fuse_proofs) {
            // the nodes nobody has taken yet (overlapped: their parents may still
            // be running; A/B barrier schedule: after every parent is done)
            if (!fuse_ovl) __syncthreads();
#pragma unroll 1
            for (int node = claim_node(); node < pn_end; node = claim_node()) node_proof_at(node);
        }
    }
}

// ------------------------------------------------------------- node proofs
// TurboSHAKE128(seed, dst(ctx, NODE_PROOF), le16(BITS) || le16(l) || path)
// (vidpf.py:366-380), XORed with the proof CW when the node's control bit is
// set (vidpf.py:321-323).  The prefix le16(len(dst)) || dst || u8(16) is
// pre-absorbed (PrefixState); the body plus the domain byte (<= 14 words)
// lands at the uniform fill position f: a switch on f/4 selects a straight-
// line XOR pattern, so no LDS staging and no per-lane indexing is needed.
struct ProofArgs {
    int oh_gstride;      // words per report group of the (tiled) proof buffer
    int bin_rstride;     // words between consecutive words of a report
    int level;
    int n_nodes;
    int npw;             // nodes per wave
    int path_bytes;      // ceil((level + 1) / 8)
    const uint32_t* child_path;  // [n_nodes][8]
    const uint32_t* cs;          // child seeds of this level [node][5]
    uint32_t* onehot;            // [n_nodes * 8]
    const PrefixState* np;       // node-proof prefix state (device memory)
    int f;                       // its fill position
};

__global__ __launch_bounds__(256) void k_node_proof(McParams p, Planes pl, ProofArgs a) {
    const int S = pl.stride;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = blockIdx.x * 64 + lane;
    const uint32_t lb = (uint32_t)r * 4u;
    const int nbeg = (blockIdx.y * 4 + wave) * a.npw;
    if (nbeg >= a.n_nodes) return;
    const int nend = min(nbeg + a.npw, a.n_nodes);
    const int l = a.level;
    uint32_t* ohg = a.onehot + (size_t)blockIdx.x * a.oh_gstride;  // tiled proof buffer of this group
    const uint32_t lt = (uint32_t)lane * 4u;
    uint32_t pcw[8];
#pragma unroll
    for (int j = 0; j < 8; j++) pcw[j] = pld(pl.cw_proof + ((size_t)l * 8 + j) * S, lb);
    for (int node = nbeg; node < nend; node++) {
        uint32_t seed[4];
#pragma unroll
        for (int i = 0; i < 4; i++) seed[i] = pld(a.cs + ((size_t)node * 5 + i) * S, lb);
        const uint32_t t = pld(a.cs + ((size_t)node * 5 + 4) * S, lb);
        node_proof_one(a.np, a.f, p.bits, l, a.path_bytes, seed, a.child_path + node * 8, t, pcw,
                       [&](int j, uint32_t w) { pst(ohg + ((size_t)node * 8 + j) * a.bin_rstride, lt, w); });
    }
}

// ------------------------------------------------------------- binder absorb
// Continues the one-hot (sponge 0) or payload (sponge 1) TurboSHAKE over the
// words one level produced.  Positions are uniform (tracked by the host).
// Level buffers (proofs, payload differences) are TILED, not planes: word m
// of report r sits at  seg + (r / 64) * gstride + m * 64 + r % 64,  so a
// sponge wave (one report group) streams one contiguous region block after
// block, and a level-kernel store of one word for 64 reports is still one
// 256-byte row.
struct AbsorbArgs {
    const uint32_t* seg[2];
    int gstride[2];  // words per report group of each segment (planes: 64)
    int rstride;     // words between consecutive stream words of a report (tiled: 64, planes: stride)
    int nbytes[2];
    int f[2];
    int prio;  // s_setprio of the sponge waves (0..3)
    int dbg;   // timing experiments only (results wrong): 1 no loads, 2 no permutations, 4 neither (sleeps)
    int which0;  // sponge of grid row 0 (0 one-hot, 1 payload): a launch covers which0 .. which0 + gridDim.y - 1
};
MH_D void absorb_setprio(int prio) {
    switch (prio) {
        case 0: break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// The next block's 43 source words are loaded before the current block's
// permutation, so their HBM/L2 latency hides under ~2.3k VALU instructions.
// Blocks whose words are all in range (every block but the first and last of
// a launch) use plain loads: a zero-select right after a load would force a
// vmcnt(0) wait per word.
__global__ __launch_bounds__(256) void k_absorb(Planes pl, AbsorbArgs a) {
    // The sponge chain is the latency-critical path and runs beside the
    // level-eval waves: win every issue arbitration on the shared SIMD.
    absorb_setprio(a.prio);
    const int r = blockIdx.x * 256 + threadIdx.x;
    const int which = a.which0 + (int)blockIdx.y;
    if (r >= pl.stride) return;
    const int nb = a.nbytes[which];
    if (nb == 0) return;
    const int S = pl.stride;
    uint32_t* sp = which == 0 ? pl.sp_onehot : pl.sp_payload;
    const uint32_t* seg = a.seg[which] + (size_t)(r >> 6) * a.gstride[which];  // this wave's tile group
    const uint32_t lb = (uint32_t)r * 4u;
    const uint32_t lt = (uint32_t)(r & 63) * 4u;  // lane offset inside a tile row
    const uint32_t rowb = (uint32_t)a.rstride * 4u;  // bytes between stream words
    KState s;
#pragma unroll
    for (int i = 0; i < 25; i++) s.a[i] = u32x2{pld(sp + (size_t)(2 * i) * S, lb), pld(sp + (size_t)(2 * i + 1) * S, lb)};
    const int f = a.f[which];
    const int q = f >> 2;
    const int sh = f & 3;
    const int off = sh ? 1 : 0;           // window starts one word early when shifted
    const int amt = (32 - 8 * sh) & 31;  // block word j = alignbit(w[j+1], w[j], amt)
    const int nw = (nb + 3) >> 2;
    const int end = f + nb;
    auto load_block = [&](int b, uint32_t* w) {
        const int base = KECCAK_RATE_WORDS * b - q - off;
        if (base >= 0 && base + KECCAK_RATE_WORDS < nw) {
            const __amdgpu_buffer_rsrc_t rs = mh_rsrc(seg + (size_t)base * a.rstride);
            // the row offset is a running SGPR sum made opaque at every step,
            // so the compiler cannot hoist 43 loop-invariant offsets (which it
            // would spill to VGPRs and then waterfall)
            uint32_t so = 0;
#pragma unroll
            for (int j = 0; j < KECCAK_RATE_WORDS + 1; j++) {
                w[j] = pld_so(rs, lt, so);
                so += rowb;
                asm volatile("" : "+s"(so));
            }
        } else {
#pragma unroll
            for (int j = 0; j < KECCAK_RATE_WORDS + 1; j++) {
                const int m = base + j;
                const int mc = m < 0 ? 0 : (m >= nw ? nw - 1 : m);
                w[j] = pld(seg + (size_t)mc * a.rstride, lt);
            }
#pragma unroll
            for (int j = 0; j < KECCAK_RATE_WORDS + 1; j++) {
                const int m = base + j;
                w[j] = (m >= 0 && m < nw) ? w[j] : 0u;
            }
        }
    };
    // one block buffer, next block's loads issued after the XOR (see k_absorb_pair)
    uint32_t cur[KECCAK_RATE_WORDS + 1];
    load_block(0, cur);
    for (int b = 0;; b++) {
        const bool full = end >= KECCAK_RATE * (b + 1);
        const bool more = end > KECCAK_RATE * (b + 1);
#pragma unroll
        for (int j = 0; j < KECCAK_RATE_WORDS; j++) kxor_word(s, j, __builtin_amdgcn_alignbit(cur[j + 1], cur[j], amt));
        if (!full) break;
        asm volatile("" ::: "memory");
        if (more) load_block(b + 1, cur);
#ifdef MASTIC_EXPERIMENT_KNOBS
        if (a.dbg == 3)
            keccak_p12<2>(s);  // A/B only: rolled rounds (small code; same results)
        else
#endif
            keccak_p12(s);
        if (!more) break;
    }
#pragma unroll
    for (int i = 0; i < 25; i++) {
        pst(sp + (size_t)(2 * i) * S, lb, s.a[i].lo);
        pst(sp + (size_t)(2 * i + 1) * S, lb, s.a[i].hi);
    }
}

// Two lanes per sponge (keccak_p12_pair): lane h of report r holds state
// words 2i + h.  Block word j = alignbit(w[j+1], w[j], amt) as above; lane h
// needs the j = 2i + h, i.e. stream words base + h + k, k < 42, which it loads
// itself (the plane offset h*S is part of its per-lane buffer offset).
// Each lane keeps only its own stream words of a block, 2i + h (22 words):
// the word after each, 2i + h + 1, is the partner lane's word i (h = 0) or
// i + 1 (h = 1), fetched with one DPP swap per word when the fill offset is not
// a multiple of 4 (shifted byte image).  22 VGPRs of block buffer instead of
// 42, so the kernel fits 5 waves per SIMD without spills.
#ifndef ABSORB_MIN_WAVES
#define ABSORB_MIN_WAVES 5
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ABSORB_MIN_WAVES)))
void k_absorb_pair(Planes pl, AbsorbArgs a) {
    absorb_setprio(a.prio);
    // (launched with optional dynamic LDS that is never touched: it only caps
    // how many absorb workgroups share a CU, see mastic_ctx::absorb_lds)
    const int h = threadIdx.x & 1;
    const int r = blockIdx.x * (int)(blockDim.x >> 1) + (int)(threadIdx.x >> 1);
    const int which = a.which0 + (int)blockIdx.y;
    if (r >= pl.stride) return;  // both lanes of a pair leave together
    const int nb = a.nbytes[which];
    if (nb == 0) return;
    const int S = pl.stride;
    uint32_t* sp = which == 0 ? pl.sp_onehot : pl.sp_payload;
    const uint32_t* seg = a.seg[which] + (size_t)(r >> 6) * a.gstride[which];  // this wave's tile group
    const uint32_t lbh = ((uint32_t)h * (uint32_t)S + (uint32_t)r) * 4u;  // state plane h of the pair
    const uint32_t lt = (uint32_t)(r & 63) * 4u;                            // lane offset in a tile row
    const uint32_t rowb = (uint32_t)a.rstride * 4u;                          // bytes between stream words
    const uint32_t lth = lt + (uint32_t)h * rowb;                           // ... of the next word for h = 1
    const uint32_t rowb2 = 2u * rowb;                                        // own words are every other word
    KHalf s;
#pragma unroll
    for (int i = 0; i < 25; i++) s.a[i] = pld(sp + (size_t)(2 * i) * S, lbh);
    const int f = a.f[which];
    const int q = f >> 2;
    const int sh = f & 3;
    const int off = sh ? 1 : 0;
    const int amt = (32 - 8 * sh) & 31;
    const int nw = (nb + 3) >> 2;
    const int end = f + nb;
    constexpr int NL = KECCAK_RATE_WORDS / 2 + 1;  // words loaded per lane and block: base + 2k + h, k < 22
    auto load_block = [&](int b, uint32_t* w) {
        const int base = KECCAK_RATE_WORDS * b - q - off;
        if (base >= 0 && base + KECCAK_RATE_WORDS + 1 < nw) {
            const __amdgpu_buffer_rsrc_t rs = mh_rsrc(seg + (size_t)base * a.rstride);
            uint32_t so = 0;  // running opaque row offset, as in k_absorb
#pragma unroll
            for (int k = 0; k < NL; k++) {
                w[k] = pld_so(rs, lth, so);
                so += rowb2;
                asm volatile("" : "+s"(so));
            }
        } else {
            // first / last block of the launch: clamped loads, zero outside
            // [0, nw); the word index is per lane (h), so it goes into the
            // lane offset (the descriptor, from a pointer, must be uniform)
#pragma unroll
            for (int k = 0; k < NL; k++) {
                const int m = base + 2 * k + h;
                const int mc = m < 0 ? 0 : (m >= nw ? nw - 1 : m);
                w[k] = pld(seg, (uint32_t)mc * rowb + lt);
            }
#pragma unroll
            for (int k = 0; k < NL; k++) {
                const int m = base + 2 * k + h;
                w[k] = (m >= 0 && m < nw) ? w[k] : 0u;
            }
        }
    };
    // One block buffer.  Per block: XOR the current block (waits for its
    // loads), THEN issue the next block's loads into the same registers, then
    // permute: the loads in flight during the permutation are exactly the
    // ones the next XOR waits for (vmcnt counts in issue order; loads issued
    // before the XOR would make its wait drain them too and expose the whole
    // memory latency once per block).
    uint32_t cur[NL];
    if (a.dbg == 1 || a.dbg == 4) {
#pragma unroll
        for (int k = 0; k < NL; k++) cur[k] = lt + k;
    } else {
        load_block(0, cur);
    }
    for (int b = 0;; b++) {
        const bool full = end >= KECCAK_RATE * (b + 1);
        const bool more = end > KECCAK_RATE * (b + 1);
#pragma unroll
        for (int i = 0; i < 21; i++) {
            // stream word 2i + h + 1: the partner's word i (h = 0) or i + 1 (h = 1)
            uint32_t nxt = 0u;
            if (sh) {
                const uint32_t x0 = pair_swap(cur[i]), x1 = pair_swap(cur[i + 1]);
                nxt = h ? x1 : x0;
            }
            s.a[i] ^= __builtin_amdgcn_alignbit(nxt, cur[i], amt);
        }
        if (!full) break;
        asm volatile("" ::: "memory");
        if (more && a.dbg != 1 && a.dbg != 4) load_block(b + 1, cur);
        if (a.dbg == 0 || a.dbg == 1) keccak_p12_pair(s, h != 0);
        else if (a.dbg == 4) __builtin_amdgcn_s_sleep(72);  // resident, ~4.6k cycles per block, no VALU
        if (!more) break;
    }
#pragma unroll
    for (int i = 0; i < 25; i++) pst(sp + (size_t)(2 * i) * S, lbh, s.a[i]);
}

// ------------------------------------------------------------- finalize
// payload_check, onehot_check, counter_check, eval_proof (mastic.py:277-306).
struct FinalArgs {
    int agg_id;
    int f_onehot;
    int f_payload;
};

template <class F>
__global__ __launch_bounds__(256) void k_finalize(McParams p, Planes pl, FinalArgs a, const PrefixState* pfx) {
    __shared__ uint32_t V[24 * 256];
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= pl.stride) return;
    const int S = pl.stride;
    uint32_t oh[8], pc[8];
    {
        KState s;
#pragma unroll
        for (int i = 0; i < 25; i++) s.a[i] = u32x2{pl.sp_onehot[(2 * i) * S + r], pl.sp_onehot[(2 * i + 1) * S + r]};
        sponge_pad(s, a.f_onehot, 0x01);
#pragma unroll
        for (int j = 0; j < 8; j++) oh[j] = kword(s, j);
#pragma unroll
        for (int i = 0; i < 25; i++) s.a[i] = u32x2{pl.sp_payload[(2 * i) * S + r], pl.sp_payload[(2 * i + 1) * S + r]};
        sponge_pad(s, a.f_payload, 0x01);
#pragma unroll
        for (int j = 0; j < 8; j++) pc[j] = kword(s, j);
    }
    typename F::E cnt = F::add(pl_load<F>(pl.rootsum, 0, S, r), F::from_u64((uint64_t)a.agg_id));
    // body = onehot_check || counter_check || payload_check
    const int t = threadIdx.x;
    for (int j = 0; j < 8; j++) V[j * 256 + t] = oh[j];
    for (int j = 0; j < F::W32; j++) V[(8 + j) * 256 + t] = F::word(cnt, j);
    for (int j = 0; j < 8; j++) V[(8 + F::W32 + j) * 256 + t] = pc[j];
    KState s;
    int f;
    load_prefix(pfx, PFX_EVAL, s, f);
    f = sponge_absorb_words(s, f, 64 + F::ENC, [&](int m) { return V[m * 256 + t]; });
    sponge_pad(s, f, 0x01);
#pragma unroll
    for (int j = 0; j < 8; j++) pl.eval_proof[j * S + r] = kword(s, j);
}

// ------------------------------------------------------------- FLP randomness
template <class F, class Put>
MH_D void squeeze_elems(KState& s, int count, Put put) {
    sponge_squeeze_vec<F::W32>(
        s, count, [&](const uint32_t* w) { return F::valid(F::from_words(w)); },
        [&](int e, const uint32_t* w) { put(e, F::from_words(w)); });
}

struct FlpArgs {
    int agg_id;
    int level;
};

template <class F>
__global__ __launch_bounds__(256) void k_flp_rand(McParams p, Planes pl, FlpArgs a, const PrefixState* pfx) {
    typedef typename F::E E;
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= pl.stride) return;
    const int S = pl.stride;
    // beta share (get_beta_share, vidpf.py:263-279): w_L0 + w_R0, negated by the helper
    for (int e = 0; e < p.value_len; e++) {
        E x = pl_load<F>(pl.rootsum, e, S, r);
        pl_store<F>(pl.beta, e, S, r, a.agg_id ? F::neg(x) : x);
    }
    KState s;
    int f;
    // query rand: TS(verify_key, dst_alg(ctx, QUERY_RAND), nonce || le16(level))
    load_prefix(pfx, PFX_QUERY, s, f);
    f = sponge_absorb_words(s, f, 18, [&](int m) {
        return m < 4 ? pl.nonce[m * S + r] : (uint32_t)(a.level & 0xffff);
    });
    sponge_pad(s, f, 0x01);
    squeeze_elems<F>(s, p.query_rand_len, [&](int e, E x) { pl_store<F>(pl.qr, e, S, r, x); });
    // proof share: leader from the input share, helper expands its seed
    if (a.agg_id == 0) {
        for (int k = 0; k < p.proof_len * F::W32; k++) pl.proof[(size_t)k * S + r] = pl.lps[(size_t)k * S + r];
    } else {
        load_prefix(pfx, PFX_PROOF_SHARE, s, f);
        f = sponge_absorb_words(s, f, 32, [&](int m) { return pl.seed[m * S + r]; });
        sponge_pad(s, f, 0x01);
        squeeze_elems<F>(s, p.proof_len, [&](int e, E x) { pl_store<F>(pl.proof, e, S, r, x); });
    }
    if (p.joint_rand_len > 0) {
        // part = TS(seed, dst_alg(JOINT_RAND_PART), nonce || encode(beta_share[1:]))
        load_prefix(pfx, PFX_JR_PART, s, f);
        const int mw = p.meas_len * F::W32;
        f = sponge_absorb_words(s, f, 32 + 16 + mw * 4, [&](int m) {
            if (m < 8) return pl.seed[m * S + r];
            if (m < 12) return pl.nonce[(m - 8) * S + r];
            return pl.beta[(size_t)(F::W32 + m - 12) * S + r];
        });
        sponge_pad(s, f, 0x01);
        uint32_t part[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            part[j] = kword(s, j);
            pl.jr_part[j * S + r] = part[j];
        }
        // seed = TS(b'', dst_alg(JOINT_RAND_SEED), part_0 || part_1)
        load_prefix(pfx, PFX_JR_SEED, s, f);
        const bool leader = a.agg_id == 0;
        f = sponge_absorb_words(s, f, 64, [&](int m) {
            const bool own = leader ? (m < 8) : (m >= 8);
            const int j = m & 7;
            return own ? pl.jr_part[j * S + r] : pl.peer[j * S + r];
        });
        sponge_pad(s, f, 0x01);
#pragma unroll
        for (int j = 0; j < 8; j++) pl.jr_seed[j * S + r] = kword(s, j);
        // joint rand = TS(seed, dst_alg(JOINT_RAND), b'').next_vec(JRL)
        load_prefix(pfx, PFX_JR, s, f);
        f = sponge_absorb_words(s, f, 32, [&](int m) { return pl.jr_seed[m * S + r]; });
        sponge_pad(s, f, 0x01);
        squeeze_elems<F>(s, p.joint_rand_len, [&](int e, E x) { pl_store<F>(pl.jr, e, S, r, x); });
    }
}

template <class F>
__global__ __launch_bounds__(256) void k_flp_query(McParams p, Planes pl, FlpConsts<F> c) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= pl.stride) return;
    const int S = pl.stride;
    const bool ok = flp_query<F>(p, c, pl.beta + (size_t)F::W32 * S, pl.proof, pl.qr, pl.jr, pl.verifier, S, r);
    if (!ok) pl.status[r] = -2;  // test point is a root of unity
}

// ------------------------------------------------------------- fold
// agg_share[i] = sum over valid reports of out[i]  (agg_update + merge).
// Workgroup (row, y) sums reports [y * chunk, (y + 1) * chunk) of one output
// element into agg_words[y][row]; with gridDim.y > 1 the per-chunk partials
// are then merged by k_fold_shares.  Four independent accumulators keep four
// loads in flight per lane (a level of a sweep has few rows and ~1M reports:
// one workgroup per row walking all reports was load-latency bound, ~7 ms).
template <class F>
__global__ __launch_bounds__(256) void k_fold(const uint32_t* out, int n, int stride, const uint8_t* valid, int chunk,
                                              uint32_t* agg_words) {
    typedef typename F::E E;
    __shared__ E red[256];
    const int row = blockIdx.x;
    const int r0 = blockIdx.y * chunk;
    const int r1 = min(n, r0 + chunk);
    auto get = [&](int r) {
        const E x = pl_load<F>(out, row, stride, r);
        return (valid && !valid[r]) ? F::zero() : x;
    };
    E a0 = F::zero(), a1 = F::zero(), a2 = F::zero(), a3 = F::zero();
    int r = r0 + (int)threadIdx.x;
    for (; r + 768 < r1; r += 1024) {
        const E x0 = get(r), x1 = get(r + 256), x2 = get(r + 512), x3 = get(r + 768);
        a0 = F::add(a0, x0);
        a1 = F::add(a1, x1);
        a2 = F::add(a2, x2);
        a3 = F::add(a3, x3);
    }
    for (; r < r1; r += 256) a0 = F::add(a0, get(r));
    const E acc = F::add(F::add(a0, a1), F::add(a2, a3));
    agg_words += (size_t)blockIdx.y * gridDim.x * F::W32;
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] = F::add(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        E x = red[0];
        for (int i = 0; i < F::W32; i++) agg_words[(size_t)row * F::W32 + i] = F::word(x, i);
    }
}

// out[e] = sum_s in[s][e] (mod p): merges the agg shares gathered from the
// ranks of a multi-GPU job (RCCL's sum is not GF(p) addition).
template <class F>
__global__ __launch_bounds__(256) void k_fold_shares(const uint32_t* in, int n_shares, int n_elems, uint32_t* out) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= n_elems) return;
    typename F::E acc = F::zero();
    for (int s = 0; s < n_shares; s++) {
        uint32_t w[F::W32];
        for (int i = 0; i < F::W32; i++) w[i] = in[((size_t)s * n_elems + e) * F::W32 + i];
        acc = F::add(acc, F::from_words(w));
    }
    for (int i = 0; i < F::W32; i++) out[(size_t)e * F::W32 + i] = F::word(acc, i);
}

// ------------------------------------------------------------- proof tree
// VIDPF-proof aggregation mode (draft-mouris-cfrg-mastic.md, "Plain
// Heavy-Hitters with VIDPF-Proof Aggregation"): the aggregators compute
// identical eval proofs iff a report is valid, so they compare Merkle trees
// over the batch's eval proofs instead of exchanging every prep share, and
// descend into differing subtrees to isolate invalid reports.  The draft
// leaves the hash unspecified; here a node of two children is
//   XofTurboShake128(b'', dst(ctx, USAGE_PROOF_TREE = 12), left || right).next(32)
// and the last node of an odd level is promoted unchanged.  Nodes are 32-byte
// rows (node-major), levels concatenated leaves first.
__global__ __launch_bounds__(256) void k_proof_tree_leaves(const uint32_t* eval_proof, int n, int stride,
                                                          uint32_t* leaves) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (int j = 0; j < 8; j++) leaves[(size_t)i * 8 + j] = eval_proof[(size_t)j * stride + i];
}

__global__ __launch_bounds__(256) void k_proof_tree_level(const PrefixState* pfx, const uint32_t* in, int n_in,
                                                         uint32_t* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n_out = (n_in + 1) >> 1;
    if (i >= n_out) return;
    const uint32_t* lr = in + (size_t)(2 * i) * 8;  // left || right: 16 consecutive words
    if (2 * i + 1 >= n_in) {
#pragma unroll
        for (int j = 0; j < 8; j++) out[(size_t)i * 8 + j] = lr[j];
        return;
    }
    KState s;
    int f;
    load_prefix(pfx, PFX_TREE, s, f);
    f = sponge_absorb_words(s, f, 64, [&](int m) { return lr[m]; });
    sponge_pad(s, f, 0x01);
    sponge_squeeze_words(s, 8, [&](int j, uint32_t w) { out[(size_t)i * 8 + j] = w; });
}

// ------------------------------------------------------------- decide
// prep_shares_to_prep (mastic.py:320-362) for a batch of report pairs.
// prep share wire: eval_proof || [jr_part] || [verifier]  (mastic.py:543-552)
template <class F>
__global__ __launch_bounds__(256) void k_decide(McParams p, int n, int stride, int weight_check,
                                                const uint8_t* ps0, const uint8_t* ps1, int ps_size,
                                                uint32_t* ver_scratch, const PrefixState* pfx,
                                                uint8_t* msg_out, uint8_t* status_out) {
    typedef typename F::E E;
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const uint8_t* a = ps0 + (size_t)ps_size * r;
    const uint8_t* b = ps1 + (size_t)ps_size * r;
    // status: 1 = valid, 0 = VIDPF verification failed, 2 = FLP verification failed
    uint8_t st = 1;
    for (int i = 0; i < 32; i++)
        if (a[i] != b[i]) st = 0;
    if (st && weight_check) {
        const int jr = p.joint_rand_len > 0 ? 32 : 0;
        const uint8_t* va = a + 32 + jr;
        const uint8_t* vb = b + 32 + jr;
        for (int e = 0; e < p.verifier_len; e++) {
            uint32_t wa[F::W32], wb[F::W32];
            for (int i = 0; i < F::W32; i++) {
                wa[i] = ld_u32_bytes(va + e * F::ENC + 4 * i);
                wb[i] = ld_u32_bytes(vb + e * F::ENC + 4 * i);
            }
            E xa = F::from_words(wa), xb = F::from_words(wb);
            if (!F::valid(xa) || !F::valid(xb)) st = 2;
            pl_store<F>(ver_scratch, e, stride, r, F::add(xa, xb));
        }
        if (st == 1 && !flp_decide<F>(p, ver_scratch, stride, r)) st = 2;
        if (st == 1 && p.joint_rand_len > 0) {
            KState s;
            int f;
            load_prefix(pfx, PFX_JR_SEED, s, f);
            f = sponge_absorb_words(s, f, 64, [&](int m) {
                return m < 8 ? ld_u32_bytes(a + 32 + 4 * m) : ld_u32_bytes(b + 32 + 4 * (m - 8));
            });
            sponge_pad(s, f, 0x01);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                uint32_t w = kword(s, j);
                for (int i = 0; i < 4; i++) msg_out[(size_t)32 * r + 4 * j + i] = (uint8_t)(w >> (8 * i));
            }
        }
    }
    status_out[r] = st;
}

// ------------------------------------------------------------- wire encoding
// Planes -> report-major wire bytes on the device (mastic.py:537-552): row r
// of the output is the concatenation of up to 3 plane segments (seg[k]:
// words[k] planes of stride S), i.e. the prep share eval_proof || [jr_part]
// || [verifier] (encode_vec is little-endian words, the planes' byte order),
// or an out share (encode_vec of the truncated vector).  Consecutive threads
// on consecutive words of a row; a grid-stride loop over the output words (a
// grid's work-items must stay below 2^32, an output may be larger: C2's
// 12,288 x 10k-prefix out shares are 2.5e9 words).
struct RowSegs {
    const uint32_t* seg[3];
    int words[3];
};
__global__ __launch_bounds__(256) void k_gather_rows(RowSegs sg, int n, int stride, uint32_t* out) {
    const size_t row_words = (size_t)sg.words[0] + sg.words[1] + sg.words[2];
    const size_t total = (size_t)n * row_words;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const int r = (int)(i / row_words);
        int k = (int)(i - (size_t)r * row_words);
        int s = 0;
        while (k >= sg.words[s]) {
            k -= sg.words[s];
            s++;
        }
        out[i] = sg.seg[s][(size_t)k * stride + r];
    }
}

// Both aggregators' prep_shares_to_prep + prep_next outcome per report, from
// k_decide's code, the two query statuses and (weight check with joint
// randomness) the joint-rand confirmation of each aggregator
// (mastic.py:364-377): accept = 1 iff all pass.
__global__ __launch_bounds__(256) void k_accept(int n, int stride, int check_jr, const uint8_t* code,
                                                const int32_t* st0, const int32_t* st1, const uint8_t* msg,
                                                const uint32_t* jrs0, const uint32_t* jrs1, uint8_t* accept) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    bool ok = code[r] == 1 && st0[r] == 0 && st1[r] == 0;
    if (check_jr) {
        for (int j = 0; j < 8; j++) {
            const uint32_t m = ld_u32_bytes(msg + (size_t)32 * r + 4 * j);
            ok = ok && m == jrs0[(size_t)j * stride + r] && m == jrs1[(size_t)j * stride + r];
        }
    }
    accept[r] = ok ? 1 : 0;
}

// Test hook (mastic_set_test_sponge_delay): one wave idles `ticks` periods of
// the constant wall clock, holding the stream it is queued on, so the work a
// prep_init queues there afterwards completes late.  No memory access.
__global__ __launch_bounds__(64) void k_spin(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
