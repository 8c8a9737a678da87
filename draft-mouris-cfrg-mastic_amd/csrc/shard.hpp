// Client-side Mastic.shard on the GPU (poc/mastic.py:91-185 with
// Vidpf.gen, poc/vidpf.py:103-211): one lane = one report.  Used to
// synthesise reports at scale (bench) and behind the drop-in `shard`.
// Writes the wire encodings straight into the report buffers.
#pragma once
#include "kernels.hpp"

struct ShardArgs {
    int n;
    int stride;
    const uint8_t* alphas;  // [n][ceil(bits/8)] MSB-first
    const uint8_t* betas;   // [n][meas_len * enc] encoded measurement (beta[1:])
    const uint8_t* nonces;  // [n][16]
    const uint8_t* rands;   // [n][rand_size]
    uint8_t* pub;           // [n][public share]
    uint8_t* in0;           // [n][leader input share]
    uint8_t* in1;           // [n][helper input share]
    // scratch planes
    uint32_t* beta;    // [vl*w32]
    uint32_t* rke;     // [44]
    uint32_t* rkc;     // [44]
    uint32_t* bs;      // [2][vl*w32]  beta shares (joint rand)
    uint32_t* jr;      // [jrl*w32]
    uint32_t* prand;   // [arity*w32]
    uint32_t* vals;    // [arity*P*w32]
    uint32_t* coef;    // [arity*P*w32]
    uint32_t* proof;   // [proof_len*w32]
    uint32_t* hps;     // [proof_len*w32] helper proof share
    uint32_t* misc;    // [32]  nonce(4) | seeds
};

MH_D void st_u32_bytes(uint8_t* p, uint32_t w) {
    p[0] = (uint8_t)w;
    p[1] = (uint8_t)(w >> 8);
    p[2] = (uint8_t)(w >> 16);
    p[3] = (uint8_t)(w >> 24);
}

template <class F>
__global__ __launch_bounds__(256) void k_shard(McParams p, ShardArgs a, const PrefixState* pfx,
                                               FlpConsts<F> fc, const typename F::E* alpha_inv_pows) {
    typedef typename F::E E;
    __shared__ uint32_t T[AES_LDS_WORDS];
    __shared__ uint32_t V[16 * 256];
    aes_lds_fill(T, threadIdx.x, 256);
    __syncthreads();
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= a.n) return;
    const int S = a.stride;
    const int t = threadIdx.x;
    AesLds TL{T + (threadIdx.x & 31)};
    const int vl = p.value_len;
    const int ab = (p.bits + 7) / 8;
    const uint8_t* alpha = a.alphas + (size_t)ab * r;
    const uint8_t* rnd = a.rands + (size_t)mc_rand_size(p) * r;
    const uint8_t* nc = a.nonces + (size_t)16 * r;
    uint8_t* pub = a.pub + (size_t)mc_public_share_size(p) * r;
    const int nctrl = (2 * p.bits + 7) / 8;
    uint32_t* nonce = a.misc;  // planes 0..3

    // beta = [1] || encoded measurement
    pl_store<F>(a.beta, 0, S, r, F::from_u64(1));
    for (int e = 1; e < vl; e++) {
        uint32_t w[F::W32];
        for (int i = 0; i < F::W32; i++) w[i] = ld_u32_bytes(a.betas + ((size_t)r * p.meas_len + e - 1) * F::ENC + 4 * i);
        pl_store<F>(a.beta, e, S, r, F::from_words(w));
    }
    for (int i = 0; i < 4; i++) nonce[i * S + r] = ld_u32_bytes(nc + 4 * i);

    // fixed AES keys for this nonce
    for (int which = 0; which < 2; which++) {
        KState s;
        int f;
        load_prefix(pfx, which == 0 ? PFX_EXT : PFX_CONV, s, f);
        f = sponge_absorb_words(s, f, 16, [&](int m) { return nonce[m * S + r]; });
        sponge_pad(s, f, 0x02);
        uint32_t key[4] = {s.a[0].lo, s.a[0].hi, s.a[1].lo, s.a[1].hi};
        uint32_t rk[44];
        aes128_expand(TL, key, rk);
        uint32_t* dst = which == 0 ? a.rke : a.rkc;
        for (int i = 0; i < 44; i++) dst[i * S + r] = rk[i];
    }
    uint32_t rke_w[44], rkc_w[44];
#pragma unroll
    for (int i = 0; i < 44; i++) {
        rke_w[i] = a.rke[i * S + r];
        rkc_w[i] = a.rkc[i * S + r];
    }
    const RkRegs rke{rke_w}, rkc{rkc_w};
    KState s0;
    int f0;
    load_prefix(pfx, PFX_NODE, s0, f0);

    // ---- Vidpf.gen
    uint32_t seed[2][4];
    for (int i = 0; i < 4; i++) {
        seed[0][i] = ld_u32_bytes(rnd + 4 * i);
        seed[1][i] = ld_u32_bytes(rnd + 16 + 4 * i);
    }
    uint32_t ctrl[2] = {0u, 1u};
    uint32_t ctrl_byte = 0;
    for (int lv = 0; lv < p.bits; lv++) {
        const uint32_t bit = (alpha[lv >> 3] >> (7 - (lv & 7))) & 1u;
        uint32_t ex[2][2][4], tt[2][2];
        for (int ag = 0; ag < 2; ag++)
            for (int c = 0; c < 2; c++) {
                uint32_t b[4];
                fixed_key_block(TL, rke, seed[ag], (uint32_t)c, b);
                tt[ag][c] = b[0] & 1u;
                b[0] &= ~1u;
                for (int i = 0; i < 4; i++) ex[ag][c][i] = b[i];
            }
        uint32_t scw[4];
        for (int i = 0; i < 4; i++) scw[i] = bit ? (ex[0][0][i] ^ ex[1][0][i]) : (ex[0][1][i] ^ ex[1][1][i]);
        const uint32_t cw0 = tt[0][0] ^ tt[1][0] ^ (bit ^ 1u);
        const uint32_t cw1 = tt[0][1] ^ tt[1][1] ^ bit;
        const uint32_t cwk = bit ? cw1 : cw0;
        uint32_t sk[2][4];
        for (int ag = 0; ag < 2; ag++) {
            uint32_t tk = bit ? tt[ag][1] : tt[ag][0];
            for (int i = 0; i < 4; i++) sk[ag][i] = bit ? ex[ag][1][i] : ex[ag][0][i];
            if (ctrl[ag]) {
                for (int i = 0; i < 4; i++) sk[ag][i] ^= scw[i];
                tk ^= cwk;
            }
            ctrl[ag] = tk;
        }
        // convert: next seeds and payload correction word
        ConvStream<F> cs0, cs1;
        cs0.init(sk[0]);
        cs1.init(sk[1]);
        fixed_key_block(TL, rkc, sk[0], 0u, seed[0]);
        fixed_key_block(TL, rkc, sk[1], 0u, seed[1]);
        uint8_t* wdst = pub + nctrl + 16 * p.bits + (size_t)lv * vl * F::ENC;
        for (int e = 0; e < vl; e++) {
            E w0 = cs0.next(TL, rkc);
            E w1 = cs1.next(TL, rkc);
            E wc = F::add(F::sub(pl_load<F>(a.beta, e, S, r), w0), w1);
            if (ctrl[1]) wc = F::neg(wc);
            for (int i = 0; i < F::W32; i++) st_u32_bytes(wdst + e * F::ENC + 4 * i, F::word(wc, i));
        }
        // proof correction word
        const int pb = (lv + 1 + 7) / 8;
        const int rem = lv + 1 - 8 * (pb - 1);
        uint32_t pcw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int ag = 0; ag < 2; ag++) {
            for (int i = 0; i < 4; i++) V[i * 256 + t] = seed[ag][i];
            V[4 * 256 + t] = (uint32_t)p.bits | ((uint32_t)lv << 16);
            for (int w = 0; w < (pb + 3) / 4; w++) {
                uint32_t word = 0;
                for (int k = 0; k < 4; k++) {
                    int bi = 4 * w + k;
                    if (bi < pb) {
                        uint32_t byte = alpha[bi];
                        if (bi == pb - 1) byte &= (0xFF00u >> rem) & 0xFFu;
                        word |= byte << (8 * k);
                    }
                }
                V[(5 + w) * 256 + t] = word;
            }
            KState s = s0;
            int f = sponge_absorb_words(s, f0, 20 + pb, [&](int m) { return V[m * 256 + t]; });
            sponge_pad(s, f, 0x01);
#pragma unroll
            for (int j = 0; j < 8; j++) pcw[j] ^= kword(s, j);
        }
        for (int i = 0; i < 4; i++) st_u32_bytes(pub + nctrl + 16 * lv + 4 * i, scw[i]);
        uint8_t* pdst = pub + nctrl + 16 * p.bits + (size_t)p.bits * vl * F::ENC + 32 * lv;
        for (int j = 0; j < 8; j++) st_u32_bytes(pdst + 4 * j, pcw[j]);
        ctrl_byte |= (cw0 | (cw1 << 1)) << (2 * (lv & 3));
        if ((lv & 3) == 3 || lv == p.bits - 1) {
            pub[lv >> 2] = (uint8_t)ctrl_byte;
            ctrl_byte = 0;
        }
    }

    // ---- FLP randomness and proof
    const uint8_t* prove_seed = rnd + 32;
    const uint8_t* helper_seed = rnd + 64;
    const uint8_t* leader_seed = rnd + 96;
    uint32_t part[2][8];
    if (p.joint_rand_len > 0) {
        // get_beta_share for both aggregators, from the level-0 correction word
        const uint8_t* scw0 = pub + nctrl;
        const uint32_t cc = pub[0] & 3u;
        const uint8_t* wcw0 = pub + nctrl + 16 * p.bits;
        for (int ag = 0; ag < 2; ag++) {
            uint32_t key[4];
            for (int i = 0; i < 4; i++) key[i] = ld_u32_bytes(rnd + 16 * ag + 4 * i);
            ConvStream<F> cst[2];
            uint32_t tcs[2];
            for (int c = 0; c < 2; c++) {
                uint32_t b[4];
                fixed_key_block(TL, rke, key, (uint32_t)c, b);
                uint32_t tc = b[0] & 1u;
                b[0] &= ~1u;
                if (ag) {  // root control bit = agg_id
                    for (int i = 0; i < 4; i++) b[i] ^= ld_u32_bytes(scw0 + 4 * i);
                    tc ^= (cc >> c) & 1u;
                }
                cst[c].init(b);
                tcs[c] = tc;
            }
            for (int e = 0; e < vl; e++) {
                uint32_t w[F::W32];
                for (int i = 0; i < F::W32; i++) w[i] = ld_u32_bytes(wcw0 + e * F::ENC + 4 * i);
                E cw = F::from_words(w);
                E x0 = cst[0].next(TL, rkc);
                E x1 = cst[1].next(TL, rkc);
                if (tcs[0]) x0 = F::add(x0, cw);
                if (tcs[1]) x1 = F::add(x1, cw);
                E sum = F::add(x0, x1);
                pl_store<F>(a.bs + (size_t)ag * vl * F::W32 * S, e, S, r, ag ? F::neg(sum) : sum);
            }
            // part_ag = TS(seed_ag, JOINT_RAND_PART, nonce || encode(beta_share[1:]))
            const uint8_t* sd = ag == 0 ? leader_seed : helper_seed;
            for (int i = 0; i < 8; i++) a.misc[(4 + i) * S + r] = ld_u32_bytes(sd + 4 * i);
            const uint32_t* bsp = a.bs + (size_t)ag * vl * F::W32 * S;
            KState s;
            int f;
            load_prefix(pfx, PFX_JR_PART, s, f);
            f = sponge_absorb_words(s, f, 48 + p.meas_len * F::ENC, [&](int m) {
                if (m < 8) return a.misc[(4 + m) * S + r];
                if (m < 12) return nonce[(m - 8) * S + r];
                return bsp[(size_t)(F::W32 + m - 12) * S + r];
            });
            sponge_pad(s, f, 0x01);
#pragma unroll
            for (int j = 0; j < 8; j++) part[ag][j] = kword(s, j);
        }
        for (int j = 0; j < 8; j++) {
            a.misc[(4 + j) * S + r] = part[0][j];
            a.misc[(12 + j) * S + r] = part[1][j];
        }
        KState s;
        int f;
        load_prefix(pfx, PFX_JR_SEED, s, f);
        f = sponge_absorb_words(s, f, 64, [&](int m) { return a.misc[(4 + m) * S + r]; });
        sponge_pad(s, f, 0x01);
#pragma unroll
        for (int j = 0; j < 8; j++) a.misc[(20 + j) * S + r] = kword(s, j);
        load_prefix(pfx, PFX_JR, s, f);
        f = sponge_absorb_words(s, f, 32, [&](int m) { return a.misc[(20 + m) * S + r]; });
        sponge_pad(s, f, 0x01);
        squeeze_elems<F>(s, p.joint_rand_len, [&](int e, E x) { pl_store<F>(a.jr, e, S, r, x); });
    }
    {
        KState s;
        int f;
        for (int i = 0; i < 8; i++) a.misc[(4 + i) * S + r] = ld_u32_bytes(prove_seed + 4 * i);
        load_prefix(pfx, PFX_PROVE_RAND, s, f);
        f = sponge_absorb_words(s, f, 32, [&](int m) { return a.misc[(4 + m) * S + r]; });
        sponge_pad(s, f, 0x01);
        squeeze_elems<F>(s, p.prove_rand_len, [&](int e, E x) { pl_store<F>(a.prand, e, S, r, x); });
    }
    flp_prove<F>(p, fc, alpha_inv_pows, a.beta + (size_t)F::W32 * S, a.jr, a.prand, a.vals, a.coef, a.proof, S, r);
    {
        KState s;
        int f;
        for (int i = 0; i < 8; i++) a.misc[(4 + i) * S + r] = ld_u32_bytes(helper_seed + 4 * i);
        load_prefix(pfx, PFX_PROOF_SHARE, s, f);
        f = sponge_absorb_words(s, f, 32, [&](int m) { return a.misc[(4 + m) * S + r]; });
        sponge_pad(s, f, 0x01);
        squeeze_elems<F>(s, p.proof_len, [&](int e, E x) { pl_store<F>(a.hps, e, S, r, x); });
    }
    // ---- input shares (mastic.py:516-529)
    uint8_t* o0 = a.in0 + (size_t)mc_input_share_size(p, 0) * r;
    uint8_t* o1 = a.in1 + (size_t)mc_input_share_size(p, 1) * r;
    for (int i = 0; i < 16; i++) {
        o0[i] = rnd[i];
        o1[i] = rnd[16 + i];
    }
    uint8_t* q0 = o0 + 16;
    for (int e = 0; e < p.proof_len; e++) {
        E x = F::sub(pl_load<F>(a.proof, e, S, r), pl_load<F>(a.hps, e, S, r));
        for (int i = 0; i < F::W32; i++) st_u32_bytes(q0 + e * F::ENC + 4 * i, F::word(x, i));
    }
    q0 += (size_t)p.proof_len * F::ENC;
    uint8_t* q1 = o1 + 16;
    for (int i = 0; i < 32; i++) q1[i] = helper_seed[i];
    q1 += 32;
    if (p.joint_rand_len > 0) {
        for (int i = 0; i < 32; i++) q0[i] = leader_seed[i];
        for (int j = 0; j < 8; j++) {
            st_u32_bytes(q0 + 32 + 4 * j, part[1][j]);
            st_u32_bytes(q1 + 4 * j, part[0][j]);
        }
    }
}
