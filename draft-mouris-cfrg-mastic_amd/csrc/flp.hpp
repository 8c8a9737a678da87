// FLP of [BBCGGI19] (vdaf_poc.flp_bbcggi19 at draft-irtf-cfrg-vdaf-13) for the
// five Mastic circuits: query and decide on the aggregator side, prove on the
// client side.  One lane = one report; vectors live in word planes
// [word][stride] so that every access is coalesced across lanes.
//
// Query evaluates each wire polynomial at the test point t through the
// Lagrange basis of the P-th roots of unity,
//     wire_j(t) = sum_k wire_j[k] * L_k(t),  L_k(t) = (t^P - 1) a^k / (P (t - a^k)),
// which equals interpolate-then-evaluate exactly (same polynomial, exact field
// arithmetic) while touching only the CALLS + 1 non-zero wire values.
#pragma once
#include "field.hpp"
#include "params.hpp"

// Element load/store on word planes: word i of element elt at
// plane0 + (elt * W32 + i) * rowstride (rowstride = the plane stride, or the
// tile row stride of the binder buffers).  plane0, elt and rowstride must be
// wave-uniform; lane_bytes is the lane's byte offset in a row.  One buffer
// descriptor per element and the word's row offset in soffset: a 4-word
// Field128 element costs one descriptor (a few SALU) instead of one per word.
template <class F>
MH_D typename F::E pl_load_rows(const uint32_t* plane0, int elt, int rowstride, uint32_t lane_bytes) {
    const __amdgpu_buffer_rsrc_t rs = mh_rsrc(plane0 + (size_t)elt * F::W32 * rowstride);
    const uint32_t rb = (uint32_t)rowstride * 4u;
    uint32_t w[F::W32];
#pragma unroll
    for (int i = 0; i < F::W32; i++) w[i] = pld_so(rs, lane_bytes, (uint32_t)i * rb);
    return F::from_words(w);
}
template <class F>
MH_D void pl_store_rows(uint32_t* plane0, int elt, int rowstride, uint32_t lane_bytes, typename F::E x) {
    const __amdgpu_buffer_rsrc_t rs = mh_rsrc(plane0 + (size_t)elt * F::W32 * rowstride);
    const uint32_t rb = (uint32_t)rowstride * 4u;
#pragma unroll
    for (int i = 0; i < F::W32; i++) pst_so(rs, lane_bytes, (uint32_t)i * rb, F::word(x, i));
}
// r is the lane's report (column) of planes of stride `stride`
template <class F>
MH_D typename F::E pl_load(const uint32_t* plane0, int elt, int stride, int r) {
    return pl_load_rows<F>(plane0, elt, stride, (uint32_t)r * 4u);
}
template <class F>
MH_D void pl_store(uint32_t* plane0, int elt, int stride, int r, typename F::E x) {
    pl_store_rows<F>(plane0, elt, stride, (uint32_t)r * 4u, x);
}

// Field constants needed by the FLP, computed once on the host.
template <class F>
struct FlpConsts {
    typename F::E alpha;      // primitive P-th root of unity
    typename F::E inv_p;      // 1/P
    typename F::E inv2;       // shares_inv = 1/2 (query, num_shares = 2)
    typename F::E offset;     // Sum / Multihot offset as a field element
    typename F::E offset_h;   // offset * inv2
};

// Inputs of gadget call k (1-based): emit(j, x_j) for j < arity.
// m(i) reads the measurement (share) element i, jr(i) joint rand i.
template <class F, class MeasFn, class JrFn, class Emit>
MH_D void flp_call_inputs(const McParams& p, int k, typename F::E shares_inv, MeasFn m, JrFn jr, Emit emit) {
    typedef typename F::E E;
    if (p.gadget == G_MUL) {
        E m0 = m(0);
        emit(0, m0);
        emit(1, m0);
    } else if (p.gadget == G_RANGE2) {
        emit(0, m(k - 1));
    } else {
        int i = k - 1;
        E r = jr(i);
        E rp = r;
        for (int j = 0; j < p.chunk; j++) {
            int idx = i * p.chunk + j;
            E me = idx < p.meas_len ? m(idx) : F::zero();
            emit(2 * j, F::mul(rp, me));
            emit(2 * j + 1, F::sub(me, shares_inv));
            rp = F::mul(rp, r);
        }
    }
}

// Gadget G on inputs x(0..arity).
template <class F, class X>
MH_D typename F::E flp_gadget_eval(const McParams& p, X x) {
    typedef typename F::E E;
    if (p.gadget == G_MUL) return F::mul(x(0), x(1));
    if (p.gadget == G_RANGE2) {
        E a = x(0);
        return F::sub(F::mul(a, a), a);
    }
    E acc = F::zero();
    for (int j = 0; j < p.chunk; j++) acc = F::add(acc, F::mul(x(2 * j), x(2 * j + 1)));
    return acc;
}

// Horner evaluation of the gadget polynomial stored at proof elements
// [arity, arity + deg*(P-1) + 1).
template <class F>
MH_D typename F::E flp_gpoly_eval(const McParams& p, const uint32_t* proof, int stride, int r,
                                  typename F::E x) {
    typedef typename F::E E;
    int glen = p.degree * (p.P - 1) + 1;
    E acc = F::zero();
    for (int i = glen - 1; i >= 0; i--) acc = F::add(F::mul(acc, x), pl_load<F>(proof, p.arity + i, stride, r));
    return acc;
}

// Writes verifier = [v, wire_0(t)..wire_{arity-1}(t), gpoly(t)] into `ver`.
// Returns false when the test point is a root of unity (query aborts).
template <class F>
MH_D bool flp_query(const McParams& p, const FlpConsts<F>& c, const uint32_t* meas, const uint32_t* proof,
                    const uint32_t* qr, const uint32_t* jrand, uint32_t* ver, int stride, int r) {
    typedef typename F::E E;
    auto m = [&](int i) { return pl_load<F>(meas, i, stride, r); };
    auto jr = [&](int i) { return pl_load<F>(jrand, i, stride, r); };
    const bool reduce = p.eval_output_len > 1;
    const E t = pl_load<F>(qr, reduce ? p.eval_output_len : 0, stride, r);

    E tp = t;  // t^P, P a power of two
    for (int s = 1; s < p.P; s <<= 1) tp = F::mul(tp, tp);
    const E one = F::from_u64(1);
    if (F::eq(tp, one)) return false;
    const E tp1 = F::sub(tp, one);

    // wire accumulators live in the verifier planes 1..arity
    E ak = one;  // alpha^k
    {
        E lk = F::mul(F::mul(tp1, c.inv_p), finv<F>(F::sub(t, ak)));
        for (int j = 0; j < p.arity; j++)
            pl_store<F>(ver, 1 + j, stride, r, F::mul(pl_load<F>(proof, j, stride, r), lk));
    }
    E v = F::zero();
    E circ = F::zero();
    for (int k = 1; k <= p.calls; k++) {
        ak = F::mul(ak, c.alpha);
        const E lk = F::mul(F::mul(F::mul(tp1, ak), c.inv_p), finv<F>(F::sub(t, ak)));
        flp_call_inputs<F>(p, k, c.inv2, m, jr, [&](int j, E x) {
            pl_store<F>(ver, 1 + j, stride, r, F::add(pl_load<F>(ver, 1 + j, stride, r), F::mul(x, lk)));
        });
        const E g = flp_gpoly_eval<F>(p, proof, stride, r, ak);
        if (p.circuit == MC_SUM)
            v = F::add(v, F::mul(pl_load<F>(qr, k - 1, stride, r), g));  // out[k-1] = g
        else if (p.circuit == MC_COUNT)
            circ = g;
        else
            circ = F::add(circ, g);  // range check
    }
    if (p.circuit == MC_COUNT) {
        v = F::sub(circ, m(0));
    } else if (p.circuit == MC_SUM) {
        E lo = F::zero(), hi = F::zero();
        for (int i = p.wbits - 1; i >= 0; i--) {
            lo = F::add(F::add(lo, lo), m(i));
            hi = F::add(F::add(hi, hi), m(p.wbits + i));
        }
        E rc = F::sub(F::add(c.offset_h, lo), hi);
        v = F::add(v, F::mul(pl_load<F>(qr, 2 * p.wbits, stride, r), rc));
    } else if (p.circuit == MC_SUMVEC) {
        v = circ;
    } else if (p.circuit == MC_HISTOGRAM) {
        E s = F::neg(c.inv2);
        for (int i = 0; i < p.meas_len; i++) s = F::add(s, m(i));
        v = F::add(F::mul(pl_load<F>(qr, 0, stride, r), circ), F::mul(pl_load<F>(qr, 1, stride, r), s));
    } else {  // MC_MULTIHOT
        E w = F::zero();
        for (int i = 0; i < p.length; i++) w = F::add(w, m(i));
        E rep = F::zero();
        for (int i = p.wbits - 1; i >= 0; i--) rep = F::add(F::add(rep, rep), m(p.length + i));
        E wc = F::sub(F::add(c.offset_h, w), rep);
        v = F::add(F::mul(pl_load<F>(qr, 0, stride, r), circ), F::mul(pl_load<F>(qr, 1, stride, r), wc));
    }
    pl_store<F>(ver, 0, stride, r, v);
    pl_store<F>(ver, 1 + p.arity, stride, r, flp_gpoly_eval<F>(p, proof, stride, r, t));
    return true;
}

// decide on a summed verifier held in planes: v == 0 and G(x) == y.
template <class F>
MH_D bool flp_decide(const McParams& p, const uint32_t* ver, int stride, int r) {
    if (!F::is_zero(pl_load<F>(ver, 0, stride, r))) return false;
    typename F::E y = flp_gadget_eval<F>(p, [&](int j) { return pl_load<F>(ver, 1 + j, stride, r); });
    return F::eq(y, pl_load<F>(ver, 1 + p.arity, stride, r));
}

// prove (client): proof = wire seeds || gadget polynomial, num_shares = 1.
// vals, coef: scratch planes [arity * P] each; alpha_inv_pows: table a^-i, i < P.
template <class F>
MH_D void flp_prove(const McParams& p, const FlpConsts<F>& c, const typename F::E* alpha_inv_pows,
                    const uint32_t* meas, const uint32_t* jrand, const uint32_t* prove_rand,
                    uint32_t* vals, uint32_t* coef, uint32_t* proof, int stride, int r) {
    typedef typename F::E E;
    auto m = [&](int i) { return pl_load<F>(meas, i, stride, r); };
    auto jr = [&](int i) { return pl_load<F>(jrand, i, stride, r); };
    const E one = F::from_u64(1);
    const int P = p.P;
    for (int j = 0; j < p.arity; j++) pl_store<F>(vals, j * P, stride, r, pl_load<F>(prove_rand, j, stride, r));
    for (int k = 1; k <= p.calls; k++)
        flp_call_inputs<F>(p, k, one, m, jr, [&](int j, E x) { pl_store<F>(vals, j * P + k, stride, r, x); });
    // interpolate: coeff_i = (1/P) sum_{k <= calls} y_k a^{-ik}  (y_k = 0 for k > calls)
    for (int j = 0; j < p.arity; j++) {
        for (int i = 0; i < P; i++) {
            E s = F::zero();
            for (int k = 0; k <= p.calls; k++)
                s = F::add(s, F::mul(pl_load<F>(vals, j * P + k, stride, r), alpha_inv_pows[(i * k) & (P - 1)]));
            pl_store<F>(coef, j * P + i, stride, r, F::mul(s, c.inv_p));
        }
    }
    for (int i = 0; i < p.arity; i++) pl_store<F>(proof, i, stride, r, pl_load<F>(prove_rand, i, stride, r));
    const int glen = 2 * P - 1;
    for (int i = 0; i < glen; i++) {
        E s = F::zero();
        int lo = i - (P - 1) > 0 ? i - (P - 1) : 0;
        int hi = i < P - 1 ? i : P - 1;
        if (p.gadget == G_RANGE2) {
            for (int a = lo; a <= hi; a++)
                s = F::add(s, F::mul(pl_load<F>(coef, a, stride, r), pl_load<F>(coef, i - a, stride, r)));
            if (i < P) s = F::sub(s, pl_load<F>(coef, i, stride, r));
        } else {
            int pairs = p.gadget == G_MUL ? 1 : p.chunk;
            for (int q = 0; q < pairs; q++) {
                const int w0 = (2 * q) * P, w1 = (2 * q + 1) * P;
                for (int a = lo; a <= hi; a++)
                    s = F::add(s, F::mul(pl_load<F>(coef, w0 + a, stride, r), pl_load<F>(coef, w1 + i - a, stride, r)));
            }
        }
        pl_store<F>(proof, p.arity + i, stride, r, s);
    }
}
