// Square-root-free ECDSA verify ("twist path"), one lane = one (pubkey, msg32, r, s) tuple.
//
// The reference decompresses a 33-byte key with a field square root (eckey_impl.h:17-35,
// ge_set_xo_var: ~266 modmuls, 11 % of a verify) before secp256k1_ecdsa_verify
// (ecdsa_impl.h:207-275).  Here the key's y is never computed.  With v = x^3 + 7 and w = y_Q the
// key's (unknown) y, the isomorphism (X, Y) -> (X w^2, Y w^3) maps Q to Q_w = (x v, v^2), which is
// rational, onto E_w: y^2 = x^3 + 7 v^3.  The Jacobian formulas never use b, so
//   B = u2 * Q_w     is computed on E_w (GLV, signed odd windows, shared-Z table: ecdsa_lane.h),
//   A = u1 * G       is computed on E itself by a fixed-base comb (no doublings, tables in HBM),
// and B maps back to E as the Jacobian point (X2, Y2, Zb w), Zb = Z2 sigma.  Adding A + B on E
// with Jacobian formulas leaves w only in odd powers, so the reference's final test
//   x(A + B) == r   (ecdsa_impl.h:241-273; also r + n when r < p - n)
// becomes  alpha + w beta == 0  with alpha, beta, K computable without w:
//   U1 = X1 Zb^2 v, U2 = X2 Z1^2, S1 = w s1 with s1 = Y1 Zb^3 v, S2 = Y2 Z1^3, H = U2 - U1,
//   K = Z3^2 = Z1^2 Zb^2 v H^2,
//   alpha = r K - S2^2 - v s1^2 + H^3 + 2 U1 H^2,   beta = 2 S2 s1.
// So the tuple is valid iff gamma = -alpha / beta is THE square root of v the key names: gamma^2
// == v and gamma has the key's parity (compressed), or gamma == y (uncompressed: y^2 == v is
// checked in prep, as ge_is_valid_var does).  A non-residue v (an invalid compressed key) can
// never pass gamma^2 == v.  beta^-1 is batched across tuples (Montgomery's trick in
// ecdsa_tfin_kernel: ~3 mults per tuple plus a shared inversion) instead of one square root each.
// Rare exceptional configurations (A or B at infinity, x(A) == x(B), beta == 0: reachable only by
// adversarial inputs) take an exact fallback: the square root after all, then the plain Jacobian
// sum and the reference's x-test.
#pragma once
#include <stddef.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "ecdsa_lane.h"

namespace bcc {

#ifndef BCC_COMB_BITS
#define BCC_COMB_BITS 16  // 16 windows x 32768 points = 32 MiB of tables (MALL-resident); 15 additions
#endif
constexpr int WC = BCC_COMB_BITS;                 // comb window: 2^(WC-1) odd multiples per window
constexpr int CTAB = 1 << (WC - 1);
constexpr int CTOP = (256 + WC - 1) / WC - 1;     // top window index (19 for WC = 13)
constexpr int CWIN = CTOP + 1;                    // windows
static_assert(WC * CTOP + 1 + (WC - 1) >= 256, "top comb digit must cover bit 255");

// extra ladder-state flags of the twist path (LS_VALID / LS_NEG0 / LS_NEG1 / LS_CORR0 as before)
enum : u32 {
    LS_NEGU1 = 1u << 7,   // u1 was even: the comb runs on n - u1 and A is negated
    LS_U1ZERO = 1u << 8,  // u1 == 0: A is the point at infinity
    LS_COMP = 1u << 9,    // compressed key (02 / 03): the y to match is named by its parity
    LS_PAR = 1u << 10,    // ... and that parity is odd (03)
};

// host-side state of the twist path (the device keeps the same words in wave-blocked scratch)
struct TwistState {
    u32 k[4][4];  // k1 (Q), k2 (lambda Q), u1 words 0..3, u1 words 4..7
    u32 flags;
    fe sigma;     // scale of the Q table's curve relative to E_w
    sc r;
    fe v;         // x^3 + 7
    fe ychk;      // uncompressed keys: y
    BCC_HD u32 kword(int s, int w) const { return k[s][w]; }
    BCC_HD void get_r(sc& o) const { o = r; }
    BCC_HD void get_v(fe& o) const { o = v; }
    BCC_HD void get_y(fe& o) const { o = ychk; }
};

// word li (0..7, 8 == 0) of u1 from the state's slots 2 and 3
template <class ST>
BCC_HD u32 u1_word(const ST& st, int li) {
    return li < 4 ? st.kword(2, li) : li < 8 ? st.kword(3, li - 4) : 0u;
}

// signed odd fixed-window digit of the odd 256-bit u1 at bit position pos (a multiple of WC)
template <class ST>
BCC_HD u32 comb_digit(const ST& st, int pos, bool& neg) {
    const int b = pos + 1, li = b >> 5, sh = b & 31;
    const u32 a = u1_word(st, li), c = u1_word(st, li + 1);
    u32 v = sh ? ((a >> sh) | (c << (32 - sh))) : a;
    v &= (1u << WC) - 1u;
    if (pos == WC * CTOP) {
        neg = false;
        return v;
    }
    const u32 half = 1u << (WC - 1), mask = half - 1u;
    const bool positive = (v & half) != 0;
    neg = !positive;
    return positive ? (v & mask) : (~v & mask);
}

// Host comb tables: xy[((win * CTAB) + i) * 2 + {0, 1}] = affine (2i+1) 2^(WC win) G.
struct GCombArray {
    const fe* xy;
    BCC_HD void get(int win, int i, fe& x, fe& y) const {
        x = xy[((size_t)win * CTAB + i) * 2 + 0];
        y = xy[((size_t)win * CTAB + i) * 2 + 1];
    }
};

// Prep, key half: key parse without a square root and the Q_w table (nothing here depends on
// the signature or the message, so K_tkey can run beside the sighash kernels).  Returns false
// (st.flags = 0) on the reference's pubkey parse failures other than "x^3 + 7 is not a square",
// which the final test catches; else st.flags = LS_VALID | LS_COMP / LS_PAR.
template <class QT>
BCC_HD bool twist_prep_key(u32 tag, const fe& px, const fe& py, QT& qt, TwistState& st) {
    st.flags = 0;
    const bool compressed = (tag == 2u || tag == 3u);
    const bool full = (tag == 4u || tag == 6u || tag == 7u);
    if (!compressed && !full) return false;
    if (!fe_lt_p(px)) return false;
    fe v;
    curve_rhs(v, px);
    u32 flags = LS_VALID;
    if (compressed) {
        flags |= LS_COMP | (tag == 3u ? LS_PAR : 0u);
        st.ychk = fe_zero();
    } else {  // ge_set_xy + ge_is_valid_var, hybrid parity (eckey_impl.h:24-33)
        if (!fe_lt_p(py)) return false;
        if (tag != 4u && (py.v[0] & 1u) != (tag == 7u ? 1u : 0u)) return false;
        fe t;
        fe_sqr(t, py);
        if (!fe_equal(t, v)) return false;
        st.ychk = py;
    }
    st.v = v;
    // Q_w = (x v, v^2): Q on E_w; the table lands on E_w scaled once more by st.sigma
    fe qx, qy;
    fe_mul(qx, px, v);
    fe_sqr(qy, v);
    build_q_table_coz(qx, qy, qt, st.sigma);
    st.flags = flags;
    return true;
}

// Prep, the signature half (after twist_prep_key; `flags` = its st.flags): r / s range checks
// (ecdsa_impl.h:216-222), u2 = r s^-1 and its GLV split, the odd fix-ups.  Nothing here reads the
// message, so the Q ladder (B = u2 Q_w) can run beside the sighash kernels.  Returns false
// (st.flags = 0) when the tuple is rejected outright; *sinv_out (optional) receives s^-1.
BCC_HD bool twist_prep_u2(u32 flags, const sc& r_in, const sc& s_in, const sc* sinv_pre,
                          TwistState& st, sc* sinv_out = nullptr) {
    const u32 N[8] = BCC_N_LIMBS;
    st.flags = 0;
    if (!(flags & LS_VALID)) return false;
    if (u256_is_zero(r_in.v) || u256_is_zero(s_in.v)) return false;
    if (!u256_lt(r_in.v, N) || !u256_lt(s_in.v, N)) return false;
    sc sinv, u2, k1, k2;
    if (sinv_pre) sinv = *sinv_pre;
    else sc_inv(sinv, s_in);
    if (sinv_out) *sinv_out = sinv;
    sc_mul(u2, r_in, sinv);
    // u2 = k1 + lambda k2 for the Q ladder, both halves odd (corrections at the end)
    sc_split_lambda(k1, k2, u2);
    if ((k1.v[4] | k1.v[5] | k1.v[6] | k1.v[7]) != 0) {
        sc_neg(k1, k1);
        flags |= LS_NEG0;
    }
    if ((k2.v[4] | k2.v[5] | k2.v[6] | k2.v[7]) != 0) {
        sc_neg(k2, k2);
        flags |= LS_NEG1;
    }
    for (int i = 0; i < 4; i++) {
        st.k[0][i] = k1.v[i];
        st.k[1][i] = k2.v[i];
    }
    for (int s = 0; s < 2; s++) {
        if ((st.k[s][0] & 1u) == 0) flags |= LS_CORR0 << s;
        st.k[s][0] |= 1u;
    }
    st.flags = flags;
    st.r = r_in;
    return true;
}

// Prep, the message half: u1 = (m mod n) s^-1 for the comb, odd by negation (u1 G = -((n - u1) G),
// so A needs no correction); sets LS_U1ZERO / LS_NEGU1 in *flags and the u1 words k2 (0..3) and
// k3 (4..7).
BCC_HD void twist_prep_u1(const sc& m_in, const sc& sinv, u32* flags, u32 (&k2)[4], u32 (&k3)[4]) {
    const u32 N[8] = BCC_N_LIMBS;
    sc m = m_in, u1;
    if (!u256_lt(m.v, N)) {
        u32 tmp[8];
        u256_sub(tmp, m.v, N);
        for (int i = 0; i < 8; i++) m.v[i] = tmp[i];
    }
    sc_mul(u1, m, sinv);
    if (sc_is_zero(u1)) {
        *flags |= LS_U1ZERO;
        u1.v[0] = 1u;
    } else if ((u1.v[0] & 1u) == 0) {
        sc_neg(u1, u1);
        *flags |= LS_NEGU1;
    }
    for (int i = 0; i < 4; i++) {
        k2[i] = u1.v[i];
        k3[i] = u1.v[4 + i];
    }
}

// Prep, scalar half: both of the above.
BCC_HD bool twist_prep_scalars(u32 flags, const sc& r_in, const sc& s_in, const sc& m_in,
                               const sc* sinv_pre, TwistState& st) {
    sc sinv;
    if (!twist_prep_u2(flags, r_in, s_in, sinv_pre, st, &sinv)) return false;
    twist_prep_u1(m_in, sinv, &st.flags, st.k[2], st.k[3]);
    return true;
}

// Prep: both halves (the rejections of either set st.flags = 0).
template <class QT>
BCC_HD bool twist_prep_lane(u32 tag, const fe& px, const fe& py, const sc& r_in, const sc& s_in,
                            const sc& m_in, const sc* sinv_pre, QT& qt, TwistState& st) {
    if (!twist_prep_key(tag, px, py, qt, st)) return false;
    return twist_prep_scalars(st.flags, r_in, s_in, m_in, sinv_pre, st);
}

// B = u2 Q_w: Strauss over the two GLV halves with shared doublings (the Q slots of
// ladder_accumulate), then the odd-fix corrections.  acc on E_w scaled by sigma; returns inf.
template <class ST, class QT>
BCC_HD bool twist_accumulate_q(const ST& st, const QT& qt, gej& acc) {
    const bool neg0 = (st.flags & LS_NEG0) != 0, neg1 = (st.flags & LS_NEG1) != 0;
    const fe one = fe_one();
    bool inf = false;
    {
        bool ng;
        u32 idx = digit_index(st.kword(0, 0), st.kword(0, 1), st.kword(0, 2), st.kword(0, 3), TOPQ,
                              WQ, TOPQ, ng);
        qt.get((int)idx, 0, acc.x);
        qt.get((int)idx, 2, acc.y);
        if (neg0) fe_neg(acc.y, acc.y);
        acc.z = one;
    }
#pragma unroll 1
    for (int pos = TOPQ; pos >= -1; pos--) {
        if (pos >= 0 && pos != TOPQ && !inf) {
            gej t;
            gej_double(t, acc);
            acc = t;
        }
        if (pos >= 0 && (pos % WQ) != 0) continue;
#pragma unroll 1
        for (int slot = 0; slot < 2; slot++) {
            const bool kneg = slot == 0 ? neg0 : neg1;
            u32 idx;
            bool sneg;
            if (pos >= 0) {
                if (slot == 0 && pos == TOPQ) continue;  // initial value
                bool dneg;
                idx = digit_index(st.kword(slot, 0), st.kword(slot, 1), st.kword(slot, 2),
                                  st.kword(slot, 3), pos, WQ, TOPQ, dneg);
                sneg = dneg ^ kneg;
            } else {
                if (!(st.flags & (LS_CORR0 << slot))) continue;  // per lane
                idx = 0;
                sneg = !kneg;
            }
            fe px, py;
            qt.get_pair((int)idx, slot, px, py);  // (x or beta*x, y)
            if (sneg) fe_neg(py, py);
            acc_add(acc, inf, px, py, one, false);
        }
    }
    return inf;
}

// One GLV half of B (round 5, the latency mode of small rounds): slot 0 accumulates k1 Q over the
// table's (x, y), slot 1 k2 lambda Q over its (beta x, y), each with its own 124 doublings and
// odd-fix correction, so two lanes run the halves side by side and B = B_0 + B_1
// (twist_keyq2_kernel).  The same digits and additions as twist_accumulate_q's slot.  Returns inf.
template <class ST, class QT>
BCC_HD bool twist_accumulate_q_half(const ST& st, const QT& qt, gej& acc, int slot) {
    const bool kneg = (st.flags & (slot == 0 ? LS_NEG0 : LS_NEG1)) != 0;
    const fe one = fe_one();
    bool inf = false;
    {
        bool ng;
        const u32 idx = digit_index(st.kword(slot, 0), st.kword(slot, 1), st.kword(slot, 2),
                                    st.kword(slot, 3), TOPQ, WQ, TOPQ, ng);
        qt.get_pair((int)idx, slot, acc.x, acc.y);
        if (kneg) fe_neg(acc.y, acc.y);
        acc.z = one;
    }
#pragma unroll 1
    for (int pos = TOPQ; pos >= -1; pos--) {
        if (pos >= 0 && pos != TOPQ && !inf) {
            gej t;
            gej_double(t, acc);
            acc = t;
        }
        if (pos >= 0 && ((pos % WQ) != 0 || pos == TOPQ)) continue;
        u32 idx;
        bool sneg;
        if (pos >= 0) {
            bool dneg;
            idx = digit_index(st.kword(slot, 0), st.kword(slot, 1), st.kword(slot, 2),
                              st.kword(slot, 3), pos, WQ, TOPQ, dneg);
            sneg = dneg ^ kneg;
        } else {
            if (!(st.flags & (LS_CORR0 << slot))) continue;  // per lane
            idx = 0;
            sneg = !kneg;
        }
        fe px, py;
        qt.get_pair((int)idx, slot, px, py);
        if (sneg) fe_neg(py, py);
        acc_add(acc, inf, px, py, one, false);
    }
    return inf;
}

// A = u1 G on E by the fixed-base comb: one addition per window, no doublings.  Returns inf.
template <class ST, class GC>
BCC_HD bool twist_accumulate_g(const ST& st, const GC& gc, gej& acc) {
    const fe one = fe_one();
    bool inf = false;
    {
        bool ng;
        u32 idx = comb_digit(st, WC * CTOP, ng);
        gc.get(CTOP, (int)idx, acc.x, acc.y);
        acc.z = one;
    }
#pragma unroll 1
    for (int win = CTOP - 1; win >= 0; win--) {
        bool neg;
        u32 idx = comb_digit(st, WC * win, neg);
        fe px, py;
        gc.get(win, (int)idx, px, py);
        if (neg) fe_neg(py, py);
        acc_add(acc, inf, px, py, one, false);
    }
    if (st.flags & LS_NEGU1) fe_neg(acc.y, acc.y);
    if (st.flags & LS_U1ZERO) inf = true;
    return inf;
}

// The w-free final quantities of A + B (see the header).  A on E, B on E_w scaled by sigma.
// Returns false for the exceptional configurations (x(A) == x(B), beta == 0).
BCC_HD bool twist_combine(const gej& A, const gej& B, const fe& sigma, const fe& v, const sc& r,
                          fe& al, fe& be, fe& K) {
    // ordered so that A and B die early (the ladder kernel runs at <= 128 VGPRs)
    fe zb, zb2, z12, u1, u2, s1, s2, h, hh, t;
    fe_mul(zb, B.z, sigma);
    fe_sqr(zb2, zb);
    fe_sqr(z12, A.z);
    fe_mul(u2, B.x, z12);          // U2 = X2 Z1^2
    fe_mul(t, z12, A.z);
    fe_mul(s2, B.y, t);            // S2 = Y2 Z1^3
    fe_mul(t, A.y, zb2);
    fe_mul(t, t, zb);
    fe_mul(s1, t, v);              // S1 = w s1, s1 = Y1 Zb^3 v
    fe_mul(t, A.x, zb2);
    fe_mul(u1, t, v);              // U1 = X1 Zb^2 v
    fe_sub(h, u2, u1);
    if (fe_is_zero(h)) return false;
    fe_mul(be, s2, s1);
    fe_shl<1>(be, be);             // beta = 2 S2 s1
    if (fe_is_zero(be)) return false;
    fe_sqr(hh, h);
    fe_mul(t, z12, zb2);
    fe_mul(t, t, v);
    fe_mul(K, t, hh);              // K = Z3^2
    fe xr;
    for (int i = 0; i < 8; i++) xr.v[i] = r.v[i];  // r < n < p
    fe_mul(al, xr, K);
    fe_sqr(t, s2);
    fe_sub(al, al, t);
    fe_sqr(t, s1);
    fe_mul(t, t, v);
    fe_sub(al, al, t);
    fe_mul(t, hh, h);
    fe_add(al, al, t);
    fe_mul(t, u1, hh);
    fe_shl<1>(t, t);
    fe_add(al, al, t);             // alpha = r K - S2^2 - v s1^2 + H^3 + 2 U1 H^2
    return true;
}

// gamma = -alpha beta^-1 is the key's y?
BCC_HD bool twist_is_key_y(const fe& al, const fe& binv, const fe& v, const fe& ychk, u32 flags) {
    fe g, g2;
    fe_mul(g, al, binv);
    fe_neg(g, g);
    fe_normalize(g);
    fe_sqr(g2, g);
    if (!fe_equal(g2, v)) return false;
    if (flags & LS_COMP) return (g.v[0] & 1u) == ((flags & LS_PAR) ? 1u : 0u);
    return fe_equal(g, ychk);
}

// The verdict of a normal lane from (alpha, K) and beta^-1: x(R) == r, or x(R) == r + n when
// r < p - n (ecdsa_impl.h:241-273).
BCC_HD int twist_final(const fe& al, const fe& K, const fe& binv, const fe& v, const fe& ychk,
                       u32 flags, const sc& r) {
    if (twist_is_key_y(al, binv, v, ychk, flags)) return 1;
    const u32 PMN[8] = BCC_PMN_LIMBS;
    if (!u256_lt(r.v, PMN)) return 0;
    const u32 N[8] = BCC_N_LIMBS;
    fe nf, t, al2;
    fe_set(nf, N);
    fe_mul(t, K, nf);
    fe_add(al2, al, t);            // (r + n) K - ...
    return twist_is_key_y(al2, binv, v, ychk, flags) ? 1 : 0;
}

// r = a + b, both Jacobian and finite, with the exceptional cases of gej_add_var
// (group_impl.h:388-444): a == b doubles, a == -b gives infinity.
BCC_HD void gej_add_gej(gej& r, bool& inf, const gej& a, const gej& b) {
    fe z22, z12, u1, u2, s1, s2, h, rr, hh, hhh, v, t;
    fe_sqr(z22, b.z);
    fe_sqr(z12, a.z);
    fe_mul(u1, a.x, z22);
    fe_mul(u2, b.x, z12);
    fe_mul(s1, a.y, z22);
    fe_mul(s1, s1, b.z);
    fe_mul(s2, b.y, z12);
    fe_mul(s2, s2, a.z);
    fe_sub(h, u2, u1);
    fe_sub(rr, s2, s1);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr)) {
            gej_double(r, a);
            inf = false;
        } else {
            inf = true;
            r = a;
        }
        return;
    }
    fe_sqr(hh, h);
    fe_mul(hhh, h, hh);
    fe_mul(v, u1, hh);
    fe_mul(t, a.z, b.z);
    fe_mul(r.z, t, h);
    fe_sqr(t, rr);
    fe_sub(t, t, hhh);
    fe_sub(t, t, v);
    fe_sub(r.x, t, v);             // X3 = R^2 - H^3 - 2V
    fe_sub(t, v, r.x);
    fe_mul(t, rr, t);
    fe_mul(hhh, s1, hhh);
    fe_sub(r.y, t, hhh);           // Y3 = R (V - X3) - S1 H^3
    inf = false;
}

// Exact fallback for the exceptional lanes: the key's y by the square root after all (or the
// uncompressed y), B back on E, the plain Jacobian sum and the reference's x-test.
BCC_HD int twist_exceptional(const gej& A, bool ainf, const gej& B, bool binf, const fe& sigma,
                             const fe& v, const fe& ychk, u32 flags, const sc& r) {
    const u32 N[8] = BCC_N_LIMBS;
    fe w;
    if (flags & LS_COMP) {
        if (!fe_sqrt(w, v)) return 0;  // ge_set_xo_var: x^3 + 7 is not a square
        fe_normalize(w);
        if ((w.v[0] & 1u) != ((flags & LS_PAR) ? 1u : 0u)) fe_neg(w, w);
    } else {
        w = ychk;
    }
    if (ainf && binf) return 0;
    gej be = B, R;
    bool rinf = false;
    fe zb;
    fe_mul(zb, B.z, sigma);
    fe_mul(be.z, zb, w);               // B on E: (X2, Y2, Zb w)
    if (binf) R = A;
    else if (ainf) R = be;
    else gej_add_gej(R, rinf, A, be);
    if (rinf) return 0;                // R = infinity (ecdsa_impl.h:225-227)
    fe z2, lhs, xr;
    fe_sqr(z2, R.z);
    for (int i = 0; i < 8; i++) xr.v[i] = r.v[i];
    fe_mul(lhs, xr, z2);
    if (fe_equal(lhs, R.x)) return 1;
    const u32 PMN[8] = BCC_PMN_LIMBS;
    if (!u256_lt(r.v, PMN)) return 0;
    u32 xn[8];
    u256_add(xn, r.v, N);
    for (int i = 0; i < 8; i++) xr.v[i] = xn[i];
    fe_mul(lhs, xr, z2);
    return fe_equal(lhs, R.x) ? 1 : 0;
}

// Status of a lane after the twist ladder.
enum : u32 { TW_REJECT = 0, TW_NORMAL = 1, TW_EXCEPT = 2 };

// Whole verify on one lane (host tests): prep, both accumulations, combine, a per-lane
// inversion instead of the batched one.
template <class QT, class GC>
BCC_HD int ecdsa_verify_twist_lane(u32 tag, const fe& px, const fe& py, const sc& r,
                                   const sc& s, const sc& m, QT& qt, const GC& gc) {
    TwistState st;
    if (!twist_prep_lane(tag, px, py, r, s, m, nullptr, qt, st)) return 0;
    gej A, B;
    const bool binf = twist_accumulate_q(st, qt, B);
    const bool ainf = twist_accumulate_g(st, gc, A);
    fe al, be, K;
    if (binf || ainf || !twist_combine(A, B, st.sigma, st.v, st.r, al, be, K))
        return twist_exceptional(A, ainf, B, binf, st.sigma, st.v, st.ychk, st.flags, st.r);
    fe binv;
    fe_inv(binv, be);
    return twist_final(al, K, binv, st.v, st.ychk, st.flags, st.r);
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host-only form of B = u2 Q_w for one lane (the engine's host verification path): a lone CPU
// thread pays for every addition, so the GLV halves are recoded as width-5 wNAF (digits odd in
// [-15, 15] or 0: the same 8-entry table, ≈43 additions instead of the SIMT path's 63 + 2 fixed-
// window ones, and no odd-fix corrections), the variable-time recoding the reference uses on the
// CPU too (ecmult_impl.h:155-199, 531-558).  `k` are the raw halves (|k| < 2^128, their signs in
// LS_NEG0 / LS_NEG1).  Same result as twist_accumulate_q; returns inf.
inline int wnaf5_128(int8_t (&d)[132], const u32 (&k)[4]) {
    typedef unsigned __int128 u128;
    u128 lo = (u128)((uint64_t)k[2] | (uint64_t)k[3] << 32) << 64 | ((uint64_t)k[0] | (uint64_t)k[1] << 32);
    uint64_t hi = 0;  // bits from 128 up (the value stays below 2^128 + 16)
    int n = 0;
    while (lo | hi) {
        int v = 0;
        if (lo & 1) {
            v = (int)(lo & 31);
            if (v >= 16) v -= 32;
            if (v > 0) {
                lo -= (u128)v;  // the low 5 bits are v: no borrow
            } else {
                const u128 o = lo;
                lo += (u128)(-v);
                if (lo < o) hi++;
            }
        }
        d[n++] = (int8_t)v;  // at most 130 digits
        lo = lo >> 1 | (u128)(hi & 1) << 127;
        hi >>= 1;
    }
    return n;
}

template <class ST, class QT>
inline bool twist_accumulate_q_wnaf(const ST& st, const u32 (&k1)[4], const u32 (&k2)[4], const QT& qt,
                                    gej& acc) {
    int8_t d[2][132];
    const int n0 = wnaf5_128(d[0], k1), n1 = wnaf5_128(d[1], k2);
    const bool kneg[2] = {(st.flags & LS_NEG0) != 0, (st.flags & LS_NEG1) != 0};
    const fe one = fe_one();
    bool inf = true;
    acc.x = acc.y = fe_zero();
    acc.z = one;
    for (int i = std::max(n0, n1) - 1; i >= 0; i--) {
        if (!inf) {
            gej t;
            gej_double(t, acc);
            acc = t;
        }
        for (int slot = 0; slot < 2; slot++) {
            const int v = i < (slot ? n1 : n0) ? d[slot][i] : 0;
            if (v == 0) continue;
            fe px, py;
            qt.get_pair((v < 0 ? -v : v) >> 1, slot, px, py);  // (|v| - 1) / 2 for odd |v|
            if ((v < 0) != kneg[slot]) fe_neg(py, py);
            acc_add(acc, inf, px, py, one, false);
        }
    }
    return inf;
}

// Whole ECDSA verify on one lane for the host (host_verify.cpp): the twist path with the wNAF Q
// half above and the host's variable-time inverses (modinv_host.h).  Same verdicts as
// ecdsa_verify_twist_lane.
template <class QT, class GC>
inline int ecdsa_verify_twist_host(u32 tag, const fe& px, const fe& py, const sc& r, const sc& s,
                                   const sc& m, QT& qt, const GC& gc) {
    TwistState st;
    if (!twist_prep_key(tag, px, py, qt, st)) return 0;
    sc sinv;
    if (!twist_prep_u2(st.flags, r, s, nullptr, st, &sinv)) return 0;
    u32 k1[4], k2[4];  // the raw GLV halves: undo twist_prep_u2's odd fix-up
    for (int i = 0; i < 4; i++) {
        k1[i] = st.k[0][i];
        k2[i] = st.k[1][i];
    }
    if (st.flags & LS_CORR0) k1[0] &= ~1u;
    if (st.flags & (LS_CORR0 << 1)) k2[0] &= ~1u;
    twist_prep_u1(m, sinv, &st.flags, st.k[2], st.k[3]);
    gej A, B;
    const bool binf = twist_accumulate_q_wnaf(st, k1, k2, qt, B);
    const bool ainf = twist_accumulate_g(st, gc, A);
    fe al, be, K;
    if (binf || ainf || !twist_combine(A, B, st.sigma, st.v, st.r, al, be, K))
        return twist_exceptional(A, ainf, B, binf, st.sigma, st.v, st.ychk, st.flags, st.r);
    fe binv;
    fe_inv(binv, be);
    return twist_final(al, K, binv, st.v, st.ychk, st.flags, st.r);
}
#endif

// ------------------------------------------------------------------------------------------
// BIP340 on the same path (secp256k1_schnorrsig_verify, modules/schnorrsig/main_impl.h:190-237):
// the x-only key's even-y lift (extrakeys/main_impl.h:21-39) is never computed either.
// R = s G - e P = A + B with A = s G (comb) and B = (-e) P_w (Q ladder on E_w).  Besides
// x(R) == r (alpha + w beta == 0, as for ECDSA) the reference needs y(R) even.  With the same
// quantities, Y3 = c0 + w c1 and Z3 = w Z1 Zb H, so
//   y(R) = (c0 w + v c1) / Dd,   Dd = v^2 D^3,  D = Z1 Zb H,
//   M = U1 H^2 - X3r,  X3r = S2^2 + v s1^2 - H^3 - 2 U1 H^2,
//   c0 = S2 (M - 2 v s1^2),  c1 = s1 (2 S2^2 - M - H^3),
// and w = gamma once gamma has passed.  beta and Dd are inverted together (one batched inversion
// of beta Dd per tuple).
// ------------------------------------------------------------------------------------------

// Prep: rx < p (main_impl.h:207), s < n (:211-214), x < p (extrakeys), the challenge e, u1 = s
// for the comb and u2 = -e for the Q ladder, the Q_w table.  The key parity to match is even.
template <class QT>
BCC_HD bool schnorr_twist_prep(const fe& px, const fe& rx, const sc& s_in, const sc& m, QT& qt,
                               TwistState& st) {
    const u32 N[8] = BCC_N_LIMBS;
    st.flags = 0;
    if (!fe_lt_p(rx)) return false;
    if (!u256_lt(s_in.v, N)) return false;
    if (!fe_lt_p(px)) return false;
    fe v;
    curve_rhs(v, px);
    sc e, u2, u1 = s_in, k1, k2;
    schnorr_challenge(e, rx, px, m);
    sc_neg(u2, e);
    u32 flags = LS_VALID | LS_COMP;  // even y: LS_PAR clear
    sc_split_lambda(k1, k2, u2);
    if ((k1.v[4] | k1.v[5] | k1.v[6] | k1.v[7]) != 0) {
        sc_neg(k1, k1);
        flags |= LS_NEG0;
    }
    if ((k2.v[4] | k2.v[5] | k2.v[6] | k2.v[7]) != 0) {
        sc_neg(k2, k2);
        flags |= LS_NEG1;
    }
    if (sc_is_zero(u1)) {
        flags |= LS_U1ZERO;
        u1.v[0] = 1u;
    } else if ((u1.v[0] & 1u) == 0) {
        sc_neg(u1, u1);
        flags |= LS_NEGU1;
    }
    for (int i = 0; i < 4; i++) {
        st.k[0][i] = k1.v[i];
        st.k[1][i] = k2.v[i];
        st.k[2][i] = u1.v[i];
        st.k[3][i] = u1.v[4 + i];
    }
    for (int q = 0; q < 2; q++) {
        if ((st.k[q][0] & 1u) == 0) flags |= LS_CORR0 << q;
        st.k[q][0] |= 1u;
    }
    st.flags = flags;
    for (int i = 0; i < 8; i++) st.r.v[i] = rx.v[i];
    st.v = v;
    st.ychk = fe_zero();
    fe qx, qy;
    fe_mul(qx, px, v);
    fe_sqr(qy, v);
    build_q_table_coz(qx, qy, qt, st.sigma);
    return true;
}

// alpha, beta as twist_combine, plus Dd, c0, c1 for the y-parity of R.  False for the exceptional
// configurations (x(A) == x(B), beta == 0; Dd == 0 follows from H == 0).
BCC_HD bool schnorr_twist_combine(const gej& A, const gej& B, const fe& sigma, const fe& v,
                                  const fe& rx, fe& al, fe& be, fe& dd, fe& c0, fe& c1) {
    fe zb, zb2, z12, u1, u2, s1, s2, h, hh, t, x3r, m;
    fe_mul(zb, B.z, sigma);
    fe_sqr(zb2, zb);
    fe_sqr(z12, A.z);
    fe_mul(u2, B.x, z12);          // U2 = X2 Z1^2
    fe_mul(t, z12, A.z);
    fe_mul(s2, B.y, t);            // S2 = Y2 Z1^3
    fe_mul(t, A.y, zb2);
    fe_mul(t, t, zb);
    fe_mul(s1, t, v);              // s1 = Y1 Zb^3 v
    fe_mul(t, A.x, zb2);
    fe_mul(u1, t, v);              // U1 = X1 Zb^2 v
    fe_sub(h, u2, u1);
    if (fe_is_zero(h)) return false;
    fe_mul(be, s2, s1);
    fe_shl<1>(be, be);             // beta = 2 S2 s1
    if (fe_is_zero(be)) return false;
    fe_mul(t, A.z, zb);
    fe_mul(t, t, h);               // D = Z1 Zb H
    fe_sqr(dd, t);
    fe_mul(dd, dd, t);
    fe_sqr(t, v);
    fe_mul(dd, dd, t);             // Dd = v^2 D^3
    fe_sqr(hh, h);
    fe_mul(t, z12, zb2);
    fe_mul(t, t, v);
    fe K;
    fe_mul(K, t, hh);              // K = Z3^2
    fe h3, s22, vs12, u1h2;
    fe_mul(h3, hh, h);
    fe_mul(u1h2, u1, hh);
    fe_sqr(s22, s2);
    fe_sqr(t, s1);
    fe_mul(vs12, t, v);
    fe_add(x3r, s22, vs12);
    fe_sub(x3r, x3r, h3);
    fe_sub(x3r, x3r, u1h2);
    fe_sub(x3r, x3r, u1h2);        // X3r = S2^2 + v s1^2 - H^3 - 2 U1 H^2
    fe_mul(al, rx, K);
    fe_sub(al, al, x3r);           // alpha = r K - X3r
    fe_sub(m, u1h2, x3r);          // M = U1 H^2 - X3r
    fe_sub(t, m, vs12);
    fe_sub(t, t, vs12);
    fe_mul(c0, s2, t);             // c0 = S2 (M - 2 v s1^2)
    fe_shl<1>(t, s22);
    fe_sub(t, t, m);
    fe_sub(t, t, h3);
    fe_mul(c1, s1, t);             // c1 = s1 (2 S2^2 - M - H^3)
    return true;
}

// The verdict of a normal BIP340 lane from ic = (beta Dd)^-1.
BCC_HD int schnorr_twist_final(const fe& al, const fe& be, const fe& dd, const fe& c0,
                               const fe& c1, const fe& ic, const fe& v) {
    fe binv, dinv, g, g2, y, t;
    fe_mul(binv, dd, ic);
    fe_mul(dinv, be, ic);
    fe_mul(g, al, binv);
    fe_neg(g, g);
    fe_normalize(g);
    fe_sqr(g2, g);
    if (!fe_equal(g2, v)) return 0;          // x(R) != r, or x^3 + 7 not a square
    if (g.v[0] & 1u) return 0;               // gamma is not the even-y lift: x(R) != r
    fe_mul(y, c0, g);
    fe_mul(t, v, c1);
    fe_add(y, y, t);
    fe_mul(y, y, dinv);
    fe_normalize(y);
    return (y.v[0] & 1u) == 0 ? 1 : 0;       // y(R) even (main_impl.h:234-236)
}

// Exact fallback for the exceptional BIP340 lanes: the even-y lift by the square root, the plain
// Jacobian sum, x(R) == r and y(R) even with a per-lane inversion.
BCC_HD int schnorr_twist_exceptional(const gej& A, bool ainf, const gej& B, bool binf,
                                     const fe& sigma, const fe& v, const fe& rx) {
    fe w;
    if (!fe_sqrt(w, v)) return 0;
    fe_normalize(w);
    if (w.v[0] & 1u) fe_neg(w, w);
    if (ainf && binf) return 0;
    gej be = B, R;
    bool rinf = false;
    fe zb;
    fe_mul(zb, B.z, sigma);
    fe_mul(be.z, zb, w);
    if (binf) R = A;
    else if (ainf) R = be;
    else gej_add_gej(R, rinf, A, be);
    if (rinf) return 0;
    fe z2, lhs, zi;
    fe_sqr(z2, R.z);
    fe_mul(lhs, rx, z2);
    if (!fe_equal(lhs, R.x)) return 0;
    fe_inv(zi, R.z);
    return schnorr_y_even(R.y, zi) ? 1 : 0;
}

// Whole BIP340 verify on one lane (host tests).
template <class QT, class GC>
BCC_HD int schnorr_verify_twist_lane(const fe& px, const fe& rx, const sc& s, const sc& m,
                                     QT& qt, const GC& gc) {
    TwistState st;
    if (!schnorr_twist_prep(px, rx, s, m, qt, st)) return 0;
    gej A, B;
    const bool binf = twist_accumulate_q(st, qt, B);
    const bool ainf = twist_accumulate_g(st, gc, A);
    fe al, be, dd, c0, c1;
    if (binf || ainf || !schnorr_twist_combine(A, B, st.sigma, st.v, rx, al, be, dd, c0, c1))
        return schnorr_twist_exceptional(A, ainf, B, binf, st.sigma, st.v, rx);
    fe c, ic;
    fe_mul(c, be, dd);
    fe_inv(ic, c);
    return schnorr_twist_final(al, be, dd, c0, c1, ic, st.v);
}

// Host build of the comb tables: per window the odd multiples of 2^(WC win) G in Jacobian
// coordinates, then one batched normalisation (Montgomery's trick) per window.  The window bases
// come from one doubling chain; the windows themselves are independent and built on up to CWIN
// threads (std::thread; the 16-bit comb is 0.5 M points).
inline void build_g_comb_window(fe* xy, int win, const gej& base) {
    std::vector<gej> pts(CTAB);
    std::vector<fe> pre(CTAB);
    {
        gej b2;
        gej_double(b2, base);
        pts[0] = base;
        for (int i = 1; i < CTAB; i++) {
            bool inf_unused;
            gej_add_gej(pts[i], inf_unused, pts[i - 1], b2);
        }
        fe acc = fe_one();
        for (int i = 0; i < CTAB; i++) {
            pre[i] = acc;                  // Z_0 ... Z_{i-1}
            fe_mul(acc, acc, pts[i].z);
        }
        fe inv;
        fe_inv(inv, acc);
        for (int i = CTAB - 1; i >= 0; i--) {
            fe zi, zi2, zi3, x, y;
            fe_mul(zi, inv, pre[i]);       // Z_i^-1
            fe_mul(inv, inv, pts[i].z);
            fe_sqr(zi2, zi);
            fe_mul(zi3, zi2, zi);
            fe_mul(x, pts[i].x, zi2);
            fe_mul(y, pts[i].y, zi3);
            fe_normalize(x);
            fe_normalize(y);
            xy[((size_t)win * CTAB + i) * 2 + 0] = x;
            xy[((size_t)win * CTAB + i) * 2 + 1] = y;
        }
    }
}

inline void build_g_comb(fe* xy) {
    std::vector<gej> bases(CWIN);
    {
        const u32 X[8] = BCC_GX_LIMBS, Y[8] = BCC_GY_LIMBS;
        fe_set(bases[0].x, X);
        fe_set(bases[0].y, Y);
        bases[0].z = fe_one();
    }
    for (int win = 1; win < CWIN; win++) {  // 2^(WC win) G, Jacobian
        gej b = bases[win - 1];
        for (int i = 0; i < WC; i++) {
            gej t;
            gej_double(t, b);
            b = t;
        }
        bases[win] = b;
    }
    const unsigned hw = std::thread::hardware_concurrency();
    const int nth = std::max(1, std::min<int>(CWIN, hw ? (int)hw : 1));
    std::vector<std::thread> th;
    for (int k = 1; k < nth; k++)
        th.emplace_back([&, k] {
            for (int win = k; win < CWIN; win += nth) build_g_comb_window(xy, win, bases[win]);
        });
    for (int win = 0; win < CWIN; win += nth) build_g_comb_window(xy, win, bases[win]);
    for (auto& t : th) t.join();
}

}  // namespace bcc
