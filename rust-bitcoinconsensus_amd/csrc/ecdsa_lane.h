// Per-lane building blocks of the signature ladders (one lane = one tuple), shared by the
// verification path (ecdsa_twist.h: ECDSA per secp256k1_ecdsa_verify, secp256k1.c:423-438 +
// ecdsa_impl.h:207-275; BIP340 per secp256k1_schnorrsig_verify, modules/schnorrsig/
// main_impl.h:190-237) and the synthetic-input generators (keygen and signing below):
//   signed odd fixed-window recoding (every digit nonzero, so every lane of a wave adds at the
//   same bit positions: no wNAF divergence), the shared-Z odd-multiples table of Q on an
//   isomorphic curve (no inversion), the mixed addition into an accumulator, the BIP340
//   challenge, and the affine G tables of the generators' fixed-base ladder.
// (The round-1 verify lanes -- key decompression by a square root, G tables in LDS -- were retired
// with their kernels in round 4; ecdsa_twist.h is the verification path.)
#pragma once
#include "secp256k1_device.h"
#include "sha256_device.h"

namespace bcc {

// window widths
#ifndef BCC_WQ_BITS
#define BCC_WQ_BITS 4
#endif
constexpr int WQ = BCC_WQ_BITS;               // Q / lambda*Q digits: table of 2^(WQ-1) odd multiples
#ifndef BCC_WG_BITS
#define BCC_WG_BITS 10
#endif
constexpr int WG = BCC_WG_BITS;               // G / 2^128*G digits: tables of 2^(WG-1) odd multiples
constexpr int QTAB = 1 << (WQ - 1);           // 8 for WQ = 4
constexpr int GTAB = 1 << (WG - 1);
constexpr int TOPQ = (127 / WQ) * WQ;         // top digit position for 128-bit scalars (124)
static_assert(TOPQ + WQ >= 128, "top Q digit must cover bit 127");
constexpr int TOPG = (127 / WG) * WG;         // top G digit position: 120 for WG = 8, 10, 12
static_assert(TOPG + WG >= 128 && TOPG <= TOPQ, "top G digit must cover bit 127 inside the ladder");

// (k >> pos) & (2^w - 1) for a 128-bit k (4 limbs), 0 <= pos < 128, w <= 31
BCC_HD u32 bits_at(u32 l0, u32 l1, u32 l2, u32 l3, int pos, int w) {
    int li = pos >> 5, sh = pos & 31;
    u32 a = li == 0 ? l0 : li == 1 ? l1 : li == 2 ? l2 : l3;
    u32 b = li == 0 ? l1 : li == 1 ? l2 : li == 2 ? l3 : 0u;
    u32 v = sh ? ((a >> sh) | (b << (32 - sh))) : a;
    return v & ((1u << w) - 1u);
}

// Signed odd fixed-window recoding of an ODD scalar k < 2^128, closed form:
//   k = sum_i d_i 2^(w i),  d_i = 2*((k >> (w i + 1)) mod 2^w) + 1 - 2^w   (i < top)
//   d_top = 2*(k >> (w top + 1)) + 1            (positive, < 2^w for k < 2^128)
// Returns the table index (|d| - 1) / 2 and sets neg = (d < 0).
BCC_HD u32 digit_index(u32 l0, u32 l1, u32 l2, u32 l3, int pos, int w, int top, bool& neg) {
    u32 v = bits_at(l0, l1, l2, l3, pos + 1, w);
    if (pos == top) {
        neg = false;
        return v;
    }
    u32 half = 1u << (w - 1), mask = half - 1u;
    bool positive = (v & half) != 0;
    neg = !positive;
    return positive ? (v & mask) : (~v & mask);
}

// Per-lane Q table: entry i holds x, beta*x, y of (2i+1)Q on the shared-Z curve E'.
// Host version: a plain array (device version lives in ecdsa_verify.hip).
struct QTableArray {
    fe e[QTAB][3];
    BCC_HD void put(int i, int f, const fe& a) { e[i][f] = a; }
    BCC_HD void get(int i, int f, fe& a) const { a = e[i][f]; }
    BCC_HD void get_pair(int i, int which, fe& x, fe& y) const {
        x = e[i][which];
        y = e[i][2];
    }
};

// Host version of the G tables: affine (2i+1) * 2^(128 tab) * G.
struct GTableArray {
    const fe* xy;  // [2][GTAB][2]
    BCC_HD void get(int tab, int i, fe& x, fe& y) const {
        x = xy[(tab * GTAB + i) * 2 + 0];
        y = xy[(tab * GTAB + i) * 2 + 1];
    }
};

// acc += point; the point is (px, py) affine on E (use_zinv, scale sigma) or on E' (plain).
// Handles acc == infinity (rare) by materialising the point on E'.
BCC_HD void acc_add(gej& acc, bool& inf, const fe& px, const fe& py, const fe& sigma,
                    bool use_zinv) {
    if (inf) {  // rare: only after an adversarial cancellation
        if (use_zinv) {
            fe s2, s3;
            fe_sqr(s2, sigma);
            fe_mul(s3, s2, sigma);
            fe_mul(acc.x, px, s2);
            fe_mul(acc.y, py, s3);
        } else {
            acc.x = px;
            acc.y = py;
        }
        acc.z = fe_one();
        inf = false;
        return;
    }
    gej r;
    bool rinf;
    gej_add_zinv(r, rinf, acc, px, py, sigma, use_zinv);
    acc = r;
    inf = rinf;
}

// TwistState::flags bits (ecdsa_twist.h): valid, negated GLV halves, odd-fix corrections
enum : u32 {
    LS_VALID = 1u, LS_NEG0 = 2u, LS_NEG1 = 4u, LS_CORR0 = 8u,  // LS_CORR0 << slot
};

// Q table: odd multiples {1,3,..,15}Q on E' with one shared Z (ecmult_odd_multiples_table +
// ge_globalz_set_table_gej restated, ecmult_impl.h:85-143), plus the lambda images beta*x; returns
// sigma, the scale of E' (total Z of the table).  Built by co-Z arithmetic (Meloni's ZADDU; DBLU
// for the first doubling): every T_i = T_{i-1} + 2Q is one co-Z addition that also re-expresses
// 2Q with T_i's Z (4M + 2S instead of a mixed addition's 8M + 3S); the Z ratios
// h_i = X_{2Q} - X_{T_{i-1}} then rescale every entry to the common Z by a backward H-product.
template <class QT>
BCC_HD void build_q_table_coz(const fe& qx, const fe& qy, QT& qt, fe& sigma) {
    fe dx, dy, tx, ty;
    {  // DBLU: D = 2Q with Z = 2y, T_0 = Q with the same Z
        fe b, e, l, sx, m, t;
        fe_sqr(b, qx);             // x^2
        fe_sqr(e, qy);             // y^2
        fe_sqr(l, e);              // y^4
        fe_add(t, qx, e);
        fe_sqr(t, t);
        fe_sub(t, t, b);
        fe_sub(t, t, l);
        fe_shl<1>(sx, t);          // S = 4 x y^2 (= x (2y)^2)
        fe_shl<1>(m, b);
        fe_add(m, m, b);           // M = 3 x^2
        fe_sqr(t, m);
        fe_shl<1>(dx, sx);
        fe_sub(dx, t, dx);         // X(2Q) = M^2 - 2S
        fe_sub(t, sx, dx);
        fe_mul(t, m, t);
        fe_shl<3>(ty, l);          // 8 y^4 (= y (2y)^3)
        fe_sub(dy, t, ty);         // Y(2Q) = M (S - X) - 8 y^4
        tx = sx;
    }
    qt.put(0, 0, tx);
    qt.put(0, 2, ty);
    for (int i = 1; i < QTAB; i++) {  // ZADDU(D, T_{i-1}) -> T_i = D + T_{i-1}, D co-Z with T_i
        fe h, c, w1, w2, d, a1, t, ry;
        fe_sub(h, dx, tx);         // Z_i = Z_{i-1} h
        fe_sqr(c, h);
        fe_mul(w1, dx, c);
        fe_mul(w2, tx, c);
        fe_sub(ry, dy, ty);
        fe_sqr(d, ry);
        fe_sub(t, w1, w2);
        fe_mul(a1, dy, t);
        fe_sub(t, d, w1);
        fe_sub(tx, t, w2);         // X3 = (Yd - Yt)^2 - W1 - W2
        fe_sub(t, w1, tx);
        fe_mul(t, ry, t);
        fe_sub(ty, t, a1);         // Y3 = (Yd - Yt)(W1 - X3) - A1
        dx = w1;                   // D re-expressed with Z_i
        dy = a1;
        qt.put(i, 0, tx);
        qt.put(i, 2, ty);
        qt.put(i, 1, h);           // slot 1 holds h_i until the rescale pass
    }
    fe f = fe_one(), f2, f3, beta;
    {
        const u32 bl[8] = BCC_BETA_LIMBS;
        fe_set(beta, bl);
    }
    for (int i = QTAB - 1; i >= 0; i--) {  // entry i times f_i = prod_{j>i} h_j = Z_last / Z_i
        fe ex, ey, h;
        qt.get(i, 0, ex);
        qt.get(i, 2, ey);
        if (i > 0) qt.get(i, 1, h);
        if (i < QTAB - 1) {
            fe_sqr(f2, f);
            fe_mul(f3, f2, f);
            fe_mul(ex, ex, f2);
            fe_mul(ey, ey, f3);
        }
        fe bx;
        fe_mul(bx, ex, beta);
        qt.put(i, 0, ex);
        qt.put(i, 1, bx);
        qt.put(i, 2, ey);
        if (i > 0) fe_mul(f, f, h);
    }
    fe y2;
    fe_shl<1>(y2, qy);
    fe_mul(sigma, f, y2);          // Z_last = 2y prod h_i
}

// x^3 + 7
BCC_HD void curve_rhs(fe& r, const fe& x) {
    fe seven = fe_const(7, 0, 0, 0, 0, 0, 0, 0);
    fe_sqr(r, x);
    fe_mul(r, r, x);
    fe_add(r, r, seven);
}

// ------------------------------------------------------------------------------------------
// BIP340 (config C5): secp256k1_schnorrsig_verify, modules/schnorrsig/main_impl.h:190-237
// ------------------------------------------------------------------------------------------

// e = SHA256(SHA256(tag) || SHA256(tag) || rx || px || m) mod n, tag = "BIP0340/challenge":
// the 64-byte tag prefix is the fixed midstate of secp256k1_schnorrsig_sha256_tagged
// (main_impl.h:98-109), so the challenge is two compressions (96 message bytes + padding,
// total length 160 bytes).  rx, px, m are the raw 32-byte strings read as big-endian integers
// (rx, px < p, so their fe_get_b32 serialisations are those same bytes).
BCC_HD void schnorr_challenge(sc& e, const fe& rx, const fe& px, const sc& m) {
    const u32 N[8] = BCC_N_LIMBS;
    u32 s[8] = {0x9cecba11u, 0x23925381u, 0x11679112u, 0xd1627e0fu,
                0x97c87550u, 0x003cc765u, 0x90f61164u, 0x33e9b66au};
    u32 w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        w[j] = rx.v[7 - j];                      // big-endian word j of the 32-byte string
        w[8 + j] = px.v[7 - j];
    }
    sha256_compress(s, w);
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = m.v[7 - j];
    w[8] = 0x80000000u;
#pragma unroll
    for (int j = 9; j < 15; j++) w[j] = 0;
    w[15] = 160 * 8;
    sha256_compress(s, w);
#pragma unroll
    for (int i = 0; i < 8; i++) e.v[i] = s[7 - i];
    if (!u256_lt(e.v, N)) {                      // scalar_set_b32 reduction (main_impl.h:124)
        u32 tmp[8];
        u256_sub(tmp, e.v, N);
        for (int i = 0; i < 8; i++) e.v[i] = tmp[i];
    }
}

// y = ye * zinv^3 normalised; true when even (!secp256k1_fe_is_odd).
BCC_HD bool schnorr_y_even(const fe& ye, const fe& zinv) {
    fe z2, z3, y;
    fe_sqr(z2, zinv);
    fe_mul(z3, z2, zinv);
    fe_mul(y, ye, z3);
    fe_normalize(y);
    return (y.v[0] & 1u) == 0;
}

// k*G -> affine (x, y), normalized.  Used by the synthetic-workload generator (keygen, signing),
// not by verification.  Same signed-odd-window ladder as the verify loop, G slots only.
// Returns false for k == 0 (mod n) or a zero result.
template <class GT>
BCC_HD bool ecmult_gen_lane(const sc& k_in, fe& xo, fe& yo, const GT& gt) {
    if (sc_is_zero(k_in)) return false;
    u32 c0 = k_in.v[0], c1 = k_in.v[1], c2 = k_in.v[2], c3 = k_in.v[3];
    u32 d0 = k_in.v[4], d1 = k_in.v[5], d2 = k_in.v[6], d3 = k_in.v[7];
    bool corr2 = (c0 & 1u) == 0, corr3 = (d0 & 1u) == 0;
    c0 |= 1u;
    d0 |= 1u;
    fe one = fe_one();
    gej acc;
    bool inf = false;
    {
        bool ng;
        u32 idx = digit_index(c0, c1, c2, c3, TOPG, WG, TOPG, ng);
        gt.get(0, (int)idx, acc.x, acc.y);
        acc.z = one;
    }
    for (int pos = TOPG; pos >= 0; pos--) {
        if (pos != TOPG && !inf) {
            gej t;
            gej_double(t, acc);
            acc = t;
        }
        if (pos % WG) continue;
        for (int slot = 2; slot < 4; slot++) {
            if (slot == 2 && pos == TOPG) continue;
            bool dneg;
            u32 idx = slot == 2 ? digit_index(c0, c1, c2, c3, pos, WG, TOPG, dneg)
                                : digit_index(d0, d1, d2, d3, pos, WG, TOPG, dneg);
            fe px, py;
            gt.get(slot - 2, (int)idx, px, py);
            if (dneg) fe_neg(py, py);
            acc_add(acc, inf, px, py, one, false);
        }
    }
    for (int slot = 2; slot < 4; slot++) {
        if (!(slot == 2 ? corr2 : corr3)) continue;
        fe px, py;
        gt.get(slot - 2, 0, px, py);
        fe_neg(py, py);
        acc_add(acc, inf, px, py, one, false);
    }
    if (inf) return false;
    fe zi, zi2, zi3;
    fe_inv(zi, acc.z);
    fe_sqr(zi2, zi);
    fe_mul(zi3, zi2, zi);
    fe_mul(xo, acc.x, zi2);
    fe_mul(yo, acc.y, zi3);
    fe_normalize(xo);
    fe_normalize(yo);
    return true;
}

// ECDSA signing for the generator: r = x(kG) mod n, s = k^-1 (m + r d) mod n, low-S.
template <class GT>
BCC_HD bool ecdsa_sign_lane(const sc& d, const sc& m_in, const sc& k, sc& r, sc& s, const GT& gt) {
    const u32 N[8] = BCC_N_LIMBS;
    fe rx, ry;
    if (!ecmult_gen_lane(k, rx, ry, gt)) return false;
    for (int i = 0; i < 8; i++) r.v[i] = rx.v[i];
    if (!u256_lt(r.v, N)) {
        u32 t[8];
        u256_sub(t, r.v, N);
        for (int i = 0; i < 8; i++) r.v[i] = t[i];
    }
    if (sc_is_zero(r)) return false;
    sc m = m_in, kinv, t;
    if (!u256_lt(m.v, N)) {
        u32 tt[8];
        u256_sub(tt, m.v, N);
        for (int i = 0; i < 8; i++) m.v[i] = tt[i];
    }
    sc_inv(kinv, k);
    sc_mul(t, r, d);
    sc_add(t, t, m);
    sc_mul(s, kinv, t);
    if (sc_is_zero(s)) return false;
    // low-S: s > n/2 -> n - s  (n/2 = 7FFFFFFF FFFFFFFF FFFFFFFF FFFFFFFF 5D576E73 57A4501D DFE92F46 681B20A0)
    const u32 H[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                      0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
    if (u256_lt(H, s.v)) sc_neg(s, s);
    return true;
}

// BIP340 signing for the generator (secp256k1_schnorrsig_sign, main_impl.h:127-188, with the
// caller's nonce k instead of the BIP340 nonce function): the key is negated when its point
// has odd y, R = kG with k negated when R has odd y, sig = x(R) || k + e d.  Returns false for
// d or k == 0.  xonly receives P.x.
template <class GT>
BCC_HD bool schnorr_sign_lane(const sc& d_in, const sc& m, const sc& k_in, fe& rx, sc& s,
                              fe& xonly, const GT& gt) {
    fe px, py, ry;
    if (!ecmult_gen_lane(d_in, px, py, gt)) return false;
    if (!ecmult_gen_lane(k_in, rx, ry, gt)) return false;
    sc d = d_in, k = k_in, e, t;
    if (py.v[0] & 1u) sc_neg(d, d);
    if (ry.v[0] & 1u) sc_neg(k, k);
    xonly = px;
    schnorr_challenge(e, rx, px, m);
    sc_mul(t, e, d);
    sc_add(s, t, k);
    return true;
}

// Affine G tables: xy[(tab*GTAB + i)*2 + {0,1}] = (2i+1) * 2^(128 tab) * G.  Host-side build
// (once per process; exact group arithmetic, then one inversion per point).
inline void build_g_tables(fe* xy) {
    fe gx, gy;
    {
        const u32 X[8] = BCC_GX_LIMBS, Y[8] = BCC_GY_LIMBS;
        fe_set(gx, X);
        fe_set(gy, Y);
    }
    gej base;
    base.x = gx; base.y = gy; base.z = fe_one();
    for (int tab = 0; tab < 2; tab++) {
        if (tab == 1) {  // base = 2^128 G
            for (int i = 0; i < 128; i++) {
                gej t;
                gej_double(t, base);
                base = t;
            }
        }
        gej b2;
        gej_double(b2, base);
        // b2 to affine for mixed adds
        fe zi, zi2, zi3, b2x, b2y;
        fe_inv(zi, b2.z);
        fe_sqr(zi2, zi);
        fe_mul(zi3, zi2, zi);
        fe_mul(b2x, b2.x, zi2);
        fe_mul(b2y, b2.y, zi3);
        gej cur = base;
        for (int i = 0; i < GTAB; i++) {
            if (i > 0) {
                gej nxt;
                bool inf_unused;
                fe one = fe_one();
                gej_add_zinv(nxt, inf_unused, cur, b2x, b2y, one, false);
                cur = nxt;
            }
            fe x, y;
            fe_inv(zi, cur.z);
            fe_sqr(zi2, zi);
            fe_mul(zi3, zi2, zi);
            fe_mul(x, cur.x, zi2);
            fe_mul(y, cur.y, zi3);
            fe_normalize(x);
            fe_normalize(y);
            xy[(tab * GTAB + i) * 2 + 0] = x;
            xy[(tab * GTAB + i) * 2 + 1] = y;
        }
    }
}

}  // namespace bcc
