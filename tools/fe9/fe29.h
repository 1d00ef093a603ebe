// Fp in radix 2^29 for the verify hot path: nine 29-bit limbs, value = sum v[i] 2^(29 i).
//
// Why this representation on gfx950 (measured, profiles/r02a): the signature kernels are
// VALU-issue bound (~95 % of the SIMDs' issue slots), and on MI355X almost every integer VALU op
// costs a half-rate slot (v_mad_u64_u32, v_addc_co_u32, v_alignbit_b32, v_lshrrev_b64 all run at
// ~34 T lane-ops/s; only plain adds / logic ops run at ~59 T).  With 32-bit limbs every partial
// product needs a v_mad_u64_u32 AND a v_addc_co_u32 to catch the 64-bit accumulator's carry, plus
// register moves between columns and carry-chain add / sub with a fold of the 2^256 wrap.  With
// 29-bit limbs a column of nine products stays below 2^64, so
//   * a product is 81 bare v_mad_u64_u32 + one v_and / v_lshrrev_b64 pair per column;
//   * the reduction by 2^261 == 2^37 + 31264 (mod p) is three v_mad_u64_u32 per limb, and a
//     small constant factor k of the result (2XY^2 ... 9X^4 in the doubling) rides along for free
//     by scaling the fold constants (fe9_mul_k / fe9_sqr_k);
//   * add / sub / double are one plain op per limb: limbs are LAZY, with explicit bounds.
// The same C code runs on the host (tests/native) and on the device: the CPU tests exercise the
// arithmetic the GPU executes (no inline asm).
//
// Reference semantics restated: field_10x26_impl.h (the reference's 32-bit field: 26-bit limbs,
// lazy magnitudes, 2^260 == 0x3D10 * 2^... fold) and field_impl.h:39-263 (sqrt / inverse chains).
//
// Bounds (B = largest limb value; "N" = normalised: every limb <= 2^29 + 1):
//   fe9_mul_k(a, b)    needs B(a) * B(b) <= 2^60.8; returns N        (9 B(a) B(b) + 2^35 < 2^64)
//   fe9_sqr_k(a)       needs B(a) <= 2^30.4;        returns N
//   fe9_add(a, b)      B(a) + B(b)
//   fe9_shl1(a)        2 B(a)
//   fe9_sub(a, b)      needs B(b) <= 2^29 + 1 (b normalised); returns B(a) + 2^30
//   fe9_sub2(a, b)     needs B(b) <= 2^30 + 2;      returns B(a) + 2^31
//   fe9_norm(a)        needs B(a) <= 2^31.9;        returns N
// k in fe9_mul_k / fe9_sqr_k is a small constant (1..9) multiplied into the result.
#pragma once
#include "secp256k1_device.h"

namespace bcc {

struct fe9 {
    u32 v[9];
};

constexpr u32 M29 = 0x1FFFFFFFu;

// acc + a * b as ONE v_mad_u64_u32 whose 64-bit addend is the running accumulator.  Left to
// itself the compiler re-associates a column's nine products into a separate sum and adds the
// carry afterwards (one extra 64-bit add per column); the empty asm pins the order.
#ifndef BCC_FE9_CHAIN
#define BCC_FE9_CHAIN 1
#endif
BCC_HD void mad_acc(u64& acc, u32 a, u32 b) {
#if defined(__HIP_DEVICE_COMPILE__) && BCC_FE9_CHAIN >= 2
    asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
#else
    acc += (u64)a * b;
#if defined(__HIP_DEVICE_COMPILE__) && BCC_FE9_CHAIN == 1
    asm volatile("" : "+v"(acc));
#endif
#endif
}

// 48 p with every limb raised to >= 2^29 + 2^27 by borrowing from the next one (computed by
// tools/fe9/derive_constants.py): a - b + K48 never underflows a limb for normalised b.
#define BCC_K48_LIMBS {0x3fff48d0u, 0x3ffffe7eu, 0x3ffffffeu, 0x3ffffffeu, 0x3ffffffeu, \
                       0x3ffffffeu, 0x3ffffffeu, 0x3ffffffeu, 0x2ffffffeu}
// p in radix 2^29 (canonical digits)
#define BCC_P29_LIMBS {0x1ffffc2fu, 0x1ffffff7u, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, \
                       0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x00ffffffu}

BCC_HD fe9 fe9_zero() {
    fe9 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = 0;
    return r;
}
BCC_HD fe9 fe9_one() {
    fe9 r = fe9_zero();
    r.v[0] = 1;
    return r;
}
BCC_HD fe9 fe9_small(u32 c) {  // c < 2^29
    fe9 r = fe9_zero();
    r.v[0] = c;
    return r;
}

// ---- conversions ---------------------------------------------------------------------------
// 8 x 32 (any value < 2^256) -> 9 x 29, normalised (v[8] < 2^24)
BCC_HD void fe9_from_fe(fe9& r, const fe& a) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int bit = 29 * i, w = bit >> 5, s = bit & 31;
        const u32 lo = a.v[w] >> s;
        const u32 hi = (s > 3 && w + 1 < 8) ? (a.v[w + 1] << (32 - s)) : 0u;
        r.v[i] = (lo | hi) & M29;
    }
}

// one carry pass: digits 0..7 < 2^29, value unchanged, v[8] takes the rest (inputs < 2^32 - 8)
BCC_HD void fe9_carry(fe9& r) {
    u32 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const u32 x = r.v[i] + c;
        r.v[i] = x & M29;
        c = x >> 29;
    }
    r.v[8] += c;
}

// value (< 2^262) -> 8 x 32 weak (< 2^256, congruent), via canonical digits and one fold of the
// bits at 2^256 and above
BCC_HD void fe9_to_fe_weak(fe& r, const fe9& a_in) {
    fe9 a = a_in;
    fe9_carry(a);
    const u32 top = a.v[8] >> 24;  // bits 256.. (value < 2^262: top < 2^6)
    a.v[8] &= 0xFFFFFFu;
    u32 w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {  // w[j] = bits [32 j, 32 j + 32) of the 256-bit digit string
        const int i = (32 * j) / 29, s = (32 * j) % 29;
        u32 x = a.v[i] >> s;
        if (29 - s < 32 && i + 1 < 9) x |= a.v[i + 1] << (29 - s);
        if (58 - s < 32 && i + 2 < 9) x |= a.v[i + 2] << (58 - s);
        w[j] = x;
    }
    // + top * (2^32 + 977): at most one further wrap, which adds 2^32 + 977 once more
    u64 c = (u64)w[0] + (u64)top * 977u;
    r.v[0] = lo32(c);
    c = (c >> 32) + (u64)w[1] + top;
    r.v[1] = lo32(c);
#pragma unroll
    for (int j = 2; j < 8; j++) {
        c = (c >> 32) + w[j];
        r.v[j] = lo32(c);
    }
    if (c >> 32) {
        c = (u64)r.v[0] + 977u;
        r.v[0] = lo32(c);
        c = (c >> 32) + (u64)r.v[1] + 1u;
        r.v[1] = lo32(c);
#pragma unroll
        for (int j = 2; j < 8; j++) {
            c = (c >> 32) + r.v[j];
            r.v[j] = lo32(c);
        }
    }
}

// canonical 8 x 32 (< p)
BCC_HD void fe9_to_fe(fe& r, const fe9& a) {
    fe9_to_fe_weak(r, a);
    fe_normalize(r);
}

// ---- lazy linear ops -----------------------------------------------------------------------
BCC_HD void fe9_add(fe9& r, const fe9& a, const fe9& b) {
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + b.v[i];
}
BCC_HD void fe9_shl1(fe9& r, const fe9& a) {
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = a.v[i] << 1;
}
// a - b + 48 p (b normalised)
BCC_HD void fe9_sub(fe9& r, const fe9& a, const fe9& b) {
    const u32 K[9] = BCC_K48_LIMBS;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + (K[i] - b.v[i]);
}
// a - b + 96 p (b with limbs <= 2^30 + 2, e.g. the double of a normalised value)
BCC_HD void fe9_sub2(fe9& r, const fe9& a, const fe9& b) {
    const u32 K[9] = BCC_K48_LIMBS;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + (2u * K[i] - b.v[i]);
}
// -a + 48 p (a normalised)
BCC_HD void fe9_neg(fe9& r, const fe9& a) {
    const u32 K[9] = BCC_K48_LIMBS;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = K[i] - a.v[i];
}

// weak normalisation: limbs <= 2^31.9 -> N
BCC_HD void fe9_norm(fe9& r) {
    u32 c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const u32 x = r.v[i] + c;
        r.v[i] = x & M29;
        c = x >> 29;
    }
    // c * 2^261 == c * 31264 + c * 256 * 2^29  (c < 2^3)
    const u32 x0 = r.v[0] + c * 31264u;
    r.v[0] = x0 & M29;
    const u32 x1 = r.v[1] + (c << 8) + (x0 >> 29);
    r.v[1] = x1 & M29;
    r.v[2] += x1 >> 29;
}

// ---- multiplication ------------------------------------------------------------------------
// t (18 columns: t[0..16] < 2^29, t[17] < 2^32) -> K * t mod p, normalised.
//   2^261 == 2^37 + 31264 (mod p):  column j >= 9 adds 31264 t_j to limb j - 9 and 256 t_j to
//   limb j - 8; column 17 (2^493 == 31264 2^232 + 65536 2^29 + 8003584) adds 31264 t_17 to
//   limb 8, 65536 t_17 to limb 1 and 8003584 t_17 to limb 0.  Every term is one
//   v_mad_u64_u32 into a 64-bit running carry; the factor K scales the constants.
template <u32 K>
BCC_HD void fe9_reduce(fe9& r, const u32 (&t)[18]) {
    constexpr u32 C0 = 31264u * K, C1 = 256u * K, CA = 8003584u * K, CB = 65536u * K;
    u64 acc = (u64)t[0] * K;
    mad_acc(acc, t[9], C0);
    mad_acc(acc, t[17], CA);
    r.v[0] = lo32(acc) & M29;
    acc >>= 29;
    mad_acc(acc, t[1], K);
    mad_acc(acc, t[10], C0);
    mad_acc(acc, t[9], C1);
    mad_acc(acc, t[17], CB);
    r.v[1] = lo32(acc) & M29;
    acc >>= 29;
#pragma unroll
    for (int i = 2; i < 8; i++) {
        mad_acc(acc, t[i], K);
        mad_acc(acc, t[i + 9], C0);
        mad_acc(acc, t[i + 8], C1);
        r.v[i] = lo32(acc) & M29;
        acc >>= 29;
    }
    mad_acc(acc, t[8], K);
    mad_acc(acc, t[17], C0);
    mad_acc(acc, t[16], C1);
    r.v[8] = lo32(acc) & M29;
    const u32 c = (u32)(acc >> 29);  // < 2^21.2: the coefficient of 2^261
    const u64 x0 = (u64)c * 31264u + r.v[0];
    r.v[0] = lo32(x0) & M29;
    const u32 x1 = r.v[1] + (c << 8) + (u32)(x0 >> 29);
    r.v[1] = x1 & M29;
    r.v[2] += x1 >> 29;
}

// r = K a b mod p
template <u32 K>
BCC_HD void fe9_mul_k(fe9& r, const fe9& a, const fe9& b) {
    u32 t[18];
    u64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#if BCC_FE9_CHAIN == 3
        // two half-columns as independent chains (more ILP per wave), joined by one 64-bit add
        u64 acc2 = 0;
        int n = 0;
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++, n++) {
            if (n & 1) mad_acc(acc2, a.v[i], b.v[k - i]);
            else mad_acc(acc, a.v[i], b.v[k - i]);
        }
        acc += acc2;
#else
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) mad_acc(acc, a.v[i], b.v[k - i]);
#endif
        t[k] = lo32(acc) & M29;
        acc >>= 29;
    }
    t[17] = lo32(acc);
    fe9_reduce<K>(r, t);
}

// r = K a^2 mod p: cross products once against the doubled limbs, plus the squares
template <u32 K>
BCC_HD void fe9_sqr_k(fe9& r, const fe9& a) {
    u32 d[9], t[18];
#pragma unroll
    for (int i = 0; i < 9; i++) d[i] = a.v[i] << 1;
    u64 acc = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; i++) mad_acc(acc, d[i], a.v[k - i]);
        if ((k & 1) == 0) mad_acc(acc, a.v[k / 2], a.v[k / 2]);
        t[k] = lo32(acc) & M29;
        acc >>= 29;
    }
    t[17] = lo32(acc);
    fe9_reduce<K>(r, t);
}

BCC_HD void fe9_mul(fe9& r, const fe9& a, const fe9& b) { fe9_mul_k<1>(r, a, b); }
BCC_HD void fe9_sqr(fe9& r, const fe9& a) { fe9_sqr_k<1>(r, a); }

// ---- exact tests ---------------------------------------------------------------------------
// a == 0 (mod p), a normalised (value < 2^261 + 2^60).  Every nonzero multiple q p (q <= 32) has
// digits 2..7 all ones, so a value whose digits 2..7 are neither all ones nor all zero is
// nonzero mod p; only the rest (adversarial inputs) pays for the exact test.
BCC_HD bool fe9_is_zero(const fe9& a_in) {
    fe9 a = a_in;
    fe9_carry(a);  // canonical digits (N has v[2] <= 2^29 + 1)
    u32 ones = M29, any = 0;
#pragma unroll
    for (int i = 2; i < 8; i++) {
        ones &= a.v[i];
        any |= a.v[i];
    }
    if (ones != M29 && any != 0) return false;
    fe w;
    fe9_to_fe_weak(w, a);
    return fe_is_zero(w);
}

BCC_HD bool fe9_equal(const fe9& a, const fe9& b) {  // both normalised
    fe9 d;
    fe9_sub(d, a, b);
    fe9_norm(d);
    return fe9_is_zero(d);
}

// parity of the canonical value (a normalised)
BCC_HD bool fe9_is_odd(const fe9& a) {
    fe w;
    fe9_to_fe(w, a);
    return (w.v[0] & 1u) != 0;
}

BCC_HD void fe9_sqr_n(fe9& r, const fe9& a, int n) {
    r = a;
#pragma unroll 1
    for (int i = 0; i < n; i++) fe9_sqr(r, r);
}

// x223 = a^(2^223 - 1), x22, x2: the common prefix of the (p+1)/4 and p-2 chains
// (field_impl.h:39-137 / 229-263 addition chains)
BCC_HD void fe9_chain_x223(fe9& x223, fe9& x22, fe9& x2, const fe9& a) {
    fe9 x3, x6, x9, x11, x44, x88, x176, x220, t;
    fe9_sqr(x2, a);
    fe9_mul(x2, x2, a);
    fe9_sqr(x3, x2);
    fe9_mul(x3, x3, a);
    fe9_sqr_n(t, x3, 3);
    fe9_mul(x6, t, x3);
    fe9_sqr_n(t, x6, 3);
    fe9_mul(x9, t, x3);
    fe9_sqr_n(t, x9, 2);
    fe9_mul(x11, t, x2);
    fe9_sqr_n(t, x11, 11);
    fe9_mul(x22, t, x11);
    fe9_sqr_n(t, x22, 22);
    fe9_mul(x44, t, x22);
    fe9_sqr_n(t, x44, 44);
    fe9_mul(x88, t, x44);
    fe9_sqr_n(t, x88, 88);
    fe9_mul(x176, t, x88);
    fe9_sqr_n(t, x176, 44);
    fe9_mul(x220, t, x44);
    fe9_sqr_n(t, x220, 3);
    fe9_mul(x223, t, x3);
}

// r = a^((p+1)/4); true when r^2 == a (secp256k1_fe_sqrt semantics)
BCC_HD bool fe9_sqrt(fe9& r, const fe9& a) {
    fe9 x223, x22, x2, t;
    fe9_chain_x223(x223, x22, x2, a);
    fe9_sqr_n(t, x223, 23);
    fe9_mul(t, t, x22);
    fe9_sqr_n(t, t, 6);
    fe9_mul(t, t, x2);
    fe9_sqr(t, t);
    fe9_sqr(r, t);
    fe9_sqr(t, r);
    return fe9_equal(t, a);
}

// r = a^(p-2)
BCC_HD void fe9_inv(fe9& r, const fe9& a) {
    fe9 x223, x22, x2, t;
    fe9_chain_x223(x223, x22, x2, a);
    fe9_sqr_n(t, x223, 23);
    fe9_mul(t, t, x22);
    fe9_sqr_n(t, t, 5);
    fe9_mul(t, t, a);
    fe9_sqr_n(t, t, 3);
    fe9_mul(t, t, x2);
    fe9_sqr_n(t, t, 2);
    fe9_mul(r, t, a);
}

// ---- group law on Jacobian coordinates (every coordinate normalised) -----------------------
struct gej9 {
    fe9 x, y, z;
};

// 2a, a not infinity (no 2-torsion: never infinity).  dbl-2009-l restated with the products
// taken directly where the radix-2^29 arithmetic makes that cheaper than the squaring trick:
//   A = X^2, B = Y^2, D = 4 X B, F = 9 A^2 (= E^2, E = 3A), Z3 = 2 Y Z,
//   X3 = F - 2D, Y3 = 3 A (D - X3) - 8 B^2.     4M + 4S (k-scaled reductions, no 2M+5S adds)
BCC_HD void gej9_double(gej9& r, const gej9& a) {
    fe9 A, B, C8, D, F, t;
    fe9_sqr(A, a.x);
    fe9_sqr(B, a.y);
    fe9_sqr_k<8>(C8, B);         // 8 Y^4
    fe9_mul_k<4>(D, a.x, B);     // 4 X Y^2
    fe9_sqr_k<9>(F, A);          // 9 X^4
    fe9_mul_k<2>(r.z, a.y, a.z); // 2 Y Z
    fe9_shl1(t, D);              // <= 2^30 + 2
    fe9_sub2(r.x, F, t);         // <= 2^29 + 1 + 2^31
    fe9_norm(r.x);
    fe9_sub(t, D, r.x);          // <= 2^29 + 1 + 2^30
    fe9_mul_k<3>(t, A, t);       // 3 A (D - X3)
    fe9_sub(r.y, t, C8);
    fe9_norm(r.y);
}

// r = a + b, b = (bx, by) affine on the curve scaled by 1/bzinv (bzinv used iff use_zinv), 8M+3S
// (+1M with zinv); exceptional cases (a == b: double, a == -b: infinity) exactly as
// gej_add_zinv_var / gej_add_ge_var (group_impl.h:388-491).  a must not be infinity.
BCC_HD void gej9_add_zinv(gej9& r, bool& inf, const gej9& a, const fe9& bx, const fe9& by,
                          const fe9& bzinv, bool use_zinv, fe9* hout = nullptr) {
    fe9 az, z12, u2, s2, h, rr, hh, hhh, v, t;
    if (use_zinv) fe9_mul(az, a.z, bzinv);
    else az = a.z;
    fe9_sqr(z12, az);
    fe9_mul(u2, bx, z12);
    fe9_mul(s2, by, z12);
    fe9_mul(s2, s2, az);
    fe9_sub(h, u2, a.x);
    fe9_norm(h);
    fe9_sub(rr, s2, a.y);
    fe9_norm(rr);
    if (fe9_is_zero(h)) {  // rare, adversarial only
        if (fe9_is_zero(rr)) {
            gej9_double(r, a);
            inf = false;
        } else {
            inf = true;
            r = a;
        }
        return;
    }
    if (hout) *hout = h;
    fe9_sqr(hh, h);
    fe9_mul(hhh, h, hh);
    fe9_mul(v, a.x, hh);
    fe9_mul(r.z, a.z, h);
    fe9_sqr(t, rr);
    fe9_sub(t, t, hhh);          // <= 2^29 + 1 + 2^30
    fe9_shl1(u2, v);             // 2V <= 2^30 + 2
    fe9_sub2(r.x, t, u2);        // X3 = R^2 - H^3 - 2V
    fe9_norm(r.x);
    fe9_sub(t, v, r.x);
    fe9_mul(t, rr, t);
    fe9_mul(hhh, a.y, hhh);
    fe9_sub(r.y, t, hhh);        // Y3 = R (V - X3) - Y1 H^3
    fe9_norm(r.y);
    inf = false;
}

}  // namespace bcc
