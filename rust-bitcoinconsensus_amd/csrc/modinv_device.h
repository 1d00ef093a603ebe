// Modular inverse for the GPU lanes: Bernstein-Yang "safegcd" divsteps (Bernstein & Yang, "Fast
// constant-time gcd computation and modular inversion", 2019), restated for 64-wide SIMT lanes.
//
// The divsteps run 30 at a time on the low words of (f, g) as a branchless select chain (every lane
// of a wave executes the same instructions), their 2^30-scaled transition matrix is then applied
// to f, g and to the Bezout coefficients d, e held in nine signed 30-bit limbs with 64-bit products
// (v_mad_i64_i32).  25 batches (750 >= 741 divsteps) bound any 256-bit input; a wave stops early
// once g is zero in every lane (about 19 batches for random inputs).  About 2.5x fewer
// instructions than the Fermat chains (255 squarings + the multiplications of the addition chain)
// it replaces in K_inv (s^-1 mod n) and K_tfin (beta^-1 mod p), and far less latency for a lone
// wave.  The inverted values are public (signatures, curve points), as for the reference's
// secp256k1_scalar_inverse_var / secp256k1_fe_inv_var (ecdsa_impl.h:229, group_impl.h).
// Checked against integer inverses in tools/safegcd/check.py (host prototype, p and n, 40k random
// and edge operands) and on the GPU by tests/test_field_gpu.py (mi_fe_selftest ops 10 / 11).
#pragma once
#include <stdint.h>

// one out-of-line copy per kernel (a 25-batch loop is too large to inline at every call site)
#if defined(__HIPCC__)
#define BCC_MI30_FN __host__ __device__ __attribute__((noinline)) inline
#else
#define BCC_MI30_FN inline
#endif

namespace bcc {
namespace mi30 {

constexpr int32_t M30 = (1 << 30) - 1;

// value = v[0] + v[1] 2^30 + ... + v[8] 2^240; v[0..7] in [0, 2^30), v[8] signed
struct S30 {
    int32_t v[9];
};

BCC_HD S30 from_u32(const uint32_t (&a)[8]) {
    S30 r;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int b = 30 * i, w = b >> 5, s = b & 31;
        const uint32_t lo = w < 8 ? a[w] >> s : 0u;
        const uint32_t hi = (s && w + 1 < 8) ? a[w + 1] << (32 - s) : 0u;
        r.v[i] = (int32_t)((lo | hi) & (i < 8 ? (uint32_t)M30 : 0xFFFFFFFFu));
    }
    return r;
}

BCC_HD void to_u32(uint32_t (&r)[8], const S30& a) {  // a in [0, 2^256), canonical limbs
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int b = 30 * i, w = b >> 5, s = b & 31;
        const uint32_t x = (uint32_t)a.v[i];
        if (w < 8) r[w] |= x << s;
        if (s > 2 && w + 1 < 8) r[w + 1] |= x >> (32 - s);
    }
}

// 30 divsteps on the low words of (f, g), eta = -delta: 2^30 f' = u f + v g, 2^30 g' = q f + r g.
// A step: g odd and delta > 0 -> (f, g) = (g, (g - f) / 2), delta = 1 - delta; g odd otherwise
// -> g = (g + f) / 2, delta = 1 + delta; g even -> g = g / 2, delta = 1 + delta.
BCC_HD int32_t divsteps30(int32_t eta, uint32_t f, uint32_t g, int32_t (&t)[4]) {
    int32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll 2
    for (int i = 0; i < 30; i++) {
        const bool odd = (g & 1u) != 0;
        const bool sw = odd && eta < 0;
        const uint32_t gpf = g + f, gmf = g - f;
        const int32_t qpu = q + u, qmu = q - u, rpv = r + v, rmv = r - v;
        const uint32_t nf = sw ? g : f;
        const uint32_t ng = sw ? gmf : (odd ? gpf : g);
        const int32_t nu = sw ? q : u, nv = sw ? r : v;
        const int32_t nq = sw ? qmu : (odd ? qpu : q), nr = sw ? rmv : (odd ? rpv : r);
        eta = (sw ? -eta : eta) - 1;
        f = nf;
        g = ng >> 1;
        u = nu * 2;
        v = nv * 2;
        q = nq;
        r = nr;
    }
    t[0] = u;
    t[1] = v;
    t[2] = q;
    t[3] = r;
    return eta;
}

// (f, g) <- (u f + v g, q f + r g) / 2^30 (exact)
BCC_HD void update_fg(S30& f, S30& g, const int32_t (&t)[4]) {
    int64_t cf = (int64_t)t[0] * f.v[0] + (int64_t)t[1] * g.v[0];
    int64_t cg = (int64_t)t[2] * f.v[0] + (int64_t)t[3] * g.v[0];
    cf >>= 30;
    cg >>= 30;
#pragma unroll
    for (int i = 1; i < 9; i++) {
        cf += (int64_t)t[0] * f.v[i] + (int64_t)t[1] * g.v[i];
        cg += (int64_t)t[2] * f.v[i] + (int64_t)t[3] * g.v[i];
        f.v[i - 1] = (int32_t)cf & M30;
        g.v[i - 1] = (int32_t)cg & M30;
        cf >>= 30;
        cg >>= 30;
    }
    f.v[8] = (int32_t)cf;
    g.v[8] = (int32_t)cg;
}

// a += m & mask (mask 0 or -1), canonical limbs out
BCC_HD void cadd(S30& a, const S30& m, int32_t mask) {
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += a.v[i] + (m.v[i] & mask);
        a.v[i] = c & M30;
        c >>= 30;
    }
    a.v[8] += c + (m.v[8] & mask);
}

// a in (-m, 2m) -> [0, m)
BCC_HD void normalize(S30& a, const S30& m) {
    cadd(a, m, a.v[8] >> 31);  // negative: + m
    S30 t;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += a.v[i] - m.v[i];
        t.v[i] = c & M30;
        c >>= 30;
    }
    t.v[8] = a.v[8] + c - m.v[8];
    const int32_t keep = t.v[8] >> 31;  // a - m < 0: keep a
#pragma unroll
    for (int i = 0; i < 9; i++) a.v[i] = (a.v[i] & keep) | (t.v[i] & ~keep);
}

// (d, e) <- (u d + v e, q d + r e) / 2^30 mod m: multiples md, me of m in [0, 2^30) clear the low
// limbs (minv30 = m^-1 mod 2^30); d, e in [0, m) before and after (|u| + |v| <= 2^30, so the sums
// divided by 2^30 lie in (-m, 2m)).
BCC_HD void update_de(S30& d, S30& e, const int32_t (&t)[4], const S30& m, uint32_t minv30) {
    int64_t cd = (int64_t)t[0] * d.v[0] + (int64_t)t[1] * e.v[0];
    int64_t ce = (int64_t)t[2] * d.v[0] + (int64_t)t[3] * e.v[0];
    const int32_t md = (int32_t)((0u - (uint32_t)cd) * minv30 & (uint32_t)M30);
    const int32_t me = (int32_t)((0u - (uint32_t)ce) * minv30 & (uint32_t)M30);
    cd += (int64_t)md * m.v[0];
    ce += (int64_t)me * m.v[0];
    cd >>= 30;
    ce >>= 30;
#pragma unroll
    for (int i = 1; i < 9; i++) {
        cd += (int64_t)t[0] * d.v[i] + (int64_t)t[1] * e.v[i] + (int64_t)md * m.v[i];
        ce += (int64_t)t[2] * d.v[i] + (int64_t)t[3] * e.v[i] + (int64_t)me * m.v[i];
        d.v[i - 1] = (int32_t)cd & M30;
        e.v[i - 1] = (int32_t)ce & M30;
        cd >>= 30;
        ce >>= 30;
    }
    d.v[8] = (int32_t)cd;
    e.v[8] = (int32_t)ce;
    normalize(d, m);
    normalize(e, m);
}

BCC_HD bool is_zero(const S30& a) {
    int32_t o = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) o |= a.v[i];
    return o == 0;
}

// r = a^-1 mod m for an odd 256-bit modulus m and 0 <= a < m; r = 0 for a == 0 (as the Fermat
// chains give).  minv30 = m^-1 mod 2^30.
BCC_MI30_FN void inverse(uint32_t (&r)[8], const uint32_t (&a)[8], const uint32_t (&mm)[8],
                         uint32_t minv30) {
    const S30 M = from_u32(mm);
    S30 f = M, g = from_u32(a), d, e;
#pragma unroll
    for (int i = 0; i < 9; i++) d.v[i] = e.v[i] = 0;
    e.v[0] = 1;
    int32_t eta = -1;  // delta = 1
#pragma unroll 1
    for (int b = 0; b < 25; b++) {
#if defined(__HIP_DEVICE_COMPILE__)
        if (!__any(!is_zero(g))) break;  // wave-uniform: every lane of the wave has finished
#else
        if (is_zero(g)) break;
#endif
        int32_t t[4];
        eta = divsteps30(eta, (uint32_t)f.v[0] | ((uint32_t)f.v[1] << 30),
                         (uint32_t)g.v[0] | ((uint32_t)g.v[1] << 30), t);
        update_fg(f, g, t);
        update_de(d, e, t, M, minv30);
    }
    // f = +-1 and d a == f (mod m); f == -1: r = m - d
    const int32_t neg = f.v[8] >> 31;
    S30 n;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += M.v[i] - d.v[i];
        n.v[i] = c & M30;
        c >>= 30;
    }
    n.v[8] = M.v[8] - d.v[8] + c;
    const int32_t dz = is_zero(d) ? -1 : 0;  // m - 0 would be m: keep 0
    const int32_t take = neg & ~dz;
#pragma unroll
    for (int i = 0; i < 9; i++) d.v[i] = (d.v[i] & ~take) | (n.v[i] & take);
    to_u32(r, d);
}

}  // namespace mi30
}  // namespace bcc
