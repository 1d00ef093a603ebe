// Host-only variable-time modular inverse for the host builds of the lane code (host_verify.cpp,
// tests/native): Bernstein-Yang "safegcd" divsteps (Bernstein & Yang, "Fast constant-time gcd
// computation and modular inversion", 2019), applied 62 at a time on the low words, with the
// transition matrix then applied to the full numbers in signed radix-2^62 limbs (128-bit
// products).  Verification data is public, so variable time is fine; the reference inverts the
// same public values (ecdsa_impl.h:229 secp256k1_scalar_inverse_var, group_impl.h's
// secp256k1_fe_inv_var).  About 12 batches of 62 divsteps for a 256-bit modulus, against the 255
// squarings of a Fermat inversion.  The GPU keeps its Fermat chains (wave-uniform control flow).
#pragma once
#include <stdint.h>

namespace bcc {
namespace modinv {

typedef __int128 i128;
constexpr int64_t M62 = (int64_t)(((uint64_t)1 << 62) - 1);

// value = v[0] + v[1] 2^62 + v[2] 2^124 + v[3] 2^186 + v[4] 2^248; v[0..3] in [0, 2^62), v[4] signed
struct S62 {
    int64_t v[5];
};

inline S62 from_u32(const uint32_t a[8]) {
    uint64_t w[4];
    for (int i = 0; i < 4; i++) w[i] = (uint64_t)a[2 * i] | (uint64_t)a[2 * i + 1] << 32;
    S62 r;
    r.v[0] = (int64_t)(w[0] & (uint64_t)M62);
    r.v[1] = (int64_t)((w[0] >> 62 | w[1] << 2) & (uint64_t)M62);
    r.v[2] = (int64_t)((w[1] >> 60 | w[2] << 4) & (uint64_t)M62);
    r.v[3] = (int64_t)((w[2] >> 58 | w[3] << 6) & (uint64_t)M62);
    r.v[4] = (int64_t)(w[3] >> 56);
    return r;
}

inline void to_u32(uint32_t r[8], const S62& a) {  // a in [0, 2^256)
    const uint64_t v0 = (uint64_t)a.v[0], v1 = (uint64_t)a.v[1], v2 = (uint64_t)a.v[2],
                   v3 = (uint64_t)a.v[3], v4 = (uint64_t)a.v[4];
    const uint64_t w[4] = {v0 | v1 << 62, v1 >> 2 | v2 << 60, v2 >> 4 | v3 << 58, v3 >> 6 | v4 << 56};
    for (int i = 0; i < 4; i++) {
        r[2 * i] = (uint32_t)w[i];
        r[2 * i + 1] = (uint32_t)(w[i] >> 32);
    }
}

inline uint64_t low64(const S62& a) { return (uint64_t)a.v[0] | (uint64_t)a.v[1] << 62; }

inline bool is_zero(const S62& a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3] | a.v[4]) == 0; }

// a += k m (small k), canonical limbs out
inline void addmul(S62& a, const S62& m, int64_t k) {
    i128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (i128)a.v[i] + (i128)k * m.v[i];
        a.v[i] = (int64_t)c & M62;
        c >>= 62;
    }
    a.v[4] = (int64_t)(c + a.v[4] + (i128)k * m.v[4]);
}

// a mod m into [0, m), for |a| < 4m
inline void reduce(S62& a, const S62& m) {
    while (a.v[4] < 0) addmul(a, m, 1);
    for (;;) {
        S62 t = a;
        addmul(t, m, -1);
        if (t.v[4] < 0) return;
        a = t;
    }
}

// 2^62 times the matrix of 62 divsteps on the low words of (f, g): after them,
// 2^62 f' = u f + v g and 2^62 g' = q f + r g.  Returns the new delta.
struct Trans {
    int64_t u, v, q, r;
};
inline int64_t divsteps62(int64_t delta, uint64_t f, uint64_t g, Trans& t) {
    int64_t u = 1, v = 0, q = 0, r = 1;
    for (int i = 0; i < 62; i++) {
        if (g & 1) {
            if (delta > 0) {  // (1 - delta, g, (g - f) / 2)
                delta = 1 - delta;
                const uint64_t of = f;
                f = g;
                g = (g - of) >> 1;
                const int64_t ou = u, ov = v;
                u = 2 * q;
                v = 2 * r;
                q -= ou;
                r -= ov;
            } else {  // (1 + delta, f, (g + f) / 2)
                delta = 1 + delta;
                g = (g + f) >> 1;
                q += u;
                r += v;
                u *= 2;
                v *= 2;
            }
        } else {  // (1 + delta, f, g / 2)
            delta = 1 + delta;
            g >>= 1;
            u *= 2;
            v *= 2;
        }
    }
    t = Trans{u, v, q, r};
    return delta;
}

// (f, g) <- (u f + v g, q f + r g) / 2^62 (exact)
inline void update_fg(S62& f, S62& g, const Trans& t) {
    i128 cf = (i128)t.u * f.v[0] + (i128)t.v * g.v[0];
    i128 cg = (i128)t.q * f.v[0] + (i128)t.r * g.v[0];
    cf >>= 62;
    cg >>= 62;
    for (int i = 1; i < 5; i++) {
        cf += (i128)t.u * f.v[i] + (i128)t.v * g.v[i];
        cg += (i128)t.q * f.v[i] + (i128)t.r * g.v[i];
        f.v[i - 1] = (int64_t)cf & M62;
        g.v[i - 1] = (int64_t)cg & M62;
        cf >>= 62;
        cg >>= 62;
    }
    f.v[4] = (int64_t)cf;
    g.v[4] = (int64_t)cg;
}

// (d, e) <- (u d + v e, q d + r e) / 2^62 mod m, d and e in [0, m) before and after
inline void update_de(S62& d, S62& e, const Trans& t, const S62& m, uint64_t minv62) {
    i128 cd = (i128)t.u * d.v[0] + (i128)t.v * e.v[0];
    i128 ce = (i128)t.q * d.v[0] + (i128)t.r * e.v[0];
    // add md m, me m so that the low 62 bits vanish
    const int64_t md = (int64_t)((0 - (uint64_t)cd) * minv62 & (uint64_t)M62);
    const int64_t me = (int64_t)((0 - (uint64_t)ce) * minv62 & (uint64_t)M62);
    cd += (i128)md * m.v[0];
    ce += (i128)me * m.v[0];
    cd >>= 62;
    ce >>= 62;
    for (int i = 1; i < 5; i++) {
        cd += (i128)t.u * d.v[i] + (i128)t.v * e.v[i] + (i128)md * m.v[i];
        ce += (i128)t.q * d.v[i] + (i128)t.r * e.v[i] + (i128)me * m.v[i];
        d.v[i - 1] = (int64_t)cd & M62;
        e.v[i - 1] = (int64_t)ce & M62;
        cd >>= 62;
        ce >>= 62;
    }
    d.v[4] = (int64_t)cd;
    e.v[4] = (int64_t)ce;
    reduce(d, m);  // |u d + v e + md m| / 2^62 < 3m
    reduce(e, m);
}

// r = a^-1 mod m for an odd 256-bit modulus m (a < 2^256, reduced first); r = 0 for a == 0 mod m,
// as the Fermat chains give.  Little-endian 32-bit limbs, r in [0, m).
inline void inverse_var(uint32_t r[8], const uint32_t a[8], const uint32_t m[8]) {
    const S62 M = from_u32(m);
    S62 g = from_u32(a);
    reduce(g, M);  // a < 2^256 < 2m
    if (is_zero(g)) {
        for (int i = 0; i < 8; i++) r[i] = 0;
        return;
    }
    const uint64_t m0 = (uint64_t)m[0] | (uint64_t)m[1] << 32;
    uint64_t inv = m0;  // m0 * m0 == 1 mod 8: 3 correct bits, doubled by each Newton step
    for (int i = 0; i < 5; i++) inv *= 2 - m0 * inv;
    const uint64_t minv62 = inv & (uint64_t)M62;
    S62 f = M, d = {{0, 0, 0, 0, 0}}, e = {{1, 0, 0, 0, 0}};
    int64_t delta = 1;
    for (int it = 0; it < 24 && !is_zero(g); it++) {  // <= 741 divsteps for 256 bits
        Trans t;
        delta = divsteps62(delta, low64(f), low64(g), t);
        update_fg(f, g, t);
        update_de(d, e, t, M, minv62);
    }
    // f == +-1 (gcd), and f == d a (mod m) throughout
    if (f.v[4] < 0) {
        S62 n = M;
        addmul(n, d, -1);  // m - d
        d = n;
        reduce(d, M);
    }
    to_u32(r, d);
}

}  // namespace modinv
}  // namespace bcc
