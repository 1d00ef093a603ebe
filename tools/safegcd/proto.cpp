// Prototype (host) of the GPU variable-time-free safegcd inverse: 30-bit batches of branchless
// divsteps on the low words, signed 30-bit limbs (9 per value), int64 products.  Checked against
// Python's pow(a, -1, m) by tools/safegcd/check.py.  Not part of the product.
#include <cstdint>
#include <cstdio>
#include <cstring>

typedef int32_t i32;
typedef int64_t i64;
typedef uint32_t u32;
constexpr i32 M30 = (1 << 30) - 1;

struct S30 { i32 v[9]; };

static S30 from_u32(const u32 a[8]) {
    S30 r;
    // bits 30i .. 30i+29
    for (int i = 0; i < 9; i++) {
        const int b = 30 * i, w = b >> 5, s = b & 31;
        u32 lo = w < 8 ? a[w] >> s : 0;
        u32 hi = (s && w + 1 < 8) ? a[w + 1] << (32 - s) : 0;
        r.v[i] = (i32)((lo | hi) & (i < 8 ? (u32)M30 : 0xFFFFFFFFu));
    }
    return r;
}
static void to_u32(u32 r[8], const S30& a) {  // a in [0, 2^256), canonical limbs
    for (int i = 0; i < 8; i++) r[i] = 0;
    for (int i = 0; i < 9; i++) {
        const int b = 30 * i, w = b >> 5, s = b & 31;
        const u32 x = (u32)a.v[i];
        if (w < 8) r[w] |= x << s;
        if (s > 2 && w + 1 < 8) r[w + 1] |= x >> (32 - s);
    }
}

struct Tr { i32 u, v, q, r; };

// 30 branchless divsteps on the low words of (f, g); eta = -delta.  2^30 f' = u f + v g,
// 2^30 g' = q f + r g.
static i32 divsteps30(i32 eta, u32 f, u32 g, Tr& t) {
    i32 u = 1, v = 0, q = 0, r = 1;
    for (int i = 0; i < 30; i++) {
        const bool odd = g & 1;
        const bool sw = odd && eta < 0;
        const u32 gpf = g + f, gmf = g - f;
        const i32 qpu = q + u, qmu = q - u, rpv = r + v, rmv = r - v;
        const u32 nf = sw ? g : f;
        const u32 ng = sw ? gmf : (odd ? gpf : g);
        const i32 nu = sw ? q : u, nv = sw ? r : v;
        const i32 nq = sw ? qmu : (odd ? qpu : q), nr = sw ? rmv : (odd ? rpv : r);
        eta = (sw ? -eta : eta) - 1;
        f = nf;
        g = ng >> 1;
        u = nu << 1;
        v = nv << 1;
        q = nq;
        r = nr;
    }
    t = Tr{u, v, q, r};
    return eta;
}

static void update_fg(S30& f, S30& g, const Tr& t) {
    i64 cf = (i64)t.u * f.v[0] + (i64)t.v * g.v[0];
    i64 cg = (i64)t.q * f.v[0] + (i64)t.r * g.v[0];
    cf >>= 30;
    cg >>= 30;
    for (int i = 1; i < 9; i++) {
        cf += (i64)t.u * f.v[i] + (i64)t.v * g.v[i];
        cg += (i64)t.q * f.v[i] + (i64)t.r * g.v[i];
        f.v[i - 1] = (i32)cf & M30;
        g.v[i - 1] = (i32)cg & M30;
        cf >>= 30;
        cg >>= 30;
    }
    f.v[8] = (i32)cf;
    g.v[8] = (i32)cg;
}

// a += (mask & m): conditional add of the modulus, canonical limbs out
static void cadd(S30& a, const S30& m, i32 mask) {
    i32 c = 0;
    for (int i = 0; i < 8; i++) {
        c += a.v[i] + (m.v[i] & mask);
        a.v[i] = c & M30;
        c >>= 30;
    }
    a.v[8] += c + (m.v[8] & mask);
}
static void csub(S30& a, const S30& m, i32 mask) {
    i32 c = 0;
    for (int i = 0; i < 8; i++) {
        c += a.v[i] - (m.v[i] & mask);
        a.v[i] = c & M30;
        c >>= 30;
    }
    a.v[8] += c - (m.v[8] & mask);
}
// a in (-m, 2m) -> [0, m)
static void norm(S30& a, const S30& m) {
    cadd(a, m, a.v[8] >> 31);  // negative: + m
    S30 t = a;
    csub(t, m, -1);
    const i32 keep = t.v[8] >> 31;  // a - m < 0: keep a
    for (int i = 0; i < 9; i++) a.v[i] = (a.v[i] & keep) | (t.v[i] & ~keep);
}

static void update_de(S30& d, S30& e, const Tr& t, const S30& m, u32 minv30) {
    i64 cd = (i64)t.u * d.v[0] + (i64)t.v * e.v[0];
    i64 ce = (i64)t.q * d.v[0] + (i64)t.r * e.v[0];
    const i32 md = (i32)(((u32)0 - (u32)cd) * minv30 & (u32)M30);
    const i32 me = (i32)(((u32)0 - (u32)ce) * minv30 & (u32)M30);
    cd += (i64)md * m.v[0];
    ce += (i64)me * m.v[0];
    cd >>= 30;
    ce >>= 30;
    for (int i = 1; i < 9; i++) {
        cd += (i64)t.u * d.v[i] + (i64)t.v * e.v[i] + (i64)md * m.v[i];
        ce += (i64)t.q * d.v[i] + (i64)t.r * e.v[i] + (i64)me * m.v[i];
        d.v[i - 1] = (i32)cd & M30;
        e.v[i - 1] = (i32)ce & M30;
        cd >>= 30;
        ce >>= 30;
    }
    d.v[8] = (i32)cd;
    e.v[8] = (i32)ce;
    norm(d, m);
    norm(e, m);
}

static bool is_zero(const S30& a) {
    i32 o = 0;
    for (int i = 0; i < 9; i++) o |= a.v[i];
    return o == 0;
}

// r = a^-1 mod m (a < m, a != 0); r = 0 for a == 0
static int inv(u32 r[8], const u32 a[8], const u32 mm[8], int max_batches) {
    const S30 M = from_u32(mm);
    u32 m0 = mm[0], x = m0;
    for (int i = 0; i < 4; i++) x *= 2 - m0 * x;
    const u32 minv30 = x & (u32)M30;
    S30 f = M, g = from_u32(a), d{}, e{};
    e.v[0] = 1;
    i32 eta = -1;
    int b = 0;
    for (; b < max_batches && !is_zero(g); b++) {
        Tr t;
        eta = divsteps30(eta, (u32)f.v[0] | ((u32)f.v[1] << 30), (u32)g.v[0] | ((u32)g.v[1] << 30), t);
        update_fg(f, g, t);
        update_de(d, e, t, M, minv30);
    }
    // f = +-1: d a == f (mod m)
    if (f.v[8] < 0) {  // f == -1: r = -d = m - d
        S30 n = M;
        for (int i = 0; i < 9; i++) n.v[i] = 0;
        csub(n, d, -1);
        cadd(n, M, n.v[8] >> 31);
        d = n;
    }
    to_u32(r, d);
    return b;
}

int main() {
    // stdin: lines "m a" as 64 hex chars each (big-endian); stdout: "r batches"
    char mh[80], ah[80];
    while (scanf("%64s %64s", mh, ah) == 2) {
        u32 m[8], a[8], r[8];
        for (int i = 0; i < 8; i++) {
            unsigned x, y;
            sscanf(mh + 8 * (7 - i), "%8x", &x);
            sscanf(ah + 8 * (7 - i), "%8x", &y);
            m[i] = x;
            a[i] = y;
        }
        int b = inv(r, a, m, 25);
        for (int i = 7; i >= 0; i--) printf("%08x", r[i]);
        printf(" %d\n", b);
    }
}
