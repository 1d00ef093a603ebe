/* oracle/bcc_oracle.c — TEST INFRASTRUCTURE ONLY (see bcc_oracle.h).
 *
 * A deliberately simple, obviously-correct restatement of the reference's signature hot path:
 * fully-reduced 4x64-bit limbs, schoolbook products, Fermat inverses, double-and-add scalar
 * multiplication, no tables, no tricks. Speed is irrelevant here; it is only a checker.
 *
 * Every routine cites the reference file:line whose observable behaviour it restates
 * (paths relative to /root/reference/depend/bitcoin/src/).
 */
#include "bcc_oracle.h"

#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ========================================================================================== */
/* SHA-256 (FIPS 180-4; crypto/sha256.cpp:78-162 Transform, :637-679 Write/Finalize)          */
/* ========================================================================================== */
typedef struct {
    uint32_t s[8];
    uint8_t buf[64];
    uint64_t bytes;
} sha256_ctx;

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void sha256_compress(uint32_t s[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

static void sha256_init(sha256_ctx* c) {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(c->s, iv, sizeof iv);
    c->bytes = 0;
}

static void sha256_write(sha256_ctx* c, const uint8_t* p, size_t n) {
    while (n > 0) {
        size_t fill = (size_t)(c->bytes & 63);
        size_t take = 64 - fill < n ? 64 - fill : n;
        memcpy(c->buf + fill, p, take);
        c->bytes += take;
        p += take;
        n -= take;
        if (((c->bytes) & 63) == 0) sha256_compress(c->s, c->buf);
    }
}

static void sha256_final(sha256_ctx* c, uint8_t out[32]) {
    uint64_t bits = c->bytes * 8;
    uint8_t pad = 0x80, zero = 0, len[8];
    sha256_write(c, &pad, 1);
    while ((c->bytes & 63) != 56) sha256_write(c, &zero, 1);
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha256_write(c, len, 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(c->s[i] >> 24);
        out[4 * i + 1] = (uint8_t)(c->s[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->s[i] >> 8);
        out[4 * i + 3] = (uint8_t)c->s[i];
    }
}

void bcco_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
    sha256_ctx c;
    sha256_init(&c);
    sha256_write(&c, msg, len);
    sha256_final(&c, out);
}

/* CHashWriter::GetHash = SHA256(SHA256(x)) (hash.h:122-127) */
void bcco_sha256d(const uint8_t* msg, size_t len, uint8_t out[32]) {
    uint8_t t[32];
    bcco_sha256(msg, len, t);
    bcco_sha256(t, 32, out);
}

/* ========================================================================================== */
/* 256-bit integers, little-endian 64-bit limbs                                               */
/* ========================================================================================== */
typedef struct { uint64_t v[4]; } u256;

static const u256 P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 N = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};

static u256 u256_from_be(const uint8_t b[32]) {
    u256 r;
    for (int i = 0; i < 4; i++) {
        uint64_t x = 0;
        for (int j = 0; j < 8; j++) x = (x << 8) | b[(3 - i) * 8 + j];
        r.v[i] = x;
    }
    return r;
}

static void u256_to_be(const u256* a, uint8_t b[32]) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}

static int u256_cmp(const u256* a, const u256* b) {
    for (int i = 3; i >= 0; i--) {
        if (a->v[i] < b->v[i]) return -1;
        if (a->v[i] > b->v[i]) return 1;
    }
    return 0;
}

static int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }

/* r = a + b, returns carry */
static uint64_t u256_add(u256* r, const u256* a, const u256* b) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
        c += (u128)a->v[i] + b->v[i];
        r->v[i] = (uint64_t)c;
        c >>= 64;
    }
    return (uint64_t)c;
}

/* r = a - b, returns borrow */
static uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        u128 t = (u128)a->v[i] - b->v[i] - borrow;
        r->v[i] = (uint64_t)t;
        borrow = (uint64_t)(t >> 64) & 1;
    }
    return borrow;
}

/* ---- modular arithmetic with a generic modulus m = 2^256 - c (p and n both have this form) ---- */
typedef struct {
    u256 m;
    uint64_t c[3]; /* 2^256 - m, little-endian, < 2^192 */
} modulus;

static const modulus MODP = {{{0xFFFFFFFEFFFFFC2FULL, ~0ULL, ~0ULL, ~0ULL}}, {0x1000003D1ULL, 0, 0}};
static const modulus MODN = {{{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, ~0ULL}},
                             {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL}};

/* reduce an up-to-8-limb value modulo m by folding 2^256 == c, then final subtraction */
static u256 mod_reduce(const modulus* md, const uint64_t* t_in, int nl) {
    uint64_t t[12];
    memset(t, 0, sizeof t);
    memcpy(t, t_in, (size_t)nl * 8);
    for (;;) {
        int hi_nonzero = 0;
        for (int i = 4; i < 12; i++) hi_nonzero |= (t[i] != 0);
        if (!hi_nonzero) break;
        uint64_t acc[12];
        memset(acc, 0, sizeof acc);
        memcpy(acc, t, 4 * 8);
        /* acc += hi * c */
        for (int i = 4; i < 12; i++) {
            if (!t[i]) continue;
            u128 carry = 0;
            for (int j = 0; j < 3; j++) {
                u128 x = (u128)t[i] * md->c[j] + acc[i - 4 + j] + carry;
                acc[i - 4 + j] = (uint64_t)x;
                carry = x >> 64;
            }
            for (int k = i - 4 + 3; carry && k < 12; k++) {
                u128 x = (u128)acc[k] + carry;
                acc[k] = (uint64_t)x;
                carry = x >> 64;
            }
        }
        memcpy(t, acc, sizeof t);
    }
    u256 r = {{t[0], t[1], t[2], t[3]}};
    while (u256_cmp(&r, &md->m) >= 0) u256_sub(&r, &r, &md->m);
    return r;
}

static u256 mod_mul(const modulus* md, const u256* a, const u256* b) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; i++) {
        u128 carry = 0;
        for (int j = 0; j < 4; j++) {
            u128 x = (u128)a->v[i] * b->v[j] + t[i + j] + carry;
            t[i + j] = (uint64_t)x;
            carry = x >> 64;
        }
        t[i + 4] = (uint64_t)carry;
    }
    return mod_reduce(md, t, 8);
}

static u256 mod_add(const modulus* md, const u256* a, const u256* b) {
    uint64_t t[5];
    u256 r;
    t[4] = u256_add(&r, a, b);
    memcpy(t, r.v, 32);
    return mod_reduce(md, t, 5);
}

static u256 mod_neg(const modulus* md, const u256* a) {
    u256 r;
    if (u256_is_zero(a)) return *a;
    u256_sub(&r, &md->m, a);
    return r;
}

static u256 mod_sub(const modulus* md, const u256* a, const u256* b) {
    u256 nb = mod_neg(md, b);
    return mod_add(md, a, &nb);
}

static u256 mod_pow(const modulus* md, const u256* a, const u256* e) {
    u256 r = {{1, 0, 0, 0}};
    for (int i = 255; i >= 0; i--) {
        r = mod_mul(md, &r, &r);
        if ((e->v[i / 64] >> (i % 64)) & 1) r = mod_mul(md, &r, a);
    }
    return r;
}

/* Fermat inverse a^(m-2) (field_impl.h:229-263 / scalar_impl.h:68-236 compute the same value) */
static u256 mod_inv(const modulus* md, const u256* a) {
    u256 e, two = {{2, 0, 0, 0}};
    u256_sub(&e, &md->m, &two);
    return mod_pow(md, a, &e);
}

/* ========================================================================================== */
/* Field Fp helpers                                                                           */
/* ========================================================================================== */
static u256 fe_mul(const u256* a, const u256* b) { return mod_mul(&MODP, a, b); }
static u256 fe_sqr(const u256* a) { return mod_mul(&MODP, a, a); }
static u256 fe_add(const u256* a, const u256* b) { return mod_add(&MODP, a, b); }
static u256 fe_sub(const u256* a, const u256* b) { return mod_sub(&MODP, a, b); }
static u256 fe_small(uint64_t k) { u256 r = {{k, 0, 0, 0}}; return r; }

/* secp256k1_fe_sqrt (field_impl.h:39-137): r = a^((p+1)/4); succeeds iff r^2 == a */
static int fe_sqrt(u256* r, const u256* a) {
    u256 e, one = {{1, 0, 0, 0}};
    u256_add(&e, &P, &one);          /* p + 1 fits: p < 2^256 - 1 */
    e.v[0] = (e.v[0] >> 2) | (e.v[1] << 62);
    e.v[1] = (e.v[1] >> 2) | (e.v[2] << 62);
    e.v[2] = (e.v[2] >> 2) | (e.v[3] << 62);
    e.v[3] = e.v[3] >> 2;
    *r = mod_pow(&MODP, a, &e);
    u256 chk = fe_sqr(r);
    return u256_cmp(&chk, a) == 0;
}

/* ========================================================================================== */
/* Group law, Jacobian coordinates with explicit infinity (group_impl.h semantics)            */
/* ========================================================================================== */
typedef struct { u256 x, y, z; int inf; } gej;

static const u256 GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const u256 GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};

static gej gej_from_affine(const u256* x, const u256* y) {
    gej r;
    r.x = *x; r.y = *y; r.z = fe_small(1); r.inf = 0;
    return r;
}

/* doubling for a = 0 (gej_double, group_impl.h:273-305 computes the same point) */
static gej gej_double(const gej* a) {
    gej r;
    if (a->inf || u256_is_zero(&a->y)) { r.inf = 1; r.x = r.y = r.z = fe_small(0); return r; }
    u256 xx = fe_sqr(&a->x), yy = fe_sqr(&a->y), yyyy = fe_sqr(&yy);
    u256 s = fe_mul(&a->x, &yy);                 /* S = 4*X*Y^2 */
    s = fe_add(&s, &s); s = fe_add(&s, &s);
    u256 m = fe_add(&xx, &xx); m = fe_add(&m, &xx); /* M = 3*X^2 */
    u256 t = fe_sqr(&m), s2 = fe_add(&s, &s);
    r.x = fe_sub(&t, &s2);                       /* X3 = M^2 - 2S */
    u256 e = fe_sub(&s, &r.x);
    u256 y8 = fe_add(&yyyy, &yyyy); y8 = fe_add(&y8, &y8); y8 = fe_add(&y8, &y8);
    t = fe_mul(&m, &e);
    r.y = fe_sub(&t, &y8);                       /* Y3 = M(S - X3) - 8Y^4 */
    t = fe_mul(&a->y, &a->z);
    r.z = fe_add(&t, &t);                        /* Z3 = 2YZ */
    r.inf = 0;
    return r;
}

/* general addition incl. P == Q (-> double) and P == -Q (-> infinity)
 * (gej_add_var, group_impl.h:307-333, same exceptional-case outcomes) */
static gej gej_add(const gej* a, const gej* b) {
    if (a->inf) return *b;
    if (b->inf) return *a;
    u256 z1z1 = fe_sqr(&a->z), z2z2 = fe_sqr(&b->z);
    u256 u1 = fe_mul(&a->x, &z2z2), u2 = fe_mul(&b->x, &z1z1);
    u256 t = fe_mul(&b->z, &z2z2);
    u256 s1 = fe_mul(&a->y, &t);
    t = fe_mul(&a->z, &z1z1);
    u256 s2 = fe_mul(&b->y, &t);
    u256 h = fe_sub(&u2, &u1), rr = fe_sub(&s2, &s1);
    if (u256_is_zero(&h)) {
        if (u256_is_zero(&rr)) return gej_double(a);
        gej inf; inf.inf = 1; inf.x = inf.y = inf.z = fe_small(0);
        return inf;
    }
    u256 hh = fe_sqr(&h), hhh = fe_mul(&h, &hh), v = fe_mul(&u1, &hh);
    gej r;
    t = fe_sqr(&rr);
    t = fe_sub(&t, &hhh);
    u256 v2 = fe_add(&v, &v);
    r.x = fe_sub(&t, &v2);
    t = fe_sub(&v, &r.x);
    t = fe_mul(&rr, &t);
    u256 w = fe_mul(&s1, &hhh);
    r.y = fe_sub(&t, &w);
    t = fe_mul(&a->z, &b->z);
    r.z = fe_mul(&t, &h);
    r.inf = 0;
    return r;
}

static gej gej_mul(const gej* p, const u256* k) {
    gej r; r.inf = 1; r.x = r.y = r.z = fe_small(0);
    for (int i = 255; i >= 0; i--) {
        r = gej_double(&r);
        if ((k->v[i / 64] >> (i % 64)) & 1) r = gej_add(&r, p);
    }
    return r;
}

static void gej_to_affine(const gej* a, u256* x, u256* y) {
    u256 zi = mod_inv(&MODP, &a->z), zi2 = fe_sqr(&zi), zi3 = fe_mul(&zi2, &zi);
    *x = fe_mul(&a->x, &zi2);
    *y = fe_mul(&a->y, &zi3);
}

static int fe_is_on_curve(const u256* x, const u256* y) {
    u256 y2 = fe_sqr(y), x3 = fe_sqr(x);
    x3 = fe_mul(&x3, x);
    u256 seven = fe_small(7);
    x3 = fe_add(&x3, &seven);
    return u256_cmp(&y2, &x3) == 0;
}

/* ========================================================================================== */
/* Pubkey parse: CPubKey filter (pubkey.h:58-94) + eckey_pubkey_parse (eckey_impl.h:17-35)    */
/* ========================================================================================== */
static int pubkey_parse(const uint8_t* pub, size_t len, u256* x, u256* y) {
    if (len == 0) return 0;
    uint8_t h = pub[0];
    size_t want = (h == 2 || h == 3) ? 33 : (h == 4 || h == 6 || h == 7) ? 65 : 0;
    if (want == 0 || len != want) return 0; /* CPubKey::IsValid / eckey size+tag test */
    *x = u256_from_be(pub + 1);
    if (u256_cmp(x, &P) >= 0) return 0;     /* fe_set_b32 rejects >= p (field_5x52_impl.h) */
    if (want == 33) {
        u256 x3 = fe_sqr(x), seven = fe_small(7);
        x3 = fe_mul(&x3, x);
        x3 = fe_add(&x3, &seven);
        if (!fe_sqrt(y, &x3)) return 0;       /* ge_set_xo_var: no square root -> invalid */
        if ((int)(y->v[0] & 1) != (h == 3)) *y = mod_neg(&MODP, y);
        return 1;
    }
    *y = u256_from_be(pub + 33);
    if (u256_cmp(y, &P) >= 0) return 0;
    if ((h == 6 || h == 7) && (int)(y->v[0] & 1) != (h == 7)) return 0; /* hybrid parity */
    return fe_is_on_curve(x, y);           /* ge_is_valid_var */
}

int bcco_pubkey_parse(const uint8_t* pub, size_t len, uint8_t xo[32], uint8_t yo[32]) {
    u256 x, y;
    if (!pubkey_parse(pub, len, &x, &y)) return 0;
    u256_to_be(&x, xo);
    u256_to_be(&y, yo);
    return 1;
}

/* ========================================================================================== */
/* Lax DER (pubkey.cpp:28-168)                                                                */
/* ========================================================================================== */
/* reads an integer's length field; returns 0 on failure */
static int der_len(const uint8_t* in, size_t inlen, size_t* pos, size_t* out) {
    if (*pos == inlen) return 0;
    size_t lenbyte = in[(*pos)++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (lenbyte > inlen - *pos) return 0;
        while (lenbyte > 0 && in[*pos] == 0) { (*pos)++; lenbyte--; }
        if (lenbyte >= 4) return 0;
        size_t v = 0;
        while (lenbyte > 0) { v = (v << 8) + in[*pos]; (*pos)++; lenbyte--; }
        *out = v;
    } else {
        *out = lenbyte;
    }
    return 1;
}

int bcco_der_parse_lax(const uint8_t* in, size_t inlen, uint8_t r[32], uint8_t s[32]) {
    size_t pos = 0, rpos, rlen, spos, slen, lenbyte;
    uint8_t tmp[64];
    memset(tmp, 0, 64);
    memset(r, 0, 32);
    memset(s, 0, 32);
    if (pos == inlen || in[pos] != 0x30) return 0;
    pos++;
    if (pos == inlen) return 0;
    lenbyte = in[pos++];
    if (lenbyte & 0x80) {                 /* sequence length: skipped, only bounds-checked */
        lenbyte -= 0x80;
        if (lenbyte > inlen - pos) return 0;
        pos += lenbyte;
    }
    if (pos == inlen || in[pos] != 0x02) return 0;
    pos++;
    if (!der_len(in, inlen, &pos, &rlen)) return 0;
    if (rlen > inlen - pos) return 0;
    rpos = pos;
    pos += rlen;
    if (pos == inlen || in[pos] != 0x02) return 0;
    pos++;
    if (!der_len(in, inlen, &pos, &slen)) return 0;
    if (slen > inlen - pos) return 0;
    spos = pos;
    int overflow = 0;
    while (rlen > 0 && in[rpos] == 0) { rlen--; rpos++; }
    if (rlen > 32) overflow = 1; else memcpy(tmp + 32 - rlen, in + rpos, rlen);
    while (slen > 0 && in[spos] == 0) { slen--; spos++; }
    if (slen > 32) overflow = 1; else memcpy(tmp + 64 - slen, in + spos, slen);
    if (!overflow) {
        /* ecdsa_signature_parse_compact: r or s >= n is an overflow (secp256k1.c:358-377) */
        u256 rv = u256_from_be(tmp), sv = u256_from_be(tmp + 32);
        if (u256_cmp(&rv, &N) >= 0 || u256_cmp(&sv, &N) >= 0) overflow = 1;
    }
    if (overflow) memset(tmp, 0, 64);
    memcpy(r, tmp, 32);
    memcpy(s, tmp + 32, 32);
    return 1;
}

/* ========================================================================================== */
/* ECDSA verify (ecdsa_impl.h:207-275)                                                        */
/* ========================================================================================== */
static int ecdsa_verify_pt(const u256* qx, const u256* qy, const u256* rv, const u256* sv,
                           const uint8_t msg32[32]) {
    if (u256_is_zero(rv) || u256_is_zero(sv)) return 0;
    if (u256_cmp(rv, &N) >= 0 || u256_cmp(sv, &N) >= 0) return 0;
    /* m = msg mod n (scalar_set_b32 with overflow reduction) */
    u256 m = u256_from_be(msg32);
    if (u256_cmp(&m, &N) >= 0) u256_sub(&m, &m, &N);
    u256 sn = mod_inv(&MODN, sv);
    u256 u1 = mod_mul(&MODN, &m, &sn), u2 = mod_mul(&MODN, rv, &sn);
    gej g = gej_from_affine(&GX, &GY), q = gej_from_affine(qx, qy);
    gej a = gej_mul(&g, &u1), b = gej_mul(&q, &u2);
    gej R = gej_add(&a, &b);
    if (R.inf) return 0;
    /* xr * Z^2 == X, or (xr + n < p and (xr + n) * Z^2 == X) */
    u256 z2 = fe_sqr(&R.z);
    u256 lhs = fe_mul(rv, &z2);
    if (u256_cmp(&lhs, &R.x) == 0) return 1;
    u256 pmn, xr2;
    u256_sub(&pmn, &P, &N);
    if (u256_cmp(rv, &pmn) >= 0) return 0;
    u256_add(&xr2, rv, &N);
    lhs = fe_mul(&xr2, &z2);
    return u256_cmp(&lhs, &R.x) == 0;
}

int bcco_ecdsa_verify_raw(const uint8_t qx[32], const uint8_t qy[32], const uint8_t r[32],
                          const uint8_t s[32], const uint8_t msg32[32]) {
    u256 x = u256_from_be(qx), y = u256_from_be(qy), rv = u256_from_be(r), sv = u256_from_be(s);
    return ecdsa_verify_pt(&x, &y, &rv, &sv, msg32);
}

/* CPubKey::Verify (pubkey.cpp:191-207): parse key, lax-DER, normalize S, verify */
int bcco_pubkey_verify(const uint8_t* pub, size_t publen, const uint8_t hash32[32],
                       const uint8_t* sig, size_t siglen) {
    u256 x, y;
    uint8_t r[32], s[32];
    if (!pubkey_parse(pub, publen, &x, &y)) return 0;
    if (!bcco_der_parse_lax(sig, siglen, r, s)) return 0;
    u256 rv = u256_from_be(r), sv = u256_from_be(s);
    /* secp256k1_ecdsa_signature_normalize (secp256k1.c:404-421): s > n/2 -> n - s */
    u256 half = N;
    half.v[0] = (half.v[0] >> 1) | (half.v[1] << 63);
    half.v[1] = (half.v[1] >> 1) | (half.v[2] << 63);
    half.v[2] = (half.v[2] >> 1) | (half.v[3] << 63);
    half.v[3] >>= 1;
    if (u256_cmp(&sv, &half) > 0) u256_sub(&sv, &N, &sv);
    return ecdsa_verify_pt(&x, &y, &rv, &sv, hash32);
}

int bcco_ecmult_gen(const uint8_t k32[32], uint8_t xo[32], uint8_t yo[32]) {
    u256 k = u256_from_be(k32);
    if (u256_cmp(&k, &N) >= 0) u256_sub(&k, &k, &N);
    if (u256_is_zero(&k)) return 0;
    gej g = gej_from_affine(&GX, &GY);
    gej r = gej_mul(&g, &k);
    u256 x, y;
    gej_to_affine(&r, &x, &y);
    u256_to_be(&x, xo);
    u256_to_be(&y, yo);
    return 1;
}

/* ========================================================================================== */
/* BIP340 Schnorr verify (modules/schnorrsig/main_impl.h:190-237)                             */
/* ========================================================================================== */
int bcco_schnorr_verify(const uint8_t sig64[64], const uint8_t msg32[32], const uint8_t xonly32[32]) {
    u256 rx = u256_from_be(sig64), s = u256_from_be(sig64 + 32), px = u256_from_be(xonly32), py;
    if (u256_cmp(&rx, &P) >= 0) return 0;
    if (u256_cmp(&s, &N) >= 0) return 0;
    /* xonly_pubkey_parse: x < p, lift with even y (modules/extrakeys/main_impl.h:21-39) */
    if (u256_cmp(&px, &P) >= 0) return 0;
    {
        u256 x3 = fe_sqr(&px), seven = fe_small(7);
        x3 = fe_mul(&x3, &px);
        x3 = fe_add(&x3, &seven);
        if (!fe_sqrt(&py, &x3)) return 0;
        if (py.v[0] & 1) py = mod_neg(&MODP, &py);
    }
    /* e = tagged_hash("BIP0340/challenge", r || P || m) mod n */
    uint8_t tag[32], buf[32 * 5];
    bcco_sha256((const uint8_t*)"BIP0340/challenge", 17, tag);
    memcpy(buf, tag, 32);
    memcpy(buf + 32, tag, 32);
    memcpy(buf + 64, sig64, 32);
    memcpy(buf + 96, xonly32, 32);
    memcpy(buf + 128, msg32, 32);
    uint8_t eh[32];
    bcco_sha256(buf, sizeof buf, eh);
    u256 e = u256_from_be(eh);
    if (u256_cmp(&e, &N) >= 0) u256_sub(&e, &e, &N);
    u256 ne = mod_neg(&MODN, &e);
    gej g = gej_from_affine(&GX, &GY), pk = gej_from_affine(&px, &py);
    gej a = gej_mul(&g, &s), b = gej_mul(&pk, &ne);
    gej R = gej_add(&a, &b);
    if (R.inf) return 0;
    u256 x, y;
    gej_to_affine(&R, &x, &y);
    if (y.v[0] & 1) return 0;
    return u256_cmp(&x, &rx) == 0;
}

/* ========================================================================================== */
/* Transaction parse (primitives/transaction.h:188-224, serialize.h:318-347) + sighash        */
/* ========================================================================================== */
typedef struct {
    const uint8_t* prevout; /* 36 bytes */
    const uint8_t* script;
    size_t scriptlen;
    uint32_t sequence;
    int has_witness;        /* scriptWitness non-empty */
} txin_t;
typedef struct {
    const uint8_t* ser; /* serialized CTxOut: value(8) || compactsize || script */
    size_t serlen;
} txout_t;
typedef struct {
    int32_t version;
    uint32_t locktime;
    size_t nin, nout, ser_size;   /* ser_size: bytes consumed */
    txin_t* vin;
    txout_t* vout;
} tx_t;

typedef struct { const uint8_t* p; size_t n, pos; int bad; } rd_t;

static const uint8_t* rd_take(rd_t* r, size_t k) {
    if (r->bad || k > r->n - r->pos) { r->bad = 1; return NULL; }
    const uint8_t* q = r->p + r->pos;
    r->pos += k;
    return q;
}
static uint64_t rd_le(rd_t* r, int k) {
    const uint8_t* q = rd_take(r, (size_t)k);
    uint64_t v = 0;
    if (!q) return 0;
    for (int i = k - 1; i >= 0; i--) v = (v << 8) | q[i];
    return v;
}
static uint64_t rd_cs(rd_t* r) {
    uint64_t c = rd_le(r, 1), v;
    if (c < 253) v = c;
    else if (c == 253) { v = rd_le(r, 2); if (v < 253) r->bad = 1; }
    else if (c == 254) { v = rd_le(r, 4); if (v < 0x10000u) r->bad = 1; }
    else { v = rd_le(r, 8); if (v < 0x100000000ULL) r->bad = 1; }
    if (v > 0x02000000) r->bad = 1;
    return v;
}

static int parse_vin(rd_t* r, tx_t* tx) {
    uint64_t n = rd_cs(r);
    if (r->bad || n > r->n) return 0;
    tx->nin = (size_t)n;
    tx->vin = (txin_t*)calloc(n ? n : 1, sizeof(txin_t));
    for (size_t i = 0; i < n; i++) {
        tx->vin[i].prevout = rd_take(r, 36);
        uint64_t sl = rd_cs(r);
        tx->vin[i].script = rd_take(r, (size_t)sl);
        tx->vin[i].scriptlen = (size_t)sl;
        tx->vin[i].sequence = (uint32_t)rd_le(r, 4);
        if (r->bad) return 0;
    }
    return 1;
}

static int parse_vout(rd_t* r, tx_t* tx) {
    uint64_t n = rd_cs(r);
    if (r->bad || n > r->n) return 0;
    tx->nout = (size_t)n;
    tx->vout = (txout_t*)calloc(n ? n : 1, sizeof(txout_t));
    for (size_t i = 0; i < n; i++) {
        size_t start = r->pos;
        rd_take(r, 8);
        uint64_t sl = rd_cs(r);
        rd_take(r, (size_t)sl);
        if (r->bad) return 0;
        tx->vout[i].ser = r->p + start;
        tx->vout[i].serlen = r->pos - start;
    }
    return 1;
}

static int tx_parse(const uint8_t* p, size_t n, tx_t* tx) {
    rd_t r = {p, n, 0, 0};
    memset(tx, 0, sizeof *tx);
    tx->version = (int32_t)rd_le(&r, 4);
    if (!parse_vin(&r, tx)) return 0;
    uint8_t flags = 0;
    if (tx->nin == 0) {
        flags = (uint8_t)rd_le(&r, 1);
        if (flags != 0) {
            free(tx->vin);
            if (!parse_vin(&r, tx)) return 0;
            if (!parse_vout(&r, tx)) return 0;
        }
    } else {
        if (!parse_vout(&r, tx)) return 0;
    }
    if (flags & 1) {
        flags ^= 1;
        int any = 0;
        for (size_t i = 0; i < tx->nin; i++) {
            uint64_t k = rd_cs(&r);
            if (k) any = 1;
            tx->vin[i].has_witness = k != 0;
            for (uint64_t j = 0; j < k && !r.bad; j++) {
                uint64_t l = rd_cs(&r);
                rd_take(&r, (size_t)l);
            }
            if (r.bad) return 0;
        }
        if (!any) return 0;
    }
    if (flags) return 0;
    tx->locktime = (uint32_t)rd_le(&r, 4);
    tx->ser_size = r.pos;
    return !r.bad;
}

static void tx_free(tx_t* tx) { free(tx->vin); free(tx->vout); }

/* growable byte buffer */
typedef struct { uint8_t* p; size_t n, cap; } buf_t;
static void bput(buf_t* b, const void* d, size_t k) {
    if (b->n + k > b->cap) {
        b->cap = (b->n + k) * 2 + 64;
        b->p = (uint8_t*)realloc(b->p, b->cap);
    }
    memcpy(b->p + b->n, d, k);
    b->n += k;
}
static void bput_le(buf_t* b, uint64_t v, int k) {
    uint8_t t[8];
    for (int i = 0; i < k; i++) t[i] = (uint8_t)(v >> (8 * i));
    bput(b, t, (size_t)k);
}
static void bput_cs(buf_t* b, uint64_t v) {
    if (v < 253) bput_le(b, v, 1);
    else if (v <= 0xFFFF) { bput_le(b, 253, 1); bput_le(b, v, 2); }
    else if (v <= 0xFFFFFFFFULL) { bput_le(b, 254, 1); bput_le(b, v, 4); }
    else { bput_le(b, 255, 1); bput_le(b, v, 8); }
}

/* CScript::GetOp (script.cpp:283) — returns 0 at end or on a truncated push */
static int script_getop(const uint8_t* s, size_t n, size_t* pc, uint8_t* op) {
    if (*pc >= n) return 0;
    uint8_t o = s[(*pc)++];
    *op = o;
    if (o <= 0x4e) {
        size_t sz;
        if (o < 0x4c) sz = o;
        else if (o == 0x4c) { if (n - *pc < 1) return 0; sz = s[*pc]; *pc += 1; }
        else if (o == 0x4d) { if (n - *pc < 2) return 0; sz = s[*pc] | ((size_t)s[*pc + 1] << 8); *pc += 2; }
        else { if (n - *pc < 4) return 0; sz = s[*pc] | ((size_t)s[*pc + 1] << 8) | ((size_t)s[*pc + 2] << 16) | ((size_t)s[*pc + 3] << 24); *pc += 4; }
        if (n - *pc < sz) return 0;
        *pc += sz;
    }
    return 1;
}

/* SerializeScriptCode (interpreter.cpp:1293-1312): drop OP_CODESEPARATOR opcodes */
static void put_script_code(buf_t* b, const uint8_t* s, size_t n) {
    size_t pc = 0, ncs = 0;
    uint8_t op;
    while (script_getop(s, n, &pc, &op)) if (op == 0xab) ncs++;
    bput_cs(b, n - ncs);
    size_t begin = 0;
    pc = 0;
    while (script_getop(s, n, &pc, &op)) {
        if (op == 0xab) { bput(b, s + begin, pc - begin - 1); begin = pc; }
    }
    if (begin != n) bput(b, s + begin, pc - begin);
}

int bcco_sighash(const uint8_t* txb, size_t txlen, unsigned nIn, const uint8_t* script,
                 size_t scriptlen, int hashtype, int64_t amount, int sigversion, uint8_t out[32]) {
    tx_t tx;
    if (!tx_parse(txb, txlen, &tx)) { tx_free(&tx); return 0; }
    if (nIn >= tx.nin) { tx_free(&tx); return 0; }
    int acp = (hashtype & 0x80) != 0, base = hashtype & 0x1f;
    int single = base == 3, none = base == 2;
    buf_t b = {0};
    if (sigversion == 1) {
        /* BIP143 (interpreter.cpp:1581-1625, hashes :1366-1397) */
        uint8_t hp[32] = {0}, hs[32] = {0}, ho[32] = {0};
        if (!acp) {
            buf_t t = {0};
            for (size_t i = 0; i < tx.nin; i++) bput(&t, tx.vin[i].prevout, 36);
            bcco_sha256d(t.p, t.n, hp);
            free(t.p);
        }
        if (!acp && !single && !none) {
            buf_t t = {0};
            for (size_t i = 0; i < tx.nin; i++) bput_le(&t, tx.vin[i].sequence, 4);
            bcco_sha256d(t.p, t.n, hs);
            free(t.p);
        }
        if (!single && !none) {
            buf_t t = {0};
            for (size_t i = 0; i < tx.nout; i++) bput(&t, tx.vout[i].ser, tx.vout[i].serlen);
            bcco_sha256d(t.p, t.n, ho);
            free(t.p);
        } else if (single && nIn < tx.nout) {
            bcco_sha256d(tx.vout[nIn].ser, tx.vout[nIn].serlen, ho);
        }
        bput_le(&b, (uint32_t)tx.version, 4);
        bput(&b, hp, 32);
        bput(&b, hs, 32);
        bput(&b, tx.vin[nIn].prevout, 36);
        bput_cs(&b, scriptlen);
        bput(&b, script, scriptlen);
        bput_le(&b, (uint64_t)amount, 8);
        bput_le(&b, tx.vin[nIn].sequence, 4);
        bput(&b, ho, 32);
        bput_le(&b, tx.locktime, 4);
        bput_le(&b, (uint32_t)hashtype, 4);
        bcco_sha256d(b.p, b.n, out);
    } else {
        /* legacy: SIGHASH_SINGLE bug -> uint256::ONE (interpreter.cpp:1627-1633) */
        if (single && nIn >= tx.nout) {
            memset(out, 0, 32);
            out[0] = 1;
            tx_free(&tx);
            return 1;
        }
        /* CTransactionSignatureSerializer (interpreter.cpp:1273-1364) */
        bput_le(&b, (uint32_t)tx.version, 4);
        size_t nins = acp ? 1 : tx.nin;
        bput_cs(&b, nins);
        for (size_t k = 0; k < nins; k++) {
            size_t i = acp ? nIn : k;
            bput(&b, tx.vin[i].prevout, 36);
            if (i != nIn) bput_cs(&b, 0);
            else put_script_code(&b, script, scriptlen);
            if (i != nIn && (single || none)) bput_le(&b, 0, 4);
            else bput_le(&b, tx.vin[i].sequence, 4);
        }
        size_t nouts = none ? 0 : (single ? nIn + 1 : tx.nout);
        bput_cs(&b, nouts);
        for (size_t o = 0; o < nouts; o++) {
            if (single && o != nIn) { bput_le(&b, (uint64_t)-1, 8); bput_cs(&b, 0); }
            else bput(&b, tx.vout[o].ser, tx.vout[o].serlen);
        }
        bput_le(&b, tx.locktime, 4);
        bput_le(&b, (uint32_t)hashtype, 4);
        bcco_sha256d(b.p, b.n, out);
    }
    free(b.p);
    tx_free(&tx);
    return 1;
}

/* ========================================================================================== */
/* BIP341 / BIP342 signature hash + CheckSchnorrSignature                                     */
/* ========================================================================================== */
/* std::vector<CTxOut> (serialize.h:318-347 vector rule): compactsize count, then per output
 * value(8) || compactsize || script.  Fills out[] (the serialized CTxOut of each entry). */
static int spent_parse(const uint8_t* p, size_t n, txout_t** out, size_t* cnt) {
    rd_t r = {p, n, 0, 0};
    uint64_t k = rd_cs(&r);
    if (r.bad || k > n) return 0;
    *cnt = (size_t)k;
    *out = (txout_t*)calloc(k ? k : 1, sizeof(txout_t));
    for (size_t i = 0; i < k; i++) {
        size_t start = r.pos;
        rd_take(&r, 8);
        uint64_t sl = rd_cs(&r);
        rd_take(&r, (size_t)sl);
        if (r.bad) return 0;
        (*out)[i].ser = p + start;
        (*out)[i].serlen = r.pos - start;
    }
    return r.pos == n;
}

/* SHA256(SHA256(tag) || SHA256(tag) || msg) (hash.cpp TaggedHash + CHashWriter::GetSHA256) */
static void tagged_sha256(const char* tag, const uint8_t* m, size_t n, uint8_t out[32]) {
    uint8_t th[32];
    bcco_sha256((const uint8_t*)tag, strlen(tag), th);
    sha256_ctx c;
    sha256_init(&c);
    sha256_write(&c, th, 32);
    sha256_write(&c, th, 32);
    sha256_write(&c, m, n);
    sha256_final(&c, out);
}

/* SignatureHashSchnorr (interpreter.cpp:1491-1574) with PrecomputedTransactionData::Init's
 * single-SHA256 tx hashes (:1366-1417, :1455-1471) and the annex hash of
 * VerifyWitnessProgram (:1889-1893: SHA256 of the annex serialized with its compactsize). */
int bcco_sighash_schnorr(const uint8_t* txb, size_t txlen, const uint8_t* spent, size_t spentlen,
                         unsigned nIn, int hash_type, int sigversion, const uint8_t* annex,
                         size_t annexlen, const uint8_t tapleaf32[32], uint32_t codesep_pos,
                         uint8_t out[32]) {
    tx_t tx;
    txout_t* so = NULL;
    size_t nso = 0;
    int rc = -1;
    if (!tx_parse(txb, txlen, &tx) || tx.ser_size != txlen) { tx_free(&tx); return -1; }
    if (!spent_parse(spent, spentlen, &so, &nso) || nso != tx.nin || nIn >= tx.nin) goto done;
    {
        /* m_bip341_taproot_ready (Init :1436-1452): some witness-bearing input spends a 34-byte
         * scriptPubKey starting with OP_1; SignatureHashSchnorr asserts it (:1512) */
        int ready = 0;
        for (size_t i = 0; i < tx.nin; i++) {
            const uint8_t* spk = so[i].ser + 8;
            size_t spkl = so[i].serlen - 8;
            if (tx.vin[i].has_witness && spkl == 35 && spk[0] == 34 && spk[1] == 0x51) ready = 1;
        }
        if (!ready) goto done;
    }
    rc = 0;
    {
        const int output_type = hash_type == 0 ? 1 : (hash_type & 3);
        const int input_type = hash_type & 0x80;
        if (!(hash_type <= 0x03 || (hash_type >= 0x81 && hash_type <= 0x83))) goto done;
        if (output_type == 3 && nIn >= tx.nout) goto done;
        buf_t b = {0};
        bput_le(&b, 0, 1);                          /* epoch */
        bput_le(&b, (uint64_t)hash_type, 1);
        bput_le(&b, (uint32_t)tx.version, 4);
        bput_le(&b, tx.locktime, 4);
        if (!input_type) {
            uint8_t h[32];
            buf_t t = {0};
            for (size_t i = 0; i < tx.nin; i++) bput(&t, tx.vin[i].prevout, 36);
            bcco_sha256(t.p, t.n, h); bput(&b, h, 32); t.n = 0;
            for (size_t i = 0; i < nso; i++) bput(&t, so[i].ser, 8);
            bcco_sha256(t.p, t.n, h); bput(&b, h, 32); t.n = 0;
            for (size_t i = 0; i < nso; i++) bput(&t, so[i].ser + 8, so[i].serlen - 8);
            bcco_sha256(t.p, t.n, h); bput(&b, h, 32); t.n = 0;
            for (size_t i = 0; i < tx.nin; i++) bput_le(&t, tx.vin[i].sequence, 4);
            bcco_sha256(t.p, t.n, h); bput(&b, h, 32);
            free(t.p);
        }
        if (output_type == 1) {
            uint8_t h[32];
            buf_t t = {0};
            for (size_t i = 0; i < tx.nout; i++) bput(&t, tx.vout[i].ser, tx.vout[i].serlen);
            bcco_sha256(t.p, t.n, h);
            bput(&b, h, 32);
            free(t.p);
        }
        const int ext_flag = sigversion == 1 ? 1 : 0;
        bput_le(&b, (uint64_t)((ext_flag << 1) + (annex ? 1 : 0)), 1);   /* spend_type */
        if (input_type) {
            bput(&b, tx.vin[nIn].prevout, 36);
            bput(&b, so[nIn].ser, so[nIn].serlen);
            bput_le(&b, tx.vin[nIn].sequence, 4);
        } else {
            bput_le(&b, nIn, 4);
        }
        if (annex) {
            uint8_t h[32];
            buf_t t = {0};
            bput_cs(&t, annexlen);
            bput(&t, annex, annexlen);
            bcco_sha256(t.p, t.n, h);
            bput(&b, h, 32);
            free(t.p);
        }
        if (output_type == 3) {
            uint8_t h[32];
            bcco_sha256(tx.vout[nIn].ser, tx.vout[nIn].serlen, h);
            bput(&b, h, 32);
        }
        if (sigversion == 1) {
            bput(&b, tapleaf32, 32);
            bput_le(&b, 0, 1);                      /* key_version */
            bput_le(&b, codesep_pos, 4);
        }
        tagged_sha256("TapSighash", b.p, b.n, out);
        free(b.p);
        rc = 1;
    }
done:
    free(so);
    tx_free(&tx);
    return rc;
}

/* GenericTransactionSignatureChecker::CheckSchnorrSignature (interpreter.cpp:1678-1704):
 * returns 1 (valid) or 0 with *serror = SCHNORR_SIG_SIZE / SCHNORR_SIG_HASHTYPE / SCHNORR_SIG
 * (script_error.h:73-75 values), or -1 if the tx / spent outputs do not parse or nIn is out of
 * range (the reference asserts there).  sighash32 (optional) receives the signature hash. */
int bcco_taproot_check(const uint8_t* txb, size_t txlen, const uint8_t* spent, size_t spentlen,
                       unsigned nIn, const uint8_t* sig, size_t siglen, const uint8_t pk32[32],
                       int sigversion, const uint8_t* annex, size_t annexlen,
                       const uint8_t tapleaf32[32], uint32_t codesep_pos, int* serror,
                       uint8_t* sighash32) {
    enum { ERR_SIZE = 44, ERR_HASHTYPE = 45, ERR_SIG = 46 };
    uint8_t h[32];
    *serror = 0;
    /* the checker only exists for a parsed tx with its spent outputs (PrecomputedTransactionData
     * asserts their count): inputs that do not meet that are refused before any check */
    if (bcco_sighash_schnorr(txb, txlen, spent, spentlen, nIn, 0, sigversion, annex, annexlen,
                             tapleaf32, codesep_pos, h) < 0)
        return -1;
    if (siglen != 64 && siglen != 65) { *serror = ERR_SIZE; return 0; }
    int hash_type = 0;
    if (siglen == 65) {
        hash_type = sig[64];
        if (hash_type == 0) { *serror = ERR_HASHTYPE; return 0; }
    }
    int rc = bcco_sighash_schnorr(txb, txlen, spent, spentlen, nIn, hash_type, sigversion, annex,
                                  annexlen, tapleaf32, codesep_pos, h);
    if (rc < 0) return -1;
    if (rc == 0) { *serror = ERR_HASHTYPE; return 0; }
    if (sighash32) memcpy(sighash32, h, 32);
    if (!bcco_schnorr_verify(sig, h, pk32)) { *serror = ERR_SIG; return 0; }
    return 1;
}
