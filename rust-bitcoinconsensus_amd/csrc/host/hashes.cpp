// Host hash functions (see hashes.h).  Straightforward implementations of the published
// algorithms (FIPS 180-4 SHA-256 / SHA-1, Dobbertin-Bosselaers-Preneel RIPEMD-160).
#include "hashes.h"

#include <cstdlib>
#include <cstring>
#include <utility>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace bcc {
namespace host {

namespace {

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
inline uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

void sha256_block_portable(uint32_t s[8], const uint8_t* blk) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = be32(blk + 4 * i);
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

#if defined(__x86_64__)
// The same compression with the x86 SHA extensions (sha256rnds2 / sha256msg1 / sha256msg2),
// selected at run time when the host CPU has them.  State in the ABEF / CDGH register layout
// the instructions use; message words scheduled four at a time.
__attribute__((target("sha,sse4.1"))) void sha256_block_shani(uint32_t s[8], const uint8_t* blk) {
    const __m128i BSWAP = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i tmp = _mm_loadu_si128((const __m128i*)&s[0]);
    __m128i st1 = _mm_loadu_si128((const __m128i*)&s[4]);
    tmp = _mm_shuffle_epi32(tmp, 0xB1);              // CDAB
    st1 = _mm_shuffle_epi32(st1, 0x1B);              // EFGH
    __m128i st0 = _mm_alignr_epi8(tmp, st1, 8);      // ABEF
    st1 = _mm_blend_epi16(st1, tmp, 0xF0);           // CDGH
    const __m128i save0 = st0, save1 = st1;
    __m128i w[4];
    for (int g = 0; g < 16; g++) {
        if (g < 4) {
            w[g] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(blk + 16 * g)), BSWAP);
        } else {
            __m128i t = _mm_sha256msg1_epu32(w[(g - 4) & 3], w[(g - 3) & 3]);
            t = _mm_add_epi32(t, _mm_alignr_epi8(w[(g - 1) & 3], w[(g - 2) & 3], 4));
            w[g & 3] = _mm_sha256msg2_epu32(t, w[(g - 1) & 3]);
        }
        __m128i m = _mm_add_epi32(w[g & 3], _mm_loadu_si128((const __m128i*)&K256[4 * g]));
        st1 = _mm_sha256rnds2_epu32(st1, st0, m);
        m = _mm_shuffle_epi32(m, 0x0E);
        st0 = _mm_sha256rnds2_epu32(st0, st1, m);
    }
    st0 = _mm_add_epi32(st0, save0);
    st1 = _mm_add_epi32(st1, save1);
    tmp = _mm_shuffle_epi32(st0, 0x1B);              // FEBA
    st1 = _mm_shuffle_epi32(st1, 0xB1);              // DCHG
    st0 = _mm_blend_epi16(tmp, st1, 0xF0);           // DCBA
    st1 = _mm_alignr_epi8(st1, tmp, 8);              // HGFE
    _mm_storeu_si128((__m128i*)&s[0], st0);
    _mm_storeu_si128((__m128i*)&s[4], st1);
}

// Two independent single-block compressions from the IV, interleaved: the SHA round instructions
// are latency-bound, so two chains side by side take little longer than one.
__attribute__((target("sha,sse4.1"))) void sha256_iv_block_shani_x2(const uint8_t* b0,
                                                                     const uint8_t* b1,
                                                                     uint32_t o0[8], uint32_t o1[8]) {
    const __m128i BSWAP = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    // the IV as ABEF / CDGH
    const __m128i iv0 = _mm_set_epi32(0x6a09e667, 0xbb67ae85, 0x510e527f, 0x9b05688c);
    const __m128i iv1 = _mm_set_epi32(0x3c6ef372, 0xa54ff53a, 0x1f83d9ab, 0x5be0cd19);
    __m128i a0 = iv0, a1 = iv1, c0 = iv0, c1 = iv1;
    __m128i w[4], v[4];
    for (int g = 0; g < 16; g++) {
        if (g < 4) {
            w[g] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(b0 + 16 * g)), BSWAP);
            v[g] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(b1 + 16 * g)), BSWAP);
        } else {
            __m128i t = _mm_sha256msg1_epu32(w[(g - 4) & 3], w[(g - 3) & 3]);
            __m128i u = _mm_sha256msg1_epu32(v[(g - 4) & 3], v[(g - 3) & 3]);
            t = _mm_add_epi32(t, _mm_alignr_epi8(w[(g - 1) & 3], w[(g - 2) & 3], 4));
            u = _mm_add_epi32(u, _mm_alignr_epi8(v[(g - 1) & 3], v[(g - 2) & 3], 4));
            w[g & 3] = _mm_sha256msg2_epu32(t, w[(g - 1) & 3]);
            v[g & 3] = _mm_sha256msg2_epu32(u, v[(g - 1) & 3]);
        }
        const __m128i k = _mm_loadu_si128((const __m128i*)&K256[4 * g]);
        __m128i m = _mm_add_epi32(w[g & 3], k), n = _mm_add_epi32(v[g & 3], k);
        a1 = _mm_sha256rnds2_epu32(a1, a0, m);
        c1 = _mm_sha256rnds2_epu32(c1, c0, n);
        m = _mm_shuffle_epi32(m, 0x0E);
        n = _mm_shuffle_epi32(n, 0x0E);
        a0 = _mm_sha256rnds2_epu32(a0, a1, m);
        c0 = _mm_sha256rnds2_epu32(c0, c1, n);
    }
    a0 = _mm_add_epi32(a0, iv0);
    a1 = _mm_add_epi32(a1, iv1);
    c0 = _mm_add_epi32(c0, iv0);
    c1 = _mm_add_epi32(c1, iv1);
    __m128i t0 = _mm_shuffle_epi32(a0, 0x1B), t1 = _mm_shuffle_epi32(c0, 0x1B);  // FEBA
    a1 = _mm_shuffle_epi32(a1, 0xB1);                                              // DCHG
    c1 = _mm_shuffle_epi32(c1, 0xB1);
    _mm_storeu_si128((__m128i*)&o0[0], _mm_blend_epi16(t0, a1, 0xF0));  // DCBA
    _mm_storeu_si128((__m128i*)&o0[4], _mm_alignr_epi8(a1, t0, 8));     // HGFE
    _mm_storeu_si128((__m128i*)&o1[0], _mm_blend_epi16(t1, c1, 0xF0));
    _mm_storeu_si128((__m128i*)&o1[4], _mm_alignr_epi8(c1, t1, 8));
}
#endif

using BlockFn = void (*)(uint32_t*, const uint8_t*);
BlockFn pick_sha256_block() {
#if defined(__x86_64__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1") && !getenv("BCC_NO_SHANI"))
        return sha256_block_shani;
#endif
    return sha256_block_portable;
}
const BlockFn sha256_block = pick_sha256_block();

}  // namespace

bool sha256_uses_shani() { return sha256_block != sha256_block_portable; }

Sha256::Sha256() : bytes(0) {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(s, iv, sizeof s);
}

Sha256& Sha256::write(const uint8_t* p, size_t n) {
    size_t fill = (size_t)(bytes & 63);
    bytes += n;
    if (fill) {
        size_t take = 64 - fill < n ? 64 - fill : n;
        memcpy(buf + fill, p, take);
        p += take;
        n -= take;
        if (fill + take < 64) return *this;
        sha256_block(s, buf);
    }
    while (n >= 64) {
        sha256_block(s, p);
        p += 64;
        n -= 64;
    }
    if (n) memcpy(buf, p, n);
    return *this;
}

void Sha256::finalize(uint8_t out[32]) {
    uint64_t bits = bytes * 8;
    uint8_t pad[72];
    size_t padlen = 1 + ((119 - (bytes % 64)) % 64);
    memset(pad, 0, sizeof pad);
    pad[0] = 0x80;
    for (int i = 0; i < 8; i++) pad[padlen + i] = (uint8_t)(bits >> (56 - 8 * i));
    write(pad, padlen + 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(s[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s[i] >> 8);
        out[4 * i + 3] = (uint8_t)s[i];
    }
}

void sha256(const uint8_t* p, size_t n, uint8_t out[32]) {
    if (n <= 55) {  // one padded block built in place (keys, digests): a single compression
        alignas(16) uint8_t blk[64];
        memcpy(blk, p, n);
        blk[n] = 0x80;
        memset(blk + n + 1, 0, 55 - n);
        const uint64_t bits = (uint64_t)n * 8;
        for (int i = 0; i < 8; i++) blk[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
        uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        sha256_block(st, blk);
        for (int i = 0; i < 8; i++) {
            out[4 * i] = (uint8_t)(st[i] >> 24);
            out[4 * i + 1] = (uint8_t)(st[i] >> 16);
            out[4 * i + 2] = (uint8_t)(st[i] >> 8);
            out[4 * i + 3] = (uint8_t)st[i];
        }
        return;
    }
    Sha256().write(p, n).finalize(out);
}

void sha256d(const uint8_t* p, size_t n, uint8_t out[32]) {
    uint8_t t[32];
    sha256(p, n, t);
    sha256(t, 32, out);
}

// ---------------------------------------------------------------- SHA-1 (crypto/sha1.cpp)
void sha1(const uint8_t* p, size_t n, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    uint64_t bits = (uint64_t)n * 8;
    size_t total = ((n + 8) / 64 + 1) * 64;
    for (size_t off = 0; off < total; off += 64) {
        uint8_t blk[64];
        for (int i = 0; i < 64; i++) {
            size_t k = off + i;
            uint8_t v;
            if (k < n) v = p[k];
            else if (k == n) v = 0x80;
            else if (k >= total - 8) v = (uint8_t)(bits >> (8 * (total - 1 - k)));
            else v = 0;
            blk[i] = v;
        }
        uint32_t w[80];
        for (int i = 0; i < 16; i++) w[i] = be32(blk + 4 * i);
        for (int i = 16; i < 80; i++) w[i] = rotl(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
        for (int i = 0; i < 80; i++) {
            uint32_t f, k;
            if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999; }
            else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1; }
            else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDC; }
            else { f = b ^ c ^ d; k = 0xCA62C1D6; }
            uint32_t t = rotl(a, 5) + f + e + k + w[i];
            e = d; d = c; c = rotl(b, 30); b = a; a = t;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
    }
    for (int i = 0; i < 5; i++) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

// ---------------------------------------------------------------- RIPEMD-160 (crypto/ripemd160.cpp)
namespace {
const uint8_t RL[80] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                        7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9, 5, 2, 14, 11, 8,
                        3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12,
                        1, 9, 11, 10, 0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2,
                        4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13};
const uint8_t RR[80] = {5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12,
                        6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8, 12, 4, 9, 1, 2,
                        15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13,
                        8, 6, 4, 1, 3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14,
                        12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11};
const uint8_t SL[80] = {11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8,
                        7, 6, 8, 13, 11, 9, 7, 15, 7, 12, 15, 9, 11, 7, 13, 12,
                        11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5,
                        11, 12, 14, 15, 14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12,
                        9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6};
const uint8_t SR[80] = {8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6,
                        9, 13, 15, 7, 12, 8, 9, 11, 7, 7, 12, 7, 6, 15, 13, 11,
                        9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5,
                        15, 5, 8, 11, 14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8,
                        8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11};
const uint32_t KL[5] = {0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E};
const uint32_t KR[5] = {0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000};

inline uint32_t rf(int j, uint32_t x, uint32_t y, uint32_t z) {
    switch (j / 16) {
        case 0: return x ^ y ^ z;
        case 1: return (x & y) | (~x & z);
        case 2: return (x | ~y) ^ z;
        case 3: return (x & z) | (y & ~z);
        default: return x ^ (y | ~z);
    }
}

// One compression; fully unrolled so every selector, index and rotation is a constant.
void ripemd160_block(uint32_t h[5], const uint8_t* blk) {
    uint32_t X[16];
    for (int i = 0; i < 16; i++) X[i] = le32(blk + 4 * i);
    uint32_t al = h[0], bl = h[1], cl = h[2], dl = h[3], el = h[4];
    uint32_t ar = h[0], br = h[1], cr = h[2], dr = h[3], er = h[4];
#pragma GCC unroll 80
    for (int j = 0; j < 80; j++) {
        uint32_t t = rotl(al + rf(j, bl, cl, dl) + X[RL[j]] + KL[j / 16], SL[j]) + el;
        al = el; el = dl; dl = rotl(cl, 10); cl = bl; bl = t;
        t = rotl(ar + rf(79 - j, br, cr, dr) + X[RR[j]] + KR[j / 16], SR[j]) + er;
        ar = er; er = dr; dr = rotl(cr, 10); cr = br; br = t;
    }
    uint32_t t = h[1] + cl + dr;
    h[1] = h[2] + dl + er;
    h[2] = h[3] + el + ar;
    h[3] = h[4] + al + br;
    h[4] = h[0] + bl + cr;
    h[0] = t;
}
}  // namespace

void ripemd160(const uint8_t* p, size_t n, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    size_t full = n / 64;
    for (size_t b = 0; b < full; b++) ripemd160_block(h, p + 64 * b);
    // tail + padding (one or two blocks), length little-endian
    uint8_t tail[128];
    const size_t rem = n - 64 * full, tl = rem < 56 ? 64 : 128;
    memset(tail, 0, tl);
    if (rem) memcpy(tail, p + 64 * full, rem);
    tail[rem] = 0x80;
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; i++) tail[tl - 8 + i] = (uint8_t)(bits >> (8 * i));
    ripemd160_block(h, tail);
    if (tl == 128) ripemd160_block(h, tail + 64);
    for (int i = 0; i < 5; i++) {
        out[4 * i] = (uint8_t)h[i];
        out[4 * i + 1] = (uint8_t)(h[i] >> 8);
        out[4 * i + 2] = (uint8_t)(h[i] >> 16);
        out[4 * i + 3] = (uint8_t)(h[i] >> 24);
    }
}

// RIPEMD-160 of eight 32-byte messages at once (the second half of HASH160), one message per
// 32-bit lane of AVX2 registers: the same 80 double-line steps as ripemd160_block, unrolled so
// that selectors, word indices and rotations are constants.
namespace {
#define RV_ROL(x, n) _mm256_or_si256(_mm256_slli_epi32((x), (n)), _mm256_srli_epi32((x), 32 - (n)))
__attribute__((target("avx2"))) inline __m256i rfv(int j, __m256i x, __m256i y, __m256i z) {
    const __m256i ones = _mm256_set1_epi32(-1);
    switch (j / 16) {
        case 0: return _mm256_xor_si256(_mm256_xor_si256(x, y), z);
        case 1: return _mm256_or_si256(_mm256_and_si256(x, y), _mm256_andnot_si256(x, z));
        case 2: return _mm256_xor_si256(_mm256_or_si256(x, _mm256_xor_si256(y, ones)), z);
        case 3: return _mm256_or_si256(_mm256_and_si256(x, z), _mm256_andnot_si256(z, y));
        default: return _mm256_xor_si256(x, _mm256_or_si256(y, _mm256_xor_si256(z, ones)));
    }
}

__attribute__((target("avx2"))) void ripemd160_32x8_avx2(const uint8_t* const in[8],
                                                          uint8_t* const out[8]) {
    __m256i X[16];
    for (int w = 0; w < 8; w++)
        X[w] = _mm256_setr_epi32((int)le32(in[0] + 4 * w), (int)le32(in[1] + 4 * w),
                                 (int)le32(in[2] + 4 * w), (int)le32(in[3] + 4 * w),
                                 (int)le32(in[4] + 4 * w), (int)le32(in[5] + 4 * w),
                                 (int)le32(in[6] + 4 * w), (int)le32(in[7] + 4 * w));
    X[8] = _mm256_set1_epi32(0x80);  // padding of a 32-byte message: 0x80, zeros, bit length 256
    for (int w = 9; w < 16; w++) X[w] = _mm256_setzero_si256();
    X[14] = _mm256_set1_epi32(256);
    const uint32_t H[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    __m256i al = _mm256_set1_epi32((int)H[0]), bl = _mm256_set1_epi32((int)H[1]),
            cl = _mm256_set1_epi32((int)H[2]), dl = _mm256_set1_epi32((int)H[3]),
            el = _mm256_set1_epi32((int)H[4]);
    __m256i ar = al, br = bl, cr = cl, dr = dl, er = el;
#pragma GCC unroll 80
    for (int j = 0; j < 80; j++) {
        __m256i t = _mm256_add_epi32(_mm256_add_epi32(al, rfv(j, bl, cl, dl)),
                                     _mm256_add_epi32(X[RL[j]], _mm256_set1_epi32((int)KL[j / 16])));
        t = _mm256_add_epi32(RV_ROL(t, SL[j]), el);
        al = el; el = dl; dl = RV_ROL(cl, 10); cl = bl; bl = t;
        t = _mm256_add_epi32(_mm256_add_epi32(ar, rfv(79 - j, br, cr, dr)),
                             _mm256_add_epi32(X[RR[j]], _mm256_set1_epi32((int)KR[j / 16])));
        t = _mm256_add_epi32(RV_ROL(t, SR[j]), er);
        ar = er; er = dr; dr = RV_ROL(cr, 10); cr = br; br = t;
    }
    __m256i h[5];
    h[0] = _mm256_add_epi32(_mm256_add_epi32(_mm256_set1_epi32((int)H[1]), cl), dr);
    h[1] = _mm256_add_epi32(_mm256_add_epi32(_mm256_set1_epi32((int)H[2]), dl), er);
    h[2] = _mm256_add_epi32(_mm256_add_epi32(_mm256_set1_epi32((int)H[3]), el), ar);
    h[3] = _mm256_add_epi32(_mm256_add_epi32(_mm256_set1_epi32((int)H[4]), al), br);
    h[4] = _mm256_add_epi32(_mm256_add_epi32(_mm256_set1_epi32((int)H[0]), bl), cr);
    alignas(32) uint32_t v[5][8];
    for (int k = 0; k < 5; k++) _mm256_store_si256(reinterpret_cast<__m256i*>(v[k]), h[k]);
    for (int m = 0; m < 8; m++)
        for (int k = 0; k < 5; k++)
            for (int b = 0; b < 4; b++) out[m][4 * k + b] = (uint8_t)(v[k][m] >> (8 * b));
}
#undef RV_ROL

bool have_avx2() {
    static const bool v = __builtin_cpu_supports("avx2") && !getenv("BCC_NO_AVX2");
    return v;
}

// The same with sixteen messages in the 32-bit lanes of AVX-512 registers: rotations are one
// vprold and every selector function one vpternlogd (truth tables below), about half the
// instructions of the AVX2 step per message.
template <int J>
__attribute__((target("avx512f"))) inline __m512i rf16(__m512i x, __m512i y, __m512i z) {
    // imm8 = f(x, y, z) over the truth-table index (x << 2) | (y << 1) | z
    constexpr int T = J / 16 == 0 ? 0x96   /* x ^ y ^ z */
                    : J / 16 == 1 ? 0xCA   /* (x & y) | (~x & z) */
                    : J / 16 == 2 ? 0x59   /* (x | ~y) ^ z */
                    : J / 16 == 3 ? 0xE4   /* (x & z) | (y & ~z) */
                                  : 0x2D;  /* x ^ (y | ~z) */
    return _mm512_ternarylogic_epi32(x, y, z, T);
}

template <int J>
__attribute__((target("avx512f"))) inline void rstep16(__m512i& a, __m512i& b, __m512i& c,
                                                       __m512i& d, __m512i& e, __m512i& a2,
                                                       __m512i& b2, __m512i& c2, __m512i& d2,
                                                       __m512i& e2, const __m512i* X) {
    static constexpr uint32_t KLc[5] = {0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E};
    static constexpr uint32_t KRc[5] = {0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000};
    __m512i t = _mm512_add_epi32(_mm512_add_epi32(a, rf16<J>(b, c, d)),
                                 _mm512_add_epi32(X[RL[J]], _mm512_set1_epi32((int)KLc[J / 16])));
    t = _mm512_add_epi32(_mm512_rolv_epi32(t, _mm512_set1_epi32(SL[J])), e);
    a = e; e = d; d = _mm512_rol_epi32(c, 10); c = b; b = t;
    t = _mm512_add_epi32(_mm512_add_epi32(a2, rf16<79 - J>(b2, c2, d2)),
                         _mm512_add_epi32(X[RR[J]], _mm512_set1_epi32((int)KRc[J / 16])));
    t = _mm512_add_epi32(_mm512_rolv_epi32(t, _mm512_set1_epi32(SR[J])), e2);
    a2 = e2; e2 = d2; d2 = _mm512_rol_epi32(c2, 10); c2 = b2; b2 = t;
}

template <int... J>
__attribute__((target("avx512f"))) inline void rsteps16(std::integer_sequence<int, J...>,
                                                        __m512i (&v)[10], const __m512i* X) {
    (rstep16<J>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], X), ...);
}

__attribute__((target("avx512f"))) void ripemd160_32x16_avx512(const uint8_t* const in[16],
                                                              uint8_t* const out[16]) {
    __m512i X[16];
    alignas(64) uint32_t col[16];
    for (int w = 0; w < 8; w++) {
        for (int m = 0; m < 16; m++) col[m] = le32(in[m] + 4 * w);
        X[w] = _mm512_load_si512(col);
    }
    X[8] = _mm512_set1_epi32(0x80);  // padding of a 32-byte message: 0x80, zeros, bit length 256
    for (int w = 9; w < 16; w++) X[w] = _mm512_setzero_si512();
    X[14] = _mm512_set1_epi32(256);
    const uint32_t H[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    __m512i v[10];
    for (int k = 0; k < 5; k++) v[k] = v[5 + k] = _mm512_set1_epi32((int)H[k]);
    rsteps16(std::make_integer_sequence<int, 80>{}, v, X);
    // v: al bl cl dl el | ar br cr dr er
    __m512i h[5];
    h[0] = _mm512_add_epi32(_mm512_add_epi32(_mm512_set1_epi32((int)H[1]), v[2]), v[8]);
    h[1] = _mm512_add_epi32(_mm512_add_epi32(_mm512_set1_epi32((int)H[2]), v[3]), v[9]);
    h[2] = _mm512_add_epi32(_mm512_add_epi32(_mm512_set1_epi32((int)H[3]), v[4]), v[5]);
    h[3] = _mm512_add_epi32(_mm512_add_epi32(_mm512_set1_epi32((int)H[4]), v[0]), v[6]);
    h[4] = _mm512_add_epi32(_mm512_add_epi32(_mm512_set1_epi32((int)H[0]), v[1]), v[7]);
    alignas(64) uint32_t o[5][16];
    for (int k = 0; k < 5; k++) _mm512_store_si512(o[k], h[k]);
    for (int m = 0; m < 16; m++)
        for (int k = 0; k < 5; k++) memcpy(out[m] + 4 * k, &o[k][m], 4);  // little-endian words
}

// SHA-256 of sixteen single-block messages (<= 55 bytes) in the 32-bit lanes of AVX-512
// registers: Sigma / sigma as vprold + vpternlogd, Ch / Maj one vpternlogd each.  Digests as
// big-endian bytes to out[m].
__attribute__((target("avx512f"))) void sha256_x16_avx512(const uint8_t* const p[16],
                                                         const size_t n[16], uint8_t* const out[16]) {
    alignas(64) uint8_t blk[16][64];
    for (int m = 0; m < 16; m++) {
        memcpy(blk[m], p[m], n[m]);
        blk[m][n[m]] = 0x80;
        memset(blk[m] + n[m] + 1, 0, 55 - n[m]);
        const uint64_t bits = (uint64_t)n[m] * 8;
        for (int i = 0; i < 8; i++) blk[m][56 + i] = (uint8_t)(bits >> (56 - 8 * i));
    }
    __m512i W[16];
    alignas(64) uint32_t col[16];
    for (int w = 0; w < 16; w++) {
        for (int m = 0; m < 16; m++) col[m] = be32(blk[m] + 4 * w);
        W[w] = _mm512_load_si512(col);
    }
    static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    __m512i a = _mm512_set1_epi32((int)IV[0]), b = _mm512_set1_epi32((int)IV[1]),
            c = _mm512_set1_epi32((int)IV[2]), d = _mm512_set1_epi32((int)IV[3]),
            e = _mm512_set1_epi32((int)IV[4]), f = _mm512_set1_epi32((int)IV[5]),
            g = _mm512_set1_epi32((int)IV[6]), h = _mm512_set1_epi32((int)IV[7]);
    for (int i = 0; i < 64; i++) {
        __m512i w;
        if (i < 16) {
            w = W[i];
        } else {  // W[i % 16] += sigma1(W[i-2]) + W[i-7] + sigma0(W[i-15])
            const __m512i x15 = W[(i - 15) & 15], x2 = W[(i - 2) & 15];
            const __m512i s0 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(x15, 7), _mm512_ror_epi32(x15, 18),
                                                         _mm512_srli_epi32(x15, 3), 0x96);
            const __m512i s1 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(x2, 17), _mm512_ror_epi32(x2, 19),
                                                         _mm512_srli_epi32(x2, 10), 0x96);
            w = W[i & 15] = _mm512_add_epi32(_mm512_add_epi32(W[i & 15], s0),
                                             _mm512_add_epi32(W[(i - 7) & 15], s1));
        }
        const __m512i S1 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(e, 6), _mm512_ror_epi32(e, 11),
                                                     _mm512_ror_epi32(e, 25), 0x96);
        const __m512i ch = _mm512_ternarylogic_epi32(e, f, g, 0xCA);   // (e & f) | (~e & g)
        const __m512i t1 = _mm512_add_epi32(_mm512_add_epi32(_mm512_add_epi32(h, S1), ch),
                                            _mm512_add_epi32(w, _mm512_set1_epi32((int)K256[i])));
        const __m512i S0 = _mm512_ternarylogic_epi32(_mm512_ror_epi32(a, 2), _mm512_ror_epi32(a, 13),
                                                     _mm512_ror_epi32(a, 22), 0x96);
        const __m512i maj = _mm512_ternarylogic_epi32(a, b, c, 0xE8);  // majority
        const __m512i t2 = _mm512_add_epi32(S0, maj);
        h = g; g = f; f = e; e = _mm512_add_epi32(d, t1);
        d = c; c = b; b = a; a = _mm512_add_epi32(t1, t2);
    }
    __m512i st[8] = {a, b, c, d, e, f, g, h};
    alignas(64) uint32_t o[8][16];
    for (int k = 0; k < 8; k++)
        _mm512_store_si512(o[k], _mm512_add_epi32(st[k], _mm512_set1_epi32((int)IV[k])));
    for (int m = 0; m < 16; m++)
        for (int k = 0; k < 8; k++) {
            const uint32_t x = o[k][m];
            out[m][4 * k] = (uint8_t)(x >> 24);
            out[m][4 * k + 1] = (uint8_t)(x >> 16);
            out[m][4 * k + 2] = (uint8_t)(x >> 8);
            out[m][4 * k + 3] = (uint8_t)x;
        }
}

bool have_avx512() {
    static const bool v = __builtin_cpu_supports("avx512f") && !getenv("BCC_NO_AVX512");
    return v;
}

}  // namespace

namespace {
// SHA-256 of two messages: both <= 55 bytes (one padded block each) with the SHA extensions go
// through the interleaved pair compression, anything else one by one.
void pad_block(uint8_t blk[64], const uint8_t* p, size_t n) {
    memcpy(blk, p, n);
    blk[n] = 0x80;
    memset(blk + n + 1, 0, 55 - n);
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; i++) blk[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
}
void sha256_pair(const uint8_t* p0, size_t n0, const uint8_t* p1, size_t n1, uint8_t o0[32],
                 uint8_t o1[32]) {
#if defined(__x86_64__)
    if (n0 <= 55 && n1 <= 55 && sha256_uses_shani()) {
        alignas(16) uint8_t b0[64], b1[64];
        pad_block(b0, p0, n0);
        pad_block(b1, p1, n1);
        uint32_t s0[8], s1[8];
        sha256_iv_block_shani_x2(b0, b1, s0, s1);
        for (int i = 0; i < 8; i++) {
            const uint32_t x = s0[i], y = s1[i];
            o0[4 * i] = (uint8_t)(x >> 24); o0[4 * i + 1] = (uint8_t)(x >> 16);
            o0[4 * i + 2] = (uint8_t)(x >> 8); o0[4 * i + 3] = (uint8_t)x;
            o1[4 * i] = (uint8_t)(y >> 24); o1[4 * i + 1] = (uint8_t)(y >> 16);
            o1[4 * i + 2] = (uint8_t)(y >> 8); o1[4 * i + 3] = (uint8_t)y;
        }
        return;
    }
#endif
    sha256(p0, n0, o0);
    sha256(p1, n1, o1);
}
}  // namespace

void hash160_batch(const uint8_t* const* p, const size_t* n, uint8_t* const* out, size_t count) {
    size_t i = 0;
    if (have_avx512()) {
        uint8_t d[16][32];
        const uint8_t* in[16];
        for (int k = 0; k < 16; k++) in[k] = d[k];
        uint8_t* dp[16];
        for (int k = 0; k < 16; k++) dp[k] = d[k];
        for (; i + 16 <= count; i += 16) {
            bool short_msgs = true;
            for (int k = 0; k < 16; k++) short_msgs &= n[i + k] <= 55;
            if (short_msgs) {  // compressed keys: sixteen one-block SHA-256s in one pass
                sha256_x16_avx512(p + i, n + i, dp);
            } else {
                for (int k = 0; k < 16; k += 2)
                    sha256_pair(p[i + k], n[i + k], p[i + k + 1], n[i + k + 1], d[k], d[k + 1]);
            }
            ripemd160_32x16_avx512(in, out + i);
        }
    }
    if (have_avx2()) {
        uint8_t d[8][32];
        const uint8_t* in[8];
        for (int k = 0; k < 8; k++) in[k] = d[k];
        for (; i + 8 <= count; i += 8) {
            // SHA-256 per message with the SHA extensions (an 8-lane AVX2 SHA-256 measured no
            // faster), then the eight RIPEMD-160s together
            for (int k = 0; k < 8; k += 2) sha256_pair(p[i + k], n[i + k], p[i + k + 1], n[i + k + 1], d[k], d[k + 1]);
            ripemd160_32x8_avx2(in, out + i);
        }
    }
    for (; i < count; i++) hash160(p[i], n[i], out[i]);
}

void hash160(const uint8_t* p, size_t n, uint8_t out[20]) {
    uint8_t t[32];
    sha256(p, n, t);
    ripemd160(t, 32, out);
}

}  // namespace host
}  // namespace bcc
