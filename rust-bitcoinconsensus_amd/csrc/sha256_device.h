// SHA-256 compression for one lane (FIPS 180-4; restates crypto/sha256.cpp:78-162).
// Pure 32-bit integer ALU work: ~64 rounds x ~30 VALU ops per 64-byte block.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SHA_HD __host__ __device__ __attribute__((always_inline)) inline
#else
#define SHA_HD inline
#endif

namespace bcc {

SHA_HD uint32_t sha_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); the compiler pairs two v_xor_b32 instead
SHA_HD uint32_t sha_xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

SHA_HD void sha256_init_state(uint32_t s[8]) {
    s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
    s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
}

// w[16] = the block as big-endian words (w is clobbered: message schedule in place)
SHA_HD void sha256_compress(uint32_t s[8], uint32_t w[16]) {
    const uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            uint32_t s0 = sha_xor3(sha_rotr(w15, 7), sha_rotr(w15, 18), w15 >> 3);
            uint32_t s1 = sha_xor3(sha_rotr(w2, 17), sha_rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        uint32_t t1 = h + sha_xor3(sha_rotr(e, 6), sha_rotr(e, 11), sha_rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + wi;
        uint32_t t2 = sha_xor3(sha_rotr(a, 2), sha_rotr(a, 13), sha_rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

// second hash of SHA-256d: SHA256 over the 32-byte digest (one padded block)
SHA_HD void sha256_of_digest(uint32_t out[8], const uint32_t d[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = d[i];
    w[8] = 0x80000000u;
#pragma unroll
    for (int i = 9; i < 15; i++) w[i] = 0;
    w[15] = 256;
    sha256_init_state(out);
    sha256_compress(out, w);
}

// RIPEMD-160 compression for one lane (restates crypto/ripemd160.cpp:20-239: two lines of 80
// steps over the little-endian words X[16]; the fully unrolled tables fold into constants).
SHA_HD uint32_t rmd_rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

SHA_HD uint32_t rmd_f(int j, uint32_t x, uint32_t y, uint32_t z) {
    return j < 16 ? x ^ y ^ z
         : j < 32 ? (x & y) | (~x & z)
         : j < 48 ? (x | ~y) ^ z
         : j < 64 ? (x & z) | (y & ~z)
                  : x ^ (y | ~z);
}

SHA_HD void ripemd160_compress(uint32_t h[5], const uint32_t X[16]) {
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
    const uint32_t KL[5] = {0u, 0x5a827999u, 0x6ed9eba1u, 0x8f1bbcdcu, 0xa953fd4eu};
    const uint32_t KR[5] = {0x50a28be6u, 0x5c4dd124u, 0x6d703ef3u, 0x7a6d76e9u, 0u};
    uint32_t a1 = h[0], b1 = h[1], c1 = h[2], d1 = h[3], e1 = h[4];
    uint32_t a2 = a1, b2 = b1, c2 = c1, d2 = d1, e2 = e1;
#pragma unroll
    for (int j = 0; j < 80; j++) {
        uint32_t t = rmd_rol(a1 + rmd_f(j, b1, c1, d1) + X[RL[j]] + KL[j >> 4], SL[j]) + e1;
        a1 = e1; e1 = d1; d1 = rmd_rol(c1, 10); c1 = b1; b1 = t;
        t = rmd_rol(a2 + rmd_f(79 - j, b2, c2, d2) + X[RR[j]] + KR[j >> 4], SR[j]) + e2;
        a2 = e2; e2 = d2; d2 = rmd_rol(c2, 10); c2 = b2; b2 = t;
    }
    const uint32_t t = h[1] + c1 + d2;
    h[1] = h[2] + d1 + e2;
    h[2] = h[3] + e1 + a2;
    h[3] = h[4] + a1 + b2;
    h[4] = h[0] + b1 + c2;
    h[0] = t;
}

SHA_HD uint32_t sha_bswap(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// HASH160 (RIPEMD160(SHA256(k)), crypto/hash.h CHash160) of a public key held as a tuple row:
// k = tag || x (33 bytes) for tag 2 / 3, tag || x || y (65 bytes) otherwise; x, y are the big-endian
// coordinates as eight words each (xw[0] = bytes 0-3).  out[5] = the digest as little-endian
// words (out[0] = digest bytes 0-3, the byte order of the 20-byte program).
SHA_HD void key_hash160(uint32_t tag, const uint32_t xw[8], const uint32_t yw[8], uint32_t out[5]) {
    const bool cmp = tag == 2 || tag == 3;
    uint32_t w[16], s[8];
    // bytes: tag, x[0..31] (, y[0..31]) -> big-endian words shifted by one byte
    w[0] = (tag << 24) | (xw[0] >> 8);
#pragma unroll
    for (int i = 1; i < 8; i++) w[i] = (xw[i - 1] << 24) | (xw[i] >> 8);
    sha256_init_state(s);
    if (cmp) {
        w[8] = (xw[7] << 24) | 0x00800000u;
#pragma unroll
        for (int i = 9; i < 15; i++) w[i] = 0;
        w[15] = 33 * 8;
        sha256_compress(s, w);
    } else {
        w[8] = (xw[7] << 24) | (yw[0] >> 8);
#pragma unroll
        for (int i = 9; i < 16; i++) w[i] = (yw[i - 9] << 24) | (yw[i - 8] >> 8);
        const uint32_t last = yw[7] << 24;
        sha256_compress(s, w);
        w[0] = last | 0x00800000u;
#pragma unroll
        for (int i = 1; i < 15; i++) w[i] = 0;
        w[15] = 65 * 8;
        sha256_compress(s, w);
    }
    // RIPEMD-160 of the 32-byte digest: one block, little-endian words
    uint32_t X[16];
#pragma unroll
    for (int i = 0; i < 8; i++) X[i] = sha_bswap(s[i]);
    X[8] = 0x80u;
#pragma unroll
    for (int i = 9; i < 14; i++) X[i] = 0;
    X[14] = 256;
    X[15] = 0;
    out[0] = 0x67452301u; out[1] = 0xefcdab89u; out[2] = 0x98badcfeu; out[3] = 0x10325476u;
    out[4] = 0xc3d2e1f0u;
    ripemd160_compress(out, X);
}

}  // namespace bcc
