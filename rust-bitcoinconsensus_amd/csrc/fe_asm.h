// gfx950 inline-asm building blocks for the 8x32-bit limb product (device only).
//
// Product scanning ("Comba"): column k accumulates every a[i]*b[j], i+j == k, into a 96-bit
// accumulator {acc (64), hi (32)}.  Each partial product is ONE v_mad_u64_u32 (acc += a*b, carry
// out to VCC) plus ONE v_addc_co_u32 (hi += carry): no 64-bit adds, no zero-extension moves.
// Measured issue rates (MI355X, profiles/r01_first_probe.log): both instructions ~half rate, so a
// partial product costs 4 issue slots; the portable C formulation costs ~8.
#pragma once
#include <stdint.h>

namespace bcc {

#if defined(__HIP_DEVICE_COMPILE__)

__device__ __forceinline__ void mad_cc(uint64_t& acc, uint32_t& hi, uint32_t x, uint32_t y) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(hi)
        : "v"(x), "v"(y)
        : "vcc");
}

// 256x256 -> 512, columns 0..15
__device__ __forceinline__ void mul_256x256_asm(uint32_t (&t)[16], const uint32_t (&a)[8],
                                                const uint32_t (&b)[8]) {
    uint64_t acc = (uint64_t)a[0] * b[0];
    uint32_t hi = 0;
    t[0] = (uint32_t)acc;
    acc >>= 32;
#pragma unroll
    for (int k = 1; k < 15; k++) {
#pragma unroll
        for (int i = (k > 7 ? k - 7 : 0); i <= (k < 7 ? k : 7); i++) mad_cc(acc, hi, a[i], b[k - i]);
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)hi << 32);
        hi = 0;
    }
    t[15] = (uint32_t)acc;  // column 15 holds only the final carry
    (void)hi;
}

// squaring: per column the cross products once, the 96-bit column doubled, plus the square term
__device__ __forceinline__ void sqr_256_asm(uint32_t (&t)[16], const uint32_t (&a)[8]) {
    uint64_t carry = 0;  // carry into the current column (< 2^38)
#pragma unroll
    for (int k = 0; k < 15; k++) {
        uint64_t acc = 0;
        uint32_t hi = 0;
        // cross products i < j, i + j == k
#pragma unroll
        for (int i = (k > 7 ? k - 7 : 0); i < (k + 1) / 2; i++) mad_cc(acc, hi, a[i], a[k - i]);
        // double the 96-bit column sum
        hi = (hi << 1) | (uint32_t)(acc >> 63);
        acc <<= 1;
        if ((k & 1) == 0) mad_cc(acc, hi, a[k / 2], a[k / 2]);
        uint64_t s = acc + carry;  // add the incoming carry
        hi += (s < acc ? 1u : 0u);
        t[k] = (uint32_t)s;
        carry = (s >> 32) | ((uint64_t)hi << 32);
    }
    t[15] = (uint32_t)carry;
}

__device__ __forceinline__ uint32_t addc(uint32_t x, uint32_t y, uint32_t cin, uint32_t& cout) {
    return __builtin_addc(x, y, cin, &cout);
}

// t (512 bits) mod p, weakly reduced (< 2^256): t_lo + t_hi * (2^32 + 977)
__device__ __forceinline__ void fe_reduce512_asm(uint32_t (&r)[8], const uint32_t (&t)[16]) {
    // u = t_lo + (t_hi << 32): nine limbs via one carry chain
    uint32_t u[9], c;
    u[0] = t[0];
    u[1] = addc(t[1], t[8], 0, c);
#pragma unroll
    for (int i = 2; i < 8; i++) u[i] = addc(t[i], t[7 + i], c, c);
    u[8] = t[15] + c;  // t[15] + carry cannot overflow past 2^32 here? keep the carry below
    uint32_t u8c = (u[8] < t[15]) ? 1u : 0u;
    // r = u + 977 * t_hi, column by column; each column < 2^43
    uint64_t acc = (uint64_t)t[8] * 977u + u[0];
    r[0] = (uint32_t)acc;
#pragma unroll
    for (int i = 1; i < 8; i++) {
        acc = (uint64_t)t[8 + i] * 977u + (acc >> 32) + u[i];
        r[i] = (uint32_t)acc;
    }
    // coefficient of 2^256: u8 (+ its carry) + column carry, < 2^33 + 2^11
    uint64_t top = (acc >> 32) + u[8] + ((uint64_t)u8c << 32);
    // fold top * (2^32 + 977)
    uint64_t f = top * 977u + r[0];
    r[0] = (uint32_t)f;
    uint32_t c2;
    uint64_t f1 = (uint64_t)r[1] + (uint32_t)top + (f >> 32);  // < 2^34
    r[1] = (uint32_t)f1;
    uint32_t carry = (uint32_t)(f1 >> 32) + (uint32_t)(top >> 32);  // into limb 2, <= 3
    r[2] = addc(r[2], carry, 0, c2);
#pragma unroll
    for (int i = 3; i < 8; i++) r[i] = addc(r[i], 0, c2, c2);
    if (c2) {  // wrapped past 2^256 (rare): add 2^32 + 977 once more, cannot carry again
        uint32_t c3;
        r[0] = addc(r[0], 977u, 0, c3);
        r[1] = addc(r[1], 1u, c3, c3);
#pragma unroll
        for (int i = 2; i < 8; i++) r[i] = addc(r[i], 0, c3, c3);
    }
}

#endif

}  // namespace bcc
