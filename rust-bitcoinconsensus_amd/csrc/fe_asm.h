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

// ---- 256-bit add / sub / shift mod p as single asm statements ----
// The common path is one 8-limb carry chain plus a two-limb fold of the wrap-around
// (2^256 == 2^32 + 977); the fold's carry into limb 2 (probability ~2^-64 per lane) and a
// second wrap (only for weak inputs >= p) run behind a wave-uniform branch that skips them
// unless some lane of the wave needs them.  hipcc cannot see inside, so it pads nothing.
#define BCC_FOLD_TAIL(OP0, OP1, OPC)                                              \
    "s_and_b64 %[tmp], vcc, exec\n\t"                                             \
    "s_cbranch_scc0 .Ldone%=\n\t"                                                 \
    OPC " %[r2], vcc, 0, %[r2], vcc\n\t" OPC " %[r3], vcc, 0, %[r3], vcc\n\t"     \
    OPC " %[r4], vcc, 0, %[r4], vcc\n\t" OPC " %[r5], vcc, 0, %[r5], vcc\n\t"     \
    OPC " %[r6], vcc, 0, %[r6], vcc\n\t" OPC " %[r7], vcc, 0, %[r7], vcc\n\t"     \
    "v_cndmask_b32_e64 %[t0], 0, %[k977], vcc\n\t"                                \
    "v_cndmask_b32_e64 %[t1], 0, 1, vcc\n\t"                                      \
    OP0 " %[r0], vcc, %[r0], %[t0]\n\t"                                          \
    OP1 " %[r1], vcc, %[r1], %[t1], vcc\n\t"                                     \
    OPC " %[r2], vcc, 0, %[r2], vcc\n\t" OPC " %[r3], vcc, 0, %[r3], vcc\n\t"     \
    OPC " %[r4], vcc, 0, %[r4], vcc\n\t" OPC " %[r5], vcc, 0, %[r5], vcc\n\t"     \
    OPC " %[r6], vcc, 0, %[r6], vcc\n\t" OPC " %[r7], vcc, 0, %[r7], vcc\n"       \
    ".Ldone%=:"

// The carry (borrow) of limb 7, in VCC, as t1 = c and t0 = 977 c (two selects; an add-with-carry
// plus a 24-bit multiply instead measured neutral, profiles/r02tw4).
#define BCC_CARRY_TO_T01                                                           \
    "v_cndmask_b32_e64 %[t0], 0, %[k977], vcc\n\t"                                 \
    "v_cndmask_b32_e64 %[t1], 0, 1, vcc\n\t"

#define BCC_R_OUT                                                                  \
    [r0] "=&v"(r[0]), [r1] "=&v"(r[1]), [r2] "=&v"(r[2]), [r3] "=&v"(r[3]),      \
    [r4] "=&v"(r[4]), [r5] "=&v"(r[5]), [r6] "=&v"(r[6]), [r7] "=&v"(r[7]),      \
    [t0] "=&v"(t0), [t1] "=&v"(t1), [tmp] "=&s"(tmp)

// r = a + b (weak, < 2^256)
__device__ __forceinline__ void fe_add_asm(uint32_t (&r)[8], const uint32_t (&a)[8],
                                           const uint32_t (&b)[8]) {
    uint32_t t0, t1;
    uint64_t tmp;
    asm volatile(
        "v_add_co_u32_e32 %[r0], vcc, %[a0], %[b0]\n\t"
        "v_addc_co_u32_e32 %[r1], vcc, %[a1], %[b1], vcc\n\t"
        "v_addc_co_u32_e32 %[r2], vcc, %[a2], %[b2], vcc\n\t"
        "v_addc_co_u32_e32 %[r3], vcc, %[a3], %[b3], vcc\n\t"
        "v_addc_co_u32_e32 %[r4], vcc, %[a4], %[b4], vcc\n\t"
        "v_addc_co_u32_e32 %[r5], vcc, %[a5], %[b5], vcc\n\t"
        "v_addc_co_u32_e32 %[r6], vcc, %[a6], %[b6], vcc\n\t"
        "v_addc_co_u32_e32 %[r7], vcc, %[a7], %[b7], vcc\n\t"
        BCC_CARRY_TO_T01
        "v_add_co_u32_e32 %[r0], vcc, %[r0], %[t0]\n\t"
        "v_addc_co_u32_e32 %[r1], vcc, %[r1], %[t1], vcc\n\t"
        BCC_FOLD_TAIL("v_add_co_u32_e32", "v_addc_co_u32_e32", "v_addc_co_u32_e32")
        : BCC_R_OUT
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]),
          [a4] "v"(a[4]), [a5] "v"(a[5]), [a6] "v"(a[6]), [a7] "v"(a[7]),
          [b0] "v"(b[0]), [b1] "v"(b[1]), [b2] "v"(b[2]), [b3] "v"(b[3]),
          [b4] "v"(b[4]), [b5] "v"(b[5]), [b6] "v"(b[6]), [b7] "v"(b[7]),
          [k977] "v"(977u)
        : "vcc", "scc");
}

// r = a - b (weak): a borrow out of limb 7 adds p, i.e. subtracts 2^32 + 977 mod 2^256
__device__ __forceinline__ void fe_sub_asm(uint32_t (&r)[8], const uint32_t (&a)[8],
                                           const uint32_t (&b)[8]) {
    uint32_t t0, t1;
    uint64_t tmp;
    asm volatile(
        "v_sub_co_u32_e32 %[r0], vcc, %[a0], %[b0]\n\t"
        "v_subb_co_u32_e32 %[r1], vcc, %[a1], %[b1], vcc\n\t"
        "v_subb_co_u32_e32 %[r2], vcc, %[a2], %[b2], vcc\n\t"
        "v_subb_co_u32_e32 %[r3], vcc, %[a3], %[b3], vcc\n\t"
        "v_subb_co_u32_e32 %[r4], vcc, %[a4], %[b4], vcc\n\t"
        "v_subb_co_u32_e32 %[r5], vcc, %[a5], %[b5], vcc\n\t"
        "v_subb_co_u32_e32 %[r6], vcc, %[a6], %[b6], vcc\n\t"
        "v_subb_co_u32_e32 %[r7], vcc, %[a7], %[b7], vcc\n\t"
        BCC_CARRY_TO_T01
        "v_sub_co_u32_e32 %[r0], vcc, %[r0], %[t0]\n\t"
        "v_subb_co_u32_e32 %[r1], vcc, %[r1], %[t1], vcc\n\t"
        BCC_FOLD_TAIL("v_sub_co_u32_e32", "v_subb_co_u32_e32", "v_subbrev_co_u32_e32")
        : BCC_R_OUT
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]),
          [a4] "v"(a[4]), [a5] "v"(a[5]), [a6] "v"(a[6]), [a7] "v"(a[7]),
          [b0] "v"(b[0]), [b1] "v"(b[1]), [b2] "v"(b[2]), [b3] "v"(b[3]),
          [b4] "v"(b[4]), [b5] "v"(b[5]), [b6] "v"(b[6]), [b7] "v"(b[7]),
          [k977] "v"(977u)
        : "vcc", "scc");
}

// r = a << S mod p for S in 1..3: limbs by v_alignbit, the S bits shifted out fold back as
// top * (2^32 + 977) (top * 977 < 2^13)
template <int S>
__device__ __forceinline__ void fe_shl_asm(uint32_t (&r)[8], const uint32_t (&a)[8]) {
    static_assert(S >= 1 && S <= 3, "small shifts only");
    uint32_t t0, t1;
    uint64_t tmp;
    asm volatile(
        "v_lshrrev_b32_e32 %[t1], %[rs], %[a7]\n\t"
        "v_alignbit_b32 %[r7], %[a7], %[a6], %[rs]\n\t"
        "v_alignbit_b32 %[r6], %[a6], %[a5], %[rs]\n\t"
        "v_alignbit_b32 %[r5], %[a5], %[a4], %[rs]\n\t"
        "v_alignbit_b32 %[r4], %[a4], %[a3], %[rs]\n\t"
        "v_alignbit_b32 %[r3], %[a3], %[a2], %[rs]\n\t"
        "v_alignbit_b32 %[r2], %[a2], %[a1], %[rs]\n\t"
        "v_alignbit_b32 %[r1], %[a1], %[a0], %[rs]\n\t"
        "v_lshlrev_b32_e32 %[r0], %[ls], %[a0]\n\t"
        "v_mul_u32_u24_e32 %[t0], %[k977], %[t1]\n\t"
        "v_add_co_u32_e32 %[r0], vcc, %[r0], %[t0]\n\t"
        "v_addc_co_u32_e32 %[r1], vcc, %[r1], %[t1], vcc\n\t"
        BCC_FOLD_TAIL("v_add_co_u32_e32", "v_addc_co_u32_e32", "v_addc_co_u32_e32")
        : BCC_R_OUT
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]),
          [a4] "v"(a[4]), [a5] "v"(a[5]), [a6] "v"(a[6]), [a7] "v"(a[7]),
          [rs] "i"(32 - S), [ls] "i"(S), [k977] "v"(977u)
        : "vcc", "scc");
}

__device__ __forceinline__ uint32_t addc(uint32_t x, uint32_t y, uint32_t cin, uint32_t& cout) {
    return __builtin_addc(x, y, cin, &cout);
}

// r = t mod p (weak, < 2^256) with 2^256 == 2^32 + 977: s = t_hi * 977 as a chain of
// v_mad_u64_u32 whose 64-bit addend is the previous product's high word (p >> 32: one move into a
// zero-high pair, no 64-bit add), then x = t_lo + s + (t_hi << 32) as two carry chains, then the
// top (< 2^34) folded once more; the rare wrap past 2^256 runs behind a branch.  (A per-limb asm
// carry-chain reduction with SGPR carries measured 4-6 % slower in the ladder: profiles/r02/
// ab_field_reduction_sqrtail.txt.)
__device__ __forceinline__ void fe_reduce512_v3(uint32_t (&r)[8], const uint32_t (&t)[16]) {
    uint32_t s[9];
    uint64_t p = (uint64_t)t[8] * 977u;
    s[0] = (uint32_t)p;
#pragma unroll
    for (int i = 1; i < 8; i++) {
        p = (uint64_t)t[8 + i] * 977u + (p >> 32);
        s[i] = (uint32_t)p;
    }
    s[8] = (uint32_t)(p >> 32);
    uint32_t x[9], ca, cb;
    x[0] = addc(t[0], s[0], 0, ca);
    x[1] = addc(t[1], s[1], ca, ca);
    x[1] = addc(x[1], t[8], 0, cb);
#pragma unroll
    for (int i = 2; i < 8; i++) {
        x[i] = addc(t[i], s[i], ca, ca);
        x[i] = addc(x[i], t[7 + i], cb, cb);
    }
    uint32_t dz;
    x[8] = addc(s[8], t[15], ca, ca);
    uint32_t x9 = addc(0u, 0u, ca, dz);  // the carries as values by add-with-carry (no selects)
    x[8] = addc(x[8], 0, cb, cb);
    x9 = addc(x9, 0u, cb, dz);           // top = x8 + x9 2^32 < 2^34
    uint64_t f = (uint64_t)x[8] * 977u + x[0];
    r[0] = (uint32_t)f;
    uint32_t c2;
    uint64_t f1 = (uint64_t)x[1] + x[8] + (f >> 32) + (uint64_t)x9 * 977u;  // < 2^34
    r[1] = (uint32_t)f1;
    uint32_t carry = (uint32_t)(f1 >> 32) + x9;  // into limb 2, small
    r[2] = addc(x[2], carry, 0, c2);
#pragma unroll
    for (int i = 3; i < 8; i++) r[i] = addc(x[i], 0, c2, c2);
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
