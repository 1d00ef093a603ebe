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

// A lane-mask bit (an SGPR pair written as a carry-out) as 0 / 1 in this lane.
__device__ __forceinline__ uint32_t lane_bit(uint64_t m) {
    uint32_t v;
    asm volatile("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(v) : "s"(m));
    return v;
}

// r = t mod p (weak), round 5: each high limb folds together with its low limb in ONE
// v_mad_u64_u32, D_k = t[k+8] * 977 + {t[k], t[k+8]} = t[k] + t[k+8] (2^32 + 977) at limb k, so
// the fold's two carry chains (lo + s and + hi << 32) become one chain over the overlapping D_k;
// the top word w8 folds by one more v_mad_u64_u32 over {w0, w1 + w8}.  The common path is
// 8 + 1 multiply-adds and 10 carry ops (fe_reduce512_v3: 9 + 25, plus 11 moves and the
// six-limb carry walk of its top fold).  What the common path drops is flagged in SGPR carry
// masks and added back behind one wave-uniform branch:
//   e_k  D_k >= 2^64 (t[k+8] > 2^32 - 978: p ~ 2^-22 per limb)          -> limb k + 2
//   c9   the chain's carry out of w8 (needs t[15] ~ 2^32 - 1)             -> limb 9
//   ef   the top fold's carry out of limbs 0..1 (w1 + w8 ~ 2^32 - 1)      -> limb 2
//   c2   the carry out of limb 2 after the top fold (w2 == 2^32 - 1)      -> limb 3
// Limbs 8 and 9 fold again as 2^256 == 2^32 + 977, 2^288 == 2^64 + 977 2^32.  The rare sum
// M < 2^140, so r + M wraps past 2^256 at most once and one more fold cannot carry.
__device__ __forceinline__ void fe_reduce512_v4(uint32_t (&r)[8], const uint32_t (&t)[16]) {
    uint64_t D0 = (uint64_t)t[0] | ((uint64_t)t[8] << 32), D1 = (uint64_t)t[1] | ((uint64_t)t[9] << 32),
             D2 = (uint64_t)t[2] | ((uint64_t)t[10] << 32), D3 = (uint64_t)t[3] | ((uint64_t)t[11] << 32),
             D4 = (uint64_t)t[4] | ((uint64_t)t[12] << 32), D5 = (uint64_t)t[5] | ((uint64_t)t[13] << 32),
             D6 = (uint64_t)t[6] | ((uint64_t)t[14] << 32), D7 = (uint64_t)t[7] | ((uint64_t)t[15] << 32);
    uint64_t e0, e1, e2, e3, e4, e5, e6, e7;
    asm("v_mad_u64_u32 %[d0], %[e0], %[h0], %[k], %[d0]\n\t"
        "v_mad_u64_u32 %[d1], %[e1], %[h1], %[k], %[d1]\n\t"
        "v_mad_u64_u32 %[d2], %[e2], %[h2], %[k], %[d2]\n\t"
        "v_mad_u64_u32 %[d3], %[e3], %[h3], %[k], %[d3]\n\t"
        "v_mad_u64_u32 %[d4], %[e4], %[h4], %[k], %[d4]\n\t"
        "v_mad_u64_u32 %[d5], %[e5], %[h5], %[k], %[d5]\n\t"
        "v_mad_u64_u32 %[d6], %[e6], %[h6], %[k], %[d6]\n\t"
        "v_mad_u64_u32 %[d7], %[e7], %[h7], %[k], %[d7]"
        : [d0] "+v"(D0), [d1] "+v"(D1), [d2] "+v"(D2), [d3] "+v"(D3),
          [d4] "+v"(D4), [d5] "+v"(D5), [d6] "+v"(D6), [d7] "+v"(D7),
          [e0] "=&s"(e0), [e1] "=&s"(e1), [e2] "=&s"(e2), [e3] "=&s"(e3),
          [e4] "=&s"(e4), [e5] "=&s"(e5), [e6] "=&s"(e6), [e7] "=&s"(e7)
        : [h0] "v"(t[8]), [h1] "v"(t[9]), [h2] "v"(t[10]), [h3] "v"(t[11]),
          [h4] "v"(t[12]), [h5] "v"(t[13]), [h6] "v"(t[14]), [h7] "v"(t[15]), [k] "s"(977u));
    // one chain over the overlapping D_k (w_k = D_k.lo + D_{k-1}.hi), then x1 = w1 + w8 and its
    // carry into limb 2
    uint32_t x1, r2, w3, w4, w5, w6, w7, w8;
    uint64_t c9, c2;
    {
        uint32_t w1, w2;
        asm("v_add_co_u32_e32 %[w1], vcc, %[h0], %[l1]\n\t"
            "v_addc_co_u32_e32 %[w2], vcc, %[h1], %[l2], vcc\n\t"
            "v_addc_co_u32_e32 %[w3], vcc, %[h2], %[l3], vcc\n\t"
            "v_addc_co_u32_e32 %[w4], vcc, %[h3], %[l4], vcc\n\t"
            "v_addc_co_u32_e32 %[w5], vcc, %[h4], %[l5], vcc\n\t"
            "v_addc_co_u32_e32 %[w6], vcc, %[h5], %[l6], vcc\n\t"
            "v_addc_co_u32_e32 %[w7], vcc, %[h6], %[l7], vcc\n\t"
            "v_addc_co_u32_e64 %[w8], %[c9], %[h7], 0, vcc\n\t"
            "v_add_co_u32_e32 %[x1], vcc, %[w1], %[w8]\n\t"
            "v_addc_co_u32_e64 %[r2], %[c2], %[w2], 0, vcc"
            : [w1] "=&v"(w1), [w2] "=&v"(w2), [w3] "=&v"(w3), [w4] "=&v"(w4), [w5] "=&v"(w5),
              [w6] "=&v"(w6), [w7] "=&v"(w7), [w8] "=&v"(w8), [x1] "=&v"(x1), [r2] "=&v"(r2),
              [c9] "=&s"(c9), [c2] "=&s"(c2)
            : [h0] "v"((uint32_t)(D0 >> 32)), [l1] "v"((uint32_t)D1), [h1] "v"((uint32_t)(D1 >> 32)),
              [l2] "v"((uint32_t)D2), [h2] "v"((uint32_t)(D2 >> 32)), [l3] "v"((uint32_t)D3),
              [h3] "v"((uint32_t)(D3 >> 32)), [l4] "v"((uint32_t)D4), [h4] "v"((uint32_t)(D4 >> 32)),
              [l5] "v"((uint32_t)D5), [h5] "v"((uint32_t)(D5 >> 32)), [l6] "v"((uint32_t)D6),
              [h6] "v"((uint32_t)(D6 >> 32)), [l7] "v"((uint32_t)D7), [h7] "v"((uint32_t)(D7 >> 32))
            : "vcc");
    }
    // {r0, r1} = {w0, x1} + 977 w8
    uint64_t F = (uint64_t)(uint32_t)D0 | ((uint64_t)x1 << 32), ef;
    asm("v_mad_u64_u32 %[f], %[ef], %[w8], %[k], %[f]" : [f] "+v"(F), [ef] "=s"(ef) : [w8] "v"(w8), [k] "s"(977u));
    r[0] = (uint32_t)F;
    r[1] = (uint32_t)(F >> 32);
    r[2] = r2;
    r[3] = w3;
    r[4] = w4;
    r[5] = w5;
    r[6] = w6;
    r[7] = w7;
    if (__builtin_expect((e0 | e1 | e2 | e3 | e4 | e5 | e6 | e7 | c9 | c2 | ef) != 0, 0)) {
        const uint32_t b6 = lane_bit(e6), b79 = lane_bit(e7) + lane_bit(c9);
        uint32_t m[8];
        m[0] = 977u * b6;
        m[1] = b6 + 977u * b79;
        m[2] = lane_bit(ef) + lane_bit(e0) + b79;
        m[3] = lane_bit(c2) + lane_bit(e1);
        m[4] = lane_bit(e2);
        m[5] = lane_bit(e3);
        m[6] = lane_bit(e4);
        m[7] = lane_bit(e5);
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) r[i] = addc(r[i], m[i], c, c);
        if (c) {  // at most once: r + M - 2^256 < M
            r[0] = addc(r[0], 977u, 0, c);
            r[1] = addc(r[1], 1u, c, c);
#pragma unroll
            for (int i = 2; i < 8; i++) r[i] = addc(r[i], 0, c, c);
        }
    }
}

#endif

}  // namespace bcc
