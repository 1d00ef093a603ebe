// secp256k1 arithmetic for gfx950 lanes: Fp / Fn in 8x32-bit limbs, Jacobian group law,
// GLV split and signed odd fixed-window digits.  One lane = one signature.
//
// Design notes (DESIGN.md §3 has the full story):
//  * Limbs are 32-bit so that every partial product is ONE v_mad_u64_u32
//    (32x32 + 64 -> 64) — the integer-ALU roofline unit of this engine.
//  * Field elements are kept "weakly reduced": any value < 2^256 that is congruent mod p.
//    p = 2^256 - 0x1000003D1, so a 512-bit product folds as lo + hi * (2^32 + 977).
//    Only comparisons / outputs normalise to [0, p).
//  * Scalars (mod n) are always fully reduced.
//  * Everything is __host__ __device__ so the exact lane code is unit-testable on the CPU.
//
// Reference semantics restated (paths under /root/reference/depend/bitcoin/src/secp256k1/src):
//  field arithmetic        field_5x52_int128_impl.h:18-279, field_impl.h:39-263
//  scalar arithmetic       scalar_4x64_impl.h:117-915, scalar_impl.h:68-375
//  group law              group_impl.h:273-491 (double / add_ge / add_zinv with exceptional cases)
//  GLV split              scalar_impl.h:342-375 (constants re-derived: tools/derive_glv_constants.py)
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#include "fe_asm.h"
#include "fe_asm_gen.h"
#define BCC_HD __host__ __device__ __attribute__((always_inline)) inline
#define BCC_HD_NOINLINE __host__ __device__ __attribute__((noinline))
#else
#define BCC_HD inline
#define BCC_HD_NOINLINE
#endif

#include "modinv_device.h"  // the lanes' safegcd inverse (fe_inv, sc_inv)

namespace bcc {

typedef uint32_t u32;
typedef uint64_t u64;

struct fe {
    u32 v[8];
};  // little-endian 32-bit limbs

// ------------------------------------------------------------------------------------------
// constants
// ------------------------------------------------------------------------------------------
// p = 2^256 - 2^32 - 977
#define BCC_P_LIMBS {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}
// n = group order
#define BCC_N_LIMBS {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}
// 2^256 - n (129 bits, 5 limbs)
#define BCC_NC_LIMBS {0x2FC9BEBFu, 0x402DA173u, 0x50B75FC4u, 0x45512319u, 0x1u}
// beta: cube root of unity mod p, lambda*(x,y) = (beta*x, y)
#define BCC_BETA_LIMBS {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u, 0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu}
// lambda
#define BCC_LAMBDA_LIMBS {0x1B23BD72u, 0xDF02967Cu, 0x20816678u, 0x122E22EAu, 0x8812645Au, 0xA5261C02u, 0xC05C30E0u, 0x5363AD4Cu}
// g1 = round(2^384*b2/n), g2 = round(2^384*(-b1)/n)
#define BCC_G1_LIMBS {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u, 0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u}
#define BCC_G2_LIMBS {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu, 0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u}
// -b1 mod n, -b2 mod n
#define BCC_MB1_LIMBS {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u, 0u, 0u, 0u, 0u}
#define BCC_MB2_LIMBS {0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}
// p - n (for the xr + n < p test)
#define BCC_PMN_LIMBS {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u, 0x1u, 0u, 0u, 0u}
// generator
#define BCC_GX_LIMBS {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu, 0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu}
#define BCC_GY_LIMBS {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u, 0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u}

BCC_HD void fe_set(fe& r, const u32 (&c)[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = c[i];
}
BCC_HD fe fe_const(u32 a0, u32 a1, u32 a2, u32 a3, u32 a4, u32 a5, u32 a6, u32 a7) {
    fe r;
    r.v[0] = a0; r.v[1] = a1; r.v[2] = a2; r.v[3] = a3;
    r.v[4] = a4; r.v[5] = a5; r.v[6] = a6; r.v[7] = a7;
    return r;
}
BCC_HD fe fe_zero() { return fe_const(0, 0, 0, 0, 0, 0, 0, 0); }
BCC_HD fe fe_one() { return fe_const(1, 0, 0, 0, 0, 0, 0, 0); }

BCC_HD u32 lo32(u64 x) { return (u32)x; }
BCC_HD u32 hi32(u64 x) { return (u32)(x >> 32); }

// ------------------------------------------------------------------------------------------
// 256x256 -> 512 product, operand scanning: every partial product is one v_mad_u64_u32
// ((2^32-1)^2 + 2*(2^32-1) = 2^64-1, so a*b + t + carry never overflows 64 bits)
// ------------------------------------------------------------------------------------------
BCC_HD void mul_256x256(u32 (&t)[16], const u32 (&a)[8], const u32 (&b)[8]) {
    {
        u64 c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            c = (u64)a[0] * b[j] + (c >> 32);
            t[j] = lo32(c);
        }
        t[8] = hi32(c);
    }
#pragma unroll
    for (int i = 1; i < 8; i++) {
        u64 c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            c = (u64)a[i] * b[j] + t[i + j] + (c >> 32);
            t[i + j] = lo32(c);
        }
        t[i + 8] = hi32(c);
    }
}

// squaring: cross products once, doubled, plus the diagonal (36 mads instead of 64)
BCC_HD void sqr_256(u32 (&t)[16], const u32 (&a)[8]) {
#pragma unroll
    for (int k = 0; k < 16; k++) t[k] = 0;
    // cross products a[i]*a[j], i < j
#pragma unroll
    for (int i = 0; i < 7; i++) {
        u64 c = 0;
#pragma unroll
        for (int j = i + 1; j < 8; j++) {
            c = (u64)a[i] * a[j] + t[i + j] + (c >> 32);
            t[i + j] = lo32(c);
        }
        t[i + 8] = hi32(c);
    }
    // double
    u32 carry = 0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
        u32 nc = t[k] >> 31;
        t[k] = (t[k] << 1) | carry;
        carry = nc;
    }
    // add diagonal
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 d = (u64)a[i] * a[i];
        c = (u64)t[2 * i] + lo32(d) + (c >> 32);
        t[2 * i] = lo32(c);
        c = (u64)t[2 * i + 1] + hi32(d) + (c >> 32);
        t[2 * i + 1] = lo32(c);
    }
}

// r = t mod p (weak: r < 2^256), t = lo + hi*2^256, 2^256 == 2^32 + 977 (mod p)
BCC_HD void fe_reduce512(fe& r, const u32 (&t)[16]) {
    u64 c = (u64)t[8] * 977u + t[0];
    r.v[0] = lo32(c);
#pragma unroll
    for (int i = 1; i < 8; i++) {
        c = (u64)t[8 + i] * 977u + t[i] + t[8 + i - 1] + (c >> 32);
        r.v[i] = lo32(c);
    }
    u64 top = (u64)t[15] + (c >> 32);  // < 2^33: coefficient of 2^256
    // fold top*(2^32 + 977)
    c = (u64)r.v[0] + top * 977u;
    r.v[0] = lo32(c);
    c = (u64)r.v[1] + lo32(top) + (c >> 32) + ((top >> 32) << 32);
    // (top >> 32) is 0 or 1 and belongs at limb 2; handle via carry arithmetic below
    r.v[1] = lo32(c);
    u64 cc = (c >> 32);
#pragma unroll
    for (int i = 2; i < 8; i++) {
        cc += r.v[i];
        r.v[i] = lo32(cc);
        cc >>= 32;
    }
    if (cc) {  // wrapped past 2^256 (rare): add 2^32 + 977 once more; cannot carry again
        c = (u64)r.v[0] + 977u;
        r.v[0] = lo32(c);
        c = (u64)r.v[1] + 1u + (c >> 32);
        r.v[1] = lo32(c);
        cc = c >> 32;
#pragma unroll
        for (int i = 2; i < 8; i++) {
            cc += r.v[i];
            r.v[i] = lo32(cc);
            cc >>= 32;
        }
    }
}

// Device builds use the inline-asm column products (fe_asm_gen.h) and fe_reduce512_v3 (fe_asm.h:
// the 977-products chained through their high words, two carry chains for the rest; 4.4 % fewer
// VALU instructions in the ladder than the round-1 reduction, profiles/r02tw4/ab_summary.txt);
// host builds use 4 x 64-bit limbs (below) or the portable formulation above.  All compute the
// same weak residue class.  Round 5: fe_reduce512_v4 (fe_asm.h: one multiply-add per limb pair,
// one carry chain, the rare carries behind a wave-uniform branch); BCC_RED_V4=0 keeps v3.
#ifndef BCC_RED_V4
#define BCC_RED_V4 1
#endif
// (Round 6 also replaced v4's e_k / c9 masks by a precheck of the high limbs -- all <= 2^32 - 979
// rule them out -- and measured it slower: the max over eight limbs sits on the reduction's
// critical path, C2 117.1 -> 114.5 M/s, profiles/r06/ab/reduction_precheck.txt.  Not kept.)
#if BCC_RED_V4
#define BCC_FE_REDUCE fe_reduce512_v4
#else
#define BCC_FE_REDUCE fe_reduce512_v3
#endif
// Round 5: the product columns' first multiply-adds unguarded, their rare carries flagged
// (fe_asm_gen.h mul_256x256_col_f / sqr_cross_col_f); a wave with a flagged lane redoes the product
// with the exact columns.  BCC_MUL_FLAG=0 keeps the exact columns only.
#ifndef BCC_MUL_FLAG
#define BCC_MUL_FLAG 1
#endif
// Round 6: no flags at all.  The columns' first carries are provably zero when a[0] and b[7] (a[0]
// and a[7] for a square) are at most 2^32 - 9 (tools/gen_fe_asm.py, mul_256x256_col_u); one
// compare per operand and a wave-wide ballot pick the unguarded columns or, when any lane has such
// a limb, the exact ones.  BCC_MUL_PRECHECK=0 keeps round 5's flags.
#ifndef BCC_MUL_PRECHECK
#define BCC_MUL_PRECHECK 1
#endif
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ bool any_lane_top_limbs(u32 lo_limb, u32 hi_limb) {
    return __builtin_amdgcn_ballot_w64((lo_limb > 0xFFFFFFF7u) | (hi_limb > 0xFFFFFFF7u)) != 0;
}
#endif

#if !defined(__HIP_DEVICE_COMPILE__) && defined(__SIZEOF_INT128__)
// Host builds (the engine's host verification, host_verify.cpp, and tests/native): 4 x 64-bit limbs
// with 128-bit products, the CPU's native width, over the same little-endian bytes as fe.v.
// Same contract as the 32-bit formulation: a weak residue (< 2^256) of a * b mod p.
#define BCC_FE_HOST64 1
}  // namespace bcc
#include "modinv_host.h"  // variable-time inverses of the host builds (fe_inv, sc_inv)
namespace bcc {
inline void mul_4x64(u64 (&t)[8], const u32 (&a)[8], const u32 (&b)[8]) {
    typedef unsigned __int128 u128;
    u64 x[4], y[4];
    memcpy(x, a, 32);
    memcpy(y, b, 32);
    for (int i = 0; i < 8; i++) t[i] = 0;
    for (int i = 0; i < 4; i++) {
        u64 c = 0;
        for (int j = 0; j < 4; j++) {
            const u128 p = (u128)x[i] * y[j] + t[i + j] + c;
            t[i + j] = (u64)p;
            c = (u64)(p >> 64);
        }
        t[i + 4] = c;
    }
}
inline void fe_mul_host64(fe& r, const fe& a, const fe& b) {
    typedef unsigned __int128 u128;
    u64 t[8];
    mul_4x64(t, a.v, b.v);
    // 2^256 == 0x1000003D1 (mod p): r = t_lo + t_hi * 0x1000003D1, folded twice
    const u64 C = 0x1000003D1ull;
    u64 o[4], c = 0;
    for (int i = 0; i < 4; i++) {
        const u128 p = (u128)t[4 + i] * C + t[i] + c;
        o[i] = (u64)p;
        c = (u64)(p >> 64);
    }
    u128 p = (u128)c * C + o[0];  // c < 2^34
    o[0] = (u64)p;
    u64 k = (u64)(p >> 64);
    for (int i = 1; i < 4 && k; i++) {
        const u128 q = (u128)o[i] + k;
        o[i] = (u64)q;
        k = (u64)(q >> 64);
    }
    if (k) {  // wrapped past 2^256 once more (the value is then tiny): add C again, no carry out
        p = (u128)o[0] + C;
        o[0] = (u64)p;
        k = (u64)(p >> 64);
        for (int i = 1; i < 4 && k; i++) {
            const u128 q = (u128)o[i] + k;
            o[i] = (u64)q;
            k = (u64)(q >> 64);
        }
    }
    memcpy(r.v, o, 32);
}
#endif

BCC_HD void fe_mul(fe& r, const fe& a, const fe& b) {
#if defined(BCC_FE_HOST64)
    fe_mul_host64(r, a, b);
#else
    u32 t[16];
#if defined(__HIP_DEVICE_COMPILE__)
#if BCC_MUL_PRECHECK
    if (__builtin_expect(any_lane_top_limbs(a.v[0], b.v[7]), 0)) mul_256x256_col(t, a.v, b.v);
    else mul_256x256_col_u(t, a.v, b.v);
#elif BCC_MUL_FLAG
    uint64_t ovf;
    mul_256x256_col_f(t, a.v, b.v, ovf);
    if (__builtin_expect(ovf != 0, 0)) mul_256x256_col(t, a.v, b.v);
#else
    mul_256x256_col(t, a.v, b.v);
#endif
    BCC_FE_REDUCE(r.v, t);
#else
    mul_256x256(t, a.v, b.v);
    fe_reduce512(r, t);
#endif
#endif
}

BCC_HD void fe_sqr(fe& r, const fe& a) {
#if defined(BCC_FE_HOST64)
    fe_mul_host64(r, a, a);
#else
    u32 t[16];
#if defined(__HIP_DEVICE_COMPILE__)
#if BCC_MUL_PRECHECK
    if (__builtin_expect(any_lane_top_limbs(a.v[0], a.v[7]), 0)) {
        sqr_256_col(t, a.v);
    } else {
        u32 x[16];
        sqr_cross_col_u(x, a.v);
        sqr_tail_col(t, x, a.v);
    }
#elif BCC_MUL_FLAG
    uint64_t ovf;
    u32 x[16];
    sqr_cross_col_f(x, a.v, ovf);
    if (__builtin_expect(ovf != 0, 0)) sqr_256_col(t, a.v);
    else sqr_tail_col(t, x, a.v);
#else
    sqr_256_col(t, a.v);
#endif
    BCC_FE_REDUCE(r.v, t);
#else
    sqr_256(t, a.v);
    fe_reduce512(r, t);
#endif
#endif
}

// r = a + b mod p (weak)
BCC_HD void fe_add(fe& r, const fe& a, const fe& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    fe_add_asm(r.v, a.v, b.v);
    return;
#endif
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c = (u64)a.v[i] + b.v[i] + (c >> 32);
        r.v[i] = lo32(c);
    }
    u32 k = hi32(c);  // 0/1: add k*(2^32+977)
    c = (u64)r.v[0] + 977u * k;
    r.v[0] = lo32(c);
    c = (u64)r.v[1] + k + (c >> 32);
    r.v[1] = lo32(c);
#pragma unroll
    for (int i = 2; i < 8; i++) {
        c = (u64)r.v[i] + (c >> 32);
        r.v[i] = lo32(c);
    }
    if (hi32(c)) {  // rare second wrap
        c = (u64)r.v[0] + 977u;
        r.v[0] = lo32(c);
        c = (u64)r.v[1] + 1u + (c >> 32);
        r.v[1] = lo32(c);
#pragma unroll
        for (int i = 2; i < 8; i++) {
            c = (u64)r.v[i] + (c >> 32);
            r.v[i] = lo32(c);
        }
    }
}

// r = a - b mod p (weak)
BCC_HD void fe_sub(fe& r, const fe& a, const fe& b) {
#if defined(__HIP_DEVICE_COMPILE__)
    fe_sub_asm(r.v, a.v, b.v);
    return;
#endif
    u64 c = 0;  // borrow propagation via two's complement
    u32 borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 d = (u64)a.v[i] - b.v[i] - borrow;
        r.v[i] = lo32(d);
        borrow = (u32)(d >> 63);
    }
    // if borrow: r = r + p (mod 2^256) == r - (2^32 + 977)
    u32 k = borrow;
    u64 d = (u64)r.v[0] - 977u * k;
    r.v[0] = lo32(d);
    u32 bw = (u32)(d >> 63);
    d = (u64)r.v[1] - k - bw;
    r.v[1] = lo32(d);
    bw = (u32)(d >> 63);
#pragma unroll
    for (int i = 2; i < 8; i++) {
        d = (u64)r.v[i] - bw;
        r.v[i] = lo32(d);
        bw = (u32)(d >> 63);
    }
    if (bw) {  // rare: the first correction borrowed again (b was >= p): subtract once more
        d = (u64)r.v[0] - 977u;
        r.v[0] = lo32(d);
        bw = (u32)(d >> 63);
        d = (u64)r.v[1] - 1u - bw;
        r.v[1] = lo32(d);
        bw = (u32)(d >> 63);
#pragma unroll
        for (int i = 2; i < 8; i++) {
            d = (u64)r.v[i] - bw;
            r.v[i] = lo32(d);
            bw = (u32)(d >> 63);
        }
    }
    (void)c;
}

BCC_HD void fe_neg(fe& r, const fe& a) {
    fe z = fe_zero();
    fe_sub(r, z, a);
}

// canonical representative in [0, p)
BCC_HD void fe_normalize(fe& r) {
    // r >= p  <=>  r + (2^32 + 977) >= 2^256
    u64 c = (u64)r.v[0] + 977u;
    u32 t[8];
    t[0] = lo32(c);
    c = (u64)r.v[1] + 1u + (c >> 32);
    t[1] = lo32(c);
#pragma unroll
    for (int i = 2; i < 8; i++) {
        c = (u64)r.v[i] + (c >> 32);
        t[i] = lo32(c);
    }
    bool ge = hi32(c) != 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = ge ? t[i] : r.v[i];
}

BCC_HD bool fe_is_zero_norm(const fe& a) {  // a must be normalized
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= a.v[i];
    return x == 0;
}

// a weak value (< 2^256) is 0 mod p iff it is 0 or p: no carry chain needed
BCC_HD bool fe_is_zero(const fe& a) {
    u32 z = 0, q = (a.v[0] ^ 0xFFFFFC2Fu) | (a.v[1] ^ 0xFFFFFFFEu);
#pragma unroll
    for (int i = 0; i < 8; i++) z |= a.v[i];
#pragma unroll
    for (int i = 2; i < 8; i++) q |= ~a.v[i];
    return z == 0 || q == 0;
}

BCC_HD bool fe_equal(const fe& a, const fe& b) {
    fe d;
    fe_sub(d, a, b);
    return fe_is_zero(d);
}

// a < p (a fully below 2^256)
BCC_HD bool fe_lt_p(const fe& a) {
    u64 c = (u64)a.v[0] + 977u;
    c = (u64)a.v[1] + 1u + (c >> 32);
#pragma unroll
    for (int i = 2; i < 8; i++) c = (u64)a.v[i] + (c >> 32);
    return hi32(c) == 0;
}

BCC_HD void fe_mul_int(fe& r, const fe& a, u32 k) {  // small k (< 2^20)
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c = (u64)a.v[i] * k + (c >> 32);
        r.v[i] = lo32(c);
    }
    u32 top = hi32(c);  // fold top*(2^32+977)
    c = (u64)r.v[0] + (u64)top * 977u;
    r.v[0] = lo32(c);
    c = (u64)r.v[1] + top + (c >> 32);
    r.v[1] = lo32(c);
#pragma unroll
    for (int i = 2; i < 8; i++) {
        c = (u64)r.v[i] + (c >> 32);
        r.v[i] = lo32(c);
    }
    if (hi32(c)) {
        c = (u64)r.v[0] + 977u;
        r.v[0] = lo32(c);
        c = (u64)r.v[1] + 1u + (c >> 32);
        r.v[1] = lo32(c);
#pragma unroll
        for (int i = 2; i < 8; i++) {
            c = (u64)r.v[i] + (c >> 32);
            r.v[i] = lo32(c);
        }
    }
}

// r = 2^S a (S = 1..3)
template <int S>
BCC_HD void fe_shl(fe& r, const fe& a) {
#if defined(__HIP_DEVICE_COMPILE__)
    fe_shl_asm<S>(r.v, a.v);
#else
    fe_mul_int(r, a, 1u << S);
#endif
}

BCC_HD void fe_sqr_n(fe& r, const fe& a, int n) {
    r = a;
#pragma unroll 1
    for (int i = 0; i < n; i++) fe_sqr(r, r);
}

// Common prefix of the (p+1)/4 and p-2 addition chains: returns x223 = a^(2^223-1), x22, x2.
BCC_HD void fe_chain_x223(fe& x223, fe& x22, fe& x2, const fe& a) {
    fe x3, x6, x9, x11, x44, x88, x176, x220, t;
    fe_sqr(x2, a);
    fe_mul(x2, x2, a);
    fe_sqr(x3, x2);
    fe_mul(x3, x3, a);
    fe_sqr_n(t, x3, 3);
    fe_mul(x6, t, x3);
    fe_sqr_n(t, x6, 3);
    fe_mul(x9, t, x3);
    fe_sqr_n(t, x9, 2);
    fe_mul(x11, t, x2);
    fe_sqr_n(t, x11, 11);
    fe_mul(x22, t, x11);
    fe_sqr_n(t, x22, 22);
    fe_mul(x44, t, x22);
    fe_sqr_n(t, x44, 44);
    fe_mul(x88, t, x44);
    fe_sqr_n(t, x88, 88);
    fe_mul(x176, t, x88);
    fe_sqr_n(t, x176, 44);
    fe_mul(x220, t, x44);
    fe_sqr_n(t, x220, 3);
    fe_mul(x223, t, x3);
}

// r = a^((p+1)/4); returns whether r^2 == a (secp256k1_fe_sqrt semantics, field_impl.h:39-137)
BCC_HD bool fe_sqrt(fe& r, const fe& a) {
    fe x223, x22, x2, t;
    fe_chain_x223(x223, x22, x2, a);
    fe_sqr_n(t, x223, 23);
    fe_mul(t, t, x22);
    fe_sqr_n(t, t, 6);
    fe_mul(t, t, x2);
    fe_sqr(t, t);
    fe_sqr(r, t);
    fe_sqr(t, r);
    return fe_equal(t, a);
}

// r = a^-1 mod p (0 for a == 0): the safegcd inverse, 30-bit divstep batches on the device
// (modinv_device.h), 62-bit variable-time batches on the host (modinv_host.h).  Round 4 replaced
// the Fermat chain below (kept for BCC_INV_SAFEGCD=0 builds, the A/B baseline): C2 ECDSA stage
// 10.36-10.40 -> 9.99-10.01 ms, C3 staged ECDSA stage 1.41 -> 1.09 ms (profiles/r04/ab_safegcd).
#ifndef BCC_INV_SAFEGCD
#define BCC_INV_SAFEGCD 1
#endif
BCC_HD void fe_inv(fe& r, const fe& a) {
#if defined(BCC_FE_HOST64)
    const u32 P[8] = BCC_P_LIMBS;
    modinv::inverse_var(r.v, a.v, P);
    return;
#elif BCC_INV_SAFEGCD
    const u32 P[8] = BCC_P_LIMBS;
    fe an = a;
    fe_normalize(an);  // weak input: the inverse wants a < p
    mi30::inverse(r.v, an.v, P, 0x2ddacacfu);
    return;
#endif
    fe x223, x22, x2, t;
    fe_chain_x223(x223, x22, x2, a);
    fe_sqr_n(t, x223, 23);
    fe_mul(t, t, x22);
    fe_sqr_n(t, t, 5);
    fe_mul(t, t, a);
    fe_sqr_n(t, t, 3);
    fe_mul(t, t, x2);
    fe_sqr_n(t, t, 2);
    fe_mul(r, t, a);
}

// big-endian 32 bytes -> limbs
BCC_HD u32 bswap32(u32 x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}
BCC_HD void fe_from_be_words(fe& r, const u32 (&w)[8]) {  // w = the 8 big-endian words as loaded
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = bswap32(w[7 - i]);
}
BCC_HD void fe_from_be_bytes(fe& r, const uint8_t* b) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint8_t* q = b + 4 * (7 - i);
        r.v[i] = ((u32)q[0] << 24) | ((u32)q[1] << 16) | ((u32)q[2] << 8) | q[3];
    }
}
BCC_HD void fe_to_be_bytes(uint8_t* b, const fe& a) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint8_t* q = b + 4 * (7 - i);
        q[0] = (uint8_t)(a.v[i] >> 24);
        q[1] = (uint8_t)(a.v[i] >> 16);
        q[2] = (uint8_t)(a.v[i] >> 8);
        q[3] = (uint8_t)a.v[i];
    }
}

// ------------------------------------------------------------------------------------------
// 256-bit plain integer helpers (used for scalars)
// ------------------------------------------------------------------------------------------
BCC_HD bool u256_is_zero(const u32 (&a)[8]) {
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= a[i];
    return x == 0;
}
// a < b
BCC_HD bool u256_lt(const u32 (&a)[8], const u32 (&b)[8]) {
    u32 borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 d = (u64)a[i] - b[i] - borrow;
        borrow = (u32)(d >> 63);
    }
    return borrow != 0;
}
// r = a - b, returns borrow
BCC_HD u32 u256_sub(u32 (&r)[8], const u32 (&a)[8], const u32 (&b)[8]) {
    u32 borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 d = (u64)a[i] - b[i] - borrow;
        r[i] = lo32(d);
        borrow = (u32)(d >> 63);
    }
    return borrow;
}
BCC_HD u32 u256_add(u32 (&r)[8], const u32 (&a)[8], const u32 (&b)[8]) {
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c = (u64)a[i] + b[i] + (c >> 32);
        r[i] = lo32(c);
    }
    return hi32(c);
}

// ------------------------------------------------------------------------------------------
// Scalars mod n (always fully reduced)
// ------------------------------------------------------------------------------------------
struct sc {
    u32 v[8];
};

BCC_HD void sc_cond_sub_n(sc& r, u32 carry_in) {
    // subtract n if r >= n or carry_in
    const u32 N[8] = BCC_N_LIMBS;
    u32 t[8];
    u32 borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 d = (u64)r.v[i] - N[i] - borrow;
        t[i] = lo32(d);
        borrow = (u32)(d >> 63);
    }
    bool take = carry_in || !borrow;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = take ? t[i] : r.v[i];
}

// Column accumulator (acc: 64 bits, nh: the carry word above it) of the mod-n reduction.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void sc_mac(u64& acc, u32& nh, u32 a, u32 b) {
    asm("v_mad_u64_u32 %[acc], vcc, %[a], %[b], %[acc]\n\tv_addc_co_u32_e32 %[nh], vcc, 0, %[nh], vcc"
        : [acc] "+v"(acc), [nh] "+v"(nh) : [a] "v"(a), [b] "v"(b) : "vcc");
}
#else
inline void sc_mac(u64& acc, u32& nh, u32 a, u32 b) {
    const u64 p = (u64)a * b;
    acc += p;
    nh += acc < p ? 1u : 0u;
}
#endif
BCC_HD void sc_acc(u64& acc, u32& nh, u32 a) { sc_mac(acc, nh, a, 1u); }
BCC_HD u32 sc_col_out(u64& acc, u32& nh) {  // the column's word; acc moves to the next column
    const u32 w = lo32(acc);
    acc = (acc >> 32) | ((u64)nh << 32);
    nh = 0;
    return w;
}

// reduce a 512-bit value mod n: fold 2^256 == NC (129 bits: four limbs and a top 1) three times,
// each fold by product scanning (one accumulator over the columns, no per-row carry walks), then
// subtract n at most twice.  Bounds: m < 2^386 (13 limbs), q < 2^260 (9 limbs), s < 2^256 + 2^133.
BCC_HD void sc_reduce512(sc& r, const u32 (&t)[16]) {
    const u32 NC[5] = BCC_NC_LIMBS;
    u64 acc = 0;
    u32 nh = 0;
    // step 1: m = t_lo + t_hi * NC
    u32 m[13];
#pragma unroll
    for (int k = 0; k < 13; k++) {
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (k - j >= 0 && k - j < 8) sc_mac(acc, nh, t[8 + k - j], NC[j]);
        if (k >= 4 && k < 12) sc_acc(acc, nh, t[8 + k - 4]);
        if (k < 8) sc_acc(acc, nh, t[k]);
        m[k] = sc_col_out(acc, nh);
    }
    // step 2: q = m_lo + m_hi * NC (m_hi = m[8..12] < 2^130)
    acc = 0;
    nh = 0;
    u32 q[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (k - j >= 0 && k - j < 5) sc_mac(acc, nh, m[8 + k - j], NC[j]);
        if (k >= 4) sc_acc(acc, nh, m[8 + k - 4]);
        if (k < 8) sc_acc(acc, nh, m[k]);
        q[k] = sc_col_out(acc, nh);
    }
    // step 3: s = q_lo + q[8] * NC (q[8] < 16)
    acc = 0;
    nh = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (k < 4) sc_mac(acc, nh, q[8], NC[k]);
        if (k == 4) sc_acc(acc, nh, q[8]);
        sc_acc(acc, nh, q[k]);
        r.v[k] = sc_col_out(acc, nh);
    }
    const u32 carry = lo32(acc);  // bit 256 of s
    sc_cond_sub_n(r, carry);
    sc_cond_sub_n(r, 0);
}

#if defined(BCC_FE_HOST64)
// Host builds: the same three folds by 2^256 == NC over 64-bit words (NC = 2^256 - n, 129 bits).
inline void sc_reduce512_host64(sc& r, const u64 (&t)[8]) {
    typedef unsigned __int128 u128;
    const u64 NC[3] = {0x402DA1732FC9BEBFull, 0x4551231950B75FC4ull, 1ull};
    u64 m[7] = {t[0], t[1], t[2], t[3], 0, 0, 0};  // m = t_lo + t_hi NC < 2^386
    for (int i = 0; i < 4; i++) {
        u64 c = 0;
        for (int j = 0; j < 3; j++) {
            const u128 p = (u128)t[4 + i] * NC[j] + m[i + j] + c;
            m[i + j] = (u64)p;
            c = (u64)(p >> 64);
        }
        for (int k = i + 3; k < 7; k++) {
            const u128 p = (u128)m[k] + c;
            m[k] = (u64)p;
            c = (u64)(p >> 64);
        }
    }
    u64 q[5] = {m[0], m[1], m[2], m[3], 0};  // q = m_lo + m_hi NC < 2^260 (m_hi < 2^130)
    for (int i = 0; i < 3; i++) {
        u64 c = 0;
        for (int j = 0; j < 3 && i + j < 5; j++) {
            const u128 p = (u128)m[4 + i] * NC[j] + q[i + j] + c;
            q[i + j] = (u64)p;
            c = (u64)(p >> 64);
        }
        for (int k = i + 3; k < 5; k++) {
            const u128 p = (u128)q[k] + c;
            q[k] = (u64)p;
            c = (u64)(p >> 64);
        }
    }
    u64 w[4] = {q[0], q[1], q[2], q[3]};  // w = q_lo + q[4] NC < 2^256 + 2^133
    u64 c = 0;
    for (int j = 0; j < 3; j++) {
        const u128 p = (u128)q[4] * NC[j] + w[j] + c;
        w[j] = (u64)p;
        c = (u64)(p >> 64);
    }
    const u128 p = (u128)w[3] + c;
    w[3] = (u64)p;
    memcpy(r.v, w, 32);
    sc_cond_sub_n(r, (u32)(p >> 64));
    sc_cond_sub_n(r, 0);
}
#endif

BCC_HD void sc_mul(sc& r, const sc& a, const sc& b) {
#if defined(BCC_FE_HOST64)
    u64 t[8];
    mul_4x64(t, a.v, b.v);
    sc_reduce512_host64(r, t);
#else
    u32 t[16];
#if defined(__HIP_DEVICE_COMPILE__)
    mul_256x256_col(t, a.v, b.v);
#else
    mul_256x256(t, a.v, b.v);
#endif
    sc_reduce512(r, t);
#endif
}

BCC_HD void sc_sqr(sc& r, const sc& a) {
#if defined(BCC_FE_HOST64)
    sc_mul(r, a, a);
#else
    u32 t[16];
#if defined(__HIP_DEVICE_COMPILE__)
    sqr_256_col(t, a.v);
#else
    sqr_256(t, a.v);
#endif
    sc_reduce512(r, t);
#endif
}

BCC_HD void sc_add(sc& r, const sc& a, const sc& b) {
    u32 c = u256_add(r.v, a.v, b.v);
    sc_cond_sub_n(r, c);
}

BCC_HD void sc_neg(sc& r, const sc& a) {
    const u32 N[8] = BCC_N_LIMBS;
    bool z = u256_is_zero(a.v);
    u32 t[8];
    u256_sub(t, N, a.v);
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = z ? 0u : t[i];
}

BCC_HD bool sc_is_zero(const sc& a) { return u256_is_zero(a.v); }

// r = a^(n-2) mod n by a left-to-right sliding window (w = 4) over the constant exponent: the odd
// powers a, a^3, ..., a^15 in registers, then 58 steps "square sq times, multiply by a^(2 idx + 1)"
// (252 squarings + 58 + 7 multiplications, against 254 + 191 for plain square-and-multiply).  The
// step list is a constant table, so every branch is wave-uniform and the power table is indexed
// by constants only (no scratch).  The batched path (batch_sinv_kernel) amortises this.
BCC_HD void sc_inv(sc& r, const sc& a) {
#if defined(BCC_FE_HOST64)  // host builds: the variable-time safegcd inverse (modinv_host.h)
    const u32 N[8] = BCC_N_LIMBS;
    modinv::inverse_var(r.v, a.v, N);
    return;
#elif BCC_INV_SAFEGCD  // device: the 30-bit safegcd (modinv_device.h); a < n
    const u32 N[8] = BCC_N_LIMBS;
    mi30::inverse(r.v, a.v, N, 0x2a774ec1u);
    return;
#endif
    // n - 2 = FFFFFFFF FFFFFFFF FFFFFFFF FFFFFFFE BAAEDCE6 AF48A03B BFD25E8C D036413F
    static constexpr uint8_t SQ[58] = {0, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4,
                                       4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 3, 5, 3, 4, 4, 5, 2, 5, 6,
                                       5, 4, 3, 6, 10, 4, 5, 4, 5, 6, 4, 5, 6, 10, 4, 9, 4, 1};
    static constexpr uint8_t IX[58] = {7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,
                                       7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 3, 5, 2, 2, 3, 6, 1, 3, 6,
                                       5, 6, 0, 2, 3, 3, 7, 7, 4, 5, 6, 1, 6, 6, 4, 4, 7, 0};
    sc p0 = a, p1, p2, p3, p4, p5, p6, p7, a2;
    sc_sqr(a2, a);
    sc_mul(p1, p0, a2);
    sc_mul(p2, p1, a2);
    sc_mul(p3, p2, a2);
    sc_mul(p4, p3, a2);
    sc_mul(p5, p4, a2);
    sc_mul(p6, p5, a2);
    sc_mul(p7, p6, a2);
    sc acc = p7;  // step 0: a^15
#pragma unroll 1
    for (int k = 1; k < 58; k++) {
#pragma unroll 1
        for (int q = 0; q < SQ[k]; q++) sc_sqr(acc, acc);
        switch (IX[k]) {
        case 0: sc_mul(acc, acc, p0); break;
        case 1: sc_mul(acc, acc, p1); break;
        case 2: sc_mul(acc, acc, p2); break;
        case 3: sc_mul(acc, acc, p3); break;
        case 4: sc_mul(acc, acc, p4); break;
        case 5: sc_mul(acc, acc, p5); break;
        case 6: sc_mul(acc, acc, p6); break;
        default: sc_mul(acc, acc, p7); break;
        }
    }
    r = acc;
}

// r = round(a * g / 2^384) for 256-bit a, g (scalar_mul_shift_var semantics, shift 384)
BCC_HD void sc_mul_shift_384(sc& r, const sc& a, const u32 (&g)[8]) {
    u32 t[16];
    mul_256x256(t, a.v, g);
    // bits 384.. : limbs 12..15, rounding bit = bit 383 (limb 11 bit 31)
    u32 round = t[11] >> 31;
    u64 c = (u64)t[12] + round;
    r.v[0] = lo32(c);
    c = (u64)t[13] + (c >> 32);
    r.v[1] = lo32(c);
    c = (u64)t[14] + (c >> 32);
    r.v[2] = lo32(c);
    c = (u64)t[15] + (c >> 32);
    r.v[3] = lo32(c);
    r.v[4] = r.v[5] = r.v[6] = r.v[7] = 0;
}

// GLV: k == k1 + lambda*k2 (mod n), |k1|, |k2| < 2^128 (scalar_impl.h:342-375 bounds)
BCC_HD void sc_split_lambda(sc& k1, sc& k2, const sc& k) {
    const u32 G1[8] = BCC_G1_LIMBS, G2[8] = BCC_G2_LIMBS;
    sc mb1, mb2, lam, c1, c2;
    {
        const u32 a[8] = BCC_MB1_LIMBS, b[8] = BCC_MB2_LIMBS, l[8] = BCC_LAMBDA_LIMBS;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            mb1.v[i] = a[i];
            mb2.v[i] = b[i];
            lam.v[i] = l[i];
        }
    }
    sc_mul_shift_384(c1, k, G1);
    sc_mul_shift_384(c2, k, G2);
    sc_mul(c1, c1, mb1);
    sc_mul(c2, c2, mb2);
    sc_add(k2, c1, c2);
    sc_mul(k1, k2, lam);
    sc_neg(k1, k1);
    sc_add(k1, k1, k);
}

// ------------------------------------------------------------------------------------------
// Group law (Jacobian), curve y^2 = x^3 + b for any b: the formulas never use b, so they are
// valid on every isomorphic curve E_s: y^2 = x^3 + 7 s^6 used by the shared-Z table trick.
// ------------------------------------------------------------------------------------------
struct gej {
    fe x, y, z;
};

// dbl-2009-l (a = 0): 2M + 5S.  a must not be infinity (there is no 2-torsion, so the result
// is never infinity either).
BCC_HD void gej_double(gej& r, const gej& a) {
    fe A, B, C, D, E, F, t;
    fe_sqr(A, a.x);          // A = X^2
    fe_sqr(B, a.y);          // B = Y^2
    fe_sqr(C, B);            // C = B^2
    fe_add(t, a.x, B);
    fe_sqr(t, t);            // (X+B)^2
    fe_sub(t, t, A);
    fe_sub(t, t, C);
    fe_shl<1>(D, t);         // D = 2((X+B)^2 - A - C)
    fe_shl<1>(E, A);
    fe_add(E, E, A);         // E = 3A
    fe_sqr(F, E);            // F = E^2
    fe_mul(r.z, a.y, a.z);
    fe_shl<1>(r.z, r.z);     // Z3 = 2YZ
    fe_shl<1>(t, D);
    fe_sub(r.x, F, t);       // X3 = F - 2D
    fe_sub(t, D, r.x);
    fe_mul(t, E, t);
    fe_shl<3>(C, C);
    fe_sub(r.y, t, C);       // Y3 = E(D - X3) - 8C
}

// r = a + b where b is given as an affine point (bx, by) of the curve scaled by bzinv:
// b's Jacobian form is (bx, by, 1/bzinv).  bzinv == 1 gives the plain mixed addition.
// 8M + 3S (+1M when bzinv != 1: the caller passes use_zinv).  Exceptional cases
// (a == b -> double, a == -b -> infinity) are handled exactly like gej_add_zinv_var /
// gej_add_ge_var (group_impl.h:388-491).  a must not be infinity; *inf is set on the result.
BCC_HD void gej_add_zinv(gej& r, bool& inf, const gej& a, const fe& bx, const fe& by,
                         const fe& bzinv, bool use_zinv, fe* hout = nullptr) {
    fe az, z12, u2, s2, h, rr, hh, hhh, v, t;
    if (use_zinv) fe_mul(az, a.z, bzinv);
    else az = a.z;
    fe_sqr(z12, az);             // az^2
    fe_mul(u2, bx, z12);         // U2 = bx*az^2
    fe_mul(s2, by, z12);
    fe_mul(s2, s2, az);          // S2 = by*az^3
    fe_sub(h, u2, a.x);          // H = U2 - X1
    fe_sub(rr, s2, a.y);         // R = S2 - Y1
    if (fe_is_zero(h)) {         // rare, adversarial only
        if (fe_is_zero(rr)) {
            gej_double(r, a);
            inf = false;
        } else {
            inf = true;
            r = a;
        }
        return;
    }
    if (hout) *hout = h;
    fe_sqr(hh, h);               // H^2
    fe_mul(hhh, h, hh);          // H^3
    fe_mul(v, a.x, hh);          // V = X1*H^2
    fe_mul(r.z, a.z, h);         // Z3 = Z1*H (not az: the result stays on a's curve)
    fe_sqr(t, rr);
    fe_sub(t, t, hhh);
    fe_sub(t, t, v);
    fe_sub(r.x, t, v);           // X3 = R^2 - H^3 - 2V
    fe_sub(t, v, r.x);
    fe_mul(t, rr, t);
    fe_mul(hhh, a.y, hhh);
    fe_sub(r.y, t, hhh);         // Y3 = R(V - X3) - Y1*H^3
    inf = false;
}

}  // namespace bcc
