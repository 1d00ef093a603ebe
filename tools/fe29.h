// Fp in radix 2^29: nine limbs, value = sum v[i] 2^(29 i), lazily reduced.
//
// Why: the 8 x 32-bit product needs a carry capture (v_addc) behind every v_mad_u64_u32,
// because a 32x32 product fills the whole 64-bit accumulator.  With 29-bit limbs a column of
// nine products stays below 2^63.2 for limbs up to 2^30, so the product is 81 bare
// v_mad_u64_u32 (no carries, no inline asm), and additions are limb-wise v_add_u32 with no
// carry chain.  The reduction uses 2^261 == 2^37 + 31264 (mod p)  [2^256 == 2^32 + 977,
// field_10x26_impl.h's 0x3D10 / 0x400 fold, restated for 29-bit limbs].
//
// Magnitude contract (checked by tests/native and the fe_bench cross-check):
//   * fe9_mul / fe9_sqr accept limbs < 2^30 (i.e. any sum of two outputs) and return limbs
//     < 2^29 except v[2] < 2^29 + 2^20;  value < 2^261.
//   * fe9_add of two such values gives limbs < 2^30: a valid multiplication input.
//   * fe9_sub / fe9_neg return weakly normalized values (limbs < 2^29 + 2^20).
#pragma once
#include "secp256k1_device.h"

namespace bcc {

struct fe9 {
    u32 v[9];
};

constexpr u32 M29 = 0x1FFFFFFFu;

// 8 x 32 -> 9 x 29 (any 256-bit value; no reduction needed)
BCC_HD void fe9_from_fe(fe9& r, const fe& a) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
        int bit = 29 * i, w = bit >> 5, s = bit & 31;
        u32 lo = a.v[w] >> s;
        u32 hi = (s > 3 && w + 1 < 8) ? (a.v[w + 1] << (32 - s)) : 0u;
        r.v[i] = (lo | hi) & M29;
    }
}

// carry-propagate any lazy value (limbs < 2^32 - 2^5) to limbs < 2^29 (v[2] < 2^29 + 2^20)
BCC_HD void fe9_normalize_weak(fe9& r) {
    u32 c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        u32 x = r.v[i] + c;
        r.v[i] = x & M29;
        c = x >> 29;
    }
    // c = coefficient of 2^261 (< 2^4): fold c * (2^37 + 31264)
    u32 x0 = r.v[0] + c * 31264u;
    r.v[0] = x0 & M29;
    u32 x1 = r.v[1] + (c << 8) + (x0 >> 29);
    r.v[1] = x1 & M29;
    r.v[2] += x1 >> 29;
}

// 9 x 29 (lazy) -> canonical 8 x 32 (< p)
BCC_HD void fe9_to_fe(fe& r, const fe9& a_in) {
    fe9 a = a_in;
    fe9_normalize_weak(a);
    fe9_normalize_weak(a);  // now every limb < 2^29, value < 2^261
    u32 w[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 9; i++) {  // additive packing: a limb may exceed 29 bits slightly
        int bit = 29 * i, wi = bit >> 5, s = bit & 31;
        u64 x = (u64)a.v[i] << s;
        u64 acc = (u64)w[wi] + (u32)x;
        w[wi] = (u32)acc;
        acc = (acc >> 32) + w[wi + 1] + (u32)(x >> 32);
        w[wi + 1] = (u32)acc;
        for (int j = wi + 2; j < 10; j++) {
            acc = (acc >> 32) + w[j];
            w[j] = (u32)acc;
        }
    }
    // w[8] = bits 256..260: fold w8 * (2^32 + 977)
    u64 acc = (u64)w[8] * 977u + w[0];
    w[0] = (u32)acc;
    acc = (acc >> 32) + (u64)w[1] + w[8];
    w[1] = (u32)acc;
    acc >>= 32;
    for (int i = 2; i < 8; i++) {
        acc += w[i];
        w[i] = (u32)acc;
        acc >>= 32;
    }
    // acc (0/1) = a further 2^256: add 2^32 + 977 once more (cannot carry again)
    u32 c = (u32)acc;
    acc = (u64)w[0] + 977u * c;
    w[0] = (u32)acc;
    acc = (acc >> 32) + (u64)w[1] + c;
    w[1] = (u32)acc;
    acc >>= 32;
    for (int i = 2; i < 8; i++) {
        acc += w[i];
        w[i] = (u32)acc;
        acc >>= 32;
    }
    for (int i = 0; i < 8; i++) r.v[i] = w[i];
    fe_normalize(r);
}

// acc >> 29 without 64-bit shifts (v_alignbit_b32 + v_lshrrev_b32)
BCC_HD u64 shr29(u64 acc) {
    u32 lo = (u32)acc, hi = (u32)(acc >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
    u32 nlo = __builtin_amdgcn_alignbit(hi, lo, 29);
    u32 nhi = __builtin_amdgcn_alignbit(0u, hi, 29);
#else
    u32 nlo = (lo >> 29) | (hi << 3);
    u32 nhi = hi >> 29;
#endif
    return ((u64)nhi << 32) | nlo;
}

BCC_HD u64 mad64(u32 a, u32 b, u64 c) { return (u64)a * b + c; }

// t[0..17]: 29-bit columns of a product (t[17] < 2^31) -> r (limbs < 2^29, v[2] < 2^29 + 2^20)
BCC_HD void fe9_reduce(fe9& r, const u32 (&t)[18]) {
    // r_i = t_i + 31264 t_{i+9} + 256 t_{i+8} + carry: < 2^47, so the carry fits 32 bits and
    // t_i + carry < 2^30 enters the first v_mad_u64_u32 as its 64-bit addend
    u32 carry = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        u64 c = mad64(t[i + 9], 31264u, (u64)(t[i] + carry));
        if (i > 0) c = mad64(t[i + 8], 256u, c);
        r.v[i] = (u32)c & M29;
        carry = (u32)shr29(c);
    }
    // coefficient of 2^261: carry (< 2^18) + 256 t17 (< 2^39); fold * (2^37 + 31264)
    u64 top = mad64(t[17], 256u, (u64)carry);
    u32 tl = (u32)top & M29, th = (u32)shr29(top);      // top = th 2^29 + tl, th < 2^11
    u64 x0 = mad64(tl, 31264u, (u64)r.v[0]);            // < 2^45
    r.v[0] = (u32)x0 & M29;
    // limb 1 gets 256 tl + 31264 th (th 2^29 * 31264 lands on limb 1) + carry
    u64 x1 = mad64(tl, 256u, mad64(th, 31264u, (u64)(r.v[1] + (u32)shr29(x0))));
    r.v[1] = (u32)x1 & M29;
    // limb 2 gets 256 th + carry
    r.v[2] += (th << 8) + (u32)shr29(x1);
}

}  // namespace bcc
#include "fe29_asm_gen.h"
namespace bcc {

BCC_HD void fe9_mul(fe9& r, const fe9& a, const fe9& b) {
    u32 t[18];
#if defined(__HIP_DEVICE_COMPILE__)
    mul9_cols(t, a.v, b.v);
#else
    u64 acc = 0;
    for (int k = 0; k < 17; k++) {
        for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) acc = mad64(a.v[i], b.v[k - i], acc);
        t[k] = (u32)acc & M29;
        acc >>= 29;
    }
    t[17] = (u32)acc;
#endif
    fe9_reduce(r, t);
}

BCC_HD void fe9_sqr(fe9& r, const fe9& a) {
    u32 d[9];
#pragma unroll
    for (int i = 0; i < 9; i++) d[i] = a.v[i] << 1;
    u32 t[18];
#if defined(__HIP_DEVICE_COMPILE__)
    sqr9_cols(t, a.v, d);
#else
    u64 acc = 0;
    for (int k = 0; k < 17; k++) {
        for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; i++) acc = mad64(d[i], a.v[k - i], acc);
        if ((k & 1) == 0) acc = mad64(a.v[k / 2], a.v[k / 2], acc);
        t[k] = (u32)acc & M29;
        acc >>= 29;
    }
    t[17] = (u32)acc;
#endif
    fe9_reduce(r, t);
}

}  // namespace bcc
