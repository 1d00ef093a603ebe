// ECDSA verify on gfx950: stages (b) and (c) of the hot path.  One lane = one tuple.
//
// Default, square-root-free path (ecdsa_twist.h):
//   K_inv     batch_sinv_kernel     s^-1 mod n by Montgomery's trick over strided chunks of <= 16
//                                   tuples (3 mults/tuple + one sliding-window Fermat inversion)
//   K_tprep   ecdsa_tprep_kernel    key parse without a square root, v = x^3 + 7, Q_w = (x v, v^2),
//                                   u1 u2, GLV split, co-Z Q_w table
//   K_tladder twist_ladder_kernel   B = u2 Q_w (Strauss, shared doublings), A = u1 G (fixed-base
//                                   comb from HBM tables), alpha / beta / K of the x-test
//   K_tfin    twist_fin_kernel      batched beta^-1, "gamma = -alpha / beta is the key's y",
//                                   exact fallback for the exceptional lanes
// BIP340 runs one fused prep + ladder launch (schnorr_tladder_kernel, round 4) and
// twist_fin_kernel<true>.  (The round-1
// path -- key decompression by a square root, G tables in LDS -- was retired in round 4.)
// K_inv needs only the s rows: DeviceBatch::run launches it on a side stream beside the sighash
// kernels.  Prep and ladder are separate launches so that each gets its own register allocation
// (ladder: 4 waves per SIMD).  Tuples are processed in chunks of up to 16M lanes so the per-tuple
// scratch (Q table + ladder state, ~1.4 KB) stays bounded.
//
// HBM layout (all device-resident):
//   tag[n]            u8   pubkey header byte (0 = rejected by the host length filter)
//   x[n][32], y[n][32]     pubkey coordinates, big-endian (y unused for 02/03)
//   r[n][32], s[n][32]     signature scalars after lax-DER (zero on overflow)
//   m[n][32]               sighash (raw SHA-256d bytes == big-endian integer)
//   verdict[n]        u8   1 = valid
//   scratch                per tuple s^-1, key y, key status; per chunk lane Q table (192 words)
//                          and ladder state (33 words) in wave blocks (lane_words below)
// Row loads are two 16-byte loads per lane (a wave covers one contiguous 2 KiB span); every
// scratch access of a wave is one 256-byte span.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

#include "ecdsa_lane.h"
#include "ecdsa_twist.h"
#include "gpu_common.h"
#include "pipeline.h"

namespace bcc {

// Per-lane scratch words in wave blocks: word w of lane t at
//   base[(t / 64) * (W * 64) + w * 64 + t % 64]
// so one wave's access to one word is 256 contiguous bytes and all W words of a wave's 64 lanes
// are one contiguous W * 256-byte block (few DRAM pages / TLB entries per wave, unlike a
// chunk-wide stride that puts consecutive words of a lane C * 4 bytes apart).
constexpr size_t LANE_STRIDE = 64;
__device__ __forceinline__ u32* lane_words(u32* base, size_t t, int W) {
    return base + (t >> 6) * (size_t)(W * 64) + (t & 63);
}
__device__ __forceinline__ const u32* lane_words(const u32* base, size_t t, int W) {
    return base + (t >> 6) * (size_t)(W * 64) + (t & 63);
}

// Per-lane Q table, lane-major: lane t's 1 KiB table is contiguous at base + t * QTABLE_WORDS,
// entry i at 32 words [x | y | beta*x | y] (y stored twice), so an addition reads its point
// (x, y) or (beta*x, y) as one aligned 64-byte piece with four 16-byte loads.  The ladder gathers
// by a per-lane digit index: with the entry words interleaved across lanes instead (word-major),
// each of those loads hit up to 8 table rows per wave and the L2 fetched ~3.7x the bytes used
// (rocprofv3 TCP_TCC_READ_REQ / SQ_INSTS_VMEM_RD = 14.7, 90 % L2 misses, profiles/r01g_pmc).
// Fields for put / get: 0 = x, 1 = beta*x (an H value while the table is built), 2 = y.
struct QTableGlobal {
    u32* base;
    __device__ static int field_off(int f) { return f == 0 ? 0 : f == 1 ? 16 : 8; }
    __device__ void put(int i, int f, const fe& a) {
        uint4* p = reinterpret_cast<uint4*>(base + i * 32 + field_off(f));
        p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
        p[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
        if (f == 2) {
            uint4* q = reinterpret_cast<uint4*>(base + i * 32 + 24);
            q[0] = p[0];
            q[1] = p[1];
        }
    }
    __device__ void get(int i, int f, fe& a) const {
        const uint4* p = reinterpret_cast<const uint4*>(base + i * 32 + field_off(f));
        const uint4 u = p[0], v = p[1];
        a.v[0] = u.x; a.v[1] = u.y; a.v[2] = u.z; a.v[3] = u.w;
        a.v[4] = v.x; a.v[5] = v.y; a.v[6] = v.z; a.v[7] = v.w;
    }
    // (x, y) for which == 0, (beta*x, y) for which == 1: one 64-byte piece
    __device__ void get_pair(int i, int which, fe& x, fe& y) const {
        const uint4* p = reinterpret_cast<const uint4*>(base + i * 32 + 16 * which);
        const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
        x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
        y.v[0] = c.x; y.v[1] = c.y; y.v[2] = c.z; y.v[3] = c.w;
        y.v[4] = d.x; y.v[5] = d.y; y.v[6] = d.z; y.v[7] = d.w;
    }
};
__device__ __forceinline__ u32* lane_table(u32* qtab, size_t t);
constexpr int QTABLE_WORDS = QTAB * 32;     // 256 words = 1 KiB per lane
__device__ __forceinline__ u32* lane_table(u32* qtab, size_t t) { return qtab + t * QTABLE_WORDS; }
constexpr int PRE_WORDS = 8;  // per tuple: s^-1

__device__ __forceinline__ void load_be32(fe& r, const uint8_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    u32 w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    fe_from_be_words(r, w);
}
__device__ __forceinline__ void load_be32(sc& r, const uint8_t* p) {
    fe t;
    load_be32(t, p);
#pragma unroll
    for (int k = 0; k < 8; k++) r.v[k] = t.v[k];
}
__device__ __forceinline__ void load_limbs(sc& r, const u32* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
}
__device__ __forceinline__ void store_limbs(u32* p, const sc& a) {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
    q[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}

__device__ __forceinline__ void sanitize_s(sc& s) {
    const u32 N[8] = BCC_N_LIMBS;
    if (u256_is_zero(s.v) || !u256_lt(s.v, N)) {
        s.v[0] = 1;
#pragma unroll
        for (int k = 1; k < 8; k++) s.v[k] = 0;
    }
}

// Tuples per thread of the batched inversions (K_inv: s^-1, K_tfin: beta^-1): one Fermat
// inversion per thread is shared by this many tuples (at least one wave per SIMD either way).
#ifndef BCC_INV_PER_THREAD
#define BCC_INV_PER_THREAD 16
#endif
#ifndef BCC_FIN_PER_THREAD
#define BCC_FIN_PER_THREAD 16
#endif
constexpr size_t INV_PER_THREAD = BCC_INV_PER_THREAD;
constexpr size_t FIN_PER_THREAD = BCC_FIN_PER_THREAD;

// Montgomery's simultaneous inversion over the strided chunk {t, t+T, t+2T, ...} (coalesced:
// at every step the wave touches 64 consecutive tuples).  s == 0 or s >= n is replaced by 1;
// the prep kernel rejects those tuples on the original s anyway.
__global__ __launch_bounds__(256) void batch_sinv_kernel(const uint8_t* __restrict__ ps,
                                                         u32* __restrict__ sinv, size_t n,
                                                         size_t T) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n || t >= T) return;
    sc acc, s;
    size_t last = t;
    load_be32(acc, ps + 32 * t);
    sanitize_s(acc);
    store_limbs(sinv + 8 * t, acc);
    for (size_t i = t + T; i < n; i += T) {
        load_be32(s, ps + 32 * i);
        sanitize_s(s);
        sc_mul(acc, acc, s);
        store_limbs(sinv + 8 * i, acc);  // prefix product s_t * ... * s_i
        last = i;
    }
    sc inv;
    sc_inv(inv, acc);
    for (size_t i = last; i >= t + T; i -= T) {
        load_be32(s, ps + 32 * i);
        sanitize_s(s);
        sc prev, out;
        load_limbs(prev, sinv + 8 * (i - T));
        sc_mul(out, inv, prev);  // (s_t..s_i)^-1 * (s_t..s_{i-1}) = s_i^-1
        sc_mul(inv, inv, s);     // (s_t..s_{i-1})^-1
        store_limbs(sinv + 8 * i, out);
    }
    store_limbs(sinv + 8 * t, inv);
}

#ifndef BCC_LADDER_WAVES
#define BCC_LADDER_WAVES 4  // waves per SIMD the ladder kernels are register-allocated for
#endif

// ------------------------------------------------------------------------------------------
// ECDSA, square-root-free path (ecdsa_twist.h): K_tprep -> K_tladder -> K_tfin.  The key is never
// decompressed (no K_key); A = u1 G comes from the comb tables in HBM, B = u2 Q_w from the
// lane's Q table; K_tfin inverts every lane's beta by Montgomery's trick and decides.
// Per-lane state words (wave blocks, TSTATE_WORDS per lane):
// ------------------------------------------------------------------------------------------
enum : int {
    T_K = 0,       // 16 scalar words: k1, k2, u1
    T_FLAGS = 16,
    T_SIGMA = 17,  // 8
    T_R = 25,      // 8
    T_V = 33,      // 8: x^3 + 7
    T_Y = 41,      // 8: y of an uncompressed key
    T_STAT = 49,   // TW_REJECT / TW_NORMAL / TW_EXCEPT (written by the ladder)
    T_AL = 50,     // 8: alpha
    T_BE = 58,     // 8: beta
    T_KK = 66,     // 8: K = Z3^2
    T_PRE = 74,    // 8: K_tfin's prefix product
    T_C0 = 82,     // 8: BIP340 only: c0, c1 of y(R) (T_KK then holds Dd)
    T_C1 = 90,
    TSTATE_WORDS = 98,
};

__device__ __forceinline__ void tw_store(u32* w, int at, const u32 (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++) w[(at + j) * LANE_STRIDE] = v[j];
}
__device__ __forceinline__ void tw_load(u32 (&v)[8], const u32* w, int at) {
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = w[(at + j) * LANE_STRIDE];
}

// The ladder's view of the twist state: flags and sigma in registers, the scalar words, r, v
// and y loaded at their use (address hidden from LICM as in LadderStateView).
struct TwistStateView {
    const u32* p;
    u32 flags;
    fe sigma;
    __device__ __forceinline__ u32 kword(int s, int w) const {
        const u32* q = p;
        asm volatile("" : "+v"(q));
        const __attribute__((address_space(1))) u32* g = (const __attribute__((address_space(1))) u32*)q;
        return g[(size_t)(T_K + s * 4 + w) * LANE_STRIDE];
    }
    __device__ __forceinline__ void get_r(sc& o) const { tw_load(o.v, p, T_R); }
    __device__ __forceinline__ void get_v(fe& o) const { tw_load(o.v, p, T_V); }
    __device__ __forceinline__ void get_y(fe& o) const { tw_load(o.v, p, T_Y); }
};

// comb tables in HBM: entry (win, i) = 16 words x || y, read as four 16-byte loads
struct GCombGlobal {
    const u32* base;
    __device__ void get(int win, int i, fe& x, fe& y) const {
        const uint4* q = reinterpret_cast<const uint4*>(base + ((size_t)win * CTAB + i) * 16);
        const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
        x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
        x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
        y.v[0] = c.x; y.v[1] = c.y; y.v[2] = c.z; y.v[3] = c.w;
        y.v[4] = d.x; y.v[5] = d.y; y.v[6] = d.z; y.v[7] = d.w;
    }
};

// a lane's parked Jacobian point in its own (dead after the Q loop) table words: 24 words + inf
__device__ __forceinline__ void park_gej(u32* q, const gej& a, bool inf) {
    uint4* p = reinterpret_cast<uint4*>(q);
    p[0] = make_uint4(a.x.v[0], a.x.v[1], a.x.v[2], a.x.v[3]);
    p[1] = make_uint4(a.x.v[4], a.x.v[5], a.x.v[6], a.x.v[7]);
    p[2] = make_uint4(a.y.v[0], a.y.v[1], a.y.v[2], a.y.v[3]);
    p[3] = make_uint4(a.y.v[4], a.y.v[5], a.y.v[6], a.y.v[7]);
    p[4] = make_uint4(a.z.v[0], a.z.v[1], a.z.v[2], a.z.v[3]);
    p[5] = make_uint4(a.z.v[4], a.z.v[5], a.z.v[6], a.z.v[7]);
    p[6] = make_uint4(inf ? 1u : 0u, 0u, 0u, 0u);
}
__device__ __forceinline__ bool unpark_gej(const u32* q, gej& a) {
    asm volatile("" : "+v"(q));  // a real reload: the point must not stay live in registers
    const uint4* p = reinterpret_cast<const uint4*>(q);
    uint4 u;
    u = p[0]; a.x.v[0] = u.x; a.x.v[1] = u.y; a.x.v[2] = u.z; a.x.v[3] = u.w;
    u = p[1]; a.x.v[4] = u.x; a.x.v[5] = u.y; a.x.v[6] = u.z; a.x.v[7] = u.w;
    u = p[2]; a.y.v[0] = u.x; a.y.v[1] = u.y; a.y.v[2] = u.z; a.y.v[3] = u.w;
    u = p[3]; a.y.v[4] = u.x; a.y.v[5] = u.y; a.y.v[6] = u.z; a.y.v[7] = u.w;
    u = p[4]; a.z.v[0] = u.x; a.z.v[1] = u.y; a.z.v[2] = u.z; a.z.v[3] = u.w;
    u = p[5]; a.z.v[4] = u.x; a.z.v[5] = u.y; a.z.v[6] = u.z; a.z.v[7] = u.w;
    return p[6].x != 0;
}
constexpr int PARK_B = 0, PARK_A = 32;  // word offsets in the lane's table

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void ecdsa_tprep_kernel(
    const uint8_t* __restrict__ tag, const uint8_t* __restrict__ px,
    const uint8_t* __restrict__ py, const uint8_t* __restrict__ pr, const uint8_t* __restrict__ ps,
    const uint8_t* __restrict__ pm, const u32* __restrict__ psinv, size_t base, size_t cnt,
    u32* __restrict__ qtab, u32* __restrict__ state) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const size_t i = base + t;
    fe x, y;
    sc r, s, m, si;
    load_be32(x, px + 32 * i);
    load_be32(y, py + 32 * i);
    load_be32(r, pr + 32 * i);
    load_be32(s, ps + 32 * i);
    load_be32(m, pm + 32 * i);
    load_limbs(si, psinv + 8 * i);
    QTableGlobal qt{lane_table(qtab, t)};
    TwistState st;
    twist_prep_lane(tag[i], x, y, r, s, m, &si, qt, st);
    u32* w = lane_words(state, t, TSTATE_WORDS);
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) w[(T_K + a * 4 + b) * LANE_STRIDE] = st.k[a][b];
    w[T_FLAGS * LANE_STRIDE] = st.flags;
    tw_store(w, T_SIGMA, st.sigma.v);
    tw_store(w, T_R, st.r.v);
    tw_store(w, T_V, st.v.v);
    tw_store(w, T_Y, st.ychk.v);
}

// Ladder workgroups of 256 lanes: no LDS (the comb tables are read from HBM / L2), so the only
// occupancy limit is the register file (4 waves per SIMD at <= 128 VGPRs).
#ifndef BCC_TLADDER_WG
#define BCC_TLADDER_WG 256
#endif
constexpr int TLADDER_WG = BCC_TLADDER_WG;

// The Q half of the ladder: B = u2 Q_w (or the BIP340 e P_w), parked in the lane's own table
// words (dead after the Q loop) for the G half.
__device__ __forceinline__ void twist_q_part(u32* lt, const TwistStateView& st) {
    gej B;
    const bool binf = twist_accumulate_q(st, QTableGlobal{lt}, B);
    park_gej(lt + PARK_B, B, binf);
}

// The G half: A = u1 G by the comb, B back from the table, the w-free combine; writes the lane's
// status (and alpha / beta / K, or the parked A for the exact fallback).
template <bool BIP340>
__device__ __forceinline__ void twist_g_part(u32* w, u32* lt, const u32* gcomb, TwistStateView& st) {
    u32 stat = TW_NORMAL;
    gej A, B;
    const bool ainf = twist_accumulate_g(st, GCombGlobal{gcomb}, A);
    const bool binf = unpark_gej(lt + PARK_B, B);
    fe v, al, be, K;
    sc r;
    st.get_v(v);
    st.get_r(r);  // loaded here, used last by the combine
    bool ok;
    if constexpr (BIP340) {
        fe c0, c1, rx;
#pragma unroll
        for (int j = 0; j < 8; j++) rx.v[j] = r.v[j];
        ok = !binf && !ainf && schnorr_twist_combine(A, B, st.sigma, v, rx, al, be, K, c0, c1);
        if (ok) {
            tw_store(w, T_C0, c0.v);
            tw_store(w, T_C1, c1.v);
        }
    } else {
        ok = !binf && !ainf && twist_combine(A, B, st.sigma, v, r, al, be, K);
    }
    if (!ok) {
        park_gej(lt + PARK_A, A, ainf);
        stat = TW_EXCEPT;
    } else {
        tw_store(w, T_AL, al.v);
        tw_store(w, T_BE, be.v);
        tw_store(w, T_KK, K.v);  // BIP340: Dd
    }
    w[T_STAT * LANE_STRIDE] = stat;
}

template <bool BIP340>
__global__ __launch_bounds__(TLADDER_WG) __attribute__((amdgpu_waves_per_eu(BCC_LADDER_WAVES, BCC_LADDER_WAVES))) void twist_ladder_kernel(
    u32* __restrict__ state, u32* __restrict__ qtab, const u32* __restrict__ gcomb, size_t cnt) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    u32* w = lane_words(state, t, TSTATE_WORDS);
    TwistStateView st;
    st.p = w;
    st.flags = w[T_FLAGS * LANE_STRIDE];
    if (!(st.flags & LS_VALID)) {
        w[T_STAT * LANE_STRIDE] = TW_REJECT;
        return;
    }
    tw_load(st.sigma.v, w, T_SIGMA);
    u32* lt = lane_table(qtab, t);
    twist_q_part(lt, st);
    twist_g_part<BIP340>(w, lt, gcomb, st);
}

// BIP340 in one launch per chunk (round 4, as K_keyq fuses the ECDSA key half): each lane runs
// the prep (key without a square root, e = H(r || P || m), the co-Z P_w table, the GLV split) and
// then the ladder (twist_ladder_kernel<true>'s body) on its own table and state words, so the
// prep's instructions fill the ladder's 4-wave SIMDs; as its own 3-wave launch (round 3's
// schnorr_tprep_kernel) it cost 14.2 of 149.6 ms per 16M rows.  Fused: C5 106.1-106.4 ->
// 110.9-111.8 M verifies/s in an interleaved A/B (profiles/r04/schnorr_fused).
__global__ __launch_bounds__(TLADDER_WG) __attribute__((amdgpu_waves_per_eu(BCC_LADDER_WAVES, BCC_LADDER_WAVES))) void schnorr_tladder_kernel(
    const uint8_t* __restrict__ psig, const uint8_t* __restrict__ pm,
    const uint8_t* __restrict__ ppk, size_t base, size_t cnt, u32* __restrict__ qtab,
    u32* __restrict__ state, const u32* __restrict__ gcomb) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const size_t i = base + t;
    u32* w = lane_words(state, t, TSTATE_WORDS);
    u32* lt = lane_table(qtab, t);
    {
        fe px, rx;
        sc s, m;
        load_be32(rx, psig + 64 * i);
        load_be32(s, psig + 64 * i + 32);
        load_be32(m, pm + 32 * i);
        load_be32(px, ppk + 32 * i);
        QTableGlobal qt{lt};
        TwistState st;
        schnorr_twist_prep(px, rx, s, m, qt, st);
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) w[(T_K + a * 4 + b) * LANE_STRIDE] = st.k[a][b];
        w[T_FLAGS * LANE_STRIDE] = st.flags;
        tw_store(w, T_SIGMA, st.sigma.v);
        tw_store(w, T_R, st.r.v);
        tw_store(w, T_V, st.v.v);
        tw_store(w, T_Y, st.ychk.v);
    }
    TwistStateView sv;
    sv.p = w;
    sv.flags = w[T_FLAGS * LANE_STRIDE];
    if (!(sv.flags & LS_VALID)) {
        w[T_STAT * LANE_STRIDE] = TW_REJECT;
        return;
    }
    tw_load(sv.sigma.v, w, T_SIGMA);
    twist_q_part(lt, sv);
    twist_g_part<true>(w, lt, gcomb, sv);
}

// The ECDSA ladder in two launches (ecdsa_launch_q / ecdsa_launch_after_pre): the Q half needs
// only the key and u2, so it runs on the side stream beside the sighash kernels; K_tladder_g
// forms u1 = m s^-1 from the sighash row (twist_prep_u1) and finishes the lane.
#ifndef BCC_LADDERQ_WAVES
#define BCC_LADDERQ_WAVES BCC_LADDER_WAVES
#endif
// The Q half, K_keyq (round 4: the former K_tkey + K_tscal_q + K_tladder_q in one launch, for
// rounds that fit one scratch chunk): key parse without a square root and the co-Z Q_w table, the r / s checks, u2 = r s^-1
// and its GLV split, then B = u2 Q_w.  The table build alone ran at about 60 % of the ladder's
// issue rate as its own launch (its 1 KiB lane-major table writes); fused, its instructions fill
// the same waves as the ladder's (108 VGPRs, 4 waves per SIMD, no spill).
__global__ __launch_bounds__(TLADDER_WG) __attribute__((amdgpu_waves_per_eu(BCC_LADDERQ_WAVES, BCC_LADDERQ_WAVES))) void twist_keyq_kernel(
    const uint8_t* __restrict__ tag, const uint8_t* __restrict__ px, const uint8_t* __restrict__ py,
    const uint8_t* __restrict__ pr, const uint8_t* __restrict__ ps, const u32* __restrict__ psinv,
    size_t cnt, u32* __restrict__ qtab, u32* __restrict__ state, const u32* __restrict__ emap,
    size_t ecount, size_t base) {
    const size_t t = base + (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // lanes [base, cnt)
    if (t >= cnt) return;
    if (emap && emap[t] < ecount) return;  // an early twin's result is copied (keyq_copy_kernel)
    u32* w = lane_words(state, t, TSTATE_WORDS);
    u32* lt = lane_table(qtab, t);
    {
        fe x, y;
        load_be32(x, px + 32 * t);
        load_be32(y, py + 32 * t);
        TwistState st;
        QTableGlobal qt{lt};
        bool ok = twist_prep_key(tag[t], x, y, qt, st);
        if (ok) {
            tw_store(w, T_SIGMA, st.sigma.v);
            tw_store(w, T_V, st.v.v);
            tw_store(w, T_Y, st.ychk.v);
            sc r, s, si;
            load_be32(r, pr + 32 * t);
            load_be32(s, ps + 32 * t);
            load_limbs(si, psinv + 8 * t);
            ok = twist_prep_u2(st.flags, r, s, &si, st);
        }
        if (!ok) {
            w[T_FLAGS * LANE_STRIDE] = 0u;  // K_tladder_g writes the status
            return;
        }
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) w[(T_K + a * 4 + b) * LANE_STRIDE] = st.k[a][b];
        w[T_FLAGS * LANE_STRIDE] = st.flags;
        tw_store(w, T_R, st.r.v);
    }
    TwistStateView sv;
    sv.p = w;
    sv.flags = w[T_FLAGS * LANE_STRIDE];
    tw_load(sv.sigma.v, w, T_SIGMA);
    twist_q_part(lt, sv);
}

// K_keyq's latency mode (round 5) for rounds of at most one wave per SIMD, where each verify's
// single-lane chain sets the round's length (C3: K_keyq ~0.93 ms beside a ~0.6 ms sighash front):
// two lanes per tuple.  Both parse the key and build the Q table (in their own areas of qtab2),
// lane 2t + h accumulates GLV half h (twist_accumulate_q_half: the 124 doublings, half the
// additions), lane 2t + 1 hands its point to lane 2t (cross-lane shuffles) and lane 2t parks
// B = B_0 + B_1 (the exceptional sums exact, gej_add_gej) and writes the tuple's state words as
// K_keyq does.  ~0.77x the chain of one lane, ~1.08x its instructions.
struct HalfK {  // twist_accumulate_q_half's view of one slot's k words (kword(slot, w) for its slot)
    u32 flags;
    u32 k[4];
    __device__ __forceinline__ u32 kword(int, int w) const { return k[w]; }
};
__device__ __forceinline__ void shfl_fe_xor1(fe& a) {
#pragma unroll
    for (int k = 0; k < 8; k++) a.v[k] = (u32)__shfl_xor((int)a.v[k], 1);
}
__global__ __launch_bounds__(TLADDER_WG) __attribute__((amdgpu_waves_per_eu(1, 2))) void twist_keyq2_kernel(
    const uint8_t* __restrict__ tag, const uint8_t* __restrict__ px, const uint8_t* __restrict__ py,
    const uint8_t* __restrict__ pr, const uint8_t* __restrict__ ps, const u32* __restrict__ psinv,
    size_t cnt, u32* __restrict__ qtab, u32* __restrict__ qtab2, u32* __restrict__ state,
    const u32* __restrict__ emap, size_t ecount) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t t = g >> 1;
    const int h = (int)(g & 1);
    // a pair's lanes stay together through the shuffles: a lane past the end (or an early twin's
    // pair) runs nothing, and so does its partner
    const bool live = t < cnt && !(emap && emap[t] < ecount);
    u32* lt2 = lane_table(qtab2, g);
    TwistState st;
    bool ok = false;
    if (live) {
        fe x, y;
        load_be32(x, px + 32 * t);
        load_be32(y, py + 32 * t);
        QTableGlobal qt{lt2};
        ok = twist_prep_key(tag[t], x, y, qt, st);
        if (ok) {
            sc r, s, si;
            load_be32(r, pr + 32 * t);
            load_be32(s, ps + 32 * t);
            load_limbs(si, psinv + 8 * t);
            ok = twist_prep_u2(st.flags, r, s, &si, st);
        }
    }
    u32* w = live ? lane_words(state, t, TSTATE_WORDS) : nullptr;
    if (live && h == 0) {
        if (!ok) {
            w[T_FLAGS * LANE_STRIDE] = 0u;  // K_tladder_g writes the status
        } else {
            tw_store(w, T_SIGMA, st.sigma.v);
            tw_store(w, T_V, st.v.v);
            tw_store(w, T_Y, st.ychk.v);
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 4; b++) w[(T_K + a * 4 + b) * LANE_STRIDE] = st.k[a][b];
            w[T_FLAGS * LANE_STRIDE] = st.flags;
            tw_store(w, T_R, st.r.v);
        }
    }
    gej B;
    bool binf = true;
    if (live && ok) {
        HalfK hk;  // this lane's half of the scalar words, in registers
        hk.flags = st.flags;
#pragma unroll
        for (int b = 0; b < 4; b++) hk.k[b] = h ? st.k[1][b] : st.k[0][b];
        binf = twist_accumulate_q_half(hk, QTableGlobal{lt2}, B, h);
    }
    // lane 2t + 1 -> lane 2t (every lane takes part: the partner's values arrive in lockstep)
    gej B1 = B;
    shfl_fe_xor1(B1.x);
    shfl_fe_xor1(B1.y);
    shfl_fe_xor1(B1.z);
    const bool b1inf = __shfl_xor(binf ? 1 : 0, 1) != 0;
    if (!(live && ok && h == 0)) return;
    gej S;
    bool sinf;
    if (binf) {
        S = B1;
        sinf = b1inf;
    } else if (b1inf) {
        S = B;
        sinf = false;
    } else {
        gej_add_gej(S, sinf, B, B1);
    }
    park_gej(lane_table(qtab, t) + PARK_B, S, sinf);
}

// Early Q halves (round 5, DeviceBatch::early_launch): a row whose (key, signature) bytes equal an
// early row's takes that lane's K_keyq output -- the state words K_keyq writes (the k1 / k2 words,
// flags, sigma, r, v, y: words [T_K, T_Y + 8)) and the parked B -- instead of recomputing it.
constexpr int KEYQ_STATE_WORDS = T_Y + 8;
constexpr int PARK_WORDS = 28;
__global__ __launch_bounds__(256) void keyq_copy_kernel(const u32* __restrict__ emap, size_t cnt,
                                                        size_t ecount, const u32* __restrict__ estate,
                                                        const u32* __restrict__ eqtab,
                                                        u32* __restrict__ state, u32* __restrict__ qtab) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const u32 e = emap[t];
    if (e >= ecount) return;
    const u32* src = lane_words(estate, e, TSTATE_WORDS);
    u32* dst = lane_words(state, t, TSTATE_WORDS);
#pragma unroll 7
    for (int k = 0; k < KEYQ_STATE_WORDS; k++) dst[k * LANE_STRIDE] = src[k * LANE_STRIDE];
    const uint4* ps = reinterpret_cast<const uint4*>(eqtab + (size_t)e * QTABLE_WORDS + PARK_B);
    uint4* pd = reinterpret_cast<uint4*>(qtab + t * QTABLE_WORDS + PARK_B);
#pragma unroll
    for (int k = 0; k < PARK_WORDS / 4; k++) pd[k] = ps[k];
}

// The G half keeps the combine's temporaries live beside the comb accumulator: at four waves
// per SIMD (128 VGPRs) it spills; BCC_LADDERG_WAVES selects its own occupancy (A/B builds).
#ifndef BCC_LADDERG_WAVES
#define BCC_LADDERG_WAVES BCC_LADDER_WAVES
#endif
__global__ __launch_bounds__(TLADDER_WG) __attribute__((amdgpu_waves_per_eu(BCC_LADDERG_WAVES, BCC_LADDERG_WAVES))) void twist_ladder_g_kernel(
    u32* __restrict__ state, u32* __restrict__ qtab, const u32* __restrict__ gcomb,
    const uint8_t* __restrict__ pm, const u32* __restrict__ psinv, size_t cnt, size_t base) {
    const size_t t = base + (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // lanes [base, cnt)
    if (t >= cnt) return;
    u32* w = lane_words(state, t, TSTATE_WORDS);
    u32 flags = w[T_FLAGS * LANE_STRIDE];
    if (!(flags & LS_VALID)) {
        w[T_STAT * LANE_STRIDE] = TW_REJECT;
        return;
    }
    {
        sc m, si;
        load_be32(m, pm + 32 * t);
        load_limbs(si, psinv + 8 * t);
        u32 k2[4], k3[4];
        twist_prep_u1(m, si, &flags, k2, k3);
#pragma unroll
        for (int b = 0; b < 4; b++) {
            w[(T_K + 8 + b) * LANE_STRIDE] = k2[b];
            w[(T_K + 12 + b) * LANE_STRIDE] = k3[b];
        }
        w[T_FLAGS * LANE_STRIDE] = flags;
    }
    TwistStateView st;
    st.p = w;
    st.flags = flags;
    tw_load(st.sigma.v, w, T_SIGMA);
    twist_g_part<false>(w, lane_table(qtab, t), gcomb, st);
}

// beta^-1 for every normal lane of a chunk by Montgomery's trick over the strided sub-chunk
// {t, t+T, ...} (3 mults per lane + one Fermat inversion per thread), then the verdicts; the
// exceptional lanes (adversarial only) run the exact fallback here, divergently.
template <bool BIP340>
__device__ __forceinline__ void twist_fin_elem(const u32* w, fe& c) {  // the inverted element
    tw_load(c.v, w, T_BE);
    if constexpr (BIP340) {
        fe dd;
        tw_load(dd.v, w, T_KK);
        fe_mul(c, c, dd);  // beta Dd
    }
}

template <bool BIP340>
__global__ __launch_bounds__(256) void twist_fin_kernel(u32* __restrict__ state,
                                                        const u32* __restrict__ qtab,
                                                        uint8_t* __restrict__ verdict,
                                                        size_t base, size_t cnt, size_t T,
                                                        int and_mode) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt || t >= T) return;
    fe acc = fe_one();
    size_t last = t;
    for (size_t i = t; i < cnt; i += T) {
        u32* w = lane_words(state, i, TSTATE_WORDS);
        tw_store(w, T_PRE, acc.v);  // product of the betas before i
        if (w[T_STAT * LANE_STRIDE] == TW_NORMAL) {
            fe b;
            twist_fin_elem<BIP340>(w, b);
            fe_mul(acc, acc, b);
        }
        last = i;
    }
    fe inv;
    fe_inv(inv, acc);
    for (size_t i = last + T; i > t;) {
        i -= T;
        const u32* w = lane_words(state, i, TSTATE_WORDS);
        const u32 stat = w[T_STAT * LANE_STRIDE];
        int ok = 0;
        if (stat != TW_REJECT) {
            const u32 flags = w[T_FLAGS * LANE_STRIDE];
            fe v, y;
            sc r;
            tw_load(v.v, w, T_V);
            tw_load(y.v, w, T_Y);
            tw_load(r.v, w, T_R);
            if (stat == TW_NORMAL) {
                fe pre, b, binv, al, K;
                tw_load(pre.v, w, T_PRE);
                twist_fin_elem<BIP340>(w, b);
                fe_mul(binv, inv, pre);  // element_i^-1
                fe_mul(inv, inv, b);     // (element_t ... element_{i-1})^-1
                tw_load(al.v, w, T_AL);
                tw_load(K.v, w, T_KK);
                if constexpr (BIP340) {
                    fe be, c0, c1;
                    tw_load(be.v, w, T_BE);
                    tw_load(c0.v, w, T_C0);
                    tw_load(c1.v, w, T_C1);
                    ok = schnorr_twist_final(al, be, K, c0, c1, binv, v);
                } else {
                    ok = twist_final(al, K, binv, v, y, flags, r);
                }
            } else {
                const u32* lt = lane_table(const_cast<u32*>(qtab), i);
                gej A, B;
                fe sigma;
                const bool ainf = unpark_gej(lt + PARK_A, A);
                const bool binf = unpark_gej(lt + PARK_B, B);
                tw_load(sigma.v, w, T_SIGMA);
                if constexpr (BIP340) {
                    fe rx;
#pragma unroll
                    for (int j = 0; j < 8; j++) rx.v[j] = r.v[j];
                    ok = schnorr_twist_exceptional(A, ainf, B, binf, sigma, v, rx);
                } else {
                    ok = twist_exceptional(A, ainf, B, binf, sigma, v, y, flags, r);
                }
            }
        }
        if (!and_mode) verdict[base + i] = (uint8_t)ok;
        else if (!ok) verdict[base + i] = 0;  // the caller preset the row to 1 (verdict_and)
    }
}

// ------------------------------------------------------------------------------------------
// Comb tables (one read-only copy per device) and caller-owned scratch
// ------------------------------------------------------------------------------------------
static std::mutex g_gtab_mu;
static u32* g_gcomb[64];
static int g_cus[64];

static const std::vector<fe>& host_gcomb() {
    static std::vector<fe> t;
    static std::once_flag once;
    std::call_once(once, [] {
        t.resize((size_t)CWIN * CTAB * 2);
        build_g_comb(t.data());
    });
    return t;
}

// Lanes per prep/ladder launch pair.  Larger chunks leave fewer kernel tails and fewer latency-
// bound K_tfin passes (measured on MI355X, C2 1M: 256k lanes 65.8M/s, 1M lanes 71.0M/s; C4 8M:
// 2M 75.6M/s, 4M 76.8M/s; round 3, C5 16M rows: 4M 100.1 / 100.5, 16M 107.4 / 106.7 M/s, C4 8M
// equal at 4M and 8M, profiles/r03/ab/chunk); 16M lanes cost at most ≈22 GiB of scratch per
// caller on a 288 GB device, allocated only up to the batch size.
static size_t default_chunk_lanes() {
    const char* e = getenv("BCC_CHUNK");
    return e ? (size_t)atol(e) : ((size_t)16 << 20);
}
static std::atomic<size_t> g_chunk_lanes{0};

static size_t chunk_lanes() {
    size_t v = g_chunk_lanes.load(std::memory_order_relaxed);
    if (v == 0) v = default_chunk_lanes();
    return std::max<size_t>(256, (v + 255) & ~(size_t)255);
}

// Current device, its comb tables and CU count.
static int device_tables(int* dev, const u32** gcomb, int* cus) {
    BCC_HIP_TRY(hipGetDevice(dev));
    if (*dev < 0 || *dev >= 64) return (int)hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_gtab_mu);
    if (!g_gcomb[*dev]) {
        BCC_HIP_TRY(hipDeviceGetAttribute(&g_cus[*dev], hipDeviceAttributeMultiprocessorCount, *dev));
        const auto& hc = host_gcomb();
        fe* dc = nullptr;
        BCC_HIP_TRY(hipMalloc(&dc, hc.size() * sizeof(fe)));
        BCC_HIP_TRY(hipMemcpy(dc, hc.data(), hc.size() * sizeof(fe), hipMemcpyHostToDevice));
        g_gcomb[*dev] = reinterpret_cast<u32*>(dc);
    }
    *gcomb = g_gcomb[*dev];
    *cus = g_cus[*dev];
    return 0;
}

SigScratch::~SigScratch() {
    if (dev >= 0 && (sinv || chunk || qtab2 || ev_qa || ev_ga || aux)) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(dev);
        if (aux) (void)hipStreamSynchronize((hipStream_t)aux);
        if (sinv) (void)hipFree(sinv);
        if (chunk) (void)hipFree(chunk);
        if (qtab2) (void)hipFree(qtab2);
        if (ev_qa) (void)hipEventDestroy((hipEvent_t)ev_qa);
        if (ev_ga) (void)hipEventDestroy((hipEvent_t)ev_ga);
        if (aux) (void)hipStreamDestroy((hipStream_t)aux);
        (void)hipSetDevice(cur);
    }
}

// Debug cap on the chunk scratch (tests, bcc_debug_scratch_cap_lanes): a larger request fails as
// out of memory without touching the device.
static std::atomic<size_t> g_scratch_cap{0};

static hipError_t chunk_malloc(void** p, size_t lanes) {
    const size_t cap = g_scratch_cap.load(std::memory_order_relaxed);
    if (cap && lanes > cap) return hipErrorOutOfMemory;
    return hipMalloc(p, lanes * (QTABLE_WORDS + TSTATE_WORDS) * sizeof(u32));
}

// Grows sc to n tuples (sinv rows when with_sinv) and min(n, chunk) lanes of chunk scratch;
// returns the chunk stride C.  When the device cannot hold the chunk (other callers' scratch, a
// smaller GPU) the request is halved until it fits (at least 64k lanes): the launches then loop
// over more, smaller chunks instead of failing the round.  The shortfall is remembered, so the
// calls of one round agree on C.
static int ensure_scratch(SigScratch& sc, int dev, size_t n, bool with_sinv, size_t* C) {
    if (sc.dev >= 0 && sc.dev != dev) return (int)hipErrorInvalidDevice;
    sc.dev = dev;
    const size_t want = std::min(chunk_lanes(), (n + 255) & ~(size_t)255);
    if (want > sc.chunk_cap && want != sc.chunk_short) {
        if (sc.chunk) BCC_HIP_TRY(hipFree(sc.chunk));
        sc.chunk = nullptr;
        sc.chunk_cap = 0;
        sc.chunk_short = 0;
        constexpr size_t MIN_LANES = (size_t)1 << 16;
        size_t lanes = want;
        for (;;) {
            const hipError_t e = chunk_malloc(&sc.chunk, lanes);
            if (e == hipSuccess) break;
            (void)hipGetLastError();
            sc.chunk = nullptr;
            if (e != hipErrorOutOfMemory || lanes <= MIN_LANES) return (int)e;
            lanes = std::max(MIN_LANES, (lanes / 2 + 255) & ~(size_t)255);
        }
        if (lanes < want) {
            fprintf(stderr, "[bcc] signature scratch: %zu lanes do not fit on device %d, using "
                            "chunks of %zu\n", want, dev, lanes);
            sc.chunk_short = want;
        }
        sc.chunk_cap = lanes;
    }
    if (with_sinv && n > sc.sinv_cap) {
        if (sc.sinv) BCC_HIP_TRY(hipFree(sc.sinv));
        sc.sinv = nullptr;
        sc.sinv_cap = 0;
        size_t cap = std::max<size_t>(n, 1 << 12);
        // per tuple: s^-1 (8 words), the loaded key's y (8 words) and its parse status (1 word)
        BCC_HIP_TRY(hipMalloc(&sc.sinv, cap * PRE_WORDS * sizeof(u32)));
        sc.sinv_cap = cap;
    }
    *C = std::min(want, sc.chunk_cap);
    return 0;
}

int ecdsa_launch_pre(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x,
                     const uint8_t* d_y, const uint8_t* d_s, size_t n, void* stream) {
    (void)d_tag;
    (void)d_x;
    (void)d_y;
    if (n == 0) return 0;
    int dev = 0, cus = 0;
    const u32* gcomb = nullptr;
    size_t C = 0;
    if (int e = device_tables(&dev, &gcomb, &cus)) return e;
    if (int e = ensure_scratch(sc, dev, n, true, &C)) return e;
    // K_inv: chunks of <= 16 tuples, but at least one wave per SIMD
    size_t T = std::max<size_t>((n + INV_PER_THREAD - 1) / INV_PER_THREAD, std::min<size_t>(n, (size_t)cus * 256));
    hipLaunchKernelGGL(batch_sinv_kernel, dim3((unsigned)((T + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_s, (u32*)sc.sinv, n, T);
    BCC_HIP_TRY(hipGetLastError());
    return 0;
}

// The key half runs inside the fused Q launch (twist_keyq_kernel, ecdsa_launch_q): this only
// marks the round's keys as handled there when the round fits one scratch chunk.
int ecdsa_launch_key(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x,
                     const uint8_t* d_y, size_t n, void* stream) {
    (void)d_tag;
    (void)d_x;
    (void)d_y;
    (void)stream;
    sc.key_ready = 0;
    if (n == 0 || n > chunk_lanes()) return 0;
    int dev = 0, cus = 0;
    const u32* gcomb = nullptr;
    size_t C = 0;
    if (int e = device_tables(&dev, &gcomb, &cus)) return e;
    if (int e = ensure_scratch(sc, dev, n, true, &C)) return e;
    if (n > C) return 0;  // chunked: the whole prep runs per chunk after K_inv
    sc.key_ready = n;
    return 0;
}

// Small rounds are latency-bound: at most one TLADDER_WG group per CU, every wave alone on its
// SIMD -- unless a workgroup of the sighash kernels running beside K_keyq on the other stream
// lands on the same CU and halves that SIMD's issue rate for the whole front (C3: K_keyq 0.85 ms
// alone, 1.7 ms beside the sighash front).  Such a launch therefore reserves nearly all of its
// CU's 160 KiB LDS (unused): the sighash kernels' groups (8.4 KB of LDS each) go to other CUs.
constexpr size_t KEYQ_EXCLUSIVE_LDS = 152 * 1024;

// The dynamic LDS that makes a group's total KEYQ_EXCLUSIVE_LDS (the kernel's static LDS counts:
// the two-lane kernel's low occupancy lets hipcc keep ~49 KiB of lane temporaries in LDS), or 0.
static size_t reserve_lds(const void* kernel, const char* name) {
    hipFuncAttributes fa;
    size_t fixed = 0;
    if (hipFuncGetAttributes(&fa, kernel) == hipSuccess) fixed = fa.sharedSizeBytes;
    else (void)hipGetLastError();
    const size_t dyn = fixed < KEYQ_EXCLUSIVE_LDS ? KEYQ_EXCLUSIVE_LDS - fixed : 0;
    const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    if (e == hipSuccess) return dyn;
    (void)hipGetLastError();
    fprintf(stderr, "[bcc] %s: no %zu-byte LDS reservation on this device (%s); small rounds "
                    "share CUs with the sighash kernels\n", name, dyn, hipGetErrorString(e));
    return 0;
}

static size_t keyq_lds(size_t groups, int cus, bool two_lane = false) {
    static const size_t dyn1 = reserve_lds((const void*)&twist_keyq_kernel, "K_keyq");
    static const size_t dyn2 = reserve_lds((const void*)&twist_keyq2_kernel, "K_keyq2");
    return groups <= (size_t)cus ? (two_lane ? dyn2 : dyn1) : 0;
}

// K_keyq or, for a round of at most one wave per SIMD at two lanes per tuple, its latency mode
// (twist_keyq2_kernel; BCC_KEYQ2=0 keeps K_keyq).
static const bool g_keyq2 = [] {
    const char* e = getenv("BCC_KEYQ2");
    return !(e && atoi(e) == 0);
}();
// The residency tail (round 6).  K_keyq holds BCC_LADDERQ_WAVES waves per SIMD, so one residency
// round is cus x 4 SIMDs x waves x 64 lanes (262,144 on MI355X); C2's 1M lanes are 3.81 rounds, and
// the last 0.81-full round left ~19 % of the chip idle for a whole round (~5 % of the stage;
// DESIGN §3.3).  Split at the last whole round, the tail round's idle slots take the G ladder of
// the lanes before it.  Returns the split (a multiple of the group size) or 0 for none
// (BCC_KEYQ_SPLIT=0, fewer than two rounds, or a whole number of rounds).
static const bool g_keyq_split = [] {
    const char* e = getenv("BCC_KEYQ_SPLIT");
    return !(e && atoi(e) == 0);
}();
static size_t keyq_split_at(size_t n, int cus) {
    const size_t R = (size_t)cus * 4 * BCC_LADDERQ_WAVES * 64;
    if (!g_keyq_split || R == 0 || n <= R || n % R == 0) return 0;
    return n / R * R;
}

static int launch_keyq(SigScratch& sc, int cus, const uint8_t* d_tag, const uint8_t* d_x,
                       const uint8_t* d_y, const uint8_t* d_r, const uint8_t* d_s, size_t n,
                       u32* qtab, u32* state, const u32* emap, size_t ecount, hipStream_t st) {
    sc.q_split = 0;
    if (g_keyq2 && 2 * n <= (size_t)cus * 4 * 64) {
        if (2 * n > sc.qtab2_cap) {
            if (sc.qtab2) BCC_HIP_TRY(hipFree(sc.qtab2));
            sc.qtab2 = nullptr;
            sc.qtab2_cap = 0;
            const size_t lanes = (2 * n + 255) & ~(size_t)255;
            BCC_HIP_TRY(hipMalloc(&sc.qtab2, lanes * QTABLE_WORDS * sizeof(u32)));
            sc.qtab2_cap = lanes;
        }
        const size_t groups = (2 * n + TLADDER_WG - 1) / TLADDER_WG;
        hipLaunchKernelGGL(twist_keyq2_kernel, dim3((unsigned)groups), dim3(TLADDER_WG),
                           (unsigned)keyq_lds(groups, cus, true), st, d_tag, d_x, d_y, d_r, d_s,
                           (const u32*)sc.sinv, n, qtab, (u32*)sc.qtab2, state, emap, ecount);
        return (int)hipGetLastError();
    }
    const size_t groups = (n + TLADDER_WG - 1) / TLADDER_WG;
    // a launch of several residency rounds plus a partial one: the whole rounds first, then the
    // partial round as a launch of its own, with an event between them (keyq_split_at)
    const size_t A = keyq_split_at(n, cus);
    if (A) {
        if (!sc.ev_qa) {
            hipEvent_t e = nullptr;
            BCC_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            sc.ev_qa = e;
        }
        hipLaunchKernelGGL(twist_keyq_kernel, dim3((unsigned)(A / TLADDER_WG)), dim3(TLADDER_WG), 0, st,
                           d_tag, d_x, d_y, d_r, d_s, (const u32*)sc.sinv, A, qtab, state, emap,
                           ecount, (size_t)0);
        BCC_HIP_TRY(hipGetLastError());
        BCC_HIP_TRY(hipEventRecord((hipEvent_t)sc.ev_qa, st));
        hipLaunchKernelGGL(twist_keyq_kernel, dim3((unsigned)((n - A + TLADDER_WG - 1) / TLADDER_WG)),
                           dim3(TLADDER_WG), 0, st, d_tag, d_x, d_y, d_r, d_s, (const u32*)sc.sinv,
                           n, qtab, state, emap, ecount, A);
        BCC_HIP_TRY(hipGetLastError());
        sc.q_split = A;
        return 0;
    }
    hipLaunchKernelGGL(twist_keyq_kernel, dim3((unsigned)groups), dim3(TLADDER_WG),
                       (unsigned)keyq_lds(groups, cus), st, d_tag, d_x, d_y, d_r, d_s,
                       (const u32*)sc.sinv, n, qtab, state, emap, ecount, (size_t)0);
    return (int)hipGetLastError();
}

int ecdsa_launch_q(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                   const uint8_t* d_r, const uint8_t* d_s, size_t n, void* stream) {
    sc.q_ready = 0;
    if (n == 0 || sc.key_ready != n || n > chunk_lanes()) return 0;
    int dev = 0, cus = 0;
    const u32* gcomb = nullptr;
    size_t C = 0;
    if (int e = device_tables(&dev, &gcomb, &cus)) return e;
    if (int e = ensure_scratch(sc, dev, n, true, &C)) return e;
    if (n > C) return 0;
    u32* qtab = (u32*)sc.chunk;
    u32* state = qtab + C * QTABLE_WORDS;
    if (int e = launch_keyq(sc, cus, d_tag, d_x, d_y, d_r, d_s, n, qtab, state, nullptr, 0,
                            (hipStream_t)stream))
        return e;
    sc.q_ready = n;
    return 0;
}

int ecdsa_launch_q_mapped(SigScratch& sc, const SigScratch& early, size_t early_n,
                          const uint32_t* d_emap, const uint8_t* d_tag, const uint8_t* d_x,
                          const uint8_t* d_y, const uint8_t* d_r, const uint8_t* d_s, size_t n,
                          void* stream) {
    if (!d_emap || early_n == 0 || !early.chunk)
        return ecdsa_launch_q(sc, d_tag, d_x, d_y, d_r, d_s, n, stream);
    sc.q_ready = 0;
    if (n == 0 || sc.key_ready != n || n > chunk_lanes()) return 0;
    int dev = 0, cus = 0;
    const u32* gcomb = nullptr;
    size_t C = 0;
    if (int e = device_tables(&dev, &gcomb, &cus)) return e;
    if (int e = ensure_scratch(sc, dev, n, true, &C)) return e;
    if (n > C) return 0;
    const size_t eC = std::min(chunk_lanes(), (early_n + 255) & ~(size_t)255);
    if (early.dev != dev || early_n > early.chunk_cap || eC > early.chunk_cap) return 0;  // cannot map: full K_keyq
    u32* qtab = (u32*)sc.chunk;
    u32* state = qtab + C * QTABLE_WORDS;
    const u32* eqtab = (const u32*)early.chunk;
    const u32* estate = eqtab + eC * QTABLE_WORDS;
    hipLaunchKernelGGL(keyq_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_emap, n, early_n, estate, eqtab, state, qtab);
    BCC_HIP_TRY(hipGetLastError());
    if (int e = launch_keyq(sc, cus, d_tag, d_x, d_y, d_r, d_s, n, qtab, state, d_emap, early_n,
                            (hipStream_t)stream))
        return e;
    sc.q_ready = n;
    return 0;
}

int ecdsa_launch(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                 const uint8_t* d_r, const uint8_t* d_s, const uint8_t* d_m, uint8_t* d_verdict,
                 size_t n, void* stream) {
    sc.key_ready = 0;
    sc.q_ready = 0;
    if (int e = ecdsa_launch_pre(sc, d_tag, d_x, d_y, d_s, n, stream)) return e;
    // the same split kernels as DeviceBatch::run, on one stream
    if (int e = ecdsa_launch_key(sc, d_tag, d_x, d_y, n, stream)) return e;
    if (int e = ecdsa_launch_q(sc, d_tag, d_x, d_y, d_r, d_s, n, stream)) return e;
    return ecdsa_launch_after_pre(sc, d_tag, d_x, d_y, d_r, d_s, d_m, d_verdict, n, stream);
}

int ecdsa_launch_after_pre(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x,
                           const uint8_t* d_y, const uint8_t* d_r, const uint8_t* d_s,
                           const uint8_t* d_m, uint8_t* d_verdict, size_t n, void* stream,
                           void* ev_rows_read, bool verdict_and, void* ev_q_done) {
    const int and_mode = verdict_and ? 1 : 0;
    if (n == 0) {  // nothing to launch; the stream still joins the other one
        if (ev_q_done) BCC_HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev_q_done, 0));
        return 0;
    }
    int dev = 0, cus = 0;
    const u32* gcomb = nullptr;
    size_t C = 0;
    if (int e = device_tables(&dev, &gcomb, &cus)) return e;
    if (int e = ensure_scratch(sc, dev, n, true, &C)) return e;  // sized by ecdsa_launch_pre
    hipStream_t sm = (hipStream_t)stream;
    u32* sinv = (u32*)sc.sinv;
    u32* qtab = (u32*)sc.chunk;
    u32* state = qtab + C * QTABLE_WORDS;
    const bool q_ahead = sc.q_ready == n && n <= C;
    const size_t A = q_ahead ? sc.q_split : 0;
    sc.key_ready = 0;
    sc.q_ready = 0;
    sc.q_split = 0;
    if (q_ahead && A && A < n) {
        // split K_keyq: the G ladder of lanes [0, A) as soon as their K_keyq is done, beside the
        // tail launch [A, n); the tail's G ladder after it
        if (ev_q_done) {  // K_keyq ran on another stream (DeviceBatch::run_stages)
            BCC_HIP_TRY(hipStreamWaitEvent(sm, (hipEvent_t)sc.ev_qa, 0));
            hipLaunchKernelGGL(twist_ladder_g_kernel, dim3((unsigned)(A / TLADDER_WG)), dim3(TLADDER_WG),
                               0, sm, state, qtab, gcomb, d_m, sinv, A, (size_t)0);
            BCC_HIP_TRY(hipGetLastError());
            BCC_HIP_TRY(hipStreamWaitEvent(sm, (hipEvent_t)ev_q_done, 0));
        } else {  // K_keyq queued on this stream: the first G ladder goes to the second stream
            if (!sc.aux) {
                hipStream_t a = nullptr;
                hipEvent_t g = nullptr;
                BCC_HIP_TRY(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
                BCC_HIP_TRY(hipEventCreateWithFlags(&g, hipEventDisableTiming));
                sc.aux = a;
                sc.ev_ga = g;
            }
            hipStream_t ax = (hipStream_t)sc.aux;
            BCC_HIP_TRY(hipStreamWaitEvent(ax, (hipEvent_t)sc.ev_qa, 0));
            hipLaunchKernelGGL(twist_ladder_g_kernel, dim3((unsigned)(A / TLADDER_WG)), dim3(TLADDER_WG),
                               0, ax, state, qtab, gcomb, d_m, sinv, A, (size_t)0);
            BCC_HIP_TRY(hipGetLastError());
            BCC_HIP_TRY(hipEventRecord((hipEvent_t)sc.ev_ga, ax));
            BCC_HIP_TRY(hipStreamWaitEvent(sm, (hipEvent_t)sc.ev_ga, 0));
        }
        hipLaunchKernelGGL(twist_ladder_g_kernel, dim3((unsigned)((n - A + TLADDER_WG - 1) / TLADDER_WG)),
                           dim3(TLADDER_WG), 0, sm, state, qtab, gcomb, d_m, sinv, n, A);
        BCC_HIP_TRY(hipGetLastError());
    } else if (q_ahead) {  // the key half, u2 and the Q ladder ran ahead (ecdsa_launch_q)
        if (ev_q_done) BCC_HIP_TRY(hipStreamWaitEvent(sm, (hipEvent_t)ev_q_done, 0));
        hipLaunchKernelGGL(twist_ladder_g_kernel, dim3((unsigned)((n + TLADDER_WG - 1) / TLADDER_WG)),
                           dim3(TLADDER_WG), 0, sm, state, qtab, gcomb, d_m, sinv, n, (size_t)0);
        BCC_HIP_TRY(hipGetLastError());
    }
    if (q_ahead) {
        if (ev_rows_read) BCC_HIP_TRY(hipEventRecord((hipEvent_t)ev_rows_read, sm));
        const size_t T = std::max<size_t>((n + FIN_PER_THREAD - 1) / FIN_PER_THREAD, std::min<size_t>(n, (size_t)cus * 256));
        hipLaunchKernelGGL(twist_fin_kernel<false>, dim3((unsigned)((T + 255) / 256)), dim3(256), 0,
                           sm, state, qtab, d_verdict, 0, n, T, and_mode);
        BCC_HIP_TRY(hipGetLastError());
        return 0;
    }
    // chunked (n above the scratch chunk): the whole prep, the fused ladder and K_tfin per chunk
    if (ev_q_done) BCC_HIP_TRY(hipStreamWaitEvent(sm, (hipEvent_t)ev_q_done, 0));  // K_inv's s^-1
    for (size_t base = 0; base < n; base += C) {
        const size_t cnt = std::min(C, n - base);
        hipLaunchKernelGGL(ecdsa_tprep_kernel, dim3((unsigned)((cnt + 255) / 256)),
                           dim3(256), 0, sm, d_tag, d_x, d_y, d_r, d_s, d_m, sinv, base,
                           cnt, qtab, state);
        BCC_HIP_TRY(hipGetLastError());
        if (ev_rows_read && base + cnt >= n)
            BCC_HIP_TRY(hipEventRecord((hipEvent_t)ev_rows_read, sm));
        hipLaunchKernelGGL(twist_ladder_kernel<false>,
                           dim3((unsigned)((cnt + TLADDER_WG - 1) / TLADDER_WG)),
                           dim3(TLADDER_WG), 0, sm, state, qtab, gcomb, cnt);
        BCC_HIP_TRY(hipGetLastError());
        // the batched beta inversion: sub-chunks of <= 16 lanes, at least one wave per SIMD
        const size_t T = std::max<size_t>((cnt + FIN_PER_THREAD - 1) / FIN_PER_THREAD, std::min<size_t>(cnt, (size_t)cus * 256));
        hipLaunchKernelGGL(twist_fin_kernel<false>, dim3((unsigned)((T + 255) / 256)), dim3(256), 0,
                           sm, state, qtab, d_verdict, base, cnt, T, and_mode);
        BCC_HIP_TRY(hipGetLastError());
    }
    return 0;
}

int schnorr_launch(SigScratch& sc, const uint8_t* d_sig64, const uint8_t* d_msg32,
                   const uint8_t* d_xonly32, uint8_t* d_verdict, size_t n, void* stream) {
    if (n == 0) return 0;
    int dev = 0, cus = 0;
    const u32* gcomb = nullptr;
    size_t C = 0;
    if (int e = device_tables(&dev, &gcomb, &cus)) return e;
    if (int e = ensure_scratch(sc, dev, n, false, &C)) return e;
    hipStream_t sm = (hipStream_t)stream;
    u32* qtab = (u32*)sc.chunk;
    u32* state = qtab + C * QTABLE_WORDS;
    for (size_t base = 0; base < n; base += C) {
        const size_t cnt = std::min(C, n - base);
        hipLaunchKernelGGL(schnorr_tladder_kernel,
                           dim3((unsigned)((cnt + TLADDER_WG - 1) / TLADDER_WG)), dim3(TLADDER_WG),
                           0, sm, d_sig64, d_msg32, d_xonly32, base, cnt, qtab, state, gcomb);
        BCC_HIP_TRY(hipGetLastError());
        const size_t T = std::max<size_t>((cnt + FIN_PER_THREAD - 1) / FIN_PER_THREAD, std::min<size_t>(cnt, (size_t)cus * 256));
        hipLaunchKernelGGL(twist_fin_kernel<true>, dim3((unsigned)((T + 255) / 256)), dim3(256), 0,
                           sm, state, qtab, d_verdict, base, cnt, T, 0);
        BCC_HIP_TRY(hipGetLastError());
    }
    return 0;
}

// The device-pointer ABI entries share one scratch per device (launches must be ordered on one
// stream per device, as documented in bcc_amd.h); the host-buffer entries below use a scratch and
// stream of their own per (thread, device).
static std::mutex g_shared_mu;
static SigScratch* g_shared[64];

static SigScratch* shared_scratch() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_shared_mu);
    if (!g_shared[dev]) g_shared[dev] = new SigScratch();  // lives for the process
    return g_shared[dev];
}

// Per (thread, device) context of the synchronous host-buffer entries: a stream, kernel scratch
// and one device + one pinned host buffer, grown on demand and reused by every later call (no
// per-call allocation; inputs go to HBM in one DMA copy from the pinned image).
struct ThreadCtx {
    SigScratch sc;
    hipStream_t stream = nullptr;
    int dev = -1;
    void* dbuf = nullptr;
    size_t dcap = 0;
    void* hbuf = nullptr;
    size_t hcap = 0;
    ~ThreadCtx() {
        if (dev >= 0) (void)hipSetDevice(dev);
        if (stream) (void)hipStreamDestroy(stream);
        if (dbuf) (void)hipFree(dbuf);
        if (hbuf) (void)hipHostFree(hbuf);
    }
    int reserve(size_t bytes) {
        if (bytes > dcap) {
            if (dbuf) BCC_HIP_TRY(hipFree(dbuf));
            dbuf = nullptr;
            dcap = 0;
            BCC_HIP_TRY(hipMalloc(&dbuf, bytes));
            dcap = bytes;
        }
        if (bytes > hcap) {
            if (hbuf) BCC_HIP_TRY(hipHostFree(hbuf));
            hbuf = nullptr;
            hcap = 0;
            BCC_HIP_TRY(hipHostMalloc(&hbuf, bytes, hipHostMallocDefault));
            hcap = bytes;
        }
        return 0;
    }
};

thread_local std::unique_ptr<ThreadCtx> tl_ctx[64];

// Frees the calling thread's tuple-path contexts (bcc_release_thread_state).
void release_tuple_thread_state() {
    for (auto& c : tl_ctx) c.reset();
}

static int thread_ctx(int device, ThreadCtx** out) {
    auto& ctx = tl_ctx;
    if (device < 0 || device >= 64) return (int)hipErrorInvalidDevice;
    if (!ctx[device]) {
        auto c = std::make_unique<ThreadCtx>();
        c->dev = device;
        BCC_HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        ctx[device] = std::move(c);
    }
    *out = ctx[device].get();
    return 0;
}

}  // namespace bcc

using namespace bcc;

extern "C" int bcc_set_chunk_lanes(size_t lanes) {
    bcc::g_chunk_lanes.store(lanes, std::memory_order_relaxed);
    return 0;
}

extern "C" {

// Device-pointer entry: all buffers already resident on the current device; launches on
// `stream` (hipStream_t, may be null). Returns 0 on success, else a hipError_t value.
int mi_ecdsa_verify_device(const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                           const uint8_t* d_r, const uint8_t* d_s, const uint8_t* d_m,
                           uint8_t* d_verdict, size_t n, void* stream) {
    if (n == 0) return 0;
    SigScratch* sc = shared_scratch();
    if (!sc) return (int)hipErrorInvalidDevice;
    return ecdsa_launch(*sc, d_tag, d_x, d_y, d_r, d_s, d_m, d_verdict, n, stream);
}

// BIP340 device-pointer entry: sig64 / msg32 / xonly32 rows resident on the current device
// (secp256k1_schnorrsig_verify per row, with the x-only key given as its 32 serialized bytes and
// parsed as secp256k1_xonly_pubkey_parse would; an unparsable key verifies false).
int mi_schnorr_verify_device(const uint8_t* d_sig64, const uint8_t* d_msg32,
                             const uint8_t* d_xonly32, uint8_t* d_verdict, size_t n,
                             void* stream) {
    if (n == 0) return 0;
    SigScratch* sc = shared_scratch();
    if (!sc) return (int)hipErrorInvalidDevice;
    return schnorr_launch(*sc, d_sig64, d_msg32, d_xonly32, d_verdict, n, stream);
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// BIP340 host-buffer entry: n rows of sig64 / msg32 / xonly32; synchronous on `device`.
int mi_schnorr_verify_tuples(const uint8_t* sig64, const uint8_t* msg32, const uint8_t* xonly32,
                             uint8_t* verdict, size_t n, int device) {
    if (n == 0) return 0;
    BCC_HIP_TRY(hipSetDevice(device));
    ThreadCtx* ctx = nullptr;
    if (int e = thread_ctx(device, &ctx)) return e;
    const size_t o_m = align256(64 * n), o_pk = o_m + align256(32 * n), o_v = o_pk + align256(32 * n);
    const size_t total = o_v + align256(n);
    if (int e = ctx->reserve(total)) return e;
    uint8_t* h = (uint8_t*)ctx->hbuf;
    uint8_t* d = (uint8_t*)ctx->dbuf;
    memcpy(h, sig64, 64 * n);
    memcpy(h + o_m, msg32, 32 * n);
    memcpy(h + o_pk, xonly32, 32 * n);
    int rc = 0;
    if ((rc = (int)hipMemcpyAsync(d, h, o_v, hipMemcpyHostToDevice, ctx->stream)) ||
        (rc = schnorr_launch(ctx->sc, d, d + o_m, d + o_pk, d + o_v, n, ctx->stream)) ||
        (rc = (int)hipMemcpyAsync(h + o_v, d + o_v, n, hipMemcpyDeviceToHost, ctx->stream)) ||
        (rc = (int)hipStreamSynchronize(ctx->stream))) {
        fprintf(stderr, "[bcc] mi_schnorr_verify_tuples failed: %d\n", rc);
        return rc;
    }
    memcpy(verdict, h + o_v, n);
    return 0;
}

// Host-buffer entry (the inner C ABI of SURVEY §8b): pub65[n] = header byte || x || y (y ignored
// for 02/03; header 0 = rejected by the caller's CPubKey length filter), msg32/r32/s32 big-endian.
// Copies in (one DMA copy from the thread's pinned image), verifies on `device`, copies verdicts
// out. Synchronous and reentrant: each calling thread has its own stream, scratch and buffers.
int mi_ecdsa_verify_tuples(const uint8_t* pub65, const uint8_t* msg32, const uint8_t* r32,
                           const uint8_t* s32, uint8_t* verdict, size_t n, int device) {
    if (n == 0) return 0;
    BCC_HIP_TRY(hipSetDevice(device));
    ThreadCtx* ctx = nullptr;
    if (int e = thread_ctx(device, &ctx)) return e;
    // layout: tag | x | y | r | s | m | verdict  (rows 256-byte aligned)
    const size_t tagb = align256(n), row = align256(32 * n);
    const size_t o_x = tagb, o_y = o_x + row, o_r = o_y + row, o_s = o_r + row, o_m = o_s + row,
                 o_v = o_m + row, total = o_v + tagb;
    if (int e = ctx->reserve(total)) return e;
    uint8_t* h = (uint8_t*)ctx->hbuf;
    uint8_t* d = (uint8_t*)ctx->dbuf;
    for (size_t i = 0; i < n; i++) {
        h[i] = pub65[65 * i];
        memcpy(h + o_x + 32 * i, pub65 + 65 * i + 1, 32);
        memcpy(h + o_y + 32 * i, pub65 + 65 * i + 33, 32);
    }
    memcpy(h + o_r, r32, 32 * n);
    memcpy(h + o_s, s32, 32 * n);
    memcpy(h + o_m, msg32, 32 * n);
    int rc = 0;
    if ((rc = (int)hipMemcpyAsync(d, h, o_v, hipMemcpyHostToDevice, ctx->stream)) ||
        (rc = ecdsa_launch(ctx->sc, d, d + o_x, d + o_y, d + o_r, d + o_s, d + o_m, d + o_v, n,
                           ctx->stream)) ||
        (rc = (int)hipMemcpyAsync(h + o_v, d + o_v, n, hipMemcpyDeviceToHost, ctx->stream)) ||
        (rc = (int)hipStreamSynchronize(ctx->stream))) {
        fprintf(stderr, "[bcc] mi_ecdsa_verify_tuples failed: %d\n", rc);
        return rc;
    }
    memcpy(verdict, h + o_v, n);
    return 0;
}

}  // extern "C"

extern "C" void bcc_debug_scratch_cap_lanes(size_t lanes) {
    g_scratch_cap.store(lanes, std::memory_order_relaxed);
}
