// K_der (round 5): the host half of CPubKey::Verify (pubkey.cpp:191-207) on the device, for
// bcc_pubkey_verify_batch from host buffers.  The caller's pubkey / signature blobs and their offset
// arrays go to HBM as they are (one DMA copy each, no host parse); one lane per tuple applies
//   * the CPubKey length filter (pubkey.h:58-94: 02/03 -> 33 bytes, 04/06/07 -> 65, else invalid),
//   * ecdsa_signature_parse_der_lax (pubkey.cpp:28-168): the lax length fields, leading zeros
//     stripped, an integer longer than 32 bytes or >= n -> (r, s) = (0, 0) (overflow, line 141-163),
//   * the r / s == 0 rejection of secp256k1_ecdsa_verify,
// and writes the row the ECDSA kernels read (tag 0 = rejected; x / y / r / s big-endian, y zero for
// 02/03).  The host restatement is csrc/host/sighash.cpp der_parse_lax / pubkey_size_valid; the
// parity tests run the same tuples through both (tests/test_tuples_gpu.py).
//
// Roofline: HBM / latency only -- ~150 algorithmic bytes per tuple read (pub ~33-65, sig ~71, two
// offsets, the row) and 161 written; the ~10^2 byte loads of a lane are uncoalesced but sit in the
// L2 lines its wave shares.  Small beside the ECDSA stage (~1 % of a C4 round).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pipeline.h"

namespace bcc {

namespace {

// One tuple's bytes, bounds-checked against the staged blob: a lane never reads outside
// [0, bytes) whatever the offsets say (an offset pair out of order or past the blob rejects the
// tuple; the host entry point checks the totals).
struct Span {
    const uint8_t* p;
    uint64_t len;
    bool ok;
};

__device__ __forceinline__ Span span(const uint8_t* blob, const uint64_t* off, uint64_t base,
                                     uint64_t bytes, uint32_t i) {
    const uint64_t a = off[i] - base, b = off[i + 1] - base;
    Span s{blob + a, b - a, a <= b && b <= bytes};
    if (!s.ok) s.len = 0;
    return s;
}

// the length field of an integer (pubkey.cpp:62-90 / 101-129 pattern; host der_len)
__device__ __forceinline__ bool der_len(const uint8_t* in, uint64_t inlen, uint64_t& pos,
                                        uint64_t& out) {
    if (pos == inlen) return false;
    uint64_t lenbyte = in[pos++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (lenbyte > inlen - pos) return false;
        while (lenbyte > 0 && in[pos] == 0) {
            pos++;
            lenbyte--;
        }
        if (lenbyte >= 4) return false;
        uint64_t v = 0;
        while (lenbyte > 0) {
            v = (v << 8) + in[pos];
            pos++;
            lenbyte--;
        }
        out = v;
    } else {
        out = lenbyte;
    }
    return true;
}

// 32 big-endian bytes right-aligned from in[pos .. pos + len) (len <= 32) as 8 memory-order words
__device__ __forceinline__ void load_be32(const uint8_t* in, uint64_t pos, uint32_t len, uint32_t w[8]) {
    const uint32_t lead = 32 - len;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t j = 4 * k + b;
            const uint32_t byte = j >= lead ? in[pos + j - lead] : 0u;
            v |= byte << (8 * b);
        }
        w[k] = v;
    }
}

// v >= n (the group order) for a memory-order big-endian 32-byte value
__device__ __forceinline__ bool ge_order(const uint32_t w[8]) {
    const uint32_t N[8] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFEu,
                           0xBAAEDCE6u, 0xAF48A03Bu, 0xBFD25E8Cu, 0xD0364141u};
    int64_t borrow = 0;  // v - N from the least significant word: no final borrow <=> v >= N
#pragma unroll
    for (int k = 7; k >= 0; k--) {
        const int64_t d = (int64_t)__builtin_bswap32(w[k]) - (int64_t)N[k] - borrow;
        borrow = d < 0;
    }
    return borrow == 0;
}

__device__ __forceinline__ void store32(uint8_t* dst, const uint32_t w[8]) {
    uint4* d = (uint4*)dst;
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__device__ __forceinline__ void load_bytes32(const uint8_t* p, uint32_t w[8]) {
#pragma unroll
    for (int k = 0; k < 8; k++)
        w[k] = (uint32_t)p[4 * k] | (uint32_t)p[4 * k + 1] << 8 | (uint32_t)p[4 * k + 2] << 16 |
               (uint32_t)p[4 * k + 3] << 24;
}

// ecdsa_signature_parse_der_lax (pubkey.cpp:28-168); false: the parse fails (Verify -> false)
__device__ bool der_parse_lax(const uint8_t* in, uint64_t inlen, uint32_t r[8], uint32_t s[8]) {
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = s[k] = 0;
    uint64_t pos = 0, rpos, rlen, spos, slen, lenbyte;
    if (pos == inlen || in[pos] != 0x30) return false;  // sequence tag
    pos++;
    if (pos == inlen) return false;  // sequence length (ignored beyond its own bytes)
    lenbyte = in[pos++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (lenbyte > inlen - pos) return false;
        pos += lenbyte;
    }
    if (pos == inlen || in[pos] != 0x02) return false;  // integer tag of R
    pos++;
    if (!der_len(in, inlen, pos, rlen)) return false;
    if (rlen > inlen - pos) return false;
    rpos = pos;
    pos += rlen;
    if (pos == inlen || in[pos] != 0x02) return false;  // integer tag of S
    pos++;
    if (!der_len(in, inlen, pos, slen)) return false;
    if (slen > inlen - pos) return false;
    spos = pos;
    while (rlen > 0 && in[rpos] == 0) {  // leading zeros
        rlen--;
        rpos++;
    }
    while (slen > 0 && in[spos] == 0) {
        slen--;
        spos++;
    }
    bool overflow = rlen > 32 || slen > 32;
    if (!overflow) {
        load_be32(in, rpos, (uint32_t)rlen, r);
        load_be32(in, spos, (uint32_t)slen, s);
        overflow = ge_order(r) || ge_order(s);  // secp256k1_ecdsa_signature_parse_compact
    }
    if (overflow) {
#pragma unroll
        for (int k = 0; k < 8; k++) r[k] = s[k] = 0;
    }
    return true;
}

__global__ void __launch_bounds__(256) der_rows_kernel(
    const uint8_t* __restrict__ pub, const uint64_t* __restrict__ pub_off, uint64_t pub_base,
    uint64_t pub_bytes, const uint8_t* __restrict__ sig, const uint64_t* __restrict__ sig_off,
    uint64_t sig_base, uint64_t sig_bytes, uint32_t n, uint8_t* __restrict__ tag,
    uint8_t* __restrict__ x, uint8_t* __restrict__ y, uint8_t* __restrict__ r,
    uint8_t* __restrict__ s) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Span pk = span(pub, pub_off, pub_base, pub_bytes, i);
    const Span sg = span(sig, sig_off, sig_base, sig_bytes, i);
    uint32_t h = pk.len ? pk.p[0] : 0u;
    const bool size_ok = ((h == 2 || h == 3) && pk.len == 33) ||
                         ((h == 4 || h == 6 || h == 7) && pk.len == 65);  // CPubKey::IsValid
    uint32_t rw[8], sw[8], xw[8], yw[8];
    bool ok = size_ok && sg.ok && der_parse_lax(sg.p, sg.len, rw, sw);
    if (ok) {
        uint32_t rz = 0, sz = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            rz |= rw[k];
            sz |= sw[k];
        }
        ok = rz != 0 && sz != 0;  // secp256k1_ecdsa_verify: r, s != 0
    }
#pragma unroll
    for (int k = 0; k < 8; k++) xw[k] = yw[k] = 0;
    if (ok) {
        load_bytes32(pk.p + 1, xw);
        if (pk.len == 65) load_bytes32(pk.p + 33, yw);
    } else {
        h = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) rw[k] = sw[k] = 0;
    }
    tag[i] = (uint8_t)h;
    store32(x + 32 * (size_t)i, xw);
    store32(y + 32 * (size_t)i, yw);
    store32(r + 32 * (size_t)i, rw);
    store32(s + 32 * (size_t)i, sw);
}

}  // namespace

int der_launch(const uint8_t* pub, const uint64_t* pub_off, uint64_t pub_base, uint64_t pub_bytes,
               const uint8_t* sig, const uint64_t* sig_off, uint64_t sig_base, uint64_t sig_bytes,
               size_t n, uint8_t* tag, uint8_t* x, uint8_t* y, uint8_t* r, uint8_t* s, void* stream) {
    if (n == 0) return 0;
    if (n >= ((size_t)1 << 32)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(der_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, pub, pub_off, pub_base, pub_bytes, sig, sig_off, sig_base,
                       sig_bytes, (uint32_t)n, tag, x, y, r, s);
    return (int)hipGetLastError();
}

}  // namespace bcc
