// tests/native/lane_host.cpp — TEST ONLY. Runs the product's per-lane signature code
// (rust-bitcoinconsensus_amd/csrc/ecdsa_twist.h + ecdsa_lane.h) on the CPU, so the exact arithmetic the HIP kernel
// executes can be checked against the oracle without a GPU. Never linked into the product.
#include "../../rust-bitcoinconsensus_amd/csrc/ecdsa_lane.h"
#include "../../rust-bitcoinconsensus_amd/csrc/ecdsa_twist.h"

#include <cstring>
#include <vector>

using namespace bcc;

static std::vector<fe>& gtab() {
    static std::vector<fe> t;
    if (t.empty()) {
        t.resize(2 * GTAB * 2);
        build_g_tables(t.data());
    }
    return t;
}

static std::vector<fe>& gcomb() {
    static std::vector<fe> t;
    if (t.empty()) {
        t.resize((size_t)CWIN * CTAB * 2);
        build_g_comb(t.data());
    }
    return t;
}

// the square-root-free ECDSA path (ecdsa_twist.h): the key header byte, x, y (ignored for 02/03),
// r, s and the message as 32-byte big-endian strings
extern "C" int lane_verify_twist(unsigned tag, const unsigned char* x32, const unsigned char* y32,
                                 const unsigned char* r32, const unsigned char* s32,
                                 const unsigned char* m32) {
    fe px, py, t;
    sc r, s, m;
    fe_from_be_bytes(px, x32);
    fe_from_be_bytes(py, y32);
    fe_from_be_bytes(t, r32);
    memcpy(r.v, t.v, 32);
    fe_from_be_bytes(t, s32);
    memcpy(s.v, t.v, 32);
    fe_from_be_bytes(t, m32);
    memcpy(m.v, t.v, 32);
    QTableArray qt;
    GCombArray gc{gcomb().data()};
    return ecdsa_verify_twist_lane(tag, px, py, r, s, m, qt, gc);
}

// the host engine's form of the same path (ecdsa_verify_twist_host: wNAF Q half, variable-time
// inverses), same arguments
extern "C" int lane_verify_twist_host(unsigned tag, const unsigned char* x32, const unsigned char* y32,
                                      const unsigned char* r32, const unsigned char* s32,
                                      const unsigned char* m32) {
    fe px, py, t;
    sc r, s, m;
    fe_from_be_bytes(px, x32);
    fe_from_be_bytes(py, y32);
    fe_from_be_bytes(t, r32);
    memcpy(r.v, t.v, 32);
    fe_from_be_bytes(t, s32);
    memcpy(s.v, t.v, 32);
    fe_from_be_bytes(t, m32);
    memcpy(m.v, t.v, 32);
    QTableArray qt;
    GCombArray gc{gcomb().data()};
    return ecdsa_verify_twist_host(tag, px, py, r, s, m, qt, gc);
}

// BIP340 on the square-root-free path (ecdsa_twist.h)
extern "C" int lane_schnorr_verify_twist(const unsigned char* sig64, const unsigned char* msg32,
                                         const unsigned char* xonly32) {
    fe px, rx, t;
    sc s, m;
    fe_from_be_bytes(rx, sig64);
    fe_from_be_bytes(t, sig64 + 32);
    memcpy(s.v, t.v, 32);
    fe_from_be_bytes(t, msg32);
    memcpy(m.v, t.v, 32);
    fe_from_be_bytes(px, xonly32);
    QTableArray qt;
    GCombArray gc{gcomb().data()};
    return schnorr_verify_twist_lane(px, rx, s, m, qt, gc);
}

// the generator's BIP340 signer (nonce supplied): returns 0 for d or k == 0
extern "C" int lane_schnorr_sign(const unsigned char* d32, const unsigned char* msg32,
                                 const unsigned char* k32, unsigned char* sig64,
                                 unsigned char* xonly32) {
    fe t, rx, px;
    sc d, m, k, s;
    fe_from_be_bytes(t, d32);
    memcpy(d.v, t.v, 32);
    fe_from_be_bytes(t, msg32);
    memcpy(m.v, t.v, 32);
    fe_from_be_bytes(t, k32);
    memcpy(k.v, t.v, 32);
    GTableArray gt{gtab().data()};
    if (!schnorr_sign_lane(d, m, k, rx, s, px, gt)) return 0;
    fe_to_be_bytes(sig64, rx);
    memcpy(t.v, s.v, 32);
    fe_to_be_bytes(sig64 + 32, t);
    fe_to_be_bytes(xonly32, px);
    return 1;
}

// field/scalar primitives for unit tests
extern "C" void lane_fe_mul(const unsigned char* a32, const unsigned char* b32, unsigned char* o32) {
    fe a, b, r;
    fe_from_be_bytes(a, a32);
    fe_from_be_bytes(b, b32);
    fe_mul(r, a, b);
    fe_normalize(r);
    fe_to_be_bytes(o32, r);
}
extern "C" void lane_fe_sqr(const unsigned char* a32, unsigned char* o32) {
    fe a, r;
    fe_from_be_bytes(a, a32);
    fe_sqr(r, a);
    fe_normalize(r);
    fe_to_be_bytes(o32, r);
}
extern "C" void lane_fe_addsub(const unsigned char* a32, const unsigned char* b32, unsigned char* sum,
                               unsigned char* diff) {
    fe a, b, r;
    fe_from_be_bytes(a, a32);
    fe_from_be_bytes(b, b32);
    fe_add(r, a, b);
    fe_normalize(r);
    fe_to_be_bytes(sum, r);
    fe_sub(r, a, b);
    fe_normalize(r);
    fe_to_be_bytes(diff, r);
}
extern "C" void lane_sc_mul(const unsigned char* a32, const unsigned char* b32, unsigned char* o32) {
    fe t;
    sc a, b, r;
    fe_from_be_bytes(t, a32);
    memcpy(a.v, t.v, 32);
    fe_from_be_bytes(t, b32);
    memcpy(b.v, t.v, 32);
    sc_mul(r, a, b);
    memcpy(t.v, r.v, 32);
    fe_to_be_bytes(o32, t);
}
extern "C" void lane_sc_inv(const unsigned char* a32, unsigned char* o32) {
    fe t;
    sc a, r;
    fe_from_be_bytes(t, a32);
    memcpy(a.v, t.v, 32);
    sc_inv(r, a);
    memcpy(t.v, r.v, 32);
    fe_to_be_bytes(o32, t);
}
extern "C" void lane_split(const unsigned char* k32, unsigned char* k1, unsigned char* k2) {
    fe t;
    sc k, a, b;
    fe_from_be_bytes(t, k32);
    memcpy(k.v, t.v, 32);
    sc_split_lambda(a, b, k);
    memcpy(t.v, a.v, 32);
    fe_to_be_bytes(k1, t);
    memcpy(t.v, b.v, 32);
    fe_to_be_bytes(k2, t);
}

// the GPU lanes' safegcd inverse (csrc/modinv_device.h) on the CPU: r = a^-1 mod m, little-endian
// 32-bit limbs, minv30 = m^-1 mod 2^30
extern "C" void lane_mi30_inverse(const uint32_t* a, const uint32_t* m, uint32_t minv30,
                                  uint32_t* r) {
    uint32_t aa[8], mm[8], rr[8];
    memcpy(aa, a, 32);
    memcpy(mm, m, 32);
    bcc::mi30::inverse(rr, aa, mm, minv30);
    memcpy(r, rr, 32);
}
