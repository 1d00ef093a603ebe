// Synthetic tuple sets (configs C4 / C5), staged in HBM for bench.py / tests.
//
//   bcc_tupleset_c4   deterministic (pub, msg32, DER sig) tuples, 90 % valid, 10 % spread over
//                     18 adversarial classes; the staged rows are exactly what
//                     bcc_pubkey_verify_batch's host front end (tuples.cpp) builds.
//   bcc_tupleset_c5   BIP340 (sig64, msg32, xonly32) rows, fresh GPU-signed signatures with the
//                     caller's vectors (the 15 BIP340 CSV rows) tiled in, for
//                     mi_schnorr_verify_device.
// Keys and signatures come from the engine's GPU generator kernels (gen.hip).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "pipeline.h"
#include "bcc_amd.h"
#include "bcc_bench.h"
#include "host/hashes.h"
#include "host/tuples.h"

using namespace bcc::host;

namespace {

const uint8_t N_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                          0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48,
                          0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};
const uint8_t P_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                          0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                          0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xFF, 0xFF, 0xFC, 0x2F};

// ---- generation helpers (synthetic inputs only) ----

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

bool scalar_ok(const uint8_t* k) {
    bool zero = true;
    for (int i = 0; i < 32; i++) zero &= k[i] == 0;
    return !zero && memcmp(k, N_BE, 32) < 0;
}

void derive_scalar(const uint8_t* msg, size_t len, uint8_t out[32]) {
    std::vector<uint8_t> m(msg, msg + len);
    m.push_back(0);
    for (uint8_t ctr = 0;; ctr++) {
        m.back() = ctr;
        sha256(m.data(), ctr == 0 ? len : m.size(), out);
        if (scalar_ok(out)) return;
    }
}

void tagged(const char* tag, uint64_t seed, uint64_t i, uint8_t out[32], bool scalar) {
    uint8_t buf[64];
    size_t L = strlen(tag);
    memcpy(buf, tag, L);
    for (int b = 0; b < 8; b++) buf[L + b] = (uint8_t)(seed >> (8 * b));
    for (int b = 0; b < 8; b++) buf[L + 8 + b] = (uint8_t)(i >> (8 * b));
    if (scalar)
        derive_scalar(buf, L + 16, out);
    else
        sha256(buf, L + 16, out);
}

// big-endian 256-bit helpers
void be_add_small(uint8_t* a, uint32_t v) {
    uint64_t c = v;
    for (int i = 31; i >= 0 && c; i--) {
        c += a[i];
        a[i] = (uint8_t)c;
        c >>= 8;
    }
}
void be_sub(const uint8_t* a, const uint8_t* b, uint8_t* o) {  // o = a - b (a >= b)
    int br = 0;
    for (int i = 31; i >= 0; i--) {
        int d = (int)a[i] - b[i] - br;
        br = d < 0;
        o[i] = (uint8_t)(d + (br << 8));
    }
}

// Host Fp (p = 2^256 - 0x1000003D1) with 4 x 64-bit limbs, only to pick off-curve x values.
using u128 = unsigned __int128;
struct Fe {
    uint64_t v[4];  // little-endian limbs
};
Fe fe_from_be(const uint8_t* b) {
    Fe r;
    for (int l = 0; l < 4; l++) {
        uint64_t w = 0;
        for (int k = 0; k < 8; k++) w = (w << 8) | b[(3 - l) * 8 + k];
        r.v[l] = w;
    }
    return r;
}
void fe_to_be(const Fe& a, uint8_t* b) {
    for (int l = 0; l < 4; l++)
        for (int k = 0; k < 8; k++) b[(3 - l) * 8 + k] = (uint8_t)(a.v[l] >> (56 - 8 * k));
}
Fe fe_mul(const Fe& a, const Fe& b) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)a.v[i] * b.v[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
    const uint64_t C = 0x1000003D1ULL;
    // fold hi * C into lo (twice), then conditional subtract
    u128 c = 0;
    uint64_t r[5];
    for (int i = 0; i < 4; i++) {
        c += (u128)t[4 + i] * C + t[i];
        r[i] = (uint64_t)c;
        c >>= 64;
    }
    r[4] = (uint64_t)c;
    c = (u128)r[4] * C;
    for (int i = 0; i < 4; i++) {
        c += r[i];
        r[i] = (uint64_t)c;
        c >>= 64;
    }
    if (c) {  // wrapped past 2^256: add C once more (cannot wrap again)
        u128 d = C;
        for (int i = 0; i < 4; i++) {
            d += r[i];
            r[i] = (uint64_t)d;
            d >>= 64;
        }
    }
    Fe o{{r[0], r[1], r[2], r[3]}};
    // o < 2^256; reduce mod p once if o >= p
    uint8_t be[32];
    fe_to_be(o, be);
    if (memcmp(be, P_BE, 32) >= 0) {
        u128 d = C;
        for (int i = 0; i < 4; i++) {
            d += o.v[i];
            o.v[i] = (uint64_t)d;
            d >>= 64;
        }
    }
    return o;
}
// Euler's criterion: a^((p-1)/2) == 1 (a != 0)
bool fe_is_square(const Fe& a) {
    // (p-1)/2 = 0x7FFFFFFF...FFFFFFFF 7FFFFE17
    uint8_t e[32];
    static const uint8_t ONE_BE[32] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                       0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
    be_sub(P_BE, ONE_BE, e);
    for (int i = 31; i >= 0; i--) e[i] = (uint8_t)((e[i] >> 1) | (i ? (e[i - 1] & 1) << 7 : 0));
    Fe r{{1, 0, 0, 0}};
    for (int bit = 255; bit >= 0; bit--) {
        r = fe_mul(r, r);
        if ((e[31 - bit / 8] >> (bit % 8)) & 1) r = fe_mul(r, a);
    }
    return r.v[0] == 1 && r.v[1] == 0 && r.v[2] == 0 && r.v[3] == 0;
}

// DER integer from its exact content bytes
void der_int(std::vector<uint8_t>& o, const uint8_t* c, size_t len) {
    o.push_back(0x02);
    o.push_back((uint8_t)len);
    o.insert(o.end(), c, c + len);
}
// minimal content bytes of a 32-byte big-endian value, with `extra_zeros` extra 0x00 pad bytes
// and optionally a non-zero `prefix` byte (an over-long integer)
std::vector<uint8_t> int_bytes(const uint8_t* v, int extra_zeros, int prefix) {
    int i = 0;
    while (i < 31 && v[i] == 0) i++;
    std::vector<uint8_t> b(v + i, v + 32);
    if (b[0] & 0x80) b.insert(b.begin(), 0);
    b.insert(b.begin(), (size_t)extra_zeros, 0);
    if (prefix) b.insert(b.begin(), (uint8_t)prefix);
    return b;
}
void der_sig(std::vector<uint8_t>& o, const std::vector<uint8_t>& rb, const std::vector<uint8_t>& sb) {
    o.clear();
    o.push_back(0x30);
    o.push_back((uint8_t)(4 + rb.size() + sb.size()));
    der_int(o, rb.data(), rb.size());
    der_int(o, sb.data(), sb.size());
}

}  // namespace

// ---- C4 adversarial classes -------------------------------------------------------------------
enum C4Class : uint8_t {
    C4_VALID = 0,
    C4_FLIP_R, C4_FLIP_S, C4_FLIP_MSG, C4_HIGH_S, C4_R_GE_N, C4_S_GE_N, C4_R_ZERO, C4_S_ZERO,
    C4_R_OVERLONG, C4_R_ZEROPAD, C4_PUB_NO_SQRT, C4_PUB_X_GE_P, C4_PUB_04_BAD_Y, C4_PUB_04,
    C4_PUB_HYBRID_OK, C4_PUB_HYBRID_BAD, C4_PUB_BAD_HEADER, C4_WRONG_KEY,
    C4_NCLASS
};
static const bool C4_EXPECT[C4_NCLASS] = {1, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 1, 1, 0, 0, 0};

struct bcc_tupleset {
    int device = 0;
    int kind = 0;  // 4: ECDSA (C4), 5: BIP340 (C5)
    size_t n = 0;
    // ECDSA: CPubKey::Verify inputs
    std::vector<uint8_t> pub_blob, sig_blob, msg;
    std::vector<uint64_t> pub_off, sig_off;
    // BIP340 rows
    std::vector<uint8_t> sig64, xonly;
    std::vector<uint8_t> cls, expect;
    bcc::DeviceBatch* batch = nullptr;  // C4 staged rows
    uint8_t* d_buf = nullptr;           // C5: sig64 | msg | xonly | verdict
};

extern "C" {

bcc_tupleset* bcc_tupleset_c4(size_t n, uint64_t seed, int device) {
    return bcc_tupleset_c4_range(n, seed, 0, n, device);
}

bcc_tupleset* bcc_tupleset_c4_range(size_t n, uint64_t seed, size_t first, size_t total,
                                    int device) {
    if (total < first + n || n == 0) return nullptr;
    auto* ts = new bcc_tupleset();
    ts->device = device;
    ts->kind = 4;
    ts->n = n;
    // keys for the n tuples plus the next global index (the wrong-key class takes key gi + 1)
    std::vector<uint8_t> d(32 * (n + 1)), m(32 * n), k(32 * n), px(32 * (n + 1)), py(32 * (n + 1)),
        ok(n + 1), r(32 * n), s(32 * n);
    ts->cls.resize(n);
    tagged("mi355x-c4", seed, (first + n) % total, &d[32 * n], true);
    pfor(n, 1024, [&](size_t lo, size_t hi) {
        for (size_t li = lo; li < hi; li++) {
            const size_t i = li, gi = first + li;  // local row, index in the global set
            tagged("mi355x-c4", seed, gi, &d[32 * i], true);
            tagged("mi355x-c4-msg", seed, gi, &m[32 * i], false);
            uint8_t nb[32 + 32 + 15];
            memcpy(nb, "mi355x-c4-nonce", 15);
            memcpy(nb + 15, &d[32 * i], 32);
            memcpy(nb + 47, &m[32 * i], 32);
            derive_scalar(nb, sizeof nb, &k[32 * i]);
            uint64_t u = splitmix64(seed * 0x9E37 + gi);
            ts->cls[i] = (u % 100) < 90 ? C4_VALID : (uint8_t)(1 + (u >> 8) % (C4_NCLASS - 1));
        }
    });
    if (mi_gen_pubkeys(d.data(), n + 1, px.data(), py.data(), ok.data(), device) != 0 ||
        mi_gen_sign(d.data(), m.data(), k.data(), n, r.data(), s.data(), ok.data(), device) != 0) {
        delete ts;
        return nullptr;
    }
    d.clear();
    k.clear();
    // per-tuple encodings (variable length), built in parallel then concatenated
    const unsigned T = pool_threads(n, 1024);
    std::vector<std::vector<uint8_t>> pb(T), sb(T);
    std::vector<std::vector<uint64_t>> plen(T), slen(T);
    ts->msg = m;
    ts->expect.resize(n);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; t++)
        th.emplace_back([&, t]() {
            size_t lo = n * t / T, hi = n * (t + 1) / T;
            std::vector<uint8_t> sig;
            for (size_t i = lo; i < hi; i++) {
                const uint8_t c = ts->cls[i];
                const size_t gi = first + i;
                uint64_t u = splitmix64(seed ^ (gi * 0xD1B54A32D192ED03ULL));
                uint8_t R[32], S[32], X[32], Y[32];
                memcpy(R, &r[32 * i], 32);
                memcpy(S, &s[32 * i], 32);
                memcpy(X, &px[32 * i], 32);
                memcpy(Y, &py[32 * i], 32);
                int rzeros = 0, rprefix = 0;
                uint8_t hdr = 0x02 | (Y[31] & 1);
                bool full = false;
                switch (c) {
                    case C4_FLIP_R: R[u % 32] ^= (uint8_t)(1 << ((u >> 5) % 8)); break;
                    case C4_FLIP_S: S[u % 32] ^= (uint8_t)(1 << ((u >> 5) % 8)); break;
                    case C4_FLIP_MSG: ts->msg[32 * i + u % 32] ^= (uint8_t)(1 << ((u >> 5) % 8)); break;
                    case C4_HIGH_S: be_sub(N_BE, S, S); break;
                    case C4_R_GE_N: memcpy(R, N_BE, 32); be_add_small(R, (uint32_t)(u & 0xffff)); break;
                    case C4_S_GE_N: memcpy(S, N_BE, 32); be_add_small(S, (uint32_t)(u & 0xffff)); break;
                    case C4_R_ZERO: memset(R, 0, 32); break;
                    case C4_S_ZERO: memset(S, 0, 32); break;
                    case C4_R_OVERLONG: rprefix = 1 + (int)(u % 127); break;
                    case C4_R_ZEROPAD: rzeros = 1 + (int)(u % 3); break;
                    case C4_PUB_NO_SQRT: {
                        uint8_t cand[32];
                        tagged("mi355x-c4-nosqrt", seed, gi, cand, false);
                        cand[0] &= 0x7f;  // < p
                        for (;;) {
                            Fe x = fe_from_be(cand);
                            Fe rhs = fe_mul(fe_mul(x, x), x);
                            uint8_t b[32];
                            fe_to_be(rhs, b);
                            be_add_small(b, 7);  // < p + 7: no wrap past p matters for squareness
                            if (memcmp(b, P_BE, 32) >= 0) be_sub(b, P_BE, b);
                            if (!fe_is_square(fe_from_be(b))) break;
                            be_add_small(cand, 1);
                        }
                        memcpy(X, cand, 32);
                        break;
                    }
                    case C4_PUB_X_GE_P: memcpy(X, P_BE, 32); be_add_small(X, (uint32_t)(u % 0x3D0)); break;
                    case C4_PUB_04_BAD_Y: full = true; hdr = 0x04; be_add_small(Y, 1 + (uint32_t)(u % 7)); break;
                    case C4_PUB_04: full = true; hdr = 0x04; break;
                    case C4_PUB_HYBRID_OK: full = true; hdr = 0x06 | (Y[31] & 1); break;
                    case C4_PUB_HYBRID_BAD: full = true; hdr = 0x06 | ((Y[31] & 1) ^ 1); break;
                    case C4_PUB_BAD_HEADER: hdr = 0x05; break;
                    case C4_WRONG_KEY: {  // the key of global tuple gi + 1 (row i + 1 here)
                        memcpy(X, &px[32 * (i + 1)], 32);
                        memcpy(Y, &py[32 * (i + 1)], 32);
                        hdr = 0x02 | (Y[31] & 1);
                        if ((gi + 1) % total == gi) X[31] ^= 1;
                        break;
                    }
                    default: break;
                }
                ts->expect[i] = C4_EXPECT[c];
                pb[t].push_back(hdr);
                pb[t].insert(pb[t].end(), X, X + 32);
                if (full) pb[t].insert(pb[t].end(), Y, Y + 32);
                plen[t].push_back(full ? 65 : 33);
                der_sig(sig, int_bytes(R, rzeros, rprefix), int_bytes(S, 0, 0));
                sb[t].insert(sb[t].end(), sig.begin(), sig.end());
                slen[t].push_back(sig.size());
            }
        });
    for (auto& x : th) x.join();
    ts->pub_off.assign(1, 0);
    ts->sig_off.assign(1, 0);
    for (unsigned t = 0; t < T; t++) {
        ts->pub_blob.insert(ts->pub_blob.end(), pb[t].begin(), pb[t].end());
        ts->sig_blob.insert(ts->sig_blob.end(), sb[t].begin(), sb[t].end());
        for (uint64_t L : plen[t]) ts->pub_off.push_back(ts->pub_off.back() + L);
        for (uint64_t L : slen[t]) ts->sig_off.push_back(ts->sig_off.back() + L);
        std::vector<uint8_t>().swap(pb[t]);
        std::vector<uint8_t>().swap(sb[t]);
    }
    // stage exactly the rows bcc_pubkey_verify_batch hands the kernels
    bcc::TupleRows rows;
    parse_rows(ts->pub_blob.data(), ts->pub_off.data(), ts->msg.data(), ts->sig_blob.data(),
               ts->sig_off.data(), n, rows);
    ts->batch = new bcc::DeviceBatch(device);
    if (ts->batch->stage(bcc::SighashJobs(), rows) != 0) {
        delete ts->batch;
        delete ts;
        return nullptr;
    }
    return ts;
}

bcc_tupleset* bcc_tupleset_c5(size_t n, uint64_t seed, const uint8_t* vec_sig64,
                              const uint8_t* vec_msg32, const uint8_t* vec_xonly32,
                              const uint8_t* vec_expect, size_t nvec, int device) {
    return bcc_tupleset_c5_range(n, seed, 0, vec_sig64, vec_msg32, vec_xonly32, vec_expect, nvec,
                                 device);
}

bcc_tupleset* bcc_tupleset_c5_range(size_t n, uint64_t seed, size_t first,
                                    const uint8_t* vec_sig64, const uint8_t* vec_msg32,
                                    const uint8_t* vec_xonly32, const uint8_t* vec_expect,
                                    size_t nvec, int device) {
    auto* ts = new bcc_tupleset();
    ts->device = device;
    ts->kind = 5;
    ts->n = n;
    std::vector<uint8_t> d(32 * n), k(32 * n), ok(n);
    ts->msg.resize(32 * n);
    ts->sig64.resize(64 * n);
    ts->xonly.resize(32 * n);
    ts->cls.assign(n, 0);
    ts->expect.assign(n, 1);
    pfor(n, 1024, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; i++) {
            tagged("mi355x-c5", seed, first + i, &d[32 * i], true);
            tagged("mi355x-c5-msg", seed, first + i, &ts->msg[32 * i], false);
            uint8_t nb[32 + 32 + 15];
            memcpy(nb, "mi355x-c5-nonce", 15);
            memcpy(nb + 15, &d[32 * i], 32);
            memcpy(nb + 47, &ts->msg[32 * i], 32);
            derive_scalar(nb, sizeof nb, &k[32 * i]);
        }
    });
    if (mi_gen_schnorr_sign(d.data(), ts->msg.data(), k.data(), n, ts->sig64.data(),
                            ts->xonly.data(), ok.data(), device) != 0) {
        delete ts;
        return nullptr;
    }
    // the caller's vectors tiled at a fixed stride: row i with i % 1024 == 1 + j is vector j
    if (nvec && vec_sig64 && vec_msg32 && vec_xonly32 && vec_expect)
        for (size_t i = 0; i < n; i++) {
            size_t j = (first + i) % 1024;
            if (j == 0 || j > nvec) continue;
            j -= 1;
            memcpy(&ts->sig64[64 * i], vec_sig64 + 64 * j, 64);
            memcpy(&ts->msg[32 * i], vec_msg32 + 32 * j, 32);
            memcpy(&ts->xonly[32 * i], vec_xonly32 + 32 * j, 32);
            ts->cls[i] = (uint8_t)(1 + j);
            ts->expect[i] = vec_expect[j];
        }
    if (hipSetDevice(device) != hipSuccess || hipMalloc((void**)&ts->d_buf, 129 * n) != hipSuccess) {
        delete ts;
        return nullptr;
    }
    uint8_t* b = ts->d_buf;
    if (hipMemcpy(b, ts->sig64.data(), 64 * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b + 64 * n, ts->msg.data(), 32 * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b + 96 * n, ts->xonly.data(), 32 * n, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(ts->d_buf);
        delete ts;
        return nullptr;
    }
    return ts;
}

void bcc_tupleset_free(bcc_tupleset* ts) {
    if (!ts) return;
    delete ts->batch;
    if (ts->d_buf) {
        (void)hipSetDevice(ts->device);
        (void)hipFree(ts->d_buf);
    }
    delete ts;
}

size_t bcc_tupleset_size(const bcc_tupleset* ts) { return ts ? ts->n : 0; }

int bcc_tupleset_run(bcc_tupleset* ts, void* stream) {
    if (!ts) return -1;
    if (ts->kind == 4) return ts->batch->run_ecdsa(stream);
    const size_t n = ts->n;
    uint8_t* b = ts->d_buf;
    if (hipSetDevice(ts->device) != hipSuccess) return -1;
    return mi_schnorr_verify_device(b, b + 64 * n, b + 96 * n, b + 128 * n, n, stream);
}

int bcc_tupleset_verdicts(bcc_tupleset* ts, uint8_t* out) {
    if (!ts) return -1;
    if (ts->kind == 4) return ts->batch->fetch_verdicts(out);
    if (hipSetDevice(ts->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpy(out, ts->d_buf + 128 * ts->n, ts->n, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

void bcc_tupleset_view(const bcc_tupleset* ts, bcc_tupleset_host* v) {
    memset(v, 0, sizeof *v);
    if (!ts) return;
    v->n = ts->n;
    v->msg32 = ts->msg.data();
    v->cls = ts->cls.data();
    v->expect = ts->expect.data();
    if (ts->kind == 4) {
        v->pub_blob = ts->pub_blob.data();
        v->pub_off = ts->pub_off.data();
        v->sig_blob = ts->sig_blob.data();
        v->sig_off = ts->sig_off.data();
    } else {
        v->sig64 = ts->sig64.data();
        v->xonly32 = ts->xonly.data();
    }
}

}  // extern "C"
