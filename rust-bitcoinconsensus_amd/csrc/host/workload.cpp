// Synthetic workloads built and staged in HBM for bench.py / tests.
//
// C2: n P2WPKH spends.  Key i = SHA256("mi355x-c2" || le64(seed) || le64(i)) mod n; tx = v2,
// 1 input (prevout txid = SHA256(le64(i) || le64(seed)), vout 0, nSequence 0xffffffff), 1 P2WPKH
// output, locktime 0; amount uniform in [546, 2.1e15]; BIP143 SIGHASH_ALL signatures, low-S DER;
// witness = [sig || 01, pubkey33]; spent script 0014 || HASH160(pubkey).  Nonces are derived as
// SHA256("mi355x-c2-nonce" || d || m) mod n (deterministic; RFC6979 is not needed for a verify
// benchmark).  Public keys and signatures come from the engine's GPU generator kernels.
//
// The staged device batch is exactly what bitcoinconsensus_verify_batch hands the GPU for these
// inputs: the engine's own first-round interpreter pass (build_first_round) builds it.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../pipeline.h"
#include "bcc_amd.h"
#include "engine.h"
#include "hashes.h"
#include "script.h"
#include "tx.h"

struct bcc_workload {
    int device = 0;
    size_t n = 0;
    std::vector<uint8_t> txblob;
    std::vector<size_t> txoff;  // n + 1
    std::vector<uint8_t> spk;   // 22 bytes per item
    std::vector<int64_t> amount;
    bcc::DeviceBatch* batch = nullptr;
};

namespace {

using namespace bcc::host;

const uint8_t N_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                          0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48,
                          0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};

bool scalar_ok(const uint8_t* k) {
    bool zero = true;
    for (int i = 0; i < 32; i++) zero &= k[i] == 0;
    return !zero && memcmp(k, N_BE, 32) < 0;
}

// scalar from a hash with rejection (probability of a retry ~2^-128)
void derive_scalar(const uint8_t* msg, size_t len, uint8_t out[32]) {
    std::vector<uint8_t> m(msg, msg + len);
    m.push_back(0);
    for (uint8_t ctr = 0;; ctr++) {
        m.back() = ctr;
        sha256(m.data(), ctr == 0 ? len : m.size(), out);
        if (scalar_ok(out)) return;
    }
}

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

void put_le(std::vector<uint8_t>& o, uint64_t v, int k) {
    for (int i = 0; i < k; i++) o.push_back((uint8_t)(v >> (8 * i)));
}

template <class F>
void parallel_for(size_t n, F f) {
    unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 4096) T = 1;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; t++)
        th.emplace_back([=]() {
            size_t lo = n * t / T, hi = n * (t + 1) / T;
            f(lo, hi, t);
        });
    for (auto& x : th) x.join();
}

// DER encoding of (r, s) (strict, minimal) || hashtype
void der_encode(const uint8_t* r, const uint8_t* s, uint8_t hashtype, std::vector<uint8_t>& out) {
    auto enc = [](const uint8_t* v, std::vector<uint8_t>& o) {
        int i = 0;
        while (i < 31 && v[i] == 0) i++;
        std::vector<uint8_t> b(v + i, v + 32);
        if (b[0] & 0x80) b.insert(b.begin(), 0);
        o.push_back(0x02);
        o.push_back((uint8_t)b.size());
        o.insert(o.end(), b.begin(), b.end());
    };
    std::vector<uint8_t> body;
    enc(r, body);
    enc(s, body);
    out.clear();
    out.push_back(0x30);
    out.push_back((uint8_t)body.size());
    out.insert(out.end(), body.begin(), body.end());
    out.push_back(hashtype);
}

}  // namespace

extern "C" {

bcc_workload* bcc_workload_p2wpkh(size_t n, uint64_t seed, int device) {
    auto* w = new bcc_workload();
    w->device = device;
    w->n = n;
    std::vector<uint8_t> d(32 * n), px(32 * n), py(32 * n), ok(n), m(32 * n), k(32 * n),
        r(32 * n), s(32 * n);
    // 1. keys
    parallel_for(n, [&](size_t lo, size_t hi, unsigned) {
        uint8_t buf[9 + 16];
        memcpy(buf, "mi355x-c2", 9);
        for (size_t i = lo; i < hi; i++) {
            for (int b = 0; b < 8; b++) buf[9 + b] = (uint8_t)(seed >> (8 * b));
            for (int b = 0; b < 8; b++) buf[17 + b] = (uint8_t)((uint64_t)i >> (8 * b));
            derive_scalar(buf, sizeof buf, &d[32 * i]);
        }
    });
    if (mi_gen_pubkeys(d.data(), n, px.data(), py.data(), ok.data(), device) != 0) {
        delete w;
        return nullptr;
    }
    // 2. unsigned txs + BIP143 sighashes (host, generation only)
    w->spk.resize(22 * n);
    w->amount.resize(n);
    std::vector<std::vector<uint8_t>> pubs(n);
    parallel_for(n, [&](size_t lo, size_t hi, unsigned) {
        std::vector<uint8_t> pre;
        for (size_t i = lo; i < hi; i++) {
            std::vector<uint8_t>& pub = pubs[i];
            pub.assign(33, 0);
            pub[0] = 0x02 | (py[32 * i + 31] & 1);
            memcpy(&pub[1], &px[32 * i], 32);
            uint8_t h160[20];
            hash160(pub.data(), 33, h160);
            uint8_t* spk = &w->spk[22 * i];
            spk[0] = 0x00;
            spk[1] = 0x14;
            memcpy(spk + 2, h160, 20);
            uint64_t rnd = splitmix64(seed ^ (0xA5A5A5A5ULL * (i + 1)));
            int64_t amount = 546 + (int64_t)(rnd % (uint64_t)(2100000000000000LL - 546 + 1));
            w->amount[i] = amount;
            // outpoint
            uint8_t outpoint[36], tmp[16];
            for (int b = 0; b < 8; b++) tmp[b] = (uint8_t)((uint64_t)i >> (8 * b));
            for (int b = 0; b < 8; b++) tmp[8 + b] = (uint8_t)(seed >> (8 * b));
            sha256(tmp, 16, outpoint);
            memset(outpoint + 32, 0, 4);
            // output: P2WPKH to HASH160(le64(i) || "out")
            uint8_t otmp[11], oh[20];
            for (int b = 0; b < 8; b++) otmp[b] = (uint8_t)((uint64_t)i >> (8 * b));
            memcpy(otmp + 8, "out", 3);
            hash160(otmp, 11, oh);
            std::vector<uint8_t> txout;
            put_le(txout, (uint64_t)(amount > 1546 ? amount - 1000 : amount), 8);
            txout.push_back(22);
            txout.push_back(0x00);
            txout.push_back(0x14);
            txout.insert(txout.end(), oh, oh + 20);
            // BIP143 (interpreter.cpp:1581-1625) with SIGHASH_ALL
            uint8_t hp[32], hs[32], ho[32], seq[4] = {0xff, 0xff, 0xff, 0xff};
            sha256d(outpoint, 36, hp);
            sha256d(seq, 4, hs);
            sha256d(txout.data(), txout.size(), ho);
            pre.clear();
            put_le(pre, 2, 4);
            pre.insert(pre.end(), hp, hp + 32);
            pre.insert(pre.end(), hs, hs + 32);
            pre.insert(pre.end(), outpoint, outpoint + 36);
            pre.push_back(25);
            const uint8_t code_head[3] = {0x76, 0xa9, 0x14};
            pre.insert(pre.end(), code_head, code_head + 3);
            pre.insert(pre.end(), h160, h160 + 20);
            pre.push_back(0x88);
            pre.push_back(0xac);
            put_le(pre, (uint64_t)amount, 8);
            put_le(pre, 0xffffffffu, 4);
            pre.insert(pre.end(), ho, ho + 32);
            put_le(pre, 0, 4);
            put_le(pre, 1, 4);
            sha256d(pre.data(), pre.size(), &m[32 * i]);
            // nonce
            uint8_t nb[15 + 64];
            memcpy(nb, "mi355x-c2-nonce", 15);
            memcpy(nb + 15, &d[32 * i], 32);
            memcpy(nb + 47, &m[32 * i], 32);
            derive_scalar(nb, sizeof nb, &k[32 * i]);
            // stash outpoint + txout for assembly (reuse pre as scratch: store in pub tail)
            pub.insert(pub.end(), outpoint, outpoint + 36);
            pub.insert(pub.end(), txout.begin(), txout.end());
        }
    });
    // 3. signatures (GPU)
    if (mi_gen_sign(d.data(), m.data(), k.data(), n, r.data(), s.data(), ok.data(), device) != 0) {
        delete w;
        return nullptr;
    }
    // 4. final txs (segwit serialization)
    std::vector<std::vector<uint8_t>> txs(n);
    parallel_for(n, [&](size_t lo, size_t hi, unsigned) {
        std::vector<uint8_t> sig;
        for (size_t i = lo; i < hi; i++) {
            const std::vector<uint8_t>& aux = pubs[i];
            const uint8_t* outpoint = aux.data() + 33;
            const uint8_t* txout = aux.data() + 33 + 36;
            size_t txout_len = aux.size() - 33 - 36;
            der_encode(&r[32 * i], &s[32 * i], 0x01, sig);
            std::vector<uint8_t>& t = txs[i];
            put_le(t, 2, 4);
            t.push_back(0x00);  // segwit marker
            t.push_back(0x01);  // flag
            t.push_back(1);     // vin count
            t.insert(t.end(), outpoint, outpoint + 36);
            t.push_back(0);     // empty scriptSig
            put_le(t, 0xffffffffu, 4);
            t.push_back(1);     // vout count
            t.insert(t.end(), txout, txout + txout_len);
            t.push_back(2);     // witness stack items
            t.push_back((uint8_t)sig.size());
            t.insert(t.end(), sig.begin(), sig.end());
            t.push_back(33);
            t.insert(t.end(), aux.begin(), aux.begin() + 33);
            put_le(t, 0, 4);    // locktime
        }
    });
    w->txoff.resize(n + 1);
    size_t total = 0;
    for (size_t i = 0; i < n; i++) {
        w->txoff[i] = total;
        total += txs[i].size();
    }
    w->txoff[n] = total;
    w->txblob.resize(total);
    for (size_t i = 0; i < n; i++) memcpy(&w->txblob[w->txoff[i]], txs[i].data(), txs[i].size());
    txs.clear();
    pubs.clear();
    // 5. the engine's first round over all items (threaded, merged in item order), staged in HBM
    std::vector<bcc_batch_item> items(n);
    for (size_t i = 0; i < n; i++)
        items[i] = bcc_batch_item{&w->spk[22 * i], 22, w->amount[i], &w->txblob[w->txoff[i]],
                                  (unsigned)(w->txoff[i + 1] - w->txoff[i]), 0};
    unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<bcc::SighashJobs> pj(T);
    std::vector<bcc::TupleRows> pr(T);
    parallel_for(n, [&](size_t lo, size_t hi, unsigned t) {
        build_first_round(items.data() + lo, hi - lo, FLAGS_VERIFY_ALL, pj[t], pr[t]);
    });
    bcc::SighashJobs jobs;
    bcc::TupleRows rows;
    for (unsigned t = 0; t < T; t++) {
        append_round(jobs, rows, pj[t], pr[t]);
        pj[t] = bcc::SighashJobs();
        pr[t] = bcc::TupleRows();
    }
    w->batch = new bcc::DeviceBatch(device);
    if (w->batch->stage(jobs, rows) != 0) {
        bcc_workload_free(w);
        return nullptr;
    }
    return w;
}

void bcc_workload_free(bcc_workload* w) {
    if (!w) return;
    delete w->batch;
    delete w;
}

size_t bcc_workload_size(const bcc_workload* w) { return w ? w->n : 0; }

int bcc_workload_run(bcc_workload* w, void* stream) { return w->batch->run(stream); }
int bcc_workload_run_sighash(bcc_workload* w, void* stream) { return w->batch->run_sighash(stream); }
int bcc_workload_run_ecdsa(bcc_workload* w, void* stream) { return w->batch->run_ecdsa(stream); }

int bcc_workload_verdicts(bcc_workload* w, uint8_t* out) { return w->batch->fetch_verdicts(out); }

void bcc_workload_shape(const bcc_workload* w, size_t* tuples, size_t* sighash_blocks,
                        size_t* aux_blocks, size_t* preimages, size_t* aux_messages) {
    if (tuples) *tuples = w->batch->n_tuples();
    if (sighash_blocks) *sighash_blocks = w->batch->pre_blocks();
    if (aux_blocks) *aux_blocks = w->batch->aux_blocks();
    if (preimages) *preimages = w->batch->n_pre();
    if (aux_messages) *aux_messages = w->batch->n_aux();
}

size_t bcc_workload_item(const bcc_workload* w, size_t i, uint8_t* spk, size_t* spk_len,
                         int64_t* amount, uint8_t* tx, size_t cap) {
    if (!w || i >= w->n) return 0;
    memcpy(spk, &w->spk[22 * i], 22);
    *spk_len = 22;
    *amount = w->amount[i];
    size_t len = w->txoff[i + 1] - w->txoff[i];
    memcpy(tx, &w->txblob[w->txoff[i]], std::min(len, cap));
    return len;
}

}  // extern "C"
