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
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "pipeline.h"
#include "bcc_amd.h"
#include "bcc_bench.h"
#include "host/engine.h"
#include "host/hashes.h"
#include "host/script.h"
#include "host/sighash.h"
#include "host/tx.h"

struct bcc_workload {
    int device = 0;
    size_t n = 0;                // items (spends)
    std::vector<uint8_t> txblob;
    std::vector<size_t> txoff;   // per transaction, + 1
    std::vector<uint8_t> spkblob;
    std::vector<size_t> spkoff;  // per item, + 1
    std::vector<int64_t> amount;
    std::vector<uint32_t> item_tx, item_nin;
    std::vector<bcc_batch_item> items;  // borrowed pointers into the blobs above
    unsigned flags = bcc::host::FLAGS_VERIFY_ALL;
    std::vector<uint32_t> tuple_item;  // staged tuple row -> item
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
    T = (unsigned)std::max<size_t>(1, std::min<size_t>(T, n / 64));
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

void push_data(std::vector<uint8_t>& o, const uint8_t* p, size_t n) {
    if (n < 76) {
        o.push_back((uint8_t)n);
    } else {
        o.push_back(0x4c);  // OP_PUSHDATA1
        o.push_back((uint8_t)n);
    }
    o.insert(o.end(), p, p + n);
}

// Items from the blobs, then the engine's first interpreter round over all of them (threaded,
// merged in item order), staged in HBM: exactly the batch bitcoinconsensus_verify_batch hands the
// GPU first.  Frees w and returns nonzero on failure.
int finish(bcc_workload* w) {
    const size_t n = w->n;
    w->items.resize(n);
    for (size_t i = 0; i < n; i++) {
        size_t t = w->item_tx[i];
        w->items[i] = bcc_batch_item{&w->spkblob[w->spkoff[i]],
                                     (unsigned)(w->spkoff[i + 1] - w->spkoff[i]), w->amount[i],
                                     &w->txblob[w->txoff[t]],
                                     (unsigned)(w->txoff[t + 1] - w->txoff[t]), w->item_nin[i]};
    }
    unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<bcc::SighashJobs> pj(T);
    std::vector<bcc::TupleRows> pr(T);
    std::vector<std::vector<uint32_t>> ti(T);
    // split on transaction boundaries: items of one tx share its BIP143 aux messages
    std::vector<size_t> cut(T + 1, n);
    cut[0] = 0;
    for (unsigned t = 1; t < T; t++) {
        size_t c = std::max(cut[t - 1], n * t / T);
        while (c > 0 && c < n && w->item_tx[c] == w->item_tx[c - 1]) c++;
        cut[t] = c;
    }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; t++)
        th.emplace_back([&, t]() {
            build_first_round(w->items.data() + cut[t], cut[t + 1] - cut[t], w->flags, pj[t],
                              pr[t], &ti[t]);
        });
    for (auto& x : th) x.join();
    bcc::SighashJobs jobs;
    bcc::TupleRows rows;
    w->tuple_item.clear();
    for (unsigned t = 0; t < T; t++) {
        for (uint32_t i : ti[t]) w->tuple_item.push_back(i + (uint32_t)cut[t]);
        append_round(jobs, rows, pj[t], pr[t]);
        pj[t] = bcc::SighashJobs();
        pr[t] = bcc::TupleRows();
    }
    w->batch = new bcc::DeviceBatch(w->device);
    if (w->batch->stage(jobs, rows) != 0) {
        bcc_workload_free(w);
        return 1;
    }
    return 0;
}

}  // namespace

extern "C" {

bcc_workload* bcc_workload_p2wpkh(size_t n, uint64_t seed, int device) {
    return bcc_workload_p2wpkh_range(n, seed, 0, device);
}

bcc_workload* bcc_workload_p2wpkh_range(size_t n, uint64_t seed, size_t first, int device) {
    auto* w = new bcc_workload();
    w->device = device;
    w->n = n;
    std::vector<uint8_t> d(32 * n), px(32 * n), py(32 * n), ok(n), m(32 * n), k(32 * n),
        r(32 * n), s(32 * n);
    w->txoff.reserve(n + 1);
    // 1. keys
    parallel_for(n, [&](size_t lo, size_t hi, unsigned) {
        uint8_t buf[9 + 16];
        memcpy(buf, "mi355x-c2", 9);
        for (size_t i = lo; i < hi; i++) {
            for (int b = 0; b < 8; b++) buf[9 + b] = (uint8_t)(seed >> (8 * b));
            for (int b = 0; b < 8; b++) buf[17 + b] = (uint8_t)((uint64_t)(first + i) >> (8 * b));
            derive_scalar(buf, sizeof buf, &d[32 * i]);
        }
    });
    if (mi_gen_pubkeys(d.data(), n, px.data(), py.data(), ok.data(), device) != 0) {
        delete w;
        return nullptr;
    }
    // 2. unsigned txs + BIP143 sighashes (host, generation only)
    w->spkblob.resize(22 * n);
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
            uint8_t* spk = &w->spkblob[22 * i];
            spk[0] = 0x00;
            spk[1] = 0x14;
            memcpy(spk + 2, h160, 20);
            const uint64_t gi = first + i;  // index in the global (all-rank) set
            uint64_t rnd = splitmix64(seed ^ (0xA5A5A5A5ULL * (gi + 1)));
            int64_t amount = 546 + (int64_t)(rnd % (uint64_t)(2100000000000000LL - 546 + 1));
            w->amount[i] = amount;
            // outpoint
            uint8_t outpoint[36], tmp[16];
            for (int b = 0; b < 8; b++) tmp[b] = (uint8_t)(gi >> (8 * b));
            for (int b = 0; b < 8; b++) tmp[8 + b] = (uint8_t)(seed >> (8 * b));
            sha256(tmp, 16, outpoint);
            memset(outpoint + 32, 0, 4);
            // output: P2WPKH to HASH160(le64(i) || "out")
            uint8_t otmp[11], oh[20];
            for (int b = 0; b < 8; b++) otmp[b] = (uint8_t)(gi >> (8 * b));
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
    w->spkoff.resize(n + 1);
    w->item_tx.resize(n);
    w->item_nin.assign(n, 0);
    for (size_t i = 0; i <= n; i++) w->spkoff[i] = 22 * i;
    for (size_t i = 0; i < n; i++) w->item_tx[i] = (uint32_t)i;
    if (finish(w)) return nullptr;
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

int bcc_workload_verdicts(bcc_workload* w, uint8_t* out, size_t cap) {
    if (!w || !w->batch || !out) return -1;
    if (cap < w->batch->n_tuples()) return BCC_BENCH_ERR_CAPACITY;  // one byte per row, not per item
    return w->batch->fetch_verdicts(out);
}

void bcc_workload_shape(const bcc_workload* w, size_t* tuples, size_t* sighash_blocks,
                        size_t* aux_blocks, size_t* preimages, size_t* aux_messages) {
    if (tuples) *tuples = w->batch->n_tuples();
    if (sighash_blocks) *sighash_blocks = w->batch->pre_blocks();
    if (aux_blocks) *aux_blocks = w->batch->aux_blocks();
    if (preimages) *preimages = w->batch->n_pre();
    if (aux_messages) *aux_messages = w->batch->n_aux();
}

size_t bcc_workload_sighash_bytes(const bcc_workload* w) { return w ? w->batch->sighash_bytes() : 0; }

size_t bcc_workload_item(const bcc_workload* w, size_t i, uint8_t* spk, size_t* spk_len,
                         int64_t* amount, uint8_t* tx, size_t cap) {
    if (!w || i >= w->n) return 0;
    const bcc_batch_item& it = w->items[i];
    memcpy(spk, it.script_pubkey, std::min<size_t>(it.script_pubkey_len, 64));
    *spk_len = it.script_pubkey_len;
    *amount = it.amount;
    memcpy(tx, it.tx_to, std::min<size_t>(it.tx_to_len, cap));
    return it.tx_to_len;
}

const bcc_batch_item* bcc_workload_items(const bcc_workload* w, size_t* n) {
    if (n) *n = w ? w->n : 0;
    return w ? w->items.data() : nullptr;
}

// Mutated copies of a workload's items (agreement runs): item i is mutated with probability
// `rate` (splitmix of seed and i), kinds[i] = 0 (untouched) or 1 + the mutation: 1 flip one bit
// of the tx (any byte), 2 flip one bit in the back half of the tx (witness / signatures / the
// later inputs), 3 amount +-1, 4 flip one bit of the spent script, 5 drop the tx's last byte,
// 6 nIn = number of inputs.  A mutated item gets its own copy of the tx; the others keep sharing
// their tx buffer with their neighbours (the engine parses a shared buffer once).
struct bcc_itemset {
    std::vector<std::vector<uint8_t>> bufs;
    std::vector<bcc_batch_item> items;
};

bcc_itemset* bcc_workload_mutate(const bcc_workload* w, double rate, uint64_t seed,
                                 uint8_t* kinds) {
    if (!w) return nullptr;
    auto* m = new bcc_itemset();
    m->items = w->items;
    const uint64_t thr = (uint64_t)(rate * 18446744073709551615.0);
    for (size_t i = 0; i < w->n; i++) {
        uint64_t u = splitmix64(seed ^ (0x5851F42D4C957F2DULL * (i + 1)));
        kinds[i] = 0;
        if (u > thr) continue;
        bcc_batch_item& it = m->items[i];
        const uint64_t v = splitmix64(u);
        const int kind = 1 + (int)(v % 6);
        kinds[i] = (uint8_t)kind;
        std::vector<uint8_t> tx(it.tx_to, it.tx_to + it.tx_to_len);
        std::vector<uint8_t> spk(it.script_pubkey, it.script_pubkey + it.script_pubkey_len);
        const uint64_t r = v >> 8;
        switch (kind) {
            case 1: if (!tx.empty()) tx[r % tx.size()] ^= (uint8_t)(1u << ((r >> 32) % 8)); break;
            case 2: if (tx.size() > 1) tx[tx.size() / 2 + r % (tx.size() - tx.size() / 2)] ^= (uint8_t)(1u << ((r >> 32) % 8)); break;
            case 3: it.amount += (r & 1) ? 1 : -1; break;
            case 4: if (!spk.empty()) spk[r % spk.size()] ^= (uint8_t)(1u << ((r >> 32) % 8)); break;
            case 5: if (!tx.empty()) tx.pop_back(); break;
            case 6: {
                bcc::host::Tx t;
                if (bcc::host::parse_tx(it.tx_to, it.tx_to_len, t)) it.n_in = (unsigned)t.vin.size();
                break;
            }
        }
        m->bufs.push_back(std::move(tx));
        const std::vector<uint8_t>& tb = m->bufs.back();
        it.tx_to = tb.empty() ? nullptr : tb.data();
        it.tx_to_len = (unsigned)tb.size();
        m->bufs.push_back(std::move(spk));
        const std::vector<uint8_t>& sb = m->bufs.back();
        it.script_pubkey = sb.empty() ? nullptr : sb.data();
        it.script_pubkey_len = (unsigned)sb.size();
    }
    return m;
}

const bcc_batch_item* bcc_itemset_items(const bcc_itemset* m, size_t* n) {
    if (n) *n = m ? m->items.size() : 0;
    return m ? m->items.data() : nullptr;
}

void bcc_itemset_free(bcc_itemset* m) { delete m; }

int bcc_workload_tuple_items(const bcc_workload* w, uint32_t* out, size_t cap) {
    if (!w || !out) return -1;
    if (cap < w->tuple_item.size()) return BCC_BENCH_ERR_CAPACITY;
    if (!w->tuple_item.empty()) memcpy(out, w->tuple_item.data(), 4 * w->tuple_item.size());
    return 0;
}

int bcc_workload_msgs(bcc_workload* w, uint8_t* out, size_t cap) {
    if (!w || !w->batch || !out) return -1;
    if (cap / 32 < w->batch->n_tuples()) return BCC_BENCH_ERR_CAPACITY;
    return w->batch->fetch_msgs(out);
}

// Any caller items (copied): the engine's first interpreter round over them under `flags`,
// staged like the synthetic workloads, so tests can run the exact benchmarked path on mutated
// inputs.  Adjacent items with the same tx buffer share one copy (and its BIP143 aux hashes).
bcc_workload* bcc_workload_from_items(const bcc_batch_item* items, size_t n, unsigned flags,
                                      int device) {
    auto* w = new bcc_workload();
    w->device = device;
    w->n = n;
    w->flags = flags;
    w->spkoff.assign(1, 0);
    w->txoff.assign(1, 0);
    w->amount.resize(n);
    w->item_tx.resize(n);
    w->item_nin.resize(n);
    for (size_t i = 0; i < n; i++) {
        const bcc_batch_item& it = items[i];
        if (it.script_pubkey_len)
            w->spkblob.insert(w->spkblob.end(), it.script_pubkey, it.script_pubkey + it.script_pubkey_len);
        w->spkoff.push_back(w->spkblob.size());
        if (i == 0 || it.tx_to != items[i - 1].tx_to || it.tx_to_len != items[i - 1].tx_to_len) {
            if (it.tx_to_len) w->txblob.insert(w->txblob.end(), it.tx_to, it.tx_to + it.tx_to_len);
            w->txoff.push_back(w->txblob.size());
        }
        w->item_tx[i] = (uint32_t)(w->txoff.size() - 2);
        w->amount[i] = it.amount;
        w->item_nin[i] = it.n_in;
    }
    w->spkblob.push_back(0);  // keep data() valid for empty blobs
    w->txblob.push_back(0);
    if (finish(w)) return nullptr;
    return w;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// C3: block replay.  Transactions with the (inputs, outputs) counts given by the
// caller (the histogram of the reference's bench/data/block413567.raw, tests/golden/
// block413567_shape.json), re-signed with synthetic keys because the block's prevouts are not
// in the block.  Input type per input: 60 % P2PKH (legacy sighash), 30 % P2WPKH (BIP143),
// 10 % P2SH 2-of-3 CHECKMULTISIG (legacy, signer pair uniform over {1,2}, {1,3}, {2,3}, so
// 2-3 signature checks per input); outputs P2PKH : P2SH = 2841 : 737 as in the block.  All
// signatures SIGHASH_ALL, low-S, strict DER; a transaction with a P2WPKH input is serialized
// with witnesses (version 2), otherwise legacy (version 1).
// ------------------------------------------------------------------------------------------
namespace {

enum InType : uint8_t { IN_P2PKH = 0, IN_P2WPKH = 1, IN_MS = 2 };

struct PlanIn {
    uint8_t type;
    uint8_t pair;      // multisig signer pair: 0 {1,2}, 1 {1,3}, 2 {2,3}
    uint32_t key0;     // first key index (multisig: 3 consecutive keys)
    int64_t amount;
    uint8_t m[32];     // sighash
    uint32_t sig0;     // first signature index (multisig: 2)
};

}  // namespace

extern "C" bcc_workload* bcc_workload_block(const uint32_t* tx_nin, const uint32_t* tx_nout,
                                            size_t ntx, uint64_t seed, int device) {
    auto* w = new bcc_workload();
    w->device = device;
    // ---- plan: input types, key indices ----
    std::vector<std::vector<PlanIn>> plan(ntx);
    std::vector<size_t> tx_key0(ntx + 1, 0), tx_sig0(ntx + 1, 0), tx_item0(ntx + 1, 0);
    for (size_t j = 0; j < ntx; j++) {
        plan[j].resize(tx_nin[j]);
        size_t keys = 0, sigs = 0;
        for (uint32_t i = 0; i < tx_nin[j]; i++) {
            uint64_t r = splitmix64(seed ^ ((uint64_t)j << 20) ^ i ^ 0xC3C3C3C3ULL);
            PlanIn& p = plan[j][i];
            unsigned u = (unsigned)(r % 10);
            p.type = u < 6 ? IN_P2PKH : u < 9 ? IN_P2WPKH : IN_MS;
            p.pair = (uint8_t)((r >> 8) % 3);
            p.key0 = (uint32_t)(tx_key0[j] + keys);
            p.sig0 = (uint32_t)(tx_sig0[j] + sigs);
            p.amount = 546 + (int64_t)((r >> 16) % (uint64_t)(50000000000LL));
            keys += p.type == IN_MS ? 3 : 1;
            sigs += p.type == IN_MS ? 2 : 1;
        }
        tx_key0[j + 1] = tx_key0[j] + keys;
        tx_sig0[j + 1] = tx_sig0[j] + sigs;
        tx_item0[j + 1] = tx_item0[j] + tx_nin[j];
    }
    const size_t K = tx_key0[ntx], S = tx_sig0[ntx], n = tx_item0[ntx];
    w->n = n;
    // ---- keys (GPU) ----
    std::vector<uint8_t> d(32 * K), px(32 * K), py(32 * K), ok(std::max<size_t>(K, S));
    parallel_for(K, [&](size_t lo, size_t hi, unsigned) {
        uint8_t buf[9 + 16];
        memcpy(buf, "mi355x-c3", 9);
        for (size_t k = lo; k < hi; k++) {
            for (int b = 0; b < 8; b++) buf[9 + b] = (uint8_t)(seed >> (8 * b));
            for (int b = 0; b < 8; b++) buf[17 + b] = (uint8_t)((uint64_t)k >> (8 * b));
            derive_scalar(buf, sizeof buf, &d[32 * k]);
        }
    });
    if (mi_gen_pubkeys(d.data(), K, px.data(), py.data(), ok.data(), device) != 0) {
        delete w;
        return nullptr;
    }
    auto pub33 = [&](size_t k, uint8_t* o) {
        o[0] = 0x02 | (py[32 * k + 31] & 1);
        memcpy(o + 1, &px[32 * k], 32);
    };
    auto redeem = [&](const PlanIn& p, std::vector<uint8_t>& o) {  // OP_2 <k1> <k2> <k3> OP_3 OP_CMS
        o.clear();
        o.push_back(0x52);
        for (int q = 0; q < 3; q++) {
            uint8_t pk[33];
            pub33(p.key0 + q, pk);
            push_data(o, pk, 33);
        }
        o.push_back(0x53);
        o.push_back(0xae);
    };
    auto spk_of = [&](const PlanIn& p, std::vector<uint8_t>& o) {
        o.clear();
        uint8_t h[20];
        if (p.type == IN_MS) {
            std::vector<uint8_t> rs;
            redeem(p, rs);
            hash160(rs.data(), rs.size(), h);
            o.insert(o.end(), {0xa9, 0x14});
            o.insert(o.end(), h, h + 20);
            o.push_back(0x87);
            return;
        }
        uint8_t pk[33];
        pub33(p.key0, pk);
        hash160(pk, 33, h);
        if (p.type == IN_P2WPKH) {
            o.insert(o.end(), {0x00, 0x14});
            o.insert(o.end(), h, h + 20);
        } else {
            o.insert(o.end(), {0x76, 0xa9, 0x14});
            o.insert(o.end(), h, h + 20);
            o.insert(o.end(), {0x88, 0xac});
        }
    };
    // ---- unsigned transactions + sighashes (host, generation only) ----
    std::vector<std::vector<uint8_t>> outs(ntx);  // serialized vout section per tx
    std::vector<uint8_t> sm(32 * S), sk(32 * S), sd(32 * S);
    parallel_for(ntx, [&](size_t lo, size_t hi, unsigned) {
        std::vector<uint8_t> un, pre, code, aux;
        for (size_t j = lo; j < hi; j++) {
            std::vector<uint8_t>& vo = outs[j];
            vo.clear();
            put_compact_size(vo, tx_nout[j]);
            for (uint32_t o = 0; o < tx_nout[j]; o++) {
                uint64_t r = splitmix64(seed * 31 + ((uint64_t)j << 24) + o);
                put_le(vo, 1000 + r % 100000000ULL, 8);
                uint8_t h[20], t[12];
                for (int b = 0; b < 8; b++) t[b] = (uint8_t)(j >> (8 * b));
                for (int b = 0; b < 4; b++) t[8 + b] = (uint8_t)(o >> (8 * b));
                hash160(t, 12, h);
                if ((r >> 40) % 3578 < 2841) {  // block413567: 2841 P2PKH : 737 P2SH outputs
                    vo.push_back(25);
                    vo.insert(vo.end(), {0x76, 0xa9, 0x14});
                    vo.insert(vo.end(), h, h + 20);
                    vo.insert(vo.end(), {0x88, 0xac});
                } else {
                    vo.push_back(23);
                    vo.insert(vo.end(), {0xa9, 0x14});
                    vo.insert(vo.end(), h, h + 20);
                    vo.push_back(0x87);
                }
            }
            bool seg = false;
            for (const auto& p : plan[j]) seg |= p.type == IN_P2WPKH;
            un.clear();
            put_le(un, seg ? 2 : 1, 4);
            put_compact_size(un, tx_nin[j]);
            for (uint32_t i = 0; i < tx_nin[j]; i++) {
                uint8_t t[20], op[32];
                for (int b = 0; b < 8; b++) t[b] = (uint8_t)(j >> (8 * b));
                for (int b = 0; b < 4; b++) t[8 + b] = (uint8_t)(i >> (8 * b));
                for (int b = 0; b < 8; b++) t[12 + b] = (uint8_t)(seed >> (8 * b));
                sha256(t, 20, op);
                un.insert(un.end(), op, op + 32);
                put_le(un, i % 3, 4);
                un.push_back(0);  // scriptSig (other inputs' scriptSigs never enter a sighash)
                put_le(un, 0xffffffffu, 4);
            }
            un.insert(un.end(), vo.begin(), vo.end());
            put_le(un, 0, 4);
            Tx tx;
            if (!parse_tx(un.data(), un.size(), tx)) abort();
            for (uint32_t i = 0; i < tx_nin[j]; i++) {
                PlanIn& p = plan[j][i];
                if (p.type == IN_MS) {
                    redeem(p, code);
                } else {
                    uint8_t pk[33], h[20];
                    pub33(p.key0, pk);
                    hash160(pk, 33, h);
                    code.assign({0x76, 0xa9, 0x14});
                    code.insert(code.end(), h, h + 20);
                    code.insert(code.end(), {0x88, 0xac});
                }
                if (p.type == IN_P2WPKH) {  // BIP143 (interpreter.cpp:1581-1625)
                    Bip143Job job;
                    build_bip143_preimage(tx, i, Bytes(code.begin(), code.end()), 1, p.amount, job);
                    for (int k = 0; k < 3; k++) {
                        if (!job.need[k]) continue;
                        build_aux_message(tx, (AuxKind)k, aux);
                        sha256d(aux.data(), aux.size(), &job.preimage[job.off[k]]);
                    }
                    sha256d(job.preimage.data(), job.preimage.size(), p.m);
                } else {  // legacy (interpreter.cpp:1273-1364)
                    if (!build_legacy_preimage(tx, i, Bytes(code.begin(), code.end()), 1, pre)) abort();
                    sha256d(pre.data(), pre.size(), p.m);
                }
                const int nsig = p.type == IN_MS ? 2 : 1;
                for (int q = 0; q < nsig; q++) {
                    // signer keys: pair {1,2} {1,3} {2,3} -> key offsets
                    const int ko = p.type != IN_MS ? 0 : (q == 0 ? (p.pair == 2 ? 1 : 0)
                                                                  : (p.pair == 0 ? 1 : 2));
                    size_t sgi = p.sig0 + q;
                    memcpy(&sd[32 * sgi], &d[32 * (p.key0 + ko)], 32);
                    memcpy(&sm[32 * sgi], p.m, 32);
                    uint8_t nb[15 + 64];
                    memcpy(nb, "mi355x-c3-nonce", 15);
                    memcpy(nb + 15, &sd[32 * sgi], 32);
                    memcpy(nb + 47, p.m, 32);
                    derive_scalar(nb, sizeof nb, &sk[32 * sgi]);
                }
            }
        }
    });
    // ---- signatures (GPU) ----
    std::vector<uint8_t> r(32 * S), s(32 * S);
    if (mi_gen_sign(sd.data(), sm.data(), sk.data(), S, r.data(), s.data(), ok.data(), device) != 0) {
        delete w;
        return nullptr;
    }
    // ---- final transactions, spent scripts, amounts ----
    std::vector<std::vector<uint8_t>> txs(ntx), spks(n);
    w->amount.resize(n);
    w->item_tx.resize(n);
    w->item_nin.resize(n);
    parallel_for(ntx, [&](size_t lo, size_t hi, unsigned) {
        std::vector<uint8_t> sig, sig2, ss, rs;
        for (size_t j = lo; j < hi; j++) {
            bool seg = false;
            for (const auto& p : plan[j]) seg |= p.type == IN_P2WPKH;
            std::vector<uint8_t>& t = txs[j];
            put_le(t, seg ? 2 : 1, 4);
            if (seg) t.insert(t.end(), {0x00, 0x01});
            put_compact_size(t, tx_nin[j]);
            for (uint32_t i = 0; i < tx_nin[j]; i++) {
                const PlanIn& p = plan[j][i];
                uint8_t tb[20], op[32];
                for (int b = 0; b < 8; b++) tb[b] = (uint8_t)(j >> (8 * b));
                for (int b = 0; b < 4; b++) tb[8 + b] = (uint8_t)(i >> (8 * b));
                for (int b = 0; b < 8; b++) tb[12 + b] = (uint8_t)(seed >> (8 * b));
                sha256(tb, 20, op);
                t.insert(t.end(), op, op + 32);
                put_le(t, i % 3, 4);
                ss.clear();
                der_encode(&r[32 * p.sig0], &s[32 * p.sig0], 0x01, sig);
                if (p.type == IN_P2PKH) {
                    uint8_t pk[33];
                    pub33(p.key0, pk);
                    push_data(ss, sig.data(), sig.size());
                    push_data(ss, pk, 33);
                } else if (p.type == IN_MS) {
                    der_encode(&r[32 * (p.sig0 + 1)], &s[32 * (p.sig0 + 1)], 0x01, sig2);
                    redeem(p, rs);
                    ss.push_back(0x00);  // CHECKMULTISIG dummy (NULLDUMMY)
                    push_data(ss, sig.data(), sig.size());
                    push_data(ss, sig2.data(), sig2.size());
                    push_data(ss, rs.data(), rs.size());
                }
                put_compact_size(t, ss.size());
                t.insert(t.end(), ss.begin(), ss.end());
                put_le(t, 0xffffffffu, 4);
                size_t item = tx_item0[j] + i;
                spk_of(p, spks[item]);
                w->amount[item] = p.amount;
                w->item_tx[item] = (uint32_t)j;
                w->item_nin[item] = i;
            }
            t.insert(t.end(), outs[j].begin(), outs[j].end());
            if (seg) {
                for (uint32_t i = 0; i < tx_nin[j]; i++) {
                    const PlanIn& p = plan[j][i];
                    if (p.type != IN_P2WPKH) {
                        t.push_back(0);
                        continue;
                    }
                    uint8_t pk[33];
                    pub33(p.key0, pk);
                    der_encode(&r[32 * p.sig0], &s[32 * p.sig0], 0x01, sig);
                    t.push_back(2);
                    t.push_back((uint8_t)sig.size());
                    t.insert(t.end(), sig.begin(), sig.end());
                    t.push_back(33);
                    t.insert(t.end(), pk, pk + 33);
                }
            }
            put_le(t, 0, 4);
        }
    });
    w->txoff.resize(ntx + 1);
    size_t total = 0;
    for (size_t j = 0; j < ntx; j++) {
        w->txoff[j] = total;
        total += txs[j].size();
    }
    w->txoff[ntx] = total;
    w->txblob.resize(total);
    for (size_t j = 0; j < ntx; j++) memcpy(&w->txblob[w->txoff[j]], txs[j].data(), txs[j].size());
    w->spkoff.resize(n + 1);
    total = 0;
    for (size_t i = 0; i < n; i++) {
        w->spkoff[i] = total;
        total += spks[i].size();
    }
    w->spkoff[n] = total;
    w->spkblob.resize(total);
    for (size_t i = 0; i < n; i++) memcpy(&w->spkblob[w->spkoff[i]], spks[i].data(), spks[i].size());
    if (finish(w)) return nullptr;
    return w;
}

// The GPU sighash stage alone over n checks built by the engine's own job builder
// (host/engine.cpp add_sighash_job via build_sighash_checks): legacy SIGHASH_ALL template jobs
// (K3'), host-serialized legacy preimages (K3), the SIGHASH_SINGLE bug (row stays ONE), BIP143
// raw-tx jobs (K_wtx + K_win) and BIP143 SIGHASH_SINGLE preimages (K1 + K2 + K3).
int bcc_debug_sighash(const bcc_sighash_check* checks, size_t n, uint8_t* msg32_out, int device) {
    if (n == 0) return 0;
    if (!checks || !msg32_out) return -1;
    std::vector<bcc::host::SighashCheck> c(n);
    for (size_t i = 0; i < n; i++)
        c[i] = bcc::host::SighashCheck{checks[i].tx,       checks[i].tx_len,
                                       checks[i].script_code, checks[i].script_code_len,
                                       checks[i].n_in,     checks[i].hashtype,
                                       checks[i].amount,   checks[i].sigversion};
    bcc::SighashJobs jobs;
    bcc::TupleRows rows;
    if (bcc::host::build_sighash_checks(c.data(), n, jobs, rows) != n) return -1;
    bcc::DeviceBatch batch(device);
    int e = batch.stage(jobs, rows);
    if (!e) e = batch.run_sighash(nullptr);
    if (!e) e = batch.fetch_msgs(msg32_out);
    return e;
}
