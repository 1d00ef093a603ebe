// The engine's own verification on the host CPU: the device round of a batch (sighash jobs ->
// tuple rows -> verdicts, pipeline.h) computed by host code instead of the HIP kernels.  Used
// (a) when a device round fails twice (a GPU error must never become a consensus verdict, and the
// single-input ABI has no "no verdict" code, bitcoinconsensus.cpp:83-100), and (b) for rounds of
// at most bcc_set_host_small_round() tuples, whose GPU latency (one wave of a few hundred thousand
// dependent instructions) is far above a host verify.
//
// The verdict arithmetic is the kernels' own lane code compiled for the host: ecdsa_twist.h's
// square-root-free verify (twist_prep_lane, twist_accumulate_q/g, twist_combine, twist_final /
// twist_exceptional) over the same fixed-base comb tables; the sighash jobs are evaluated with the
// host SHA-256 (hashes.cpp) and the host preimage builders (sighash.cpp):
//   aux messages   SHA-256d of the padded message                     (K1)
//   preimages      aux digests patched in, SHA-256d                   (K2, K3)
//   template jobs  T[0, pos) || code || T[pos + 1, len) || le32(type) (K3')
//   BIP143 jobs    BIP143 preimage of the raw tx (interpreter.cpp:1581-1625), SHA-256d (K_wtx, K_win)
//   key hashes     HASH160 of the row's key against the program                        (K_h160)
// Nothing here is test infrastructure: tests/test_host_verify.py pins it against the reference's
// fixtures; the oracle is never linked.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../ecdsa_lane.h"
#include "../ecdsa_twist.h"
#include "../pipeline.h"
#include "bcc_amd.h"
#include "hashes.h"
#include "host_verify.h"
#include "sighash.h"
#include "team.h"
#include "tx.h"

namespace bcc {
namespace host {

namespace {

size_t unpadded_len(const uint8_t* m, size_t padded) {
    uint64_t bits = 0;
    for (int i = 0; i < 8; i++) bits = (bits << 8) | m[padded - 8 + i];
    return (size_t)(bits / 8);
}

const fe* comb_tables() {
    static std::vector<fe> t;
    static std::once_flag once;
    std::call_once(once, [] {
        t.resize((size_t)CWIN * CTAB * 2);
        build_g_comb(t.data());
    });
    return t.data();
}

void load_be(fe& r, const uint8_t* p) { fe_from_be_bytes(r, p); }
void load_be(sc& r, const uint8_t* p) {
    fe t;
    fe_from_be_bytes(t, p);
    memcpy(r.v, t.v, 32);
}

// Runs f(i) for i in [0, n) on up to T threads (contiguous shares).
template <class F>
void parallel_for(size_t n, unsigned T, F f) {
    T = (unsigned)std::max<size_t>(1, std::min<size_t>(T, n / 64 + 1));
    if (T <= 1) {
        for (size_t i = 0; i < n; i++) f(i);
        return;
    }
    run_team(T, [&](unsigned t) {
        for (size_t i = n * t / T; i < n * (t + 1) / T; i++) f(i);
    });
}

}  // namespace

void tpl_midstates(const uint8_t* T, uint32_t len, std::vector<uint32_t>& mid) {
    const uint32_t nm = tpl_mid_count(len);
    mid.resize(8 * (size_t)nm);
    Sha256 x;
    for (uint32_t j = 0; j < nm; j++) {
        memcpy(&mid[8 * (size_t)j], x.s, 32);
        if (j + 1 < nm) x.write(T + 64 * (size_t)j, 64);  // a whole block: compressed at once
    }
}

void tpl_job_sighash(const uint8_t* tpl, const uint8_t* code, const TplJob& t, uint8_t out[32]) {
    const uint8_t* T = tpl + t.tpl_off;
    Sha256 x;
    uint32_t q0 = 0;  // first message byte hashed here
    if (tpl_has_mid(t)) {
        const uint32_t b0 = t.pos / 64;
        memcpy(x.s, tpl + tpl_mid_offset(t.tpl_off, t.tpl_len) + 32 * (size_t)b0, 32);
        x.bytes = 64 * (uint64_t)b0;
        q0 = 64 * b0;
    }
    const uint32_t h = t.hashtype;
    const uint8_t ht[4] = {(uint8_t)h, (uint8_t)(h >> 8), (uint8_t)(h >> 16), (uint8_t)(h >> 24)};
    x.write(T + q0, t.pos - q0).write(code + t.code_off, t.code_len);
    x.write(T + t.pos + 1, t.tpl_len - t.pos - 1).write(ht, 4);
    uint8_t d[32];
    x.finalize(d);
    sha256(d, 32, out);
}

void host_sighash(const SighashJobs& j, uint8_t* msg) {
    std::vector<uint8_t> auxd(32 * j.aux_off.size());
    for (size_t a = 0; a < j.aux_off.size(); a++) {
        const uint8_t* m = &j.aux[(size_t)j.aux_off[a] * 64];
        sha256d(m, unpadded_len(m, (size_t)j.aux_nblk[a] * 64), &auxd[32 * a]);
    }
    if (!j.pre_off.empty()) {
        std::vector<uint8_t> pre(j.pre.begin(), j.pre.end());
        for (const auto& p : j.patches) memcpy(&pre[p.pre_byte], &auxd[32 * p.aux], 32);
        for (size_t k = 0; k < j.pre_off.size(); k++) {
            const uint8_t* m = &pre[(size_t)j.pre_off[k] * 64];
            sha256d(m, unpadded_len(m, (size_t)j.pre_nblk[k] * 64), msg + 32 * (size_t)j.pre_row[k]);
        }
    }
    for (const TplJob& t : j.tjobs) tpl_job_sighash(j.tpl.data(), j.code.data(), t, msg + 32 * (size_t)t.row);
    if (!j.wjobs.empty()) {
        // BIP143 from the raw tx bytes: parse each tx once, its three aux digests on first use
        std::vector<Tx> txs(j.wtx.size());
        std::vector<char> parsed(j.wtx.size(), 0);
        std::vector<uint8_t> digests(96 * j.wtx.size());
        Bip143Job job;
        std::vector<uint8_t> aux;
        for (const WinJob& w : j.wjobs) {
            const WtxRec& r = j.wtx[w.tx];
            if (!parsed[w.tx]) {
                if (!parse_tx(&j.txraw[r.tx_off], r.tx_len, txs[w.tx])) continue;  // row keeps ONE
                for (int k = 0; k < 3; k++) {
                    build_aux_message(txs[w.tx], (AuxKind)k, aux);
                    sha256d(aux.data(), aux.size(), &digests[96 * w.tx + 32 * k]);
                }
                parsed[w.tx] = 1;
            }
            const Tx& tx = txs[w.tx];
            if (w.nin >= tx.vin.size()) continue;
            const uint8_t* c = &j.code[w.code_off];
            const size_t hdr = c[0] < 253 ? 1 : c[0] == 253 ? 3 : 5;
            const Bytes code(c + hdr, c + w.code_len);
            const int64_t amount = (int64_t)((uint64_t)w.amount_hi << 32 | w.amount_lo);
            build_bip143_preimage(tx, w.nin, code, (int)w.hashtype, amount, job);
            for (int k = 0; k < 3; k++)
                if (job.need[k]) memcpy(&job.preimage[job.off[k]], &digests[96 * w.tx + 32 * k], 32);
            sha256d(job.preimage.data(), job.preimage.size(), msg + 32 * (size_t)w.row);
        }
    }
}

int host_verify_tuple(uint8_t tag, const uint8_t* x32, const uint8_t* y32, const uint8_t* r32,
                      const uint8_t* s32, const uint8_t* m32) {
    if (tag == 0) return 0;  // rejected by the host length filter
    fe px, py;
    sc r, s, m;
    load_be(px, x32);
    load_be(py, y32);
    load_be(r, r32);
    load_be(s, s32);
    load_be(m, m32);
    QTableArray qt;
    GCombArray gc{comb_tables()};
    return ecdsa_verify_twist_host(tag, px, py, r, s, m, qt, gc);  // wNAF Q half, safegcd inverses
}

void host_verify_rows(const TupleRows& rows, const uint8_t* msg, uint8_t* verdict, unsigned threads) {
    comb_tables();
    parallel_for(rows.size(), threads, [&](size_t i) {
        static const uint8_t zero[32] = {0};
        const uint8_t* y = rows.y.size() >= 32 * (i + 1) ? &rows.y[32 * i] : zero;
        verdict[i] = (uint8_t)host_verify_tuple(rows.tag[i], &rows.x[32 * i], y, &rows.r[32 * i],
                                                &rows.s[32 * i], msg + 32 * i);
    });
}

void apply_key_hashes(const TupleRows& R, uint8_t* verdict) {
    for (size_t k = 0; k < R.hrow.size(); k++) {
        const uint32_t row = R.hrow[k];
        uint8_t key[65], h[20];
        key[0] = R.tag[row];
        memcpy(key + 1, &R.x[32 * (size_t)row], 32);
        size_t n = 33;
        if (key[0] != 2 && key[0] != 3) {  // a 65-byte key (add_lazy stores its y; else zero)
            if (R.y.size() >= 32 * ((size_t)row + 1))
                memcpy(key + 33, &R.y[32 * (size_t)row], 32);
            else
                memset(key + 33, 0, 32);
            n = 65;
        }
        hash160(key, n, h);
        if (memcmp(h, &R.hprog[20 * k], 20) != 0) verdict[row] = 0;
    }
}

int host_verify_parts(const SighashJobs* const* jobs, const TupleRows* const* rows, size_t P,
                      uint8_t* verdict, unsigned threads) {
    size_t r0 = 0;
    std::vector<uint8_t> msg;
    for (size_t p = 0; p < P; p++) {
        const TupleRows& R = *rows[p];
        msg.resize(32 * R.size());
        if (R.msg_one) {  // the device initialises these rows: ONE
            for (size_t i = 0; i < R.size(); i++) {
                memset(&msg[32 * i], 0, 32);
                msg[32 * i] = 1;
            }
        } else {
            R.copy_msg(msg.data());  // rows past the stored prefix: ONE
        }
        host_sighash(*jobs[p], msg.data());
        host_verify_rows(R, msg.data(), verdict + r0, threads);
        apply_key_hashes(R, verdict + r0);
        r0 += R.size();
    }
    return 0;
}

namespace {
std::atomic<size_t> g_small_round{[] {
    const char* e = getenv("BCC_HOST_SMALL_ROUND");
    return e ? (size_t)atoll(e) : (size_t)BCC_HOST_SMALL_ROUND_DEFAULT;
}()};
std::atomic<int> g_failure_policy{[] {
    const char* e = getenv("BCC_DEVICE_FAILURE");
    return e && strcmp(e, "error") == 0 ? BCC_DEVICE_FAILURE_ERROR : BCC_DEVICE_FAILURE_HOST;
}()};
std::atomic<size_t> g_fallbacks{0};
}  // namespace

size_t host_small_round() { return g_small_round.load(std::memory_order_relaxed); }
bool host_fallback_enabled() {
    return g_failure_policy.load(std::memory_order_relaxed) == BCC_DEVICE_FAILURE_HOST;
}
void note_host_fallback() { g_fallbacks.fetch_add(1); }

}  // namespace host
}  // namespace bcc

extern "C" {

int bcc_set_host_small_round(size_t tuples) {
    bcc::host::g_small_round.store(tuples, std::memory_order_relaxed);
    return 0;
}

int bcc_set_device_failure_policy(int policy) {
    if (policy != BCC_DEVICE_FAILURE_HOST && policy != BCC_DEVICE_FAILURE_ERROR) return -1;
    bcc::host::g_failure_policy.store(policy, std::memory_order_relaxed);
    return 0;
}

size_t bcc_host_fallback_rounds(void) { return bcc::host::g_fallbacks.load(); }

int bcc_host_verify_tuples(const uint8_t* pub65, const uint8_t* msg32, const uint8_t* r32,
                           const uint8_t* s32, uint8_t* verdict, size_t n, unsigned threads) {
    if (n == 0) return 0;
    if (!pub65 || !msg32 || !r32 || !s32 || !verdict) return -1;
    bcc::host::parallel_for(n, threads ? threads : 1, [&](size_t i) {
        const uint8_t* p = pub65 + 65 * i;
        verdict[i] = (uint8_t)bcc::host::host_verify_tuple(p[0], p + 1, p + 33, r32 + 32 * i,
                                                           s32 + 32 * i, msg32 + 32 * i);
    });
    return 0;
}

}  // extern "C"
