// Tuple level of the hot path, without a script around it: bcc_pubkey_verify_batch =
// N x CPubKey(pub).Verify(hash, sig) (pubkey.cpp:191-207).  The CPubKey length filter
// (pubkey.h:58-94), lax DER (pubkey.cpp:28-168) and the r / s == 0 rule are decided on the host,
// threaded; every surviving tuple goes to the GPU ECDSA kernels (normalisation is implicit: the
// verdict is invariant under s -> n - s).
#include "tuples.h"

#include <algorithm>
#include <cstring>
#include <thread>
#include <memory>
#include <vector>

#include "bcc_amd.h"
#include "devices.h"
#include "engine.h"
#include "host_verify.h"
#include "sighash.h"

namespace bcc {
namespace host {

unsigned pool_threads(size_t n, size_t grain) {
    return (unsigned)std::max<size_t>(1, std::min<size_t>(host_threads(), n / grain));
}

// One tuple's host half of CPubKey::Verify into row i of preallocated rows.  A tuple the host
// already rejects keeps tag 0 (the kernel's "rejected" header) and zero r / s.
static void parse_row(const uint8_t* pub, size_t publen, const uint8_t* m32, const uint8_t* sig,
                      size_t siglen, bcc::TupleRows& rows, size_t i) {
    uint8_t* tag = &rows.tag[i];
    uint8_t *x = &rows.x[32 * i], *y = &rows.y[32 * i], *r = &rows.r[32 * i], *s = &rows.s[32 * i];
    memcpy(&rows.msg[32 * i], m32, 32);
    *tag = 0;
    memset(x, 0, 32);
    memset(y, 0, 32);
    memset(r, 0, 32);
    memset(s, 0, 32);
    if (!pubkey_size_valid(pub, publen)) return;     // CPubKey::IsValid
    if (!der_parse_lax(sig, siglen, r, s)) return;   // ecdsa_signature_parse_der_lax
    bool rz = true, sz = true;
    for (int k = 0; k < 32; k++) {
        rz &= r[k] == 0;
        sz &= s[k] == 0;
    }
    if (rz || sz) return;                             // ecdsa_sig_verify: r, s != 0
    *tag = pub[0];
    memcpy(x, pub + 1, 32);
    if (publen == 65) memcpy(y, pub + 33, 32);
}

static void rows_resize(bcc::TupleRows& rows, size_t n) {
    rows.tag.resize(n);
    rows.x.resize(32 * n);
    rows.y.resize(32 * n);
    rows.r.resize(32 * n);
    rows.s.resize(32 * n);
    rows.msg.resize(32 * n);
}

void parse_rows(const uint8_t* pub_blob, const uint64_t* pub_off, const uint8_t* msg32,
                const uint8_t* sig_blob, const uint64_t* sig_off, size_t n, bcc::TupleRows& rows) {
    rows_resize(rows, n);  // every field of every row is written below (reused rows stay dirty)
    rows.msg_one = rows.y_unused = false;
    rows.hrow.clear();
    rows.hprog.clear();
    pfor(n, 4096, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; i++)
            parse_row(pub_blob + pub_off[i], pub_off[i + 1] - pub_off[i], msg32 + 32 * i,
                      sig_blob + sig_off[i], sig_off[i + 1] - sig_off[i], rows, i);
    });
}

// The rows of bcc_pubkey_verify_batch, kept with the thread that parsed them (the caller, or a
// per-GPU worker) for its next call: an 8M-tuple call otherwise zero-fills and faults in 1.3 GB of
// fresh vectors on one thread before the parallel parse, and unmaps them afterwards.
thread_local bcc::TupleRows tl_pubkey_rows;

// The pipelined form (tuple_rounds): two row sets and two staged device rounds per thread.
struct TupleSlot {
    bcc::TupleRows rows;
    std::unique_ptr<bcc::StagedRound, void (*)(bcc::StagedRound*)> staged{nullptr,
                                                                         bcc::gpu_staged_free};
    int dev = -1;
    size_t lo = 0, n = 0;  // the rows' range in the caller's arrays (n == 0: nothing in flight)
};
thread_local TupleSlot tl_tuple_slots[2];

void release_pubkey_rows() {
    tl_pubkey_rows = bcc::TupleRows();
    for (auto& s : tl_tuple_slots) s = TupleSlot();
}

// One device round of rows (the tuple-level entry point's): the host lane code for a small round,
// else the device with the engine's failure handling.
int tuple_round(int dev, const bcc::TupleRows& rows, uint8_t* verdict) {
    if (rows.size() <= host_small_round()) {  // latency: the host lane code
        host_verify_rows(rows, rows.msg.data(), verdict, host_threads());
        return 0;
    }
    const bcc::SighashJobs none;
    const bcc::SighashJobs* jp = &none;
    const bcc::TupleRows* rp = &rows;
    size_t retries = 0, host_rounds = 0;
    double st = 0;
    return resilient_round(dev, &jp, &rp, 1, verdict, &st, &retries, &host_rounds,
                           "pubkey_verify_batch");
}

// Rounds of about TUPLE_ROUND tuples, pipelined: round k's rows are parsed and staged on the
// calling thread's team while round k - 1 runs, and round k's upload (its own device batch and
// streams) runs beside round k - 1's kernels.  A staging or device error sends the round through
// tuple_round (retry on a fresh batch, then the failure policy).
constexpr size_t TUPLE_ROUND = (size_t)1 << 20;

int tuple_rounds(int dev, const uint8_t* pub_blob, const uint64_t* pub_off, const uint8_t* msg32,
                 const uint8_t* sig_blob, const uint64_t* sig_off, size_t n, uint8_t* verdict) {
    auto finish = [&](TupleSlot& s) -> int {
        if (s.n == 0) return 0;
        const size_t lo = s.lo;
        s.n = 0;
        if (bcc::gpu_staged_finish(s.staged.get(), verdict + lo) == 0) return 0;
        return tuple_round(dev, s.rows, verdict + lo);
    };
    int err = 0;
    size_t k = 0;
    for (size_t lo = 0; lo < n && !err; lo += TUPLE_ROUND, k++) {
        TupleSlot& s = tl_tuple_slots[k & 1];
        const size_t m = std::min(TUPLE_ROUND, n - lo);
        if (int e = finish(s)) err = e;  // (only after an error) this slot's last round
        parse_rows(pub_blob, pub_off + lo, msg32 + 32 * lo, sig_blob, sig_off + lo, m, s.rows);
        if (!s.staged || s.dev != dev) {
            s.staged.reset(bcc::gpu_staged_new(dev));
            s.dev = dev;
        }
        const bcc::SighashJobs none;
        const bcc::SighashJobs* jp = &none;
        const bcc::TupleRows* rp = &s.rows;
        double st = 0;
        s.lo = lo;
        s.n = m;
        if (injected_device_fault() != 0 ||
            bcc::gpu_staged_stage(s.staged.get(), &jp, &rp, 1, &st) != 0 ||
            bcc::gpu_staged_launch(s.staged.get(), nullptr) != 0) {
            s.n = 0;
            if (int e = tuple_round(dev, s.rows, verdict + lo)) err = e;
        }
        if (int e = finish(tl_tuple_slots[(k + 1) & 1])) err = err ? err : e;  // round k - 1
    }
    for (auto& s : tl_tuple_slots)
        if (int e = finish(s)) err = err ? err : e;
    return err;
}

}  // namespace host
}  // namespace bcc

extern "C" int bcc_pubkey_verify_batch(const uint8_t* pub_blob, const uint64_t* pub_off,
                                       const uint8_t* msg32, const uint8_t* sig_blob,
                                       const uint64_t* sig_off, uint8_t* verdict, size_t n,
                                       int device) {
    if (n == 0) return 0;
    if (!pub_off || !sig_off || !msg32 || !verdict) return -1;
    bcc::host::ActiveCaller active;
    std::vector<int> devs = device < 0 ? bcc::host::device_list() : std::vector<int>{device};
    const size_t D = std::min<size_t>(devs.size(), (n + 4095) / 4096);
    std::vector<std::function<int()>> jobs;
    for (size_t d = 0; d < D; d++) {
        const size_t lo = n * d / D, hi = n * (d + 1) / D;
        jobs.push_back([=] {  // contiguous equal range on devs[d] (offsets stay absolute)
            if (hi - lo >= 2 * bcc::host::TUPLE_ROUND)
                return bcc::host::tuple_rounds(devs[d], pub_blob, pub_off + lo, msg32 + 32 * lo,
                                               sig_blob, sig_off + lo, hi - lo, verdict + lo);
            bcc::TupleRows& rows = bcc::host::tl_pubkey_rows;
            bcc::host::parse_rows(pub_blob, pub_off + lo, msg32 + 32 * lo, sig_blob, sig_off + lo,
                                  hi - lo, rows);
            return bcc::host::tuple_round(devs[d], rows, verdict + lo);
        });
    }
    devs.resize(D);
    return bcc::host::run_on_devices(devs, jobs);
}
