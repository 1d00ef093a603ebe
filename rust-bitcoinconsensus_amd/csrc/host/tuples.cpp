// Tuple level of the hot path, without a script around it: bcc_pubkey_verify_batch =
// N x CPubKey(pub).Verify(hash, sig) (pubkey.cpp:191-207).  The CPubKey length filter
// (pubkey.h:58-94), lax DER (pubkey.cpp:28-168) and the r / s == 0 rule are decided on the device
// (round 5: K_der, der.hip, over the caller's blobs copied as they are); the host restatement here
// (parse_rows) serves small rounds on the host lane code and the device-failure path.  Every
// surviving tuple goes to the GPU ECDSA kernels (normalisation is implicit: the verdict is
// invariant under s -> n - s).
#include "tuples.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
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
    // a tuple's offsets must lie in order inside the round's [off[0], off[n]] (as K_der checks);
    // otherwise it is invalid (its bytes are never read)
    const uint64_t p0 = pub_off[0], p1 = pub_off[n], s0 = sig_off[0], s1 = sig_off[n];
    pfor(n, 4096, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; i++) {
            const uint64_t pa = pub_off[i], pb = pub_off[i + 1], sa = sig_off[i], sb = sig_off[i + 1];
            const bool ok = p0 <= pa && pa <= pb && pb <= p1 && s0 <= sa && sa <= sb && sb <= s1;
            parse_row(pub_blob + (ok ? pa : p0), ok ? pb - pa : 0, msg32 + 32 * i,
                      sig_blob + (ok ? sa : s0), ok ? sb - sa : 0, rows, i);
        }
    });
}

// The rows of bcc_pubkey_verify_batch, kept with the thread that parsed them (the caller, or a
// per-GPU worker) for its next call: an 8M-tuple call otherwise zero-fills and faults in 1.3 GB of
// fresh vectors on one thread before the parallel parse, and unmaps them afterwards.
thread_local bcc::TupleRows tl_pubkey_rows;

// The pipelined form (tuple_rounds): two staged device rounds per thread (and the host rows a
// failed round is re-run from).
struct TupleSlot {
    bcc::TupleRows rows;
    std::unique_ptr<bcc::StagedRound, void (*)(bcc::StagedRound*)> staged{nullptr,
                                                                         bcc::gpu_staged_free};
    int dev = -1;
    size_t lo = 0, n = 0;  // the rows' range in the caller's arrays (n == 0: nothing in flight)
};

// A round's raw tuples go to the device as they are (K_der) unless their blobs are unusually large
// (more than DER_BLOB_LIMIT bytes for the round: the pinned image would grow with them); such a round
// is parsed on the host (parse_rows) and its fixed-size rows staged instead.
constexpr uint64_t DER_BLOB_LIMIT = (uint64_t)1 << 31;
bool der_on_device(const bcc::DerTuples& t) { return t.pub_bytes() + t.sig_bytes() <= DER_BLOB_LIMIT; }
// three: rounds k - 1 and k on the device while round k + 1 is staged (round 5; two slots made the
// staging of round k + 1 wait for round k - 1, which shares the GPU with round k: 8 ms idle gaps)
constexpr unsigned TUPLE_SLOTS_MAX = 3;
thread_local TupleSlot tl_tuple_slots[TUPLE_SLOTS_MAX];

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

// Pipelined rounds (sizes below): round k's raw tuples are copied into its pinned image by the
// calling thread's team while round k - 1 runs, and round k's upload (its own device batch and
// streams) runs beside round k - 1's kernels.  A staging or device error sends the round through
// the host parse and tuple_round (retry on a fresh batch, then the failure policy).  Measured on
// 8M C4 tuples (profiles/r05/c4_der): 256k-first doubling to 2M rounds 100-101 M/s, fixed 1M
// rounds 90 M/s, a 4M cap 95 M/s; the host side is ~13 ms of copying in ~80 ms.  With two slots
// round k + 1 was staged only after round k - 1 finished, and k - 1 shares the GPU with round k
// (timeline_2slots.txt: 8 ms idle before the last round); three slots: 126.4-126.8 M/s against
// 103.8-104.9 with two (slots.txt), the staged kernels alone 131.
constexpr size_t TUPLE_ROUND = (size_t)1 << 20;
static size_t env_size(const char* name, size_t dflt) {
    const char* e = getenv(name);
    return e && atoll(e) > 0 ? (size_t)atoll(e) : dflt;
}
// Round sizes: the first round (the only one whose staging and upload the GPU waits for) is small,
// and each next one doubles up to the cap while the previous round's kernels hide its staging and
// upload (~1 + 2.8 ms per 1M tuples against ~8 ms of kernels); a remainder under half the cap joins
// the last round (fewer kernel tails).
static const size_t g_tuple_first = env_size("BCC_TUPLE_FIRST", TUPLE_ROUND / 4);
static const size_t g_tuple_round = env_size("BCC_TUPLE_ROUND", 2 * TUPLE_ROUND);
static const bool g_tuple_ramp = env_size("BCC_TUPLE_RAMP", 1) != 0;
static const bool g_tuple_trace = getenv("BCC_TUPLE_TRACE") != nullptr;
static const unsigned g_tuple_slots = (unsigned)std::min<size_t>(3, std::max<size_t>(2, env_size("BCC_TUPLE_SLOTS", 3)));

// Raw tuples [lo, lo + m) of the caller's arrays.
static bcc::DerTuples der_range(const uint8_t* pub_blob, const uint64_t* pub_off, const uint8_t* msg32,
                                const uint8_t* sig_blob, const uint64_t* sig_off, size_t lo, size_t m) {
    bcc::DerTuples t;
    t.pub_blob = pub_blob;
    t.pub_off = pub_off + lo;
    t.msg32 = msg32 + 32 * lo;
    t.sig_blob = sig_blob;
    t.sig_off = sig_off + lo;
    t.n = m;
    return t;
}

// One round of raw tuples: K_der + the kernels on the device; a host-lane round, an oversized
// blob or a device error (retried on a fresh batch, then the failure policy: tuple_round) goes
// through the host rows.
int der_round(int dev, const bcc::DerTuples& t, bcc::TupleRows& rows, uint8_t* verdict) {
    if (t.n > host_small_round() && der_on_device(t) && injected_device_fault() == 0 &&
        bcc::gpu_verify_der(dev, t, verdict) == 0)
        return 0;
    parse_rows(t.pub_blob, t.pub_off, t.msg32, t.sig_blob, t.sig_off, t.n, rows);
    return tuple_round(dev, rows, verdict);
}

int tuple_rounds(int dev, const uint8_t* pub_blob, const uint64_t* pub_off, const uint8_t* msg32,
                 const uint8_t* sig_blob, const uint64_t* sig_off, size_t n, uint8_t* verdict) {
    auto host_rows = [&](TupleSlot& s) -> bcc::TupleRows& {  // a failed round's rows, on the host
        const bcc::DerTuples t = der_range(pub_blob, pub_off, msg32, sig_blob, sig_off, s.lo, s.n);
        parse_rows(t.pub_blob, t.pub_off, t.msg32, t.sig_blob, t.sig_off, t.n, s.rows);
        return s.rows;
    };
    auto finish = [&](TupleSlot& s) -> int {
        if (s.n == 0) return 0;
        const size_t lo = s.lo;
        if (bcc::gpu_staged_finish(s.staged.get(), verdict + lo) == 0) {
            s.n = 0;
            return 0;
        }
        bcc::TupleRows& rows = host_rows(s);
        s.n = 0;
        return tuple_round(dev, rows, verdict + lo);
    };
    int err = 0;
    size_t k = 0;
    using clk = std::chrono::steady_clock;
    auto sec = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
    const auto c0 = clk::now();
    double t_stage = 0, t_wait = 0;
    size_t m = 0;
    for (size_t lo = 0; lo < n && !err; lo += m, k++) {
        TupleSlot& s = tl_tuple_slots[k % g_tuple_slots];
        m = k == 0 ? g_tuple_first : g_tuple_ramp ? std::min(2 * m, g_tuple_round) : g_tuple_round;
        if (m >= n - lo || n - lo - m < m / 2) m = n - lo;
        auto w0 = clk::now();
        if (int e = finish(s)) err = e;  // (only after an error) this slot's last round
        t_wait += sec(w0);
        w0 = clk::now();
        if (!s.staged || s.dev != dev) {
            s.staged.reset(bcc::gpu_staged_new(dev));
            s.dev = dev;
        }
        const bcc::DerTuples t = der_range(pub_blob, pub_off, msg32, sig_blob, sig_off, lo, m);
        double st = 0;
        s.lo = lo;
        s.n = m;
        bool staged;
        if (der_on_device(t)) {
            staged = injected_device_fault() == 0 &&
                     bcc::gpu_staged_stage_der(s.staged.get(), t, &st) == 0 &&
                     bcc::gpu_staged_launch(s.staged.get(), nullptr) == 0;
        } else {  // oversized blobs: host rows, staged
            parse_rows(t.pub_blob, t.pub_off, t.msg32, t.sig_blob, t.sig_off, m, s.rows);
            const bcc::SighashJobs none;
            const bcc::SighashJobs* jp = &none;
            const bcc::TupleRows* rp = &s.rows;
            staged = injected_device_fault() == 0 &&
                     bcc::gpu_staged_stage(s.staged.get(), &jp, &rp, 1, &st) == 0 &&
                     bcc::gpu_staged_launch(s.staged.get(), nullptr) == 0;
        }
        if (!staged) {
            static std::atomic<int> warned{0};
            if (warned.fetch_add(1) < 3)
                fprintf(stderr, "[bcc] pubkey_verify_batch: round of %zu tuples not staged on device %d; "
                                "running it through the host parse and the general path\n", m, dev);
            bcc::TupleRows& rows = host_rows(s);
            s.n = 0;
            if (int e = tuple_round(dev, rows, verdict + lo)) err = e;
        }
        t_stage += sec(w0);
        if (g_tuple_trace)
            fprintf(stderr, "[bcc] tup k=%zu m=%zu launched %lld\n", k, m,
                    (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now().time_since_epoch()).count());
        w0 = clk::now();
        // the round that next reuses a slot: k + 1 - slots (with 3 slots round k - 2)
        if (int e = finish(tl_tuple_slots[(k + 1) % g_tuple_slots])) err = err ? err : e;
        t_wait += sec(w0);
        if (g_tuple_trace)
            fprintf(stderr, "[bcc] tup k=%zu finished_prev %lld\n", k,
                    (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now().time_since_epoch()).count());
    }
    const auto w0 = clk::now();
    for (auto& s : tl_tuple_slots)
        if (int e = finish(s)) err = err ? err : e;
    t_wait += sec(w0);
    if (g_tuple_trace)
        fprintf(stderr, "[bcc] tuple_rounds: %zu tuples, %zu rounds, %.2f ms: stage+launch %.2f ms, "
                        "waits %.2f ms\n", n, k, 1e3 * sec(c0), 1e3 * t_stage, 1e3 * t_wait);
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
    if (pub_off[n] < pub_off[0] || sig_off[n] < sig_off[0]) return -1;  // offsets run backwards
    // Offsets must be non-decreasing over the whole call: every round checks a tuple against its
    // own round's [off[lo], off[lo + m]] span (the bytes it uploads), so with offsets out of order
    // a tuple's verdict would depend on how the call is cut into rounds and devices.  One O(n) pass
    // on the team (~1 ms for 8M tuples) rejects such a call instead.
    {
        std::atomic<bool> bad{false};
        bcc::host::pfor(n, 1 << 16, [&](size_t lo, size_t hi) {
            bool b = false;
            for (size_t i = lo; i < hi; i++)
                b |= (pub_off[i + 1] < pub_off[i]) | (sig_off[i + 1] < sig_off[i]);
            if (b) bad.store(true, std::memory_order_relaxed);
        });
        if (bad.load()) return -1;
    }
    bcc::host::ActiveCaller active;
    std::vector<int> devs = device < 0 ? bcc::host::device_list() : std::vector<int>{device};
    const size_t D = std::min<size_t>(devs.size(), (n + 4095) / 4096);
    std::vector<std::function<int()>> jobs;
    for (size_t d = 0; d < D; d++) {
        const size_t lo = n * d / D, hi = n * (d + 1) / D;
        jobs.push_back([=] {  // contiguous equal range on devs[d] (offsets stay absolute)
            // (a range the host small round covers goes to the host lane code in one round: the
            // pipelined rounds are device rounds)
            if (hi - lo >= 2 * bcc::host::g_tuple_first && hi - lo > bcc::host::host_small_round())
                return bcc::host::tuple_rounds(devs[d], pub_blob, pub_off + lo, msg32 + 32 * lo,
                                               sig_blob, sig_off + lo, hi - lo, verdict + lo);
            return bcc::host::der_round(devs[d],
                                        bcc::host::der_range(pub_blob, pub_off, msg32, sig_blob,
                                                             sig_off, lo, hi - lo),
                                        bcc::host::tl_pubkey_rows, verdict + lo);
        });
    }
    devs.resize(D);
    return bcc::host::run_on_devices(devs, jobs);
}
