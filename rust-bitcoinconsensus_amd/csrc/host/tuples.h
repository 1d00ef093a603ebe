// Host front end of the tuple-level entry point (tuples.cpp): the CPubKey::Verify checks that
// need no secp256k1 arithmetic, turning (pub, msg32, DER sig) tuples into GPU tuple rows.
#pragma once
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

#include "../pipeline.h"
#include "team.h"

namespace bcc {
namespace host {

// Threaded pool helpers (up to host_threads() threads, at least `grain` items per thread).
unsigned pool_threads(size_t n, size_t grain);
// f(lo, hi) over contiguous chunks of [0, n) on pool_threads(n, grain) threads
template <class F>
void pfor(size_t n, size_t grain, F f) {
    const unsigned T = pool_threads(n, grain);
    if (T == 1) {
        f(0, n);
        return;
    }
    run_team(T, [&](unsigned t) { f(n * t / T, n * (t + 1) / T); });
}

// rows[i] for tuple i (rows resized to n): tag 0 (rejected on the host) unless the pubkey passes
// the CPubKey length filter, the signature parses laxly and r, s != 0.
void parse_rows(const uint8_t* pub_blob, const uint64_t* pub_off, const uint8_t* msg32,
                const uint8_t* sig_blob, const uint64_t* sig_off, size_t n, TupleRows& rows);

// Frees the calling thread's reused bcc_pubkey_verify_batch rows (bcc_release_thread_state).
void release_pubkey_rows();

}  // namespace host
}  // namespace bcc
