// A persistent team of host worker threads per calling thread.
//
// Every host pass of a batch (deserialization, interpreter shards, stitching, staging fills) is a
// fork/join over T contiguous shares.  Creating T - 1 std::threads per pass costs ~15-30 us each
// in the forking thread (a C3 block call makes about five such passes), so the workers are kept:
// team(t) is the calling thread's own team, created on first use, grown on demand, parked on a
// condition variable between passes and joined when the calling thread exits.  Teams are never
// shared between callers, so concurrent verify_batch callers do not serialise on each other (the
// same rule as Core's CCheckQueue per-caller control, checkqueue.h:30-170).
#pragma once
#include <functional>

namespace bcc {
namespace host {

// Runs f(t) for t in [0, T): t = 0 on the calling thread, the rest on the calling thread's team.
// Returns when every f(t) has returned.  T <= 1 runs f(0) inline.
void run_team(unsigned T, const std::function<void(unsigned)>& f);

// Joins the calling thread's team (bcc_release_thread_state).
void release_team();

}  // namespace host
}  // namespace bcc
