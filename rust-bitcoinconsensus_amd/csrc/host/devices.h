// Node sharding: the set of GPUs the library spreads a batch over, and one
// persistent host worker thread per GPU.
#pragma once
#include <functional>
#include <future>
#include <vector>

namespace bcc {
namespace host {

// The configured devices: bcc_set_devices(), else BCC_DEVICES="0,1,..", else the single device
// of bcc_set_device() / BCC_DEVICE (default 0).
std::vector<int> device_list();

// Runs jobs[d]() for every d concurrently, job d on the persistent worker thread of devs[d], so
// that each device keeps its thread-local device batch, stream and kernel scratch from call to
// call.  A single job runs inline on the calling thread (the single-device engine is per calling
// thread, reentrant).  Returns the first nonzero job result, else 0.
int run_on_devices(const std::vector<int>& devs, const std::vector<std::function<int()>>& jobs);

// Runs job() on the persistent pipeline worker thread (bitcoinconsensus_verify_batch overlaps a
// chunk's device rounds with the next chunk's host pass there; the worker's thread-local device
// batch is the pipeline's arena).
std::future<int> run_async(std::function<int()> job);

// Runs f() once on every persistent worker thread that exists (device workers and the pipeline
// worker) and waits: releases the state those threads keep for themselves.
void run_on_all_workers(const std::function<void()>& f);

// Marks a caller inside a batch entry point (verify_batch, the tuple and Taproot batches) for its
// lifetime.  bcc_release_thread_state releases the shared workers' state only while no caller is
// active: their device batches and scratch serve every caller's rounds.
struct ActiveCaller {
    ActiveCaller();
    ~ActiveCaller();
    ActiveCaller(const ActiveCaller&) = delete;
    ActiveCaller& operator=(const ActiveCaller&) = delete;
};
// Callers inside an entry point other than the calling thread's own (0 for a lone caller).
size_t other_active_callers();

// Contiguous split of `weights` (in order) into k groups of about equal total weight; returns the
// k + 1 group boundaries (indices into weights).
std::vector<size_t> split_balanced(const std::vector<size_t>& weights, size_t k);

// The CPUs this process may actually keep busy: the smaller of its affinity mask and its cgroup
// CPU bandwidth quota (cgroup v2 cpu.max, or v1 cfs_quota_us / cfs_period_us), rounded down, at
// least 1.  A quota is a per-period budget: a process that keeps more threads than the quota busy
// for a whole period exhausts it early and is throttled until the period ends.
unsigned cpu_share();

// Host worker threads of one batch pass (verify_batch's interpreter shards, the tuple and Taproot
// front ends, host-verified rounds): bcc_set_host_threads(), else BCC_HOST_THREADS, else the
// affinity CPUs, or 3 x cpu_share() under a smaller quota (capped at 64; devices.cpp says why).
unsigned host_threads();

}  // namespace host
}  // namespace bcc
