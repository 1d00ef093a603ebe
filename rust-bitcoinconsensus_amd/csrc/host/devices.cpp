// Node sharding: per-GPU persistent worker threads.
//
// The reference has no multi-GPU code; its batching precedent is Core's CCheckQueue
// (depend/bitcoin/src/checkqueue.h:30-170), a pool of host workers draining one queue of script
// checks.  Here every configured GPU gets one worker thread that owns that device's HIP stream,
// device arena, pinned staging buffer and kernel scratch (the thread-local DeviceBatch /
// ThreadCtx caches); a batch's device round is cut into contiguous, equally weighted groups of
// whole transactions, one per GPU, which run concurrently, and the verdicts land in the caller's
// array at each group's row offset (the host-side gather).  No collective sits on this path.
#include "devices.h"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "bcc_amd.h"

namespace bcc {
namespace host {

int current_device();  // engine.cpp: bcc_set_device / BCC_DEVICE

namespace {

std::mutex g_devs_mu;
std::vector<int> g_devs;  // explicit list (bcc_set_devices); empty: environment / single device
bool g_devs_env_read = false;

class Worker {
public:
    Worker() : th_([this] { loop(); }) {}
    ~Worker() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    std::future<int> submit(std::function<int()> f) {
        auto task = std::make_shared<std::packaged_task<int()>>(std::move(f));
        std::future<int> fut = task->get_future();
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back([task] { (*task)(); });
        }
        cv_.notify_one();
        return fut;
    }

private:
    void loop() {
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                job = std::move(q_.front());
                q_.pop_front();
            }
            job();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
    std::thread th_;
};

std::mutex g_workers_mu;
std::map<int, std::unique_ptr<Worker>>& workers() {
    static auto* w = new std::map<int, std::unique_ptr<Worker>>();  // lives for the process
    return *w;
}

Worker& worker(int dev) {
    std::lock_guard<std::mutex> lk(g_workers_mu);
    auto& w = workers()[dev];
    if (!w) w.reset(new Worker());
    return *w;
}

}  // namespace

std::vector<int> device_list() {
    std::lock_guard<std::mutex> lk(g_devs_mu);
    if (g_devs.empty() && !g_devs_env_read) {
        g_devs_env_read = true;
        if (const char* e = getenv("BCC_DEVICES")) {
            std::string s(e);
            size_t p = 0;
            while (p < s.size()) {
                size_t q = s.find(',', p);
                if (q == std::string::npos) q = s.size();
                if (q > p) g_devs.push_back(atoi(s.substr(p, q - p).c_str()));
                p = q + 1;
            }
        }
    }
    if (!g_devs.empty()) return g_devs;
    return {current_device()};
}

int run_on_devices(const std::vector<int>& devs, const std::vector<std::function<int()>>& jobs) {
    if (jobs.size() == 1) return jobs[0]();
    std::vector<std::future<int>> f;
    f.reserve(jobs.size());
    for (size_t d = 0; d < jobs.size(); d++) f.push_back(worker(devs[d]).submit(jobs[d]));
    int rc = 0;
    for (auto& x : f) {
        int r = x.get();
        if (r && !rc) rc = r;
    }
    return rc;
}

void run_on_all_workers(const std::function<void()>& f) {
    std::vector<Worker*> ws;
    {
        std::lock_guard<std::mutex> lk(g_workers_mu);
        for (auto& kv : workers())
            if (kv.second) ws.push_back(kv.second.get());
    }
    std::vector<std::future<int>> fut;
    for (Worker* w : ws) fut.push_back(w->submit([f] {
        f();
        return 0;
    }));
    for (auto& x : fut) x.get();
}

namespace {
std::atomic<size_t> g_active_callers{0};
thread_local size_t tl_active_depth = 0;
}  // namespace

ActiveCaller::ActiveCaller() {
    if (tl_active_depth++ == 0) g_active_callers.fetch_add(1);
}
ActiveCaller::~ActiveCaller() {
    if (--tl_active_depth == 0) g_active_callers.fetch_sub(1);
}
size_t other_active_callers() {
    return g_active_callers.load() - (tl_active_depth ? 1 : 0);
}

std::future<int> run_async(std::function<int()> job) {
    return worker(-1).submit(std::move(job));  // key -1: the pipeline worker (no device of its own)
}

namespace {

// cgroup v2 "max 100000" / "1600000 100000", or v1 quota / period files; 0 = no quota
double cgroup_quota_cpus() {
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long period = 0;
        const int k = fscanf(f, "%31s %lld", q, &period);
        fclose(f);
        if (k == 2 && strcmp(q, "max") != 0 && period > 0) return (double)atoll(q) / (double)period;
        if (k >= 1) return 0;
    }
    long long quota = -1, period = 0;
    if (FILE* f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
        if (fscanf(f, "%lld", &quota) != 1) quota = -1;
        fclose(f);
    }
    if (FILE* f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
        if (fscanf(f, "%lld", &period) != 1) period = 0;
        fclose(f);
    }
    return quota > 0 && period > 0 ? (double)quota / (double)period : 0;
}

std::atomic<unsigned> g_host_threads{0};  // bcc_set_host_threads (0: default)

}  // namespace

namespace {
unsigned affinity_cpus() {
    static const unsigned n = [] {
        unsigned c = std::max(1u, std::thread::hardware_concurrency());
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) c = std::max(1, CPU_COUNT(&set));
        return c;
    }();
    return n;
}
}  // namespace

unsigned cpu_share() {
    static const unsigned share = [] {
        unsigned n = affinity_cpus();
        const double q = cgroup_quota_cpus();
        if (q > 0) n = std::min<unsigned>(n, std::max(1u, (unsigned)q));
        return n;
    }();
    return share;
}

// Default: the CPUs the process may run on, capped at the CFS quota (cpu.max) when there is one.
// Rounds 3-4 used three times the quota: 16 threads then kept only 8 CPUs busy, which round 5
// traced to false sharing in the parse pass (per-shard vector headers on shared cache lines, each
// push_back taking the line from the other workers: 10x the single-threaded cost per item), not to
// the quota.  With that fixed, 20 back-to-back 1M-input C2 calls on the GPU box (quota 16,
// profiles/r05/dropin): 16 threads 36.5-37.5 M inputs/s at 0.245 CPU-s per 1M inputs, 24 threads
// 36.8-39.0 at 0.27-0.32, 48 threads 31.6-38.0 at 0.40-0.51.
unsigned host_threads() {
    if (unsigned v = g_host_threads.load(std::memory_order_relaxed)) return v;
    static const unsigned dflt = [] {
        if (const char* e = getenv("BCC_HOST_THREADS"))
            if (atoi(e) > 0) return (unsigned)atoi(e);
        const unsigned aff = affinity_cpus(), share = cpu_share();
        const unsigned n = std::min(aff, share);
        return std::min(64u, n);
    }();
    return dflt;
}

std::vector<size_t> split_balanced(const std::vector<size_t>& w, size_t k) {
    size_t total = 0;
    for (size_t x : w) total += x;
    std::vector<size_t> b(k + 1, w.size());
    b[0] = 0;
    size_t acc = 0, i = 0;
    for (size_t g = 1; g < k; g++) {
        const size_t want = total * g / k;
        while (i < w.size() && acc + w[i] / 2 < want) acc += w[i++];
        b[g] = i;
    }
    return b;
}

}  // namespace host
}  // namespace bcc

using namespace bcc::host;

extern "C" {

int bcc_set_devices(const int* devices, int n) {
    // validate everything first: a rejected call leaves the configured list unchanged
    if (n < 0 || (n > 0 && !devices)) return -1;
    std::vector<int> next;
    for (int i = 0; i < n; i++) {
        if (devices[i] < 0) return -1;
        next.push_back(devices[i]);
    }
    std::lock_guard<std::mutex> lk(g_devs_mu);
    g_devs.swap(next);
    g_devs_env_read = true;  // an explicit call overrides BCC_DEVICES
    return 0;
}

int bcc_set_host_threads(unsigned n) {
    if (n > 1024) return -1;
    g_host_threads.store(n, std::memory_order_relaxed);
    return 0;
}

unsigned bcc_get_host_threads(void) { return host_threads(); }

unsigned bcc_cpu_share(void) { return cpu_share(); }

int bcc_get_devices(int* out, int cap) {
    const std::vector<int> d = device_list();
    for (int i = 0; i < (int)d.size() && i < cap; i++) out[i] = d[i];
    return (int)d.size();
}

}  // extern "C"
