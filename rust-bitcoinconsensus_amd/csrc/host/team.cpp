// Persistent per-caller worker teams (team.h).
#include "team.h"

#include "devices.h"

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <set>
#include <string>
#include <cstdlib>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace bcc {
namespace host {

namespace {

// Dispatch: the caller publishes the pass (job, worker count) under the mutex and bumps an
// atomic generation; workers that finished a pass within the last SPIN_US poll that generation
// (yielding the CPU between polls) instead of sleeping on the condition variable, so the next pass
// of the same call starts without a futex wake-up per worker (~70 us for a 48-thread team on the
// GPU box's 16-CPU quota: C3 runs about six passes per call).  The caller likewise polls for the
// pass's end before it sleeps.  Idle workers (between calls) sleep.
// Worker placement (BCC_TEAM_AFFINITY; round 6 diagnosis of the drop-in's run-to-run spread on the
// shared GPU box): "none" leaves the workers to the scheduler; "node" confines them to the NUMA
// node the team's creator runs on; "core" additionally gives worker i its own physical core of that
// node (the first logical CPU of each core, in the process's affinity mask).  The calling thread
// itself is never re-pinned.
enum class Affinity { NONE, NODE, CORE };

Affinity affinity_mode() {
    static const Affinity m = [] {
        const char* e = getenv("BCC_TEAM_AFFINITY");
        const std::string v = e ? e : "none";
        return v == "node" ? Affinity::NODE : v == "core" ? Affinity::CORE : Affinity::NONE;
    }();
    return m;
}

std::vector<int> parse_cpulist(const std::string& spec) {
    std::vector<int> out;
    size_t i = 0;
    while (i < spec.size()) {
        size_t j = spec.find(',', i);
        if (j == std::string::npos) j = spec.size();
        const std::string part = spec.substr(i, j - i);
        const size_t d = part.find('-');
        if (!part.empty()) {
            const int a = atoi(part.c_str());
            const int b = d == std::string::npos ? a : atoi(part.c_str() + d + 1);
            for (int c = a; c <= b; c++) out.push_back(c);
        }
        i = j + 1;
    }
    return out;
}

std::string read_line(const std::string& path) {
    std::ifstream f(path);
    std::string s;
    std::getline(f, s);
    return s;
}

// CPUs of the NUMA node of `cpu` that this process may run on; with one_per_core, only the first
// logical CPU of each physical core.  Empty when sysfs says nothing.
std::vector<int> node_cpus(int cpu, bool one_per_core) {
    cpu_set_t aff;
    CPU_ZERO(&aff);
    if (sched_getaffinity(0, sizeof aff, &aff) != 0) return {};
    for (int node = 0; node < 64; node++) {
        const std::vector<int> cpus =
            parse_cpulist(read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
        if (std::find(cpus.begin(), cpus.end(), cpu) == cpus.end()) continue;
        std::vector<int> out;
        for (int c : cpus) {
            if (c >= CPU_SETSIZE || !CPU_ISSET(c, &aff)) continue;
            if (one_per_core) {
                const std::vector<int> sib = parse_cpulist(read_line(
                    "/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/thread_siblings_list"));
                if (!sib.empty() && sib[0] != c) continue;
            }
            out.push_back(c);
        }
        return out;
    }
    return {};
}

class Team {
public:
    ~Team() { stop(); }

    void run(unsigned T, const std::function<void(unsigned)>& f) {
        grow(T - 1);
        bool wake;
        // polling only when the team fits the CPU share: beyond it a polling worker takes a CPU
        // (and CFS quota) from one that has work
        const bool spin = T <= cpu_share();
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            T_ = T;
            spin_ = spin;
            pending_.store(T - 1, std::memory_order_relaxed);
            gen_.store(gen_.load(std::memory_order_relaxed) + 1, std::memory_order_release);
            wake = sleepers_ > 0;
        }
        if (wake) cv_.notify_all();
        std::exception_ptr err;
        try {
            f(0);
        } catch (...) {
            err = std::current_exception();
        }
        // every worker must be done with f before it goes out of scope, even when f(0) threw
        if (spin) spin_until([this] { return pending_.load(std::memory_order_acquire) == 0; });
        std::unique_lock<std::mutex> lk(mu_);
        caller_waits_ = true;
        done_.wait(lk, [this] { return pending_.load(std::memory_order_acquire) == 0; });
        caller_waits_ = false;
        job_ = nullptr;
        if (!err) err = worker_err_;
        worker_err_ = nullptr;
        lk.unlock();
        if (err) std::rethrow_exception(err);
    }

    void stop() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
        th_.clear();
        stop_ = false;
    }

private:
    static constexpr int SPIN_US = 50;

    template <class P>
    static bool spin_until(P done) {
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned i = 0;; i++) {
            if (done()) return true;
            if ((i & 63) == 63 &&
                std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(SPIN_US))
                return false;
            std::this_thread::yield();
        }
    }

    void grow(unsigned workers) {
        if (th_.size() < workers && !placed_) {
            placed_ = true;
            const Affinity m = affinity_mode();
            if (m != Affinity::NONE) {
                const int cpu = sched_getcpu();
                if (cpu >= 0) cpus_ = node_cpus(cpu, m == Affinity::CORE);
                // the creator's own core goes last: the caller runs share 0 there
                if (m == Affinity::CORE && !cpus_.empty()) {
                    auto it = std::find(cpus_.begin(), cpus_.end(), cpu);
                    if (it != cpus_.end()) std::rotate(cpus_.begin(), it + 1, cpus_.end());
                }
            }
        }
        while (th_.size() < workers) {
            const unsigned id = (unsigned)th_.size() + 1;
            uint64_t seen;
            {
                std::lock_guard<std::mutex> lk(mu_);
                seen = gen_.load(std::memory_order_relaxed);  // a new worker waits for the next pass
            }
            th_.emplace_back([this, id, seen] { loop(id, seen); });
            if (!cpus_.empty()) {
                cpu_set_t set;
                CPU_ZERO(&set);
                if (affinity_mode() == Affinity::CORE) {
                    CPU_SET(cpus_[(id - 1) % cpus_.size()], &set);
                } else {
                    for (int c : cpus_) CPU_SET(c, &set);
                }
                (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof set, &set);
            }
        }
    }

    void loop(unsigned id, uint64_t seen) {
        for (;;) {
            if (spin_.load(std::memory_order_relaxed))
                spin_until([&] { return gen_.load(std::memory_order_acquire) != seen; });
            std::unique_lock<std::mutex> lk(mu_);
            if (gen_.load(std::memory_order_relaxed) == seen && !stop_) {
                sleepers_++;
                cv_.wait(lk, [&] { return stop_ || gen_.load(std::memory_order_relaxed) != seen; });
                sleepers_--;
            }
            if (stop_) return;
            seen = gen_.load(std::memory_order_relaxed);
            if (id >= T_) continue;  // this pass needs fewer workers
            const std::function<void(unsigned)>* f = job_;
            lk.unlock();
            std::exception_ptr err;
            try {
                (*f)(id);
            } catch (...) {
                err = std::current_exception();
            }
            lk.lock();
            if (err && !worker_err_) worker_err_ = err;  // rethrown by run() on the caller
            if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1 && caller_waits_)
                done_.notify_one();
        }
    }

    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    const std::function<void(unsigned)>* job_ = nullptr;
    std::exception_ptr worker_err_;
    unsigned T_ = 0, sleepers_ = 0;
    std::atomic<unsigned> pending_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> spin_{false};  // the last pass's team fit the CPU share
    bool stop_ = false, caller_waits_ = false;
    bool placed_ = false;   // the workers' CPUs are chosen (BCC_TEAM_AFFINITY)
    std::vector<int> cpus_;  // ... and these are they (empty: no affinity)
};

thread_local std::unique_ptr<Team> tl_team;
thread_local bool tl_in_team_run = false;  // a nested pass from f(0) gets plain threads

}  // namespace

void run_team(unsigned T, const std::function<void(unsigned)>& f) {
    if (T <= 1) {
        f(0);
        return;
    }
    if (tl_in_team_run) {
        std::vector<std::exception_ptr> errs(T);
        auto guarded = [&](unsigned t) {
            try {
                f(t);
            } catch (...) {
                errs[t] = std::current_exception();
            }
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < T; t++) th.emplace_back(guarded, t);
        guarded(0);
        for (auto& x : th) x.join();
        for (auto& e : errs)
            if (e) std::rethrow_exception(e);
        return;
    }
    if (!tl_team) tl_team.reset(new Team());
    struct InRun {  // cleared however run() leaves
        InRun() { tl_in_team_run = true; }
        ~InRun() { tl_in_team_run = false; }
    } in_run;
    tl_team->run(T, f);
}

void release_team() { tl_team.reset(); }

}  // namespace host
}  // namespace bcc
