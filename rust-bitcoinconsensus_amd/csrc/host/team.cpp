// Persistent per-caller worker teams (team.h).
#include "team.h"

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

class Team {
public:
    ~Team() { stop(); }

    void run(unsigned T, const std::function<void(unsigned)>& f) {
        grow(T - 1);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            T_ = T;
            pending_ = T - 1;
            gen_++;
        }
        cv_.notify_all();
        std::exception_ptr err;
        try {
            f(0);
        } catch (...) {
            err = std::current_exception();
        }
        // every worker must be done with f before it goes out of scope, even when f(0) threw
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
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
    void grow(unsigned workers) {
        while (th_.size() < workers) {
            const unsigned id = (unsigned)th_.size() + 1;
            uint64_t seen;
            {
                std::lock_guard<std::mutex> lk(mu_);
                seen = gen_;  // a new worker waits for the next pass, not the one in flight
            }
            th_.emplace_back([this, id, seen] { loop(id, seen); });
        }
    }

    void loop(unsigned id, uint64_t seen) {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
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
            if (--pending_ == 0) done_.notify_one();
        }
    }

    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    const std::function<void(unsigned)>* job_ = nullptr;
    std::exception_ptr worker_err_;
    unsigned T_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
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
