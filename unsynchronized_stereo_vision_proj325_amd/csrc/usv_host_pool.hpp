// usv_host_pool.hpp -- persistent host worker threads for the C ABI's host-parallel loops (the host distance
// expansion, the sharded engine's per-GPU input copies).  Starting threads per call cost more than the work they
// did: a 1080p distance map took 0.50 ms with 16 threads started per call and 0.08 ms on persistent ones
// (scripts/probes/expand_probe.py, profiles/probes_r05/expand_probe_r05.txt).  Internal to libusv.so.
#pragma once
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace usv {

// run(n, fn) executes fn(0) .. fn(n - 1) and returns when all are done.  The pool keeps at most
// max_threads() - 1 workers (the calling thread is the other one); with more parts than threads, thread i runs
// parts i, i + threads, ...  Workers start on first use, grow on demand up to that cap and are joined by the
// destructor.
//
// One call at a time uses the workers.  A call that finds them busy (another thread is inside run) does not
// wait: it runs its parts on threads of its own, started for that call, so two frame streams on two threads still
// expand at the same time.  After fork() the child has none of the parent's worker threads and may have inherited
// a locked mutex, so a pool used in a process other than the one that created it never touches its own state:
// it too runs on per-call threads (and its destructor leaves the parent's thread handles alone).
class HostPool {
  public:
    HostPool() : pid_(getpid()) {}
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    ~HostPool() {
        if (getpid() != pid_) {
            // forked copy: the threads behind these handles do not exist here; joining or destroying a joinable
            // std::thread would hang or terminate, so the handles are leaked
            new std::vector<std::thread>(std::move(workers_));
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

    static int max_threads() {
        static const int n = [] {
            const unsigned h = std::thread::hardware_concurrency();
            return h == 0 ? 16 : (int)std::min(h, 256u);
        }();
        return n;
    }

    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 0) return;
        const int nt = std::min(n, max_threads());
        // strided parts of one of nt threads
        const std::function<void(int)> part = [&](int i) {
            for (int p = i; p < n; p += nt) fn(p);
        };
        if (nt == 1) {
            part(0);
            return;
        }
        if (getpid() != pid_) {
            run_detached(nt, part);
            return;
        }
        std::unique_lock<std::mutex> call(call_mu_, std::try_to_lock);
        if (!call.owns_lock()) {
            run_detached(nt, part);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            while ((int)workers_.size() < nt - 1) {
                const int id = (int)workers_.size();
                workers_.emplace_back([this, id] { loop(id); });
            }
            fn_ = &part;
            parts_ = nt;
            pending_ = nt - 1;
            ++gen_;
        }
        cv_.notify_all();
        part(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

    pid_t owner() const { return pid_; }

  private:
    // threads started for this call only (the pool is busy, or this is a forked child)
    static void run_detached(int nt, const std::function<void(int)>& part) {
        std::vector<std::thread> ts;
        ts.reserve(nt - 1);
        for (int i = 1; i < nt; ++i) ts.emplace_back(part, i);
        part(0);
        for (auto& t : ts) t.join();
    }
    void loop(int id) {
        unsigned long long seen = 0;
        for (;;) {
            const std::function<void(int)>* fn;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (id + 1 >= parts_) continue;  // not needed by this call
                fn = fn_;
            }
            (*fn)(id + 1);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    const pid_t pid_;
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* fn_ = nullptr;
    int parts_ = 0, pending_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};

}  // namespace usv
