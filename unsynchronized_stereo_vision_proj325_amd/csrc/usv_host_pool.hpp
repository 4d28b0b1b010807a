// usv_host_pool.hpp -- persistent host worker threads for the C ABI's host-parallel loops (the host distance
// expansion, the sharded engine's per-GPU input copies).  Starting threads per call cost more than the work they
// did: a 1080p distance map took 0.50 ms with 16 threads started per call and 0.08 ms on persistent ones
// (scripts/probes/expand_probe.py, profiles/probes_r05/expand_probe_r05.txt).  Internal to libusv.so.
#pragma once
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace usv {

// run(n, fn) executes fn(0) .. fn(n - 1), part 0 on the calling thread and part i on worker i - 1, and returns when
// all are done.  Calls are serialised.  Workers start on first use, grow on demand and are joined by the destructor.
class HostPool {
  public:
    HostPool() = default;
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

    void run(int n, const std::function<void(int)>& fn) {
        std::lock_guard<std::mutex> call(call_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            while ((int)workers_.size() < n - 1) {
                const int id = (int)workers_.size();
                workers_.emplace_back([this, id] { loop(id); });
            }
            fn_ = &fn;
            parts_ = n;
            pending_ = n - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

  private:
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
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* fn_ = nullptr;
    int parts_ = 0, pending_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};

}  // namespace usv
