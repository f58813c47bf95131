// host_pool.h — the persistent host thread pool behind the engines' parallel
// host sections (spade_engine batch bookkeeping, K0 token staging).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>

namespace fsm {

// A persistent pool of host threads for the per-batch bookkeeping (deep lattices
// run dozens of parallel sections per mine: creating threads for each cost more
// than the work).  One section at a time; a caller that finds the pool busy (a
// concurrent mine on another context) runs its section inline.  Never destroyed:
// the workers are detached and idle between sections.  A task that throws
// (bad_alloc in a fill, FSM_ELIMIT) never unwinds past a running section: the
// first exception is kept, the section drains (no worker is left inside the
// caller's frame), then it is rethrown on the caller's thread.
// Wake-up: a finished worker spins on the section generation for a while
// (kSpinNs) before it sleeps on the condition variable, and the caller waits for
// the section's end by spinning too: a mine's sections come in bursts, and a
// futex wake of 15 workers per section cost more than the short sections' work
// (D1M measured 0.3-0.5 ms per mine for a handful of them).
class HostPool {
  public:
    static HostPool& get() {
        static HostPool* p = new HostPool();
        return *p;
    }
    // fn(t) for t in [0, n): task 0 and any unclaimed ones on the caller, the rest on workers
    bool run(int64_t n, const std::function<void(int64_t)>& fn) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        while (int64_t(workers_) < n - 1) {
            std::thread(&HostPool::work, this).detach();
            ++workers_;
        }
        job_.store(&fn);
        n_.store(n);
        next_.store(1);
        left_.store(n);
        open_.store(true);
        gen_.fetch_add(1);
        if (sleepers_.load() > 0) {
            std::lock_guard<std::mutex> g(mu_);
            cv_.notify_all();
        }
        guarded(fn, 0);
        for (int64_t t; (t = next_.fetch_add(1)) < n;) guarded(fn, t);
        open_.store(false);  // no worker joins this section from here on
        for (int spin = 0; left_.load() != 0 || inside_.load() != 0; ++spin)
            if (spin > 4096) std::this_thread::yield();
        std::exception_ptr ex;
        {
            std::lock_guard<std::mutex> g(mu_);
            std::swap(ex, err_);
        }
        if (ex) std::rethrow_exception(ex);
        return true;
    }

  private:
    static constexpr int64_t kSpinNs = 200000;  // a worker's spin before it sleeps
    // one task: a throw is recorded (the first one wins) instead of unwinding
    void guarded(const std::function<void(int64_t)>& fn, int64_t t) {
        try {
            fn(t);
        } catch (...) {
            std::lock_guard<std::mutex> g(mu_);
            if (!err_) err_ = std::current_exception();
        }
        left_.fetch_sub(1);
    }
    void work() {
        uint64_t seen = gen_.load();
        for (;;) {
            const auto t0 = std::chrono::steady_clock::now();
            for (int spin = 0; gen_.load() == seen; ++spin) {
                if ((spin & 255) == 255 &&
                    std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() >
                        kSpinNs) {
                    std::unique_lock<std::mutex> g(mu_);
                    sleepers_.fetch_add(1);
                    cv_.wait(g, [&] { return gen_.load() != seen; });
                    sleepers_.fetch_sub(1);
                    break;
                }
            }
            const uint64_t g = gen_.load();
            seen = g;
            inside_.fetch_add(1);
            // a section that closed (or a newer one that has not opened) is left alone
            if (open_.load() && gen_.load() == g) {
                const std::function<void(int64_t)>* job = job_.load();
                const int64_t n = n_.load();
                for (int64_t t; (t = next_.fetch_add(1)) < n;) guarded(*job, t);
            }
            inside_.fetch_sub(1);
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_;
    std::exception_ptr err_;
    std::atomic<const std::function<void(int64_t)>*> job_{nullptr};
    std::atomic<int64_t> n_{0}, next_{0}, left_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> inside_{0}, sleepers_{0};
    std::atomic<bool> open_{false};
    size_t workers_ = 0;
};

// fn(t, i0, i1) over nthr contiguous slices of [0, n) on the host pool
template <class F> inline void par_slices(int64_t nthr, int64_t n, F&& fn) {
    if (nthr <= 1) {
        fn(int64_t(0), int64_t(0), n);
        return;
    }
    const std::function<void(int64_t)> task = [&fn, nthr, n](int64_t t) { fn(t, n * t / nthr, n * (t + 1) / nthr); };
    if (!HostPool::get().run(nthr, task))
        for (int64_t t = 0; t < nthr; ++t) task(t);
}
inline int64_t host_threads() { return int64_t(std::clamp(std::thread::hardware_concurrency(), 1u, 16u)); }

}  // namespace fsm
