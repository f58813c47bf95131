// host_pool.h — the persistent host thread pool behind the engines' parallel
// host sections (spade_engine batch bookkeeping, K0 token staging).
#pragma once

#include <algorithm>
#include <atomic>
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
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            n_ = n;
            next_.store(1);
            left_ = n;
            ++gen_;
        }
        cv_.notify_all();
        guarded(fn, 0);
        for (int64_t t; (t = next_.fetch_add(1)) < n;) guarded(fn, t);
        std::exception_ptr ex;
        {
            std::unique_lock<std::mutex> g(mu_);
            // every worker that joined this section has left it before the next can start
            done_cv_.wait(g, [&] { return left_ == 0 && active_ == 0; });
            job_ = nullptr;
            std::swap(ex, err_);
        }
        if (ex) std::rethrow_exception(ex);
        return true;
    }

  private:
    // one task: a throw is recorded (the first one wins) instead of unwinding
    void guarded(const std::function<void(int64_t)>& fn, int64_t t) {
        try {
            fn(t);
        } catch (...) {
            std::lock_guard<std::mutex> g(mu_);
            if (!err_) err_ = std::current_exception();
        }
        finish_one();
    }
    void finish_one() {
        std::lock_guard<std::mutex> g(mu_);
        if (--left_ == 0 && active_ == 0) done_cv_.notify_all();
    }
    void work() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int64_t)>* job;
            int64_t n;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen && job_ != nullptr; });
                seen = gen_;
                job = job_;
                n = n_;
                ++active_;
            }
            for (int64_t t; (t = next_.fetch_add(1)) < n;) guarded(*job, t);
            std::lock_guard<std::mutex> g(mu_);
            if (--active_ == 0 && left_ == 0) done_cv_.notify_all();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int64_t)>* job_ = nullptr;
    std::exception_ptr err_;
    int64_t n_ = 0, left_ = 0, active_ = 0;
    uint64_t gen_ = 0;
    std::atomic<int64_t> next_{0};
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
