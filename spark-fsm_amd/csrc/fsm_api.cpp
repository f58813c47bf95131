// fsm_api.cpp — the extern "C" boundary (include/fsm.h).  Every entry point
// catches everything: no C++ exception crosses the ABI, failures come back as
// FSM_E* codes with the message in fsm_last_error (the Scala shim turns them
// into java.lang.Exception so TrainActor records FAILURE, TrainActor.scala:65-67).
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <new>
#include <thread>

#include "comm.h"
#include "dev_db.h"
#include "device_util.h"
#include "fsm_internal.h"
#include "host_pool.h"

using fsm::Error;

namespace {

thread_local std::string g_err;  // errors before a context exists

// FSM_SEGV_TRACE=1: a host fault prints the faulting thread's native backtrace to stderr,
// then the previous handler runs (debugging aid for Python / C hosts; resolve with
// addr2line).  Never installed inside a JVM: HotSpot handles SIGSEGV itself (implicit null
// checks, safepoints), and backtrace() is not async-signal-safe.
struct sigaction g_prev_sa[3];
const int kTraceSigs[3] = {SIGSEGV, SIGBUS, SIGABRT};
void segv_trace(int sig, siginfo_t* info, void* uc) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    const char msg[] = "[fsm] fatal signal; native backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(fr, n, 2);
    for (int k = 0; k < 3; ++k) {
        if (kTraceSigs[k] != sig) continue;
        const struct sigaction& p = g_prev_sa[k];
        if (p.sa_flags & SA_SIGINFO) {
            if (p.sa_sigaction) p.sa_sigaction(sig, info, uc);
            return;
        }
        if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN) {
            p.sa_handler(sig);
            return;
        }
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
void maybe_install_segv_trace() {
    static const bool once = [] {
        const char* v = std::getenv("FSM_SEGV_TRACE");
        if (v && v[0] == '1' && !dlsym(RTLD_DEFAULT, "JNI_CreateJavaVM")) {
            struct sigaction sa;
            std::memset(&sa, 0, sizeof(sa));
            sa.sa_sigaction = segv_trace;
            sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
            sigemptyset(&sa.sa_mask);
            for (int k = 0; k < 3; ++k) sigaction(kTraceSigs[k], &sa, &g_prev_sa[k]);
        }
        return true;
    }();
    (void)once;
}

int fail(fsm_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg; else g_err = msg;
    return code;
}

template <class F> int guarded(fsm_ctx* ctx, F&& f) {
    try {
        if (ctx) ctx->err.clear();
        fsm::PoolScope pool_scope(ctx ? ctx->pool : nullptr);
        f();
        return FSM_OK;
    } catch (const Error& e) {
        return fail(ctx, e.code, e.what());
    } catch (const std::bad_alloc&) {
        return fail(ctx, FSM_ENOMEM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(ctx, FSM_EDEVICE, e.what());
    } catch (...) {
        return fail(ctx, FSM_EDEVICE, "unknown error");
    }
}

// per-mine stats start from zero; the DB-build figures of the last fsm_db_* stay
void reset_stats(fsm_ctx* ctx) {
    const fsm_stats prev = ctx->stats;
    ctx->stats = fsm_stats{};
    ctx->stats.ms_flatten = prev.ms_flatten;
    ctx->stats.ms_upload = prev.ms_upload;
    ctx->stats.k0_device = prev.k0_device;
    ctx->stats.db_parses = prev.db_parses;
    ctx->stats.db_replicas = prev.db_replicas;
    ctx->kstats.clear();
}

template <class T> T* host_copy(const fsm::DevBuf& d, size_t n, hipStream_t s) {
    T* h = static_cast<T*>(std::malloc(std::max<size_t>(n, 1) * sizeof(T)));
    if (!h) throw Error(FSM_ENOMEM, "malloc failed");
    if (n) {
        const hipError_t e = hipMemcpyAsync(h, d.p, n * sizeof(T), hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) {
            std::free(h);
            throw Error(FSM_EDEVICE, std::string("hipMemcpyAsync failed: ") + hipGetErrorString(e));
        }
    }
    return h;
}

int group_make_db(fsm_ctx* ctx, int32_t mode, const fsm::Source& src, fsm_db** out);

int make_db(fsm_ctx* ctx, int32_t mode, const fsm::Source& src, fsm_db** out) {
    if (!ctx || !out) return fail(ctx, FSM_EINVAL, "null argument");
    *out = nullptr;
    if (src.n < 0 || (src.n > 0 && !src.sids)) return fail(ctx, FSM_EINVAL, "bad record arrays");
    if (mode != FSM_MODE_SPADE && mode != FSM_MODE_TSR) return fail(ctx, FSM_EINVAL, "mode must be SPADE(0) or TSR(1)");
    if (ctx->group) return group_make_db(ctx, mode, src, out);
    fsm_db* db = new (std::nothrow) fsm_db();
    if (!db) return fail(ctx, FSM_ENOMEM, "host allocation failed");
    db->ctx = ctx;
    db->mode = mode;
    const int rc = guarded(ctx, [&] {
        FSM_HIP(hipSetDevice(ctx->opts.device));
        ctx->stats.k0_device = 0;
        ctx->stats.db_parses = 1;  // this call's one pass over the caller's input
        ctx->stats.db_replicas = 0;
        if (fsm::k0_build(ctx, mode, src, db)) return;  // K0 on the GPU (token input)
        const double t0 = fsm::now_ms();
        if (mode == FSM_MODE_SPADE) fsm::flatten_spade(src, db->spade);
        else fsm::flatten_tsr(src, db->tsr);
        const double t1 = fsm::now_ms();
        if (mode == FSM_MODE_SPADE) fsm::spade_upload(ctx, db);
        else fsm::tsr_upload(ctx, db);
        // the engines read only the resident arrays and the item dictionary from here on
        // (the host copy of the rows is not kept: D1M's is about 300 MB)
        std::vector<uint32_t>().swap(db->spade.row_off);
        std::vector<uint32_t>().swap(db->spade.ent_item);
        std::vector<uint64_t>().swap(db->spade.ent_mask);
        std::vector<uint32_t>().swap(db->tsr.row_off);
        std::vector<uint32_t>().swap(db->tsr.ent_item);
        std::vector<uint32_t>().swap(db->tsr.ent_first);
        std::vector<uint32_t>().swap(db->tsr.ent_last);
        ctx->stats.ms_flatten = t1 - t0;
        ctx->stats.ms_upload = fsm::now_ms() - t1;
    });
    if (rc != FSM_OK) {
        fsm_db_free(db);
        return rc;
    }
    *out = db;
    return FSM_OK;
}

}  // namespace


// ------------------------------------------------------------------ in-process rank groups
// fsm_opts.ndevices > 1: one context drives N rank contexts (rank r on devices[r]), each
// with its own stream, pool, DB replica and an in-process communicator (comm.cpp).  The
// engines run unchanged on the rank contexts: the sharded mine of DESIGN.md §6, with
// the ranks as threads of the caller's process instead of processes.  Rank 0 runs on the
// calling thread, ranks 1..N-1 on persistent worker threads (each keeps its device
// current), so one call on the group context is one call for the caller.
//
// Bounded calls.  The caller (the JVM actor, TrainActor.scala:56-67) must get an error,
// never a hang: a hub barrier waits at most FSM_COMM_TIMEOUT_S for its peers (comm.cpp),
// and once rank 0 has returned the group waits at most that long for the other ranks,
// then aborts the hub (a rank blocked in a collective leaves with FSM_ECOMM) and, if a
// rank still has not returned after a short grace, reports it as stalled with FSM_ECOMM.
// The stalled rank's job (a closure holding everything it writes) stays alive with its
// thread; the group refuses calls until that rank has returned, and its contexts and DBs
// are leaked rather than freed under it if the caller destroys them first.
namespace fsm {

struct Group {
    std::shared_ptr<InProcHub> hub;
    std::vector<fsm_ctx*> ranks;
    std::vector<int> rc;
    std::vector<std::string> err;  // per-rank messages of steps without a rank context
    // set while a rank of an earlier call has not returned (shared with the group's DBs)
    std::shared_ptr<std::atomic<bool>> stuck = std::make_shared<std::atomic<bool>>(false);
    std::string stuck_msg;
    static constexpr int kStalled = -2;  // run(): a rank did not return within the limit

    explicit Group(int n)
        : hub(make_inproc_hub(n)), ranks(size_t(n), nullptr), rc(size_t(n), 0), err(size_t(n)) {
        try {
            for (int r = 1; r < n; ++r) th_.emplace_back([this, r] { work(r); });
        } catch (...) {  // (a half-built Group runs no destructor: join what started)
            stop_threads();
            throw;
        }
    }
    ~Group() { stop_threads(); }
    Group(const Group&) = delete;
    Group& operator=(const Group&) = delete;
    int n() const { return int(ranks.size()); }

    // fn(r) on every rank at once (rank 0 on the caller); a rank that fails aborts the hub so
    // that no peer stays blocked in a collective.  Returns the rank whose error to report
    // (the first one that did not fail only because a peer did), -1, or kStalled (stuck_msg).
    // fn is copied: a rank that outlives the call keeps its own reference to it.
    int run(std::function<int(int)> fn) {
        if (!ready()) return kStalled;
        auto job = std::make_shared<const std::function<int(int)>>(std::move(fn));
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = job;
            left_ = n() - 1;
            for (int r = 0; r < n(); ++r) done_r_[size_t(r)].store(0);
            ++gen_;
        }
        cv_.notify_all();
        one(*job, 0);
        const double lim = comm_timeout_ms("FSM_COMM_TIMEOUT_S");
        {
            std::unique_lock<std::mutex> g(mu_);
            auto all_done = [&] { return left_ == 0; };
            // a call still waiting for its ranks after 60 s reports where they are (stderr, once)
            const double first = std::min(lim, 60000.0);
            bool ok = done_.wait_for(g, std::chrono::duration<double, std::milli>(first), all_done);
            if (!ok && lim > first) {
                std::fprintf(stderr, "[fsm] rank group: %d of %d ranks still running after %.0f s (done:%s); %s\n",
                             left_, n(), first / 1000.0, done_list().c_str(), inproc_state(*hub).c_str());
                ok = done_.wait_for(g, std::chrono::duration<double, std::milli>(lim - first), all_done);
            }
            if (!ok) {
                // release every rank blocked in a collective, then give them a moment to return
                g.unlock();
                inproc_abort(*hub);
                g.lock();
                ok = done_.wait_for(g, std::chrono::seconds(2), all_done);
            }
            job_.reset();
            if (!ok) {
                std::string who;
                for (int r = 0; r < n(); ++r)
                    if (!done_r_[size_t(r)].load()) who += (who.empty() ? "" : ", ") + std::to_string(r);
                stuck_msg = "in-process rank group: rank(s) " + who + " did not return within FSM_COMM_TIMEOUT_S (" +
                            std::to_string(int(lim / 1000.0)) + " s); the call is aborted";
                stuck->store(true);
                return kStalled;
            }
        }
        inproc_reset(*hub);
        // the failing rank to report: one whose own message is not a peer's failure, preferably
        // one that failed before the hub was aborted
        int first = -1, best = 4;
        for (int r = 0; r < n(); ++r) {
            if (rc[size_t(r)] == FSM_OK) continue;
            const std::string& m = ranks[size_t(r)] ? ranks[size_t(r)]->err : err[size_t(r)];
            const bool msg_peer = m.find("peer rank failed") != std::string::npos;
            const int score = (msg_peer ? 2 : 0) + (after_abort_[size_t(r)] ? 1 : 0);
            if (score < best) {
                best = score;
                first = r;
            }
        }
        return first;
    }

    // true once every rank of every earlier call has returned (re-arms a stalled group)
    bool ready() {
        if (!stuck->load()) return true;
        std::lock_guard<std::mutex> g(mu_);
        if (left_ != 0) return false;
        inproc_reset(*hub);
        stuck->store(false);
        return true;
    }
    // wait up to ms for a stalled rank to return; false: it is still running
    bool drain(double ms) {
        if (!stuck->load()) return true;
        std::unique_lock<std::mutex> g(mu_);
        return done_.wait_for(g, std::chrono::duration<double, std::milli>(ms), [&] { return left_ == 0; });
    }

  private:
    void stop_threads() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
        th_.clear();
    }
    std::string done_list() const {
        std::string st;
        for (int r = 0; r < n(); ++r) st += " " + std::to_string(done_r_[size_t(r)].load());
        return st;
    }
    void one(const std::function<int(int)>& fn, int r) {
        int c;
        try {
            c = fn(r);
        } catch (...) {
            c = FSM_EDEVICE;
        }
        rc[size_t(r)] = c;
        // a rank that fails once the hub is already aborted failed because a peer did
        after_abort_[size_t(r)] = c != FSM_OK && inproc_aborted(*hub);
        if (c != FSM_OK) inproc_abort(*hub);
        done_r_[size_t(r)].store(1);
    }
    void work(int r) {
        uint64_t seen = 0;
        for (;;) {
            std::shared_ptr<const std::function<int(int)>> job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
            }
            if (job) one(*job, r);
            std::lock_guard<std::mutex> g(mu_);
            if (--left_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::shared_ptr<const std::function<int(int)>> job_;
    uint64_t gen_ = 0;
    int left_ = 0;
    bool stop_ = false;
    std::vector<char> after_abort_ = std::vector<char>(size_t(FSM_MAX_DEVICES), 0);
    std::vector<std::atomic<int>> done_r_ = std::vector<std::atomic<int>>(size_t(FSM_MAX_DEVICES));
};

}  // namespace fsm

namespace {

// the group's result: rank `who`'s error (message and code) on the group context,
// its statistics otherwise
int group_finish(fsm_ctx* ctx, int who) {
    fsm::Group& g = *ctx->group;
    if (who == fsm::Group::kStalled) {
        ctx->err = g.stuck_msg.empty() ? std::string("in-process rank group: a rank of an earlier call has not returned")
                                       : g.stuck_msg;
        return FSM_ECOMM;
    }
    fsm_ctx* r0 = g.ranks[0];
    if (r0) {
        ctx->stats = r0->stats;
        ctx->kstats = r0->kstats;
        // the DB-build counters summed over the ranks (one parse per group DB)
        ctx->stats.db_parses = ctx->stats.db_replicas = 0;
        for (fsm_ctx* rk : g.ranks)
            if (rk) {
                ctx->stats.db_parses += rk->stats.db_parses;
                ctx->stats.db_replicas += rk->stats.db_replicas;
            }
    }
    if (who < 0) {
        ctx->err.clear();
        return FSM_OK;
    }
    ctx->err = g.ranks[size_t(who)] ? g.ranks[size_t(who)]->err : g.err[size_t(who)];
    if (ctx->err.empty()) ctx->err = "rank " + std::to_string(who) + " failed";
    return g.rc[size_t(who)];
}

// the collective checks of fsm_comm_selftest on one rank's communicator
void comm_selftest(fsm::Comm& comm) {
    const uint32_t N = uint32_t(comm.nranks()), r = uint32_t(comm.rank());
    {
        // FSM_INJECT_FAIL="<rank>,selftest": that rank fails before its first collective (the
        // in-process transport must then release its peers with FSM_ECOMM, not leave them blocked)
        const char* v = std::getenv("FSM_INJECT_FAIL");
        char ph[16] = {0};
        int fr = -1;
        if (v && std::sscanf(v, "%d,%15s", &fr, ph) == 2 && fr == int(r) && !std::strcmp(ph, "selftest"))
            throw Error(FSM_ELIMIT, "selftest: injected failure (FSM_INJECT_FAIL)");
    }
    fsm::maybe_stall(int(r), "selftest");
    std::vector<uint32_t> v(1000);
    for (uint32_t i = 0; i < v.size(); ++i) v[i] = r + i;
    comm.host_allreduce_u32(v.data(), v.size(), nullptr);
    for (uint32_t i = 0; i < v.size(); ++i)
        if (v[i] != N * i + N * (N - 1) / 2) throw Error(FSM_ECOMM, "selftest: all-reduce mismatch");
    std::vector<uint8_t> mine(size_t(r) * 3 + 1);
    for (size_t j = 0; j < mine.size(); ++j) mine[j] = uint8_t(r * 7 + j);
    std::vector<size_t> sizes;
    // (the work-stealing counter of the claim test below is reset before this gather, which
    // also agrees on whether every rank has the shared counters)
    const int64_t key = comm.next_key();
    comm.reset_counter(key);
    uint32_t ex = comm.has_fetch_add() ? 1u : 0u;
    const std::vector<uint8_t> all = comm.gather_blobs(mine, sizes, nullptr, nullptr, &ex, 1);
    size_t at = 0;
    for (uint32_t q = 0; q < N; ++q) {
        if (sizes[q] != size_t(q) * 3 + 1) throw Error(FSM_ECOMM, "selftest: gather size mismatch");
        for (size_t j = 0; j < sizes[q]; ++j)
            if (all[at + j] != uint8_t(q * 7 + j)) throw Error(FSM_ECOMM, "selftest: gather data mismatch");
        at += sizes[q];
    }
    if (at != all.size()) throw Error(FSM_ECOMM, "selftest: gather length mismatch");
    if (ex != N && std::getenv("FSM_SELFTEST_REQUIRE_CLAIMS"))
        throw Error(FSM_ECOMM, "selftest: the ranks have no common work-stealing counter");
    if (ex == N) {
        // claims: the ranks take ranges of r + 1 units of [0, 997) from the shared counter
        // until it runs out; every unit must be claimed exactly once
        constexpr int64_t kUnits = 997;
        std::vector<uint8_t> got;
        for (;;) {
            const int64_t old = comm.fetch_add(key, int64_t(r) + 1);
            if (old < 0) throw Error(FSM_ECOMM, "selftest: fetch_add failed");
            if (old >= kUnits) break;
            for (int64_t u = old; u < std::min<int64_t>(old + r + 1, kUnits); ++u) {
                const uint16_t v16 = uint16_t(u);
                got.push_back(uint8_t(v16 & 0xFF));
                got.push_back(uint8_t(v16 >> 8));
            }
        }
        std::vector<size_t> csz;
        const std::vector<uint8_t> claimed = comm.gather_blobs(got, csz, nullptr);
        std::vector<int> seen(kUnits, 0);
        for (size_t j = 0; j + 1 < claimed.size(); j += 2) {
            const size_t u = size_t(claimed[j]) | (size_t(claimed[j + 1]) << 8);
            if (u >= size_t(kUnits)) throw Error(FSM_ECOMM, "selftest: claimed unit out of range");
            ++seen[u];
        }
        for (int64_t u = 0; u < kUnits; ++u)
            if (seen[size_t(u)] != 1) throw Error(FSM_ECOMM, "selftest: a unit was claimed " +
                                                                 std::to_string(seen[size_t(u)]) + " times");
    }
    // a root-only gather: rank 0 gets every blob in rank order (the others may get nothing)
    std::vector<size_t> rsz;
    const std::vector<uint8_t> root = comm.gather_blobs(mine, rsz, nullptr, nullptr, nullptr, 0, true);
    if (r == 0 && root != all) throw Error(FSM_ECOMM, "selftest: root-only gather mismatch");
}

// a device copy of `bytes` from src on device sdev to dst on device ddev (stream-ordered on s)
void copy_dev(void* dst, int ddev, const void* src, int sdev, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    if (ddev == sdev) FSM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    else FSM_HIP(hipMemcpyPeerAsync(dst, ddev, src, sdev, bytes, s));
}

// rank context c's replica of the group DB `src` (rank 0's, already built): the resident
// arrays copied device to device (over xGMI between GPUs) and the host metadata the
// engines read; TSR's vertical lists and sid bitmaps are rebuilt from the rows on c's device
int replicate_db(fsm_ctx* c, const fsm_db* src, fsm_db** out) {
    *out = nullptr;
    fsm_db* db = new (std::nothrow) fsm_db();
    if (!db) return fail(c, FSM_ENOMEM, "host allocation failed");
    db->ctx = c;
    db->mode = src->mode;
    const int rc = guarded(c, [&] {
        const double t0 = fsm::now_ms();
        FSM_HIP(hipSetDevice(c->opts.device));
        const int sd = src->ctx->opts.device, dd = c->opts.device;
        if (dd != sd) {
            const hipError_t e = hipDeviceEnablePeerAccess(sd, 0);  // (without it the copy is staged)
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        }
        hipStream_t s = c->stream;
        if (src->mode == FSM_MODE_SPADE) {
            const SpadeDevDB* a = src->spade_dev;
            auto d = std::make_unique<SpadeDevDB>();
            d->R = a->R;
            d->E = a->E;
            d->U = a->U;
            d->W = a->W;
            d->row_off.alloc(size_t(a->R + 1) * 4);
            d->item.alloc(std::max<size_t>(size_t(a->E), 1) * 4);
            d->mask.alloc(std::max<size_t>(size_t(a->E), 1) * 8 * size_t(a->W));
            copy_dev(d->row_off.p, dd, a->row_off.p, sd, size_t(a->R + 1) * 4, s);
            copy_dev(d->item.p, dd, a->item.p, sd, size_t(a->E) * 4, s);
            copy_dev(d->mask.p, dd, a->mask.p, sd, size_t(a->E) * 8 * size_t(a->W), s);
            FSM_HIP(hipStreamSynchronize(s));
            db->spade.total = src->spade.total;
            db->spade.W = src->spade.W;
            db->spade.max_occ = src->spade.max_occ;
            db->spade.item_val = src->spade.item_val;
            db->spade_dev = d.release();
        } else {
            const TsrDevDB* a = src->tsr_dev;
            auto d = std::make_unique<TsrDevDB>();
            d->N = a->N;
            d->E = a->E;
            d->U = a->U;
            d->row_off.alloc(size_t(a->N + 1) * 4);
            for (fsm::DevBuf* b : {&d->item, &d->first, &d->last}) b->alloc(std::max<size_t>(size_t(a->E), 1) * 4);
            copy_dev(d->row_off.p, dd, a->row_off.p, sd, size_t(a->N + 1) * 4, s);
            copy_dev(d->item.p, dd, a->item.p, sd, size_t(a->E) * 4, s);
            copy_dev(d->first.p, dd, a->first.p, sd, size_t(a->E) * 4, s);
            copy_dev(d->last.p, dd, a->last.p, sd, size_t(a->E) * 4, s);
            fsm::tsr_finish(c, d.get());  // synchronizes
            db->tsr.total = src->tsr.total;
            db->tsr.item_val = src->tsr.item_val;
            db->tsr_dev = d.release();
        }
        c->stats.db_parses = 0;
        c->stats.db_replicas = 1;
        c->stats.k0_device = 0;
        c->stats.ms_flatten = 0;
        c->stats.ms_upload = fsm::now_ms() - t0;
    });
    if (rc != FSM_OK) {
        fsm_db_free(db);
        return rc;
    }
    *out = db;
    return FSM_OK;
}

// The group's DB: parsed and flattened ONCE (rank 0, on the calling thread: the host
// flatten + upload or K0 on its device), then every other rank copies rank 0's resident
// arrays device to device.  The caller's input arrays are read by the calling thread only.
int group_make_db(fsm_ctx* ctx, int32_t mode, const fsm::Source& src, fsm_db** out) {
    fsm::Group& g = *ctx->group;
    if (!g.ready()) return group_finish(ctx, fsm::Group::kStalled);
    fsm_db* db = new (std::nothrow) fsm_db();
    if (!db) return fail(ctx, FSM_ENOMEM, "host allocation failed");
    db->ctx = ctx;
    db->mode = mode;
    db->group_stuck = g.stuck;
    db->parts.assign(size_t(g.n()), nullptr);
    int rc = make_db(g.ranks[0], mode, src, &db->parts[0]);
    if (rc != FSM_OK) {
        ctx->err = g.ranks[0]->err;
    } else {
        fsm_db* const base = db->parts[0];
        std::vector<fsm_ctx*> ranks = g.ranks;
        const int who = g.run([db, base, ranks](int r) {
            return r == 0 ? FSM_OK : replicate_db(ranks[size_t(r)], base, &db->parts[size_t(r)]);
        });
        rc = group_finish(ctx, who);
    }
    if (rc != FSM_OK) {
        fsm_db_free(db);
        return rc;
    }
    *out = db;
    return FSM_OK;
}

}  // namespace

void fsm::set_thread_error(const std::string& msg) { g_err = msg; }

extern "C" {

int fsm_abi_version(void) { return FSM_ABI_VERSION; }

int fsm_comm_unique_id(uint8_t out[128]) {
    if (!out) return FSM_EINVAL;
    std::memset(out, 0, 128);
    return guarded(nullptr, [&] { fsm::rccl_unique_id(out); });
}

int fsm_shard_plan(const uint64_t* volume, int64_t n, int32_t nranks, int32_t* owner) {
    if (n < 0 || nranks < 1 || (n > 0 && (!volume || !owner))) return fail(nullptr, FSM_EINVAL, "bad shard plan arguments");
    return guarded(nullptr, [&] { fsm::shard_plan(volume, n, nranks, owner); });
}

int fsm_comm_selftest(const fsm_opts* opts) {
    if (opts && opts->ndevices > 1 && opts->nranks <= 1) {
        // the in-process transport on ndevices host threads (no GPU)
        if (opts->ndevices > FSM_MAX_DEVICES) return fail(nullptr, FSM_EINVAL, "ndevices exceeds FSM_MAX_DEVICES");
        const int N = opts->ndevices;
        // (heap: a rank that stalls past FSM_COMM_TIMEOUT_S keeps the group; it is then leaked)
        auto* gp = new fsm::Group(N);
        auto hub = gp->hub;
        const int who = gp->run([gp, hub](int r) {
            const int c = guarded(nullptr, [&] {
                auto comm = fsm::make_inproc_comm(hub, r);
                comm_selftest(*comm);
            });
            if (c != FSM_OK) gp->err[size_t(r)] = g_err;
            return c;
        });
        if (who == fsm::Group::kStalled) return fail(nullptr, FSM_ECOMM, gp->stuck_msg);  // (gp leaked)
        const int code = who < 0 ? FSM_OK : gp->rc[size_t(who)];
        const std::string msg = who < 0 ? std::string() : "rank " + std::to_string(who) + ": " + gp->err[size_t(who)];
        delete gp;
        return who < 0 ? FSM_OK : fail(nullptr, code, msg);
    }
    if (!opts || opts->nranks < 2) return fail(nullptr, FSM_EINVAL, "selftest needs nranks >= 2 or ndevices >= 2");
    return guarded(nullptr, [&] {
        if (!opts->host_comm) FSM_HIP(hipSetDevice(opts->device));
        auto comm = fsm::make_comm(*opts);
        comm_selftest(*comm);
    });
}

}  // extern "C"

namespace {

// one context on one device; comm: the in-process communicator of a group's rank
// (nullptr: make_comm from the options)
int create_one(const fsm_opts& opts, std::unique_ptr<fsm::Comm> comm, fsm_ctx** out, int dev_share = 1) {
    *out = nullptr;
    fsm_ctx* ctx = new (std::nothrow) fsm_ctx();
    if (!ctx) return fail(nullptr, FSM_ENOMEM, "host allocation failed");
    ctx->opts = opts;
    ctx->dev_share = std::max(dev_share, 1);
    if (ctx->opts.nranks <= 0) ctx->opts.nranks = 1;
    const int rc = guarded(ctx, [&] {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
            throw Error(FSM_EDEVICE, "no HIP device available (libfsm requires an MI355X / gfx950 GPU)");
        if (ctx->opts.device < 0 || ctx->opts.device >= ndev)
            throw Error(FSM_EINVAL, "device ordinal " + std::to_string(ctx->opts.device) + " out of range");
        FSM_HIP(hipSetDevice(ctx->opts.device));
        hipDeviceProp_t prop;
        FSM_HIP(hipGetDeviceProperties(&prop, ctx->opts.device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            throw Error(FSM_EDEVICE, std::string("libfsm is built for gfx950; device is ") + prop.gcnArchName);
        FSM_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->pool = std::make_shared<fsm::Pool>(ctx->opts.device);
        ctx->comm = comm ? comm.release() : fsm::make_comm(ctx->opts).release();
        // the host side a DB build and a mine use from their first call: the staging
        // ring (two 4 MiB pinned slots, each DMA'd once: the first DMA from a pinned
        // buffer is slow) and the host thread pool's workers
        {
            // (from the context's own pool: guarded() captured the pool before it existed)
            fsm::PoolScope ps(ctx->pool);
            const size_t rb = size_t(4) << 20;
            fsm::DevBuf warm(rb);
            for (int slot = 2; slot <= 3; ++slot) {
                std::memset(ctx->stage_host(slot, rb), 0, rb);
                ctx->stage_copy(slot, warm.p, rb);
            }
            FSM_HIP(hipStreamSynchronize(ctx->stream));
        }
        fsm::par_slices(fsm::host_threads(), fsm::host_threads(), [](int64_t, int64_t, int64_t) {});
    });
    if (rc != FSM_OK) {
        g_err = ctx->err;
        fsm_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return FSM_OK;
}

// fsm_opts.ndevices > 1: the group context and its rank contexts, each made on its own
// thread (its device current there from then on)
int create_group(const fsm_opts& opts, fsm_ctx** out) {
    const int N = opts.ndevices;
    if (N > FSM_MAX_DEVICES) return fail(nullptr, FSM_EINVAL, "ndevices exceeds FSM_MAX_DEVICES");
    if (opts.nranks > 1) return fail(nullptr, FSM_EINVAL, "ndevices > 1 (in-process ranks) excludes nranks > 1");
    fsm_ctx* ctx = new (std::nothrow) fsm_ctx();
    if (!ctx) return fail(nullptr, FSM_ENOMEM, "host allocation failed");
    ctx->opts = opts;
    ctx->opts.device = opts.devices[0];
    ctx->opts.nranks = 1;
    int rc = FSM_OK;
    try {
        ctx->group = std::make_unique<fsm::Group>(N);
    } catch (const std::exception& e) {
        rc = fail(nullptr, FSM_ENOMEM, std::string("cannot start the rank threads: ") + e.what());
    }
    if (rc == FSM_OK) {
        fsm::Group& g = *ctx->group;
        // ranks sharing a device split its default memory budgets (fsm_ctx::dev_share)
        std::vector<int> share(size_t(N), 0);
        for (int r = 0; r < N; ++r)
            for (int q = 0; q < N; ++q) share[size_t(r)] += opts.devices[q] == opts.devices[r] ? 1 : 0;
        fsm::Group* gp = &g;
        const int who = g.run([gp, opts, N, share](int r) {
            fsm_opts o = opts;
            o.ndevices = 0;
            o.device = opts.devices[r];
            o.nranks = N;
            o.rank = r;
            o.host_comm = nullptr;
            const int c = create_one(o, fsm::make_inproc_comm(gp->hub, r), &gp->ranks[size_t(r)], share[size_t(r)]);
            if (c != FSM_OK) gp->err[size_t(r)] = g_err;  // (thread-local on this rank's thread)
            else gp->ranks[size_t(r)]->result_root_only = true;
            return c;
        });
        if (who == fsm::Group::kStalled) rc = fail(nullptr, FSM_ECOMM, g.stuck_msg);
        else if (who >= 0)
            rc = fail(nullptr, g.rc[size_t(who)], "rank " + std::to_string(who) + " (device " +
                                                      std::to_string(opts.devices[who]) + "): " + g.err[size_t(who)]);
    }
    if (rc != FSM_OK) {
        const std::string keep = g_err;
        fsm_ctx_destroy(ctx);
        g_err = keep;
        return rc;
    }
    *out = ctx;
    return FSM_OK;
}

}  // namespace

extern "C" {

int fsm_ctx_create(const fsm_opts* opts, fsm_ctx** out) {
    maybe_install_segv_trace();
    if (!out) return FSM_EINVAL;
    *out = nullptr;
    fsm_opts o{};
    if (opts) o = *opts;
    if (o.ndevices > 1) return create_group(o, out);
    return create_one(o, nullptr, out);
}

void fsm_ctx_destroy(fsm_ctx* ctx) {
    if (!ctx) return;
    if (ctx->group) {
        fsm::Group& g = *ctx->group;
        // a rank still inside a timed-out call keeps running on the rank contexts: wait for it
        // (bounded), else leak the group and its contexts rather than free them under it
        if (!g.drain(fsm::comm_timeout_ms("FSM_COMM_TIMEOUT_S")) || !g.ready()) {
            (void)ctx->group.release();
            delete ctx;
            return;
        }
        // each rank context is destroyed on its own thread (its device current there)
        fsm::Group* gp = &g;
        (void)g.run([gp](int r) {
            fsm_ctx_destroy(gp->ranks[size_t(r)]);
            gp->ranks[size_t(r)] = nullptr;
            return FSM_OK;
        });
        if (g.stuck->load()) (void)ctx->group.release();  // (a rank stalled in the destroy itself)
        else ctx->group.reset();
        delete ctx;
        return;
    }
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (hipEvent_t e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->stage_ev)
        if (e) (void)hipEventDestroy(e);
    delete ctx->comm;
    if (ctx->pool) ctx->pool->trim();  // this context's cached blocks only; live DBs keep their pool alive
    ctx->pool.reset();
    if (ctx->stream) {
        fsm::scan_release(ctx->stream);
        (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
}

int fsm_get_kernel_stats(const fsm_ctx* ctx, fsm_kernel_stat* out, int32_t max, int32_t* n) {
    if (!ctx || !n || max < 0 || (max > 0 && !out)) return FSM_EINVAL;
    *n = int32_t(ctx->kstats.size());
    for (int32_t k = 0; k < max && k < *n; ++k) out[k] = ctx->kstats[size_t(k)];
    return FSM_OK;
}

const char* fsm_last_error(const fsm_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int fsm_get_stats(const fsm_ctx* ctx, fsm_stats* out) {
    if (!ctx || !out) return FSM_EINVAL;
    *out = ctx->stats;
    return FSM_OK;
}

int fsm_db_from_spmf(fsm_ctx* ctx, int32_t mode, const int32_t* sids, const char* const* lines, const int64_t* lens,
                     int64_t n, fsm_db** out) {
    if (n > 0 && (!lines || !lens)) return fail(ctx, FSM_EINVAL, "null lines/lens");
    fsm::Source src;
    src.sids = sids;
    src.lines = lines;
    src.lens = lens;
    src.n = n;
    return make_db(ctx, mode, src, out);
}

int fsm_db_from_tokens(fsm_ctx* ctx, int32_t mode, const int32_t* sids, const int64_t* seq_off,
                       const int64_t* tokens, int64_t n, fsm_db** out) {
    if (n > 0 && (!seq_off || (!tokens && seq_off[n] > 0))) return fail(ctx, FSM_EINVAL, "null token arrays");
    fsm::Source src;
    src.sids = sids;
    src.seq_off = seq_off;
    src.tokens = tokens;
    src.n = n;
    return make_db(ctx, mode, src, out);
}

int fsm_db_export(fsm_ctx* ctx, const fsm_db* db, fsm_db_image** out) {
    if (!ctx || !db || !out) return fail(ctx, FSM_EINVAL, "null argument");
    *out = nullptr;
    if (db->ctx != ctx) return fail(ctx, FSM_EINVAL, "db belongs to another context");
    if (ctx->group) {  // rank 0's replica (every rank holds the same DB)
        const int rc = fsm_db_export(ctx->group->ranks[0], db->parts[0], out);
        if (rc != FSM_OK) ctx->err = ctx->group->ranks[0]->err;
        return rc;
    }
    auto* img = static_cast<fsm_db_image*>(std::calloc(1, sizeof(fsm_db_image)));
    if (!img) return fail(ctx, FSM_ENOMEM, "calloc failed");
    const int rc = guarded(ctx, [&] {
        FSM_HIP(hipSetDevice(ctx->opts.device));
        hipStream_t s = ctx->stream;
        img->mode = db->mode;
        if (db->mode == FSM_MODE_SPADE) {
            const SpadeDevDB* d = db->spade_dev;
            img->mask_words = d->W;
            img->rows = d->R;
            img->entries = d->E;
            img->max_occ = db->spade.max_occ;
            img->row_off = host_copy<uint32_t>(d->row_off, size_t(d->R + 1), s);
            img->item = host_copy<uint32_t>(d->item, size_t(d->E), s);
            img->mask = host_copy<uint64_t>(d->mask, size_t(d->E) * size_t(d->W), s);
            img->items = int64_t(db->spade.item_val.size());
            img->item_val = static_cast<int32_t*>(std::malloc(std::max<size_t>(db->spade.item_val.size(), 1) * 4));
            if (!img->item_val) throw Error(FSM_ENOMEM, "malloc failed");
            std::memcpy(img->item_val, db->spade.item_val.data(), db->spade.item_val.size() * 4);
        } else {
            const TsrDevDB* d = db->tsr_dev;
            img->rows = d->N;
            img->entries = d->E;
            img->row_off = host_copy<uint32_t>(d->row_off, size_t(d->N + 1), s);
            img->item = host_copy<uint32_t>(d->item, size_t(d->E), s);
            img->first = host_copy<uint32_t>(d->first, size_t(d->E), s);
            img->last = host_copy<uint32_t>(d->last, size_t(d->E), s);
            img->items = int64_t(db->tsr.item_val.size());
            img->item_val = static_cast<int32_t*>(std::malloc(std::max<size_t>(db->tsr.item_val.size(), 1) * 4));
            if (!img->item_val) throw Error(FSM_ENOMEM, "malloc failed");
            std::memcpy(img->item_val, db->tsr.item_val.data(), db->tsr.item_val.size() * 4);
        }
        FSM_HIP(hipStreamSynchronize(s));
    });
    if (rc != FSM_OK) {
        fsm_db_image_free(img);
        return rc;
    }
    *out = img;
    return FSM_OK;
}

void fsm_db_image_free(fsm_db_image* img) {
    if (!img) return;
    std::free(img->row_off);
    std::free(img->item);
    std::free(img->mask);
    std::free(img->first);
    std::free(img->last);
    std::free(img->item_val);
    std::free(img);
}

void fsm_db_free(fsm_db* db) {
    if (!db) return;
    // a group DB whose group has a rank still inside a timed-out call: that rank may read
    // its replica, so the DB is leaked instead (fsm_api.cpp, Group)
    if (db->group_stuck && db->group_stuck->load()) return;
    for (fsm_db* p : db->parts) fsm_db_free(p);
    fsm::spade_release(db);
    fsm::tsr_release(db);
    delete db;
}

int fsm_spade_mine(fsm_ctx* ctx, fsm_db* db, double support, int32_t dfs, fsm_patterns** out) {
    (void)dfs;  // DFS vs BFS only changes the discovery order, not the pattern set
    if (!ctx || !db || !out) return fail(ctx, FSM_EINVAL, "null argument");
    *out = nullptr;
    if (db->ctx != ctx) return fail(ctx, FSM_EINVAL, "db belongs to another context");
    if (db->mode != FSM_MODE_SPADE) return fail(ctx, FSM_EINVAL, "db was not flattened for SPADE");
    if (ctx->group) {
        fsm::Group& g = *ctx->group;
        // the closure owns everything a rank writes (a rank may outlive a timed-out call)
        auto res = std::make_shared<std::vector<fsm_patterns*>>(size_t(g.n()), nullptr);
        const std::vector<fsm_ctx*> ranks = g.ranks;
        const std::vector<fsm_db*> parts = db->parts;
        const int who = g.run([res, ranks, parts, support, dfs](int r) {
            return fsm_spade_mine(ranks[size_t(r)], parts[size_t(r)], support, dfs, &(*res)[size_t(r)]);
        });
        const int rc = group_finish(ctx, who);
        if (who == fsm::Group::kStalled) return rc;  // (the results of the returned ranks are leaked)
        for (size_t r = 1; r < res->size(); ++r) fsm_patterns_free((*res)[r]);  // (empty: root-only output)
        if (rc != FSM_OK) fsm_patterns_free((*res)[0]);
        else *out = (*res)[0];
        return rc;
    }
    return guarded(ctx, [&] {
        FSM_HIP(hipSetDevice(ctx->opts.device));
        reset_stats(ctx);
        const bool prof = fsm::host_prof_start();
        try {
            fsm::spade_mine(ctx, db, support, out);
        } catch (...) {
            if (prof) fsm::host_prof_stop();
            throw;
        }
        if (prof) fsm::host_prof_stop();
    });
}

int fsm_tsr_mine(fsm_ctx* ctx, fsm_db* db, int32_t k, double minconf, fsm_rules** out) {
    if (!ctx || !db || !out) return fail(ctx, FSM_EINVAL, "null argument");
    *out = nullptr;
    if (db->ctx != ctx) return fail(ctx, FSM_EINVAL, "db belongs to another context");
    if (db->mode != FSM_MODE_TSR) return fail(ctx, FSM_EINVAL, "db was not flattened for TSR");
    if (k < 1) return fail(ctx, FSM_EINVAL, "TSR: k must be >= 1 (got " + std::to_string(k) + ")");
    if (ctx->group) {
        fsm::Group& g = *ctx->group;
        auto res = std::make_shared<std::vector<fsm_rules*>>(size_t(g.n()), nullptr);
        const std::vector<fsm_ctx*> ranks = g.ranks;
        const std::vector<fsm_db*> parts = db->parts;
        const int who = g.run([res, ranks, parts, k, minconf](int r) {
            return fsm_tsr_mine(ranks[size_t(r)], parts[size_t(r)], k, minconf, &(*res)[size_t(r)]);
        });
        const int rc = group_finish(ctx, who);
        if (who == fsm::Group::kStalled) return rc;
        for (size_t r = 1; r < res->size(); ++r) fsm_rules_free((*res)[r]);  // (the replay is replicated)
        if (rc != FSM_OK) fsm_rules_free((*res)[0]);
        else *out = (*res)[0];
        return rc;
    }
    return guarded(ctx, [&] {
        FSM_HIP(hipSetDevice(ctx->opts.device));
        reset_stats(ctx);
        const bool prof = fsm::host_prof_start();
        try {
            fsm::tsr_mine(ctx, db, k, minconf, out);
        } catch (...) {
            if (prof) fsm::host_prof_stop();
            throw;
        }
        if (prof) fsm::host_prof_stop();
    });
}

// (result arrays may be big host blocks: fsm::big_give frees malloc'ed ones, caches the others)
void fsm_patterns_free(fsm_patterns* p) {
    if (!p) return;
    fsm::big_give(p->support);
    fsm::big_give(p->pat_off);
    fsm::big_give(p->set_off);
    fsm::big_give(p->items);
    std::free(p);
}

void fsm_rules_free(fsm_rules* r) {
    if (!r) return;
    fsm::big_give(r->support);
    fsm::big_give(r->confidence);
    fsm::big_give(r->ante_off);
    fsm::big_give(r->ante);
    fsm::big_give(r->cons_off);
    fsm::big_give(r->cons);
    std::free(r);
}

}  // extern "C"
