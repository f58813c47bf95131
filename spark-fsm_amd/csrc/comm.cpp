// comm.cpp — the two collectives the sharded SPADE path needs:
// an in-place u32 sum all-reduce (F1 histogram, statistics) and an all-gather
// of equal-sized byte blocks (frequent-pair records, pattern CSRs).
//
//   RcclComm  one rank per GPU over RCCL (xGMI inside a node).  librccl is
//             dlopen'ed on first use, so that libfsm loads and runs single-GPU
//             without it, and binds to the librccl.so.1 a host process (PyTorch)
//             has already loaded instead of a second copy.
//   HostComm  host callbacks supplied by the caller (fsm_host_comm): used to
//             run several ranks on one GPU (tests) or over any host transport.
//             Device buffers are staged through host memory around the callback.
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>

#include <rccl/rccl.h>

#include "comm.h"

namespace fsm {
namespace {

struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
    ncclResult_t (*comm_get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    static std::string err;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            err = std::string("cannot load librccl.so.1: ") + dlerror();
            return;
        }
        api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        api.comm_init_rank_config =
            reinterpret_cast<decltype(api.comm_init_rank_config)>(dlsym(h, "ncclCommInitRankConfig"));
        api.comm_get_async_error =
            reinterpret_cast<decltype(api.comm_get_async_error)>(dlsym(h, "ncclCommGetAsyncError"));
        api.comm_abort = reinterpret_cast<decltype(api.comm_abort)>(dlsym(h, "ncclCommAbort"));
        api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(dlsym(h, "ncclAllReduce"));
        api.all_gather = reinterpret_cast<decltype(api.all_gather)>(dlsym(h, "ncclAllGather"));
        api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(h, "ncclGetErrorString"));
        if (!api.get_unique_id || !api.comm_init_rank_config || !api.comm_get_async_error || !api.comm_abort ||
            !api.comm_destroy || !api.all_reduce || !api.all_gather || !api.error_string) {
            err = "librccl.so.1 lacks an expected symbol";
            api = RcclApi{};
        }
    });
    if (!api.all_reduce) throw Error(FSM_ECOMM, err.empty() ? "RCCL unavailable" : err);
    return api;
}

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Error(FSM_ECOMM, std::string(what) + ": " + rccl().error_string(r));
}

// The communicator is created non-blocking, so that a peer that never joins (it
// failed before its own init) cannot block this rank forever: the init is polled
// up to FSM_COMM_INIT_TIMEOUT_S seconds (default 300), then aborted with FSM_ECOMM.
// Non-blocking communicators may return ncclInProgress from a collective's enqueue
// as well; wait() polls the communicator's state until the enqueue has completed.
// The work-stealing counters of the ranks of one node: a POSIX shared-memory segment
// named after the communicator's unique id.  Every rank opens it BEFORE the collective
// that completes the communicator's setup (so every rank has it open once that returns);
// rank 0 then unlinks the name (the mappings stay until each rank unmaps).  Slots are
// reused every kSlots keys: reset(key) zeroes key's slot on rank 0 before the
// collective that precedes its first claim.
class ShmCounters {
  public:
    static constexpr size_t kSlots = 512;  // + 1 probe slot (counters_shared)
    explicit ShmCounters(const uint8_t id[128]) {
        uint64_t h = 1469598103934665603ull;  // FNV-1a of the unique id
        for (int k = 0; k < 128; ++k) h = (h ^ id[k]) * 1099511628211ull;
        std::snprintf(name_, sizeof(name_), "/fsm-claims-%016llx", (unsigned long long)h);
        const int fd = shm_open(name_, O_CREAT | O_RDWR, 0600);
        if (fd < 0) return;
        if (ftruncate(fd, off_t((kSlots + 1) * sizeof(int64_t))) == 0) {
            void* p = mmap(nullptr, (kSlots + 1) * sizeof(int64_t), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (p != MAP_FAILED) ctr_ = static_cast<int64_t*>(p);
        }
        close(fd);
    }
    ~ShmCounters() {
        if (ctr_) munmap(ctr_, (kSlots + 1) * sizeof(int64_t));
    }
    ShmCounters(const ShmCounters&) = delete;
    ShmCounters& operator=(const ShmCounters&) = delete;
    void unlink_name() { shm_unlink(name_); }  // rank 0, once every rank has opened it
    bool ok() const { return ctr_ != nullptr; }
    int64_t fetch_add(int64_t key, int64_t inc) {
        return ctr_ ? __atomic_fetch_add(&ctr_[size_t(key) % kSlots], inc, __ATOMIC_SEQ_CST) : -1;
    }
    void reset(int64_t key) {
        // slot key % kSlots was last used kSlots keys ago, long past that mine's final gather
        if (ctr_) __atomic_store_n(&ctr_[size_t(key) % kSlots], int64_t(0), __ATOMIC_SEQ_CST);
    }
    void set_probe(int64_t v) {
        if (ctr_) __atomic_store_n(&ctr_[kSlots], v, __ATOMIC_SEQ_CST);
    }
    int64_t probe() const { return ctr_ ? __atomic_load_n(&ctr_[kSlots], __ATOMIC_SEQ_CST) : 0; }

  private:
    char name_[64] = {0};
    int64_t* ctr_ = nullptr;
};


// Whether every rank's ShmCounters are ONE segment (ranks on one node sharing /dev/shm):
// rank 0 stores a nonce in the probe slot, the nonce is all-gathered, every rank reads
// the slot back, and the ranks all-reduce whether they saw it.  Ranks on another node
// (or in a container with its own /dev/shm) have a segment of their own under the same
// name; without this check each such group would claim every class and the gathered
// output would hold duplicates.  Collective; false on every rank unless all agree.
bool counters_shared(Comm& c, ShmCounters& shm) {
    int64_t nonce = 0;
    if (c.rank() == 0) {
        nonce = int64_t((uint64_t(std::chrono::steady_clock::now().time_since_epoch().count()) * 0x9E3779B97F4A7C15ull ^
                         (uint64_t(getpid()) << 20)) | 1u) & INT64_MAX;
        shm.set_probe(nonce);
    }
    std::vector<int64_t> all(size_t(c.nranks()), 0);
    c.host_allgather(&nonce, all.data(), sizeof(int64_t), nullptr);
    uint32_t ok = shm.ok() && shm.probe() == all[0] ? 1u : 0u;
    c.host_allreduce_u32(&ok, 1, nullptr);
    return ok == uint32_t(c.nranks());
}

bool id_set(const uint8_t id[128]) {
    for (int k = 0; k < 128; ++k)
        if (id[k]) return true;
    return false;
}

class RcclComm final : public Comm {
  public:
    RcclComm(int nranks, int rank, const uint8_t id[128]) : Comm(nranks, rank), shm_(id) {
        ncclUniqueId uid;
        std::memcpy(uid.internal, id, sizeof(uid.internal));
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclResult_t r = rccl().comm_init_rank_config(&comm_, nranks, uid, rank, &cfg);
        if (r != ncclSuccess && r != ncclInProgress) {
            if (comm_) (void)rccl().comm_abort(comm_);
            comm_ = nullptr;
            nccl_check(r, "ncclCommInitRankConfig");
        }
        try {
            wait("ncclCommInitRankConfig", comm_timeout_ms("FSM_COMM_INIT_TIMEOUT_S"));
        } catch (...) {
            shm_.unlink_name();
            throw;
        }
        // every rank has the segment open once the setup completed: each unlinks the name (the
        // first call removes it; on a multi-node job every node's segment goes)
        shm_.unlink_name();
        shared_ = counters_shared(*this, shm_);
    }
    ~RcclComm() override {
        if (comm_) (void)rccl().comm_destroy(comm_);
    }
    bool has_fetch_add() const override { return shared_; }
    int64_t fetch_add(int64_t key, int64_t inc) override { return shm_.fetch_add(key, inc); }
    void reset_counter(int64_t key) override {
        if (rank() == 0) shm_.reset(key);
    }
    void host_allreduce_u32(uint32_t* h, size_t n, hipStream_t s) override {
        if (!n) return;
        auto* d = static_cast<uint32_t*>(staging(n * 4));
        FSM_HIP(hipMemcpyAsync(d, h, n * 4, hipMemcpyHostToDevice, s));
        allreduce_u32(d, n, s);
        FSM_HIP(hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
    }
    void host_allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        if (!bytes) return;
        const size_t all = bytes * size_t(nranks());
        auto* d = static_cast<uint8_t*>(staging(all + ((bytes + 255) & ~size_t(255))));
        uint8_t* ds = d + all;  // the send block after the receive blocks
        FSM_HIP(hipMemcpyAsync(ds, send, bytes, hipMemcpyHostToDevice, s));
        allgather(ds, d, bytes, s);
        FSM_HIP(hipMemcpyAsync(recv, d, all, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
    }
    void allreduce_u32(uint32_t* dev, size_t n, hipStream_t s) override {
        if (n) enqueued(rccl().all_reduce(dev, dev, n, ncclUint32, ncclSum, comm_, s), "ncclAllReduce");
    }
    void allgather(const void* dev_send, void* dev_recv, size_t bytes, hipStream_t s) override {
        if (bytes) enqueued(rccl().all_gather(dev_send, dev_recv, bytes, ncclUint8, comm_, s), "ncclAllGather");
    }

  private:
    void enqueued(ncclResult_t r, const char* what) {
        if (r == ncclInProgress) wait(what, comm_timeout_ms("FSM_COMM_TIMEOUT_S"));
        else nccl_check(r, what);
    }
    // poll until the communicator leaves ncclInProgress (abort past limit_ms)
    void wait(const char* what, double limit_ms) {
        const double t0 = now_ms();
        for (int polls = 0;; ) {
            ncclResult_t st = ncclSuccess;
            nccl_check(rccl().comm_get_async_error(comm_, &st), "ncclCommGetAsyncError");
            if (st == ncclSuccess) return;
            if (st != ncclInProgress) {
                (void)rccl().comm_abort(comm_);
                comm_ = nullptr;
                nccl_check(st, what);
            }
            if (now_ms() - t0 > limit_ms) {
                (void)rccl().comm_abort(comm_);
                comm_ = nullptr;
                throw Error(FSM_ECOMM, std::string(what) + ": timed out waiting for the peer ranks "
                                                           "(FSM_COMM_INIT_TIMEOUT_S / FSM_COMM_TIMEOUT_S)");
            }
            // a short spin first (a collective's enqueue normally completes within microseconds),
            // then 100 us sleeps: a rank whose peer died does not burn a core until the limit
            if (++polls > 64) std::this_thread::sleep_for(std::chrono::microseconds(100));
            else std::this_thread::yield();
        }
    }
    // persistent device staging of the host-memory collectives (grown on demand)
    void* staging(size_t bytes) {
        if (stage_.bytes < bytes) stage_.alloc(std::max(bytes, std::max<size_t>(2 * stage_.bytes, size_t(1) << 16)));
        return stage_.p;
    }
    ShmCounters shm_;
    bool shared_ = false;
    ncclComm_t comm_ = nullptr;
    DevBuf stage_;
};

// Host callbacks.  Without a fetch_add callback but with a unique id in fsm_opts, the
// ranks (one node) share the RCCL communicator's shared-memory counters instead: the
// segment is opened before a first all-reduce and unlinked by rank 0 after it.
class HostComm final : public Comm {
  public:
    HostComm(int nranks, int rank, const fsm_host_comm& cb, const uint8_t id[128]) : Comm(nranks, rank), cb_(cb) {
        if (!cb_.allreduce_u32 || !cb_.allgather) throw Error(FSM_EINVAL, "fsm_host_comm: missing callback");
        if (!cb_.fetch_add && id_set(id)) {
            shm_ = std::make_unique<ShmCounters>(id);
            uint32_t one = 1;
            host_allreduce_u32(&one, 1, nullptr);  // every rank has the segment open
            shm_->unlink_name();
            shared_ = counters_shared(*this, *shm_);
        }
    }
    void allreduce_u32(uint32_t* dev, size_t n, hipStream_t s) override {
        std::vector<uint32_t> h(n);
        if (n) FSM_HIP(hipMemcpyAsync(h.data(), dev, n * 4, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
        if (cb_.allreduce_u32(cb_.user, h.data(), int64_t(n)) != 0)
            throw Error(FSM_ECOMM, "host all-reduce callback failed");
        if (n) FSM_HIP(hipMemcpyAsync(dev, h.data(), n * 4, hipMemcpyHostToDevice, s));
        FSM_HIP(hipStreamSynchronize(s));
    }
    void allgather(const void* dev_send, void* dev_recv, size_t bytes, hipStream_t s) override {
        std::vector<uint8_t> snd(bytes), rcv(bytes * size_t(nranks()));
        if (bytes) FSM_HIP(hipMemcpyAsync(snd.data(), dev_send, bytes, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
        if (cb_.allgather(cb_.user, snd.data(), rcv.data(), int64_t(bytes)) != 0)
            throw Error(FSM_ECOMM, "host all-gather callback failed");
        if (bytes) FSM_HIP(hipMemcpyAsync(dev_recv, rcv.data(), rcv.size(), hipMemcpyHostToDevice, s));
        FSM_HIP(hipStreamSynchronize(s));
    }
    void host_allreduce_u32(uint32_t* h, size_t n, hipStream_t) override {
        if (cb_.allreduce_u32(cb_.user, h, int64_t(n)) != 0) throw Error(FSM_ECOMM, "host all-reduce callback failed");
    }
    void host_allgather(const void* send, void* recv, size_t bytes, hipStream_t) override {
        if (cb_.allgather(cb_.user, send, recv, int64_t(bytes)) != 0)
            throw Error(FSM_ECOMM, "host all-gather callback failed");
    }
    bool has_fetch_add() const override { return cb_.fetch_add != nullptr || shared_; }
    int64_t fetch_add(int64_t key, int64_t inc) override {
        if (cb_.fetch_add) return cb_.fetch_add(cb_.user, key, inc);  // (keys are never reused: no reset)
        return shm_ ? shm_->fetch_add(key, inc) : -1;
    }
    void reset_counter(int64_t key) override {
        if (!cb_.fetch_add && shm_ && rank() == 0) shm_->reset(key);
    }

  private:
    fsm_host_comm cb_;
    std::unique_ptr<ShmCounters> shm_;
    bool shared_ = false;
};

}  // namespace

void Comm::host_allreduce_u32(uint32_t* h, size_t n, hipStream_t s) {
    DevBuf d(std::max<size_t>(n, 1) * 4);
    if (n) FSM_HIP(hipMemcpyAsync(d.p, h, n * 4, hipMemcpyHostToDevice, s));
    allreduce_u32(d.as<uint32_t>(), n, s);
    if (n) FSM_HIP(hipMemcpyAsync(h, d.p, n * 4, hipMemcpyDeviceToHost, s));
    FSM_HIP(hipStreamSynchronize(s));
}

void Comm::host_allgather(const void* send, void* recv, size_t bytes, hipStream_t s) {
    DevBuf ds(std::max<size_t>(bytes, 1)), dr(std::max<size_t>(bytes * size_t(nranks()), 1));
    if (bytes) FSM_HIP(hipMemcpyAsync(ds.p, send, bytes, hipMemcpyHostToDevice, s));
    allgather(ds.p, dr.p, bytes, s);
    if (bytes) FSM_HIP(hipMemcpyAsync(recv, dr.p, bytes * size_t(nranks()), hipMemcpyDeviceToHost, s));
    FSM_HIP(hipStreamSynchronize(s));
}

std::vector<uint8_t> Comm::gather_blobs(const std::vector<uint8_t>& mine, std::vector<size_t>& sizes, hipStream_t s,
                                        Agreement* agr, uint32_t* extra, size_t n_extra, bool root_only) {
    const int N = nranks();
    // (lo, hi) u32 halves of each rank's size | 8 failure flags | the caller's extra values
    std::vector<uint32_t> sz(size_t(N) * 2 + 8 + n_extra, 0);
    sz[size_t(rank()) * 2] = uint32_t(mine.size() & 0xFFFFFFFFu);
    sz[size_t(rank()) * 2 + 1] = uint32_t(uint64_t(mine.size()) >> 32);
    if (agr) agr->flags(sz.data() + size_t(N) * 2);
    for (size_t k = 0; k < n_extra; ++k) sz[size_t(N) * 2 + 8 + k] = extra[k];
    host_allreduce_u32(sz.data(), sz.size(), s);
    if (agr) agr->check(sz.data() + size_t(N) * 2);
    for (size_t k = 0; k < n_extra; ++k) extra[k] = sz[size_t(N) * 2 + 8 + k];
    sizes.assign(size_t(N), 0);
    for (int r = 0; r < N; ++r) sizes[size_t(r)] = size_t(sz[size_t(r) * 2]) | (size_t(sz[size_t(r) * 2 + 1]) << 32);
    return gather_var(mine, sizes, s, root_only);
}

std::vector<uint8_t> Comm::gather_var(const std::vector<uint8_t>& mine, const std::vector<size_t>& sizes,
                                      hipStream_t s, bool /*root_only*/) {
    const int N = nranks();
    size_t mx = 0;
    for (size_t v : sizes) mx = std::max(mx, v);
    mx = (mx + 7) & ~size_t(7);
    std::vector<uint8_t> snd(mx, 0), all(mx * size_t(N));
    if (!mine.empty()) std::memcpy(snd.data(), mine.data(), mine.size());
    host_allgather(snd.data(), all.data(), mx, s);
    std::vector<uint8_t> out;
    for (int r = 0; r < N; ++r)
        out.insert(out.end(), all.begin() + ptrdiff_t(size_t(r) * mx), all.begin() + ptrdiff_t(size_t(r) * mx + sizes[size_t(r)]));
    return out;
}

void rccl_unique_id(uint8_t out[128]) {
    ncclUniqueId uid;
    nccl_check(rccl().get_unique_id(&uid), "ncclGetUniqueId");
    std::memcpy(out, uid.internal, 128);
}

double comm_timeout_ms(const char* var) {
    const char* tv = std::getenv(var);
    return 1000.0 * (tv ? std::max(0.1, std::atof(tv)) : 300.0);
}

std::unique_ptr<Comm> make_comm(const fsm_opts& o) {
    if (o.nranks <= 1) return nullptr;
    if (o.rank < 0 || o.rank >= o.nranks) throw Error(FSM_EINVAL, "rank out of range");
    if (o.host_comm) return std::make_unique<HostComm>(o.nranks, o.rank, *o.host_comm, o.unique_id);
    return std::make_unique<RcclComm>(o.nranks, o.rank, o.unique_id);
}

}  // namespace fsm

namespace fsm {

void shard_plan(const uint64_t* volume, int64_t n, int32_t nranks, int32_t* owner) {
    std::vector<int64_t> idx(size_t(std::max<int64_t>(n, 0)));
    for (int64_t i = 0; i < n; ++i) idx[size_t(i)] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return volume[a] > volume[b]; });
    std::vector<uint64_t> load(size_t(nranks), 0);
    for (int64_t i : idx) {
        int32_t best = 0;
        for (int32_t r = 1; r < nranks; ++r)
            if (load[size_t(r)] < load[size_t(best)]) best = r;
        owner[i] = best;
        load[size_t(best)] += volume[i];
    }
}

}  // namespace fsm

namespace fsm {

void Agreement::agree(hipStream_t s) {
    if (!comm) return;
    std::vector<uint32_t> v(8, 0u);
    flags(v.data());
    comm->host_allreduce_u32(v.data(), v.size(), s);
    check(v.data());
}

void Agreement::check(const uint32_t* v) const {
    if (code) throw Error(code, msg);
    for (int c = 1; c < 8; ++c)
        if (v[c])
            throw Error(c, std::string(what) + ": a peer rank failed (FSM error " + std::to_string(c) +
                               "); the sharded mine is aborted on every rank");
}

void maybe_stall(int rank, const char* phase) {
    const char* v = std::getenv("FSM_INJECT_STALL");
    if (!v) return;
    char ph[16] = {0};
    int r = -1;
    double sec = 0;
    if (std::sscanf(v, "%d,%15[^,],%lf", &r, ph, &sec) == 3 && r == rank && !std::strcmp(ph, phase) && sec > 0)
        std::this_thread::sleep_for(std::chrono::duration<double>(sec));
}

void Agreement::maybe_inject(const char* phase) const {
    if (comm) maybe_stall(comm->rank(), phase);
    const char* v = std::getenv("FSM_INJECT_FAIL");
    if (!v || !comm) return;
    char ph[16] = {0};
    int r = -1;
    if (std::sscanf(v, "%d,%15s", &r, ph) == 2 && r == comm->rank() && !std::strcmp(ph, phase))
        throw Error(FSM_ELIMIT, std::string(what) + ": injected failure (FSM_INJECT_FAIL, " + phase + ")");
}

}  // namespace fsm

// ------------------------------------------------------------------ in-process ranks
namespace fsm {

class InProcHub {
  public:
    explicit InProcHub(int n) : n_(n), post_(size_t(n), nullptr) {
        for (auto& c : ctr_) c.store(0);
        for (auto& b : in_bar_) b.store(-1);
    }
    int n() const { return n_; }
    // every rank's pointer of the current exchange (valid between the two barriers)
    void post(int rank, const void* p) { post_[size_t(rank)] = p; }
    const void* posted(int rank) const { return post_[size_t(rank)]; }
    // Generation barrier: a short spin (the ranks usually arrive within microseconds of
    // each other), then a condition-variable wait.  Throws FSM_ECOMM once aborted.
    // the generation a rank waits in (-1: not in a barrier), for the group's hang report
    struct InBar {
        std::atomic<int64_t>& a;
        InBar(std::atomic<int64_t>& x, int64_t v) : a(x) { a.store(v); }
        ~InBar() { a.store(-1); }
    };
    void barrier(int rank) {
        std::unique_lock<std::mutex> g(mu_);
        if (broken_) throw broken_error();
        const uint64_t my = gen_;
        InBar ib(in_bar_[size_t(rank) % in_bar_.size()], int64_t(my));
        if (++arrived_ == n_) {
            arrived_ = 0;
            gen_ = my + 1;
            agen_.store(my + 1, std::memory_order_release);
            g.unlock();
            cv_.notify_all();
            return;
        }
        g.unlock();
        for (int i = 0; i < 4000; ++i) {
            if (agen_.load(std::memory_order_acquire) != my) return;
            if (abroken_.load(std::memory_order_relaxed)) break;
            if (i > 256) std::this_thread::yield();
        }
        g.lock();
        const auto lim = std::chrono::duration<double, std::milli>(comm_timeout_ms("FSM_COMM_TIMEOUT_S"));
        if (!cv_.wait_for(g, lim, [&] { return gen_ != my || broken_; })) {
            // a peer never arrived: break the hub so every other waiter leaves too
            broken_ = true;
            abroken_.store(true);
            g.unlock();
            cv_.notify_all();
            throw Error(FSM_ECOMM, "in-process rank group: rank " + std::to_string(rank) +
                                       " timed out waiting for its peers (FSM_COMM_TIMEOUT_S); the call is aborted");
        }
        if (gen_ == my) throw broken_error();
    }
    void abort() {
        {
            std::lock_guard<std::mutex> g(mu_);
            broken_ = true;
            abroken_.store(true);
        }
        cv_.notify_all();
    }
    bool aborted() {
        std::lock_guard<std::mutex> g(mu_);
        return broken_;
    }
    void reset() {  // every rank has returned from its call
        std::lock_guard<std::mutex> g(mu_);
        broken_ = false;
        abroken_.store(false);
        arrived_ = 0;
    }
    std::atomic<int64_t>& counter(int64_t key) { return ctr_[size_t(key) % kSlots]; }
    std::string state() {
        std::string s = "hub: " + std::to_string(n_) + " ranks, barrier generation " + std::to_string(gen_) + ", " +
                        std::to_string(arrived_) + " arrived, broken " + std::to_string(int(broken_)) + "; in barrier:";
        for (int r = 0; r < n_; ++r) s += " " + std::to_string(in_bar_[size_t(r) % in_bar_.size()].load());
        return s;
    }

  private:
    static Error broken_error() {
        return Error(FSM_ECOMM, "in-process rank group: a peer rank failed; the call is aborted on every rank");
    }
    static constexpr size_t kSlots = 512;
    const int n_;
    std::vector<const void*> post_;
    std::mutex mu_;
    std::condition_variable cv_;
    int arrived_ = 0;
    uint64_t gen_ = 0;
    bool broken_ = false;
    std::atomic<uint64_t> agen_{0};
    std::atomic<bool> abroken_{false};
    std::atomic<int64_t> ctr_[kSlots];
    std::array<std::atomic<int64_t>, 64> in_bar_;
};

namespace {

class InProcComm final : public Comm {
  public:
    InProcComm(std::shared_ptr<InProcHub> hub, int rank) : Comm(hub->n(), rank), hub_(std::move(hub)) {}
    bool has_fetch_add() const override { return true; }
    int64_t fetch_add(int64_t key, int64_t inc) override { return hub_->counter(key).fetch_add(inc); }
    void reset_counter(int64_t key) override {
        // (the collective that follows on every rank orders this before any claim)
        if (rank() == 0) hub_->counter(key).store(0);
    }
    void host_allreduce_u32(uint32_t* h, size_t n, hipStream_t) override {
        std::vector<uint32_t> sum(n, 0u);
        hub_->post(rank(), h);
        hub_->barrier(rank());
        for (int r = 0; r < nranks(); ++r) {
            const auto* v = static_cast<const uint32_t*>(hub_->posted(r));
            for (size_t i = 0; i < n; ++i) sum[i] += v[i];
        }
        hub_->barrier(rank());  // every rank has read every buffer before any is overwritten
        if (n) std::memcpy(h, sum.data(), n * 4);
    }
    void host_allgather(const void* send, void* recv, size_t bytes, hipStream_t) override {
        hub_->post(rank(), send);
        hub_->barrier(rank());
        for (int r = 0; r < nranks(); ++r)
            if (bytes) std::memcpy(static_cast<uint8_t*>(recv) + size_t(r) * bytes, hub_->posted(r), bytes);
        hub_->barrier(rank());
    }
    void allreduce_u32(uint32_t* dev, size_t n, hipStream_t s) override {
        std::vector<uint32_t> h(n);
        if (n) FSM_HIP(hipMemcpyAsync(h.data(), dev, n * 4, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
        host_allreduce_u32(h.data(), n, s);
        if (n) FSM_HIP(hipMemcpyAsync(dev, h.data(), n * 4, hipMemcpyHostToDevice, s));
        FSM_HIP(hipStreamSynchronize(s));
    }
    void allgather(const void* dev_send, void* dev_recv, size_t bytes, hipStream_t s) override {
        std::vector<uint8_t> snd(bytes), rcv(bytes * size_t(nranks()));
        if (bytes) FSM_HIP(hipMemcpyAsync(snd.data(), dev_send, bytes, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
        host_allgather(snd.data(), rcv.data(), bytes, s);
        if (bytes) FSM_HIP(hipMemcpyAsync(dev_recv, rcv.data(), rcv.size(), hipMemcpyHostToDevice, s));
        FSM_HIP(hipStreamSynchronize(s));
    }

  protected:
    // blobs read in place from the posting ranks (no padding); with root_only only rank 0 copies
    std::vector<uint8_t> gather_var(const std::vector<uint8_t>& mine, const std::vector<size_t>& sizes, hipStream_t,
                                    bool root_only) override {
        std::vector<uint8_t> out;
        hub_->post(rank(), mine.data());
        hub_->barrier(rank());
        if (!root_only || rank() == 0) {
            size_t tot = 0;
            for (size_t v : sizes) tot += v;
            out.resize(tot);
            size_t at = 0;
            for (int r = 0; r < nranks(); ++r) {
                if (sizes[size_t(r)]) std::memcpy(out.data() + at, hub_->posted(r), sizes[size_t(r)]);
                at += sizes[size_t(r)];
            }
        }
        hub_->barrier(rank());
        return out;
    }

  private:
    std::shared_ptr<InProcHub> hub_;
};

}  // namespace

std::shared_ptr<InProcHub> make_inproc_hub(int nranks) { return std::make_shared<InProcHub>(nranks); }
std::unique_ptr<Comm> make_inproc_comm(const std::shared_ptr<InProcHub>& hub, int rank) {
    return std::make_unique<InProcComm>(hub, rank);
}
void inproc_abort(InProcHub& hub) { hub.abort(); }
std::string inproc_state(InProcHub& hub) { return hub.state(); }
bool inproc_aborted(InProcHub& hub) { return hub.aborted(); }
void inproc_reset(InProcHub& hub) { hub.reset(); }

}  // namespace fsm
