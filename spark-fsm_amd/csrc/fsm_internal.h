// fsm_internal.h — shared host-side types of libfsm (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/fsm.h"

namespace fsm {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define FSM_HIP(x)                                                                        \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess)                                                             \
            throw ::fsm::Error(FSM_EDEVICE, std::string(#x) + " failed: " + hipGetErrorString(e_) + \
                                                " (" __FILE__ ":" + std::to_string(__LINE__) + ")"); \
    } while (0)

// After every kernel launch: report launch errors with the kernel's name; with
// FSM_DEBUG_SYNC=1 in the environment also synchronize to localize device faults.
bool debug_sync();
void check_launch(const char* what, hipStream_t s, const char* file, int line);
#define FSM_LAUNCHED(name, stream) ::fsm::check_launch(name, stream, __FILE__, __LINE__)

// eid-mask words per SPADE entry at most: 65,536 distinct timestamps per sequence
// (the first / last eid of an entry are 16-bit fields of the slab's lohi word)
constexpr uint32_t kMaxMaskWords = 1024;

inline double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// Per-kernel timing with HIP events on one stream: begin() before a launch,
// end() after it with the launch's algorithmic bytes; finish() folds the
// events into fsm_kernel_stat rows (summed per kernel name).
struct KernelClock {
    struct Rec {
        std::string name;
        std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
        int64_t bytes = 0;
        int64_t survey = 0;  // SURVEY §8(d) bytes (fsm_kernel_stat.survey_bytes)
    };
    hipStream_t s = nullptr;
    std::vector<Rec> recs;
    // FSM_KCLOCK=0 (read per mine): no events around the launches.  Each timed launch costs
    // two event records on the stream (about 0.15 ms of a 5 ms D1M mine), so bench.py times
    // its steps without them and takes the kernel times from an instrumented warmup mine
    bool on = true;
    explicit KernelClock(hipStream_t st) : s(st) {
        const char* v = std::getenv("FSM_KCLOCK");
        on = !(v && v[0] == '0');
    }
    KernelClock(const KernelClock&) = delete;
    KernelClock& operator=(const KernelClock&) = delete;
    ~KernelClock() { release(); }
    size_t begin(const char* name);
    void end(size_t idx, int64_t alg_bytes, int64_t survey_bytes = 0);
    void add_bytes(size_t idx, int64_t alg_bytes, int64_t survey_bytes = 0) {  // known after a later sync
        recs[idx].bytes += alg_bytes;
        recs[idx].survey += survey_bytes;
    }
    void finish(std::vector<fsm_kernel_stat>& out);
    void release();
};

// The clock of the mine call running on this thread: library-internal kernels
// launched from shared helpers (the scan) record into it when it is set.
KernelClock*& thread_clock();
struct ClockScope {
    KernelClock* prev;
    explicit ClockScope(KernelClock* c) : prev(thread_clock()) { thread_clock() = c; }
    ~ClockScope() { thread_clock() = prev; }
    ClockScope(const ClockScope&) = delete;
    ClockScope& operator=(const ClockScope&) = delete;
};

// Device memory pool: hipMalloc/hipFree synchronize and cost milliseconds for
// the multi-hundred-MB frontier slabs, so freed blocks are cached per size
// class (power of two >= 4 KiB) and reused by later batches and later calls.
// One pool per context (its device and its one stream): a block released while
// kernels queued on that stream may still read it is only ever handed out
// again to later work on the same stream, so stream order keeps it safe, and
// blocks never cross devices or contexts.  The pool is shared-owned by every
// block it handed out, so DBs may outlive their context's destroy call.
struct Pool {
    explicit Pool(int dev) : device(dev) {}
    ~Pool();
    Pool(const Pool&) = delete;
    Pool& operator=(const Pool&) = delete;
    void* alloc(size_t bytes, size_t* granted);
    void give(void* p, size_t granted);
    void trim();  // hipFree every cached block
    size_t cached_blocks();
    const int device;

  private:
    std::mutex mu_;
    std::multimap<size_t, void*> free_;
};
// The pool of the context whose API call runs on this thread (set by the
// entry points through PoolScope); outside any call, a per-device default.
std::shared_ptr<Pool>& thread_pool();
std::shared_ptr<Pool> default_pool(int device);
struct PoolScope {
    std::shared_ptr<Pool> prev;
    explicit PoolScope(std::shared_ptr<Pool> p) : prev(thread_pool()) { thread_pool() = std::move(p); }
    ~PoolScope() { thread_pool() = std::move(prev); }
    PoolScope(const PoolScope&) = delete;
    PoolScope& operator=(const PoolScope&) = delete;
};

// dst (device) <- src (a mapped pinned host pointer's device address), `bytes` a multiple of 4:
// a copy kernel on stream s (device_util.hip)
void copy_from_mapped(void* dst, const void* src, size_t bytes, hipStream_t s);

// Big host blocks (device_util.hip): 2 MiB aligned, MADV_HUGEPAGE; blocks of 32 MiB and more
// are cached across mines (1 GiB per process) instead of returned to the OS.  big_take(bytes):
// bytes a multiple of kHugeBlock; big_give(p): any pointer from big_take or malloc (freed then)
constexpr size_t kHugeBlock = size_t(2) << 20;
void* big_take(size_t bytes);
void big_give(void* p);

// Mapped pinned host memory (kernels write results straight into it; the host
// reads them after a stream sync, with no copy launch).
struct PinnedBuf {
    void* host = nullptr;
    void* dev = nullptr;
    explicit PinnedBuf(size_t bytes) {
        if (hipHostMalloc(&host, bytes ? bytes : 16, hipHostMallocMapped) != hipSuccess)
            throw Error(FSM_ENOMEM, "hipHostMalloc failed");
        if (hipHostGetDevicePointer(&dev, host, 0) != hipSuccess) {
            (void)hipHostFree(host);
            throw Error(FSM_EDEVICE, "hipHostGetDevicePointer failed");
        }
    }
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { (void)hipHostFree(host); }
};

// Owning device allocation from the current pool, RAII.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    std::shared_ptr<Pool> pool;
    DevBuf() = default;
    explicit DevBuf(size_t n) { alloc(n); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes), pool(std::move(o.pool)) { o.p = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            p = o.p;
            bytes = o.bytes;
            pool = std::move(o.pool);
            o.p = nullptr;
            o.bytes = 0;
        }
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t n);
    void release() {
        if (p) pool->give(p, bytes);
        p = nullptr;
        bytes = 0;
        pool.reset();
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// ---------------------------------------------------------------- flat DBs
// SPADE: one row per distinct sequence id (records with equal sids merged, as
// IDListBitmap.registerBit(sid, ts) merges them, SPADE.scala:74,90); entries
// are the distinct items of the row (ascending dense id) with the bitmask of
// the row's rank-compressed timestamps (eids) at which they occur.
struct FlatSpade {
    int64_t total = 0;                 // input records = sequences.count()
    int W = 1;                         // u64 words per eid mask (power of two)
    int64_t max_occ = 0;               // max (item, eid) occurrences in one row = longest pattern
    std::vector<int32_t> item_val;     // dense item id -> item value (ascending)
    std::vector<uint32_t> row_off;     // [rows+1]
    std::vector<uint32_t> ent_item;    // dense item id
    std::vector<uint64_t> ent_mask;    // [entries * W]
};

// TSR: one row per sequence (sid == position), entries = distinct items with
// their first / last itemset index (the Vertical maps, TSR.scala:52-94).
struct FlatTsr {
    int64_t total = 0;
    std::vector<int32_t> item_val;
    std::vector<uint32_t> row_off;     // [total+1]
    std::vector<uint32_t> ent_item;
    std::vector<uint32_t> ent_first;
    std::vector<uint32_t> ent_last;
};

struct Source {
    // exactly one of (lines, tokens) is set
    const int32_t* sids = nullptr;
    const char* const* lines = nullptr;
    const int64_t* lens = nullptr;
    const int64_t* seq_off = nullptr;
    const int64_t* tokens = nullptr;
    int64_t n = 0;
};

// the message fsm_last_error(NULL) returns (context-free entry points)
void set_thread_error(const std::string& msg);

void flatten_spade(const Source& src, FlatSpade& out);
void flatten_tsr(const Source& src, FlatTsr& out);

}  // namespace fsm

struct SpadeDevDB;
struct TsrDevDB;
namespace fsm {
class Comm;
struct Group;
}

struct fsm_ctx {
    fsm_opts opts{};
    std::string err;
    fsm_stats stats{};
    hipStream_t stream = nullptr;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    fsm::Comm* comm = nullptr;  // nranks > 1 (owned)
    // fsm_opts.ndevices > 1: the rank contexts this context drives in-process (fsm_api.cpp)
    std::unique_ptr<fsm::Group> group;
    bool result_root_only = false;  // a rank context of a group: only rank 0's result is returned
    int dev_share = 1;  // rank contexts of this group on the same device: default budgets are split
    std::shared_ptr<fsm::Pool> pool;  // device blocks of this context (see fsm::Pool)
    std::vector<fsm_kernel_stat> kstats;  // of the last mine call
    std::unique_ptr<fsm::PinnedBuf> pin;  // small mapped readback slots, made on first use
    uint64_t* pinned_u64() {              // 16 u64 slots of pinned host memory
        if (!pin) pin = std::make_unique<fsm::PinnedBuf>(128);
        return static_cast<uint64_t*>(pin->host);
    }
    // mapped pinned host memory of at least `bytes` (kernels write results straight into it);
    // grown on demand, kept for the context's lifetime
    std::unique_ptr<fsm::PinnedBuf> pin_big;
    size_t pin_big_bytes = 0;
    fsm::PinnedBuf* pinned_big(size_t bytes) {
        if (!pin_big || pin_big_bytes < bytes) {
            const size_t nb = std::max<size_t>(bytes, std::max<size_t>(2 * pin_big_bytes, size_t(1) << 20));
            pin_big.reset();
            pin_big = std::make_unique<fsm::PinnedBuf>(nb);
            pin_big_bytes = nb;
        }
        return pin_big.get();
    }
    // H2D staging slots (pinned, grown on demand, kept for the context's lifetime): a
    // slot is rewritten only after the copy that last read it has completed (its event)
    static constexpr int kStageSlots = 4;
    std::unique_ptr<fsm::PinnedBuf> stage[kStageSlots];
    size_t stage_bytes[kStageSlots] = {0, 0, 0, 0};
    hipEvent_t stage_ev[kStageSlots] = {nullptr, nullptr, nullptr, nullptr};
    bool stage_pending[kStageSlots] = {false, false, false, false};
    void* stage_host(int i, size_t bytes) {
        if (stage_pending[i]) {
            FSM_HIP(hipEventSynchronize(stage_ev[i]));
            stage_pending[i] = false;
        }
        if (!stage[i] || stage_bytes[i] < bytes) {
            const size_t nb = std::max<size_t>(bytes, std::max<size_t>(2 * stage_bytes[i], size_t(1) << 20));
            stage[i].reset();
            stage[i] = std::make_unique<fsm::PinnedBuf>(nb);
            stage_bytes[i] = nb;
        }
        return stage[i]->host;
    }
    // Async H2D of the slot's first `bytes`.  Up to kStageKernelMax bytes (a multiple of 4) go
    // through a copy kernel on the stream that reads the mapped slot over PCIe: an SDMA copy
    // costs the next kernel a cross-engine wait of about 20 us (the gaps after every small
    // upload in the D1M kernel timeline), a kernel on the same queue none.
    static constexpr size_t kStageKernelMax = size_t(2) << 20;
    void stage_copy(int i, void* dst, size_t bytes) {
        if (!bytes) return;
        if (!stage_ev[i]) FSM_HIP(hipEventCreateWithFlags(&stage_ev[i], hipEventDisableTiming));
        if (bytes <= kStageKernelMax && bytes % 4 == 0) fsm::copy_from_mapped(dst, stage[i]->dev, bytes, stream);
        else FSM_HIP(hipMemcpyAsync(dst, stage[i]->host, bytes, hipMemcpyHostToDevice, stream));
        FSM_HIP(hipEventRecord(stage_ev[i], stream));
        stage_pending[i] = true;
    }
};

struct fsm_db {
    fsm_ctx* ctx = nullptr;
    int mode = 0;
    std::vector<fsm_db*> parts;  // a group context's DB: one replica per rank context (owned)
    std::shared_ptr<std::atomic<bool>> group_stuck;  // the group's stalled-rank flag (group DBs)
    fsm::FlatSpade spade;
    fsm::FlatTsr tsr;
    SpadeDevDB* spade_dev = nullptr;
    TsrDevDB* tsr_dev = nullptr;
};

namespace fsm {
// engines (spade_engine.hip / tsr_engine.hip)
void spade_upload(fsm_ctx* ctx, fsm_db* db);
void spade_release(fsm_db* db);
void spade_mine(fsm_ctx* ctx, fsm_db* db, double support, fsm_patterns** out);
void tsr_upload(fsm_ctx* ctx, fsm_db* db);
void tsr_release(fsm_db* db);
void tsr_mine(fsm_ctx* ctx, fsm_db* db, int32_t k, double minconf, fsm_rules** out);
// FSM_HOST_PROF=<file>: SIGPROF sampling of the host side of a mine (host_prof.cpp)
bool host_prof_start();
void host_prof_stop();
}  // namespace fsm
