// device_util.hip — single-pass exclusive scan (decoupled look-back), the
// device memory pool and kernel timing.
#include <sys/mman.h>

#include <cstdlib>
#include <map>
#include <mutex>

#include <cstdio>

#include "device_util.h"

namespace fsm {
namespace {

// One launch per scan: tiles of 4096 elements are claimed in order through a
// ticket, each wave scans 16 coalesced 64-element chunks of its 1024, the
// block combines its 4 waves in LDS, then thread 0 publishes the tile's
// aggregate and walks back over its predecessors' status words until it meets
// an inclusive prefix (flag and value packed in one u64, so relaxed agent-scope
// atomics are enough).  Ticket order means every tile a block waits on has
// already started, so the walk always ends.  No tile-sum buffers and no host
// synchronisation: the only scratch is the per-stream status array, cleared
// by one memset per scan.
constexpr int kScanT = 256;
constexpr int kScanV = 16;
constexpr int kScanTile = kScanT * kScanV;
constexpr uint64_t kStAgg = uint64_t(1) << 62, kStPre = uint64_t(2) << 62, kStVal = kStAgg - 1;

template <class T>
__global__ __launch_bounds__(kScanT) void k_scan(const T* __restrict__ in, uint64_t* __restrict__ out, size_t n,
                                                 uint32_t* __restrict__ ticket, uint64_t* __restrict__ state) {
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_excl;
    __shared__ uint64_t wsum[kScanT / 64];
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const unsigned lane = lane_id(), wave = threadIdx.x >> 6;
    const size_t wbase = size_t(tile) * kScanTile + size_t(wave) * 64 * kScanV;
    uint64_t r[kScanV];
    uint64_t run = 0;
#pragma unroll
    for (int k = 0; k < kScanV; ++k) {
        const size_t i = wbase + size_t(k) * 64 + lane;
        const uint64_t x = i < n ? uint64_t(in[i]) : 0ull;
        const uint64_t inc = wave_incl_scan(x);
        r[k] = run + inc - x;
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) wsum[wave] = run;
    __syncthreads();
    uint64_t woff = 0, tot = 0;
#pragma unroll
    for (unsigned w = 0; w < kScanT / 64; ++w) {
        woff += w < wave ? wsum[w] : 0ull;
        tot += wsum[w];
    }
    if (threadIdx.x == 0) {
        uint64_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(&state[0], kStPre | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&state[tile], kStAgg | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = int64_t(tile) - 1;
            for (;;) {
                const uint64_t st = __hip_atomic_load(&state[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (st == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += st & kStVal;
                if (st & kStPre) break;
                --j;
            }
            __hip_atomic_store(&state[tile], kStPre | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_excl = excl;
        if ((size_t(tile) + 1) * kScanTile >= n) out[n] = excl + tot;  // the last tile writes the total
    }
    __syncthreads();
    const uint64_t base = s_excl + woff;
#pragma unroll
    for (int k = 0; k < kScanV; ++k) {
        const size_t i = wbase + size_t(k) * 64 + lane;
        if (i < n) out[i] = base + r[k];
    }
}

struct ScanScratch {
    void* p = nullptr;
    size_t bytes = 0;
};
std::mutex g_scan_mu;
std::map<hipStream_t, ScanScratch>& scan_scratch() {
    static auto* m = new std::map<hipStream_t, ScanScratch>();  // leaked on exit on purpose
    return *m;
}

template <class T> void scan_impl(const T* in, uint64_t* out, size_t n, hipStream_t s) {
    if (n == 0) {
        FSM_HIP(hipMemsetAsync(out, 0, sizeof(uint64_t), s));
        return;
    }
    const size_t nt = (n + kScanTile - 1) / kScanTile;
    if (nt >= (size_t(1) << 31)) throw Error(FSM_ELIMIT, "scan: too many elements");
    const size_t need = (nt + 1) * sizeof(uint64_t);  // [ticket | state[nt]]
    void* scr;
    {
        std::lock_guard<std::mutex> g(g_scan_mu);
        ScanScratch& sc = scan_scratch()[s];
        if (sc.bytes < need) {
            if (sc.p) {
                FSM_HIP(hipStreamSynchronize(s));
                FSM_HIP(hipFree(sc.p));
                sc.p = nullptr;
                sc.bytes = 0;
            }
            const size_t want = std::max<size_t>(need, size_t(1) << 16);
            FSM_HIP(hipMalloc(&sc.p, want));
            sc.bytes = want;
        }
        scr = sc.p;
    }
    FSM_HIP(hipMemsetAsync(scr, 0, need, s));
    KernelClock* clk = thread_clock();
    const size_t tk = clk ? clk->begin("k_scan") : 0;
    hipLaunchKernelGGL(k_scan<T>, dim3(unsigned(nt)), dim3(kScanT), 0, s, in, out, n, static_cast<uint32_t*>(scr),
                       static_cast<uint64_t*>(scr) + 1);
    FSM_LAUNCHED("k_scan", s);
    if (clk) clk->end(tk, int64_t(n * (sizeof(T) + 8) + 8));
}

}  // namespace

KernelClock*& thread_clock() {
    thread_local KernelClock* c = nullptr;
    return c;
}

void scan_release(hipStream_t s) {
    std::lock_guard<std::mutex> g(g_scan_mu);
    auto& m = scan_scratch();
    auto it = m.find(s);
    if (it == m.end()) return;
    if (it->second.p) (void)hipFree(it->second.p);
    m.erase(it);
}

void scan_exclusive(const uint32_t* in, uint64_t* out, size_t n, hipStream_t s) { scan_impl<uint32_t>(in, out, n, s); }
void scan_exclusive(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s) { scan_impl<uint64_t>(in, out, n, s); }

Pool::~Pool() { trim(); }

void* Pool::alloc(size_t bytes, size_t* granted) {
    // size classes: powers of two up to 1 MiB, then sz/16 steps
    size_t sz = 4096;
    while (sz < bytes) sz <<= 1;
    if (sz > (size_t(1) << 20)) {
        const size_t step = sz >> 4;  // sz/2 < bytes <= sz: round bytes up to sz/16 steps
        sz = (bytes + step - 1) / step * step;
    }
    {
        std::lock_guard<std::mutex> g(mu_);
        auto it = free_.lower_bound(sz);  // smallest cached block that fits, at most 2x larger
        if (it != free_.end() && it->first <= 2 * sz) {
            void* p = it->second;
            *granted = it->first;
            free_.erase(it);
            return p;
        }
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, sz);
    if (e != hipSuccess) {
        trim();  // give cached blocks back and retry once
        e = hipMalloc(&p, sz);
        if (e != hipSuccess)
            throw Error(FSM_ENOMEM, "hipMalloc(" + std::to_string(sz) + " bytes) failed: " + hipGetErrorString(e));
    }
    *granted = sz;
    return p;
}

void Pool::give(void* p, size_t granted) {
    std::lock_guard<std::mutex> g(mu_);
    free_.emplace(granted, p);
}

void Pool::trim() {
    std::lock_guard<std::mutex> g(mu_);
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    for (auto& kv : free_) (void)hipFree(kv.second);
    free_.clear();
    if (cur >= 0 && cur != device) (void)hipSetDevice(cur);
}

size_t Pool::cached_blocks() {
    std::lock_guard<std::mutex> g(mu_);
    return free_.size();
}

std::shared_ptr<Pool>& thread_pool() {
    thread_local std::shared_ptr<Pool> p;
    return p;
}

std::shared_ptr<Pool> default_pool(int device) {
    static std::mutex mu;
    static auto* pools = new std::map<int, std::shared_ptr<Pool>>();  // leaked on exit on purpose
    std::lock_guard<std::mutex> g(mu);
    std::shared_ptr<Pool>& q = (*pools)[device];
    if (!q) q = std::make_shared<Pool>(device);
    return q;
}

void DevBuf::alloc(size_t n) {
    release();
    std::shared_ptr<Pool> q = thread_pool();
    if (!q) {
        int dev = 0;
        FSM_HIP(hipGetDevice(&dev));
        q = default_pool(dev);
    }
    p = q->alloc(n ? n : 16, &bytes);
    pool = std::move(q);
}

__global__ __launch_bounds__(256) void k_copy_mapped(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16,
                                                    const uint32_t* __restrict__ src4, uint32_t* __restrict__ dst4,
                                                    size_t n4) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    for (size_t i = 4 * n16 + size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) dst4[i] = src4[i];
}

void copy_from_mapped(void* dst, const void* src, size_t bytes, hipStream_t s) {
    const size_t n4 = bytes / 4, n16 = bytes / 16;
    const unsigned grid = unsigned(std::min<size_t>((std::max<size_t>(n16, 1) + 255) / 256, 1024));
    hipLaunchKernelGGL(k_copy_mapped, dim3(grid), dim3(256), 0, s, static_cast<const uint4*>(src),
                       static_cast<uint4*>(dst), n16, static_cast<const uint32_t*>(src), static_cast<uint32_t*>(dst), n4);
    FSM_LAUNCHED("k_copy_mapped", s);
}

// Big host blocks (>= 4 MiB: the member tables, class records and pattern-node chunks of
// deep lattices) are kept after a mine instead of returned to the OS, up to kCacheCap bytes
// per process, and handed to the next mine: a fresh block costs its first touch (the kernel
// zeroes every transparent huge page on its first fault), about a third of SIGN's host time
// (5.9M pattern nodes, hundreds of MB of tables per mine).  Blocks are 2 MiB aligned and
// marked MADV_HUGEPAGE.
#ifndef FSM_BIGBLOCK_MIN_MB
#define FSM_BIGBLOCK_MIN_MB 32
#endif
struct BigBlocks {
    static constexpr size_t kHuge = size_t(2) << 20;
    static constexpr size_t kCacheCap = size_t(1) << 30;
    // below this size glibc's own heap already recycles freed blocks (its mmap threshold
    // rises to 32 MiB after the first free): only larger ones come through the cache
    static constexpr size_t kMin = size_t(FSM_BIGBLOCK_MIN_MB) << 20;
    static BigBlocks& get() {
        static BigBlocks* b = new BigBlocks();  // (leaked on exit on purpose)
        return *b;
    }
    void* take(size_t bytes) {  // bytes: a multiple of kHuge
        if (bytes < kMin) {
            void* q = std::aligned_alloc(kHuge, bytes);
            if (!q) throw std::bad_alloc();
            (void)madvise(q, bytes, MADV_HUGEPAGE);
            return q;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            auto it = free_.lower_bound(bytes);
            if (it != free_.end() && it->first <= 2 * bytes) {
                void* p = it->second;
                const size_t sz = it->first;
                held_ -= sz;
                free_.erase(it);
                sizes_[p] = sz;
                return p;
            }
        }
        void* p = std::aligned_alloc(kHuge, bytes);
        if (!p) throw std::bad_alloc();
        (void)madvise(p, bytes, MADV_HUGEPAGE);
        std::lock_guard<std::mutex> g(mu_);
        sizes_[p] = bytes;
        return p;
    }
    void give(void* p) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = sizes_.find(p);
        const size_t sz = it == sizes_.end() ? 0 : it->second;
        if (it != sizes_.end()) sizes_.erase(it);
        if (sz == 0 || sz > kCacheCap) {
            std::free(p);
            return;
        }
        while (held_ + sz > kCacheCap && !free_.empty()) {  // the largest cached ones go first
            auto last = std::prev(free_.end());
            held_ -= last->first;
            std::free(last->second);
            free_.erase(last);
        }
        free_.emplace(sz, p);
        held_ += sz;
    }

  private:
    std::mutex mu_;
    std::multimap<size_t, void*> free_;
    std::map<void*, size_t> sizes_;  // blocks handed out (their granted size)
    size_t held_ = 0;
};

void* big_take(size_t bytes) { return BigBlocks::get().take(bytes); }
void big_give(void* p) {
    if (p) BigBlocks::get().give(p);
}

bool debug_sync() {
    static const bool on = [] {
        const char* v = std::getenv("FSM_DEBUG_SYNC");
        return v && v[0] == '1';
    }();
    return on;
}

void check_launch(const char* what, hipStream_t s, const char* file, int line) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug_sync()) {
        e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (e != hipSuccess)
        throw Error(FSM_EDEVICE, std::string("kernel ") + what + ": " + hipGetErrorString(e) + " (" + file + ":" +
                                     std::to_string(line) + ")");
}

size_t KernelClock::begin(const char* name) {
    size_t idx = recs.size();
    for (size_t k = 0; k < recs.size(); ++k)
        if (recs[k].name == name) idx = k;
    if (idx == recs.size()) recs.push_back(Rec{name, {}, 0, 0});
    if (!on) return idx;
    hipEvent_t a, b;
    FSM_HIP(hipEventCreate(&a));
    if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        throw Error(FSM_EDEVICE, "hipEventCreate failed");
    }
    recs[idx].ev.push_back({a, b});
    FSM_HIP(hipEventRecord(a, s));
    return idx;
}

void KernelClock::end(size_t idx, int64_t alg_bytes, int64_t survey_bytes) {
    if (on) FSM_HIP(hipEventRecord(recs[idx].ev.back().second, s));
    recs[idx].bytes += alg_bytes;
    recs[idx].survey += survey_bytes;
}

void KernelClock::finish(std::vector<fsm_kernel_stat>& out) {
    FSM_HIP(hipStreamSynchronize(s));
    out.clear();
    for (auto& r : recs) {
        fsm_kernel_stat k{};
        std::snprintf(k.name, sizeof(k.name), "%s", r.name.c_str());
        k.launches = int64_t(r.ev.size());
        k.alg_bytes = r.bytes;
        k.survey_bytes = r.survey;
        for (auto& e : r.ev) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) k.ms += ms;
        }
        out.push_back(k);
    }
    release();
}

void KernelClock::release() {
    for (auto& r : recs)
        for (auto& e : r.ev) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
    recs.clear();
}

}  // namespace fsm
