// device_util.hip — three-phase exclusive scan (tile scan -> scan of tile sums
// -> add), 2048 elements per 256-thread tile, wave64 shuffles + LDS.
#include <cstdlib>
#include <map>
#include <mutex>

#include <cstdio>

#include "device_util.h"

namespace fsm {
namespace {

constexpr int kScanT = 256;
constexpr int kScanV = 8;
constexpr int kScanTile = kScanT * kScanV;

template <class T>
__global__ __launch_bounds__(kScanT) void k_scan_tile(const T* __restrict__ in, uint64_t* __restrict__ out,
                                                      uint64_t* __restrict__ tile_sum, size_t n) {
    __shared__ uint64_t wsum[kScanT / 64];
    const size_t base = size_t(blockIdx.x) * kScanTile + size_t(threadIdx.x) * kScanV;
    uint64_t v[kScanV];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanV; ++k) {
        const size_t i = base + size_t(k);
        v[k] = i < n ? uint64_t(in[i]) : 0ull;
        s += v[k];
    }
    const uint64_t incl = wave_incl_scan(s);
    const unsigned wave = threadIdx.x >> 6;
    if (lane_id() == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t woff = 0;
    for (unsigned w = 0; w < wave; ++w) woff += wsum[w];
    uint64_t run = woff + incl - s;
#pragma unroll
    for (int k = 0; k < kScanV; ++k) {
        const size_t i = base + size_t(k);
        if (i < n) out[i] = run;
        run += v[k];
    }
    if (threadIdx.x == kScanT - 1) tile_sum[blockIdx.x] = woff + incl;
}

__global__ __launch_bounds__(kScanT) void k_scan_add(uint64_t* __restrict__ out, const uint64_t* __restrict__ tile_off,
                                                     size_t n) {
    const uint64_t add = tile_off[blockIdx.x];
    const size_t base = size_t(blockIdx.x) * kScanTile + size_t(threadIdx.x) * kScanV;
#pragma unroll
    for (int k = 0; k < kScanV; ++k) {
        const size_t i = base + size_t(k);
        if (i < n) out[i] += add;
    }
}

template <class T> void scan_impl(const T* in, uint64_t* out, size_t n, hipStream_t s) {
    if (n == 0) {
        FSM_HIP(hipMemsetAsync(out, 0, sizeof(uint64_t), s));
        return;
    }
    const size_t nt = (n + kScanTile - 1) / kScanTile;
    if (nt == 1) {
        hipLaunchKernelGGL(k_scan_tile<T>, dim3(1), dim3(kScanT), 0, s, in, out, out + n, n);
        FSM_LAUNCHED("k_scan_tile", s);
        return;
    }
    DevBuf sums((nt) * sizeof(uint64_t));
    DevBuf offs((nt + 1) * sizeof(uint64_t));
    hipLaunchKernelGGL(k_scan_tile<T>, dim3(unsigned(nt)), dim3(kScanT), 0, s, in, out, sums.as<uint64_t>(), n);
    FSM_LAUNCHED("k_scan_tile", s);
    scan_impl<uint64_t>(sums.as<uint64_t>(), offs.as<uint64_t>(), nt, s);
    hipLaunchKernelGGL(k_scan_add, dim3(unsigned(nt)), dim3(kScanT), 0, s, out, offs.as<uint64_t>(), n);
    FSM_LAUNCHED("k_scan_add", s);
    FSM_HIP(hipMemcpyAsync(out + n, offs.as<uint64_t>() + nt, sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    FSM_HIP(hipStreamSynchronize(s));  // sums/offs are released on return
}

}  // namespace

void scan_exclusive(const uint32_t* in, uint64_t* out, size_t n, hipStream_t s) { scan_impl<uint32_t>(in, out, n, s); }
void scan_exclusive(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s) { scan_impl<uint64_t>(in, out, n, s); }

namespace {
std::mutex g_pool_mu;
std::multimap<size_t, void*>& pool_map() {
    static auto* m = new std::multimap<size_t, void*>();  // leaked on exit on purpose
    return *m;
}
}  // namespace

void* pool_alloc(size_t bytes, size_t* granted) {
    // size classes: powers of two up to 1 MiB, then sz/16 steps
    size_t sz = 4096;
    while (sz < bytes) sz <<= 1;
    if (sz > (size_t(1) << 20)) {
        const size_t step = sz >> 4;  // sz/2 < bytes <= sz: round bytes up to sz/16 steps
        sz = (bytes + step - 1) / step * step;
    }
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        auto& m = pool_map();
        auto it = m.lower_bound(sz);  // smallest cached block that fits, at most 2x larger
        if (it != m.end() && it->first <= 2 * sz) {
            void* p = it->second;
            *granted = it->first;
            m.erase(it);
            return p;
        }
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, sz);
    if (e != hipSuccess) {
        pool_trim();  // give cached blocks back and retry once
        e = hipMalloc(&p, sz);
        if (e != hipSuccess)
            throw Error(FSM_ENOMEM, "hipMalloc(" + std::to_string(sz) + " bytes) failed: " + hipGetErrorString(e));
    }
    *granted = sz;
    return p;
}

void pool_free(void* p, size_t granted) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    pool_map().emplace(granted, p);
}

void pool_trim() {
    std::lock_guard<std::mutex> g(g_pool_mu);
    for (auto& kv : pool_map()) (void)hipFree(kv.second);
    pool_map().clear();
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
    if (idx == recs.size()) recs.push_back(Rec{name, {}, 0});
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

void KernelClock::end(size_t idx, int64_t alg_bytes) {
    FSM_HIP(hipEventRecord(recs[idx].ev.back().second, s));
    recs[idx].bytes += alg_bytes;
}

void KernelClock::finish(std::vector<fsm_kernel_stat>& out) {
    FSM_HIP(hipStreamSynchronize(s));
    out.clear();
    for (auto& r : recs) {
        fsm_kernel_stat k{};
        std::snprintf(k.name, sizeof(k.name), "%s", r.name.c_str());
        k.launches = int64_t(r.ev.size());
        k.alg_bytes = r.bytes;
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
