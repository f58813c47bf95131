// device_util.h — small CDNA4 building blocks shared by the engines:
// wave64 lane masks, a three-phase exclusive scan (u32/u64 -> u64 offsets),
// and eid-mask helpers for W-word masks.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fsm_internal.h"

namespace fsm {

constexpr uint32_t kNone = 0xFFFFFFFFu;

__device__ __forceinline__ unsigned lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint64_t lanemask_lt() {
    const unsigned l = lane_id();
    return l ? (~0ull >> (64u - l)) : 0ull;
}

// inclusive wave64 scan of v
template <class T> __device__ __forceinline__ T wave_incl_scan(T v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (int(lane_id()) >= d) v += o;
    }
    return v;
}

// --- W-word eid masks ----------------------------------------------------
template <int W> struct Mask {
    uint64_t w[W];
};

template <int W> __device__ __forceinline__ void load_mask(const uint64_t* __restrict__ p, uint64_t (&m)[W]) {
    if constexpr (W == 1) {
        m[0] = p[0];
    } else {
#pragma unroll
        for (int k = 0; k < W; k += 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(p + k);
            m[k] = v.x;
            m[k + 1] = v.y;
        }
    }
}

template <int W> __device__ __forceinline__ void store_mask(uint64_t* __restrict__ p, const uint64_t (&m)[W]) {
    if constexpr (W == 1) {
        p[0] = m[0];
    } else {
#pragma unroll
        for (int k = 0; k < W; k += 2) {
            ulonglong2 v;
            v.x = m[k];
            v.y = m[k + 1];
            *reinterpret_cast<ulonglong2*>(p + k) = v;
        }
    }
}

// first / last set bit (mask known non-zero)
template <int W> __device__ __forceinline__ uint32_t mask_lo(const uint64_t (&m)[W]) {
#pragma unroll
    for (int k = 0; k < W; ++k)
        if (m[k]) return uint32_t(k * 64 + __builtin_ctzll(m[k]));
    return 0;
}
template <int W> __device__ __forceinline__ uint32_t mask_hi(const uint64_t (&m)[W]) {
#pragma unroll
    for (int k = W - 1; k >= 0; --k)
        if (m[k]) return uint32_t(k * 64 + 63 - __builtin_clzll(m[k]));
    return 0;
}

// ---------------------------------------------------------------- scans
// exclusive scan in[0..n) -> out[0..n], out[n] = total (u64 offsets)
void scan_exclusive(const uint32_t* in, uint64_t* out, size_t n, hipStream_t s);
void scan_exclusive(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s);

}  // namespace fsm
