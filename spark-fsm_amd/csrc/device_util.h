// device_util.h — small CDNA4 building blocks shared by the engines:
// wave64 lane masks, a single-pass decoupled look-back exclusive scan (u32/u64 -> u64 offsets),
// and eid-mask helpers for W-word masks.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fsm_internal.h"

namespace fsm {

constexpr uint32_t kNone = 0xFFFFFFFFu;

__device__ __forceinline__ unsigned lane_id() { return threadIdx.x & 63u; }

// wave64 ballot of a condition.  HIP's __ballot(int) turns the condition into an int
// first (v_cndmask 0/1, then v_cmp_ne on it: two VALU per ballot on gfx950); the
// builtin takes the i1 and reads the compare's lane mask (SGPR pair) directly.
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

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

// first / last set bit (mask known non-zero).  Branch-free (selects only): an
// earlier early-return form was lowered into divergent branches whose register
// shuffling lost mask words in k_emit<4> (hipcc 7.2, gfx950).
template <int W> __device__ __forceinline__ uint32_t mask_lo(const uint64_t (&m)[W]) {
    uint32_t lo = 0;
#pragma unroll
    for (int k = W - 1; k >= 0; --k) lo = m[k] ? uint32_t(k * 64 + __builtin_ctzll(m[k])) : lo;
    return lo;
}
template <int W> __device__ __forceinline__ uint32_t mask_hi(const uint64_t (&m)[W]) {
    uint32_t hi = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) hi = m[k] ? uint32_t(k * 64 + 63 - __builtin_clzll(m[k])) : hi;
    return hi;
}
// clear every eid <= lo (temporal join: bits strictly after the first bit of L(i))
template <int W> __device__ __forceinline__ void mask_clear_upto(uint64_t (&m)[W], uint32_t lo) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const int sh = int(lo) + 1 - k * 64;  // bits [0, sh) of word k are cleared
        const uint64_t keep = sh <= 0 ? ~0ull : (sh >= 64 ? 0ull : (~0ull << sh));
        m[k] &= keep;
    }
}

// --- runtime-width masks (W == 0: more than 64 words, up to kMaxMaskWords) --
// Sequences with more than 4,096 distinct timestamps take the W = 0 kernel
// instantiations: masks are not held in registers but read from HBM (L1/L2)
// word by word, `wd` words each.  mask_words<W>(wd) is the per-entry stride.
template <int W> __device__ __forceinline__ uint32_t mask_words(uint32_t wd) { return W ? uint32_t(W) : wd; }

// a mask operand: in registers (W > 0) or by address (W == 0)
// load(p, wd, lh) / and_any(b, wd, lh_b): W >= 2 skips the partner's mask when the
// two entries' eid ranges (lohi: first | last set eid << 16) do not overlap
template <int W> struct MaskV {
    uint64_t w[W];
    uint32_t lh = 0;
    __device__ __forceinline__ void load(const uint64_t* __restrict__ p, uint32_t) { load_mask<W>(p, w); }
    __device__ __forceinline__ void load(const uint64_t* __restrict__ p, uint32_t, uint32_t l) {
        lh = l;
        load_mask<W>(p, w);
    }
    __device__ __forceinline__ bool and_any(const uint64_t* __restrict__ b, uint32_t) const {
        uint64_t bm[W];
        load_mask<W>(b, bm);
        uint64_t acc = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) acc |= w[k] & bm[k];
        return acc != 0;
    }
    __device__ __forceinline__ bool and_any(const uint64_t* __restrict__ b, uint32_t wd, uint32_t lb) const {
        if constexpr (W >= 2)
            if (max(lh & 0xFFFFu, lb & 0xFFFFu) > min(lh >> 16, lb >> 16)) return false;
        return and_any(b, wd);
    }
};
template <> struct MaskV<0> {
    const uint64_t* p;
    __device__ __forceinline__ void load(const uint64_t* __restrict__ q, uint32_t) { p = q; }
    __device__ __forceinline__ void load(const uint64_t* __restrict__ q, uint32_t, uint32_t) { p = q; }
    __device__ __forceinline__ bool and_any(const uint64_t* __restrict__ b, uint32_t wd) const {
        for (uint32_t k = 0; k < wd; ++k)
            if (p[k] & b[k]) return true;
        return false;
    }
    __device__ __forceinline__ bool and_any(const uint64_t* __restrict__ b, uint32_t wd, uint32_t) const {
        return and_any(b, wd);
    }
};

// copy src -> dst (wd words), returning first | last set eid << 16 (src non-zero)
__device__ __forceinline__ uint32_t mask_copy_lohi_dyn(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                       uint32_t wd) {
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t k = 0; k < wd; ++k) {
        const uint64_t v = src[k];
        dst[k] = v;
        if (v) {
            if (lo == 0xFFFFFFFFu) lo = k * 64 + uint32_t(__builtin_ctzll(v));
            hi = k * 64 + 63 - uint32_t(__builtin_clzll(v));
        }
    }
    return (lo == 0xFFFFFFFFu ? 0u : lo) | (hi << 16);
}

// ---------------------------------------------------------------- scans
// exclusive scan in[0..n) -> out[0..n], out[n] = total (u64 offsets)
void scan_exclusive(const uint32_t* in, uint64_t* out, size_t n, hipStream_t s);
void scan_exclusive(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s);
// free the scan scratch of a stream that is about to be destroyed
void scan_release(hipStream_t s);

}  // namespace fsm
