// k0_build.hip — K0: the vertical DB built on the GPU from the
// token stream of fsm_db_from_tokens, in place of the host flatten for that
// path.  It restates, per sequence:
//   SPADE  SPADE.scala:53-106 (registerBit(sid, timestamp) of every item of a
//          closed itemset; implicit timestamps 1, 2, 3 ...; rank-compressed
//          to eids = rank among the row's non-empty closed itemsets) and
//          SPADE.newSequence's token rules (:151-210: -1 closes an itemset,
//          -2 is ignored, items after the last -1 are dropped);
//   TSR    TSR.scala:52-94 (first / last itemset index of each item, the
//          index counting every -1) with TSR.newSequence (:109-143).
// The output is byte-for-byte the host flatten's (flatten.cpp), which stays
// the path for text input and for the inputs this builder declines (sids not
// strictly increasing, rows of more than 8192 tokens, item ranges over 2^27,
// and every input the reference rejects, so the host reports the exact error).
//
//   staging       the int64 token stream narrowed to int32 on host threads into
//                 pinned double-buffered chunks (DMA of one chunk overlaps the
//                 narrowing of the next), with the item-value range, the int32
//                 range check and TSR item presence computed on the way
//   k0_rows       one wave per row of <= 64 tokens, pass 1 (count) and pass 2
//                 (write): itemset index by ballot prefix counts, eids, the
//                 (value, eid) pairs sorted across the wave (bitonic, shuffles),
//                 equal items merged by a segmented OR (SPADE) or head / tail
//                 lanes (TSR first / last), written at the row's scan offset;
//                 pass 1 marks item presence in an LDS-privatized value bitmap
//   k0_long       the same for rows of 65..8192 tokens: one block per row,
//                 block scans and a bitonic sort in LDS
//   dictionary    presence bitmap -> word popcount scan -> dense ids (rank of
//                 the value) and the ascending value table
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "dev_db.h"
#include "device_util.h"
#include "host_pool.h"

namespace fsm {
namespace {

constexpr uint32_t kK0Wave = 64;         // tokens of a row for the wave path
constexpr uint32_t kK0Long = 8192;       // tokens of a row for the block path
constexpr uint32_t kK0LongThreads = 256;
constexpr uint32_t kK0Threads = 1024;    // k0_rows block (16 waves)
constexpr uint32_t kK0LdsWords = 16384;  // presence bitmap privatized in LDS up to 2^19 values
constexpr int kSpade = 0, kTsr = 1;

struct K0Stats {       // device-side maxima / flags of pass 1
    uint32_t max_eids;  // SPADE: non-empty closed itemsets of a row (mask width)
    uint32_t max_occ;   // SPADE: closed item tokens of a row (longest pattern)
    uint32_t neg_item;  // TSR: a closed item < 0 (the reference throws)
    uint32_t pad;
};
struct K0Range {
    int32_t vmin, vmax;  // over item tokens (not -1 / -2)
    uint32_t bad;        // a token outside int32
    uint32_t any_nonneg; // TSR: some token > -1 (TSR.scala:41-43 needs one)
};

__device__ __forceinline__ uint64_t lanemask_le() {
    const unsigned l = lane_id();
    return l == 63 ? ~0ull : ((2ull << l) - 1ull);
}

// dense id of an item value: its rank among the present values
__device__ __forceinline__ uint32_t value_rank(int32_t v, int32_t vmin, const uint32_t* __restrict__ bm,
                                               const uint64_t* __restrict__ wpre) {
    const uint32_t b = uint32_t(int64_t(v) - vmin), w = b >> 5;
    return uint32_t(wpre[w]) + uint32_t(__popc(bm[w] & ((1u << (b & 31u)) - 1u)));
}

struct K0Out {  // pass 2 destinations
    uint32_t* item;
    uint64_t* mask;   // SPADE [E * W]
    uint32_t* first;  // TSR
    uint32_t* last;
    const uint64_t* off;  // row entry offsets (scan of pass 1 counts)
    const uint32_t* bm;   // presence bitmap
    const uint64_t* wpre; // word popcount prefix
    int W;
};

// One wave, one row of L <= 64 tokens.
template <int kMode, bool kWrite>
__device__ __forceinline__ void k0_wave_row(const int32_t* __restrict__ tok, uint64_t t0, uint32_t L, uint32_t r,
                                            int32_t vmin, uint32_t* __restrict__ cnt, uint32_t* lbm, uint32_t* gbm,
                                            K0Stats& st, const K0Out& o) {
    const uint32_t lane = lane_id();
    const uint64_t lt = lanemask_lt();
    const bool valid = lane < L;
    const int64_t v64 = valid ? tok[t0 + lane] : -2;
    const int32_t v = int32_t(v64);
    const bool sep = v64 == -1, itm = valid && v64 != -1 && v64 != -2;
    const uint64_t sepb = ballot(sep), itb = ballot(itm);
    const uint32_t k = uint32_t(__popcll(sepb & lt));  // itemset index
    const uint32_t nsep = uint32_t(__popcll(sepb));
    const bool closed = itm && k < nsep;  // items after the last -1 are dropped
    uint32_t pay = k;                     // TSR: the itemset index
    uint32_t neids = 0;
    if (kMode == kSpade) {
        // a -1 at lane p closes a non-empty itemset iff an item lies between it and the previous -1
        const uint64_t prev = sepb & lt;
        const uint64_t after_prev = prev ? ~((2ull << (63 - __clzll(prev))) - 1ull) : ~0ull;
        const bool ne = sep && (itb & lt & after_prev) != 0ull;
        const uint64_t neb = ballot(ne);
        pay = uint32_t(__popcll(neb & lt));  // eid: non-empty closed itemsets before this item
        neids = uint32_t(__popcll(neb));
    }
    uint64_t key = closed ? ((uint64_t(uint32_t(v) ^ 0x80000000u) << 32) | pay) : ~0ull;
    // bitonic sort of the 64 keys, ascending by lane
#pragma unroll
    for (uint32_t kk = 2; kk <= 64; kk <<= 1) {
#pragma unroll
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            const uint64_t o2 = __shfl_xor(key, int(j), 64);
            const bool up = (lane & kk) == 0, lower = (lane & j) == 0;
            key = (lower == up) ? min(key, o2) : max(key, o2);
        }
    }
    const bool vk = key != ~0ull;
    const uint32_t hv = uint32_t(key >> 32);  // value ^ sign, ascending
    const uint32_t pk = uint32_t(key);
    const uint32_t hv_prev = uint32_t(__shfl_up(int(hv), 1, 64));
    const uint32_t hv_next = uint32_t(__shfl_down(int(hv), 1, 64));
    const bool vk_next = __shfl_down(int(vk), 1, 64) != 0 && lane < 63;
    const bool head = vk && (lane == 0 || hv_prev != hv);
    const bool tail = vk && (!vk_next || hv_next != hv);
    const uint64_t headb = ballot(head);
    const uint32_t nent = uint32_t(__popcll(headb));
    const int32_t val = int32_t(hv ^ 0x80000000u);
    if (!kWrite) {
        if (lane == 0) cnt[r] = nent;
        if (kMode == kSpade) {
            st.max_eids = max(st.max_eids, neids);
            st.max_occ = max(st.max_occ, uint32_t(__popcll(ballot(closed))));
        } else if (ballot(head && val < 0)) {
            st.neg_item = 1;
        }
        if (head) {
            const uint32_t b = uint32_t(int64_t(val) - vmin);
            atomicOr(lbm ? &lbm[b >> 5] : &gbm[b >> 5], 1u << (b & 31u));
        }
        return;
    }
    // head lane of each lane's segment, entry index of the segment
    const uint64_t hle = headb & lanemask_le();
    const uint32_t hl = hle ? 63u - uint32_t(__clzll(hle)) : 0u;
    const uint32_t idx = uint32_t(__popcll(hle)) - 1u;
    const uint64_t off = o.off[r];
    if (kMode == kSpade) {
        uint64_t m = vk ? (1ull << pk) : 0ull;  // pk < 64: <= 32 itemsets in 64 tokens
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t om = __shfl_up(m, int(d), 64);
            if (lane >= d && lane - d >= hl) m |= om;
        }
        if (tail) {
            const uint64_t e = off + idx;
            o.item[e] = value_rank(val, vmin, o.bm, o.wpre);
            o.mask[e * uint64_t(o.W)] = m;
            for (int w = 1; w < o.W; ++w) o.mask[e * uint64_t(o.W) + uint64_t(w)] = 0ull;
        }
    } else {
        const uint32_t first = uint32_t(__shfl(int(pk), int(hl), 64));
        if (tail) {
            const uint64_t e = off + idx;
            o.item[e] = value_rank(val, vmin, o.bm, o.wpre);
            o.first[e] = first;
            o.last[e] = pk;
        }
    }
}

// Rows of <= 64 tokens, one wave each (grid-stride over waves); rows of more
// are left to k0_long.  Pass 1 keeps the presence bitmap in LDS when it fits.
template <int kMode, bool kWrite>
__global__ __launch_bounds__(kK0Threads) void k0_rows(const uint64_t* __restrict__ so, uint32_t n,
                                                      const int32_t* __restrict__ tok, int32_t vmin, uint32_t nw,
                                                      uint32_t* __restrict__ cnt, uint32_t* __restrict__ gbm,
                                                      K0Stats* __restrict__ gst, K0Out o) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lbm_s[];
    uint32_t* lbm = nullptr;
    const bool use_lds = !kWrite && nw <= kK0LdsWords;
    if (use_lds) {
        lbm = lbm_s;
        for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) lbm[w] = 0;
        __syncthreads();
    }
    K0Stats st{0, 0, 0, 0};
    const uint32_t wstride = (gridDim.x * blockDim.x) >> 6;
    const uint64_t base = so[0];
    for (uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += wstride) {
        const uint64_t t0 = so[r] - base, L = so[r + 1] - so[r];
        if (L > kK0Wave) continue;  // k0_long
        k0_wave_row<kMode, kWrite>(tok, t0, uint32_t(L), r, vmin, cnt, lbm, gbm, st, o);
    }
    if (!kWrite) {
        if (lane_id() == 0) {
            if (st.max_eids) atomicMax(&gst->max_eids, st.max_eids);
            if (st.max_occ) atomicMax(&gst->max_occ, st.max_occ);
            if (st.neg_item) atomicOr(&gst->neg_item, 1u);
        }
        if (use_lds) {
            __syncthreads();
            for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x)
                if (lbm[w]) atomicOr(&gbm[w], lbm[w]);
        }
    }
}

// exclusive scan of a[0..n) in LDS by one block (n <= kK0Long), returns the total
__device__ uint32_t block_excl_scan(uint32_t* a, uint32_t n, uint32_t* wtot) {
    constexpr uint32_t per = kK0Long / kK0LongThreads;  // 32 consecutive elements per thread
    const uint32_t t = threadIdx.x, b = t * per;
    uint32_t s = 0;
    for (uint32_t q = 0; q < per; ++q) s += b + q < n ? a[b + q] : 0u;
    const uint32_t incl = wave_incl_scan(s);
    if (lane_id() == 63) wtot[t >> 6] = incl;
    __syncthreads();
    uint32_t woff = 0, total = 0;
    for (uint32_t w = 0; w < kK0LongThreads / 64; ++w) {
        woff += w < (t >> 6) ? wtot[w] : 0u;
        total += wtot[w];
    }
    uint32_t run = woff + incl - s;
    for (uint32_t q = 0; q < per; ++q)
        if (b + q < n) {
            const uint32_t x = a[b + q];
            a[b + q] = run;
            run += x;
        }
    __syncthreads();
    return total;
}

// One block per row of 65..8192 tokens (rows listed by the host).
template <int kMode, bool kWrite>
__global__ __launch_bounds__(kK0LongThreads) void k0_long(const uint32_t* __restrict__ rows, const uint64_t* __restrict__ so,
                                                          const int32_t* __restrict__ tok, int32_t vmin,
                                                          uint32_t* __restrict__ cnt, uint32_t* __restrict__ gbm,
                                                          K0Stats* __restrict__ gst, K0Out o) {
    __shared__ uint64_t key[kK0Long];  // the tokens, then (in place) the pairs' sort keys
    __shared__ uint32_t a[kK0Long];    // token flags / prefix counts, later the entry index of each sorted pair
    __shared__ uint32_t b2[kK0Long];   // per itemset: non-empty flag -> eid
    __shared__ uint32_t wtot[kK0LongThreads / 64];
    __shared__ uint32_t s_red[3];
    const uint32_t r = rows[blockIdx.x];
    const uint64_t t0 = so[r] - so[0];
    const uint32_t L = uint32_t(so[r + 1] - so[r]);
    const uint32_t tid = threadIdx.x;
    for (uint32_t t = tid; t < L; t += blockDim.x) {
        const int64_t v = tok[t0 + t];
        key[t] = uint64_t(v);
        a[t] = v == -1 ? 1u : 0u;
    }
    if (tid < 3) s_red[tid] = 0;
    __syncthreads();
    const uint32_t nsep = block_excl_scan(a, L, wtot);  // a[t] = itemset index of token t
    uint32_t neids = 0;
    if (kMode == kSpade) {
        for (uint32_t q = tid; q < nsep; q += blockDim.x) b2[q] = 0;
        __syncthreads();
        for (uint32_t t = tid; t < L; t += blockDim.x) {
            const int64_t v = int64_t(key[t]);
            if (v != -1 && v != -2 && a[t] < nsep) b2[a[t]] = 1u;  // itemset a[t] is non-empty
        }
        __syncthreads();
        neids = block_excl_scan(b2, nsep, wtot);  // b2[k] = eid of itemset k
    }
    // pairs of closed items, padded to a power of two with the sentinel
    uint32_t P = 1;
    while (P < L) P <<= 1;
    uint32_t occ = 0;
    for (uint32_t t = tid; t < P; t += blockDim.x) {
        uint64_t kv = ~0ull;
        const int64_t v = t < L ? int64_t(key[t]) : -2;
        if (v != -1 && v != -2 && a[t] < nsep) {
            const uint32_t pay = kMode == kSpade ? b2[a[t]] : a[t];
            kv = (uint64_t(uint32_t(int32_t(v)) ^ 0x80000000u) << 32) | pay;
            ++occ;
        }
        key[t] = kv;
    }
    __syncthreads();
    for (uint32_t kk = 2; kk <= P; kk <<= 1)
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t t = tid; t < P; t += blockDim.x) {
                const uint32_t u = t ^ j;
                if (u > t) {
                    const uint64_t x = key[t], y = key[u];
                    const bool up = (t & kk) == 0;
                    if ((x > y) == up) {
                        key[t] = y;
                        key[u] = x;
                    }
                }
            }
            __syncthreads();
        }
    // segment heads -> entry index of every pair
    for (uint32_t t = tid; t < L; t += blockDim.x)
        a[t] = key[t] != ~0ull && (t == 0 || (key[t - 1] >> 32) != (key[t] >> 32)) ? 1u : 0u;
    __syncthreads();
    const uint32_t nent = block_excl_scan(a, L, wtot);  // a[t] = index of the first head at or after t
    if (!kWrite) {
        uint32_t neg = 0;
        for (uint32_t t = tid; t < L; t += blockDim.x) {
            const uint64_t kv = key[t];
            if (kv == ~0ull || (t > 0 && (key[t - 1] >> 32) == (kv >> 32))) continue;  // heads only
            const int32_t val = int32_t(uint32_t(kv >> 32) ^ 0x80000000u);
            neg |= val < 0 ? 1u : 0u;
            const uint32_t b = uint32_t(int64_t(val) - vmin);
            atomicOr(&gbm[b >> 5], 1u << (b & 31u));
        }
        atomicAdd(&s_red[0], occ);
        if (neg) atomicOr(&s_red[1], 1u);
        __syncthreads();
        if (tid == 0) {
            cnt[r] = nent;
            if (kMode == kSpade) {
                atomicMax(&gst->max_eids, neids);
                atomicMax(&gst->max_occ, s_red[0]);
            } else if (s_red[1]) {
                atomicOr(&gst->neg_item, 1u);
            }
        }
        return;
    }
    const uint64_t off = o.off[r];
    if (kMode == kSpade) {
        const uint32_t W = uint32_t(o.W);  // the mask words were zeroed by a memset before this pass
        for (uint32_t t = tid; t < L; t += blockDim.x) {
            const uint64_t kv = key[t];
            if (kv == ~0ull) continue;
            const bool hd = t == 0 || (key[t - 1] >> 32) != (kv >> 32);
            const uint32_t e = hd ? a[t] : a[t] - 1;  // a[t] counts heads before t
            const uint32_t pay = uint32_t(kv);
            atomicOr(reinterpret_cast<unsigned long long*>(&o.mask[(off + e) * W + (pay >> 6)]),
                     (unsigned long long)(1ull << (pay & 63u)));
            if (hd) o.item[off + e] = value_rank(int32_t(uint32_t(kv >> 32) ^ 0x80000000u), vmin, o.bm, o.wpre);
        }
    } else {
        for (uint32_t t = tid; t < L; t += blockDim.x) {
            const uint64_t kv = key[t];
            if (kv == ~0ull) continue;
            const bool hd = t == 0 || (key[t - 1] >> 32) != (kv >> 32);
            const bool tl = t + 1 == L || key[t + 1] == ~0ull || (key[t + 1] >> 32) != (kv >> 32);
            const uint32_t e = hd ? a[t] : a[t] - 1;
            if (hd) {
                o.item[off + e] = value_rank(int32_t(uint32_t(kv >> 32) ^ 0x80000000u), vmin, o.bm, o.wpre);
                o.first[off + e] = uint32_t(kv);
            }
            if (tl) o.last[off + e] = uint32_t(kv);
        }
    }
}

__global__ __launch_bounds__(256) void k0_popc(const uint32_t* __restrict__ bm, uint32_t nw, uint32_t* __restrict__ pc) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x)
        pc[w] = uint32_t(__popc(bm[w]));
}

__global__ __launch_bounds__(256) void k0_values(const uint32_t* __restrict__ bm, const uint64_t* __restrict__ wpre,
                                                 uint32_t nw, int32_t vmin, int32_t* __restrict__ ival) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
        uint32_t x = bm[w];
        uint64_t at = wpre[w];
        while (x) {
            const uint32_t bit = uint32_t(__builtin_ctz(x));
            ival[at++] = int32_t(int64_t(vmin) + int64_t(w) * 32 + bit);
            x &= x - 1u;
        }
    }
}

__global__ __launch_bounds__(256) void k0_rowoff(const uint64_t* __restrict__ off, uint64_t n,
                                                 uint32_t* __restrict__ out) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i <= n; i += uint64_t(gridDim.x) * blockDim.x)
        out[i] = uint32_t(off[i]);
}

bool k0_disabled() {
    const char* v = std::getenv("FSM_K0");
    return v && !std::strcmp(v, "host");
}

// The row offsets and the token stream (int64, T tokens from seq_off[0],
// narrowed to int32) staged on the host pool through a ring of two pinned
// context slots of kStageBytes and DMA'd (the filling of one chunk overlaps the
// DMA of the other; the slots stay allocated for the context's lifetime).  The
// value range, an out-of-int32 token (bad) and TSR's "some token > -1" are
// gathered by the narrowing (branch-free, vectorizable).  Returns after the
// last copy.  Measured on MI355X (tools/micro/): pinned H2D 47-53 GB/s, pinned
// allocation about 0.12 ms per MiB, and a first pageable copy of the caller's
// arrays about 1 GB/s, so everything goes through the small pinned ring.
constexpr uint64_t kStageBytes = uint64_t(4) << 20;

K0Range k0_stage(fsm_ctx* ctx, const Source& src, int64_t n, uint64_t T, DevBuf& d_so, DevBuf& d_tok) {
    const char* ev = std::getenv("FSM_K0_THREADS");  // tuning
    const int64_t nthr = ev ? std::clamp<int64_t>(std::atoll(ev), 1, 64) : host_threads();
    const double ts0 = now_ms();
    int k = 0;  // chunks staged so far (ring position)
    // fill(h, a, m): write elements [a, a + m) of a stream into pinned h (per host thread)
    auto stream = [&](char* dst, uint64_t nel, uint32_t esz, auto&& fill) {
        const uint64_t per = kStageBytes / esz;
        for (uint64_t a = 0; a < nel; a += per, ++k) {
            const uint64_t m = std::min<uint64_t>(per, nel - a);
            const int slot = 2 + (k & 1);
            char* h = static_cast<char*>(ctx->stage_host(slot, kStageBytes));
            par_slices(m >= (uint64_t(1) << 15) ? nthr : 1, int64_t(m),
                       [&](int64_t t, int64_t i0, int64_t i1) { fill(t, h, a, uint64_t(i0), uint64_t(i1)); });
            ctx->stage_copy(slot, dst + a * esz, m * esz);
        }
    };
    stream(static_cast<char*>(d_so.p), uint64_t(n + 1), 8, [&](int64_t, char* h, uint64_t a, uint64_t i0, uint64_t i1) {
        std::memcpy(h + i0 * 8, src.seq_off + a + i0, (i1 - i0) * 8);
    });
    const int64_t* tok = src.tokens + src.seq_off[0];
    std::vector<int64_t> lo(static_cast<size_t>(nthr), INT64_MAX), hi(static_cast<size_t>(nthr), INT64_MIN);
    stream(static_cast<char*>(d_tok.p), T, 4, [&](int64_t t, char* h, uint64_t a, uint64_t i0, uint64_t i1) {
        int32_t* o = reinterpret_cast<int32_t*>(h);
        const int64_t* in = tok + a;
        int64_t l = lo[size_t(t)], u = hi[size_t(t)];
        for (uint64_t i = i0; i < i1; ++i) {
            const int64_t v = in[i];
            o[i] = int32_t(v);
            const bool sep = uint64_t(v + 2) < 2u;  // -2 or -1
            l = std::min(l, sep ? INT64_MAX : v);
            u = std::max(u, sep ? INT64_MIN : v);
        }
        lo[size_t(t)] = l;
        hi[size_t(t)] = u;
    });
    const double tf = now_ms();
    FSM_HIP(hipStreamSynchronize(ctx->stream));
    int64_t l = INT64_MAX, u = INT64_MIN;
    for (int64_t t = 0; t < nthr; ++t) {
        l = std::min(l, lo[size_t(t)]);
        u = std::max(u, hi[size_t(t)]);
    }
    K0Range rng{INT32_MAX, INT32_MIN, 0, 0};
    if (l <= u) {  // some item token
        rng.bad = l < INT32_MIN || u > INT32_MAX;
        rng.vmin = int32_t(std::max<int64_t>(l, INT32_MIN));
        rng.vmax = int32_t(std::min<int64_t>(u, INT32_MAX));
        rng.any_nonneg = u > -1;
    }
    if (const char* v = std::getenv("FSM_HOST_TRACE"); v && v[0] == '1')
        std::fprintf(stderr, "[fsm k0] staging: %d chunks in %.2f ms, final sync %.2f ms\n", k, tf - ts0, now_ms() - tf);
    return rng;
}

}  // namespace

bool k0_build(fsm_ctx* ctx, int mode, const Source& src, fsm_db* db) {
    if (!src.tokens || src.lines || src.n <= 0 || k0_disabled()) return false;
    const int64_t n = src.n;
    if (n >= int64_t(UINT32_MAX)) return false;
    const double t0 = now_ms();
    // host checks (the reference's errors and the merged-sid case go to the host flatten)
    // (rows checked over the host pool; the long rows collected in row order)
    const int64_t nthr = n >= (int64_t(1) << 16) ? host_threads() : 1;
    std::vector<std::vector<uint32_t>> lr(static_cast<size_t>(nthr));
    std::vector<uint8_t> ok(static_cast<size_t>(nthr), 1);
    par_slices(nthr, n, [&](int64_t t, int64_t a, int64_t z) {
        for (int64_t r = a; r < z; ++r) {
            const bool bad_sid = mode == FSM_MODE_SPADE ? (src.sids[r] < 0 || (r > 0 && src.sids[r] <= src.sids[r - 1]))
                                                        : src.sids[r] != int32_t(r);
            const int64_t L = src.seq_off[r + 1] - src.seq_off[r];
            if (bad_sid || L < 0 || L > int64_t(kK0Long)) {
                ok[size_t(t)] = 0;
                return;
            }
            if (L > int64_t(kK0Wave)) lr[size_t(t)].push_back(uint32_t(r));
        }
    });
    std::vector<uint32_t> longrows;
    for (int64_t t = 0; t < nthr; ++t) {
        if (!ok[size_t(t)]) return false;
        longrows.insert(longrows.end(), lr[size_t(t)].begin(), lr[size_t(t)].end());
    }
    const double t_val = now_ms();
    hipStream_t s = ctx->stream;
    const uint64_t T = uint64_t(src.seq_off[n] - src.seq_off[0]);
    DevBuf d_so(size_t(n + 1) * 8), d_tok(std::max<uint64_t>(T, 1) * 4);
    const double t_alloc = now_ms();
    const K0Range rng = k0_stage(ctx, src, n, T, d_so, d_tok);
    const double t_up = now_ms();
    if (rng.bad) return false;                                       // host reports the bad token
    if (mode == FSM_MODE_TSR && !rng.any_nonneg) return false;      // "no items" error on the host
    const bool any_item = rng.vmin <= rng.vmax;
    const int32_t vmin = any_item ? rng.vmin : 0;
    const int64_t range = any_item ? int64_t(rng.vmax) - vmin + 1 : 1;
    if (range > (int64_t(1) << 27)) return false;
    const uint32_t nw = uint32_t((range + 31) / 32);
    // pass 1: entries per row, presence bitmap, maxima
    DevBuf d_cnt(size_t(n) * 4), d_bm(size_t(nw) * 4), d_st(sizeof(K0Stats)), d_long(std::max<size_t>(longrows.size(), 1) * 4);
    FSM_HIP(hipMemsetAsync(d_bm.p, 0, size_t(nw) * 4, s));
    FSM_HIP(hipMemsetAsync(d_st.p, 0, sizeof(K0Stats), s));
    if (!longrows.empty())
        FSM_HIP(hipMemcpyAsync(d_long.p, longrows.data(), longrows.size() * 4, hipMemcpyHostToDevice, s));
    const unsigned grid_rows = unsigned(std::min<uint64_t>((uint64_t(n) * 64 + kK0Threads - 1) / kK0Threads, 2048));
    const size_t lds = nw <= kK0LdsWords ? size_t(nw) * 4 : 0;
    K0Out o{};
#define K0_PASS(MODE, WR)                                                                                         \
    do {                                                                                                          \
        hipLaunchKernelGGL((k0_rows<MODE, WR>), dim3(grid_rows), dim3(kK0Threads), WR ? 0 : lds, s,               \
                           d_so.as<uint64_t>(), uint32_t(n), d_tok.as<int32_t>(), vmin, nw, d_cnt.as<uint32_t>(), \
                           d_bm.as<uint32_t>(), d_st.as<K0Stats>(), o);                                           \
        FSM_LAUNCHED("k0_rows", s);                                                                               \
        if (!longrows.empty()) {                                                                                  \
            hipLaunchKernelGGL((k0_long<MODE, WR>), dim3(unsigned(longrows.size())), dim3(kK0LongThreads), 0, s,  \
                               d_long.as<uint32_t>(), d_so.as<uint64_t>(), d_tok.as<int32_t>(), vmin,            \
                               d_cnt.as<uint32_t>(), d_bm.as<uint32_t>(), d_st.as<K0Stats>(), o);                 \
            FSM_LAUNCHED("k0_long", s);                                                                           \
        }                                                                                                         \
    } while (0)
    if (mode == FSM_MODE_SPADE) K0_PASS(kSpade, false);
    else K0_PASS(kTsr, false);
    // offsets and the dictionary
    DevBuf d_off(size_t(n + 1) * 8), d_pc(size_t(nw) * 4), d_wpre(size_t(nw + 1) * 8);
    scan_exclusive(d_cnt.as<uint32_t>(), d_off.as<uint64_t>(), size_t(n), s);
    hipLaunchKernelGGL(k0_popc, dim3(unsigned(std::min<uint32_t>((nw + 255) / 256, 4096))), dim3(256), 0, s,
                       d_bm.as<uint32_t>(), nw, d_pc.as<uint32_t>());
    FSM_LAUNCHED("k0_popc", s);
    scan_exclusive(d_pc.as<uint32_t>(), d_wpre.as<uint64_t>(), size_t(nw), s);
    uint64_t E = 0, U = 0;
    K0Stats st{};
    FSM_HIP(hipMemcpyAsync(&E, d_off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
    FSM_HIP(hipMemcpyAsync(&U, d_wpre.as<uint64_t>() + nw, 8, hipMemcpyDeviceToHost, s));
    FSM_HIP(hipMemcpyAsync(&st, d_st.p, sizeof(st), hipMemcpyDeviceToHost, s));
    FSM_HIP(hipStreamSynchronize(s));
    if (E >= (uint64_t(1) << 32)) return false;                    // host reports the limit
    if (mode == FSM_MODE_SPADE && st.max_eids > 4096) return false;  // wider masks: the host flatten (or its limit)
    if (mode == FSM_MODE_TSR && st.neg_item) return false;           // host reports the negative item
    std::vector<int32_t> ival(U);
    DevBuf d_ival(std::max<uint64_t>(U, 1) * 4);
    if (U) {
        hipLaunchKernelGGL(k0_values, dim3(unsigned(std::min<uint32_t>((nw + 255) / 256, 4096))), dim3(256), 0, s,
                           d_bm.as<uint32_t>(), d_wpre.as<uint64_t>(), nw, vmin, d_ival.as<int32_t>());
        FSM_LAUNCHED("k0_values", s);
        FSM_HIP(hipMemcpyAsync(ival.data(), d_ival.p, U * 4, hipMemcpyDeviceToHost, s));
    }
    // pass 2: the rows, written at their offsets
    o.off = d_off.as<uint64_t>();
    o.bm = d_bm.as<uint32_t>();
    o.wpre = d_wpre.as<uint64_t>();
    const unsigned g_off = unsigned(std::min<uint64_t>((uint64_t(n) + 256) / 256, 4096));
    if (mode == FSM_MODE_SPADE) {
        int W = 1;
        while (uint32_t(W) * 64 < st.max_eids) W *= 2;
        auto d = std::make_unique<SpadeDevDB>();
        d->R = n;
        d->E = int64_t(E);
        d->U = int64_t(U);
        d->W = W;
        d->row_off.alloc(size_t(n + 1) * 4);
        d->item.alloc(std::max<uint64_t>(E, 1) * 4);
        d->mask.alloc(std::max<uint64_t>(E, 1) * 8 * uint64_t(W));
        hipLaunchKernelGGL(k0_rowoff, dim3(g_off), dim3(256), 0, s, d_off.as<uint64_t>(), uint64_t(n),
                           d->row_off.as<uint32_t>());
        FSM_LAUNCHED("k0_rowoff", s);
        if (!longrows.empty())  // k0_long ORs eid bits into zeroed masks
            FSM_HIP(hipMemsetAsync(d->mask.p, 0, std::max<uint64_t>(E, 1) * 8 * uint64_t(W), s));
        o.item = d->item.as<uint32_t>();
        o.mask = d->mask.as<uint64_t>();
        o.W = W;
        K0_PASS(kSpade, true);
        FSM_HIP(hipStreamSynchronize(s));
        FlatSpade& f = db->spade;
        f = FlatSpade();
        f.total = n;
        f.W = W;
        f.max_occ = int64_t(st.max_occ);
        f.item_val = std::move(ival);
        db->spade_dev = d.release();
    } else {
        auto d = std::make_unique<TsrDevDB>();
        d->N = n;
        d->E = int64_t(E);
        d->U = int64_t(U);
        d->row_off.alloc(size_t(n + 1) * 4);
        d->item.alloc(std::max<uint64_t>(E, 1) * 4);
        d->first.alloc(std::max<uint64_t>(E, 1) * 4);
        d->last.alloc(std::max<uint64_t>(E, 1) * 4);
        hipLaunchKernelGGL(k0_rowoff, dim3(g_off), dim3(256), 0, s, d_off.as<uint64_t>(), uint64_t(n),
                           d->row_off.as<uint32_t>());
        FSM_LAUNCHED("k0_rowoff", s);
        o.item = d->item.as<uint32_t>();
        o.first = d->first.as<uint32_t>();
        o.last = d->last.as<uint32_t>();
        K0_PASS(kTsr, true);
        tsr_finish(ctx, d.get());  // synchronizes
        FlatTsr& f = db->tsr;
        f = FlatTsr();
        f.total = n;
        f.item_val = std::move(ival);
        db->tsr_dev = d.release();
    }
#undef K0_PASS
    ctx->stats.ms_upload = t_up - t0;
    ctx->stats.ms_flatten = now_ms() - t_up;
    if (const char* v = std::getenv("FSM_HOST_TRACE"); v && v[0] == '1')
        std::fprintf(stderr, "[fsm k0] rows checked %.2f ms, device allocation %.2f ms, tokens staged + uploaded %.2f ms, "
                     "device build %.2f ms\n", t_val - t0, t_alloc - t_val, t_up - t_alloc, ctx->stats.ms_flatten);
    ctx->stats.k0_device = 1;
    return true;
}

}  // namespace fsm
