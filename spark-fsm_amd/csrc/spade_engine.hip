// spade_engine.hip — SPADE frequent-sequence mining on MI355X (SURVEY §8a rows
// a2-a5; the [EXT] SpadeAlgorithm of SPADE.scala:132-135).
//
// Layout.  A batch of prefix equivalence classes [P] lives in HBM as runs: one
// run per (class, sequence containing P), holding one entry per member m of [P]
// (m = P->x or P x) present in that sequence, sorted by member id:
//     cid  u32  class of the entry (index into the batch's class table)
//     mem  u32  member id = rank(x) << 1 | type   (type 0 = sequence-ext, 1 = itemset-ext)
//     lohi u32  first | last set eid of the entry's mask (16 bits each)
//     pos  u32  offset-in-run << 16 | run length
//     mask u64[W] eid bitmask (the id-list entry (sid, eids) of member m)
// The entries of member m across all runs of its class ARE its id-list L(m).
// Runs are laid out in parent-entry order (see k_emit).
//
// Kernels (one launch each per class batch):
//   k_count        every (entry i, entry j) pair of a run evaluates the temporal /
//                  equality join predicate of SURVEY A.2 and bumps the pair's
//                  support counter: ALL n^2 candidate joins of a class in one
//                  streaming pass over its entries (vs n^2 separate list merges).
//   root F2        the root class (the F x 2F pair matrix, by far the largest):
//                  one enumeration writes every entry's keys as a run, runs are
//                  indexed by rank group and counted in LDS (k_root_* / k_group_*).
//   k_freq_*       one wave per member row of the counter matrix: ballot the
//                  frequent candidates (support >= minsup), give them child member
//                  ids (wave prefix popcount), compact them for the host.
//   k_emit         (entry, frequent child) pairs flattened across the lanes:
//                  binary-search the partner entry in the (member-sorted) run,
//                  write the child runs at scan offsets into the next slab.
// The root class is the flattened DB restricted to frequent items (F1 = k_f1,
// row filter = k_root_count / k_root_write).
#include <algorithm>
#include <sys/mman.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <numeric>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>

#include "comm.h"
#include "dev_db.h"
#include "device_util.h"
#include "host_pool.h"


namespace fsm {
// sparse_count.hip
void sparse_sort_rle(const uint64_t* keys, uint64_t* sorted, uint64_t n, unsigned end_bit, uint64_t* uniq,
                     uint32_t* counts, uint32_t* nruns, hipStream_t s);
namespace {

constexpr uint32_t kSeq = 0, kItm = 1;
constexpr uint32_t kFreqOnePassRows = 16384;  // counter rows of a batch up to which k_freq_recs extracts in one pass
constexpr uint32_t kChunk = 512;         // class entries per k_count block (FSM_COUNT_CHUNK; swept on MI355X)
constexpr uint32_t kGroupCounters = 32768;  // root F2: u32 LDS counters of one rank group (128 KiB)
constexpr uint32_t kMaxGroups = 16384;      // root F2 rank groups: LDS cursors of k_f2_keys (64 KiB)
constexpr int kBlock = 256;


struct DClass {
    uint64_t cnt_off;     // counter matrix of the class
    uint32_t D;           // member id space (2 * ranks)
    uint32_t cbase;       // offset of the class's members in per-member arrays
    uint32_t mshift;      // counter row of member mi = mi >> mshift (root: 1, only SEQ members)
    uint32_t rstride;     // counters between consecutive rows (D, or a power of two >= D in keyed batches)
    uint32_t pad[2];
};
struct DRow {
    uint32_t cls, mi;
};
struct FreqRec {
    uint32_t row, slot, sup, cid;
};

struct SlabPtrs {
    uint32_t* cid;  // class of the entry (index into the batch's class table)
    uint32_t* mem;
    uint32_t* lohi;
    uint32_t* pos;
    uint64_t* mask;
    uint32_t* lim = nullptr;  // emit target: set when a child run exceeds 65535 entries (pos fields)
};

// W = 1 slabs keep no lohi word: an entry's first / last eid are the lowest / highest bit
// of its one mask word (ctz / clz), 20 B per entry instead of 24.  FSM_W1_LOHI=1 (a build
// flag, tools/build_variant.sh) stores it as the wider slabs do, for A/B runs.
#ifndef FSM_W1_LOHI
#define FSM_W1_LOHI 0
#endif
template <int W> constexpr bool kLhDerived = W == 1 && !FSM_W1_LOHI;
inline bool lh_derived(int W) { return W == 1 && !FSM_W1_LOHI; }
__device__ __forceinline__ uint32_t lh_of_word(uint64_t m) {
    return uint32_t(__builtin_ctzll(m)) | ((63u - uint32_t(__builtin_clzll(m))) << 16);
}
// the lohi word of slab entry e (W: the slab's mask words; 0 = runtime width)
template <int W>
__device__ __forceinline__ uint32_t slab_lh(const uint32_t* __restrict__ lohi, const uint64_t* __restrict__ mask,
                                            size_t e) {
    if constexpr (kLhDerived<W>) return lh_of_word(mask[e]);
    else return lohi[e];
}

// ------------------------------------------------------------------ kernels

// K1: F1 histogram = distinct-sid support per item (entries are distinct per
// (row, item)); LDS-privatized per block when the item dictionary fits.
// SPADE.scala:113-126 `idList.getSupport()`.
__global__ __launch_bounds__(kBlock) void k_f1(const uint32_t* __restrict__ item, uint64_t e0, uint64_t e1,
                                               uint32_t* __restrict__ f1, uint32_t U, int use_lds) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    if (use_lds) {
        for (uint32_t u = threadIdx.x; u < U; u += blockDim.x) h[u] = 0;
        __syncthreads();
    }
    for (uint64_t e = e0 + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < e1;
         e += uint64_t(gridDim.x) * blockDim.x) {
        if (use_lds) atomicAdd(&h[item[e]], 1u);
        else atomicAdd(&f1[item[e]], 1u);
    }
    if (use_lds) {
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < U; u += blockDim.x)
            if (h[u]) atomicAdd(&f1[u], h[u]);
    }
}

__global__ __launch_bounds__(kBlock) void k_root_count(const uint32_t* __restrict__ row_off,
                                                       const uint32_t* __restrict__ item,
                                                       const uint32_t* __restrict__ rank, uint64_t r0, uint64_t r1,
                                                       uint32_t* __restrict__ cnt, uint32_t* __restrict__ flag) {
    const uint64_t r = r0 + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= r1) return;
    uint32_t c = 0;
    for (uint32_t e = row_off[r]; e < row_off[r + 1]; ++e) c += rank[item[e]] != kNone;
    cnt[r - r0] = c;
    if (c > 0xFFFFu) atomicOr(flag, 1u);
}

// one wave per DB row: ballot the frequent items, write them compacted
template <int W>
__global__ __launch_bounds__(kBlock) void k_root_write(const uint32_t* __restrict__ row_off,
                                                       const uint32_t* __restrict__ item,
                                                       const uint64_t* __restrict__ mask,
                                                       const uint32_t* __restrict__ rank, uint64_t r0, uint64_t r1,
                                                       const uint64_t* __restrict__ off, SlabPtrs o, uint32_t wd) {
    const uint64_t r = r0 + ((uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
    if (r >= r1) return;
    const uint64_t ob = off[r - r0];
    const uint32_t len = uint32_t(off[r - r0 + 1] - ob);
    const uint32_t e1 = row_off[r + 1];
    uint32_t k = 0;
    for (uint32_t b = row_off[r]; b < e1; b += 64) {
        const uint32_t e = b + lane_id();
        const uint32_t rk = e < e1 ? rank[item[e]] : kNone;
        const bool fr = rk != kNone;
        const uint64_t bal = ballot(fr);
        if (fr) {
            const uint32_t p = k + uint32_t(__popcll(bal & lanemask_lt()));
            const uint64_t d = ob + p;
            o.mem[d] = rk << 1 | kSeq;
            o.pos[d] = (p << 16) | len;
            if constexpr (W == 0) {
                o.lohi[d] = mask_copy_lohi_dyn(mask + size_t(e) * wd, o.mask + size_t(d) * wd, wd);
            } else {
                uint64_t m[W];
                load_mask<W>(mask + size_t(e) * W, m);
                if constexpr (!kLhDerived<W>) o.lohi[d] = mask_lo<W>(m) | (mask_hi<W>(m) << 16);
                store_mask<W>(o.mask + size_t(d) * W, m);
            }
        }
        k += uint32_t(__popcll(bal));
    }
}

template <int W> __device__ __forceinline__ bool and_nonzero(const uint64_t (&a)[W], const uint64_t* __restrict__ b) {
    uint64_t bm[W];
    load_mask<W>(b, bm);
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) acc |= a[k] & bm[k];
    return acc != 0;
}

// K2/K3/K4: all candidate joins of every class of the batch, one pass.
template <int W>
__global__ __launch_bounds__(kBlock) void k_count(uint32_t E, const uint32_t* __restrict__ cid,
                                                  const DClass* __restrict__ cls,
                                                  const uint32_t* __restrict__ mem, const uint32_t* __restrict__ lohi,
                                                  const uint32_t* __restrict__ pos, const uint64_t* __restrict__ mask,
                                                  uint32_t mlo, uint32_t mhi, uint32_t chunk,
                                                  uint32_t* __restrict__ cnt,
                                                  unsigned long long* __restrict__ tests, uint32_t wd) {
    const uint32_t mw = mask_words<W>(wd);
    __shared__ uint32_t blk_tests;
    if (threadIdx.x == 0) blk_tests = 0;
    __syncthreads();
    uint32_t my_tests = 0;  // (entry, partner) join tests executed (fsm_stats.pair_tests)
    const uint32_t e1 = uint32_t(min(uint64_t(E), (uint64_t(blockIdx.x) + 1) * chunk));
    for (uint32_t e = blockIdx.x * chunk + threadIdx.x; e < e1; e += blockDim.x) {
        const uint32_t mi = mem[e], p = pos[e];
        if (mi - mlo >= mhi - mlo) continue;  // member rows of another rank (sharded root)
        my_tests += p & 0xFFFFu;
        const DClass c = cls[cid[e]];
        const uint32_t lh_i = slab_lh<W>(lohi, mask, e), lo_i = lh_i & 0xFFFFu;
        const uint32_t ti = mi & 1u, ri = mi >> 1;
        const uint32_t rb = e - (p >> 16), rl = p & 0xFFFFu;
        MaskV<W> mk;
        mk.load(mask + size_t(e) * mw, wd, lh_i);
        uint32_t* rowc = cnt + c.cnt_off + uint64_t(mi >> c.mshift) * c.rstride;
        for (uint32_t q = 0; q < rl; ++q) {
            const uint32_t f = rb + q;
            const uint32_t mj = mem[f];
            const uint32_t tj = mj & 1u, rj = mj >> 1;
            const uint32_t lh_f = slab_lh<W>(lohi, mask, f);
            if (tj == kSeq) {
                // P x -> y  /  P->x -> y : bits of L(j) strictly after first bit of L(i)
                if ((lh_f >> 16) > lo_i) atomicAdd(rowc + (rj << 1), 1u);
                // P->(x y), y > x : L(i) & L(j)
                if (ti == kSeq && rj > ri && mk.and_any(mask + size_t(f) * mw, wd, lh_f))
                    atomicAdd(rowc + (rj << 1 | 1u), 1u);
            } else if (ti == kItm && rj > ri && mk.and_any(mask + size_t(f) * mw, wd, lh_f)) {
                // P(x y), y > x
                atomicAdd(rowc + (rj << 1 | 1u), 1u);
            }
        }
    }
    atomicAdd(&blk_tests, my_tests);
    __syncthreads();
    if (threadIdx.x == 0 && blk_tests) atomicAdd(tests, (unsigned long long)blk_tests);
}

// Keyed class counting (batches of >= kKeyedMinEntries entries; FSM_COUNT_PATH
// selects): k_count's device-scope atomics execute at the memory side (15.5M of
// them at D1M, 92 % of wave cycles waiting: profiles/r2/atomics).  Here the
// batch's counters are laid out in groups of kGroupCounters (rows never straddle
// a group) and counted like the root F2: k_cnt_plan histograms each entry's key
// capacity by group per entry block, k_cnt_keys writes every successful join as
// a u16 key (the counter's offset in its group) into region (group, block), and
// k_f2_count<true> streams a group's regions into LDS counters and writes the
// group's counters out whole (no memset, no global atomics).
constexpr uint32_t kKeyedMinEntries = 1u << 20;
constexpr uint32_t kGroupShift = 15;  // kGroupCounters = 1 << kGroupShift

__device__ __forceinline__ uint64_t row_base(const DClass& c, uint32_t mi) {
    return c.cnt_off + uint64_t(mi >> c.mshift) * c.rstride;
}

__global__ __launch_bounds__(1024) void k_cnt_plan(uint32_t E, uint32_t epb, const uint32_t* __restrict__ cid,
                                                   const DClass* __restrict__ cls, const uint32_t* __restrict__ mem,
                                                   const uint32_t* __restrict__ pos, uint32_t mlo, uint32_t mhi,
                                                   uint32_t G, uint32_t nblk, uint32_t* __restrict__ cap) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) h[g] = 0;
    __syncthreads();
    const uint32_t e0 = blockIdx.x * epb, e1 = min(E, e0 + epb);
    for (uint32_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const uint32_t mi = mem[e];
        if (mi - mlo >= mhi - mlo) continue;
        const uint32_t p = pos[e], rl = p & 0xFFFFu, off = p >> 16;
        // temporal: any partner (itself included); equality: partners of higher rank (after it)
        atomicAdd(&h[uint32_t(row_base(cls[cid[e]], mi) >> kGroupShift)], 2 * rl - 1 - off);
    }
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) cap[uint64_t(g) * nblk + blockIdx.x] = (h[g] + 7u) & ~7u;
}

// the join tests of k_count for entry i against partner f; calls key(col) per successful join
template <int W, class K>
__device__ __forceinline__ void class_joins(uint32_t ti, uint32_t ri, uint32_t lo_i, const MaskV<W>& mk,
                                            uint32_t f, const uint32_t* __restrict__ mem,
                                            const uint32_t* __restrict__ lohi, const uint64_t* __restrict__ mask,
                                            uint32_t wd, K&& key) {
    const uint32_t mw = mask_words<W>(wd);
    const uint32_t mj = mem[f];
    const uint32_t tj = mj & 1u, rj = mj >> 1;
    const uint32_t lh_f = slab_lh<W>(lohi, mask, f);
    if (tj == kSeq) {
        if ((lh_f >> 16) > lo_i) key(rj << 1);
        if (ti == kSeq && rj > ri && mk.and_any(mask + size_t(f) * mw, wd, lh_f)) key(rj << 1 | 1u);
    } else if (ti == kItm && rj > ri && mk.and_any(mask + size_t(f) * mw, wd, lh_f)) {
        key(rj << 1 | 1u);
    }
}

template <int W>
__global__ __launch_bounds__(1024) void k_cnt_keys(uint32_t E, uint32_t epb, const uint32_t* __restrict__ cid,
                                                   const DClass* __restrict__ cls, const uint32_t* __restrict__ mem,
                                                   const uint32_t* __restrict__ lohi, const uint32_t* __restrict__ pos,
                                                   const uint64_t* __restrict__ mask, uint32_t mlo, uint32_t mhi,
                                                   uint32_t G, uint32_t nblk, const uint64_t* __restrict__ base,
                                                   uint32_t* __restrict__ fill, uint16_t* __restrict__ keys,
                                                   unsigned long long* __restrict__ tests, uint32_t wd) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];  // region cursors [G]
    __shared__ uint32_t blk_tests;
    const uint32_t b = blockIdx.x;
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) cur[g] = uint32_t(base[uint64_t(g) * nblk + b]);
    if (threadIdx.x == 0) blk_tests = 0;
    __syncthreads();
    uint32_t my_tests = 0;
    const uint32_t e0 = b * epb, e1 = min(E, e0 + epb);
    const uint32_t lane = lane_id();
    for (uint32_t b0 = e0; b0 < e1; b0 += blockDim.x) {  // wave-uniform trip count (ballots below)
        const uint32_t e = b0 + threadIdx.x;
        uint32_t mi = e < e1 ? mem[e] : 0u;
        const bool live = e < e1 && mi - mlo < mhi - mlo;
        uint32_t n = 0, g = 0, kb = 0, rl = 0, rb = 0, lo_i = 0, ti = 0, ri = 0;
        MaskV<W> mk;
        if (live) {
            const uint32_t p = pos[e];
            rl = p & 0xFFFFu;
            rb = e - (p >> 16);
            my_tests += rl;
            const uint64_t rbase = row_base(cls[cid[e]], mi);
            g = uint32_t(rbase >> kGroupShift);
            kb = uint32_t(rbase) & (kGroupCounters - 1u);
            const uint32_t lh_i = slab_lh<W>(lohi, mask, e);
            lo_i = lh_i & 0xFFFFu;
            ti = mi & 1u;
            ri = mi >> 1;
            mk.load(mask + size_t(e) * mask_words<W>(wd), wd, lh_i);
            for (uint32_t q = 0; q < rl; ++q)
                class_joins<W>(ti, ri, lo_i, mk, rb + q, mem, lohi, mask, wd, [&](uint32_t) { ++n; });
        }
        // region slots: with few groups every lane of a wave would hit the same LDS
        // cursors, so the wave reserves once per distinct group among its lanes
        uint32_t at = 0;
        if (G <= 64) {
            for (uint64_t todo = ballot(n > 0); todo;) {
                const int lead = __ffsll((unsigned long long)todo) - 1;
                const uint32_t lg = uint32_t(__shfl(int(g), lead, 64));
                const bool in = n > 0 && g == lg;
                const uint64_t m = ballot(in);
                const uint32_t v = in ? n : 0u;
                const uint32_t incl = wave_incl_scan(v);
                const uint32_t tot = uint32_t(__shfl(int(incl), 63, 64));
                uint32_t base = 0;
                if (int(lane) == lead) base = atomicAdd(&cur[lg], tot);
                base = uint32_t(__shfl(int(base), lead, 64));
                if (in) at = base + incl - v;
                todo &= ~m;
            }
        } else if (n) {
            at = atomicAdd(&cur[g], n);
        }
        if (n) {
            for (uint32_t q = 0; q < rl; ++q)
                class_joins<W>(ti, ri, lo_i, mk, rb + q, mem, lohi, mask, wd,
                               [&](uint32_t col) { keys[at++] = uint16_t(kb + col); });
        }
    }
    atomicAdd(&blk_tests, my_tests);
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x)
        fill[uint64_t(g) * nblk + b] = cur[g] - uint32_t(base[uint64_t(g) * nblk + b]);
    if (threadIdx.x == 0 && blk_tests) atomicAdd(tests, (unsigned long long)blk_tests);
}

// ---- Sparse class count (batches whose dense D x D counter matrices would be far
// larger than their joins: a class with tens of thousands of frequent children,
// mostly absent from one another's sequences).  k_sparse_cap sums every entry's key
// capacity (temporal: any partner; equality: partners after it); k_sparse_keys
// writes every successful join as the u64 key (member slot cbase + mi) << 32 |
// column; sparse_sort_rle (sparse_count.hip: rocPRIM radix sort + run-length
// encode) leaves the non-zero counters in (slot, column) order; k_sparse_flag +
// scan + k_sparse_recs keep the frequent ones as FreqRec in (row, slot) order.
__global__ __launch_bounds__(kBlock) void k_sparse_cap(uint32_t E, const uint32_t* __restrict__ mem,
                                                       const uint32_t* __restrict__ pos, uint32_t mlo, uint32_t mhi,
                                                       unsigned long long* __restrict__ cap) {
    __shared__ unsigned long long bs;
    if (threadIdx.x == 0) bs = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < E; e += gridDim.x * blockDim.x) {
        const uint32_t mi = mem[e], p = pos[e];
        if (mi - mlo < mhi - mlo) c += 2ull * (p & 0xFFFFu) - 1ull - (p >> 16);
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, 64);
    if (lane_id() == 0) atomicAdd(&bs, c);
    __syncthreads();
    if (threadIdx.x == 0 && bs) atomicAdd(cap, bs);
}

template <int W>
__global__ __launch_bounds__(kBlock) void k_sparse_keys(uint32_t E, const uint32_t* __restrict__ cid,
                                                        const DClass* __restrict__ cls, const uint32_t* __restrict__ mem,
                                                        const uint32_t* __restrict__ lohi,
                                                        const uint32_t* __restrict__ pos,
                                                        const uint64_t* __restrict__ mask, uint32_t mlo, uint32_t mhi,
                                                        uint32_t wd, unsigned long long* __restrict__ keys,
                                                        unsigned long long* __restrict__ cursor,
                                                        unsigned long long* __restrict__ tests) {
    const uint32_t lane = lane_id();
    uint32_t my_tests = 0;
    // wave-uniform trip count (the key reservation is a wave scan)
    for (uint32_t b0 = blockIdx.x * blockDim.x; b0 < E; b0 += gridDim.x * blockDim.x) {
        const uint32_t e = b0 + threadIdx.x;
        const uint32_t mi = e < E ? mem[e] : 0u;
        const bool live = e < E && mi - mlo < mhi - mlo;
        uint32_t n = 0, rl = 0, rb = 0, lo_i = 0, ti = 0, ri = 0, slot = 0;
        MaskV<W> mk;
        if (live) {
            const uint32_t p = pos[e];
            rl = p & 0xFFFFu;
            rb = e - (p >> 16);
            my_tests += rl;
            slot = cls[cid[e]].cbase + mi;
            const uint32_t lh_i = slab_lh<W>(lohi, mask, e);
            lo_i = lh_i & 0xFFFFu;
            ti = mi & 1u;
            ri = mi >> 1;
            mk.load(mask + size_t(e) * mask_words<W>(wd), wd, lh_i);
            for (uint32_t q = 0; q < rl; ++q)
                class_joins<W>(ti, ri, lo_i, mk, rb + q, mem, lohi, mask, wd, [&](uint32_t) { ++n; });
        }
        const uint32_t incl = wave_incl_scan(n), tot = uint32_t(__shfl(int(incl), 63, 64));
        unsigned long long base = 0;
        if (lane == 63 && tot) base = atomicAdd(cursor, (unsigned long long)tot);
        base = __shfl(base, 63, 64);
        if (n) {
            unsigned long long at = base + incl - n;
            const unsigned long long hi = (unsigned long long)slot << 32;
            for (uint32_t q = 0; q < rl; ++q)
                class_joins<W>(ti, ri, lo_i, mk, rb + q, mem, lohi, mask, wd, [&](uint32_t col) { keys[at++] = hi | col; });
        }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) my_tests += uint32_t(__shfl_xor(int(my_tests), d, 64));
    if (lane == 0 && my_tests) atomicAdd(tests, (unsigned long long)my_tests);
}

__global__ __launch_bounds__(kBlock) void k_sparse_flag(const uint32_t* __restrict__ counts,
                                                        const uint32_t* __restrict__ nruns, uint32_t n, uint32_t minsup,
                                                        uint32_t* __restrict__ flag) {
    const uint32_t nr = *nruns;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        flag[i] = i < nr && counts[i] >= minsup ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void k_sparse_recs(const uint64_t* __restrict__ uniq,
                                                        const uint32_t* __restrict__ counts,
                                                        const uint32_t* __restrict__ nruns,
                                                        const uint64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ slot2row, uint32_t minsup,
                                                        FreqRec* __restrict__ out) {
    const uint32_t nr = *nruns;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += gridDim.x * blockDim.x)
        if (counts[i] >= minsup) {
            const uint64_t k = uniq[i];
            out[off[i]] = FreqRec{slot2row[uint32_t(k >> 32)], uint32_t(k & 0xFFFFFFFFu), counts[i], 0u};
        }
}

__device__ __forceinline__ uint64_t lane_range(uint32_t a, uint32_t b) {  // bits [a, b), 0 <= a <= b <= 64
    const uint64_t hi = b >= 64 ? ~0ull : ((1ull << b) - 1ull);
    const uint64_t lo = a >= 64 ? ~0ull : ((1ull << a) - 1ull);
    return hi & ~lo;
}

// Root F2 (the F x 2F counter matrix, 220 MB at D1M: far beyond LDS, and
// global atomics into it run at the memory side, 1.3 TB/s of added bytes).
// Every key of a root entry lies in the counter row of its own rank, so the
// matrix is cut into rank groups of `per` ranks whose per*D counters fit
// 128 KiB of LDS, and the pairs are partitioned by group on the way out:
//   plan        per (group, row block): key capacity = sum of the entries'
//               upper bounds (temporal <= row length, equality <= partners of
//               higher rank), made by k_root_write_plan while it writes the
//               root rows; exclusive scan -> region bases, group-major
//   k_f2_keys   THE one partner enumeration: row block b writes the keys of
//               group g (u16, local to the group's counter tile) into region
//               (g, b) through an LDS cursor per group.  Rows of <= 64 entries
//               (W = 1) go lane-per-pair in power-of-two lane segments: a step
//               evaluates 64 / S entries i at once, S = row length rounded up;
//               the row's active entries are compacted into LDS (F2Act, one
//               16-byte read per step, issued a step ahead) and the segment's
//               cursor offset comes back by readlane when S >= 32
//   k_f2_count  one block per group: stream the group's regions with 16-byte
//               loads into LDS counters, then ballot out the frequent pairs
//               (support >= minsup) - the matrix itself never reaches HBM
// PMC basis (profiles/r2/baseline_sq): the row-per-step enumeration of round 1
// was instruction-issue bound (1.48 G VALU+SALU instructions, 44 % of wave
// cycles waiting to issue) and the per-run key walk latency bound (93 % waiting).
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return uint32_t(__builtin_amdgcn_readfirstlane(int(v))); }

// rank -> group by multiply-high (exact for rank < 2^16, per < 2^15)
__device__ __forceinline__ uint32_t group_of(uint32_t rank, uint32_t pm) { return __umulhi(rank, pm); }

// region (group g, row block b) in scan order: group-major [g][b], each group's keys one
// contiguous stream for k_f2_count (block-major measured no faster)
__device__ __forceinline__ uint64_t f2_region(uint32_t g, uint32_t b, uint32_t nblk) {
    return uint64_t(g) * nblk + b;
}

constexpr uint32_t kF2Threads = 1024;  // k_f2_keys / k_f2_count block
constexpr uint32_t kF2Waves = kF2Threads / 64;

// row entry staged in LDS for the lane-per-pair path (W = 1): the partner side
struct F2Ent {
    uint32_t x;     // rank (0xFFFF: an infrequent DB entry) | lo << 16
    uint32_t y;     // (unused)
    uint64_t mask;  // eid mask
};
// an active entry i of the row (compacted): group | row index << 16, key base | lo << 16, mask
struct F2Act {
    uint32_t a, b;
    uint64_t mask;
};
constexpr uint32_t kF2MaxRows = 4096;  // rows per block of k_f2_keys (row offsets staged in LDS)
constexpr uint32_t kF2RowWords = (kF2MaxRows + 1 + 3) & ~3u;  // their LDS words (what follows stays 16-byte aligned)

// Root rows fused with the F2 plan: block b builds the root runs of its row block
// (rpb rows, one wave per row in turn, as k_root_write) and histograms the key
// capacity of every entry it writes by rank group (the F2 plan) in LDS.
template <int W>
__global__ __launch_bounds__(kF2Threads) void k_root_write_plan(const uint32_t* __restrict__ row_off,
                                                               const uint32_t* __restrict__ item,
                                                               const uint64_t* __restrict__ mask,
                                                               const uint32_t* __restrict__ rank, uint32_t R,
                                                               uint32_t rpb, const uint64_t* __restrict__ off,
                                                               SlabPtrs o, uint32_t pm, uint32_t G, uint32_t nblk,
                                                               uint32_t mlo, uint32_t mhi,
                                                               uint32_t* __restrict__ cap, uint32_t amask, uint32_t wd) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) h[g] = 0;
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
    const uint32_t r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
    // the next row's bounds and first 64 ranks are loaded while the current row is
    // written (each row is a chain of dependent loads: bounds -> items -> ranks)
    uint64_t nob = 0;
    uint32_t nlen = 0, nrb = 0, ne1 = 0, nrk = kNone;
    auto fetch = [&](uint32_t rr) {
        if (rr >= r1) return;
        nob = off[rr];
        nlen = uint32_t(off[rr + 1] - nob);
        nrb = row_off[rr];
        ne1 = row_off[rr + 1];
        nrk = nrb + lane < ne1 ? rank[item[nrb + lane]] : kNone;
    };
    fetch(r0 + wave);
    for (uint32_t r = r0 + wave; r < r1; r += kF2Waves) {
        const uint64_t ob = nob;
        const uint32_t len = nlen, rb = nrb, e1 = ne1, rk0 = nrk;
        fetch(r + kF2Waves);
        uint32_t k = 0;
        for (uint32_t b0 = rb; b0 < e1; b0 += 64) {
            const uint32_t e = b0 + lane;
            const uint32_t rk = b0 == rb ? rk0 : (e < e1 ? rank[item[e]] : kNone);
            const bool fr = rk != kNone;
            const uint64_t bal = ballot(fr);
            if (fr) {
                const uint32_t p = k + uint32_t(__popcll(bal & lanemask_lt()));
                const uint64_t d = ob + p;
                o.mem[d] = rk << 1 | kSeq;
                o.pos[d] = (p << 16) | len;
                if constexpr (W == 0) {
                    o.lohi[d] = mask_copy_lohi_dyn(mask + size_t(e) * wd, o.mask + size_t(d) * wd, wd);
                } else {
                    uint64_t m[W];
                    load_mask<W>(mask + size_t(e) * W, m);
                    if constexpr (!kLhDerived<W>) o.lohi[d] = mask_lo<W>(m) | (mask_hi<W>(m) << 16);
                    store_mask<W>(o.mask + size_t(d) * W, m);
                }
                if ((rk << 1) - mlo < mhi - mlo) atomicAdd(&h[group_of(rk, pm)], 2 * len - 1 - p);
            }
            k += uint32_t(__popcll(bal));
        }
    }
    __syncthreads();
    // regions start on 16-byte boundaries (amask + 1 >= 8 keys): k_f2_count reads them in aligned chunks
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x)
        cap[f2_region(g, blockIdx.x, nblk)] = (h[g] + amask) & ~amask;
}

// ---- DB-direct root.  The root class is the DB restricted to the frequent items, so
// its kernels (F2 plan, F2 keys, root emit) read the DB rows themselves instead of a
// root slab written per mine (k_root_count + k_root_write: 0.5 ms and 24 B per entry
// at D1M, replicated on every rank of a sharded mine).  A DB entry's member id is
// rk2[item]: 2 x rank for a frequent item (a root member is a sequence-extension), and
// an ODD value for an infrequent one, 2 x (frequent items below it) - 1, so that in
// wrapped order (v + 1) the row stays sorted and an infrequent entry never equals a
// partner target (even).  Its lohi comes from the mask; its pos (offset in row << 16 |
// row length) from the DB's own pos array (k_db_pos, once per DB).
struct RootRef {
    const uint32_t* item;  // DB entry -> dense item (nullptr: not the DB-direct root)
    const uint32_t* rk2;   // dense item -> member id (above)
};
template <int W> __device__ __forceinline__ uint32_t lohi_of(const uint64_t* __restrict__ mask, size_t e) {
    uint64_t m[W];
    load_mask<W>(mask + e * W, m);
    return mask_lo<W>(m) | (mask_hi<W>(m) << 16);
}
// entry accessors of a batch slab (kRoot = false) or of the DB-direct root (kRoot = true)
// (WL: the slab's own mask width for its lohi words, W's when W > 0)
template <int W, bool kRoot, int WL = W> struct Ent {
    static constexpr bool kRootEnt = kRoot;
    const uint32_t* __restrict__ cid;
    const uint32_t* __restrict__ mem;
    const uint32_t* __restrict__ lohi;
    const uint64_t* __restrict__ mask;
    RootRef rr;
    __device__ __forceinline__ uint32_t c(size_t e) const {
        if constexpr (kRoot) return 0u; else return cid[e];
    }
    __device__ __forceinline__ uint32_t m(size_t e) const { return mem[e]; }  // (DB-direct root: the plan's member ids)
    __device__ __forceinline__ uint32_t lh(size_t e) const {
        if constexpr (kRoot) return lohi_of<W>(mask, e); else return slab_lh<WL>(lohi, mask, e);
    }
};
// member ids in the wrapped order of the DB-direct root (identity order for batch slabs,
// whose member ids stay below 2^31)
__device__ __forceinline__ bool mem_less(uint32_t a, uint32_t b) { return a + 1u < b + 1u; }

// pos of every DB entry: offset in its row << 16 | row length (rows <= 65535 entries;
// longer ones raise *flag and the mine keeps the root slab)
__global__ __launch_bounds__(kBlock) void k_db_pos(const uint32_t* __restrict__ row_off, uint32_t R,
                                                   uint32_t* __restrict__ pos, uint32_t* __restrict__ flag) {
    const uint32_t r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (r >= R) return;
    const uint32_t rb = row_off[r], re = row_off[r + 1], len = re - rb;
    if (len > 0xFFFFu) {
        if (lane_id() == 0) atomicOr(flag, 1u);
        return;
    }
    for (uint32_t e = rb + lane_id(); e < re; e += 64) pos[e] = ((e - rb) << 16) | len;
}

// F2 plan of the DB-direct root: block b histograms, by rank group, the key capacity of
// the frequent entries of its rpb rows that lie in the member range [mlo, mhi)
// (temporal <= row's frequent entries, equality <= frequent partners after it).
// tri (the unordered-pair layout below, gtab != nullptr): capacity 1 + 3 (partners after it),
// the group from the rank's table entry.
__global__ __launch_bounds__(kF2Threads) void k_f2_plan_db(const uint32_t* __restrict__ row_off,
                                                          const uint32_t* __restrict__ item,
                                                          const uint32_t* __restrict__ rk2, uint32_t R, uint32_t rpb,
                                                          uint32_t pm, uint32_t G, uint32_t nblk, uint32_t mlo,
                                                          uint32_t mhi, uint32_t* __restrict__ cap, uint32_t amask,
                                                          uint32_t* __restrict__ mem_out,
                                                          const uint32_t* __restrict__ gtab) {
    extern __shared__ __attribute__((aligned(16))) uint32_t h[];
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) h[g] = 0;
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
    for (uint32_t r = r0 + wave; r < r1; r += kF2Waves) {
        const uint32_t rb = row_off[r], e1 = row_off[r + 1];
        // the row's frequent entries (first chunk kept in registers: rows are short)
        uint32_t v0 = kNone, len = 0;
        for (uint32_t b0 = rb; b0 < e1; b0 += 64) {
            const uint32_t e = b0 + lane;
            const uint32_t v = e < e1 ? rk2[item[e]] : kNone;
            if (e < e1) mem_out[e] = v;  // the entries' member ids, read by the F2 keys and the root emit
            if (b0 == rb) v0 = v;
            len += uint32_t(__popcll(ballot(e < e1 && !(v & 1u))));
        }
        uint32_t k = 0;
        for (uint32_t b0 = rb; b0 < e1; b0 += 64) {
            const uint32_t e = b0 + lane;
            const uint32_t v = b0 == rb ? v0 : (e < e1 ? rk2[item[e]] : kNone);
            const bool fr = e < e1 && !(v & 1u);
            const uint64_t bal = ballot(fr);
            const uint32_t p = k + uint32_t(__popcll(bal & lt));
            if (fr && v - mlo < mhi - mlo) {
                if (gtab) atomicAdd(&h[gtab[v >> 1] >> kGroupShift], 1 + 3 * (len - 1 - p));
                else atomicAdd(&h[group_of(v >> 1, pm)], 2 * len - 1 - p);
            }
            k += uint32_t(__popcll(bal));
        }
    }
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) cap[f2_region(g, blockIdx.x, nblk)] = (h[g] + amask) & ~amask;
}

// kRoot: the rows are the DB's (row_off32), entries read through rr (DB-direct root)
template <int W, bool kRoot>
__global__ __launch_bounds__(kF2Threads) void k_f2_keys(const uint64_t* __restrict__ roff,
                                                        const uint32_t* __restrict__ row_off32, RootRef rr,
                                                        uint32_t R, uint32_t rpb,
                                                        const uint32_t* __restrict__ mem,
                                                        const uint32_t* __restrict__ lohi,
                                                        const uint64_t* __restrict__ mask, uint32_t D, uint32_t per,
                                                        uint32_t pm, uint32_t G, uint32_t nblk, uint32_t mlo,
                                                        uint32_t mhi, const uint64_t* __restrict__ base,
                                                        uint32_t* __restrict__ fill, uint16_t* __restrict__ keys,
                                                        unsigned long long* __restrict__ nkeys_total, uint32_t wd) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    F2Ent* stage_all = reinterpret_cast<F2Ent*>(smem);  // kF2Waves x 64 entries
    uint32_t* srow = smem + kF2Waves * 64 * (sizeof(F2Ent) / 4);  // row offsets of the block [rpb + 1]
    uint32_t* actx_all = srow + kF2RowWords;                        // kF2Waves x 64 active entries (F2Act)
    uint32_t* cur = actx_all + kF2Waves * 64 * (sizeof(F2Act) / 4); // region cursors [G]
    __shared__ uint32_t blk_keys;
    const uint32_t b = blockIdx.x;
    const uint32_t r0 = b * rpb, r1 = min(R, r0 + rpb);
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) cur[g] = uint32_t(base[f2_region(g, b, nblk)]);
    for (uint32_t r = r0 + threadIdx.x; r <= r1; r += blockDim.x) srow[r - r0] = kRoot ? row_off32[r] : uint32_t(roff[r]);
    if (threadIdx.x == 0) blk_keys = 0;
    const Ent<W == 0 ? 1 : W, kRoot, W> en_{nullptr, mem, lohi, mask, rr};
    __syncthreads();
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    F2Ent* stage = stage_all + wave * 64;
    F2Act* sact = reinterpret_cast<F2Act*>(actx_all) + wave * 64;
    const uint64_t lt = lanemask_lt();
    uint32_t my_keys = 0;
    // the next row's entries are loaded while the current row is enumerated
    uint32_t nrb = 0, nrl = 0, nme = 0, nlh = 0;
    uint64_t nmk = 0;
    auto fetch = [&](uint32_t rr) {
        if (rr >= r1) return;
        nrb = srow[rr - r0];
        nrl = srow[rr - r0 + 1] - nrb;
        if (W == 1 && nrl <= 64 && lane < nrl) {
            nme = mem[nrb + lane];
            nmk = mask[nrb + lane];
            if constexpr (kRoot || kLhDerived<W>) nlh = lh_of_word(nmk);
            else nlh = lohi[nrb + lane];
        }
    };
    fetch(r0 + wave);
    for (uint32_t r = r0 + wave; r < r1; r += kF2Waves) {
        const uint32_t rb = rfl(nrb), rl = rfl(nrl), me = nme, lh = nlh;
        const uint64_t mk = nmk;
        fetch(r + kF2Waves);
        if (rl == 0) continue;
        if (W == 1 && rl <= 64) {
            // ---- lane-per-pair: segments of S lanes, lane s0 + j tests partner j.  The
            // active entries i are compacted into LDS with all a step needs (one 16-byte read,
            // issued a step ahead); the segment's cursor offset comes back by readlane (S >= 32)
            const bool act = lane < rl && !(me & 1u) && me - mlo < mhi - mlo;
            const uint64_t actb = ballot(act);
            const uint32_t nact = uint32_t(__popcll(actb));
            const uint32_t ri = me >> 1, g = group_of(ri, pm);
            if (lane < rl) {
                F2Ent en;
                en.x = ((me & 1u) ? 0xFFFFu : ri) | ((lh & 0xFFFFu) << 16);
                en.y = 0u;
                en.mask = mk;
                stage[lane] = en;
            }
            if (act) sact[__popcll(actb & lt)] = F2Act{g | (lane << 16), ((ri - g * per) * D) | ((lh & 0xFFFFu) << 16), mk};
            __builtin_amdgcn_wave_barrier();
            if (nact) {
                const uint32_t lg = rl <= 1 ? 0u : 32u - uint32_t(__clz(rl - 1));  // S = 2^lg >= rl
                const uint32_t S = 1u << lg, k = 64u >> lg;
                const uint32_t j = lane & (S - 1), s0 = lane & ~(S - 1), sub = lane >> lg;
                const uint64_t segm = S == 64 ? ~0ull : (((1ull << S) - 1ull) << s0);
                const uint64_t seg_lt = lt & segm;
                const F2Ent ej = stage[j < rl ? j : 0];
                const bool vj = j < rl && (ej.x & 0xFFFFu) != 0xFFFFu;
                const uint32_t hi_j = uint32_t(__shfl(int(lh), int(j), 64)) >> 16;
                const uint32_t rj2 = (ej.x & 0xFFFFu) << 1;
                F2Act A = sact[min(sub, nact - 1)];
                for (uint32_t i0 = 0; i0 < nact; i0 += k) {
                    const uint32_t ia = i0 + sub;
                    const bool vi = ia < nact;
                    const F2Act An = sact[min(ia + k, nact - 1)];  // the next step's entry
                    const uint32_t gi = A.a & 0xFFFFu, i = A.a >> 16, li = A.b >> 16;
                    const bool t_ok = vi && vj && hi_j > li;
                    const bool e_ok = vi && vj && j > i && (ej.mask & A.mask) != 0ull;
                    const uint64_t tb = ballot(t_ok), eb = ballot(e_ok);
                    const uint32_t nt = uint32_t(__popcll(tb & segm)), n = nt + uint32_t(__popcll(eb & segm));
                    uint32_t off = 0;
                    if (lane == s0 && n) off = atomicAdd(&cur[gi], n);
                    if (S == 64)
                        off = uint32_t(__builtin_amdgcn_readlane(int(off), 0));
                    else if (S == 32) {
                        const uint32_t o0 = uint32_t(__builtin_amdgcn_readlane(int(off), 0));
                        const uint32_t o1 = uint32_t(__builtin_amdgcn_readlane(int(off), 32));
                        off = lane < 32 ? o0 : o1;
                    }
                    else
                        off = uint32_t(__shfl(int(off), int(s0), 64));
                    const uint32_t key = (A.b & 0xFFFFu) + rj2;
                    if (t_ok) keys[off + uint32_t(__popcll(tb & seg_lt))] = uint16_t(key);
                    if (e_ok) keys[off + nt + uint32_t(__popcll(eb & seg_lt))] = uint16_t(key | 1u);
                    A = An;
                }
            }
            __builtin_amdgcn_wave_barrier();
        } else {
            // ---- generic: entry i wave-uniform, partners in chunks of 64 lanes (any W, any length)
            for (uint32_t i = 0; i < rl; ++i) {
                const uint32_t me = rfl(kRoot ? en_.m(rb + i) : mem[rb + i]);
                if ((me & 1u) || !(me - mlo < mhi - mlo)) continue;
                const uint32_t ri = me >> 1, g = group_of(ri, pm);
                const uint32_t li = rfl(en_.lh(rb + i)) & 0xFFFFu;
                const uint32_t kb = (ri - g * per) * D;
                MaskV<W> mi;  // entry i's mask, wave-uniform (by address when W == 0)
                if constexpr (W == 0) {
                    mi.load(mask + size_t(rb + i) * wd, wd);
                } else {
#pragma unroll
                    for (int w = 0; w < W; ++w) {
                        const uint64_t v = mask[size_t(rb + i) * W + w];
                        mi.w[w] = uint64_t(rfl(uint32_t(v))) | (uint64_t(rfl(uint32_t(v >> 32))) << 32);
                    }
                }
                for (uint32_t c0 = 0; c0 < rl; c0 += 64) {
                    const uint32_t q = c0 + lane;
                    const bool v = q < rl;
                    bool t_ok = false, e_ok = false;
                    uint32_t rq = 0;
                    if (v) {
                        const uint32_t mq = kRoot ? en_.m(rb + q) : mem[rb + q];
                        rq = mq >> 1;
                        if (!(mq & 1u)) {
                            t_ok = (en_.lh(rb + q) >> 16) > li;
                            if (q > i) e_ok = mi.and_any(mask + size_t(rb + q) * mask_words<W>(wd), wd);
                        }
                    }
                    const uint64_t tb = ballot(t_ok), eb = ballot(e_ok);
                    const uint32_t nt = uint32_t(__popcll(tb)), n = nt + uint32_t(__popcll(eb));
                    if (n == 0) continue;
                    uint32_t off = 0;
                    if (lane == 0) off = atomicAdd(&cur[g], n);
                    off = rfl(off);
                    const uint32_t key = kb + (rq << 1);
                    if (t_ok) keys[off + uint32_t(__popcll(tb & lt))] = uint16_t(key);
                    if (e_ok) keys[off + nt + uint32_t(__popcll(eb & lt))] = uint16_t(key | 1u);
                }
            }
        }
    }
    __syncthreads();
    // the fills of the groups of the member range [mlo, mhi) only (a pass over other groups
    // leaves theirs as an earlier pass wrote them); the block's key count is their sum
    const uint32_t glo = (mlo >> 1) / per, ghi = mhi == kNone ? G : min(G, ((mhi >> 1) + per - 1) / per);
    for (uint32_t g = glo + threadIdx.x; g < ghi; g += blockDim.x) {
        const uint32_t f = cur[g] - uint32_t(base[f2_region(g, b, nblk)]);
        fill[uint64_t(g) * nblk + b] = f;
        my_keys += f;
    }
    atomicAdd(&blk_keys, my_keys);
    __syncthreads();
    if (threadIdx.x == 0 && blk_keys) atomicAdd(nkeys_total, (unsigned long long)blk_keys);
}

// ---- Root F2 over unordered pairs (the "tri" layout, DB-direct root, W = 1).  The counts
// of the ordered pairs (i -> j) and (j -> i), of the itemset pair (i, j), i < j by rank, and of
// the repeat (i -> i) all sit in the counter tile of the lower rank i: row i holds
// tri_len(i) = 1 + 3 (F - 1 - i) counters [t_ii | for j = i+1 .. F-1: t_ij, t_ji, e_ij].
// Groups are contiguous rank ranges whose rows fit kGroupCounters (gtab[rank] = group << 15 |
// the row's first counter in the group tile).  One test of an unordered pair of a row then
// yields all three of its keys, every key goes to the group of the lower rank, and the
// pairs of a row are folded: a lane segment of S >= n + 1 lanes holds the partners j >= i of
// entry i and those of entry n - 1 - i together, so the enumeration evaluates each unordered
// pair once (half the tests of the ordered scheme) on (nearly) every lane.  A lane takes its
// key slots with one LDS atomic on its group's cursor (the lanes of one entry share it).
__host__ __device__ __forceinline__ uint32_t tri_len(uint32_t F, uint32_t i) { return 1u + 3u * (F - 1u - i); }
// the first counter of row i in a group that starts at row a (rows a .. i - 1 before it)
__host__ __device__ __forceinline__ uint32_t tri_base(uint32_t F, uint32_t a, uint32_t i) {
    const uint32_t m = i - a;
    // sum_{r=a}^{i-1} (1 + 3 (F - 1 - r)); (a + i - 1) m is even (the two factors' sum is odd)
    return m + 3u * (m * (F - 1u) - (a + i - 1u) * m / 2u);
}

// The keys of the unordered pairs (ie, je) of one wave step, je == ie the repeat.  The lanes of
// one entry ie form a contiguous run [st, en] (a sub-segment); its keys take one region cursor
// reservation (the run's first lane), and are written per kind in contiguous blocks: the
// (i -> j) keys of the run, then its (j -> i), then its (i, j) keys.  Lane offsets come from
// mbcnt prefixes packed three to a word (byte fields), the run's totals from the prefixes at
// its ends (two bpermutes), the reserved offset back from the first lane (one bpermute).
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(src << 2), int(v)));
}
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}
// compare lane masks straight from v_cmp (a ballot of a combined bool is materialised as
// v_cndmask + v_cmp first); predicates: LLVM's ICMP_EQ 32, NE 33, ULT 36
__device__ __forceinline__ uint64_t lt_mask(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 36); }
__device__ __forceinline__ uint64_t eq_mask(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 32); }
__device__ __forceinline__ uint64_t nz_mask(uint64_t a) { return __builtin_amdgcn_uicmpl(a, 0ull, 33); }

// M0 / M1 / M2: the lanes with an (i -> j) / (j -> i) / (i, j) key (masks), t0..t2 the same as
// the lane's own conditions
__device__ __forceinline__ void tri_keys(uint64_t M0, uint64_t M1, uint64_t M2, bool t0, bool t1, bool t2,
                                         uint32_t key0, uint32_t grp, uint32_t st, uint32_t en,
                                         uint32_t* __restrict__ cur, uint16_t* __restrict__ keys) {
    if (!(M0 | M1 | M2)) return;  // (wave-uniform)
    const uint32_t pk = mbcnt64(M0) | (mbcnt64(M1) << 8) | (mbcnt64(M2) << 16);
    const uint32_t qk = pk + (uint32_t(t0) | (uint32_t(t1) << 8) | (uint32_t(t2) << 16));
    const uint32_t ps = bperm(pk, st), tot = bperm(qk, en) - ps;
    const uint32_t T0 = tot & 0xFFu, T1 = (tot >> 8) & 0xFFu, T2 = tot >> 16;
    uint32_t off = 0;
    if (lane_id() == st && (T0 | T1 | T2)) off = atomicAdd(&cur[grp], T0 + T1 + T2);
    off = bperm(off, st);
    const uint32_t loc = pk - ps;
    if (t0) keys[off + (loc & 0xFFu)] = uint16_t(key0);
    if (t1) keys[off + T0 + ((loc >> 8) & 0xFFu)] = uint16_t(key0 + 1u);
    if (t2) keys[off + T0 + T1 + (loc >> 16)] = uint16_t(key0 + 2u);
}

// The pair (ie, je) of a row staged in LDS (je == ie: the repeat), okm the lanes with a pair,
// lanes [st, en] sharing ie.  A staged entry is two 8-byte words (two arrays, so the lanes'
// consecutive je read consecutive 8-byte slots, and a 16-byte AoS entry's bank aliasing
// between the folded segments is gone): d.x = 3 rank (mod 2^16) | lo << 16 | hi << 24,
// d.y = (A + kTriA) | group << 16 with A = (first counter of its row) - 3 rank - 2, and the
// mask: the key of (i -> j) is then A_i + 3 rank_j, that of the repeat A_i + 3 rank_i + 2 (the
// row's first counter).
constexpr uint32_t kTriA = 32770u;
__device__ __forceinline__ void tri_pair(uint64_t okm, uint32_t ie, uint32_t je, uint32_t st, uint32_t en,
                                         const uint2* __restrict__ sd, const uint64_t* __restrict__ smk,
                                         uint32_t* __restrict__ cur, uint16_t* __restrict__ keys) {
    const bool ok = (okm >> lane_id()) & 1ull;
    const uint32_t qi = ok ? ie : 0u, qj = ok ? je : 0u;
    const uint2 Di = sd[qi], Dj = sd[qj];
    const uint64_t mm = smk[qi], mj = smk[qj];
    const uint32_t lo_i = (Di.x >> 16) & 0xFFu, hi_i = Di.x >> 24, lo_j = (Dj.x >> 16) & 0xFFu, hi_j = Dj.x >> 24;
    const bool self = je == ie;
    const uint64_t sm = eq_mask(je, ie);
    const uint32_t hs = self ? hi_i : hi_j;
    const uint64_t M0 = okm & lt_mask(lo_i, hs);
    const uint64_t M1 = okm & ~sm & lt_mask(lo_j, hi_i);
    const uint64_t M2 = okm & ~sm & nz_mask(mm & mj);
    const bool t0 = ok && lo_i < hs, t1 = ok && !self && lo_j < hi_i, t2 = ok && !self && (mm & mj) != 0ull;
    const uint32_t key0 = (Di.y & 0xFFFFu) - kTriA + (Dj.x & 0xFFFFu) + (self ? 2u : 0u);
    tri_keys(M0, M1, M2, t0, t1, t2, key0, Di.y >> 16, st, en, cur, keys);
}

__global__ __launch_bounds__(kF2Threads) void k_f2_tri(const uint32_t* __restrict__ row_off32,
                                                      const uint32_t* __restrict__ mem,
                                                      const uint64_t* __restrict__ mask, uint32_t R, uint32_t rpb,
                                                      const uint32_t* __restrict__ gtab, uint32_t G, uint32_t nblk,
                                                      uint32_t mlo, uint32_t mhi, const uint64_t* __restrict__ base,
                                                      uint32_t* __restrict__ fill, uint16_t* __restrict__ keys,
                                                      unsigned long long* __restrict__ nkeys_total) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint2* sd_all = reinterpret_cast<uint2*>(smem);               // kF2Waves x 64 staged entries (tri_pair):
    uint64_t* smk_all = reinterpret_cast<uint64_t*>(sd_all + kF2Waves * 64);  // words, then masks
    uint32_t* srow = smem + kF2Waves * 64 * 4;                     // row offsets of the block [rpb + 1]
    uint32_t* cur = srow + kF2RowWords;                            // region cursors [G]
    __shared__ uint32_t blk_keys;
    const uint32_t b = blockIdx.x;
    const uint32_t r0 = b * rpb, r1 = min(R, r0 + rpb);
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) cur[g] = uint32_t(base[f2_region(g, b, nblk)]);
    for (uint32_t r = r0 + threadIdx.x; r <= r1; r += blockDim.x) srow[r - r0] = row_off32[r];
    if (threadIdx.x == 0) blk_keys = 0;
    __syncthreads();
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    uint2* sd = sd_all + wave * 64;
    uint64_t* smk = smk_all + wave * 64;
    const uint64_t lt = lanemask_lt();
    // the next row's entries are loaded while the current row is enumerated
    uint32_t nrb = 0, nrl = 0, nme = 0;
    uint64_t nmk = 0;
    auto fetch = [&](uint32_t rr) {
        if (rr >= r1) return;
        nrb = srow[rr - r0];
        nrl = srow[rr - r0 + 1] - nrb;
        if (nrl <= 64 && lane < nrl) {
            nme = mem[nrb + lane];
            nmk = mask[nrb + lane];
        }
    };
    fetch(r0 + wave);
    for (uint32_t r = r0 + wave; r < r1; r += kF2Waves) {
        const uint32_t rb = rfl(nrb), rl = rfl(nrl), me = nme;
        const uint64_t mk = nmk;
        fetch(r + kF2Waves);
        if (rl == 0) continue;
        if (rl <= 64) {
            // the row's frequent entries, compacted (positions ascend with the rank); the active
            // ones (this rank's member range) are a contiguous run [a0, a1) of them
            const bool fr = lane < rl && !(me & 1u);
            const bool act = fr && me - mlo < mhi - mlo;
            const uint64_t fb = ballot(fr), ab = ballot(act);
            if (!ab) continue;
            const uint32_t n = uint32_t(__popcll(fb));
            const uint32_t a0 = uint32_t(__popcll(fb & ((1ull << __builtin_ctzll(ab)) - 1ull)));
            const uint32_t a1 = a0 + uint32_t(__popcll(ab));
            if (fr) {
                const uint32_t p = uint32_t(__popcll(fb & lt)), rk = me >> 1;
                const uint32_t gt = act ? gtab[rk] : 0u;
                const uint32_t A = (gt & (kGroupCounters - 1u)) - 3u * rk - 2u + kTriA;  // (active entries only)
                const uint32_t lh = uint32_t(__builtin_ctzll(mk)) | ((63u - uint32_t(__builtin_clzll(mk))) << 8);
                sd[p] = make_uint2(((3u * rk) & 0xFFFFu) | (lh << 16), (A & 0xFFFFu) | ((gt >> kGroupShift) << 16));
                smk[p] = mk;
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t need = 2u * n + 1u - a0 - a1;  // partners of a folded pair of entries
            if (need <= 64u) {
                const uint32_t npairs = (a1 - a0 + 1u) >> 1;
                const uint32_t lg = need <= 1u ? 0u : 32u - uint32_t(__clz(need - 1u));  // S = 2^lg >= need
                const uint32_t k = 64u >> lg, l = lane & ((1u << lg) - 1u), sub = lane >> lg;
                const uint32_t s0 = lane & ~((1u << lg) - 1u), S = 1u << lg;
                for (uint32_t f0 = 0; f0 < npairs; f0 += k) {
                    const uint32_t fp = f0 + sub;
                    const uint32_t iA = a0 + fp, iB = a1 - 1u - fp, cA = min(n - iA, S);
                    const bool second = l >= cA;
                    const uint32_t ie = second ? iB : iA, je = ie + (second ? l - cA : l);
                    const uint64_t sec = ~lt_mask(l, cA);
                    const uint64_t okm = lt_mask(fp, npairs) & lt_mask(je, n) & (~sec | lt_mask(iA, iB));
                    // the run of lanes of ie: [s0, s0 + cA) for iA, [s0 + cA, s0 + S) for iB
                    const uint32_t st = second ? s0 + cA : s0, en = second ? s0 + S - 1u : s0 + cA - 1u;
                    tri_pair(okm, ie, je, st, en, sd, smk, cur, keys);
                }
            } else {
                for (uint32_t i = a0; i < a1; ++i)
                    for (uint32_t c0 = 0; i + c0 < n; c0 += 64) {
                        const uint32_t je = i + c0 + lane;
                        tri_pair(lt_mask(je, n), i, je, 0u, 63u, sd, smk, cur, keys);
                    }
            }
            __builtin_amdgcn_wave_barrier();
        } else {
            // a row of more than 64 entries: entry i wave-uniform, its partners j >= i in chunks
            // of 64 lanes, read from the DB
            for (uint32_t ip = 0; ip < rl; ++ip) {
                const uint32_t mi = rfl(mem[rb + ip]);
                if ((mi & 1u) || !(mi - mlo < mhi - mlo)) continue;
                const uint64_t mki = mask[rb + ip];
                const uint32_t lo_i = uint32_t(__builtin_ctzll(mki)), hi_i = 63u - uint32_t(__builtin_clzll(mki));
                const uint32_t gt = gtab[mi >> 1], ri = mi >> 1;
                for (uint32_t c0 = ip; c0 < rl; c0 += 64) {
                    const uint32_t jp = c0 + lane;
                    bool ok = jp < rl;
                    uint32_t mj = 1u;
                    uint64_t mkj = 1ull;
                    if (ok) {
                        mj = mem[rb + jp];
                        mkj = mask[rb + jp];
                    }
                    ok = ok && !(mj & 1u);
                    const uint32_t lo_j = uint32_t(__builtin_ctzll(mkj)), hi_j = 63u - uint32_t(__builtin_clzll(mkj));
                    const bool self = jp == ip;
                    const bool t0 = ok && lo_i < (self ? hi_i : hi_j);
                    const bool t1 = ok && !self && lo_j < hi_i;
                    const bool t2 = ok && !self && (mki & mkj) != 0ull;
                    const uint32_t key0 = (gt & (kGroupCounters - 1u)) + (self ? 0u : 1u + 3u * ((mj >> 1) - ri - 1u));
                    tri_keys(ballot(t0), ballot(t1), ballot(t2), t0, t1, t2, key0, gt >> kGroupShift, 0u, 63u, cur, keys);
                }
            }
        }
    }
    __syncthreads();
    uint32_t my_keys = 0;
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) {
        const uint32_t f = cur[g] - uint32_t(base[f2_region(g, b, nblk)]);
        fill[uint64_t(g) * nblk + b] = f;
        my_keys += f;
    }
    atomicAdd(&blk_keys, my_keys);
    __syncthreads();
    if (threadIdx.x == 0 && blk_keys) atomicAdd(nkeys_total, (unsigned long long)blk_keys);
}

// One block per rank group.  The group's regions (one per row block, each
// starting on a 16-byte boundary, holes after their fills) are read as one
// logical stream of 8-key chunks: the block loads the regions' fills and
// bases into LDS and prefix-sums their chunk counts; every thread then takes
// 4 chunks per round (4 independent 16-byte loads in flight), finds each
// chunk's region by binary search in LDS and adds its keys into the LDS
// counters.  Then the frequent pairs of the group's counter rows
// [max(g*per, rlo), min((g+1)*per, rhi)) are balloted out with one atomic per
// wave; records come out unordered and the host sorts them.
// kOut (the keyed class count): the group's kGroupCounters counters are written
// out to cnt_out[g * kGroupCounters ...] instead of extracted.
constexpr uint32_t kF2MaxBlocks = 2048;  // row blocks (regions per group) k_f2_count can index in LDS
// kTri: the unordered-pair layout (k_f2_tri): group g holds rows tri_gr[g] .. tri_gr[g + 1] of
// tri_len(F, i) counters each, decoded back to ordered (row, slot) records at the extraction.
template <bool kOut, bool kTri = false>
__global__ __launch_bounds__(kF2Threads) void k_f2_count(const uint64_t* __restrict__ base,
                                                         const uint32_t* __restrict__ fill, uint32_t nblk,
                                                         const uint16_t* __restrict__ keys, uint32_t D, uint32_t per,
                                                         uint32_t g0, uint32_t rlo, uint32_t rhi, uint32_t minsup,
                                                         FreqRec* __restrict__ recs, uint32_t cap,
                                                         uint32_t* __restrict__ nrec, uint32_t* __restrict__ cnt_out,
                                                         uint32_t parts, const uint32_t* __restrict__ tri_gr = nullptr,
                                                         uint32_t triF = 0) {
    __shared__ uint32_t h[kGroupCounters];
    __shared__ uint32_t cpre[kF2MaxBlocks + 1];  // first logical chunk of each region
    __shared__ uint32_t cst[kF2MaxBlocks];       // first physical chunk of each region
    __shared__ uint32_t sfill[kF2MaxBlocks];     // keys in each region
    __shared__ uint32_t wsum[kF2Waves];
    // kOut with parts > 1: `parts` blocks share a group, each over its own range of regions
    const uint32_t g = g0 + blockIdx.x / parts, part = blockIdx.x % parts;
    const uint32_t rb0 = uint32_t(uint64_t(nblk) * part / parts), rb1 = uint32_t(uint64_t(nblk) * (part + 1) / parts);
    const uint32_t nr = rb1 - rb0;
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    const uint32_t nz = kOut ? kGroupCounters : (kTri ? tri_base(triF, tri_gr[g], tri_gr[g + 1]) : per * D);
    for (uint32_t t = threadIdx.x; t < nz; t += blockDim.x) h[t] = 0;
    // region chunk counts -> exclusive prefix (nblk <= 2 * blockDim.x: two per thread)
    const uint64_t gi = uint64_t(g) * nblk + rb0;
    const uint32_t s0 = 2 * threadIdx.x;
    const uint32_t f0 = s0 < nr ? fill[gi + s0] : 0u, f1 = s0 + 1 < nr ? fill[gi + s0 + 1] : 0u;
    if (s0 < nr) {
        cst[s0] = uint32_t(base[f2_region(g, rb0 + s0, nblk)]) >> 3;
        sfill[s0] = f0;
    }
    if (s0 + 1 < nr) {
        cst[s0 + 1] = uint32_t(base[f2_region(g, rb0 + s0 + 1, nblk)]) >> 3;
        sfill[s0 + 1] = f1;
    }
    const uint32_t c0 = (f0 + 7) >> 3, c1 = (f1 + 7) >> 3;
    const uint32_t pair = c0 + c1, incl = wave_incl_scan(pair);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t woff = 0, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < kF2Waves; ++w) {
        woff += w < wave ? wsum[w] : 0u;
        total += wsum[w];
    }
    const uint32_t ex = woff + incl - pair;
    if (s0 < nr) cpre[s0] = ex;
    if (s0 + 1 < nr) cpre[s0 + 1] = ex + c0;
    if (threadIdx.x == 0) cpre[nr] = total;
    __syncthreads();
    const uint4* kv = reinterpret_cast<const uint4*>(keys);
    constexpr uint32_t kU = 4;  // chunks per thread per round
    for (uint32_t q0 = threadIdx.x; q0 < total; q0 += kF2Threads * kU) {
        uint4 v[kU];
        uint32_t nv[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t c = q0 + u * kF2Threads;
            nv[u] = 0;
            if (c < total) {
                uint32_t lo = 0, hi = nr;  // region of c: the last s with cpre[s] <= c
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (cpre[mid] <= c) lo = mid; else hi = mid;
                }
                const uint32_t k = c - cpre[lo];
                nv[u] = min(8u, sfill[lo] - 8 * k);
                v[u] = kv[cst[lo] + k];
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q)
                if (q < nv[u]) atomicAdd(&h[(w[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu], 1u);
        }
    }
    __syncthreads();
    if constexpr (kOut) {
        uint32_t* o = cnt_out + uint64_t(g) * kGroupCounters;
        if (parts == 1) {  // the group's only block: every counter written (no memset)
            const uint4* hv = reinterpret_cast<const uint4*>(h);
            for (uint32_t t = threadIdx.x; t < kGroupCounters / 4; t += blockDim.x) reinterpret_cast<uint4*>(o)[t] = hv[t];
        } else {  // shared group (zeroed beforehand): contiguous adds of the non-zero counters
            for (uint32_t t = threadIdx.x; t < kGroupCounters; t += blockDim.x)
                if (h[t]) atomicAdd(o + t, h[t]);
        }
        return;
    }
    if constexpr (kTri) {
        // counter c of the tile: row i = the last row whose first counter is <= c; then the repeat
        // (i -> i) or, for the partner j = i + 1 + q / 3, (i -> j), (j -> i), (i, j) by q % 3
        const uint32_t a = tri_gr[g], z = tri_gr[g + 1];
        for (uint32_t c0 = wave * 64; c0 < nz; c0 += kF2Threads) {
            const uint32_t c = c0 + lane;
            const uint32_t val = c < nz ? h[c] : 0u;
            const bool fr = c < nz && val >= minsup;
            const uint64_t fb = ballot(fr);
            if (!fb) continue;
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(nrec, uint32_t(__popcll(fb)));
            at = rfl(at) + uint32_t(__popcll(fb & lanemask_lt()));
            if (fr && at < cap) {
                uint32_t lo = a, hi = z;  // tri_base(F, a, lo) <= c < tri_base(F, a, hi)
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (tri_base(triF, a, mid) <= c) lo = mid; else hi = mid;
                }
                const uint32_t off = c - tri_base(triF, a, lo);
                FreqRec rc{lo, 2u * lo, val, 0u};  // the repeat: (i -> i), a sequence-extension
                if (off) {
                    const uint32_t q = off - 1u, j = lo + 1u + q / 3u, code = q % 3u;
                    rc = code == 0 ? FreqRec{lo, 2u * j, val, 0u}
                                   : (code == 1 ? FreqRec{j, 2u * lo, val, 0u} : FreqRec{lo, 2u * j + 1u, val, 0u});
                }
                recs[at] = rc;
            }
        }
        return;
    }
    const uint32_t ra = max(g * per, rlo), rz = min((g + 1) * per, rhi);
    for (uint32_t row = ra; row < rz; ++row) {
        const uint32_t* hr = h + (row - g * per) * D;
        for (uint32_t cc = wave * 64; cc < D; cc += kF2Threads) {
            const uint32_t c = cc + lane;
            const uint32_t val = c < D ? hr[c] : 0u;
            const bool fr = c < D && val >= minsup;
            const uint64_t fb = ballot(fr);
            if (!fb) continue;
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(nrec, uint32_t(__popcll(fb)));
            at = rfl(at) + uint32_t(__popcll(fb & lanemask_lt()));
            if (fr && at < cap) recs[at] = FreqRec{row, c, val, 0u};
        }
    }
}

// Child class of every member slot x of a batch, from its kids CSR (unsharded
// runs): the children are created in slot order, one per slot with kids except
// a slot whose only kid is an itemset-extension (count_and_freq), so the child
// index of slot x is the number of such slots before it.  k_child_flag marks
// them, a scan numbers them, k_child_of writes the index relative to the
// emitted group [ga, gb) or kNone (no host table, no upload per emit).
__device__ __forceinline__ uint32_t child_flag(const uint32_t* __restrict__ koff, const uint32_t* __restrict__ kslot,
                                               uint32_t x) {
    const uint32_t a = koff[x], n = koff[x + 1] - a;
    return n > 1 || (n == 1 && (kslot[a] & 1u) == kSeq) ? 1u : 0u;
}
__global__ __launch_bounds__(kBlock) void k_child_flag(const uint32_t* __restrict__ koff,
                                                       const uint32_t* __restrict__ kslot, uint32_t n,
                                                       uint32_t* __restrict__ flag) {
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x)
        flag[x] = child_flag(koff, kslot, x);
}
__global__ __launch_bounds__(kBlock) void k_child_of(const uint32_t* __restrict__ koff,
                                                     const uint32_t* __restrict__ kslot,
                                                     const uint64_t* __restrict__ pre, uint32_t n, uint32_t ga,
                                                     uint32_t gb, uint32_t* __restrict__ child_of) {
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
        const uint32_t c = uint32_t(pre[x]);
        child_of[x] = child_flag(koff, kslot, x) && c >= ga && c < gb ? c - ga : kNone;
    }
}

// Ordered frequent extraction (large batches): k_freq_count -> scan -> k_freq_write
// gives the records in (row, slot) order with their child ids, no host ordering.
__global__ __launch_bounds__(kBlock) void k_freq_count(const DRow* __restrict__ rows, uint32_t nrows,
                                                       const DClass* __restrict__ cls, const uint32_t* __restrict__ cnt,
                                                       uint32_t minsup, uint32_t* __restrict__ rowcnt) {
    const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (g >= nrows) return;
    const DRow r = rows[g];
    const DClass c = cls[r.cls];
    const uint32_t* base = cnt + c.cnt_off + uint64_t(r.mi >> c.mshift) * c.rstride;
    uint32_t n = 0;
    for (uint32_t s = 0; s < c.D; s += 64) {
        const uint32_t slot = s + lane_id();
        const uint32_t v = slot < c.D ? base[slot] : 0u;
        n += __popcll(ballot(v >= minsup));
    }
    if (lane_id() == 0) rowcnt[g] = n;
}

__global__ __launch_bounds__(kBlock) void k_freq_write(const DRow* __restrict__ rows, uint32_t nrows,
                                                       const DClass* __restrict__ cls, const uint32_t* __restrict__ cnt,
                                                       uint32_t minsup, const uint64_t* __restrict__ rowoff,
                                                       uint32_t row_base, FreqRec* __restrict__ out,
                                                       uint32_t* __restrict__ kslot, uint32_t* __restrict__ kcid) {
    const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (g >= nrows) return;
    const DRow r = rows[g];
    const DClass c = cls[r.cls];
    const uint32_t* base = cnt + c.cnt_off + uint64_t(r.mi >> c.mshift) * c.rstride;
    uint64_t o = rowoff[g];
    uint32_t nrank = 0;
    const unsigned lane = lane_id();
    const uint64_t lead_lt = (1ull << (lane & ~1u)) - 1ull;
    for (uint32_t s = 0; s < c.D; s += 64) {
        const uint32_t slot = s + lane;
        const uint32_t v = slot < c.D ? base[slot] : 0u;
        const bool fr = slot < c.D && v >= minsup;
        const bool partner = __shfl_xor(int(fr), 1, 64) != 0;
        const uint64_t lead = ballot((fr || partner) && !(lane & 1u));
        const uint32_t crank = nrank + uint32_t(__popcll(lead & lead_lt));
        const uint64_t fb = ballot(fr);
        if (fr) {
            const uint64_t q = o + __popcll(fb & lanemask_lt());
            out[q] = FreqRec{row_base + g, slot, v, crank << 1 | (slot & 1u)};
            if (kslot) {  // the batch's kid table, straight into HBM (unsharded)
                kslot[q] = slot;
                kcid[q] = crank << 1 | (slot & 1u);
            }
        }
        o += uint64_t(__popcll(fb));
        nrank += uint32_t(__popcll(lead));
    }
}

// Kid offsets of every member slot x (CSR over cbase + mi): row g (slots ascend with
// the rows) writes rowoff[g] over the slots after the previous row's up to its own;
// the last row also closes the table (slots past it: nfreq).
__global__ __launch_bounds__(kBlock) void k_kid_off(const DRow* __restrict__ rows, uint32_t nrows,
                                                    const DClass* __restrict__ cls, const uint64_t* __restrict__ rowoff,
                                                    uint32_t nko, uint32_t* __restrict__ koff) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nrows) return;
    const DRow r = rows[g];
    const uint32_t x = cls[r.cls].cbase + r.mi;
    uint32_t a = 0;
    if (g > 0) {
        const DRow p = rows[g - 1];
        a = cls[p.cls].cbase + p.mi + 1;
    }
    const uint32_t v = uint32_t(rowoff[g]);
    for (uint32_t y = a; y <= x; ++y) koff[y] = v;
    if (g + 1 == nrows) {
        const uint32_t n = uint32_t(rowoff[nrows]);
        for (uint32_t y = x + 1; y < nko; ++y) koff[y] = n;
    }
}

// One-pass frequent extraction: one wave per counter row ballots the frequent
// candidates and appends FreqRec{row, slot, sup} at a block cursor reserved with
// one global atomic per block (unordered; the host orders them, order_recs).
// More than `cap` records: only counted (the host retries with the exact size).
__global__ __launch_bounds__(kBlock) void k_freq_recs(const DRow* __restrict__ rows, uint32_t nrows,
                                                      const DClass* __restrict__ cls, const uint32_t* __restrict__ cnt,
                                                      uint32_t minsup, uint32_t row_base, FreqRec* __restrict__ out,
                                                      uint32_t cap, uint32_t* __restrict__ nout) {
    __shared__ uint32_t w_n[kBlock / 64];
    __shared__ uint32_t b_at;
    const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const bool live = g < nrows;
    DRow r{0, 0};
    DClass c{0, 0, 0, 0, 0, {0, 0}};
    const uint32_t* base = cnt;
    uint32_t n = 0;
    if (live) {
        r = rows[g];
        c = cls[r.cls];
        base = cnt + c.cnt_off + uint64_t(r.mi >> c.mshift) * c.rstride;
        for (uint32_t s0 = 0; s0 < c.D; s0 += 64) {
            const uint32_t slot = s0 + lane;
            n += uint32_t(__popcll(ballot(slot < c.D && base[slot] >= minsup)));
        }
    }
    if (lane == 0) w_n[wv] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t k = 0; k < blockDim.x / 64; ++k) tot += w_n[k];
        b_at = tot ? atomicAdd(nout, tot) : 0u;
    }
    __syncthreads();
    if (!live || n == 0) return;
    uint32_t at = b_at;
    for (uint32_t k = 0; k < wv; ++k) at += w_n[k];
    for (uint32_t s0 = 0; s0 < c.D; s0 += 64) {
        const uint32_t slot = s0 + lane;
        const uint32_t v = slot < c.D ? base[slot] : 0u;
        const bool fr = slot < c.D && v >= minsup;
        const uint64_t fb = ballot(fr);
        const uint32_t x = at + uint32_t(__popcll(fb & lanemask_lt()));
        if (fr && x < cap) out[x] = FreqRec{row_base + g, slot, v, 0u};
        at += uint32_t(__popcll(fb));
    }
}

// Child rows.  Entry i (member mi, class c, sequence s) produces the whole
// run of sequence s in the child class [c, mi]: one entry per frequent child of
// mi whose join with i is non-empty (partner j found by binary search in the
// member-sorted run), in child member order.  Runs are written in parent entry
// order at exclusive-scan offsets, so every block writes one contiguous,
// coalesced stretch (no per-class cursors, no partial-line scatter).
//
// Work is flattened to (entry, kid) pairs per wave: the 64 entries of a wave
// expose their kid counts, a wave prefix sum numbers the pairs, and each lane
// takes one pair per step (owner found by a 6-step shuffle search).  Kid counts
// are heavily skewed (popular members have dozens of frequent children), so a
// thread-per-entry loop would leave most lanes idle behind the longest list.

// one lane's parent entry for the flattened (entry, kid) pair loop
struct EmitEnt {
    uint32_t k0, nk, cc, rb, re, lt;  // kids [k0, k0 + nk), child class, run [rb, re), lo | type << 16
};

template <class EntT>
__device__ __forceinline__ EmitEnt emit_ent(uint64_t e64, uint32_t E, const EntT& en, const DClass* __restrict__ cls,
                                            const uint32_t* __restrict__ pos, const uint32_t* __restrict__ kid_off,
                                            const uint32_t* __restrict__ child_of) {
    EmitEnt t{0, 0, kNone, 0, 0, 0};
    if (e64 < E) {
        const uint32_t e = uint32_t(e64);
        const DClass c = cls[en.c(e)];
        const uint32_t mi = en.m(e);
        t.cc = EntT::kRootEnt && (mi & 1u) ? kNone : child_of[c.cbase + mi];  // (infrequent DB entry: no class)
        if (t.cc != kNone) {
            t.k0 = kid_off[c.cbase + mi];
            t.nk = kid_off[c.cbase + mi + 1] - t.k0;
            const uint32_t p = pos[e];
            t.rb = e - (p >> 16);
            t.re = t.rb + (p & 0xFFFFu);
            t.lt = (en.lh(e) & 0xFFFFu) | ((mi & 1u) << 16);
        }
    }
    return t;
}

// The pair loop of one wave over its 64 entries (entry w0 + lane): every
// (entry, kid) pair binary-searches its partner in the member-sorted run and
// tests the join.  on_ok(ok, owner lane, owner entry, owner lo|type, kid q,
// partner f, kid slot, k) runs on EVERY lane each step (it may shuffle); k is
// the rank of a non-empty join within the owner's child run.  Returns the
// lane's own non-empty join count (its child run length).
template <int W, class EntT, class OnOk>
__device__ __forceinline__ uint32_t emit_pairs(const EmitEnt& t, uint64_t w0, const EntT& en,
                                               const uint64_t* __restrict__ mask,
                                               const uint32_t* __restrict__ kid_slot, uint32_t wd, OnOk&& on_ok) {
    const uint32_t lane = lane_id();
    const uint32_t incl = wave_incl_scan(t.nk), excl = incl - t.nk;
    const uint32_t total = uint32_t(__shfl(int(incl), 63, 64));
    uint32_t done = 0;  // this lane's (as owner) non-empty joins so far
    for (uint32_t p0 = 0; p0 < total; p0 += 64) {
        const uint32_t pp = p0 + lane;
        // owner: the largest lane whose first pair index <= pp
        uint32_t ow = 0;
#pragma unroll
        for (uint32_t step = 32; step > 0; step >>= 1) {
            const uint32_t cand = ow + step;
            if (uint32_t(__shfl(int(excl), int(cand), 64)) <= pp) ow = cand;
        }
        const uint32_t o_k0 = uint32_t(__shfl(int(t.k0), int(ow), 64));
        const uint32_t o_ex = uint32_t(__shfl(int(excl), int(ow), 64));
        const uint32_t o_rb = uint32_t(__shfl(int(t.rb), int(ow), 64));
        const uint32_t o_re = uint32_t(__shfl(int(t.re), int(ow), 64));
        const uint32_t o_lt = uint32_t(__shfl(int(t.lt), int(ow), 64));
        const uint32_t o_done = uint32_t(__shfl(int(done), int(ow), 64));
        const uint64_t o_e = w0 + ow;
        bool ok = false;
        uint32_t q = 0, f = 0, slot = 0;
        if (pp < total) {
            q = o_k0 + (pp - o_ex);
            slot = kid_slot[q];
            const uint32_t ct = slot & 1u;
            const uint32_t target = (slot & ~1u) | (ct == kSeq ? 0u : (o_lt >> 16));  // partner member id
            uint32_t lo = o_rb, hi = o_re;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (mem_less(en.m(mid), target)) lo = mid + 1; else hi = mid;
            }
            f = lo;
            if (f < o_re && en.m(f) == target) {
                const uint32_t f_lh = en.lh(f);
                if (ct == kSeq) {
                    ok = (f_lh >> 16) > (o_lt & 0xFFFFu);
                } else {
                    MaskV<W> mk;
                    mk.load(mask + size_t(o_e) * mask_words<W>(wd), wd, en.lh(o_e));
                    ok = mk.and_any(mask + size_t(f) * mask_words<W>(wd), wd, f_lh);
                }
            }
        }
        const uint64_t succ = ballot(ok);
        const uint32_t first = (o_ex > p0 ? o_ex : p0) - p0;  // owner's first lane in this step
        const uint32_t k = o_done + uint32_t(__popcll(succ & lane_range(first, lane)));
        on_ok(ok, ow, o_e, o_lt, q, f, slot, k);
        // each lane, as owner, adds its joins of this step
        const uint32_t a = (excl > p0 ? excl : p0), bnd = (incl < p0 + 64 ? incl : p0 + 64);
        if (bnd > a) done += uint32_t(__popcll(succ & lane_range(a - p0, bnd - p0)));
    }
    return done;
}

// one child entry: the join of parent entry o_e with partner f at slab slot d
template <int W>
__device__ __forceinline__ void emit_write(const SlabPtrs& o, uint64_t cap, uint64_t d, uint32_t cc, uint32_t kidc, uint32_t k,
                                           uint32_t n, uint64_t o_e, uint32_t o_lt, uint32_t f, uint32_t slot,
                                           const uint32_t* __restrict__ lohi, const uint64_t* __restrict__ mask,
                                           uint32_t wd) {
    if (d >= cap) return;  // a count mismatch: the host reports it, nothing lands past the slab
    if (n > 0xFFFFu) {  // a child run longer than the 16-bit pos fields: the host raises FSM_ELIMIT
        atomicOr(o.lim, 1u);
        return;
    }
    if constexpr (W == 0) {  // runtime width: word by word through HBM
        const uint64_t* src = mask + size_t(f) * wd;
        uint64_t* dst = o.mask + d * wd;
        uint32_t lo2 = 0xFFFFFFFFu, hi2 = 0;
        if ((slot & 1u) == kSeq) {
            hi2 = lohi[f] >> 16;
            const int lo = int(o_lt & 0xFFFFu);
            for (uint32_t k = 0; k < wd; ++k) {
                const int sh = lo + 1 - int(k) * 64;  // bits [0, sh) of word k are cleared
                const uint64_t v = src[k] & (sh <= 0 ? ~0ull : (sh >= 64 ? 0ull : (~0ull << sh)));
                dst[k] = v;
                if (v && lo2 == 0xFFFFFFFFu) lo2 = k * 64 + uint32_t(__builtin_ctzll(v));
            }
        } else {
            const uint64_t* mk = mask + size_t(o_e) * wd;
            for (uint32_t k = 0; k < wd; ++k) {
                const uint64_t v = src[k] & mk[k];
                dst[k] = v;
                if (v) {
                    if (lo2 == 0xFFFFFFFFu) lo2 = k * 64 + uint32_t(__builtin_ctzll(v));
                    hi2 = k * 64 + 63 - uint32_t(__builtin_clzll(v));
                }
            }
        }
        o.cid[d] = cc;
        o.mem[d] = kidc;
        o.lohi[d] = (lo2 == 0xFFFFFFFFu ? 0u : lo2) | (hi2 << 16);
        o.pos[d] = (k << 16) | n;
        return;
    } else {
    uint64_t m[W];
    load_mask<W>(mask + size_t(f) * W, m);
    uint32_t lo2, hi2;
    if ((slot & 1u) == kSeq) {
        hi2 = mask_hi<W>(m);  // the partner's last eid (its lohi; the DB-direct root has none stored)
        mask_clear_upto<W>(m, o_lt & 0xFFFFu);
        lo2 = mask_lo<W>(m);
    } else {
        uint64_t mk[W];
        load_mask<W>(mask + size_t(o_e) * W, mk);
#pragma unroll
        for (int x = 0; x < W; ++x) m[x] &= mk[x];
        lo2 = mask_lo<W>(m);
        hi2 = mask_hi<W>(m);
    }
    o.cid[d] = cc;
    o.mem[d] = kidc;
    if constexpr (!kLhDerived<W>) o.lohi[d] = lo2 | (hi2 << 16);
    o.pos[d] = (k << 16) | n;
    store_mask<W>(o.mask + d * W, m);
    }
}

// One-pass emission (default).  A block takes a chunk of kEmitRounds x 256
// parent entries; each wave joins its entries once, keeping every non-empty
// join (partner, kid, owner, rank in run) in LDS, then the block reserves its
// child entries with ONE atomic on the slab cursor and writes the runs from
// LDS.  Child runs stay contiguous and member-sorted; only their order in the
// slab follows the chunks' reservation order, which nothing downstream reads
// (k_count and k_emit address runs through pos).  A wave whose joins overflow
// its rcap (<= kEmitCap) LDS records joins again in the write phase.
#ifndef FSM_EMIT_ROUNDS
#define FSM_EMIT_ROUNDS 2
#endif
#ifndef FSM_EMIT_BLOCK
#define FSM_EMIT_BLOCK 256
#endif
constexpr int kEmitBlock = FSM_EMIT_BLOCK;  // threads of a k_emit1 block (one slab reservation per chunk)
#ifndef FSM_EMIT_RECORDS
#define FSM_EMIT_RECORDS 256
#endif
constexpr int kEmitRounds = FSM_EMIT_ROUNDS;      // 64-entry rounds per wave per chunk
constexpr uint32_t kEmitCap = FSM_EMIT_RECORDS;  // LDS join records per wave

template <int W, bool kRoot>
__global__ __launch_bounds__(kEmitBlock) void k_emit1(uint32_t E, RootRef rr, const uint32_t* __restrict__ cid,
                                                  const DClass* __restrict__ cls, const uint32_t* __restrict__ mem,
                                                  const uint32_t* __restrict__ lohi, const uint32_t* __restrict__ pos,
                                                  const uint64_t* __restrict__ mask,
                                                  const uint32_t* __restrict__ kid_off,
                                                  const uint32_t* __restrict__ kid_slot,
                                                  const uint32_t* __restrict__ kid_cid,
                                                  const uint32_t* __restrict__ child_of,
                                                  unsigned long long* __restrict__ cursor, SlabPtrs o,
                                                  uint64_t cap, uint32_t rcap, uint32_t wd,
                                                  const uint32_t* __restrict__ runs, const uint32_t* __restrict__ nruns) {
    constexpr uint32_t kWaves = kEmitBlock / 64;
    constexpr uint32_t kPer = 64 * kEmitRounds;  // entries of one wave per chunk
    __shared__ uint32_t r_f[kWaves][kEmitCap], r_q[kWaves][kEmitCap], r_ek[kWaves][kEmitCap];
    __shared__ uint32_t i_n[kWaves][kPer], i_off[kWaves][kPer], i_cc[kWaves][kPer], i_lt[kWaves][kPer];
    __shared__ uint32_t w_tot[kWaves];
    __shared__ unsigned long long b_base;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint64_t chunk = uint64_t(kEmitBlock) * kEmitRounds;
    const Ent<W == 0 ? 1 : W, kRoot, W> en{cid, mem, lohi, mask, rr};
    // segments: the whole batch [0, E), or (runs != nullptr) each listed run, one block per run
    const uint32_t nseg = runs ? *nruns : 1u;
    for (uint32_t sg = runs ? blockIdx.x : 0u; sg < nseg; sg += runs ? gridDim.x : nseg) {
    const uint32_t sa = runs ? runs[sg] : 0u;
    const uint32_t Ez = runs ? sa + (pos[sa] & 0xFFFFu) : E;  // segment end
    for (uint64_t c0 = runs ? uint64_t(sa) : uint64_t(blockIdx.x) * chunk; c0 < Ez;
         c0 += runs ? chunk : uint64_t(gridDim.x) * chunk) {
        uint32_t nrec = 0, wsum = 0;
        for (int r = 0; r < kEmitRounds; ++r) {
            const uint64_t w0 = c0 + uint64_t(r) * kEmitBlock + uint64_t(w) * 64;
            const EmitEnt t = emit_ent(w0 + lane, Ez, en, cls, pos, kid_off, child_of);
            const uint32_t done = emit_pairs<W>(
                t, w0, en, mask, kid_slot, wd,
                [&](bool ok, uint32_t ow, uint64_t, uint32_t, uint32_t q, uint32_t f, uint32_t, uint32_t k) {
                    const uint64_t b = ballot(ok);
                    if (ok) {
                        const uint32_t x = nrec + uint32_t(__popcll(b & lanemask_lt()));
                        if (x < rcap) {
                            r_f[w][x] = f;
                            r_q[w][x] = q;
                            r_ek[w][x] = ((uint32_t(r) * 64u + ow) << 16) | k;
                        }
                    }
                    nrec += uint32_t(__popcll(b));
                });
            const uint32_t incl = wave_incl_scan(done);
            const uint32_t el = uint32_t(r) * 64u + lane;
            i_n[w][el] = done;
            i_off[w][el] = wsum + incl - done;
            i_cc[w][el] = t.cc;
            i_lt[w][el] = t.lt;
            wsum += uint32_t(__shfl(int(incl), 63, 64));
        }
        if (lane == 0) w_tot[w] = wsum;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long tot = 0;
            for (uint32_t k = 0; k < kWaves; ++k) tot += w_tot[k];
            b_base = tot ? atomicAdd(cursor, tot) : 0ull;
        }
        __syncthreads();
        uint64_t wb = b_base;
        for (uint32_t k = 0; k < w; ++k) wb += w_tot[k];
        if (nrec <= rcap) {
            for (uint32_t x = lane; x < nrec; x += 64) {
                const uint32_t f = r_f[w][x], q = r_q[w][x], ek = r_ek[w][x];
                const uint32_t el = ek >> 16, k = ek & 0xFFFFu;
                const uint64_t o_e = c0 + uint64_t(el >> 6) * kEmitBlock + uint64_t(w) * 64 + (el & 63u);
                emit_write<W>(o, cap, wb + i_off[w][el] + k, i_cc[w][el], kid_cid[q], k, i_n[w][el], o_e, i_lt[w][el], f,
                              kid_slot[q], lohi, mask, wd);
            }
        } else {
            for (int r = 0; r < kEmitRounds; ++r) {
                const uint64_t w0 = c0 + uint64_t(r) * kEmitBlock + uint64_t(w) * 64;
                EmitEnt t = emit_ent(w0 + lane, Ez, en, cls, pos, kid_off, child_of);
                const uint32_t el = uint32_t(r) * 64u + lane;
                const uint64_t base = wb + i_off[w][el];
                const uint32_t n_run = i_n[w][el];
                if (n_run == 0) t.nk = 0;
                emit_pairs<W>(t, w0, en, mask, kid_slot, wd,
                              [&](bool ok, uint32_t ow, uint64_t o_e, uint32_t o_lt, uint32_t q, uint32_t f,
                                  uint32_t slot, uint32_t k) {
                                  const uint32_t o_n = uint32_t(__shfl(int(n_run), int(ow), 64));
                                  const uint64_t o_base = __shfl(base, int(ow), 64);
                                  const uint32_t o_cc = uint32_t(__shfl(int(t.cc), int(ow), 64));
                                  if (ok)
                                      emit_write<W>(o, cap, o_base + k, o_cc, kid_cid[q], k, o_n, o_e, o_lt, f, slot, lohi,
                                                    mask, wd);
                              });
            }
        }
        __syncthreads();  // the LDS records are reused by the next chunk
    }
    }
}

// Window emission (W = 1).  k_emit1's partner lookups are dependent binary
// searches in HBM (86 % of wave cycles waiting); here each wave
// owns the runs STARTING in a 128-entry range of the batch and walks them in
// windows of whole runs of at most 64 entries held in registers (one entry per
// lane: member, lohi, mask).  An (entry, kid) pair finds its partner with a
// fixed 6-step shuffle lower_bound over the owner's run and takes the
// partner's lohi / mask by shuffle: no memory access between a kid's slot and
// its join result.  Join records stay in per-wave LDS (as k_emit1), the block
// reserves its child entries with one slab-cursor atomic per 512-entry chunk
// and writes the runs; a wave whose records overflow joins again while writing.
// Runs longer than 64 entries are appended to `longl` for k_emit1's run list.
// W > 1 (up to 8 words): the same windows; an equality join reads the owner's and
// the partner's masks at their known slab slots (no search), after the eid-range
// overlap test on the lohi words it already holds.
#ifndef FSM_E2_RANGE
#define FSM_E2_RANGE 192
#endif
#ifndef FSM_E2_RANGE_ROOT
#define FSM_E2_RANGE_ROOT 128
#endif
#ifndef FSM_E2_CAP
#define FSM_E2_CAP 192
#endif
#ifndef FSM_E2_BLOCK
#define FSM_E2_BLOCK 512
#endif
#ifndef FSM_E2_BLOCK_ROOT
#define FSM_E2_BLOCK_ROOT 256
#endif
// threads per block, by kind (round 6, rocprof per D1M mine: the root 0.56 ms at 256 vs 0.61 at
// 512; W = 1 lattice batches 0.32 at 256 vs 0.29 at 512; 128 is slower for both; BIBLE's W = 8
// batches are slower at 512: 256 kept there)
#ifndef FSM_E2_BLOCK_W
#define FSM_E2_BLOCK_W FSM_E2_BLOCK_ROOT
#endif
#ifndef FSM_E2_RANGE_W
#define FSM_E2_RANGE_W 64  // W > 1 lattice batches (BIBLE k_emit2<8>: 64 -6 % vs 128, 192 +6 %; rocprof)
#endif
template <bool kRoot, int W> constexpr int e2_block() {
    return kRoot ? FSM_E2_BLOCK_ROOT : (W != 1 ? FSM_E2_BLOCK_W : FSM_E2_BLOCK);
}
// entries per wave range (runs starting in it; a multiple of 64): the DB-direct root's rows are
// short runs of one class, best at 128; a W = 1 lattice batch's at 192 (round 6: rocprof per
// kernel, root 0.55 vs 0.60 ms, lattice 0.41 vs 0.32 ms per D1M mine); W > 1 lattice batches 64
static_assert(FSM_E2_RANGE % 64 == 0 && FSM_E2_RANGE_ROOT % 64 == 0, "k_emit2 wave ranges are whole lane steps");
static_assert(FSM_E2_RANGE_W % 64 == 0, "k_emit2 wave ranges are whole lane steps");
template <bool kRoot, int W> constexpr uint32_t e2_range() {
    return kRoot ? FSM_E2_RANGE_ROOT : (W != 1 ? FSM_E2_RANGE_W : FSM_E2_RANGE);
}
// owner slots per wave (a run may end 63 past the range)
template <bool kRoot, int W> constexpr uint32_t e2_own() { return e2_range<kRoot, W>() + 64; }
constexpr uint32_t kE2Cap = FSM_E2_CAP;         // LDS join records per wave

template <int W, bool kRoot>
__global__ __launch_bounds__((e2_block<kRoot, W>())) void k_emit2(uint32_t E, RootRef rr, const uint32_t* __restrict__ cid,
                                                    const DClass* __restrict__ cls, const uint32_t* __restrict__ mem,
                                                    const uint32_t* __restrict__ lohi, const uint32_t* __restrict__ pos,
                                                    const uint64_t* __restrict__ mask,
                                                    const uint32_t* __restrict__ kid_off,
                                                    const uint32_t* __restrict__ kid_slot,
                                                    const uint32_t* __restrict__ kid_cid,
                                                    const uint32_t* __restrict__ child_of,
                                                    unsigned long long* __restrict__ cursor, SlabPtrs o, uint64_t cap,
                                                    uint32_t rcap, uint32_t* __restrict__ longl,
                                                    uint32_t* __restrict__ nlong) {
    constexpr uint32_t kE2Waves = uint32_t(e2_block<kRoot, W>()) / 64;
    __shared__ uint32_t r_f[kE2Waves][kE2Cap], r_q[kE2Waves][kE2Cap], r_ek[kE2Waves][kE2Cap];
    constexpr uint32_t kE2Range = e2_range<kRoot, W>(), kE2Own = e2_own<kRoot, W>();
    __shared__ uint32_t i_n[kE2Waves][kE2Own], i_off[kE2Waves][kE2Own], i_cc[kE2Waves][kE2Own], i_lt[kE2Waves][kE2Own];
    __shared__ uint32_t w_tot[kE2Waves];
    __shared__ unsigned long long b_base;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();
    constexpr uint32_t kChunkE = kE2Waves * kE2Range;
    const Ent<W, kRoot> en{cid, mem, lohi, mask, rr};
    for (uint32_t c0 = blockIdx.x * kChunkE; c0 < E; c0 += gridDim.x * kChunkE) {
        const uint32_t wa = c0 + w * kE2Range, wz = min(E, wa + kE2Range);
        // the first run start in [wa, wz) (runs ending there started in an earlier range)
        uint32_t ef = wz;
        for (uint32_t b0 = wa; b0 < wz; b0 += 64) {
            const uint32_t e = b0 + lane;
            const uint64_t st = ballot(e < wz && (pos[e] >> 16) == 0u);
            if (st) {
                ef = b0 + uint32_t(__ffsll((unsigned long long)st)) - 1u;
                break;
            }
        }
        for (uint32_t k = lane; k < kE2Own; k += 64) i_n[w][k] = 0;
        uint32_t nrec = 0;
        // the windows of whole runs [e0, e0 + cut); pass 0 records, pass 1 (overflow) writes
        // at the bases in i_cc / i_n: on_ok(ok, f, q, owner slot, k)
        auto walk = [&](auto&& on_ok, bool keep) {
            // the next window's entry words (pos, member, class, W = 1 mask) are loaded while the
            // current window's pairs are joined: a window's dependent chain starts one load later
            uint32_t np = 0, nmi = 0, ncid = 0;
            uint64_t nmk = 0;
            auto fetch = [&](uint32_t e0n) {
                const uint32_t en_e = e0n + lane;
                np = 0u;
                if (en_e < E) {
                    np = pos[en_e];
                    nmi = en.m(en_e);
                    if constexpr (W == 1) nmk = mask[en_e];
                    if constexpr (!kRoot) ncid = cid[en_e];
                }
            };
            if (ef < wz) fetch(ef);
            for (uint32_t e0 = ef; e0 < wz;) {
                const uint32_t e = e0 + lane;
                const uint32_t p = np, cmi = nmi, ccid = ncid;
                const uint64_t cmk = nmk;
                const uint32_t len = p & 0xFFFFu;
                const bool st = e < E && (p >> 16) == 0u;
                // a run starting at lane s is in this window iff it starts in [e0, wz) and fits
                const uint64_t bad = ballot(st && (e >= wz || lane + len > 64u));
                const uint64_t sts = ballot(st);
                uint32_t cut;
                if (bad & 1ull) {  // lane 0 starts a run of more than 64 entries: k_emit1's list
                    if (keep && lane == 0) longl[atomicAdd(nlong, 1u)] = e0;
                    e0 += uint32_t(__shfl(int(len), 0, 64));
                    if (e0 < wz) fetch(e0);
                    continue;
                }
                if (bad) {
                    cut = uint32_t(__ffsll((unsigned long long)bad)) - 1u;
                } else {  // every start fits: the window ends with the last run
                    const uint32_t ls = 63u - uint32_t(__clzll(sts));
                    cut = ls + uint32_t(__shfl(int(len), int(ls), 64));
                }
                if (e0 + cut < wz) fetch(e0 + cut);
                const bool in = lane < cut;
                uint32_t mi = 0, lh = 0, cc = kNone, k0 = 0, nk = 0, lt2 = 0;
                uint64_t mk = 0;
                if (in) {
                    mi = cmi;
                    if constexpr (W == 1) {
                        mk = cmk;
                        lh = kRoot || kLhDerived<W> ? lh_of_word(mk) : lohi[e];
                    } else {
                        lh = en.lh(e);
                    }
                    const DClass c = cls[kRoot ? 0u : ccid];
                    cc = kRoot && (mi & 1u) ? kNone : child_of[c.cbase + mi];  // (infrequent DB entry: no class)
                    if (cc != kNone) {
                        k0 = kid_off[c.cbase + mi];
                        nk = kid_off[c.cbase + mi + 1] - k0;
                    }
                    lt2 = (lh & 0xFFFFu) | ((mi & 1u) << 16);
                }
                const uint32_t rs = lane - (p >> 16), re = rs + len;  // the lane's run, as lanes
                const uint32_t slot_own = e - ef;                     // owner slot of the wave
                // (entry, kid) pairs flattened over the lanes: one pair per lane per step
                const uint32_t incl = wave_incl_scan(nk), excl = incl - nk;
                const uint32_t total = uint32_t(__shfl(int(incl), 63, 64));
                uint32_t done = 0;
                // the owner lane of pair pp: the largest lane whose first pair index <= pp
                auto owner_of = [&](uint32_t pp) {
                    uint32_t ow = 0;
#pragma unroll
                    for (uint32_t stp = 32; stp > 0; stp >>= 1) {
                        const uint32_t cand = ow + stp;
                        if (uint32_t(__shfl(int(excl), int(cand), 64)) <= pp) ow = cand;
                    }
                    return ow;
                };
                // the kid slot of each step is loaded one step ahead (its owner search needs no
                // result of the step before), so the load's latency overlaps a step's shuffles
                uint32_t ow_n = owner_of(lane);
                uint32_t q_n = uint32_t(__shfl(int(k0), int(ow_n), 64)) + (lane - uint32_t(__shfl(int(excl), int(ow_n), 64)));
                uint32_t slot_n = lane < total ? kid_slot[q_n] : 0u;
                for (uint32_t p0 = 0; p0 < total; p0 += 64) {
                    const uint32_t pp = p0 + lane;
                    const uint32_t ow = ow_n, q = q_n, slot = slot_n;
                    if (p0 + 64 < total) {
                        ow_n = owner_of(pp + 64);
                        q_n = uint32_t(__shfl(int(k0), int(ow_n), 64)) + (pp + 64 - uint32_t(__shfl(int(excl), int(ow_n), 64)));
                        slot_n = pp + 64 < total ? kid_slot[q_n] : 0u;
                    }
                    const uint32_t o_ex = uint32_t(__shfl(int(excl), int(ow), 64));
                    const uint32_t o_rs = uint32_t(__shfl(int(rs), int(ow), 64));
                    const uint32_t o_re = uint32_t(__shfl(int(re), int(ow), 64));
                    const uint32_t o_lt = uint32_t(__shfl(int(lt2), int(ow), 64));
                    const uint32_t o_done = uint32_t(__shfl(int(done), int(ow), 64));
                    const uint64_t o_mk = W == 1 ? __shfl(mk, int(ow), 64) : 0ull;
                    const bool live = pp < total;
                    const uint32_t ct = slot & 1u;
                    const uint32_t target = (slot & ~1u) | (ct == kSeq ? 0u : (o_lt >> 16));  // partner member id
                    // lower_bound of target in lanes [o_rs, o_re): 6 fixed steps
                    uint32_t f = o_rs;
#pragma unroll
                    for (uint32_t stp = 32; stp > 0; stp >>= 1) {
                        const uint32_t cand = f + stp;
                        const uint32_t v = uint32_t(__shfl(int(mi), int(min(cand, 64u) - 1u), 64));
                        if (cand <= o_re && mem_less(v, target)) f = cand;
                    }
                    const uint32_t fl = min(f, 63u);
                    const uint32_t f_mi = uint32_t(__shfl(int(mi), int(fl), 64));
                    const uint32_t f_lh = uint32_t(__shfl(int(lh), int(fl), 64));
                    const uint64_t f_mk = W == 1 ? __shfl(mk, int(fl), 64) : 0ull;
                    bool ok = false;
                    if constexpr (W == 1) {
                        if (live && f < o_re && f_mi == target)
                            ok = ct == kSeq ? (f_lh >> 16) > (o_lt & 0xFFFFu) : (o_mk & f_mk) != 0ull;
                    } else {
                        const uint32_t o_lh = uint32_t(__shfl(int(lh), int(ow), 64));
                        if (live && f < o_re && f_mi == target) {
                            if (ct == kSeq) {
                                ok = (f_lh >> 16) > (o_lt & 0xFFFFu);
                            } else {
                                MaskV<W> om;
                                om.load(mask + size_t(e0 + ow) * W, uint32_t(W), o_lh);
                                ok = om.and_any(mask + size_t(e0 + f) * W, uint32_t(W), f_lh);
                            }
                        }
                    }
                    const uint64_t succ = ballot(ok);
                    const uint32_t first = (o_ex > p0 ? o_ex : p0) - p0;  // owner's first lane in this step
                    const uint32_t k = o_done + uint32_t(__popcll(succ & lane_range(first, lane)));
                    on_ok(ok, e0 + f, q, e0 + ow - ef, k);
                    const uint32_t a = (excl > p0 ? excl : p0), bnd = (incl < p0 + 64 ? incl : p0 + 64);
                    if (bnd > a) done += uint32_t(__popcll(succ & lane_range(a - p0, bnd - p0)));
                }
                if (keep && in) {
                    i_n[w][slot_own] = done;
                    i_cc[w][slot_own] = cc;
                    i_lt[w][slot_own] = lt2;
                }
                e0 += cut;
            }
        };
        walk([&](bool ok, uint32_t f, uint32_t q, uint32_t os, uint32_t k) {
                 const uint64_t b = ballot(ok);
                 if (ok) {
                     const uint32_t x = nrec + uint32_t(__popcll(b & lt));
                     if (x < rcap) {
                         r_f[w][x] = f;
                         r_q[w][x] = q;
                         r_ek[w][x] = (os << 16) | k;
                     }
                 }
                 nrec += uint32_t(__popcll(b));
             },
             true);
        // the wave's child run offsets (exclusive scan of i_n over its owner slots)
        uint32_t wsum = 0;
        for (uint32_t k0 = 0; k0 < kE2Own; k0 += 64) {
            const uint32_t v = i_n[w][k0 + lane];
            const uint32_t inc = wave_incl_scan(v);
            i_off[w][k0 + lane] = wsum + inc - v;
            wsum += uint32_t(__shfl(int(inc), 63, 64));
        }
        if (lane == 0) w_tot[w] = wsum;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long tot = 0;
            for (uint32_t k = 0; k < kE2Waves; ++k) tot += w_tot[k];
            b_base = tot ? atomicAdd(cursor, tot) : 0ull;
        }
        __syncthreads();
        uint64_t wb = b_base;
        for (uint32_t k = 0; k < w; ++k) wb += w_tot[k];
        if (nrec <= rcap) {
            for (uint32_t x = lane; x < nrec; x += 64) {
                const uint32_t f = r_f[w][x], q = r_q[w][x], ek = r_ek[w][x];
                const uint32_t os = ek >> 16, k = ek & 0xFFFFu;
                emit_write<W>(o, cap, wb + i_off[w][os] + k, i_cc[w][os], kid_cid[q], k, i_n[w][os], ef + os,
                              i_lt[w][os], f, kid_slot[q], lohi, mask, uint32_t(W));
            }
        } else {  // the records overflowed: join again, writing at the run bases
            walk([&](bool ok, uint32_t f, uint32_t q, uint32_t os, uint32_t k) {
                     if (ok)
                         emit_write<W>(o, cap, wb + i_off[w][os] + k, i_cc[w][os], kid_cid[q], k, i_n[w][os], ef + os,
                                       i_lt[w][os], f, kid_slot[q], lohi, mask, uint32_t(W));
                 },
                 false);
        }
        __syncthreads();  // the LDS records are reused by the next chunk
    }
}

// Window count (W = 1).  k_count's atomics execute at the memory side, one
// request per distinct 64-byte line of a wave-instruction (MI355X_MICROARCH
// §Global float atomics: a coalesced 256-B instruction is four requests); with
// one thread per entry the 64 lanes of an instruction add into 64 different
// counter rows.  Here each wave walks windows of whole runs (<= 64 entries, in
// registers, as k_emit2) and flattens the window's (entry, partner) pairs over
// the lanes in entry order, so the lanes of one instruction add into the rows
// of the few entries of that step, and the partner's member / lohi / mask come
// by shuffle.  Runs longer than 64 entries are counted thread-per-entry.
// W > 1 (up to 8 words): equality tests read both masks at their slab slots after
// the eid-range overlap test (as k_emit2).
#ifndef FSM_C2_RANGE
#define FSM_C2_RANGE 256
#endif
// entries per wave range (runs starting in it; round 6, rocprof per D1M mine: 64 0.88 ms,
// 128 0.57-0.60, 256 0.54-0.55, 384 / 512 0.55)
constexpr uint32_t kC2Range = FSM_C2_RANGE;

template <int W>
__global__ __launch_bounds__(kBlock) void k_count2(uint32_t E, const uint32_t* __restrict__ cid,
                                                   const DClass* __restrict__ cls, const uint32_t* __restrict__ mem,
                                                   const uint32_t* __restrict__ lohi, const uint32_t* __restrict__ pos,
                                                   const uint64_t* __restrict__ mask, uint32_t mlo, uint32_t mhi,
                                                   uint32_t* __restrict__ cnt, unsigned long long* __restrict__ tests) {
    __shared__ uint32_t blk_tests;
    if (threadIdx.x == 0) blk_tests = 0;
    __syncthreads();
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
    uint32_t my_tests = 0;
    for (uint32_t wa = wave * kC2Range; wa < E; wa += nwaves * kC2Range) {
        const uint32_t wz = min(E, wa + kC2Range);
        uint32_t e0 = wz;  // the first run start in [wa, wz)
        for (uint32_t b0 = wa; b0 < wz; b0 += 64) {
            const uint32_t e = b0 + lane;
            const uint64_t st = ballot(e < wz && (pos[e] >> 16) == 0u);
            if (st) {
                e0 = b0 + uint32_t(__ffsll((unsigned long long)st)) - 1u;
                break;
            }
        }
        // the next window's entry words are loaded while the current window's pairs are counted
        uint32_t np = 0, nmi = 0, ncid = 0;
        uint64_t nmk = 0;
        auto fetch = [&](uint32_t e0n) {
            const uint32_t en_e = e0n + lane;
            np = 0u;
            if (en_e < E) {
                np = pos[en_e];
                nmi = mem[en_e];
                ncid = cid[en_e];
                if constexpr (W == 1) nmk = mask[en_e];
            }
        };
        if (e0 < wz) fetch(e0);
        while (e0 < wz) {
            const uint32_t e = e0 + lane;
            const uint32_t p = np, cmi = nmi, ccid = ncid;
            const uint64_t cmk = nmk;
            const uint32_t len = p & 0xFFFFu;
            const bool st = e < E && (p >> 16) == 0u;
            const uint64_t bad = ballot(st && (e >= wz || lane + len > 64u));
            const uint64_t sts = ballot(st);
            if (bad & 1ull) {  // lane 0 starts a run of more than 64 entries: thread per entry
                const uint32_t rl = uint32_t(__shfl(int(len), 0, 64));
                if (e0 + rl < wz) fetch(e0 + rl);
                for (uint32_t i0 = e0; i0 < e0 + rl; i0 += 64) {
                    const uint32_t ei = i0 + lane;
                    if (ei >= e0 + rl) continue;
                    const uint32_t mi = mem[ei];
                    if (!(mi - mlo < mhi - mlo)) continue;
                    my_tests += rl;
                    const DClass c = cls[cid[ei]];
                    const uint32_t lh_i = slab_lh<W>(lohi, mask, ei), lo_i = lh_i & 0xFFFFu, ti = mi & 1u, ri = mi >> 1;
                    MaskV<W> mk;
                    mk.load(mask + size_t(ei) * W, uint32_t(W), lh_i);
                    uint32_t* rowc = cnt + c.cnt_off + uint64_t(mi >> c.mshift) * c.rstride;
                    for (uint32_t f = e0; f < e0 + rl; ++f) {
                        const uint32_t mj = mem[f], tj = mj & 1u, rj = mj >> 1, lh_f = slab_lh<W>(lohi, mask, f);
                        if (tj == kSeq) {
                            if ((lh_f >> 16) > lo_i) atomicAdd(rowc + (rj << 1), 1u);
                            if (ti == kSeq && rj > ri && mk.and_any(mask + size_t(f) * W, uint32_t(W), lh_f))
                                atomicAdd(rowc + (rj << 1 | 1u), 1u);
                        } else if (ti == kItm && rj > ri && mk.and_any(mask + size_t(f) * W, uint32_t(W), lh_f)) {
                            atomicAdd(rowc + (rj << 1 | 1u), 1u);
                        }
                    }
                }
                e0 += rl;
                continue;
            }
            uint32_t cut;
            if (bad) {
                cut = uint32_t(__ffsll((unsigned long long)bad)) - 1u;
            } else {
                const uint32_t ls = 63u - uint32_t(__clzll(sts));
                cut = ls + uint32_t(__shfl(int(len), int(ls), 64));
            }
            if (e0 + cut < wz) fetch(e0 + cut);
            const bool in = lane < cut;
            uint32_t mi = 0, lh = 0, npart = 0;
            uint64_t mk = 0, rowa = 0;
            if (in) {
                mi = cmi;
                if constexpr (W == 1) mk = cmk;
                lh = kLhDerived<W> ? lh_of_word(mk) : lohi[e];
                if (mi - mlo < mhi - mlo) {  // (sharded root: this rank's member rows only)
                    const DClass c = cls[ccid];
                    rowa = c.cnt_off + uint64_t(mi >> c.mshift) * c.rstride;
                    npart = len;  // partners: every entry of its run
                    my_tests += len;
                }
            }
            const uint32_t rs = lane - (p >> 16);  // first lane of the lane's run
            const uint32_t incl = wave_incl_scan(npart), excl = incl - npart;
            const uint32_t total = uint32_t(__shfl(int(incl), 63, 64));
            for (uint32_t p0 = 0; p0 < total; p0 += 64) {
                const uint32_t pp = p0 + lane;
                uint32_t ow = 0;  // the owner lane: the largest lane whose first pair index <= pp
#pragma unroll
                for (uint32_t stp = 32; stp > 0; stp >>= 1) {
                    const uint32_t cand = ow + stp;
                    if (uint32_t(__shfl(int(excl), int(cand), 64)) <= pp) ow = cand;
                }
                const uint32_t o_ex = uint32_t(__shfl(int(excl), int(ow), 64));
                const uint32_t o_rs = uint32_t(__shfl(int(rs), int(ow), 64));
                const uint32_t o_mi = uint32_t(__shfl(int(mi), int(ow), 64));
                const uint32_t o_lh = uint32_t(__shfl(int(lh), int(ow), 64)), o_lo = o_lh & 0xFFFFu;
                const uint64_t o_mk = W == 1 ? __shfl(mk, int(ow), 64) : 0ull;
                const uint64_t o_row = __shfl(rowa, int(ow), 64);
                const uint32_t f = min(o_rs + (pp - o_ex), 63u);  // the partner lane
                const uint32_t mj = uint32_t(__shfl(int(mi), int(f), 64));
                const uint32_t lj = uint32_t(__shfl(int(lh), int(f), 64)), hj = lj >> 16;
                const uint64_t mkj = W == 1 ? __shfl(mk, int(f), 64) : 0ull;
                if (pp < total) {
                    const uint32_t ti = o_mi & 1u, ri = o_mi >> 1, tj = mj & 1u, rj = mj >> 1;
                    uint32_t* rowc = cnt + o_row;
                    // the equality join L(i) & L(j) (W > 1: the masks at slab slots e0 + ow, e0 + f)
                    auto eq = [&]() -> bool {
                        if constexpr (W == 1) {
                            return (o_mk & mkj) != 0ull;
                        } else {
                            MaskV<W> om;
                            om.load(mask + size_t(e0 + ow) * W, uint32_t(W), o_lh);
                            return om.and_any(mask + size_t(e0 + f) * W, uint32_t(W), lj);
                        }
                    };
                    if (tj == kSeq) {
                        if (hj > o_lo) atomicAdd(rowc + (rj << 1), 1u);
                        if (ti == kSeq && rj > ri && eq()) atomicAdd(rowc + (rj << 1 | 1u), 1u);
                    } else if (ti == kItm && rj > ri && eq()) {
                        atomicAdd(rowc + (rj << 1 | 1u), 1u);
                    }
                }
            }
            e0 += cut;
        }
    }
    atomicAdd(&blk_tests, my_tests);
    __syncthreads();
    if (threadIdx.x == 0 && blk_tests) atomicAdd(tests, (unsigned long long)blk_tests);
}

// ---- A batch's frequent records in (row, slot) order on the device (unsharded, one emit
// group): each record's child member id (rank of its partner item among its row's partners,
// << 1 | type), the kid table [koff | kslot | kcid] and the member slot -> child class table,
// so the next emit launches with no host ordering between the count and it.  A row's
// records have distinct slots below its class's member id space D: a bitmap of them in LDS
// and two prefix popcounts (slots, partner items) give every record its rank, so nothing
// is sorted.  Four launches: histogram, the row tables, bucket scatter, one block per row.
// (No last-block fusion: the agent-scope fences it needs write back the XCD's L2 in every
// block, which cost 0.3 ms over ~1000 row blocks.)  Rows: the root's (row r = member 2r of
// the one root class, D = 2F) or a batch's counter rows (RkRows: class and member per row).
struct RkRows {
    const DRow* rows;     // nullptr: the root (row r: member slot 2r, D = 2F)
    const DClass* cls;
    uint32_t F;
    __device__ __forceinline__ uint32_t slot(uint32_t r) const {
        if (!rows) return 2u * r;
        const DRow d = rows[r];
        return cls[d.cls].cbase + d.mi;
    }
    __device__ __forceinline__ uint32_t width(uint32_t r) const { return rows ? cls[rows[r].cls].D : 2u * F; }
};

// exclusive scan over the block (kBlock threads) of one u32 per thread; tot = the sum
__device__ __forceinline__ uint32_t rk_block_scan(uint32_t v, uint32_t* wsum, uint32_t& tot) {
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    __syncthreads();  // (wsum's previous readers are done)
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t before = 0;
    tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBlock / 64; ++w) {
        before += w < wv ? wsum[w] : 0u;
        tot += wsum[w];
    }
    return before + inc - v;
}
// exclusive scan of get(0..m) by one block in per-thread chunks: put(i, prefix, get(i)); returns the sum
template <class Get, class Put>
__device__ uint32_t rk_scan_range(uint32_t m, uint32_t* wsum, Get get, Put put) {
    const uint32_t ch = (m + kBlock - 1) / kBlock;
    const uint32_t a = min(m, threadIdx.x * ch), z = min(m, a + ch);
    uint32_t s = 0;
    for (uint32_t i = a; i < z; ++i) s += get(i);
    uint32_t tot;
    uint32_t run = rk_block_scan(s, wsum, tot);
    for (uint32_t i = a; i < z; ++i) {
        const uint32_t g = get(i);
        put(i, run, g);
        run += g;
    }
    return tot;
}
// rowcnt[r]: the row's records | 1 << 31 if one of them has an even slot (a sequence extension)
constexpr uint32_t kRkEven = 1u << 31;
__global__ __launch_bounds__(kBlock) void k_rk_hist(const FreqRec* __restrict__ R, uint32_t n,
                                                    FreqRec* __restrict__ Rd, uint32_t* __restrict__ rowcnt) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const FreqRec r = R[p];  // (mapped pinned memory: read once, kept in HBM)
        Rd[p] = r;
        atomicAdd(&rowcnt[r.row], (r.slot & 1u) ? 1u : 1u | kRkEven);
    }
}
// one tile of kRkTile rows per block: the block sums the rows before its tile itself (all
// loads independent, no cross-block wait), then scans its tile staged through LDS.  Per row
// one packed value: records | kept << 32 (a row opens a child class unless it is empty or
// one lone itemset extension).  Out: row offsets; over the member slots x in (slot(r - 1),
// slot(r)] koff[x] = the row's offset and child_of[x] = its class at slot(r), else none
// (the last row also fills the slots above it up to nko).
constexpr uint32_t kRkV = 8, kRkTile = kBlock * kRkV;
__global__ __launch_bounds__(kBlock) void k_rk_tables(const uint32_t* __restrict__ rowcnt, uint32_t nrows,
                                                      RkRows rr, uint32_t nko, uint32_t* __restrict__ rowoff,
                                                      uint32_t* __restrict__ koff, uint32_t* __restrict__ child_of) {
    __shared__ uint64_t tileb[kRkTile];
    __shared__ uint32_t sslot[kRkTile];  // the tile's member slots (loaded with the counts)
    __shared__ uint64_t wsum[kBlock / 64];
    auto get = [&](uint32_t r) {
        const uint32_t w = rowcnt[r], c = w & ~kRkEven;
        return uint64_t(c) | uint64_t(c > 1u || (c == 1u && (w & kRkEven))) << 32;
    };
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, t0 = blockIdx.x * kRkTile;
    uint64_t acc = 0;
#pragma unroll 8
    for (uint32_t i = threadIdx.x; i < t0; i += kBlock) acc += get(i);
#pragma unroll
    for (uint32_t k = 0; k < kRkV; ++k) {
        const uint32_t i = t0 + k * kBlock + threadIdx.x;
        tileb[k * kBlock + threadIdx.x] = i < nrows ? get(i) : 0ull;
        sslot[k * kBlock + threadIdx.x] = i < nrows ? rr.slot(i) : 0u;
    }
    acc = wave_incl_scan(acc);
    if (lane == 63) wsum[wv] = acc;
    __syncthreads();
    uint64_t carry = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBlock / 64; ++w) carry += wsum[w];
    uint64_t v[kRkV], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kRkV; ++k) sum += (v[k] = tileb[threadIdx.x * kRkV + k]);
    const uint64_t inc = wave_incl_scan(sum);
    __syncthreads();  // (wsum is reused)
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint64_t run = carry;
#pragma unroll
    for (uint32_t w = 0; w < kBlock / 64; ++w) run += w < wv ? wsum[w] : 0ull;
    run += inc - sum;
    const uint32_t first = t0 + threadIdx.x * kRkV;
    // the first member slot after row first - 1 (read only for a thread that has rows)
    uint32_t prev = first == 0 || first >= nrows ? 0u : (first > t0 ? sslot[first - 1u - t0] : rr.slot(first - 1u)) + 1u;
#pragma unroll
    for (uint32_t k = 0; k < kRkV; ++k) {
        const uint32_t r = first + k;
        if (r < nrows) {
            const uint32_t off = uint32_t(run), sr = sslot[r - t0];
            for (uint32_t x = prev; x < sr; ++x) {  // member slots without a counter row
                koff[x] = off;
                child_of[x] = kNone;
            }
            rowoff[r] = off;
            koff[sr] = off;
            child_of[sr] = (v[k] >> 32) ? uint32_t(run >> 32) : kNone;
            prev = sr + 1u;
            if (r == nrows - 1u) {
                const uint32_t n = uint32_t(run + v[k]);
                rowoff[nrows] = n;
                for (uint32_t x = prev; x < nko; ++x) {
                    koff[x] = n;
                    if (x < nko - 1u) child_of[x] = kNone;
                }
            }
        }
        run += v[k];
    }
}
__global__ __launch_bounds__(kBlock) void k_rk_scatter(const FreqRec* __restrict__ Rd, uint32_t n,
                                                       const uint32_t* __restrict__ rowoff, uint32_t* __restrict__ rowcnt,
                                                       uint32_t* __restrict__ idx) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const uint32_t row = Rd[p].row;
        // (bucket order is free: ranks come from slots)
        idx[rowoff[row] + (atomicSub(&rowcnt[row], 1u) & ~kRkEven) - 1u] = p;
    }
}
__global__ __launch_bounds__(kBlock) void k_rk_row(const FreqRec* __restrict__ Rd, const uint32_t* __restrict__ idx,
                                                   const uint32_t* __restrict__ rowoff, RkRows rr, uint32_t nwmax,
                                                   FreqRec* __restrict__ out, uint32_t* __restrict__ kslot,
                                                   uint32_t* __restrict__ kcid) {
    extern __shared__ uint32_t rk_sm[];
    __shared__ uint32_t wsum[kBlock / 64];
    const uint32_t r = blockIdx.x, beg = rowoff[r], c = rowoff[r + 1] - beg;
    if (c == 0) return;  // (block-uniform)
    const uint32_t nw = (rr.width(r) + 31) / 32;  // (<= nwmax: the LDS the host sized)
    uint32_t* bm = rk_sm;       // the row's slots
    uint32_t* ps = bm + nwmax;  // slots in words < w
    uint32_t* pi = ps + nwmax;  // partner items in words < w
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) bm[w] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
        const uint32_t slot = Rd[idx[beg + i]].slot;
        atomicOr(&bm[slot >> 5], 1u << (slot & 31u));
    }
    __syncthreads();
    // one scan of (slots | partner items << 16) per word: both sums <= D < 2^16
    rk_scan_range(
        nw, wsum,
        [&](uint32_t w) {
            const uint32_t m = bm[w];
            return uint32_t(__popc(m)) | uint32_t(__popc((m | m >> 1) & 0x55555555u)) << 16;
        },
        [&](uint32_t w, uint32_t pre, uint32_t) {
            ps[w] = pre & 0xFFFFu;
            pi[w] = pre >> 16;
        });
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
        FreqRec rec = Rd[idx[beg + i]];
        const uint32_t w = rec.slot >> 5, bt = rec.slot & 31u, m = bm[w];
        const uint32_t rank = ps[w] + uint32_t(__popc(m & ((1u << bt) - 1u)));
        const uint32_t crank = pi[w] + uint32_t(__popc((m | m >> 1) & 0x55555555u & ((1u << (bt & ~1u)) - 1u)));
        rec.cid = crank << 1 | (rec.slot & 1u);
        out[beg + rank] = rec;
        kslot[beg + rank] = rec.slot;
        kcid[beg + rank] = rec.cid;
    }
}

// ------------------------------------------------------------- host side

#define FSM_W_DISPATCH(W_, MACRO) \
    switch (W_) {                 \
        case 1: MACRO(1); break;  \
        case 2: MACRO(2); break;  \
        case 4: MACRO(4); break;  \
        case 8: MACRO(8); break;  \
        case 16: MACRO(16); break; \
        case 32: MACRO(32); break; \
        case 64: MACRO(64); break; \
        default: MACRO(0); break;  \
    }

struct Slab {
    DevBuf cid, mem, lohi, pos, mask;
    uint64_t cap = 0;
    void alloc(uint64_t n, int W) {
        cid.alloc(n * 4);
        mem.alloc(n * 4);
        if (!lh_derived(W)) lohi.alloc(n * 4);
        pos.alloc(n * 4);
        mask.alloc(n * 8 * uint64_t(W));
        cap = n;
    }
    SlabPtrs ptrs() const {
        return SlabPtrs{cid.as<uint32_t>(), mem.as<uint32_t>(), lohi.as<uint32_t>(), pos.as<uint32_t>(),
                        mask.as<uint64_t>(), nullptr};
    }
};

// Allocator whose resize(n) leaves the new elements unwritten (the per-batch tables of
// millions of classes and nodes are filled by index afterwards, by host threads: a
// value-initialising resize would write every byte once more, serially)
// Arrays of 4 MiB and more come 2 MiB aligned and marked for transparent huge pages
// (a mine's Miner and batches are fresh: their tables fault in 2 MiB at a time).
template <class T> struct NoInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = NoInitAlloc<U>; };
    NoInitAlloc() = default;
    template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    static constexpr size_t kHuge = kHugeBlock;
    T* allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < 2 * kHuge) return std::allocator<T>::allocate(n);
        return static_cast<T*>(big_take((bytes + kHuge - 1) & ~(kHuge - 1)));
    }
    void deallocate(T* p, size_t n) {
        if (n * sizeof(T) < 2 * kHuge) std::allocator<T>::deallocate(p, n);
        else big_give(p);
    }
    template <class U> void construct(U*) noexcept {}
    template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
template <class T> using RawVec = std::vector<T, NoInitAlloc<T>>;

// Per-class member tables live in flat per-batch arrays (no per-class heap
// vectors: deep lattices have millions of small classes).
// One record per prefix class.  A batch's children (the classes its frequent
// candidates open) are the next batch's classes: the same record, so an emit of
// a batch's only group hands the whole array over (no per-class copy).
struct ClassMeta {
    uint64_t ri_off = 0;  // rank -> dense item id:        Batch::rank_item[ri_off + rank]
    uint64_t no_off = 0;  // member -> pattern node or -1:  Batch::node_of[no_off + member]
    uint64_t cnt_off = 0;
    uint64_t cap = 0;     // entries of the class in its batch slab (= sum of member supports)
    uint64_t sS = 0, sI = 0;  // summed supports of the members by type (sequence / itemset extension)
    uint32_t D = 0;
    uint32_t mshift = 0;
    uint32_t cbase = 0;
    uint32_t nS = 0, nI = 0;  // members by type
    uint32_t psup = 0;    // support of the class prefix P: an upper bound of the class's runs
    uint32_t pcls = 0, pmi = 0;  // as a child: the parent class and member that open it
    bool split = false;  // sharded: a heavy first-level class every rank counts; its sub-classes are split
};
using ChildInfo = ClassMeta;

// append-only array in fixed chunks: growth never copies (or faults in again) what
// is already there (pattern nodes: millions in deep lattices)
// (chunks of trivially copyable T, 2 MiB aligned and marked for transparent huge
// pages: the host threads that fill a fresh chunk fault it in 2 MiB at a time)
template <class T, int kShift = 20> struct ChunkedVec {
    struct Free {
        void operator()(T* p) const { big_give(p); }
    };
    std::vector<std::unique_ptr<T[], Free>> ch;
    size_t n = 0;
    static constexpr size_t kMask = (size_t(1) << kShift) - 1;
    size_t size() const { return n; }
    T& operator[](size_t i) { return ch[i >> kShift][i & kMask]; }
    const T& operator[](size_t i) const { return ch[i >> kShift][i & kMask]; }
    void add_chunk() {
        constexpr size_t kHuge = kHugeBlock;
        const size_t bytes = ((sizeof(T) << kShift) + kHuge - 1) & ~(kHuge - 1);
        ch.emplace_back(static_cast<T*>(big_take(bytes)));
    }
    void push_back(const T& v) {
        if ((n >> kShift) == ch.size()) add_chunk();
        ch[n >> kShift][n & kMask] = v;
        ++n;
    }
    void grow(size_t m) {  // size n + m; the new elements are written by index afterwards
        while (((n + m + kMask) >> kShift) > ch.size()) add_chunk();
        n += m;
    }
};


struct PNode {
    int32_t parent;
    uint32_t item;
    uint32_t type;
    uint32_t support;
    uint32_t len_sets;  // items << 16 | itemsets of the pattern (both < 2^16)
};

// Frequent-pair records in (row, slot) order with their child member ids: rank among
// the row's slots with a frequent temporal or equality candidate, << 1 | type (the ids
// k_freq_write assigns in-kernel).  Counting sort by row, then the few slots of a row.
// Records in (row, slot) order with their child member ids: rank among the row's slots with
// a frequent temporal or equality candidate, << 1 | type (as k_freq_write assigns them).
// off (if given) receives the row offsets [nrows + 1] of the ordered records.
void order_recs(std::vector<FreqRec>& recs, uint32_t nrows, std::vector<uint32_t>* off_out = nullptr) {
    // (scratch kept per host thread: no fresh pages per batch)
    thread_local std::vector<uint32_t> off_s, at;
    thread_local std::vector<FreqRec> tmp;
    std::vector<uint32_t>& off = off_out ? *off_out : off_s;
    off.assign(size_t(nrows) + 1, 0);
    for (const FreqRec& r : recs) ++off[size_t(r.row) + 1];
    for (uint32_t x = 0; x < nrows; ++x) off[x + 1] += off[x];
    tmp.resize(recs.size());
    at.assign(off.begin(), off.end() - 1);
    for (const FreqRec& r : recs) tmp[at[r.row]++] = r;
    for (uint32_t x = 0; x < nrows; ++x) {
        FreqRec* a = tmp.data() + off[x];
        const uint32_t n = off[x + 1] - off[x];
        if (n > 16) {
            std::sort(a, a + n, [](const FreqRec& u, const FreqRec& c) { return u.slot < c.slot; });
        } else {
            for (uint32_t i = 1; i < n; ++i) {  // (rows hold a few records: insertion sort)
                const FreqRec v = a[i];
                uint32_t j = i;
                for (; j > 0 && a[j - 1].slot > v.slot; --j) a[j] = a[j - 1];
                a[j] = v;
            }
        }
        uint32_t crank = 0;
        for (uint32_t i = 0; i < n; ++i) {
            if (i > 0 && (a[i].slot >> 1) != (a[i - 1].slot >> 1)) ++crank;
            a[i].cid = crank << 1 | (a[i].slot & 1u);
        }
    }
    recs.swap(tmp);
}

struct Batch {
    Slab slab;
    RawVec<ClassMeta> cls;
    // unsharded batches whose children fit one emit group: the children (pattern nodes and
    // the next batch's class tables) are built by emit() AFTER it has launched the emit
    // kernels, from these records (valid until the next count_and_freq), so that host work
    // overlaps the emit on the GPU instead of delaying its launch
    bool defer_children = false;
    const FreqRec* defer_R = nullptr;
    uint64_t defer_n = 0, defer_total = 0;
    const RawVec<DRow>* defer_rows = nullptr;
    const uint32_t* child_of_pre = nullptr;  // deferred, host child_of: uploaded with the kid table
    // the root's unordered-pair F2 keys, launched by run_root_db right after its plan (the host's
    // root bookkeeping then overlaps them): keys, region fills, the counters block
    // the records ordered on the device (order_device): the kid and child-class tables are
    // device-built; the ordered records reach pinned host memory at rec_ev
    bool dev_order = false;
    DevBuf ord_child_of;
    hipEvent_t rec_ev = nullptr;
    bool f2_launched = false;
    DevBuf f2_keys, f2_fill, f2_ctr_own;
    char* f2_ctr = nullptr;
    size_t f2_tk = 0;
    DevBuf d_cls;
    DevBuf kid_tab;  // frequent children of every member (CSR over cbase + mi): offsets | slots | child ids
    const uint32_t* kid_off = nullptr;
    const uint32_t* kid_slot = nullptr;
    const uint32_t* kid_cid = nullptr;
    DevBuf child_pre;  // unsharded: u64 exclusive scan of "member slot has a child class" (emit's child_of)
    uint64_t E = 0;                     // entries in the slab (runs of all classes, any order)
    uint64_t n_cnt = 0, cbase_total = 0;
    RawVec<uint32_t> rank_item;  // member tables of cls (see ClassMeta)
    RawVec<int32_t> node_of;
    RawVec<ChildInfo> children;
    RawVec<uint32_t> child_rank_item;  // member tables of children
    RawVec<int32_t> child_node_of;
    std::vector<std::pair<size_t, size_t>> groups;
    size_t next_group = 0;
    int64_t depth = 1;  // items per member pattern of this batch's classes
    bool root = false;
    DevBuf root_rows;   // root batch: u64 [R+1] slab offset of every DB row's run
    uint64_t R = 0;
    // root batch: F2 plan made by k_root_write_plan (region bases scanned, slot total read back)
    bool f2_planned = false;
    DevBuf f2_base;
    uint64_t f2_nslots = 0;
    // the root F2 in the unordered-pair layout (k_f2_tri): [gtab: F | group start ranks: G + 1]
    bool f2_tri = false;
    DevBuf f2_tri_tab;
    uint32_t f2_tri_G = 0;
    // DB-direct root (no root slab): its kernels read the DB rows through rk2 (dense item ->
    // member id, odd for an infrequent item)
    bool db_direct = false;
    DevBuf rk2;
    DevBuf mem_db;  // u32 [DB entries]: each DB entry's member id rk2[item] (written by the F2 plan)
    // sharded root with work stealing: children [0, nshared_children) are the
    // heavy classes every rank mines; the rest, largest first, are claimed in ranges from the
    // shared counter claim_key (-1: no claims; groups fixed)
    int64_t claim_key = -1;
    size_t nshared_children = 0;
    bool claims_done = false;
    int claims_made = 0;
    std::vector<uint64_t> claim_pre;  // prefix volumes of the claimable children

    // back to an empty batch: device buffers released, host vectors cleared with their
    // capacity kept (the DFS reuses popped batches: no fresh pages per batch)
    void recycle() {
        slab = Slab{};
        cls.clear();
        defer_children = false;
        defer_R = nullptr;
        defer_rows = nullptr;
        child_of_pre = nullptr;
        dev_order = false;
        ord_child_of.release();
        if (rec_ev) (void)hipEventDestroy(rec_ev);
        rec_ev = nullptr;
        f2_launched = false;
        f2_keys.release();
        f2_fill.release();
        f2_ctr_own.release();
        f2_ctr = nullptr;
        defer_n = defer_total = 0;
        d_cls.release();
        kid_tab.release();
        child_pre.release();
        kid_off = kid_slot = kid_cid = nullptr;
        E = n_cnt = cbase_total = 0;
        rank_item.clear();
        node_of.clear();
        children.clear();
        child_rank_item.clear();
        child_node_of.clear();
        groups.clear();
        next_group = 0;
        depth = 1;
        root = false;
        root_rows.release();
        R = 0;
        f2_planned = false;
        f2_base.release();
        f2_nslots = 0;
        f2_tri = false;
        f2_tri_tab.release();
        f2_tri_G = 0;
        db_direct = false;
        rk2.release();
        mem_db.release();
        claim_key = -1;
        nshared_children = 0;
        claims_done = false;
        claims_made = 0;
        claim_pre.clear();
    }
};

struct Miner {
    fsm_ctx* ctx;
    SpadeDevDB* db;
    hipStream_t s;
    int W;
    uint32_t minsup;
    uint64_t budget;
    ChunkedVec<PNode> nodes;
    KernelClock* clk = nullptr;
    // Per-mine zeroed device counters (slab cursors, record counts, the join-test total): ONE
    // memset when the mine starts instead of a fill launch per counter; zslot(n) hands out
    // 16-byte aligned slots, nullptr once the block is used up (the caller then allocates and
    // zeroes its own)
    DevBuf zblk;
    uint32_t zused = 0;
    static constexpr uint32_t kZBytes = 64u << 10;
    void* zslot(size_t bytes) {
        const uint32_t n = uint32_t((bytes + 15) & ~size_t(15));
        if (!zblk.p || zused + n > kZBytes) return nullptr;
        void* p = zblk.as<char>() + zused;
        zused += n;
        return p;
    }
    unsigned long long* d_tests = nullptr;  // u64 (a zslot): (entry, partner) join tests of the class count kernels
    // sharded mining (nranks > 1): this rank counts the root rows of ranks
    // [slice_lo, slice_hi) and mines the first-level classes shard_plan gives it
    Comm* comm = nullptr;
    uint32_t slice_lo = 0, slice_hi = kNone;
    size_t n_shared = 0;  // pattern nodes every rank holds (root + its frequent children)
    std::vector<uint8_t> node_dup;  // sharded: nodes of split classes, output by rank 0 only

    // host scratch reused by every batch (capacity kept: no fresh pages per batch)
    RawVec<DRow> rows_s;
    std::vector<FreqRec> recs_s;
    RawVec<uint32_t> ktab_s, child_of_s;
    std::vector<uint32_t> rec_off_s;  // row offsets of the records order_recs ordered last (kid offsets)
    bool rec_off_ok = false;
    RawVec<uint64_t> gs_s;
    RawVec<uint32_t> r2_s;

    double wait_ms = 0;  // host time blocked on the stream (the rest of the lattice time is host work)
    // FSM_HOST_TRACE=1: host time of the bookkeeping phases, printed at the end of the mine
    double hp[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // f2 sort, kids, children, groups, emit tables, slab alloc, count prep, count
    // finer host split (FSM_HOST_TRACE): lap(i, t) adds the time since t to hq[i] and restarts t
    double hq[16] = {};
    void lap(int i, double& t) {
        const double n = now_ms();
        hq[i] += n - t;
        t = n;
    }

    // Sharded mining: the work between two collectives runs through
    // run_or_defer; agree() before the next collective (comm.h Agreement)
    Agreement agr;
    template <class F> void run_or_defer(F&& f) { agr.run(std::forward<F>(f)); }
    void maybe_inject(const char* phase) const { agr.maybe_inject(phase); }
    void agree() { agr.agree(s); }
    void sync() {
        if (pend_check && emit_blk && !emit_copied) {  // the last emit's cursor block (check_emit)
            FSM_HIP(hipMemcpyAsync(&pend[8], emit_blk, 16, hipMemcpyDeviceToHost, s));
            emit_copied = true;
        }
        const double t = now_ms();
        FSM_HIP(hipStreamSynchronize(s));
        wait_ms += now_ms() - t;
        check_emit();
    }
    uint64_t* pend = nullptr;  // pinned slots (ctx->pinned_u64()): [8..10] the last emit's cursor block
    char* emit_blk = nullptr;  // the last emit's 32-byte device block (cursor, long runs, flag, next count)
    bool emit_copied = false;  // its read-back is enqueued
    DevBuf emit_own;           // (the block when the zeroed slots are used up)
    uint64_t pend_total = 0;
    bool pend_check = false;

    uint64_t entry_bytes() const {  // cid, mem, lohi (not at W = 1), pos, mask
        return (lh_derived(W) ? 12ull : 16ull) + 8ull * uint64_t(W);
    }
    // one (sid u32, eid mask) id-list entry, 4 + 8 ceil(E/64) bytes (12 B at W = 1)
    uint64_t survey_entry_bytes() const { return 4ull + 8ull * uint64_t(W); }

    // large per-batch tables: copied into a pinned staging slot (over the host pool
    // when large) and DMA'd asynchronously (pageable copies run at a fraction of that)
    void upload_staged(int slot, DevBuf& d, const void* src, size_t bytes) {
        d.alloc(std::max<size_t>(bytes, 4));
        if (!bytes) return;
        char* dst = static_cast<char*>(ctx->stage_host(slot, bytes));
        const char* sp = static_cast<const char*>(src);
        const int64_t nthr = bytes >= (size_t(8) << 20) ? host_threads() : 1;
        par_slices(nthr, int64_t(bytes), [&](int64_t, int64_t a, int64_t z) {
            if (z > a) std::memcpy(dst + a, sp + a, size_t(z - a));
        });
        ctx->stage_copy(slot, d.p, bytes);
    }
    // pageable H2D copies are staged before hipMemcpyAsync returns; callers keep
    // the host vectors alive until the next synchronization anyway.
    template <class T> void upload(DevBuf& d, const std::vector<T>& h) {
        d.alloc(h.size() * sizeof(T));
        if (!h.empty()) FSM_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
    }


    // class descriptors (counter matrix offsets, member bases) of a batch.  keyed:
    // counters laid out for the keyed count (a class matrix that fits one group of
    // kGroupCounters is not cut by a group boundary; larger ones start on a group
    // boundary with a power-of-two row stride, so no counter row straddles a
    // group).  Returns false (plain layout) when a row exceeds a group.
    bool prepare(Batch& b, bool keyed) {
        const int64_t ncls = int64_t(b.cls.size());
        // many classes: host-thread slices laid out from 0, then moved to their base (a
        // keyed slice starts on a group boundary, so the rules above hold across slices)
        const int64_t nthr = ncls >= (int64_t(1) << 15) ? host_threads() : 1;
        // the descriptors are written straight into the pinned staging slot (no host copy)
        DClass* hc = static_cast<DClass*>(ctx->stage_host(0, std::max<size_t>(size_t(ncls), 1) * sizeof(DClass)));
        std::vector<uint64_t> toff(size_t(nthr) + 1, 0), tcb(size_t(nthr) + 1, 0);
        std::vector<uint8_t> tok(size_t(nthr), 1);
        for (int pass = keyed ? 0 : 1; pass < 2; ++pass) {
            const bool kl = pass == 0;
            par_slices(nthr, ncls, [&](int64_t t, int64_t c0, int64_t c1) {
                uint64_t off = 0, cb = 0;
                bool ok = true;
                for (int64_t c = c0; c < c1 && ok; ++c) {
                    ClassMeta& m = b.cls[size_t(c)];
                    const uint64_t rows = m.D >> m.mshift;
                    uint32_t stride = m.D;
                    if (kl) {
                        if (rows * m.D <= kGroupCounters) {
                            if ((off & (kGroupCounters - 1)) + rows * m.D > kGroupCounters)
                                off = (off + kGroupCounters - 1) & ~uint64_t(kGroupCounters - 1);
                        } else if (m.D <= kGroupCounters) {
                            stride = m.D <= 1 ? 1u : 1u << (32 - __builtin_clz(m.D - 1));
                            off = (off + kGroupCounters - 1) & ~uint64_t(kGroupCounters - 1);
                        } else {
                            ok = false;
                        }
                    }
                    m.cnt_off = off;
                    m.cbase = uint32_t(cb);
                    off += rows * stride;
                    cb += m.D;
                    hc[size_t(c)] = DClass{m.cnt_off, m.D, m.cbase, m.mshift, stride, {0, 0}};
                }
                toff[size_t(t) + 1] = off;
                tcb[size_t(t) + 1] = cb;
                tok[size_t(t)] = ok;
            });
            bool ok = true;
            for (int64_t t = 0; t < nthr; ++t) {
                ok = ok && tok[size_t(t)];
                uint64_t next = toff[size_t(t)] + toff[size_t(t) + 1];
                if (kl && t + 1 < nthr) next = (next + kGroupCounters - 1) & ~uint64_t(kGroupCounters - 1);
                toff[size_t(t) + 1] = next;
                tcb[size_t(t) + 1] += tcb[size_t(t)];
            }
            if (!ok) continue;
            if (tcb[size_t(nthr)] >= kNone) throw Error(FSM_ELIMIT, "SPADE: class batch member space exceeds 2^32");
            if (nthr > 1)
                par_slices(nthr, ncls, [&](int64_t t, int64_t c0, int64_t c1) {
                    const uint64_t bo = toff[size_t(t)];
                    const uint32_t bc = uint32_t(tcb[size_t(t)]);
                    for (int64_t c = c0; c < c1; ++c) {
                        ClassMeta& m = b.cls[size_t(c)];
                        m.cnt_off += bo;
                        m.cbase += bc;
                        hc[size_t(c)].cnt_off = m.cnt_off;
                        hc[size_t(c)].cbase = m.cbase;
                    }
                });
            b.n_cnt = toff[size_t(nthr)];
            b.cbase_total = tcb[size_t(nthr)];
            b.d_cls.alloc(std::max<size_t>(size_t(ncls) * sizeof(DClass), 4));
            ctx->stage_copy(0, b.d_cls.p, size_t(ncls) * sizeof(DClass));
            return kl;
        }
        return false;
    }

    // FSM_COUNT_PATH=atomic|keys: force the class count path (default: keyed for
    // join-dense batches of >= kKeyedMinEntries entries; tests, profiling)
    static int count_path() {
        const char* v = std::getenv("FSM_COUNT_PATH");
        if (!v) return 0;
        return !std::strcmp(v, "keys") ? 2 : (!std::strcmp(v, "atomic") ? 1 : 0);
    }
    // Keyed counting pays one group pass per kGroupCounters counters and a key pass
    // over the entries, atomics one memory-side atomic per join: keyed when the
    // batch's joins (estimated as sum cap^2 / runs, runs <= the prefix support)
    // reach both its counters and twice its entries.
    // 0: global atomics (k_count), 1: keyed
    int count_mode(const Batch& b) const {
        const int cp = count_path();
        if (b.root || b.E == 0 || b.E >= kNone || cp == 1) return 0;
        if (cp == 2) return 1;
        static const uint64_t min_e = [] {  // FSM_KEYED_MIN overrides kKeyedMinEntries (tuning)
            const char* v = std::getenv("FSM_KEYED_MIN");
            return v ? uint64_t(std::strtoull(v, nullptr, 10)) : uint64_t(kKeyedMinEntries);
        }();
        if (b.E < min_e) return 0;
        const int64_t ncls = int64_t(b.cls.size());
        const int64_t nthr = ncls >= (int64_t(1) << 15) ? host_threads() : 1;
        std::vector<double> te(size_t(nthr), 0), tn(size_t(nthr), 0);
        par_slices(nthr, ncls, [&](int64_t t, int64_t c0, int64_t c1) {
            double e = 0, n = 0;
            for (int64_t c = c0; c < c1; ++c) {
                const ClassMeta& m = b.cls[size_t(c)];
                e += double(m.cap) * double(m.cap) / double(std::max<uint32_t>(m.psup, 1));
                n += double(m.D >> m.mshift) * double(m.D);
            }
            te[size_t(t)] = e;
            tn[size_t(t)] = n;
        });
        double est = 0, ncnt = 0;
        for (int64_t t = 0; t < nthr; ++t) {
            est += te[size_t(t)];
            ncnt += tn[size_t(t)];
        }
        if (ctx->opts.verbose)
            std::fprintf(stderr, "[fsm] batch entries %llu: estimated joins %.3g, counters %.3g\n",
                         (unsigned long long)b.E, est, ncnt);
        // measured on MI355X: keyed wins on long runs (BIBLE/SIGN-shaped batches, >= 2 joins
        // per entry); at about one join per entry (Quest D1M) its key pass costs as much as the
        // atomics
        return est >= ncnt && est >= 2.0 * double(b.E) ? 1 : 0;
    }

    // Keyed count of a (non-root) batch laid out by prepare(b, true): plan ->
    // scan -> keys -> per-group LDS count writing the counters out.  Returns
    // false when the geometry does not apply (the atomic path then runs).
    bool keyed_count(Batch& b, DevBuf& cnt) {
        const uint64_t G64 = (b.n_cnt + kGroupCounters - 1) >> kGroupShift;
        if (G64 == 0 || G64 > kMaxGroups) return false;
        const uint32_t G = uint32_t(G64), E = uint32_t(b.E);
#ifndef FSM_CK_EPB
#define FSM_CK_EPB 8192
#endif
        const uint32_t nblk = uint32_t(std::min<uint64_t>(kF2MaxBlocks, std::max<uint64_t>(1, (b.E + FSM_CK_EPB - 1) / FSM_CK_EPB)));
        const uint32_t epb = (E + nblk - 1) / nblk;
        const uint64_t nd = uint64_t(G) * nblk;
        const SlabPtrs sp = b.slab.ptrs();
        const uint32_t mlo = member_lo(b), mhi = member_hi(b);
        DevBuf cap(nd * 4), base((nd + 1) * 8), fill(nd * 4);
        size_t tk = clk->begin("k_cnt_plan");
        hipLaunchKernelGGL(k_cnt_plan, dim3(nblk), dim3(kF2Threads), size_t(G) * 4, s, E, epb, sp.cid,
                           b.d_cls.as<DClass>(), sp.mem, sp.pos, mlo, mhi, G, nblk, cap.as<uint32_t>());
        FSM_LAUNCHED("k_cnt_plan", s);
        clk->end(tk, int64_t(b.E * 12 + nd * 4));
        scan_exclusive(cap.as<uint32_t>(), base.as<uint64_t>(), nd, s);
        FSM_HIP(hipMemcpyAsync(&pend[3], base.as<uint64_t>() + nd, 8, hipMemcpyDeviceToHost, s));
        sync();
        const uint64_t nslots = pend[3];
        if (nslots >= (uint64_t(1) << 32) - 4096) return false;  // region cursors are u32
        DevBuf keys((nslots + 1024) * 2);
        tk = clk->begin("k_cnt_keys");
#define FSM_CK(WW)                                                                                                   \
    hipLaunchKernelGGL(k_cnt_keys<WW>, dim3(nblk), dim3(kF2Threads), size_t(G) * 4, s, E, epb, sp.cid,                \
                       b.d_cls.as<DClass>(), sp.mem, sp.lohi, sp.pos, sp.mask, mlo, mhi, G, nblk, base.as<uint64_t>(), \
                       fill.as<uint32_t>(), keys.as<uint16_t>(), d_tests, uint32_t(W))
        FSM_W_DISPATCH(W, FSM_CK)
#undef FSM_CK
        FSM_LAUNCHED("k_cnt_keys", s);
        clk->end(tk, int64_t(b.E * entry_bytes() + nd * 12), int64_t(b.E * survey_entry_bytes()));
        cnt.alloc(std::max<uint64_t>(G64 << kGroupShift, 1) * 4);
        // few groups: several blocks per group (each over a range of the regions) keep the CUs busy
        const uint32_t parts = std::max<uint32_t>(1, std::min<uint32_t>({64u, 512u / G, nblk}));
        if (parts > 1) FSM_HIP(hipMemsetAsync(cnt.p, 0, (G64 << kGroupShift) * 4, s));
        tk = clk->begin("k_cnt_count");
        hipLaunchKernelGGL(k_f2_count<true>, dim3(G * parts), dim3(kF2Threads), 0, s, base.as<uint64_t>(),
                           fill.as<uint32_t>(), nblk, keys.as<uint16_t>(), 0u, 0u, 0u, 0u, 0u, 0u,
                           (FreqRec*)nullptr, 0u, (uint32_t*)nullptr, cnt.as<uint32_t>(), parts);
        FSM_LAUNCHED("k_cnt_count", s);
        clk->end(tk, int64_t(G64 << kGroupShift) * 4 + int64_t(nd) * 12);
        return true;
    }

    // the sparse count for batches whose dense counter matrices exceed 4 GiB (FSM_COUNT_PATH=
    // sparse forces it: tests); sparse_count itself falls back (false) when the keys would
    // not be smaller than the matrices
    bool sparse_wanted(const Batch& b) const {
        const char* v = std::getenv("FSM_COUNT_PATH");
        if (v && !std::strcmp(v, "sparse")) return true;
        return b.n_cnt * 4 >= (uint64_t(1) << 32);
    }
    bool sparse_count(Batch& b, std::vector<FreqRec>& recs, const RawVec<DRow>& rows) {
        const SlabPtrs sp = b.slab.ptrs();
        const uint32_t E = uint32_t(b.E), mlo = member_lo(b), mhi = member_hi(b);
        const unsigned grid = unsigned(std::min<uint64_t>((b.E + kBlock - 1) / kBlock, 8192));
        DevBuf capd(8), cur(8), nruns(4);
        FSM_HIP(hipMemsetAsync(capd.p, 0, 8, s));
        hipLaunchKernelGGL(k_sparse_cap, dim3(grid), dim3(kBlock), 0, s, E, sp.mem, sp.pos, mlo, mhi,
                           capd.as<unsigned long long>());
        FSM_LAUNCHED("k_sparse_cap", s);
        FSM_HIP(hipMemcpyAsync(&pend[3], capd.p, 8, hipMemcpyDeviceToHost, s));
        sync();
        const uint64_t capk = pend[3];
        const bool forced = [] { const char* v = std::getenv("FSM_COUNT_PATH"); return v && !std::strcmp(v, "sparse"); }();
        // keys, their sorted copy, the unique keys and counts: about 28 B per key
        if (!forced && (capk * 28 >= b.n_cnt * 4 || capk * 28 > budget)) return false;
        recs.clear();
        if (capk == 0) return true;
        DevBuf keys(capk * 8), sorted(capk * 8);
        FSM_HIP(hipMemsetAsync(cur.p, 0, 8, s));
        const size_t tk = clk->begin("k_count");
#define FSM_SK(WW)                                                                                                  \
    hipLaunchKernelGGL(k_sparse_keys<WW>, dim3(grid), dim3(kBlock), 0, s, E, sp.cid, b.d_cls.as<DClass>(), sp.mem,   \
                       sp.lohi, sp.pos, sp.mask, mlo, mhi, uint32_t(W), keys.as<unsigned long long>(),              \
                       cur.as<unsigned long long>(), d_tests)
        FSM_W_DISPATCH(W, FSM_SK)
#undef FSM_SK
        FSM_LAUNCHED("k_sparse_keys", s);
        clk->end(tk, int64_t(b.E * entry_bytes()), int64_t(b.E * survey_entry_bytes()));
        FSM_HIP(hipMemcpyAsync(&pend[3], cur.p, 8, hipMemcpyDeviceToHost, s));
        sync();
        const uint64_t n = pend[3];
        if (n > capk) throw Error(FSM_EDEVICE, "SPADE sparse count: more joins than their capacity");
        if (n == 0) return true;
        unsigned end_bit = 32;
        while (end_bit < 64 && (uint64_t(1) << (end_bit - 32)) < b.cbase_total) ++end_bit;
        DevBuf uniq(n * 8), counts(n * 4);
        sparse_sort_rle(keys.as<uint64_t>(), sorted.as<uint64_t>(), n, end_bit, uniq.as<uint64_t>(),
                        counts.as<uint32_t>(), nruns.as<uint32_t>(), s);
        // member slot -> counter row (the rows' index in `rows`)
        std::vector<uint32_t> s2r(size_t(std::max<uint64_t>(b.cbase_total, 1)), kNone);
        for (size_t q = 0; q < rows.size(); ++q) s2r[b.cls[rows[q].cls].cbase + rows[q].mi] = uint32_t(q);
        DevBuf d_s2r, flag(n * 4), off((n + 1) * 8);
        upload(d_s2r, s2r);
        const unsigned g2 = unsigned(std::min<uint64_t>((n + kBlock - 1) / kBlock, 8192));
        hipLaunchKernelGGL(k_sparse_flag, dim3(g2), dim3(kBlock), 0, s, counts.as<uint32_t>(), nruns.as<uint32_t>(),
                           uint32_t(n), minsup, flag.as<uint32_t>());
        FSM_LAUNCHED("k_sparse_flag", s);
        scan_exclusive(flag.as<uint32_t>(), off.as<uint64_t>(), n, s);
        FSM_HIP(hipMemcpyAsync(&pend[3], off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
        sync();
        const uint64_t nrec = pend[3];
        if (nrec) {
            DevBuf d_recs(nrec * sizeof(FreqRec));
            hipLaunchKernelGGL(k_sparse_recs, dim3(g2), dim3(kBlock), 0, s, uniq.as<uint64_t>(), counts.as<uint32_t>(),
                               nruns.as<uint32_t>(), off.as<uint64_t>(), d_s2r.as<uint32_t>(), minsup,
                               d_recs.as<FreqRec>());
            FSM_LAUNCHED("k_sparse_recs", s);
            recs.resize(nrec);
            FSM_HIP(hipMemcpyAsync(recs.data(), d_recs.p, nrec * sizeof(FreqRec), hipMemcpyDeviceToHost, s));
            sync();
        }
        return true;
    }

    void stats_for_class(const Batch& b, const ClassMeta& m) {
        const uint64_t S = m.nS, I = m.nI, sS = m.sS, sI = m.sI;
        fsm_stats& st = ctx->stats;
        const int64_t j = int64_t(S * S + I * S + (S ? S * (S - 1) / 2 : 0) + (I ? I * (I - 1) / 2 : 0));
        st.joins += j;
        if (b.root) st.joins_root += j;
        const uint64_t in = 2 * S * sS + S * sI + I * sS + (S ? (S - 1) * sS : 0) + (I ? (I - 1) * sI : 0);
        st.bytes_join_equiv += int64_t(12 * in);
        st.classes += 1;
    }

    // FSM_DEBUG_DUMP=1: print every class row entry of small batches (debugging aid)
    void dump(Batch& b) {
        static const bool on = [] { const char* v = std::getenv("FSM_DEBUG_DUMP"); return v && v[0] == '1'; }();
        const uint64_t n = b.E;
        if (!on || n > 4096 || b.db_direct) return;
        std::vector<uint32_t> cid(n), mem(n), lohi(n), pos(n);
        std::vector<uint64_t> mk(n * uint64_t(W));
        FSM_HIP(hipMemcpyAsync(cid.data(), b.slab.cid.p, n * 4, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipMemcpyAsync(mem.data(), b.slab.mem.p, n * 4, hipMemcpyDeviceToHost, s));
        if (b.slab.lohi.p) FSM_HIP(hipMemcpyAsync(lohi.data(), b.slab.lohi.p, n * 4, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipMemcpyAsync(pos.data(), b.slab.pos.p, n * 4, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipMemcpyAsync(mk.data(), b.slab.mask.p, n * 8 * W, hipMemcpyDeviceToHost, s));
        sync();
        if (!b.slab.lohi.p)  // (W = 1: derived from the mask)
            for (uint64_t e = 0; e < n; ++e)
                lohi[e] = mk[e] ? uint32_t(__builtin_ctzll(mk[e])) | ((63u - uint32_t(__builtin_clzll(mk[e]))) << 16) : 0u;
        std::fprintf(stderr, "[dump] depth=%lld classes=%zu\n", (long long)b.depth, b.cls.size());
        for (uint64_t e = 0; e < n; ++e) {
            std::fprintf(stderr, "    e=%llu cls=%u mem=%u lo=%u hi=%u off=%u len=%u mask=", (unsigned long long)e,
                         cid[e], mem[e], lohi[e] & 0xFFFF, lohi[e] >> 16, pos[e] >> 16, pos[e] & 0xFFFF);
            for (int w = 0; w < W; ++w) std::fprintf(stderr, "%016llx ", (unsigned long long)mk[e * W + w]);
            std::fprintf(stderr, "\n");
        }
    }

    // member ids whose counter rows this rank computes (all but the sharded root)
    uint32_t member_lo(const Batch& b) const { return comm && b.root ? 2 * slice_lo : 0u; }
    uint32_t member_hi(const Batch& b) const { return comm && b.root ? 2 * slice_hi : kNone; }

    // FSM_ROOT_PATH=atomic forces the global-atomic root F2 path (tests, profiling).
    static bool root_atomic() {
        const char* v = std::getenv("FSM_ROOT_PATH");
        return v && !std::strcmp(v, "atomic");
    }
    // grid cap of k_emit (FSM_EMIT_GRID overrides, for tuning)
    static uint64_t emit_grid_cap() {
        const char* v = std::getenv("FSM_EMIT_GRID");
        return v ? std::clamp<uint64_t>(std::strtoull(v, nullptr, 10), 256, 1u << 22) : (1u << 16);
    }
    // sharded mining: a first-level class whose estimated volume exceeds this fraction of a
    // rank's fair share is split (FSM_SPLIT_FRAC overrides; 0 or less disables splitting)
    static double split_frac() {
        const char* v = std::getenv("FSM_SPLIT_FRAC");
        const double f = v ? std::atof(v) : 0.5;
        return f > 0.0 ? f : 1e300;
    }
    // FSM_COUNT_KERNEL=thread forces the thread-per-entry k_count (tests, A/B runs; default: k_count2 at W = 1)
    static bool count_window() {
        const char* v = std::getenv("FSM_COUNT_KERNEL");
        return !(v && !std::strcmp(v, "thread"));
    }
    // FSM_KIDS=host builds the kid table on the host for every batch (tests, A/B; default:
    // large unsharded batches get it from k_freq_write + k_kid_off on the device)
    static bool kids_host() {
        const char* v = std::getenv("FSM_KIDS");
        return v && !std::strcmp(v, "host");
    }
    // FSM_EMIT_PATH=chunk forces k_emit1 for every batch (tests, A/B runs; default: k_emit2 at W = 1)
    static bool emit_window() {
        const char* v = std::getenv("FSM_EMIT_PATH");
        return !(v && !std::strcmp(v, "chunk"));
    }
    // emit's child_of table: built on the device for unsharded batches of at least 2^17
    // member slots (below that the launches cost more than the host fill + copy);
    // FSM_CHILD_OF=host / device forces either (tests, A/B)
    static bool child_of_device(uint64_t slots) {
        const char* v = std::getenv("FSM_CHILD_OF");
        if (v && !std::strcmp(v, "host")) return false;
        if (v && !std::strcmp(v, "device")) return true;
        return slots >= (uint64_t(1) << 17);
    }
    // LDS join records per wave of k_emit2 (FSM_EMIT_CAP lowers it too: tests of the overflow path)
    static uint32_t emit2_cap() {
        const char* v = std::getenv("FSM_EMIT_CAP");
        return v ? uint32_t(std::min<uint64_t>(std::strtoull(v, nullptr, 10), kE2Cap)) : kE2Cap;
    }
    // LDS join records per wave of k_emit1 (FSM_EMIT_CAP lowers it: tests of the overflow path)
    static uint32_t emit_cap() {
        const char* v = std::getenv("FSM_EMIT_CAP");
        return v ? uint32_t(std::min<uint64_t>(std::strtoull(v, nullptr, 10), kEmitCap)) : kEmitCap;
    }
    // class entries per block of k_count (FSM_COUNT_CHUNK overrides, for tuning)
    static uint32_t count_chunk() {
        const char* v = std::getenv("FSM_COUNT_CHUNK");
        return v ? uint32_t(std::clamp<uint64_t>(std::strtoull(v, nullptr, 10), 256, 1u << 20)) : kChunk;
    }
    // key alignment of the root F2 regions: 8 keys, so k_f2_count reads them in 16-byte words (64 or 256
    // measured no different in round 4)
    static constexpr uint32_t kF2Align = 8;
    // records from which the kid table and the children of a batch are built on the host
    // thread pool (below: one thread); FSM_HOST_PAR_MIN overrides (tuning)
    static uint64_t par_min() {
        static const uint64_t v = [] {
            const char* e = std::getenv("FSM_HOST_PAR_MIN");
            return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : uint64_t(1) << 16;
        }();
        return v;
    }
    // whether the DB-direct root's F2 takes the unordered-pair layout (run_root_db decides it the
    // same way, unless the rank's own slice is empty)
    bool tri_expected(uint32_t F) const {
        return W == 1 && f2_tri_env() && F > 0 && tri_len(F, 0) <= kGroupCounters &&
               root_db_env() && !root_atomic();
    }
    // the root F2 in the unordered-pair layout (k_f2_tri; FSM_F2_TRI=0: the ordered layout)
    static bool f2_tri_env() {
        const char* v = std::getenv("FSM_F2_TRI");
        return !(v && v[0] == '0');
    }
    // groups of the unordered-pair layout over the rows [rlo, rhi) of F ranks: gtab[i] = group <<
    // kGroupShift | first counter of row i; gr = the groups' first rows (G + 1).  0 groups: a
    // row does not fit a tile, or too many groups (the ordered layout runs)
    static uint32_t tri_tables(uint32_t F, uint32_t rlo, uint32_t rhi, std::vector<uint32_t>& tab) {
        if (F == 0 || tri_len(F, 0) > kGroupCounters || rlo >= rhi) return 0;
        tab.assign(size_t(F), 0u);
        std::vector<uint32_t> gr{rlo};
        uint32_t acc = 0;
        for (uint32_t i = rlo; i < rhi; ++i) {
            const uint32_t L = tri_len(F, i);
            if (acc + L > kGroupCounters) {
                gr.push_back(i);
                acc = 0;
            }
            tab[i] = uint32_t(gr.size() - 1) << kGroupShift | acc;
            acc += L;
        }
        gr.push_back(rhi);
        const uint32_t G = uint32_t(gr.size() - 1);
        if (G > kMaxGroups || G >= (1u << (32 - kGroupShift))) return 0;
        tab.insert(tab.end(), gr.begin(), gr.end());
        return G;
    }
    // row blocks of the root F2 (FSM_F2_BLOCKS overrides the target count, for tuning)
    static uint32_t f2_blocks() {
        const char* v = std::getenv("FSM_F2_BLOCKS");
        return v ? uint32_t(std::clamp<uint64_t>(std::strtoull(v, nullptr, 10), 1, kF2MaxBlocks)) : 1024u;
    }

    // Root F2 by rank groups (plan / k_f2_keys / k_f2_count): the
    // frequent (rank, slot) pairs of this rank's slice, sorted by (row, slot),
    // with their child member ids.  Returns false when a counter row does not
    // fit the LDS group tile, the groups are too many or the key slots exceed
    // 2^32 (the caller then takes the global-atomic path).
    // root F2 geometry: rank groups of `per` counter rows (128 KiB of LDS), row blocks of
    // rpb rows; ok = false when the group path does not apply (the atomic path runs)
    struct F2Geo {
        bool ok = false;
        uint32_t D = 0, F = 0, per = 0, G = 0, pm = 0, mlo = 0, mhi = 0, R = 0, rpb = 0, nblk = 0;
        uint64_t nd = 0;
    };
    F2Geo f2_geometry(const Batch& b, uint32_t D, uint64_t nent, uint64_t Rrows) const {
        F2Geo g;
        const uint32_t F = D / 2;
        if (nent == 0 || D > kGroupCounters || Rrows == 0 || F >= (1u << 15) || root_atomic()) return g;
        g.D = D;
        g.F = F;
        g.per = kGroupCounters / D;
        g.G = (F + g.per - 1) / g.per;
        if (g.G > kMaxGroups) return g;
        g.pm = uint32_t(((uint64_t(1) << 32) + g.per - 1) / g.per);  // group_of multiplier
        g.mlo = member_lo(b);
        g.mhi = member_hi(b);
        g.R = uint32_t(Rrows);
        const uint32_t nb_want = std::min<uint32_t>(f2_blocks(), kF2MaxBlocks);
        g.rpb = std::min<uint32_t>(kF2MaxRows, std::max<uint32_t>(16u, (g.R + nb_want - 1) / nb_want));
        if (uint64_t(g.rpb) * kF2MaxBlocks < g.R) return g;  // more rows than the LDS-indexed blocks cover
        g.nblk = (g.R + g.rpb - 1) / g.rpb;
        g.nd = uint64_t(g.G) * g.nblk;
        g.ok = true;
        return g;
    }

    bool root_f2(Batch& b, std::vector<FreqRec>& recs) {
        const ClassMeta& m = b.cls[0];
        if (b.root_rows.p == nullptr && !b.db_direct) return false;
        const F2Geo geo = f2_geometry(b, m.D, m.cap, b.R);
        if (!geo.ok) return false;
        const uint32_t D = geo.D, F = geo.F, per = geo.per, G = geo.G, pm = geo.pm, mlo = geo.mlo, mhi = geo.mhi;
        const uint32_t rlo = comm ? slice_lo : 0u, rhi = comm ? std::min(slice_hi, F) : F;
        const uint32_t R = geo.R, rpb = geo.rpb, nblk = geo.nblk;
        if (b.f2_tri) return root_f2_tri(b, recs, geo, rlo, rhi);
        const uint64_t nd = geo.nd;
        const SlabPtrs sp = b.slab.ptrs();
        const int64_t E0 = int64_t(m.cap);
        if (!b.f2_planned) return false;  // the plan is made while the root rows are written
        DevBuf base = std::move(b.f2_base), fill(nd * 4);
        const uint64_t nslots = b.f2_nslots;

        if (nslots >= (uint64_t(1) << 32) - 4096) return false;  // region cursors are u32
        // the one enumeration (keys padded: k_f2_count reads whole 16-byte words past a region's end)
        DevBuf keys((nslots + 1024) * 2), ctr_own;
        // u64 key count | u32 frequent-record count, read back together
        char* ctr = static_cast<char*>(zslot(16));
        if (!ctr) {
            ctr_own.alloc(16);
            FSM_HIP(hipMemsetAsync(ctr_own.p, 0, 16, s));
            ctr = ctr_own.as<char>();
        }
        unsigned long long* nk = reinterpret_cast<unsigned long long*>(ctr);
        uint32_t* d_nrec = reinterpret_cast<uint32_t*>(ctr + 8);
        const size_t kshm = size_t(kF2Waves) * 64 * (sizeof(F2Ent) + sizeof(F2Act)) + size_t(kF2RowWords) * 4 + size_t(G) * 4;
        // count + frequent pairs of this rank's slice
        const uint32_t g0 = rlo / per, g1 = rhi == 0 ? 0u : (rhi - 1) / per + 1;
        uint32_t cap_recs = uint32_t(std::min<uint64_t>(uint64_t(rhi - rlo) * D, uint64_t(1) << 20));
        DevBuf d_recs;
        unsigned long long nkeys = 0;
        size_t tk_cnt = 0, tk_keys = 0;
        // (one pass over every group of the slice: passes over group ranges, which keep a pass's
        // keys on-die, measured slower in round 4: each pass enumerates the rows again)
        for (int attempt = 0;; ++attempt) {
            d_recs.alloc(std::max<uint32_t>(cap_recs, 1) * sizeof(FreqRec));
            if (attempt > 0) FSM_HIP(hipMemsetAsync(d_nrec, 0, 4, s));
            {
                const uint32_t pg0 = g0, pg1 = g1, prlo = rlo, prhi = rhi;
                if (attempt == 0) {  // a retry (record overflow) counts from the keys already written
                    const uint32_t pmlo = mlo, pmhi = mhi;
                    tk_keys = clk->begin("k_f2_keys");
#define FSM_F2K(WW)                                                                                                   \
    hipLaunchKernelGGL((k_f2_keys<WW, false>), dim3(nblk), dim3(kF2Threads), kshm, s, b.root_rows.as<uint64_t>(),      \
                       (const uint32_t*)nullptr, RootRef{nullptr, nullptr}, R, rpb, sp.mem, sp.lohi, sp.mask, D, per,  \
                       pm, G, nblk, pmlo, pmhi, base.as<uint64_t>(), fill.as<uint32_t>(), keys.as<uint16_t>(),        \
                       nk, uint32_t(W))
#define FSM_F2KD(WW)                                                                                                  \
    hipLaunchKernelGGL((k_f2_keys<WW, true>), dim3(nblk), dim3(kF2Threads), kshm, s, (const uint64_t*)nullptr,         \
                       db->row_off.as<uint32_t>(), RootRef{db->item.as<uint32_t>(), b.rk2.as<uint32_t>()}, R, rpb,     \
                       b.mem_db.as<uint32_t>(), (const uint32_t*)nullptr, db->mask.as<uint64_t>(), D, per, pm, G,      \
                       nblk, pmlo, pmhi, base.as<uint64_t>(), fill.as<uint32_t>(), keys.as<uint16_t>(),               \
                       nk, uint32_t(WW))
                    if (b.db_direct) {
                        switch (W) {
                            case 1: FSM_F2KD(1); break;
                            case 2: FSM_F2KD(2); break;
                            case 4: FSM_F2KD(4); break;
                            default: FSM_F2KD(8); break;
                        }
                    } else {
                        FSM_W_DISPATCH(W, FSM_F2K)
                    }
#undef FSM_F2K
#undef FSM_F2KD
                    FSM_LAUNCHED("k_f2_keys", s);
                    // reads the slab (mem, lohi, mask) and the region bases, writes the fills;
                    // + 2 B per key actually written, added once the count is back
                    // DB-direct: the DB rows (item + mask per entry) instead of the slab's (mem, lohi, mask)
                    const int64_t rowb = b.db_direct ? db->E * int64_t(4 + 8 * W) : E0 * int64_t(8 + 8 * W);
                    clk->end(tk_keys, rowb + int64_t(nd) * 12, E0 * 8);
                }
                tk_cnt = clk->begin("k_f2_count");
                if (pg1 > pg0)
                    hipLaunchKernelGGL(k_f2_count<false>, dim3(pg1 - pg0), dim3(kF2Threads), 0, s, base.as<uint64_t>(),
                                       fill.as<uint32_t>(), nblk, keys.as<uint16_t>(), D, per, pg0, prlo, prhi, minsup,
                                       d_recs.as<FreqRec>(), cap_recs, d_nrec, (uint32_t*)nullptr, 1u);
                FSM_LAUNCHED("k_f2_count", s);
                clk->end(tk_cnt, int64_t(pg1 - pg0) * nblk * 12);
            }
            pend[2] = pend[3] = 0;
            FSM_HIP(hipMemcpyAsync(&pend[2], ctr, 16, hipMemcpyDeviceToHost, s));  // (one copy: both counts)
            sync();
            nkeys = pend[2];
            const uint32_t nrec = uint32_t(pend[3] & 0xFFFFFFFFu);
            if (nrec <= cap_recs || attempt > 0) {
                if (nrec > cap_recs) throw Error(FSM_EDEVICE, "SPADE root F2: frequent pair buffer overflow");
                recs.resize(nrec);
                if (nrec)
                    FSM_HIP(hipMemcpyAsync(recs.data(), d_recs.p, size_t(nrec) * sizeof(FreqRec), hipMemcpyDeviceToHost,
                                           s));
                sync();
                break;
            }
            cap_recs = nrec;  // rare: more frequent pairs than the first buffer held; count again
        }
        clk->add_bytes(tk_keys, int64_t(nkeys) * 2);
        clk->add_bytes(tk_cnt, int64_t(nkeys) * 2 + int64_t(recs.size() * sizeof(FreqRec)));
        ctx->stats.root_keys += int64_t(nkeys);
        // (row, slot) order and child member ids: rank among the row's slots with a frequent
        // temporal or equality candidate, << 1 | type (as k_freq_write assigns them)
        const double th0 = now_ms();
        order_recs(recs, F, &rec_off_s);
        rec_off_ok = true;
        hp[0] += now_ms() - th0;
        return true;
    }
    // The root F2 in the unordered-pair layout (k_f2_plan_db with the group table, k_f2_tri,
    // k_f2_count<false, true>): the frequent ordered pairs of the rows [rlo, rhi), as records
    // in (row, slot) order.  A pair (i, j) counts where the lower rank i is owned, so a rank's
    // records also hold rows j above its slice (the sharded gather orders them again).
    // the k_f2_tri launch of the root (once; false: the slot count exceeds the u32 cursors)
    bool launch_f2_tri(Batch& b, const F2Geo& geo) {
        if (b.f2_launched) return true;
        const uint32_t G = b.f2_tri_G, R = geo.R, rpb = geo.rpb, nblk = geo.nblk;
        const uint64_t nd = uint64_t(G) * nblk;
        const uint64_t nslots = b.f2_nslots;
        if (nslots >= (uint64_t(1) << 32) - 4096) return false;
        b.f2_fill.alloc(nd * 4);
        b.f2_keys.alloc((nslots + 1024) * 2);
        // u64 key count | u32 frequent-record count, read back together
        b.f2_ctr = static_cast<char*>(zslot(16));
        if (!b.f2_ctr) {
            b.f2_ctr_own.alloc(16);
            FSM_HIP(hipMemsetAsync(b.f2_ctr_own.p, 0, 16, s));
            b.f2_ctr = b.f2_ctr_own.as<char>();
        }
        const uint32_t* gtab = b.f2_tri_tab.as<uint32_t>();
        const size_t kshm = size_t(kF2Waves) * 64 * 16 + size_t(kF2RowWords) * 4 + size_t(G) * 4;
        b.f2_tk = clk->begin("k_f2_keys");
        hipLaunchKernelGGL(k_f2_tri, dim3(nblk), dim3(kF2Threads), kshm, s, db->row_off.as<uint32_t>(),
                           b.mem_db.as<uint32_t>(), db->mask.as<uint64_t>(), R, rpb, gtab, G, nblk, geo.mlo, geo.mhi,
                           b.f2_base.as<uint64_t>(), b.f2_fill.as<uint32_t>(), b.f2_keys.as<uint16_t>(),
                           reinterpret_cast<unsigned long long*>(b.f2_ctr));
        FSM_LAUNCHED("k_f2_tri", s);
        clk->end(b.f2_tk, db->E * 12 + int64_t(nd) * 12, int64_t(b.cls[0].cap) * 8);
        b.f2_launched = true;
        return true;
    }

    bool root_f2_tri(Batch& b, std::vector<FreqRec>& recs, const F2Geo& geo, uint32_t rlo, uint32_t rhi) {
        const uint32_t F = geo.F, G = b.f2_tri_G, nblk = geo.nblk;
        if (!launch_f2_tri(b, geo)) return false;
        DevBuf base = std::move(b.f2_base), fill = std::move(b.f2_fill), keys = std::move(b.f2_keys),
               ctr_own = std::move(b.f2_ctr_own);
        char* ctr = b.f2_ctr;
        const size_t tk_keys = b.f2_tk;
        uint32_t* d_nrec = reinterpret_cast<uint32_t*>(ctr + 8);
        const uint32_t* gtab = b.f2_tri_tab.as<uint32_t>();
        const uint32_t* gr = gtab + F;
        // count + frequent pairs (a retry when the first record buffer was too small)
        // the records land in mapped pinned host memory, the counts in pinned slots: one sync
        uint32_t cap_recs = uint32_t(std::min<uint64_t>(uint64_t(rhi - rlo) * 2 * F, uint64_t(1) << 20));
        size_t tk_cnt = 0;
        unsigned long long nkeys = 0;
        for (int attempt = 0;; ++attempt) {
            PinnedBuf* pb = ctx->pinned_big(size_t(std::max<uint32_t>(cap_recs, 1)) * sizeof(FreqRec));
            if (attempt > 0) FSM_HIP(hipMemsetAsync(d_nrec, 0, 4, s));
            tk_cnt = clk->begin("k_f2_count");
            hipLaunchKernelGGL((k_f2_count<false, true>), dim3(G), dim3(kF2Threads), 0, s, base.as<uint64_t>(),
                               fill.as<uint32_t>(), nblk, keys.as<uint16_t>(), 2 * F, 0u, 0u, rlo, rhi, minsup,
                               static_cast<FreqRec*>(pb->dev), cap_recs, d_nrec, (uint32_t*)nullptr, 1u,
                               gr, F);
            FSM_LAUNCHED("k_f2_count", s);
            clk->end(tk_cnt, int64_t(G) * nblk * 12);
            pend[2] = pend[3] = 0;
            FSM_HIP(hipMemcpyAsync(&pend[2], ctr, 16, hipMemcpyDeviceToHost, s));  // (one copy: both counts)
            sync();
            nkeys = pend[2];
            const uint32_t nrec = uint32_t(pend[3] & 0xFFFFFFFFu);
            if (nrec <= cap_recs || attempt > 0) {
                if (nrec > cap_recs) throw Error(FSM_EDEVICE, "SPADE root F2: frequent pair buffer overflow");
                const FreqRec* hr = static_cast<const FreqRec*>(pb->host);
                double tr = now_ms();
                if (b.f2_tri && F < (1u << 15) && order_device(b, pb, nrec, F, RkRows{nullptr, nullptr, F}, 2 * F, 2 * size_t(F) + 1)) {
                    recs.clear();
                    lap(14, tr);
                    clk->add_bytes(tk_keys, int64_t(nkeys) * 2);
                    clk->add_bytes(tk_cnt, int64_t(nkeys) * 2 + int64_t(nrec) * int64_t(sizeof(FreqRec)));
                    ctx->stats.root_keys += int64_t(nkeys);
                    return true;
                }
                recs.assign(hr, hr + nrec);
                lap(14, tr);
                break;
            }
            cap_recs = nrec;
        }
        clk->add_bytes(tk_keys, int64_t(nkeys) * 2);
        clk->add_bytes(tk_cnt, int64_t(nkeys) * 2 + int64_t(recs.size() * sizeof(FreqRec)));
        ctx->stats.root_keys += int64_t(nkeys);
        const double th0 = now_ms();
        double to_ = now_ms();
        order_recs(recs, F, &rec_off_s);
        lap(15, to_);
        rec_off_ok = true;
        hp[0] += now_ms() - th0;
        return true;
    }
    // FSM_DEVORDER=0: a batch's records ordered on the host (A/B)
    static bool devorder_env() {  // (read per batch: the tests switch it within one process)
        const char* v = std::getenv("FSM_DEVORDER");
        return !(v && v[0] == '0');
    }
    // A batch's nrec frequent records (unordered, mapped pinned memory pb) ordered on the device
    // with the kid table [koff: nko | kslot | kcid] and the child-class table (k_rk_*), written
    // back into pb in order (event b.rec_ev), and the batch set up for a deferred emit whose slab
    // is sized by every record's support (the lone itemset extensions' entries are counted out
    // when the children are built).  rr: the counter rows (nrows), dmax: the largest member id
    // space of a row's class.  false: the host orders them (sharded, claims, over budget).
    bool order_device(Batch& b, PinnedBuf* pb, uint32_t nrec, uint32_t nrows, RkRows rr, uint32_t dmax, size_t nko) {
        if (comm || nrec == 0 || nrows == 0 || !devorder_env() || defer_env() == 0 || b.claim_key >= 0 ||
            dmax >= (1u << 16) || nko >= kNone)
            return false;
        const FreqRec* hr = static_cast<const FreqRec*>(pb->host);
        uint64_t sumsup = 0;
        for (uint32_t q = 0; q < nrec; ++q) sumsup += hr[q].sup;
        // a row's c records give its child class D <= 2c <= 2 dmax members: sum (2c)^2 4 B <= 16 nrec dmax
        if (sumsup * entry_bytes() + 16ull * nrec * dmax > budget || sumsup > (uint64_t(1) << 31)) return false;
        const uint32_t n = nrec;
        FreqRec* R = static_cast<FreqRec*>(pb->dev);
        DevBuf Rd(size_t(n) * sizeof(FreqRec)), rowcnt(size_t(nrows) * 4), rowoff(size_t(nrows + 1) * 4),
            idx(size_t(n) * 4);
        b.kid_tab.alloc((nko + 2 * size_t(n)) * 4);
        b.ord_child_of.alloc(std::max<size_t>(nko - 1, 1) * 4);
        uint32_t* cnt = rowcnt.as<uint32_t>();  // row counts | kRkEven
        FSM_HIP(hipMemsetAsync(cnt, 0, size_t(nrows) * 4, s));
        const unsigned gn = unsigned(std::min<uint64_t>((uint64_t(n) + kBlock - 1) / kBlock, 1024));
        hipLaunchKernelGGL(k_rk_hist, dim3(gn), dim3(kBlock), 0, s, R, n, Rd.as<FreqRec>(), cnt);
        FSM_LAUNCHED("k_rk_hist", s);
        uint32_t* koff = b.kid_tab.as<uint32_t>();
        hipLaunchKernelGGL(k_rk_tables, dim3((nrows + kRkTile - 1) / kRkTile), dim3(kBlock), 0, s, cnt, nrows, rr,
                           uint32_t(nko), rowoff.as<uint32_t>(), koff, b.ord_child_of.as<uint32_t>());
        FSM_LAUNCHED("k_rk_tables", s);
        hipLaunchKernelGGL(k_rk_scatter, dim3(gn), dim3(kBlock), 0, s, Rd.as<FreqRec>(), n, rowoff.as<uint32_t>(), cnt,
                           idx.as<uint32_t>());
        FSM_LAUNCHED("k_rk_scatter", s);
        const uint32_t nwmax = (dmax + 31) / 32;
        const size_t lds = size_t(3) * nwmax * 4;  // (dmax < 2^16: at most 24 KiB)
        // the ordered records go straight back over the unordered ones in pinned memory
        // (k_rk_hist has copied those into HBM)
        hipLaunchKernelGGL(k_rk_row, dim3(nrows), dim3(kBlock), lds, s, Rd.as<FreqRec>(), idx.as<uint32_t>(),
                           rowoff.as<uint32_t>(), rr, nwmax, R, koff + nko, koff + nko + n);
        FSM_LAUNCHED("k_rk_row", s);
        if (!b.rec_ev) FSM_HIP(hipEventCreateWithFlags(&b.rec_ev, hipEventDisableTiming));
        FSM_HIP(hipEventRecord(b.rec_ev, s));
        b.kid_off = b.kid_tab.as<uint32_t>();
        b.kid_slot = b.kid_off + nko;
        b.kid_cid = b.kid_slot + n;
        b.child_of_pre = b.ord_child_of.as<uint32_t>();
        b.dev_order = true;
        b.defer_children = true;
        b.defer_R = hr;
        b.defer_n = nrec;
        b.defer_total = sumsup;  // (an upper bound: emit() counts the children's entries exactly)
        b.defer_rows = &rows_s;
        b.children.clear();
        b.groups.assign(1, {size_t(0), size_t(0)});  // (the child count: set by emit())
        b.next_group = 0;
        return true;
    }

    // The children loop of count_and_freq split over host threads (unsharded, large
    // batches; same tables, same node ids: node of record q = first + q).  Every step
    // runs over the same host-thread slices: row groups of the records (counts, then
    // positions) -> per-group sizes and per-slice sums -> slice bases -> fill, each
    // slice initialising its own ranges of the member tables.
    void children_parallel(Batch& b, const FreqRec* R, uint64_t nfreq, const RawVec<DRow>& rows) {
        double tl = now_ms();
        const int64_t nthr = host_threads();
        std::vector<int64_t> tg(size_t(nthr) + 1, 0);
        par_slices(nthr, int64_t(nfreq), [&](int64_t t, int64_t q0, int64_t q1) {
            int64_t c = 0;
            for (int64_t q = q0; q < q1; ++q) c += q == 0 || R[q].row != R[q - 1].row;
            tg[size_t(t) + 1] = c;
        });
        for (int64_t t = 0; t < nthr; ++t) tg[size_t(t) + 1] += tg[size_t(t)];
        const int64_t ng = tg[size_t(nthr)];
        RawVec<uint64_t>& gs = gs_s;  // first record of each row group
        gs.resize(size_t(ng) + 1);
        par_slices(nthr, int64_t(nfreq), [&](int64_t t, int64_t q0, int64_t q1) {
            int64_t at = tg[size_t(t)];
            for (int64_t q = q0; q < q1; ++q)
                if (q == 0 || R[q].row != R[q - 1].row) gs[size_t(at++)] = uint64_t(q);
        });
        gs[size_t(ng)] = nfreq;
        lap(0, tl);
        // r2: member ranks of each group's child (bit 31: the child is kept; a lone
        // itemset-extension opens no class)
        RawVec<uint32_t>& r2 = r2_s;
        r2.resize(size_t(ng));
        std::vector<uint64_t> tri(size_t(nthr) + 1, 0), tk(size_t(nthr) + 1, 0);
        par_slices(nthr, ng, [&](int64_t t, int64_t i0, int64_t i1) {
            uint64_t sri = 0, sk = 0;
            for (int64_t i = i0; i < i1; ++i) {
                uint32_t maxcid = 0;
                for (uint64_t q = gs[size_t(i)]; q < gs[size_t(i) + 1]; ++q) maxcid = std::max(maxcid, R[q].cid);
                const uint32_t r = (maxcid >> 1) + 1;
                const uint64_t nch = gs[size_t(i) + 1] - gs[size_t(i)];
                const bool keep = !(nch == 1 && (R[gs[size_t(i)]].slot & 1u) == kItm);
                r2[size_t(i)] = r | (keep ? 0x80000000u : 0u);
                sri += r;
                sk += keep;
            }
            tri[size_t(t) + 1] = sri;
            tk[size_t(t) + 1] = sk;
        });
        for (int64_t t = 0; t < nthr; ++t) {
            tri[size_t(t) + 1] += tri[size_t(t)];
            tk[size_t(t) + 1] += tk[size_t(t)];
        }
        lap(1, tl);
        b.child_rank_item.resize(tri[size_t(nthr)]);
        b.child_node_of.resize(2 * tri[size_t(nthr)]);
        b.children.resize(tk[size_t(nthr)]);
        const size_t node0 = nodes.size();
        nodes.grow(nfreq);
        lap(3, tl);
        std::vector<int64_t> jb(size_t(nthr), 0);
        std::vector<int> bad(size_t(nthr), 0);
        par_slices(nthr, ng, [&](int64_t t, int64_t i0, int64_t i1) {
            int64_t acc = 0;
            uint64_t ri = tri[size_t(t)], kidx = tk[size_t(t)];
            for (int64_t i = i0; i < i1; ++i) {
                const uint64_t q0 = gs[size_t(i)], q1 = gs[size_t(i) + 1];
                const uint32_t r = r2[size_t(i)] & 0x7FFFFFFFu;
                const DRow pr = rows[R[q0].row];
                const ClassMeta& pm = b.cls[pr.cls];
                const int32_t parent = b.node_of[pm.no_off + pr.mi];
                const uint32_t pls = nodes[size_t(parent)].len_sets;
                if ((pls >> 16) >= 0xFFFFu) bad[size_t(t)] |= 1;
                ChildInfo ch;
                ch.pcls = pr.cls;
                ch.pmi = pr.mi;
                ch.D = 2 * r;
                ch.ri_off = ri;
                ch.no_off = 2 * ri;
                ch.psup = nodes[size_t(parent)].support;
                std::fill_n(b.child_rank_item.data() + ri, r, 0u);
                std::fill_n(b.child_node_of.data() + 2 * ri, 2 * r, -1);
                for (uint64_t q = q0; q < q1; ++q) {
                    const FreqRec& fr = R[q];
                    const uint32_t item = b.rank_item[pm.ri_off + (fr.slot >> 1)];
                    const size_t node = node0 + q;
                    nodes[node] = PNode{parent, item, fr.slot & 1u, fr.sup, pls + (1u << 16) + ((fr.slot & 1u) == kSeq)};
                    b.child_rank_item[ch.ri_off + (fr.cid >> 1)] = item;
                    b.child_node_of[ch.no_off + fr.cid] = int32_t(node);
                    ch.cap += fr.sup;
                    if ((fr.slot & 1u) == kSeq) { ++ch.nS; ch.sS += fr.sup; } else { ++ch.nI; ch.sI += fr.sup; }
                    acc += int64_t(12ull * fr.sup);
                }
                ri += r;
                if (r2[size_t(i)] >> 31) b.children[kidx++] = ch;
            }
            jb[size_t(t)] = acc;
        });
        lap(4, tl);
        for (int64_t t = 0; t < nthr; ++t) {
            if (bad[size_t(t)] & 1) throw Error(FSM_ELIMIT, "SPADE: a pattern exceeds 65534 items");
            ctx->stats.bytes_join_equiv += jb[size_t(t)];
        }
    }

    // count kernel + frequent-candidate extraction; fills b.children / b.groups / kids
    void count_and_freq(Batch& b) {
        const double tc0 = now_ms();
        rec_off_ok = false;
        double tl = tc0;
        // FSM_HOST_TRACE=2: one line per batch with its host phases (diagnostics)
        struct BatchTrace {
            Miner* m;
            Batch* b;
            double h0[8], t0;
            ~BatchTrace() {
                std::fprintf(stderr, "[fsm batch] depth %lld root %d E %llu classes %zu children %zu: %.3f ms (", (long long)b->depth,
                             int(b->root), (unsigned long long)b->E, b->cls.size(), b->children.size(), now_ms() - t0);
                for (int i = 0; i < 8; ++i) std::fprintf(stderr, " %.3f", m->hp[i] - h0[i]);
                std::fprintf(stderr, " )\n");
            }
        };
        static const bool btrace = [] { const char* v = std::getenv("FSM_HOST_TRACE"); return v && v[0] == '2'; }();
        std::unique_ptr<BatchTrace> bt;
        if (btrace) {
            bt = std::make_unique<BatchTrace>();
            bt->m = this;
            bt->b = &b;
            for (int i = 0; i < 8; ++i) bt->h0[i] = hp[i];
            bt->t0 = tc0;
        }
        dump(b);
        const int cmode = count_mode(b);
        lap(5, tl);
        const bool keyed_layout = prepare(b, cmode != 0);
        lap(6, tl);
        const bool shard = comm && b.root;  // root rows split over ranks, frequent pairs all-gathered
        const int64_t ncls = int64_t(b.cls.size());
        const int64_t nthr = ncls >= (int64_t(1) << 15) ? host_threads() : 1;
        // the root and split classes are counted by every rank: their stats come from rank 0
        if (comm || nthr == 1) {
            for (auto& m : b.cls)
                if (!comm || (!shard && !m.split) || comm->rank() == 0) stats_for_class(b, m);
        } else {  // unsharded, many classes: the same sums over host threads
            std::vector<int64_t> sj(size_t(nthr), 0), sb(size_t(nthr), 0);
            par_slices(nthr, ncls, [&](int64_t t, int64_t c0, int64_t c1) {
                int64_t j = 0, bb = 0;
                for (int64_t c = c0; c < c1; ++c) {
                    const ClassMeta& m = b.cls[size_t(c)];
                    const uint64_t S = m.nS, I = m.nI, sS = m.sS, sI = m.sI;
                    j += int64_t(S * S + I * S + (S ? S * (S - 1) / 2 : 0) + (I ? I * (I - 1) / 2 : 0));
                    bb += int64_t(12 * (2 * S * sS + S * sI + I * sS + (S ? (S - 1) * sS : 0) + (I ? (I - 1) * sI : 0)));
                }
                sj[size_t(t)] = j;
                sb[size_t(t)] = bb;
            });
            for (int64_t t = 0; t < nthr; ++t) {
                ctx->stats.joins += sj[size_t(t)];
                if (b.root) ctx->stats.joins_root += sj[size_t(t)];
                ctx->stats.bytes_join_equiv += sb[size_t(t)];
            }
            ctx->stats.classes += ncls;
        }
        lap(7, tl);
        fsm_stats& st = ctx->stats;
        st.batches += 1;
        const uint64_t tot_ent = b.E;
        st.entries += int64_t(tot_ent);
        st.bytes_streamed += int64_t(tot_ent * entry_bytes());
        st.bytes_count_alg += int64_t(tot_ent * entry_bytes());
        // member rows of the counter matrix
        RawVec<DRow>& rows = rows_s;
        rows.clear();
        if (nthr == 1) {
            for (size_t c = 0; c < b.cls.size(); ++c)
                for (uint32_t mi = 0; mi < b.cls[c].D; ++mi)
                    if (b.node_of[b.cls[c].no_off + mi] >= 0) rows.push_back(DRow{uint32_t(c), mi});
        } else {  // a class's rows are its members (nS + nI of them): slice sums, then a parallel fill
            std::vector<uint64_t> ro(size_t(nthr) + 1, 0);
            par_slices(nthr, ncls, [&](int64_t t, int64_t c0, int64_t c1) {
                uint64_t n = 0;
                for (int64_t c = c0; c < c1; ++c) n += b.cls[size_t(c)].nS + b.cls[size_t(c)].nI;
                ro[size_t(t) + 1] = n;
            });
            for (int64_t t = 0; t < nthr; ++t) ro[size_t(t) + 1] += ro[size_t(t)];
            rows.resize(ro[size_t(nthr)]);
            par_slices(nthr, ncls, [&](int64_t t, int64_t c0, int64_t c1) {
                uint64_t at = ro[size_t(t)];
                for (int64_t c = c0; c < c1; ++c) {
                    const ClassMeta& m = b.cls[size_t(c)];
                    for (uint32_t mi = 0; mi < m.D; ++mi)
                        if (b.node_of[m.no_off + mi] >= 0) rows[at++] = DRow{uint32_t(c), mi};
                }
            });
        }
        // root rows are rows[r] = rank r: a shard extracts its own slice of them
        const uint32_t rlo = shard ? std::min<uint32_t>(slice_lo, uint32_t(rows.size())) : 0u;
        const uint32_t rhi = shard ? std::min<uint32_t>(slice_hi, uint32_t(rows.size())) : uint32_t(rows.size());
        const uint32_t nrows = rhi - rlo;
        std::vector<FreqRec>& recs = recs_s;
        recs.clear();
        const FreqRec* ext = nullptr;  // ordered extraction: the records in pinned host memory
        uint64_t ext_n = 0;
        bool kids_dev = false;  // the kid table was built on the device (k_freq_write + k_kid_off)
        DevBuf cnt;
        lap(8, tl);
        hp[6] += now_ms() - tc0;  // prepare + stats + rows
        const double tc1 = now_ms();
        auto compute = [&] {
        // the root: pairs counted per rank group, only the frequent ones leave the device
        const bool root_done = b.E && b.root && !root_atomic() && root_f2(b, recs);
        if (b.db_direct && b.E && !root_done)
            throw Error(FSM_EDEVICE, "SPADE internal error: the DB-direct root F2 did not apply");
        if (b.E) st.count_launches += 1;
        // huge, sparse counter matrices: the joins sorted instead (records in (row, slot) order)
        const bool sparse_done = !root_done && b.E && sparse_wanted(b) && sparse_count(b, recs, rows);
        if (sparse_done) {
            order_recs(recs, uint32_t(rows.size()), &rec_off_s);
            rec_off_ok = true;
            return;
        }
        const bool keyed_done = !root_done && keyed_layout && keyed_count(b, cnt);
        uint32_t* d_nz = nullptr;  // a zeroed u32 after the counters (the extraction's record count)
        if (!root_done && !keyed_done) {
            cnt.alloc((b.n_cnt + 1) * 4);
            FSM_HIP(hipMemsetAsync(cnt.p, 0, (b.n_cnt + 1) * 4, s));
            d_nz = cnt.as<uint32_t>() + b.n_cnt;
        }
        if (!root_done) {
            if (b.E && !keyed_done) {
                const SlabPtrs sp = b.slab.ptrs();
                const uint32_t cchunk = count_chunk();
#define FSM_COUNT(WW)                                                                                   \
    hipLaunchKernelGGL(k_count<WW>, dim3(unsigned((b.E + cchunk - 1) / cchunk)), dim3(kBlock), 0, s,   \
                       uint32_t(b.E), sp.cid, b.d_cls.as<DClass>(), sp.mem, sp.lohi, sp.pos, sp.mask,           \
                       member_lo(b), member_hi(b), cchunk, cnt.as<uint32_t>(), d_tests,    \
                       uint32_t(W))
                const size_t tk = clk->begin("k_count");
                if ((W == 1 || W == 2 || W == 4 || W == 8) && count_window()) {
                    const unsigned g = unsigned(std::min<uint64_t>((b.E + 4 * kC2Range - 1) / (4 * kC2Range), 1u << 16));
#define FSM_COUNT2(WW)                                                                                  \
    hipLaunchKernelGGL(k_count2<WW>, dim3(g), dim3(kBlock), 0, s, uint32_t(b.E), sp.cid, b.d_cls.as<DClass>(), \
                       sp.mem, sp.lohi, sp.pos, sp.mask, member_lo(b), member_hi(b), cnt.as<uint32_t>(),      \
                       d_tests)
                    switch (W) {
                        case 1: FSM_COUNT2(1); break;
                        case 2: FSM_COUNT2(2); break;
                        case 4: FSM_COUNT2(4); break;
                        default: FSM_COUNT2(8); break;
                    }
#undef FSM_COUNT2
                } else {
                    FSM_W_DISPATCH(W, FSM_COUNT)
                }
#undef FSM_COUNT
                FSM_LAUNCHED("k_count", s);
                clk->end(tk, int64_t(b.E * entry_bytes() + b.n_cnt * 4), int64_t(b.E * survey_entry_bytes()));
            }
            DevBuf d_rows;
            upload_staged(1, d_rows, rows.data() + rlo, size_t(nrows) * sizeof(DRow));
            const unsigned grid = unsigned((uint64_t(nrows) * 64 + kBlock - 1) / kBlock);
            if (nrows > kFreqOnePassRows) {
                // large batches: ordered extraction (the host ordering and the mapped-memory
                // reads of millions of records cost more than the extra sync)
                DevBuf rowcnt((size_t(nrows) + 1) * 4), rowoff((size_t(nrows) + 1) * 8);
                {
                    const size_t tk = clk->begin("k_freq_count");
                    hipLaunchKernelGGL(k_freq_count, dim3(grid), dim3(kBlock), 0, s, d_rows.as<DRow>(), nrows,
                                       b.d_cls.as<DClass>(), cnt.as<uint32_t>(), minsup, rowcnt.as<uint32_t>());
                    FSM_LAUNCHED("k_freq_count", s);
                    clk->end(tk, int64_t(uint64_t(nrows) * (b.n_cnt / std::max<uint64_t>(rows.size(), 1)) * 4));
                }
                scan_exclusive(rowcnt.as<uint32_t>(), rowoff.as<uint64_t>(), nrows, s);
                FSM_HIP(hipMemcpyAsync(&pend[1], rowoff.as<uint64_t>() + nrows, 8, hipMemcpyDeviceToHost, s));
                sync();
                const uint64_t nf = pend[1];
                if (nf) {  // records straight into mapped pinned host memory, read there after the sync
                    PinnedBuf* pb = ctx->pinned_big(nf * sizeof(FreqRec));
                    // unsharded: the kid table [koff | kslot | kcid] is built here, in HBM
                    const bool dk = !comm && !kids_host() && rlo == 0 && nrows == rows.size();
                    const size_t nko = size_t(b.cbase_total) + 1;
                    uint32_t *kslot = nullptr, *kcid = nullptr;
                    if (dk) {
                        b.kid_tab.alloc((nko + 2 * size_t(nf)) * 4);
                        kslot = b.kid_tab.as<uint32_t>() + nko;
                        kcid = kslot + nf;
                    }
                    const size_t tk = clk->begin("k_freq_write");
                    hipLaunchKernelGGL(k_freq_write, dim3(grid), dim3(kBlock), 0, s, d_rows.as<DRow>(), nrows,
                                       b.d_cls.as<DClass>(), cnt.as<uint32_t>(), minsup, rowoff.as<uint64_t>(), rlo,
                                       static_cast<FreqRec*>(pb->dev), kslot, kcid);
                    FSM_LAUNCHED("k_freq_write", s);
                    if (dk) {
                        hipLaunchKernelGGL(k_kid_off, dim3(unsigned((nrows + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                                           d_rows.as<DRow>(), nrows, b.d_cls.as<DClass>(), rowoff.as<uint64_t>(),
                                           uint32_t(nko), b.kid_tab.as<uint32_t>());
                        FSM_LAUNCHED("k_kid_off", s);
                        kids_dev = true;
                    }
                    clk->end(tk, int64_t(uint64_t(nrows) * (b.n_cnt / std::max<uint64_t>(rows.size(), 1)) * 4 +
                                         nf * sizeof(FreqRec)));
                    sync();
                    ext = static_cast<const FreqRec*>(pb->host);
                    ext_n = nf;
                }
                return;
            }
            // one pass, unordered records at block cursors; rare overflow: extract again at the exact size
            uint32_t cap_recs = uint32_t(std::min<uint64_t>(std::max<uint64_t>(uint64_t(nrows) * 4, 4096), b.n_cnt));
            // the records land in mapped pinned host memory: one stream sync per batch
            DevBuf d_n;
            uint32_t* dn = d_nz;  // zeroed with the counters (a retry or the keyed count: its own)
            // the last emit's block has a zeroed counter for this count: both come back in one copy
            const bool ride = pend_check && emit_blk && !emit_copied;
            if (ride) dn = reinterpret_cast<uint32_t*>(emit_blk + 16);
            for (int attempt = 0; nrows; ++attempt) {
                PinnedBuf* pb = ctx->pinned_big(size_t(std::max<uint32_t>(cap_recs, 1)) * sizeof(FreqRec));
                if (attempt > 0 || dn == nullptr) {
                    if (d_n.p == nullptr) d_n.alloc(4);
                    dn = d_n.as<uint32_t>();
                    FSM_HIP(hipMemsetAsync(dn, 0, 4, s));
                }
                const size_t tk = clk->begin("k_freq_recs");
                hipLaunchKernelGGL(k_freq_recs, dim3(grid), dim3(kBlock), 0, s, d_rows.as<DRow>(), nrows,
                                   b.d_cls.as<DClass>(), cnt.as<uint32_t>(), minsup, rlo,
                                   static_cast<FreqRec*>(pb->dev), cap_recs, dn);
                FSM_LAUNCHED("k_freq_recs", s);
                clk->end(tk, int64_t(uint64_t(nrows) * (b.n_cnt / std::max<uint64_t>(rows.size(), 1)) * 4));
                uint32_t nf = 0;
                if (ride && attempt == 0) {
                    FSM_HIP(hipMemcpyAsync(&pend[8], emit_blk, 24, hipMemcpyDeviceToHost, s));
                    emit_copied = true;
                    sync();
                    nf = uint32_t(pend[10] & 0xFFFFFFFFu);
                } else {
                    FSM_HIP(hipMemcpyAsync(&pend[1], dn, 4, hipMemcpyDeviceToHost, s));
                    sync();
                    nf = uint32_t(pend[1] & 0xFFFFFFFFu);
                }
                if (nf <= cap_recs) {
                    // unsharded, one emit group: ordered on the device, the children deferred to emit()
                    if (nf && rlo == 0 && nrows == rows.size() && !comm && !kids_host()) {
                        uint32_t dmax = 0;
                        for (const ClassMeta& m : b.cls) dmax = std::max(dmax, m.D);
                        if (order_device(b, pb, nf, nrows, RkRows{d_rows.as<DRow>(), b.d_cls.as<DClass>(), 0u}, dmax,
                                         size_t(b.cbase_total) + 1)) {
                            recs.clear();
                            return;
                        }
                    }
                    const FreqRec* hr = static_cast<const FreqRec*>(pb->host);
                    recs.assign(hr, hr + nf);
                    break;
                }
                if (attempt > 0) throw Error(FSM_EDEVICE, "SPADE: frequent candidate buffer overflow");
                cap_recs = nf;
            }
            order_recs(recs, rhi, &rec_off_s);
            rec_off_ok = rhi == rows.size();
        }
        };
        if (shard) {  // a failure here or in run_root reaches every rank in the gather below
            run_or_defer(compute);
        } else {
            compute();
        }
        const FreqRec* R = ext ? ext : recs.data();
        uint64_t nfreq = ext ? ext_n : recs.size();
        cnt.release();
        hp[7] += now_ms() - tc1;  // device count + extraction + ordering (incl. waits)
        if (shard) {  // every rank gets every frequent pair, in row order (slices ascend with the rank)
            if (agr.code) nfreq = 0;
            std::vector<uint8_t> mine(nfreq * sizeof(FreqRec));
            if (nfreq) std::memcpy(mine.data(), R, mine.size());
            std::vector<size_t> sizes;
            // the claim counter of this mine's first-level classes is reset before this gather
            // (the collective every rank passes before its first claim); the same all-reduce
            // carries the failure agreement and, at the first sharded mine, whether every rank
            // has the shared counters
            b.claim_key = comm->next_key();
            comm->reset_counter(b.claim_key);
            uint32_t ex = comm->has_fetch_add() && claims_env() ? 1u : 0u;
            const std::vector<uint8_t> all = comm->gather_blobs(mine, sizes, s, &agr, &ex, 1);
            if (comm->claim_mode < 0) comm->claim_mode = ex == uint32_t(comm->nranks()) ? 1 : 0;
            nfreq = all.size() / sizeof(FreqRec);
            recs.resize(nfreq);
            if (nfreq) std::memcpy(recs.data(), all.data(), all.size());
            // the unordered-pair F2 gives a rank records of rows above its slice: (row, slot)
            // order and the child ids over the whole set.  Every rank orders them, whatever its
            // own F2 layout (a rank with an empty slice runs the ordered one): the ranks must
            // derive identical children, or their collective sequences part
            order_recs(recs, uint32_t(rows.size()), &rec_off_s);
            rec_off_ok = true;
            R = recs.data();
        }
        double th = now_ms();
        // kids CSR over (cbase + mi): the frequent children of every member, by slot
        // one table, one H2D copy: [koff: cbase_total + 1 | kslot: nfreq | kcid: nfreq]
        if (b.dev_order) {  // kid and child-class tables built on the device; emit() builds the children
            hp[1] += now_ms() - th;
            return;
        }
        const size_t nko = size_t(b.cbase_total) + 1;
        bool defer_checked = false;
        if (kids_dev) {
            b.kid_off = b.kid_tab.as<uint32_t>();
            b.kid_slot = b.kid_off + nko;
            b.kid_cid = b.kid_slot + nfreq;
        } else {
        // deferred children (one group, unsharded; decided here, the children are built by emit()):
        // the host child_of table (member slot -> child class) rides in the same upload
        b.child_of_pre = nullptr;
        double tl3 = now_ms();
        const bool defer = defer_ok(b, R, nfreq, rows);
        lap(12, tl3);
        defer_checked = true;
        const bool pre_co = defer && !child_of_device(b.cbase_total);
        const size_t nco = pre_co ? size_t(b.cbase_total) : 0;
        // the table is filled straight into the pinned staging slot it is DMA'd from
        const size_t kbytes = (nko + 2 * size_t(nfreq) + nco) * 4;
        uint32_t* koff = static_cast<uint32_t*>(ctx->stage_host(2, kbytes));
        uint32_t* kslot = koff + nko;
        uint32_t* kcid = kslot + nfreq;
        double tl2 = th;
        lap(9, tl2);
        // records are in (row, slot) order, and a row's member slot cbase + mi ascends
        // with the row: koff[x] = records of slots < x
        const int64_t nthk = nfreq >= par_min() ? host_threads() : 1;
        if (rec_off_ok && rec_off_s.size() == rows.size() + 1) {
            // from the row offsets of the ordering: slots (s(r-1), s(r)] take off[r]
            uint64_t x = 0;
            for (size_t r = 0; r < rows.size(); ++r) {
                const uint64_t sr = uint64_t(b.cls[rows[r].cls].cbase) + rows[r].mi;
                const uint32_t o = rec_off_s[r];
                for (; x <= sr && x < nko; ++x) koff[x] = o;
            }
            for (; x < nko; ++x) koff[x] = uint32_t(nfreq);
        } else {  // (records ordered on the device: a merge, threads split x)
            auto slot_of = [&](uint64_t q) { return uint64_t(b.cls[rows[R[q].row].cls].cbase) + rows[R[q].row].mi; };
            par_slices(nthk, int64_t(nko), [&](int64_t, int64_t x0, int64_t x1) {
                uint64_t lo = 0, hi = nfreq;  // first record with slot >= x0
                while (lo < hi) {
                    const uint64_t mid = (lo + hi) / 2;
                    if (slot_of(mid) < uint64_t(x0)) lo = mid + 1; else hi = mid;
                }
                uint64_t q = lo;
                for (int64_t x = x0; x < x1; ++x) {
                    while (q < nfreq && slot_of(q) < uint64_t(x)) ++q;
                    koff[x] = uint32_t(q);
                }
            });
        }
        par_slices(nthk, int64_t(nfreq), [&](int64_t, int64_t q0, int64_t q1) {
            for (int64_t q = q0; q < q1; ++q) {  // recs are ordered by (row, slot) = CSR order
                kslot[q] = R[q].slot;
                kcid[q] = R[q].cid;
            }
        });
        lap(10, tl2);
        if (pre_co) {  // the member slots that open a class, numbered in record order (as emit's)
            uint32_t* co = kcid + nfreq;
            std::fill(co, co + nco, kNone);
            uint32_t k = 0;
            for (uint64_t q = 0; q < nfreq;) {
                uint64_t q2 = q;
                while (q2 < nfreq && R[q2].row == R[q].row) ++q2;
                if (!(q2 - q == 1 && (R[q].slot & 1u) == kItm)) {
                    const DRow pr = rows[R[q].row];
                    co[b.cls[pr.cls].cbase + pr.mi] = k++;
                }
                q = q2;
            }
        }
        lap(13, tl2);
        b.kid_tab.alloc(std::max<size_t>(kbytes, 4));
        ctx->stage_copy(2, b.kid_tab.p, kbytes);
        lap(11, tl2);
        b.kid_off = b.kid_tab.as<uint32_t>();
        b.kid_slot = b.kid_off + nko;
        b.kid_cid = b.kid_slot + nfreq;
        if (pre_co) b.child_of_pre = b.kid_cid + nfreq;
        if (defer) {  // emit() builds the children after launching its kernels
            hp[1] += now_ms() - th;
            return;
        }
        }
        hp[1] += now_ms() - th;
        th = now_ms();
        // emit() builds the children after launching its kernels (one group, unsharded)
        if (!defer_checked && defer_ok(b, R, nfreq, rows)) {
            hp[2] += now_ms() - th;
            return;
        }
        make_children(b, R, nfreq, rows);
        if (shard) {
            // first-level classes: largest-first by estimated id-list volume (the
            // class's entries), same plan on every rank; keep this rank's share.
            // A class heavier than split_frac() of a rank's fair share is split instead:
            // every rank counts it, and its sub-classes are planned over the ranks.
            n_shared = nodes.size();
            const size_t nc = b.children.size();
            const uint64_t N = uint64_t(comm->nranks());
            uint64_t tot = 0;
            for (const ChildInfo& c : b.children) tot += c.cap;
            std::vector<uint64_t> vol;
            std::vector<size_t> idx;
            std::vector<uint8_t> heavy(nc, 0);
            for (size_t k = 0; k < nc; ++k) {
                heavy[k] = nc > 1 && double(b.children[k].cap) * double(N) > split_frac() * double(tot);
                if (!heavy[k]) {
                    vol.push_back(b.children[k].cap);
                    idx.push_back(k);
                }
            }
            size_t nheavy = 0;
            for (size_t k = 0; k < nc; ++k) {
                b.children[k].split = heavy[k] != 0;
                nheavy += heavy[k];
            }
            // Claims pay where a static plan balances badly: few first-level classes per rank
            // (deep, skewed lattices: BIBLE / SIGN shapes).  With many small classes (Quest D1M:
            // about 5,000) the largest-first plan is within a few percent, and every claim costs
            // an emit pass over all the DB rows (0.3 ms at D1M), so the static plan runs (one
            // pass per rank).  FSM_SPADE_CLAIMS=1 forces claims, =0 the static plan.
            const bool claims_pay = claims_forced() || nc < kClaimClassesPerRank * uint64_t(comm->nranks());
            if (comm->claim_mode == 1 && claims_pay) {
                // work stealing: heavy classes first (every rank), then the rest largest first;
                // the groups after the shared ones are claimed from the shared counter
                std::vector<size_t> ord(idx);
                std::stable_sort(ord.begin(), ord.end(),
                                 [&](size_t x, size_t y) { return b.children[x].cap > b.children[y].cap; });
                RawVec<ChildInfo> all;
                for (size_t k = 0; k < nc; ++k)
                    if (heavy[k]) all.push_back(std::move(b.children[k]));
                const size_t h = all.size();
                for (size_t k : ord) all.push_back(std::move(b.children[k]));
                b.children = std::move(all);
                b.nshared_children = h;
            } else {
                std::vector<int32_t> owner(vol.size());
                shard_plan(vol.data(), int64_t(vol.size()), comm->nranks(), owner.data());
                std::vector<uint8_t> keep(nc, 0);
                for (size_t q = 0; q < idx.size(); ++q) keep[idx[q]] = owner[q] == comm->rank();
                RawVec<ChildInfo> kept;
                for (size_t k = 0; k < nc; ++k)
                    if (heavy[k] || keep[k]) kept.push_back(std::move(b.children[k]));
                b.children = std::move(kept);
                b.claim_key = -1;
            }
            if (ctx->opts.verbose)
                std::fprintf(stderr, "[fsm] rank %d: %zu first-level classes, %zu %s, %zu heavy (split)\n",
                             comm->rank(), nc, b.children.size(), b.claim_key >= 0 ? "claimable" : "kept", nheavy);
        } else if (comm) {
            // sub-classes of a split class: LPT over that class's sub-classes alone
            // (the same on every rank whatever the batching), this rank keeps its share
            RawVec<ChildInfo> kept;
            for (size_t k = 0; k < b.children.size();) {
                size_t k2 = k;
                const uint32_t pc = b.children[k].pcls;
                while (k2 < b.children.size() && b.children[k2].pcls == pc) ++k2;
                if (!b.cls[pc].split) {
                    for (size_t x = k; x < k2; ++x) kept.push_back(std::move(b.children[x]));
                } else {
                    std::vector<uint64_t> vol(k2 - k);
                    std::vector<int32_t> owner(k2 - k);
                    for (size_t x = k; x < k2; ++x) vol[x - k] = b.children[x].cap;
                    shard_plan(vol.data(), int64_t(vol.size()), comm->nranks(), owner.data());
                    for (size_t x = k; x < k2; ++x)
                        if (owner[x - k] == comm->rank()) kept.push_back(std::move(b.children[x]));
                }
                k = k2;
            }
            for (ChildInfo& c : kept) c.split = false;
            b.children = std::move(kept);
        }
        hp[2] += now_ms() - th;
        th = now_ms();
        if (b.claim_key >= 0) {
            // work stealing: the shared (heavy) groups now, the claimed ones as they come
            b.groups.clear();
            b.next_group = 0;
            append_groups(b, 0, b.nshared_children);
            const size_t h = b.nshared_children, n = b.children.size() - h;
            b.claim_pre.assign(n + 1, 0);
            for (size_t k = 0; k < n; ++k) b.claim_pre[k + 1] = b.claim_pre[k] + b.children[h + k].cap;
            hp[3] += now_ms() - th;
            return;
        }
        // groups of children that fit the frontier budget
        b.groups.clear();
        b.next_group = 0;
        size_t gs = 0;
        uint64_t acc = 0;
        const uint64_t max_ent = uint64_t(1) << 31;
        uint64_t acc_ent = 0;
        const int64_t nch = int64_t(b.children.size());
        bool one = false;  // many children: the common case (all fit one group) from threaded sums
        if (nch >= (int64_t(1) << 16)) {
            const int64_t nthr = host_threads();
            std::vector<uint64_t> tn(size_t(nthr), 0), te(size_t(nthr), 0);
            par_slices(nthr, nch, [&](int64_t t, int64_t k0, int64_t k1) {
                uint64_t n = 0, e = 0;
                for (int64_t k = k0; k < k1; ++k) {
                    const ChildInfo& c = b.children[size_t(k)];
                    n += c.cap * entry_bytes() + uint64_t(c.D) * c.D * 4;
                    e += c.cap;
                }
                tn[size_t(t)] = n;
                te[size_t(t)] = e;
            });
            uint64_t n = 0, e = 0;
            for (int64_t t = 0; t < nthr; ++t) {
                n += tn[size_t(t)];
                e += te[size_t(t)];
            }
            one = n <= budget && e <= max_ent;
        }
        if (one) gs = b.children.size();
        for (size_t k = one ? b.children.size() : 0; k < b.children.size(); ++k) {
            const uint64_t need = b.children[k].cap * entry_bytes() + uint64_t(b.children[k].D) * b.children[k].D * 4;
            if (k > gs && (acc + need > budget || acc_ent + b.children[k].cap > max_ent)) {
                b.groups.push_back({gs, k});
                gs = k;
                acc = 0;
                acc_ent = 0;
            }
            acc += need;
            acc_ent += b.children[k].cap;
        }
        if (one) b.groups.push_back({0, b.children.size()});
        else if (gs < b.children.size()) b.groups.push_back({gs, b.children.size()});
        hp[3] += now_ms() - th;
        if (ctx->opts.verbose)
            std::fprintf(stderr, "[fsm] batch: classes=%zu entries=%llu freq=%llu children=%zu groups=%zu\n",
                         b.cls.size(), (unsigned long long)tot_ent, (unsigned long long)nfreq,
                         b.children.size(), b.groups.size());
    }

    // the children of a counted batch (new pattern nodes, the next batch's class records and
    // member tables) in deterministic (row, slot) order
    void make_children(Batch& b, const FreqRec* R, uint64_t nfreq, const RawVec<DRow>& rows) {
        fsm_stats& st = ctx->stats;
        b.children.clear();
        b.child_rank_item.clear();
        b.child_node_of.clear();
        b.children.reserve(nfreq);
        b.child_rank_item.reserve(nfreq + 16);
        b.child_node_of.reserve(2 * nfreq + 16);
        if (!comm && nfreq >= par_min()) {
            children_parallel(b, R, nfreq, rows);
        } else
        for (size_t q = 0; q < nfreq;) {
            const uint32_t row = R[q].row;
            const DRow pr = rows[row];
            const ClassMeta& pm = b.cls[pr.cls];
            size_t q2 = q;
            uint32_t maxcid = 0;
            while (q2 < nfreq && R[q2].row == row) { maxcid = std::max(maxcid, R[q2].cid); ++q2; }
            ChildInfo ch;
            ch.pcls = pr.cls;
            ch.pmi = pr.mi;
            const uint32_t R2 = (maxcid >> 1) + 1;
            ch.D = 2 * R2;
            ch.ri_off = b.child_rank_item.size();
            ch.no_off = b.child_node_of.size();
            b.child_rank_item.resize(ch.ri_off + R2, 0);
            b.child_node_of.resize(ch.no_off + ch.D, -1);
            const int32_t parent = b.node_of[pm.no_off + pr.mi];
            const uint32_t pls = nodes[size_t(parent)].len_sets;
            ch.psup = nodes[size_t(parent)].support;
            if ((pls >> 16) >= 0xFFFFu) throw Error(FSM_ELIMIT, "SPADE: a pattern exceeds 65534 items");
            const bool dup = comm && pm.split && comm->rank() != 0;  // a split class's nodes: rank 0 outputs them
            uint32_t last_type = 0;
            for (size_t k = q; k < q2; ++k) {
                const FreqRec& fr = R[k];
                const uint32_t item = b.rank_item[pm.ri_off + (fr.slot >> 1)];
                const int32_t node = int32_t(nodes.size());
                nodes.push_back(PNode{parent, item, fr.slot & 1u, fr.sup, pls + (1u << 16) + ((fr.slot & 1u) == kSeq)});
                if (dup) {
                    node_dup.resize(nodes.size(), 0);
                    node_dup[size_t(node)] = 1;
                }
                b.child_rank_item[ch.ri_off + (fr.cid >> 1)] = item;
                b.child_node_of[ch.no_off + fr.cid] = node;
                ch.cap += fr.sup;
                if ((fr.slot & 1u) == kSeq) { ++ch.nS; ch.sS += fr.sup; } else { ++ch.nI; ch.sI += fr.sup; }
                if (!dup) st.bytes_join_equiv += int64_t(12ull * fr.sup);
                last_type = fr.slot & 1u;
            }
            const size_t nch = q2 - q;
            if (!(nch == 1 && last_type == kItm)) b.children.push_back(std::move(ch));
            q = q2;
        }
    }

    // The one-group test of count_and_freq's group split, from the records alone (before the
    // children exist): unsharded, no claims, every kept child in one group.  Then the batch
    // records what emit() needs (the group, the child entry total) and defers the children.
    bool defer_ok(Batch& b, const FreqRec* R, uint64_t nfreq, const RawVec<DRow>& rows) {
        b.defer_children = false;
        if (comm || b.claim_key >= 0 || nfreq == 0 || defer_env() == 0) return false;
        // the rows' sums over host-thread slices of the records (a slice takes the rows that start
        // in it, whole; SIGN-shaped batches hold millions of records)
        const int64_t nthr = nfreq >= par_min() ? host_threads() : 1;
        std::vector<uint64_t> sl(size_t(nthr) * 3, 0);  // need, ent, nkept per slice
        const size_t eb = entry_bytes();
        par_slices(nthr, int64_t(nfreq), [&](int64_t t, int64_t q0, int64_t q1) {
            uint64_t q = uint64_t(q0), need = 0, ent = 0, nkept = 0;
            while (q0 > 0 && q < uint64_t(q1) && R[q].row == R[q - 1].row) ++q;  // (a row that started before)
            while (q < uint64_t(q1)) {
                const uint32_t row = R[q].row;
                uint64_t q2 = q, sup = 0;
                uint32_t maxcid = 0;
                while (q2 < nfreq && R[q2].row == row) {
                    maxcid = std::max(maxcid, R[q2].cid);
                    sup += R[q2].sup;
                    ++q2;
                }
                if (!(q2 - q == 1 && (R[q].slot & 1u) == kItm)) {
                    const uint64_t D = 2ull * ((maxcid >> 1) + 1);
                    need += sup * eb + D * D * 4;
                    ent += sup;
                    ++nkept;
                }
                q = q2;
            }
            sl[size_t(t) * 3] = need;
            sl[size_t(t) * 3 + 1] = ent;
            sl[size_t(t) * 3 + 2] = nkept;
        });
        uint64_t need = 0, ent = 0, nkept = 0;
        for (int64_t t = 0; t < nthr; ++t) {
            need += sl[size_t(t) * 3];
            ent += sl[size_t(t) * 3 + 1];
            nkept += sl[size_t(t) * 3 + 2];
        }
        if (need > budget || ent > (uint64_t(1) << 31) || nkept == 0) return false;
        b.children.clear();
        b.groups.assign(1, {size_t(0), size_t(nkept)});
        b.next_group = 0;
        b.defer_children = true;
        b.defer_R = R;
        b.defer_n = nfreq;
        b.defer_total = ent;
        b.defer_rows = &rows;
        return true;
    }
    // FSM_EMIT_DEFER=0: children built before the emit launch (A/B)
    static int defer_env() {  // (read per batch: the tests switch it within one process)
        const char* e = std::getenv("FSM_EMIT_DEFER");
        return e && e[0] == '0' ? 0 : 1;
    }

    // groups of children [a, z) that fit the frontier budget, appended to b.groups
    void append_groups(Batch& b, size_t a, size_t z) {
        const uint64_t max_ent = uint64_t(1) << 31;
        size_t gs = a;
        uint64_t acc = 0, acc_ent = 0;
        for (size_t k = a; k < z; ++k) {
            const ChildInfo& c = b.children[k];
            const uint64_t need = c.cap * entry_bytes() + uint64_t(c.D) * c.D * 4;
            if (k > gs && (acc + need > budget || acc_ent + c.cap > max_ent)) {
                b.groups.push_back({gs, k});
                gs = k;
                acc = acc_ent = 0;
            }
            acc += need;
            acc_ent += c.cap;
        }
        if (gs < z) b.groups.push_back({gs, z});
    }
    // FSM_SPADE_CLAIMS=0: the sharded lattice splits the first-level classes by the static
    // plan even when the shared counters exist (tests, A/B)
    static bool claims_env() {
        const char* v = std::getenv("FSM_SPADE_CLAIMS");
        return !(v && v[0] == '0');
    }
    static bool claims_forced() {
        const char* v = std::getenv("FSM_SPADE_CLAIMS");
        return v && v[0] == '1';
    }
    // below this many first-level classes per rank the sharded lattice claims its classes
    static constexpr uint64_t kClaimClassesPerRank = 64;
    // a rank's first claim takes this fraction of its fair share of the claimable volume
    // (FSM_CLAIM_FIRST); later claims half of the remaining volume's fair share, at least
    // 1/8 of the fair share (guided self-scheduling: few claims, each an emit pass over the DB).
    // A value >= the rank count makes a first claim take every class (the regression test of
    // a first claim that covers the whole class list)
    static double claim_first() {
        const char* v = std::getenv("FSM_CLAIM_FIRST");
        return v ? std::clamp(std::atof(v), 0.01, 64.0) : 0.7;
    }
    // Claim the next range of first-level classes from the shared counter and append its
    // groups; false when every class is claimed.  Two atomics: a read of the counter to
    // size the claim by the remaining volume, then the add that takes it.
    bool claim_more(Batch& b) {
        if (b.claim_key < 0 || b.claims_done) return false;
        const size_t h = b.nshared_children, n = b.children.size() - h;
        const int64_t pos0 = comm->fetch_add(b.claim_key, 0);
        if (pos0 < 0) throw Error(FSM_ECOMM, "SPADE: work-stealing counter failed");
        if (uint64_t(pos0) >= n) {
            b.claims_done = true;
            return false;
        }
        const uint64_t N = uint64_t(comm->nranks()), tot = b.claim_pre[n], rem = tot - b.claim_pre[size_t(pos0)];
        uint64_t target = b.claims_made == 0 ? uint64_t(claim_first() * double(tot) / double(N))
                                              : std::max(rem / (2 * N), tot / (8 * N));
        target = std::max<uint64_t>(target, 1);
        // the fewest classes from pos0 whose volume reaches the target
        const uint64_t want = b.claim_pre[size_t(pos0)] + target;
        size_t m = size_t(std::lower_bound(b.claim_pre.begin() + pos0 + 1, b.claim_pre.end(), want) -
                          b.claim_pre.begin()) - size_t(pos0);
        m = std::clamp<size_t>(m, 1, n - size_t(pos0));
        const int64_t old = comm->fetch_add(b.claim_key, int64_t(m));
        if (old < 0) throw Error(FSM_ECOMM, "SPADE: work-stealing counter failed");
        if (uint64_t(old) >= n) {
            b.claims_done = true;
            return false;
        }
        append_groups(b, h + size_t(old), h + std::min<size_t>(size_t(old) + m, n));
        ++b.claims_made;
        ctx->stats.rank_claims += 1;
        return true;
    }

    // emit child rows of group g of batch b into a new batch (k_emit1: one
    // pass, LDS join records, slab cursor)
    void emit(Batch& b, size_t g, Batch& nb) {
        const double th = now_ms();
        const auto [ga, gb] = b.groups[g];
        // unsharded, large batches: the child class of each member slot comes from the kids
        // CSR on the device (k_child_of); sharded runs keep only their share of the
        // children, so the host builds the table
        const bool dev_child_of = comm == nullptr && !b.dev_order && child_of_device(b.cbase_total);
        RawVec<uint32_t>& child_of = child_of_s;
        if (!dev_child_of && !(b.defer_children && b.child_of_pre)) child_of.assign(b.cbase_total, kNone);
        uint64_t total = 0;
        const bool deferred = b.defer_children;  // (one group; the children are built after the launch)
        if (deferred) {
            total = b.defer_total;
            if (!dev_child_of && !b.child_of_pre) {  // the member slots that open a class, numbered in record order
                const FreqRec* R = b.defer_R;
                const RawVec<DRow>& rows = *b.defer_rows;
                uint32_t k = 0;
                for (uint64_t q = 0; q < b.defer_n;) {
                    uint64_t q2 = q;
                    while (q2 < b.defer_n && R[q2].row == R[q].row) ++q2;
                    if (!(q2 - q == 1 && (R[q].slot & 1u) == kItm)) {
                        const DRow pr = rows[R[q].row];
                        child_of[b.cls[pr.cls].cbase + pr.mi] = k++;
                    }
                    q = q2;
                }
            }
        }
        if (b.root && !deferred)  // the root entries this rank joins as the owner: its first-level classes' prefix supports
            for (size_t k = ga; k < gb; ++k) ctx->stats.rank_root_owned += int64_t(b.children[k].psup);
        // the only group: the children and their member tables move over whole (swapped:
        // the parent, released after this emit and recycled, keeps nb's old capacity)
        // (not a claiming root: it stays on the stack for its next claim, which reads its children;
        // a first claim covering every class would otherwise leave it with nb's old ones)
        const bool whole = !deferred && ga == 0 && gb == b.children.size() && b.groups.size() == 1 && b.claim_key < 0;
        if (deferred) {
        } else if (whole) {
            nb.cls.clear();
            nb.rank_item.clear();
            nb.node_of.clear();
            std::swap(nb.cls, b.children);
            std::swap(nb.rank_item, b.child_rank_item);
            std::swap(nb.node_of, b.child_node_of);
            const int64_t n = int64_t(nb.cls.size());
            const ClassMeta* pc = b.cls.data();
            ClassMeta* cc = nb.cls.data();
            uint32_t* co = child_of.data();
            std::vector<uint64_t> tt(16, 0);
            const int64_t nthr = n >= (int64_t(1) << 16) ? host_threads() : 1;
            par_slices(nthr, n, [&](int64_t t, int64_t k0, int64_t k1) {
                uint64_t acc = 0;
                for (int64_t k = k0; k < k1; ++k) {
                    if (!dev_child_of) co[pc[cc[k].pcls].cbase + cc[k].pmi] = uint32_t(k);
                    acc += cc[k].cap;
                }
                tt[size_t(t)] = acc;
            });
            for (uint64_t v : tt) total += v;
        } else {
            nb.cls.resize(gb - ga);
            for (size_t k = ga; k < gb; ++k) {
                const ChildInfo& ch = b.children[k];
                ClassMeta& m = nb.cls[k - ga];
                m = ch;
                m.ri_off = nb.rank_item.size();
                m.no_off = nb.node_of.size();
                nb.rank_item.insert(nb.rank_item.end(), b.child_rank_item.begin() + int64_t(ch.ri_off),
                                    b.child_rank_item.begin() + int64_t(ch.ri_off + ch.D / 2));
                nb.node_of.insert(nb.node_of.end(), b.child_node_of.begin() + int64_t(ch.no_off),
                                  b.child_node_of.begin() + int64_t(ch.no_off + ch.D));
                if (!dev_child_of) child_of[b.cls[ch.pcls].cbase + ch.pmi] = uint32_t(k - ga);
                total += ch.cap;
            }
        }
        if (total >= kNone) throw Error(FSM_ELIMIT, "SPADE: class batch exceeds 2^32 entries");
        const double th2 = now_ms();
        hp[4] += th2 - th;
        nb.slab.alloc(total, W);
        hp[5] += now_ms() - th2;
        nb.E = total;
        DevBuf d_child_of, d_long;  // (freed into the stream-ordered pool: later launches on this stream reuse them)
        if (dev_child_of) {
            const uint32_t n = uint32_t(b.cbase_total);
            d_child_of.alloc(std::max<size_t>(n, 1) * 4);
            if (n) {
                if (b.child_pre.p == nullptr) {  // the slot numbering, once per batch (every group reuses it)
                    DevBuf flag(size_t(n) * 4);
                    b.child_pre.alloc((size_t(n) + 1) * 8);
                    const unsigned gr = unsigned(std::min<uint64_t>((n + kBlock - 1) / kBlock, 8192));
                    hipLaunchKernelGGL(k_child_flag, dim3(gr), dim3(kBlock), 0, s, b.kid_off, b.kid_slot, n,
                                       flag.as<uint32_t>());
                    FSM_LAUNCHED("k_child_flag", s);
                    scan_exclusive(flag.as<uint32_t>(), b.child_pre.as<uint64_t>(), n, s);
                }
                const unsigned gr = unsigned(std::min<uint64_t>((n + kBlock - 1) / kBlock, 8192));
                hipLaunchKernelGGL(k_child_of, dim3(gr), dim3(kBlock), 0, s, b.kid_off, b.kid_slot,
                                   b.child_pre.as<uint64_t>(), n, uint32_t(ga), uint32_t(gb), d_child_of.as<uint32_t>());
                FSM_LAUNCHED("k_child_of", s);
            }
        } else if (!(deferred && b.child_of_pre)) {
            upload_staged(3, d_child_of, child_of.data(), child_of.size() * 4);
        }
        // (deferred with the host table: it came up with the kid table)
        const uint32_t* cof = deferred && b.child_of_pre ? b.child_of_pre : d_child_of.as<uint32_t>();
        ctx->stats.bytes_streamed += int64_t((total + b.E) * entry_bytes());
        if (b.E) {
            // the DB-direct root is read from the DB rows themselves (pos: the DB's row
            // positions, members through rk2, lohi from the masks)
            const bool rootdb = b.db_direct;
            const uint64_t Eg = rootdb ? uint64_t(db->E) : b.E;  // entries the kernels walk
            SlabPtrs sp = b.slab.ptrs();
            RootRef rr{nullptr, nullptr};
            if (rootdb) {
                sp = SlabPtrs{nullptr, b.mem_db.as<uint32_t>(), nullptr, db->pos.as<uint32_t>(), db->mask.as<uint64_t>(),
                              nullptr};
                rr = RootRef{db->item.as<uint32_t>(), b.rk2.as<uint32_t>()};
            }
            SlabPtrs op = nb.slab.ptrs();
            // u64 slab cursor | u32 long-run count (k_emit2) | u32 run-length flag
            // (32 bytes: the next count's record counter rides along, read back with it)
            char* cursor = static_cast<char*>(zslot(32));
            if (!cursor) {
                emit_own.alloc(32);
                FSM_HIP(hipMemsetAsync(emit_own.p, 0, 32, s));
                cursor = emit_own.as<char>();
            }
            op.lim = reinterpret_cast<uint32_t*>(cursor + 12);
            const uint64_t chunk = uint64_t(kEmitBlock) * kEmitRounds;
            const unsigned grid = unsigned(std::min<uint64_t>((Eg + chunk - 1) / chunk, emit_grid_cap()));
            const size_t tk = clk->begin("k_emit");
            if ((W == 1 || W == 2 || W == 4 || W == 8) && emit_window()) {
                // windows of whole runs in registers; the runs of more than 64 entries go to
                // k_emit1's run list (device-side count: no host round trip)
                // (grid: the entries over one block's wave ranges, per kernel kind, capped)
                d_long.alloc(std::max<uint64_t>(Eg / 65 + 1, 1) * 4);
#define FSM_EMIT2(WW, RT)                                                                                       \
    hipLaunchKernelGGL((k_emit2<WW, RT>), dim3(unsigned(std::min<uint64_t>(                                         \
                           (Eg + uint64_t(e2_block<RT, WW>() / 64) * e2_range<RT, WW>() - 1) /                     \
                           (uint64_t(e2_block<RT, WW>() / 64) * e2_range<RT, WW>()), emit_grid_cap()))),           \
                       dim3(e2_block<RT, WW>()), 0, s, uint32_t(Eg), rr, sp.cid,                                     \
                       b.d_cls.as<DClass>(), sp.mem, sp.lohi, sp.pos, sp.mask, b.kid_off, b.kid_slot, b.kid_cid,   \
                       cof, reinterpret_cast<unsigned long long*>(cursor), op, nb.slab.cap, emit2_cap(),   \
                       d_long.as<uint32_t>(), reinterpret_cast<uint32_t*>(cursor + 8));               \
    FSM_LAUNCHED("k_emit2", s);                                                                                    \
    hipLaunchKernelGGL((k_emit1<WW, RT>), dim3(256), dim3(kEmitBlock), 0, s, uint32_t(Eg), rr, sp.cid,              \
                       b.d_cls.as<DClass>(), sp.mem, sp.lohi, sp.pos, sp.mask, b.kid_off, b.kid_slot, b.kid_cid,   \
                       cof, reinterpret_cast<unsigned long long*>(cursor), op, nb.slab.cap, emit_cap(),    \
                       uint32_t(WW), d_long.as<uint32_t>(), reinterpret_cast<const uint32_t*>(cursor + 8)); \
    FSM_LAUNCHED("k_emit1", s);
                switch (W * 2 + (rootdb ? 1 : 0)) {
                    case 2: FSM_EMIT2(1, false) break;
                    case 3: FSM_EMIT2(1, true) break;
                    case 4: FSM_EMIT2(2, false) break;
                    case 5: FSM_EMIT2(2, true) break;
                    case 8: FSM_EMIT2(4, false) break;
                    case 9: FSM_EMIT2(4, true) break;
                    case 16: FSM_EMIT2(8, false) break;
                    default: FSM_EMIT2(8, true) break;
                }
#undef FSM_EMIT2
            } else {
#define FSM_EMIT1(WW)                                                                                               \
    hipLaunchKernelGGL((k_emit1<WW, false>), dim3(grid), dim3(kEmitBlock), 0, s, uint32_t(Eg), rr, sp.cid,                \
                       b.d_cls.as<DClass>(), sp.mem, sp.lohi, sp.pos, sp.mask, b.kid_off, b.kid_slot,                   \
                       b.kid_cid, cof, reinterpret_cast<unsigned long long*>(cursor), op,  \
                       nb.slab.cap, emit_cap(), uint32_t(W), (const uint32_t*)nullptr, (const uint32_t*)nullptr)
#define FSM_EMIT1R(WW)                                                                                              \
    hipLaunchKernelGGL((k_emit1<WW, true>), dim3(grid), dim3(kEmitBlock), 0, s, uint32_t(Eg), rr, sp.cid,                 \
                       b.d_cls.as<DClass>(), sp.mem, sp.lohi, sp.pos, sp.mask, b.kid_off, b.kid_slot,                   \
                       b.kid_cid, cof, reinterpret_cast<unsigned long long*>(cursor), op,  \
                       nb.slab.cap, emit_cap(), uint32_t(W), (const uint32_t*)nullptr, (const uint32_t*)nullptr)
                if (rootdb) {
                    switch (W) {
                        case 1: FSM_EMIT1R(1); break;
                        case 2: FSM_EMIT1R(2); break;
                        case 4: FSM_EMIT1R(4); break;
                        default: FSM_EMIT1R(8); break;
                    }
                } else {
                    FSM_W_DISPATCH(W, FSM_EMIT1)
                }
#undef FSM_EMIT1
#undef FSM_EMIT1R
                FSM_LAUNCHED("k_emit", s);
            }
            // reads every parent entry once (DB-direct root: the DB entry's item, pos and mask),
            // writes every child entry once
            const uint64_t rd = rootdb ? Eg * (8 + 8 * uint64_t(W)) : b.E * entry_bytes();
            clk->end(tk, int64_t(rd + total * entry_bytes()), int64_t((b.E + total) * survey_entry_bytes()));
            // the cursor block is read back with the next count's record count (or at the next
            // sync): pend[8] = entries written, pend[9] = long runs | run-length flag << 32
            emit_blk = cursor;
            emit_copied = false;
        } else {
            emit_blk = nullptr;
            pend[8] = 0;
            pend[9] = 0;
        }
        // no sync: the host prepares the next count while the emit runs; the runs must add
        // up exactly to the capacities (sum of child supports), checked at the next sync
        pend_total = total;
        pend_check = true;
        if (deferred) {
            // the children, while the emit runs: pattern nodes and the next batch's class tables,
            // moved over whole (the only group)
            const double td = now_ms();
            b.defer_children = false;
            if (b.dev_order) FSM_HIP(hipEventSynchronize(b.rec_ev));  // the ordered records (pinned)
            make_children(b, b.defer_R, b.defer_n, *b.defer_rows);
            if (b.dev_order) {
                // the exact child entries (the slab was sized by every record's support)
                uint64_t exact = 0;
                for (const ChildInfo& c : b.children) exact += c.cap;
                if (exact > nb.slab.cap)
                    throw Error(FSM_EDEVICE, "SPADE internal error: root children exceed their slab");
                nb.E = exact;
                pend_total = exact;
                b.groups[0].second = b.children.size();
            } else if (b.children.size() != gb) {
                throw Error(FSM_EDEVICE, "SPADE internal error: deferred children do not match the emit group");
            }
            if (b.root)
                for (const ChildInfo& c : b.children) ctx->stats.rank_root_owned += int64_t(c.psup);
            nb.cls.clear();
            nb.rank_item.clear();
            nb.node_of.clear();
            std::swap(nb.cls, b.children);
            std::swap(nb.rank_item, b.child_rank_item);
            std::swap(nb.node_of, b.child_node_of);
            hp[2] += now_ms() - td;
        }
    }
    // the deferred emit check (after a stream sync)
    void check_emit() {
        if (!pend_check) return;
        pend_check = false;
        const uint64_t written = pend[8];
        if (pend[9] >> 32)
            throw Error(FSM_ELIMIT, "SPADE: a class holds more than 65535 entries of one sequence");
        if (written != pend_total)
            throw Error(FSM_EDEVICE, "SPADE emit: wrote " + std::to_string(written) + " child entries, expected " +
                                         std::to_string(pend_total));
    }

    // FSM_ROOT_DB=0 keeps the root slab (k_root_count + k_root_write) for every mine (tests, A/B)
    static bool root_db_env() {
        const char* v = std::getenv("FSM_ROOT_DB");
        return !(v && v[0] == '0');
    }
    // the DB's row positions for the DB-direct root (once per DB); false = a row is too long
    bool ensure_db_pos() {
        if (db->pos_state == 0) {
            const uint32_t R = uint32_t(db->R);
            db->pos.alloc(std::max<int64_t>(db->E, 1) * 4);
            DevBuf flag(4);
            FSM_HIP(hipMemsetAsync(flag.p, 0, 4, s));
            if (R)
                hipLaunchKernelGGL(k_db_pos, dim3(unsigned((uint64_t(R) * 64 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                                   db->row_off.as<uint32_t>(), R, db->pos.as<uint32_t>(), flag.as<uint32_t>());
            FSM_LAUNCHED("k_db_pos", s);
            pend[6] = 0;
            FSM_HIP(hipMemcpyAsync(&pend[6], flag.p, 4, hipMemcpyDeviceToHost, s));
            sync();
            db->pos_state = (pend[6] & 0xFFFFFFFFu) ? -1 : 1;
            if (db->pos_state < 0) db->pos.release();
        }
        return db->pos_state > 0;
    }

    // The DB-direct root: no root slab.  The F2 plan (key capacities per rank group and row
    // block, and the root entry count) is made from the DB rows; the F2 keys and the root
    // emit read the same rows.  Returns false (nothing launched that matters) when the
    // geometry does not apply: the caller then builds the root slab.
    bool run_root_db(Batch& root, const std::vector<uint32_t>& freq_items, const std::vector<uint32_t>& f1,
                     const std::vector<uint32_t>& rank) {
        if (!(W == 1 || W == 2 || W == 4 || W == 8) || !root_db_env() || root_atomic() || db->R == 0) return false;
        const uint32_t F = uint32_t(freq_items.size());
        root.root = true;
        const F2Geo geo = f2_geometry(root, 2 * F, uint64_t(db->E), uint64_t(db->R));
        if (!geo.ok || !ensure_db_pos()) {
            root.root = false;
            return false;
        }
        // rk2: 2 rank for a frequent item; 2 (frequent items below it) - 1 for an infrequent one
        std::vector<uint32_t> rk2(size_t(db->U));
        uint32_t below = 0;
        for (size_t u = 0; u < rk2.size(); ++u) {
            if (rank[u] != kNone) {
                rk2[u] = 2 * rank[u];
                ++below;
            } else {
                rk2[u] = 2 * below - 1u;  // wraps to 0xFFFFFFFF below the first frequent item
            }
        }
        upload_staged(0, root.rk2, rk2.data(), rk2.size() * 4);  // (pinned: the copy does not block the host)
        // the unordered-pair layout (W = 1): its own groups over this rank's rows
        uint32_t G = geo.G;
        uint64_t nd = geo.nd;
        root.f2_tri = false;
        if (W == 1 && f2_tri_env()) {
            std::vector<uint32_t> tab;
            const uint32_t rlo = geo.mlo / 2, rhi = geo.mhi == kNone ? F : std::min(geo.mhi / 2, F);
            const uint32_t TG = tri_tables(F, rlo, rhi, tab);
            if (TG) {
                upload_staged(1, root.f2_tri_tab, tab.data(), tab.size() * 4);
                root.f2_tri = true;
                root.f2_tri_G = TG;
                G = TG;
                nd = uint64_t(TG) * geo.nblk;
            }
        }
        root.mem_db.alloc(std::max<int64_t>(db->E, 1) * 4);
        DevBuf cap(nd * 4);
        root.f2_base.alloc((nd + 1) * 8);
        const size_t tk = clk->begin("k_f2_plan");
        hipLaunchKernelGGL(k_f2_plan_db, dim3(geo.nblk), dim3(kF2Threads), size_t(G) * 4, s,
                           db->row_off.as<uint32_t>(), db->item.as<uint32_t>(), root.rk2.as<uint32_t>(), geo.R,
                           geo.rpb, geo.pm, G, geo.nblk, geo.mlo, geo.mhi, cap.as<uint32_t>(), kF2Align - 1,
                           root.mem_db.as<uint32_t>(), root.f2_tri ? root.f2_tri_tab.as<uint32_t>() : nullptr);
        FSM_LAUNCHED("k_f2_plan", s);
        clk->end(tk, int64_t(db->R) * 4 + db->E * 8 + int64_t(nd) * 4);
        scan_exclusive(cap.as<uint32_t>(), root.f2_base.as<uint64_t>(), nd, s);
        pend[2] = 0;
        FSM_HIP(hipMemcpyAsync(&pend[2], root.f2_base.as<uint64_t>() + nd, 8, hipMemcpyDeviceToHost, s));
        root_meta(root, freq_items, f1);
        // the root entries: one per (sequence, frequent item), so the frequent items' supports add up to them
        uint64_t E0 = 0;
        for (uint32_t it : freq_items) E0 += f1[it];
        sync();
        if (E0 >= kNone) throw Error(FSM_ELIMIT, "SPADE: more than 2^32 root entries");
        if (pend[2] >= (uint64_t(1) << 32) - 4096) {  // region cursors are u32: the slab path counts it
            root.recycle();
            nodes.n = 0;
            return false;
        }
        root.E = E0;
        root.R = uint64_t(db->R);
        root.cls[0].cap = E0;
        ctx->stats.root_entries = int64_t(E0);
        root.f2_planned = true;
        root.f2_nslots = pend[2];
        root.db_direct = true;
        // the pair keys start now: the host's root bookkeeping (class record, member rows,
        // descriptors) overlaps them (count_and_freq -> root_f2_tri takes the count from here)
        if (root.f2_tri && !comm) (void)launch_f2_tri(root, f2_geometry(root, 2 * F, E0, uint64_t(db->R)));
        return true;
    }

    // the root class record (one class: every frequent item a sequence-extension member)
    // and the 1-pattern nodes
    void root_meta(Batch& root, const std::vector<uint32_t>& freq_items, const std::vector<uint32_t>& f1) {
        const uint32_t F = uint32_t(freq_items.size());
        ClassMeta m;
        m.D = 2 * F;
        m.mshift = 1;  // root members are all sequence-extensions: counter rows by rank
        m.ri_off = 0;
        m.no_off = 0;
        root.rank_item.assign(freq_items.begin(), freq_items.end());
        root.node_of.assign(m.D, -1);
        for (uint32_t r = 0; r < F; ++r) {
            root.node_of[2 * r] = int32_t(nodes.size());
            nodes.push_back(PNode{-1, freq_items[r], kSeq, f1[freq_items[r]], (1u << 16) | 1u});
        }
        m.cap = 0;  // set from the read-back count
        m.nS = F;
        for (uint32_t r = 0; r < F; ++r) m.sS += f1[freq_items[r]];
        root.cls.push_back(std::move(m));
        root.root = true;
    }

    void run_root(Batch& root, const std::vector<uint32_t>& freq_items, const std::vector<uint32_t>& f1) {
        const int64_t R = db->R;
        const uint64_t r0 = 0, r1 = uint64_t(R);
        // rank map (dense item -> frequent rank)
        std::vector<uint32_t> rank(size_t(db->U), kNone);
        for (size_t r = 0; r < freq_items.size(); ++r) rank[freq_items[r]] = uint32_t(r);
        if (run_root_db(root, freq_items, f1, rank)) return;
        ctx->stats.rank_root_slab = R ? db->E : 0;  // (an upper bound: the root entries are read back below)
        DevBuf d_rank, rcnt((r1 - r0 + 1) * 4), roff((r1 - r0 + 1) * 8), flag(4);
        upload(d_rank, rank);
        FSM_HIP(hipMemsetAsync(flag.p, 0, 4, s));
        if (r1 > r0) {
            const size_t tk = clk->begin("k_root_count");
            hipLaunchKernelGGL(k_root_count, dim3(unsigned((r1 - r0 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                               db->row_off.as<uint32_t>(), db->item.as<uint32_t>(), d_rank.as<uint32_t>(), r0, r1,
                               rcnt.as<uint32_t>(), flag.as<uint32_t>());
            FSM_LAUNCHED("k_root_count", s);
            clk->end(tk, int64_t((r1 - r0) * 12 + uint64_t(db->E) * 8));
        }
        scan_exclusive(rcnt.as<uint32_t>(), roff.as<uint64_t>(), r1 - r0, s);
        // the root entry count and the row-length flag are read back with the F2 plan's
        // slot total at the one sync below: the root slab is sized by the DB's entries
        pend[4] = 0;
        pend[5] = 0;
        FSM_HIP(hipMemcpyAsync(&pend[4], roff.as<uint64_t>() + (r1 - r0), 8, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipMemcpyAsync(&pend[5], flag.p, 4, hipMemcpyDeviceToHost, s));
        const uint64_t Ecap = uint64_t(std::max<int64_t>(db->E, 1));
        root.slab.alloc(Ecap, W);
        FSM_HIP(hipMemsetAsync(root.slab.cid.p, 0, Ecap * 4, s));
        // the root batch's F2 geometry (its slab is this root slab): plan fused into the write
        const uint32_t F = uint32_t(freq_items.size());
        size_t tk_rw = size_t(-1);
        root.root = true;
        const F2Geo geo = f2_geometry(root, 2 * F, Ecap, r1 - r0);
        if (r1 > r0 && geo.ok) {
            const SlabPtrs op = root.slab.ptrs();
            DevBuf cap(geo.nd * 4);
            root.f2_base.alloc((geo.nd + 1) * 8);
            const size_t tk = clk->begin("k_root_write");
#define FSM_ROOTWP(WW)                                                                                            \
    hipLaunchKernelGGL(k_root_write_plan<WW>, dim3(geo.nblk), dim3(kF2Threads), size_t(geo.G) * 4, s,              \
                       db->row_off.as<uint32_t>(), db->item.as<uint32_t>(), db->mask.as<uint64_t>(),               \
                       d_rank.as<uint32_t>(), geo.R, geo.rpb, roff.as<uint64_t>(), op, geo.pm, geo.G, geo.nblk,    \
                       geo.mlo, geo.mhi, cap.as<uint32_t>(), kF2Align - 1, uint32_t(W))
            FSM_W_DISPATCH(W, FSM_ROOTWP)
#undef FSM_ROOTWP
            FSM_LAUNCHED("k_root_write", s);
            clk->end(tk, int64_t(uint64_t(db->E) * (8 + 8 * uint64_t(W)) + geo.nd * 4));
            tk_rw = tk;
            scan_exclusive(cap.as<uint32_t>(), root.f2_base.as<uint64_t>(), geo.nd, s);
            FSM_HIP(hipMemcpyAsync(&pend[2], root.f2_base.as<uint64_t>() + geo.nd, 8, hipMemcpyDeviceToHost, s));
            root.f2_planned = true;
        } else if (r1 > r0) {
            const SlabPtrs op = root.slab.ptrs();
            const unsigned grid = unsigned(((r1 - r0) * 64 + kBlock - 1) / kBlock);
            const size_t tk = clk->begin("k_root_write");
#define FSM_ROOTW(WW)                                                                                         \
    hipLaunchKernelGGL(k_root_write<WW>, dim3(grid), dim3(kBlock), 0, s, db->row_off.as<uint32_t>(),           \
                       db->item.as<uint32_t>(), db->mask.as<uint64_t>(), d_rank.as<uint32_t>(), r0, r1,       \
                       roff.as<uint64_t>(), op, uint32_t(W))
            FSM_W_DISPATCH(W, FSM_ROOTW)
#undef FSM_ROOTW
            FSM_LAUNCHED("k_root_write", s);
            clk->end(tk, int64_t(uint64_t(db->E) * (8 + 8 * uint64_t(W))));
            tk_rw = tk;
        }
        root_meta(root, freq_items, f1);
        root.root_rows = std::move(roff);
        root.R = r1 - r0;
        sync();
        const uint64_t E0 = pend[4];
        if (pend[5] & 0xFFFFFFFFu) throw Error(FSM_ELIMIT, "SPADE: a sequence has more than 65535 distinct frequent items");
        if (E0 >= kNone) throw Error(FSM_ELIMIT, "SPADE: more than 2^32 root entries");
        root.E = E0;
        root.cls[0].cap = E0;
        ctx->stats.root_entries = int64_t(E0);
        ctx->stats.rank_root_slab = int64_t(E0);
        if (tk_rw != size_t(-1)) clk->add_bytes(tk_rw, int64_t(E0 * (16 + 8 * uint64_t(W))));
        if (root.f2_planned) root.f2_nslots = pend[2];
    }

};

// malloc'd array without value-initialisation, released to the caller (freed by fsm_patterns_free)
template <class T> struct MallocArr {
    T* p = nullptr;
    size_t n = 0;
    MallocArr() = default;
    explicit MallocArr(size_t n_) { alloc(n_); }
    void alloc(size_t n_) {
        big_give(p);
        p = nullptr;
        n = n_;
        // large result arrays: big host blocks (2 MiB aligned, transparent huge pages, the
        // largest reused from earlier mines: a dense mine's CSR is hundreds of MB of pages);
        // fsm_patterns_free / fsm_rules_free hand them back through big_give
        const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        if (bytes >= 4 * kHugeBlock) p = static_cast<T*>(big_take((bytes + kHugeBlock - 1) & ~(kHugeBlock - 1)));
        else p = static_cast<T*>(std::malloc(bytes));
        if (!p) throw Error(FSM_ENOMEM, "malloc failed");
    }
    MallocArr(const MallocArr&) = delete;
    MallocArr& operator=(const MallocArr&) = delete;
    ~MallocArr() { big_give(p); }
    T& operator[](size_t i) { return p[i]; }
    T* release() {
        T* r = p;
        p = nullptr;
        return r;
    }
};

template <class T> void copy_out(T*& dst, const std::vector<T>& src) {
    dst = static_cast<T*>(std::malloc(std::max<size_t>(src.size(), 1) * sizeof(T)));
    if (!dst) throw Error(FSM_ENOMEM, "malloc failed");
    if (!src.empty()) std::memcpy(dst, src.data(), src.size() * sizeof(T));
}

// the work counters of a sharded mine that are summed over the ranks (joins etc. are
// counted where the work ran)
constexpr size_t kSumStats = 11;
void sum_stats_fields(fsm_stats& st, int64_t* f[kSumStats]) {
    int64_t* g[kSumStats] = {&st.joins, &st.classes, &st.batches, &st.entries, &st.bytes_join_equiv,
                             &st.bytes_streamed, &st.bytes_count_alg, &st.count_launches, &st.joins_root,
                             &st.root_keys, &st.pair_tests};
    for (size_t k = 0; k < kSumStats; ++k) f[k] = g[k];
}

// every rank's pattern CSR, concatenated in rank order, on every rank, with the summed work
// counters; one gather, which also carries the failure agreement of the mine (agr)
// root_only (ranks of one in-process group): only rank 0's result is returned, the others
// get an empty CSR and copy nothing
void gather_patterns(Comm* comm, hipStream_t s, std::vector<int32_t>& sup, std::vector<int64_t>& pat_off,
                     std::vector<int64_t>& set_off, std::vector<int32_t>& items, fsm_stats& st, Agreement* agr,
                     bool root_only) {
    // blob (int32): stats (2 x kSumStats), n, n_sets, n_items, sup[n], sets-per-pattern[n],
    // set sizes[n_sets], items[n_items]
    const size_t n = sup.size(), ns = set_off.size() - 1, ni = items.size();
    if (n > size_t(INT32_MAX) || ns > size_t(INT32_MAX) || ni > size_t(INT32_MAX))
        throw Error(FSM_ELIMIT, "SPADE: pattern output of one rank exceeds 2^31 entries");
    int64_t* f[kSumStats];
    sum_stats_fields(st, f);
    std::vector<int32_t> b;
    b.reserve(2 * kSumStats + 3 + 2 * n + ns + ni);
    for (size_t k = 0; k < kSumStats; ++k) {
        int32_t w[2];
        std::memcpy(w, f[k], 8);
        b.push_back(w[0]);
        b.push_back(w[1]);
    }
    b.push_back(int32_t(n));
    b.push_back(int32_t(ns));
    b.push_back(int32_t(ni));
    b.insert(b.end(), sup.begin(), sup.end());
    for (size_t k = 0; k < n; ++k) b.push_back(int32_t(pat_off[k + 1] - pat_off[k]));
    for (size_t k = 0; k < ns; ++k) b.push_back(int32_t(set_off[k + 1] - set_off[k]));
    b.insert(b.end(), items.begin(), items.end());
    std::vector<uint8_t> mine(b.size() * 4);
    std::memcpy(mine.data(), b.data(), mine.size());
    std::vector<size_t> sizes;
    const std::vector<uint8_t> all = comm->gather_blobs(mine, sizes, s, agr, nullptr, 0, root_only);
    sup.clear();
    items.clear();
    pat_off.assign(1, 0);
    set_off.assign(1, 0);
    if (root_only && comm->rank() != 0) return;
    for (size_t k = 0; k < kSumStats; ++k) *f[k] = 0;
    size_t at = 0;
    for (size_t r = 0; r < sizes.size(); ++r) {
        std::vector<int32_t> v(sizes[r] / 4);
        if (!v.empty()) std::memcpy(v.data(), all.data() + at, sizes[r]);
        at += sizes[r];
        for (size_t k = 0; k < kSumStats; ++k) {
            int64_t x;
            std::memcpy(&x, v.data() + 2 * k, 8);
            *f[k] += x;
        }
        const int32_t* q = v.data() + 2 * kSumStats;
        const size_t rn = size_t(q[0]), rs = size_t(q[1]), ri = size_t(q[2]);
        const int32_t* p = q + 3;
        sup.insert(sup.end(), p, p + rn);
        for (size_t k = 0; k < rn; ++k) pat_off.push_back(pat_off.back() + p[rn + k]);
        for (size_t k = 0; k < rs; ++k) set_off.push_back(set_off.back() + p[2 * rn + k]);
        items.insert(items.end(), p + 2 * rn + rs, p + 2 * rn + rs + ri);
    }
}


}  // namespace

void spade_upload(fsm_ctx* ctx, fsm_db* db) {
    const FlatSpade& f = db->spade;
    auto* d = new SpadeDevDB();
    try {
        d->R = int64_t(f.row_off.size()) - 1;
        d->E = int64_t(f.ent_item.size());
        d->U = int64_t(f.item_val.size());
        d->W = f.W;
        d->row_off.alloc(f.row_off.size() * 4);
        d->item.alloc(std::max<size_t>(f.ent_item.size(), 1) * 4);
        d->mask.alloc(std::max<size_t>(f.ent_mask.size(), 1) * 8);
        FSM_HIP(hipMemcpyAsync(d->row_off.p, f.row_off.data(), f.row_off.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        if (d->E) {
            FSM_HIP(hipMemcpyAsync(d->item.p, f.ent_item.data(), f.ent_item.size() * 4, hipMemcpyHostToDevice, ctx->stream));
            FSM_HIP(hipMemcpyAsync(d->mask.p, f.ent_mask.data(), f.ent_mask.size() * 8, hipMemcpyHostToDevice, ctx->stream));
        }
        FSM_HIP(hipStreamSynchronize(ctx->stream));
    } catch (...) {
        delete d;
        throw;
    }
    db->spade_dev = d;
}

void spade_release(fsm_db* db) {
    delete db->spade_dev;
    db->spade_dev = nullptr;
}

void spade_mine(fsm_ctx* ctx, fsm_db* db, double support, fsm_patterns** out) {
    const double t0 = now_ms();
    SpadeDevDB* d = db->spade_dev;
    const int64_t total = db->spade.total;
    Miner mn{ctx, d, ctx->stream, d->W, 1, 0, {}};
    KernelClock clock(ctx->stream);
    ClockScope clock_scope(&clock);
    mn.clk = &clock;
    mn.comm = ctx->comm;
    mn.agr.comm = ctx->comm;
    mn.agr.what = "SPADE";
    Comm* comm = ctx->comm;
    ctx->stats.mask_words = d->W;
    // minsupp = Math.ceil(support * total) (SPADE.scala:113), >= 1 for the lattice
    const double ms = std::ceil(support * double(total));
    const bool none = !(ms == ms) || ms > double(INT32_MAX);
    mn.minsup = none ? 0x7FFFFFFFu : (ms < 1.0 ? 1u : uint32_t(ms));
    size_t free_b = 0, total_b = 0;
    FSM_HIP(hipMemGetInfo(&free_b, &total_b));
    mn.budget = ctx->opts.mem_budget > 0 ? uint64_t(ctx->opts.mem_budget) : uint64_t(free_b / 2) / uint64_t(ctx->dev_share);
    mn.pend = ctx->pinned_u64();
    mn.zblk.alloc(Miner::kZBytes);
    FSM_HIP(hipMemsetAsync(mn.zblk.p, 0, Miner::kZBytes, ctx->stream));
    mn.d_tests = static_cast<unsigned long long*>(mn.zslot(8));

    // ---- F1 (K1)
    std::vector<uint32_t> f1(size_t(d->U), 0);
    {
        DevBuf d_f1(std::max<int64_t>(d->U, 1) * 4);
        FSM_HIP(hipMemsetAsync(d_f1.p, 0, size_t(d->U) * 4, ctx->stream));
        // sharded: each rank histograms its slice of the entries, then one all-reduce
        const uint64_t e0 = comm ? uint64_t(d->E) * uint64_t(comm->rank()) / uint64_t(comm->nranks()) : 0;
        const uint64_t e1 = comm ? uint64_t(d->E) * uint64_t(comm->rank() + 1) / uint64_t(comm->nranks()) : uint64_t(d->E);
        if (e1 > e0) {
            const int use_lds = d->U <= 16384;
            const unsigned grid = unsigned(std::min<uint64_t>((e1 - e0 + kBlock - 1) / kBlock, use_lds ? 1024 : 8192));
            const size_t tk = clock.begin("k_f1");
            hipLaunchKernelGGL(k_f1, dim3(grid), dim3(kBlock), use_lds ? size_t(d->U) * 4 : 0, ctx->stream,
                               d->item.as<uint32_t>(), e0, e1, d_f1.as<uint32_t>(), uint32_t(d->U), use_lds);
            FSM_LAUNCHED("k_f1", ctx->stream);
            clock.end(tk, int64_t((e1 - e0) * 4 + uint64_t(d->U) * 4), int64_t((e1 - e0) * 4));
        }
        if (comm) comm->allreduce_u32(d_f1.as<uint32_t>(), size_t(d->U), ctx->stream);
        // (through pinned memory: a pageable read-back is staged by the runtime)
        PinnedBuf* pb = ctx->pinned_big(std::max<size_t>(size_t(d->U) * 4, 4));
        if (d->U) FSM_HIP(hipMemcpyAsync(pb->host, d_f1.p, size_t(d->U) * 4, hipMemcpyDeviceToHost, ctx->stream));
        FSM_HIP(hipStreamSynchronize(ctx->stream));
        if (d->U) std::memcpy(f1.data(), pb->host, size_t(d->U) * 4);
    }
    std::vector<uint32_t> freq;
    if (!none)
        for (int64_t i = 0; i < d->U; ++i)
            if (f1[size_t(i)] >= mn.minsup) freq.push_back(uint32_t(i));

    if (comm && !freq.empty()) {
        // root counter rows: contiguous rank slices of about equal F2 work.  The ordered
        // enumeration tests every entry against its whole row (work ~ the entry count); the
        // unordered one (k_f2_tri) only against the partners above it, so an entry of rank k
        // weighs sup(k) x (the root entries of ranks >= k): rows are sorted by rank
        const bool tri = mn.tri_expected(uint32_t(freq.size()));
        uint64_t tot_e = 0;
        for (uint32_t it : freq) tot_e += f1[it];
        std::vector<uint64_t> w(freq.size());
        uint64_t tot = 0, above = tot_e;
        for (size_t k = 0; k < freq.size(); ++k) {
            const uint64_t e = f1[freq[k]];
            w[k] = tri ? e * ((above + (e + 1) / 2) >> 4) + 1 : e;  // (>> 4: the sum stays in 64 bits)
            above -= e;
            tot += w[k];
        }
        const uint64_t N = uint64_t(comm->nranks()), r = uint64_t(comm->rank());
        uint64_t acc = 0;
        mn.slice_lo = mn.slice_hi = uint32_t(freq.size());
        for (size_t k = 0; k < freq.size(); ++k) {
            if (mn.slice_lo == freq.size() && acc * N >= tot * r) mn.slice_lo = uint32_t(k);
            if (acc * N >= tot * (r + 1)) { mn.slice_hi = uint32_t(k); break; }
            acc += w[k];
        }
        if (mn.slice_hi < mn.slice_lo) mn.slice_hi = mn.slice_lo;
    }
    // the root entries this rank joins as the owner in the F2 (its rank slice; all unsharded)
    for (size_t k = comm ? mn.slice_lo : 0; k < (comm ? std::min<size_t>(mn.slice_hi, freq.size()) : freq.size()); ++k)
        ctx->stats.rank_root_owned += int64_t(f1[freq[k]]);
    std::vector<std::unique_ptr<Batch>> stack;
    if (!freq.empty()) {
        auto root = std::make_unique<Batch>();
        root->root = true;  // (even if run_root fails below: every rank then takes the root's gather)
        mn.run_or_defer([&] {  // agreed on in the root count
            mn.maybe_inject("root");
            mn.run_root(*root, freq, f1);
        });
        const double t1 = now_ms();
        ctx->stats.ms_f1 = t1 - t0;
        mn.count_and_freq(*root);
        ctx->stats.ms_f2 = now_ms() - t1;
        stack.push_back(std::move(root));
    } else {
        ctx->stats.ms_f1 = now_ms() - t0;
    }
    const double t2 = now_ms();
    // ---- lattice: DFS over class batches (each group of children = one batch);
    // sharded: rank-local, failures agreed on before the pattern gather
    mn.run_or_defer([&] {
    mn.maybe_inject("lattice");
    std::vector<std::unique_ptr<Batch>> spare;  // popped batches, recycled
    auto pop = [&] {
        stack.back()->recycle();
        spare.push_back(std::move(stack.back()));
        stack.pop_back();
    };
    while (!stack.empty()) {
        Batch& top = *stack.back();
        if (top.next_group >= top.groups.size() && !mn.claim_more(top)) {
            pop();
            continue;
        }
        const size_t g = top.next_group++;
        std::unique_ptr<Batch> nb;
        if (spare.empty()) {
            nb = std::make_unique<Batch>();
        } else {
            nb = std::move(spare.back());
            spare.pop_back();
        }
        nb->depth = top.depth + 1;
        // a pattern cannot hold more items than the longest sequence has (item, eid) occurrences
        if (nb->depth > db->spade.max_occ)
            throw Error(FSM_EDEVICE, "SPADE internal error: lattice depth " + std::to_string(nb->depth) +
                                         " exceeds the longest sequence (" + std::to_string(db->spade.max_occ) + ")");
        mn.emit(top, g, *nb);
        if (top.next_group >= top.groups.size() && top.claim_key < 0) {
            // parent fully emitted: release it before descending (a claiming root stays until
            // its claims run out)
            pop();
        }
        mn.count_and_freq(*nb);
        stack.push_back(std::move(nb));
    }
    mn.sync();  // the last deferred emit check, before the agreement
    });
    // sharded: a failure from here on is agreed on in the pattern gather (no round trip of its own)
    mn.run_or_defer([&] {
        unsigned long long tests = 0;
        FSM_HIP(hipMemcpyAsync(&tests, mn.d_tests, 8, hipMemcpyDeviceToHost, ctx->stream));
        mn.sync();
        ctx->stats.pair_tests = int64_t(tests);
    });
    ctx->stats.ms_lattice = now_ms() - t2;
    if (const char* v = std::getenv("FSM_HOST_TRACE"); v && v[0] == '1')
        std::fprintf(stderr, "[fsm host] f2 sort %.3f, kids %.3f, children %.3f, groups %.3f, emit tables %.3f, "
                     "slab alloc %.3f, count prep %.3f, count+extract %.3f, gpu wait %.3f ms\n", mn.hp[0], mn.hp[1],
                     mn.hp[2], mn.hp[3], mn.hp[4], mn.hp[5], mn.hp[6], mn.hp[7], mn.wait_ms);
    if (const char* v = std::getenv("FSM_HOST_TRACE"); v && v[0] == '1') {
        std::fprintf(stderr, "[fsm host laps]");
        for (int i = 0; i < 16; ++i) std::fprintf(stderr, " %d:%.2f", i, mn.hq[i]);
        std::fprintf(stderr, "\n");
    }
    mn.run_or_defer([&] { clock.finish(ctx->kstats); });
    for (const fsm_kernel_stat& k : ctx->kstats) {
        const std::string nm = k.name;
        if (nm == "k_count" || nm.rfind("k_root_keys", 0) == 0 || nm == "k_group_count") ctx->stats.ms_count_kernel += k.ms;
        if (nm.rfind("k_emit", 0) == 0) ctx->stats.ms_emit_kernel += k.ms;
    }

    // ---- output CSR in discovery order (the reference's order is discovery order too);
    // sharded: rank 0 holds the shared root levels, every rank its own classes.
    // Every node carries its pattern's item and itemset counts, so the output is
    // split over host threads in two passes: per-thread totals, then each thread
    // writes its offsets and fills its patterns by walking their parents (the
    // fresh output pages are first touched by the threads that fill them).
    const double to0 = now_ms();
    ctx->stats.ms_gpu_wait = mn.wait_ms;
    MallocArr<int32_t> sup, items;
    MallocArr<int64_t> pat_off, set_off;
    int64_t n = 0;
    mn.run_or_defer([&] {
    const auto& nodes = mn.nodes;
    const int64_t NN = int64_t(nodes.size());
    const int64_t first = (comm && comm->rank() != 0) ? int64_t(mn.n_shared) : 0;
    // this rank's output nodes: [first, NN) minus the nodes of split classes rank 0 outputs
    std::vector<int32_t> outn;
    const bool any_dup = !mn.node_dup.empty();
    if (any_dup) {
        outn.reserve(size_t(NN - first));
        for (int64_t k = first; k < NN; ++k)
            if (size_t(k) >= mn.node_dup.size() || !mn.node_dup[size_t(k)]) outn.push_back(int32_t(k));
    }
    auto node_at = [&](int64_t k) -> int64_t { return any_dup ? int64_t(outn[size_t(k)]) : first + k; };
    n = any_dup ? int64_t(outn.size()) : NN - first;
    const int64_t nthr = n >= (int64_t(1) << 16) ? host_threads() : 1;
    auto par = [&](auto&& fn) { par_slices(nthr, n, fn); };  // fn(t, k0, k1) over nthr slices of [0, n)
    std::vector<int64_t> tsets(size_t(nthr) + 1, 0), titems(size_t(nthr) + 1, 0);
    par([&](int64_t t, int64_t k0, int64_t k1) {
        int64_t a = 0, c = 0;
        for (int64_t k = k0; k < k1; ++k) {
            const uint32_t ls = nodes[size_t(node_at(k))].len_sets;
            a += ls & 0xFFFFu;
            c += ls >> 16;
        }
        tsets[size_t(t) + 1] = a;
        titems[size_t(t) + 1] = c;
    });
    for (int64_t t = 0; t < nthr; ++t) {
        tsets[size_t(t) + 1] += tsets[size_t(t)];
        titems[size_t(t) + 1] += titems[size_t(t)];
    }
    // the output arrays are filled in place (malloc'd, handed to the caller:
    // no zero-fill and no second copy of multi-hundred-MB pattern sets)
    sup.alloc(static_cast<size_t>(n));
    pat_off.alloc(static_cast<size_t>(n) + 1);
    set_off.alloc(static_cast<size_t>(tsets[size_t(nthr)]) + 1);
    items.alloc(static_cast<size_t>(titems[size_t(nthr)]));
    pat_off[size_t(n)] = tsets[size_t(nthr)];
    set_off[set_off.n - 1] = titems[size_t(nthr)];
    const int32_t* ival = db->spade.item_val.data();
    if (first == 0 && !any_dup && nthr > 1) {
        // Every node is output at its own index and its parent precedes it, so a pattern
        // is its parent's pattern plus one item: offsets first, then one parallel pass per
        // pattern length copying the parent's items and itemset starts (written by the
        // previous pass) instead of walking the whole parent chain per pattern.
        std::vector<uint32_t> tmax(size_t(nthr), 0);
        par([&](int64_t t, int64_t k0, int64_t k1) {
            int64_t ps = tsets[size_t(t)], pi = titems[size_t(t)];
            uint32_t mx = 0;
            for (int64_t k = k0; k < k1; ++k) {
                const uint32_t ls = nodes[size_t(k)].len_sets;
                pat_off[size_t(k)] = ps;
                set_off[size_t(ps)] = pi;  // the first itemset starts at the pattern's first item
                ps += ls & 0xFFFFu;
                pi += ls >> 16;
                mx = std::max(mx, ls >> 16);
            }
            tmax[size_t(t)] = mx;
        });
        const uint32_t maxL = *std::max_element(tmax.begin(), tmax.end());
        // node indices bucketed by pattern length (threads' counts, then their slots)
        std::vector<int64_t> cnt(size_t(nthr) * (maxL + 2), 0);
        par([&](int64_t t, int64_t k0, int64_t k1) {
            int64_t* c = cnt.data() + size_t(t) * (maxL + 2);
            for (int64_t k = k0; k < k1; ++k) ++c[nodes[size_t(k)].len_sets >> 16];
        });
        std::vector<int64_t> lstart(maxL + 2, 0);
        int64_t acc = 0;
        for (uint32_t L = 0; L <= maxL; ++L) {
            lstart[L] = acc;
            for (int64_t t = 0; t < nthr; ++t) {
                int64_t& c = cnt[size_t(t) * (maxL + 2) + L];
                const int64_t v = c;
                c = acc;
                acc += v;
            }
        }
        lstart[maxL + 1] = acc;
        RawVec<uint32_t> order(static_cast<size_t>(n));
        par([&](int64_t t, int64_t k0, int64_t k1) {
            int64_t* c = cnt.data() + size_t(t) * (maxL + 2);
            for (int64_t k = k0; k < k1; ++k) order[size_t(c[nodes[size_t(k)].len_sets >> 16]++)] = uint32_t(k);
        });
        for (uint32_t L = 1; L <= maxL; ++L) {
            const int64_t a = lstart[L], z = lstart[L + 1];
            if (z <= a) continue;
            par_slices(z - a >= (int64_t(1) << 12) ? nthr : 1, z - a, [&](int64_t, int64_t i0, int64_t i1) {
                for (int64_t i = a + i0; i < a + i1; ++i) {
                    const int64_t k = order[size_t(i)];
                    const PNode& nd = nodes[size_t(k)];
                    const int64_t ps = pat_off[size_t(k)], pi = set_off[size_t(ps)];
                    sup[size_t(k)] = int32_t(nd.support);
                    if (nd.parent < 0) {
                        items[size_t(pi)] = ival[nd.item];
                        continue;
                    }
                    const int64_t pp = nd.parent, pps = pat_off[size_t(pp)], pns = pat_off[size_t(pp) + 1] - pps;
                    const int64_t ppi = set_off[size_t(pps)];
                    std::memcpy(&items[size_t(pi)], &items[size_t(ppi)], size_t(L - 1) * sizeof(int32_t));
                    items[size_t(pi + L - 1)] = ival[nd.item];
                    for (int64_t q = 1; q < pns; ++q) set_off[size_t(ps + q)] = set_off[size_t(pps + q)] - ppi + pi;
                    if (nd.type == kSeq) set_off[size_t(ps + pns)] = pi + L - 1;
                }
            });
        }
    } else
    par([&](int64_t t, int64_t k0, int64_t k1) {
        int64_t ps = tsets[size_t(t)], pi = titems[size_t(t)];
        for (int64_t k = k0; k < k1; ++k) {
            const int64_t nk = node_at(k);
            const uint32_t ls = nodes[size_t(nk)].len_sets;
            pat_off[size_t(k)] = ps;
            ps += ls & 0xFFFFu;
            pi += ls >> 16;
            int64_t pos = pi, sidx = ps;
            for (int32_t q = int32_t(nk); q >= 0; q = nodes[size_t(q)].parent) {
                const PNode& nd = nodes[size_t(q)];
                items[size_t(--pos)] = ival[nd.item];
                if (nd.parent < 0 || nd.type == kSeq) set_off[size_t(--sidx)] = pos;
            }
            sup[size_t(k)] = int32_t(nodes[size_t(nk)].support);
        }
    });
    });
    ctx->stats.ms_output = now_ms() - to0;
    auto* p = static_cast<fsm_patterns*>(std::calloc(1, sizeof(fsm_patterns)));
    if (!p) throw Error(FSM_ENOMEM, "calloc failed");
    p->total = total;
    p->minsup = int32_t(std::min<uint32_t>(mn.minsup, 0x7FFFFFFFu));
    if (comm) {  // every rank's CSR, concatenated in rank order (after the failure agreement)
        if (mn.agr.code) n = 0;
        std::vector<int32_t> vs, vi;
        std::vector<int64_t> vp{0}, vo{0};
        if (!mn.agr.code) {
            vs.assign(sup.p, sup.p + sup.n);
            vi.assign(items.p, items.p + items.n);
            vp.assign(pat_off.p, pat_off.p + pat_off.n);
            vo.assign(set_off.p, set_off.p + set_off.n);
        }
        gather_patterns(comm, ctx->stream, vs, vp, vo, vi, ctx->stats, &mn.agr, ctx->result_root_only);
        n = int64_t(vs.size());
        p->n_sets = int64_t(vo.size()) - 1;
        p->n_items = int64_t(vi.size());
        copy_out(p->support, vs);
        copy_out(p->pat_off, vp);
        copy_out(p->set_off, vo);
        copy_out(p->items, vi);
    } else {
        p->n_sets = int64_t(set_off.n) - 1;
        p->n_items = int64_t(items.n);
        p->support = sup.release();
        p->pat_off = pat_off.release();
        p->set_off = set_off.release();
        p->items = items.release();
    }
    p->n = n;
    ctx->stats.patterns = n;
    ctx->stats.ms_mine = now_ms() - t0;
    *out = p;
}

}  // namespace fsm
