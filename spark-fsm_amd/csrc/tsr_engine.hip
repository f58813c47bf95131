// tsr_engine.hip — Top-K Sequential Rules (TSR.scala:102-105, [EXT]
// TSRAlgorithm) on MI355X.
//
// HBM layout (uploaded once by fsm_db_from_*):
//   horizontal rows  row_off[N+1]; per entry item / first / last (u32), the
//                    entries of a row sorted by item (binary-searchable)
//   vertical lists   vert_off[U+1], vert_sid / vert_item: the sids of each
//                    item (built on the GPU by k_vcount + scan + k_vscatter)
//
// The counts are computed on the GPU; the order-dependent top-k bookkeeping
// (save / registerAsCandidate / popMaximum with the rising minsup) is replayed
// on the host in exactly the reference's order, so the result is bit-identical
// to the CPU restatement whatever the GPU scheduling:
//   pair phase   k_pairs: for a block of items i, every s in sids(i) scans the
//                tail of row s (items j > i) and counts i=>j (first_i < last_j)
//                and j=>i (first_j < last_i) into a dense block x U matrix;
//                k_pairs_compact (wave ballot) emits the pairs that can reach
//                the block's starting minsup, in (i, j) order.
//   expansions   k_expand: one thread per sid of the rarest item of the rule;
//                binary-searches the rule's items in the row, derives firstX /
//                lastY, and histograms the expandL (c before lastY) / expandR
//                (c after firstX) candidates plus |sids(X u {c})|;
//                k_expand_compact pulls the candidates with count >= minsup and
//                re-zeroes the histograms.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <memory>
#include <queue>
#include <set>
#include <unordered_map>
#include <unordered_set>

#include "comm.h"
#include "dev_db.h"
#include "device_util.h"


namespace fsm {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxSide = 64;
constexpr int kCollectBlocks = 8;   // collect blocks per rule slot (FSM_TSR_GRID sweep: 4-8 best)
constexpr int kExpBatch = 384;      // rules expanded per launch (speculative, committed in order; FSM_TSR_BATCH; swept on MI355X)
constexpr int kExpBatchWide = 768;  // the same when the pair phase ends at minsup >= kWideMinsup (swept on MI355X)
constexpr uint32_t kWideMinsup = 32;
constexpr int kMaxBatch = 1024;  // FSM_TSR_BATCH ceiling (the slot searches of the kernels)
constexpr int kExpandBlocks = 4096; // bitmap path: at most this many expansion blocks per rule slot
constexpr int kExpSpb = 128;        // bitmap path: expected domain sids per expansion block (FSM_TSR_SPB; swept: 64-512)
constexpr int kDlBlocks = 512;      // bitmap path: |sids(X u {c})| blocks
constexpr int kDlUnroll = 8;        // k_dl: independent words / sids per thread per round
constexpr int kSpecDepth = 6;       // child speculation: levels per launch
constexpr int kSpecMax = 2;         // child speculation: rules per level, in batches (2 x B)
constexpr int kExpSets = 2;         // launch sets (buffers, stream, events) in flight
// FSM_TSR_GRID="expand,collect,dl" overrides the per-launch grids (tuning sweeps)
struct TsrGrid {
    unsigned expand = kExpandBlocks, collect = kCollectBlocks, dl = kDlBlocks;
    TsrGrid() {
        if (const char* v = std::getenv("FSM_TSR_GRID")) {
            unsigned a = 0, b = 0, c = 0;
            if (std::sscanf(v, "%u,%u,%u", &a, &b, &c) == 3 && a && b && c && a <= 4096 && b <= 4096 && c <= 4096) {
                expand = a;
                collect = b;
                dl = c;
            }
        }
    }
};

__global__ __launch_bounds__(kBlock) void k_vcount(const uint32_t* __restrict__ item, uint64_t E,
                                                   uint32_t* __restrict__ cnt) {
    for (uint64_t e = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += uint64_t(gridDim.x) * blockDim.x)
        atomicAdd(&cnt[item[e]], 1u);
}

__global__ __launch_bounds__(kBlock) void k_vscatter(const uint32_t* __restrict__ row_off,
                                                     const uint32_t* __restrict__ item, uint64_t N,
                                                     const uint64_t* __restrict__ voff, uint32_t* __restrict__ cursor,
                                                     uint32_t* __restrict__ vsid, uint32_t* __restrict__ vitem) {
    const uint64_t s = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (s >= N) return;
    for (uint32_t e = row_off[s]; e < row_off[s + 1]; ++e) {
        const uint32_t it = item[e];
        const uint64_t d = voff[it] + atomicAdd(&cursor[it], 1u);
        vsid[d] = uint32_t(s);
        vitem[d] = it;
    }
}

__device__ __forceinline__ uint32_t row_find(const uint32_t* __restrict__ item, uint32_t lo, uint32_t hi,
                                             uint32_t key) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (item[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void k_pairs(const uint32_t* __restrict__ vsid, const uint32_t* __restrict__ vitem,
                                                  uint64_t v0, uint64_t v1, uint32_t a, uint32_t U, uint32_t t,
                                                  uint32_t slo, uint32_t shi,
                                                  const uint32_t* __restrict__ sup,
                                                  const uint32_t* __restrict__ row_off,
                                                  const uint32_t* __restrict__ item, const uint32_t* __restrict__ first,
                                                  const uint32_t* __restrict__ last, uint32_t* __restrict__ scr) {
    const uint64_t v = v0 + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (v >= v1) return;
    const uint32_t i = vitem[v];
    if (sup[i] < t) return;
    const uint32_t s = vsid[v];
    if (s - slo >= shi - slo) return;  // sharded pair phase: another rank's sequences
    const uint32_t rb = row_off[s], re = row_off[s + 1];
    const uint32_t k = row_find(item, rb, re, i);
    const uint32_t fi = first[k], li = last[k];
    uint32_t* row = scr + uint64_t(i - a) * U * 2;
    for (uint32_t q = k + 1; q < re; ++q) {
        const uint32_t j = item[q];
        if (sup[j] < t) continue;
        if (fi < last[q]) atomicAdd(row + 2 * j, 1u);       // i => j
        if (first[q] < li) atomicAdd(row + 2 * j + 1, 1u);  // j => i
    }
}

// Rows restricted to the items with support >= t (one wave per row, ballot
// compaction, item order kept): pass 1 counts (out == nullptr), pass 2 writes
// item / first / last and the item's support (read beside the entry by the
// expansions: no dependent support lookup per entry).
__global__ __launch_bounds__(kBlock) void k_rows_keep(const uint32_t* __restrict__ row_off,
                                                      const uint32_t* __restrict__ item,
                                                      const uint32_t* __restrict__ first,
                                                      const uint32_t* __restrict__ last,
                                                      const uint32_t* __restrict__ isup, uint32_t t, uint64_t N,
                                                      uint32_t* __restrict__ cnt, const uint64_t* __restrict__ off,
                                                      uint32_t* __restrict__ o_item, uint32_t* __restrict__ o_first,
                                                      uint32_t* __restrict__ o_last, uint32_t* __restrict__ o_sup) {
    const uint64_t wstride = (uint64_t(gridDim.x) * blockDim.x) >> 6;
    for (uint64_t r = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; r < N; r += wstride) {
        const uint32_t rb = row_off[r], re = row_off[r + 1];
        uint64_t o = off ? off[r] : 0;
        uint32_t n = 0;
        for (uint32_t e0 = rb; e0 < re; e0 += 64) {
            const uint32_t e = e0 + lane_id();
            const uint32_t c = e < re ? item[e] : 0u;
            const uint32_t sp = e < re ? isup[c] : 0u;
            const bool keep = e < re && sp >= t;
            const uint64_t b = ballot(keep);
            if (off && keep) {
                const uint64_t d = o + uint32_t(__popcll(b & lanemask_lt()));
                o_item[d] = c;
                o_first[d] = first[e];
                o_last[d] = last[e];
                o_sup[d] = sp;
            }
            o += uint32_t(__popcll(b));
            n += uint32_t(__popcll(b));
        }
        if (!off && lane_id() == 0) cnt[r] = n;
    }
}

__global__ __launch_bounds__(kBlock) void k_off32(const uint64_t* __restrict__ off, uint64_t n,
                                                  uint32_t* __restrict__ out) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i <= n; i += uint64_t(gridDim.x) * blockDim.x)
        out[i] = uint32_t(off[i]);
}

struct PairRec {
    uint32_t i, j, ij, ji;
};

// one wave per item row of the block: count (out == nullptr) or write (+ re-zero the
// counters when `zero`; the sharded pair phase still reads them afterwards)
__global__ __launch_bounds__(kBlock) void k_pairs_compact(uint32_t* __restrict__ scr, uint32_t a, uint32_t nb,
                                                          uint32_t U, uint32_t t, uint32_t* __restrict__ rowcnt,
                                                          const uint64_t* __restrict__ rowoff,
                                                          PairRec* __restrict__ out, int zero) {
    const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (g >= nb) return;
    const uint32_t i = a + g;
    uint32_t* row = scr + uint64_t(g) * U * 2;
    uint64_t o = out ? rowoff[g] : 0;
    uint32_t n = 0;
    for (uint32_t j0 = i + 1; j0 < U; j0 += 64) {
        const uint32_t j = j0 + lane_id();
        uint32_t ij = 0, ji = 0;
        if (j < U) { ij = row[2 * j]; ji = row[2 * j + 1]; }
        const bool keep = j < U && (ij >= t || ji >= t);
        const uint64_t b = ballot(keep);
        if (out) {
            if (keep) out[o + __popcll(b & lanemask_lt())] = PairRec{i, j, ij, ji};
            if (zero && j < U && (ij | ji)) { row[2 * j] = 0; row[2 * j + 1] = 0; }
            o += uint64_t(__popcll(b));
        } else {
            n += uint32_t(__popcll(b));
        }
    }
    if (!out && lane_id() == 0) rowcnt[g] = n;
}

// sharded pair phase: this rank's partial (ij, ji) of every candidate key (i, j)
__global__ __launch_bounds__(kBlock) void k_pairs_gather(const uint32_t* __restrict__ scr, uint32_t a, uint32_t U,
                                                         const uint2* __restrict__ keys, uint32_t n,
                                                         uint32_t* __restrict__ out) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const uint2 k = keys[q];
    const uint32_t* row = scr + uint64_t(k.x - a) * U * 2;
    out[2 * q] = row[2 * k.y];
    out[2 * q + 1] = row[2 * k.y + 1];
}

struct Side {
    uint32_t nx, ny, doL, doR;
    uint32_t maxX, maxY;
    uint32_t drv;    // bitmap path: the rarest item of X u Y
    uint32_t lmode;  // bitmap path: 1 = the domain from drv's sid list (short) probed in the other bitmaps;
                     // 2 = the domain from the parent rule's kept rows (pl, pn) and the new item pc
    uint32_t pc;     // lmode 2: the item the rule added to its parent (to X when pleft, else to Y)
    uint32_t pleft;
    uint32_t pn;     // lmode 2: the parent's kept rows
    uint32_t kb;     // this rule's kept rows: at most kb (its support) ...
    uint64_t pl;     // lmode 2: the parent's first entry in the kept-rows arena
    uint64_t ko;     // ... written from arena entry ko (kNoList: none kept)
    uint32_t xid;    // the item set X's interned id (Replay::XIntern: the |sids(X u {c})| memo's exact key)
    uint32_t klo;    // bitmap path: the lowest kid ever counted, min(max X, max Y) + 1 (as kids)
    uint32_t X[kMaxSide];
    uint32_t Y[kMaxSide];
};

__device__ __forceinline__ bool in_sorted(const uint32_t* s, uint32_t n, uint32_t c) {
    for (uint32_t k = 0; k < n; ++k) {
        if (s[k] == c) return true;
        if (s[k] > c) return false;
    }
    return false;
}

// expansion control block (device memory), reset by k_expand_collect
struct ExpCtl {
    uint32_t nx;     // |sids(X)| seen by this expansion
    uint32_t nlist;  // items touched (list entries)
    uint32_t nout;   // candidates kept
    uint32_t done;   // collect blocks finished
    uint32_t nsid;   // bitmap path: domain sids (holding X u Y: the bitmap AND)
    uint32_t nent;   // bitmap path: row entries of the domain sids (SURVEY's scan)
    uint32_t nhold;  // bitmap path: domain rows where X => Y holds (with a candidate past mlo)
    uint32_t nwalk;  // bitmap path: row entries the row kernel walks (those rows' suffixes)
    uint32_t nkeep;  // bitmap path: domain rows kept for the rule's children (k_exp_rows, pass 0)
    uint32_t pad[3];
};
constexpr uint64_t kNoList = ~uint64_t(0);

// histogram bump (no returned value: the lanes' atomics stay in flight) that
// also records the item the first time it is touched in this expansion, so the
// collect pass visits only touched items
__device__ __forceinline__ void bump(uint32_t* __restrict__ h, uint32_t c, uint32_t* __restrict__ seen,
                                     uint32_t* __restrict__ list, ExpCtl* __restrict__ ctl) {
    atomicAdd(&h[c], 1u);
    if (__hip_atomic_load(&seen[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
        atomicExch(&seen[c], 1u) == 0u)
        list[atomicAdd(&ctl->nlist, 1u)] = c;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = max(v, uint32_t(__shfl_xor(int(v), d, 64)));
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = min(v, uint32_t(__shfl_xor(int(v), d, 64)));
    return v;
}

// One wave per sid of the driver item (rows are up to thousands of items long
// on Kosarak-shaped data: the lanes split the binary searches and the row
// scans, so one long row does not serialize a thread).
// A batch of up to kExpBatch rules (slot b: rule side, driver sid range,
// histograms / touched list / control at slot offsets) in one launch; waves
// are numbered across slots by the prefix wave_off.
__global__ __launch_bounds__(kBlock) void k_expand(const Side* __restrict__ sides,
                                                   const uint64_t* __restrict__ drv_off,
                                                   const uint64_t* __restrict__ wave_off, uint32_t nslot,
                                                   const uint32_t* __restrict__ vert_sid,
                                                   const uint32_t* __restrict__ row_off,
                                                   const uint32_t* __restrict__ item,
                                                   const uint32_t* __restrict__ first,
                                                   const uint32_t* __restrict__ last, uint32_t U,
                                                   uint32_t* __restrict__ TLb, uint32_t* __restrict__ DLb,
                                                   uint32_t* __restrict__ TRb, uint32_t* __restrict__ seenb,
                                                   uint32_t* __restrict__ listb, ExpCtl* __restrict__ ctlb,
                                                   const uint32_t* __restrict__ isup, uint32_t t) {
    const uint64_t w = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    if (w >= wave_off[nslot]) return;
    uint32_t b = 0;  // slot of this wave: the last b with wave_off[b] <= w
    for (uint32_t step = kMaxBatch / 2; step > 0; step >>= 1)
        if (b + step < nslot && wave_off[b + step] <= w) b += step;
    const Side& side = sides[b];
    const uint64_t U64 = U;
    uint32_t* TL = TLb + b * U64;
    uint32_t* DL = DLb + b * U64;
    uint32_t* TR = TRb + b * U64;
    uint32_t* seen = seenb + b * U64;
    uint32_t* list = listb + b * U64;
    ExpCtl* ctl = ctlb + b;
    const uint32_t lane = lane_id();
    const uint32_t s = vert_sid[drv_off[b] + (w - wave_off[b])];
    const uint32_t rb = row_off[s], re = row_off[s + 1];
    bool ok = true;
    uint32_t fX = 0;
    for (uint32_t k = lane; k < side.nx; k += 64) {
        const uint32_t q = row_find(item, rb, re, side.X[k]);
        if (q >= re || item[q] != side.X[k]) ok = false;
        else fX = max(fX, first[q]);
    }
    if (ballot(!ok)) return;  // s not in sids(X)
    fX = wave_max(fX);
    if (lane == 0) atomicAdd(&ctl->nx, 1u);
    if (side.doL) {  // |sids(X u {c})| for candidate left extensions
        const uint32_t q0 = row_find(item, rb, re, side.maxX + 1);
        for (uint32_t q = q0 + lane; q < re; q += 64)
            if (isup[item[q]] >= t && !in_sorted(side.Y, side.ny, item[q])) bump(DL, item[q], seen, list, ctl);
    }
    uint32_t lY = 0xFFFFFFFFu;
    for (uint32_t k = lane; k < side.ny; k += 64) {
        const uint32_t q = row_find(item, rb, re, side.Y[k]);
        if (q >= re || item[q] != side.Y[k]) ok = false;
        else lY = min(lY, last[q]);
    }
    if (ballot(!ok)) return;  // s not in sids(Y)
    lY = wave_min(lY);
    if (fX >= lY) return;  // X => Y does not hold in s
    if (side.doL) {        // expandL: c > max(X), c not in Y, c before lastY(s)
        const uint32_t q0 = row_find(item, rb, re, side.maxX + 1);
        for (uint32_t q = q0 + lane; q < re; q += 64) {
            const uint32_t c = item[q];
            if (first[q] < lY && isup[c] >= t && !in_sorted(side.Y, side.ny, c)) bump(TL, c, seen, list, ctl);
        }
    }
    if (side.doR) {        // expandR: c > max(Y), c not in X, c after firstX(s)
        const uint32_t q0 = row_find(item, rb, re, side.maxY + 1);
        for (uint32_t q = q0 + lane; q < re; q += 64) {
            const uint32_t c = item[q];
            if (last[q] > fX && isup[c] >= t && !in_sorted(side.X, side.nx, c)) bump(TR, c, seen, list, ctl);
        }
    }
}

struct ExpRec {
    uint32_t c, tl, dl, tr;
};
struct ExpHdr {
    uint32_t nout, nx, nsid, nent, nhold, nwalk;
    uint32_t ln;  // bitmap path: the rows the rule kept (in the arena at its slot's ko, if <= kb)
    uint32_t pad;
};

// List path: visit the items this expansion touched, keep the counts >= t
// (records to mapped pinned host memory, any order; the host sorts them by
// item) and re-zero the counters and the touched marks.
__global__ __launch_bounds__(kBlock) void k_expand_collect(uint32_t* __restrict__ TLb, uint32_t* __restrict__ DLb,
                                                           uint32_t* __restrict__ TRb, uint32_t* __restrict__ seenb,
                                                           const uint32_t* __restrict__ listb,
                                                           ExpCtl* __restrict__ ctlb, uint32_t U, uint32_t t,
                                                           ExpRec* __restrict__ outb, uint32_t cap) {
    const uint64_t b = blockIdx.y, U64 = U;
    uint32_t* TL = TLb + b * U64;
    uint32_t* DL = DLb + b * U64;
    uint32_t* TR = TRb + b * U64;
    uint32_t* seen = seenb + b * U64;
    const uint32_t* list = listb + b * U64;
    ExpCtl* ctl = ctlb + b;
    ExpRec* out = outb + b * uint64_t(cap);
    const uint32_t n = ctl->nlist;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t c = list[i];
        const uint32_t tl = TL[c], dl = DL[c], tr = TR[c];
        TL[c] = 0;
        DL[c] = 0;
        TR[c] = 0;
        seen[c] = 0;
        if (tl >= t || tr >= t) {
            const uint32_t idx = atomicAdd(&ctl->nout, 1u);
            if (idx < cap) out[idx] = ExpRec{c, tl, dl, tr};
        }
    }
}

// Publish every slot's header and reset its control block for the next
// launch.  Runs in the kernel after the collect (k_dl, or k_publish on the
// list path): the kernel boundary orders it after every collect block, with
// no cross-block completion counter (an agent-scope fence per block writes
// back the XCD's L2, which cost more than the collect itself).
__device__ __forceinline__ void publish_slots(ExpCtl* __restrict__ ctlb, ExpHdr* __restrict__ hdrb, uint32_t nslot) {
    for (uint32_t b = threadIdx.x; b < nslot; b += blockDim.x) {
        ExpCtl& c = ctlb[b];
        hdrb[b].ln = c.nkeep;
        c.nkeep = 0;
        hdrb[b].nout = c.nout;
        hdrb[b].nx = c.nx;
        hdrb[b].nsid = c.nsid;
        hdrb[b].nent = c.nent;
        hdrb[b].nhold = c.nhold;
        hdrb[b].nwalk = c.nwalk;
        c.nhold = 0;
        c.nwalk = 0;
        c.nx = 0;
        c.nlist = 0;
        c.nout = 0;
        c.done = 0;
        c.nsid = 0;
        c.nent = 0;
    }
}

__global__ __launch_bounds__(kBlock) void k_publish(ExpCtl* __restrict__ ctlb, ExpHdr* __restrict__ hdrb,
                                                    uint32_t nslot) {
    publish_slots(ctlb, hdrb, nslot);
}

// ---- sid bitmaps: one bit per sequence per item.  They replace
// the driver item's sid list as the expansion domain: the sids holding every
// item of X u Y come from one AND over |X|+|Y| bitmaps, and |sids(X u {c})|
// of the left-extension candidates that survive from AND + popcount, so no
// expansion walks the rows of all sids(X) any more.
__global__ __launch_bounds__(kBlock) void k_bitmap_build(const uint32_t* __restrict__ vsid,
                                                         const uint32_t* __restrict__ vitem, uint64_t E,
                                                         uint32_t NW, uint32_t* __restrict__ bm) {
    for (uint64_t e = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += uint64_t(gridDim.x) * blockDim.x) {
        const uint32_t sid = vsid[e];
        atomicOr(&bm[uint64_t(vitem[e]) * NW + (sid >> 5)], 1u << (sid & 31u));
    }
}

// ---- bitmap path: expansion rows packed for the expansions.  After the pair
// phase only the items with support >= its minsup (K "kept" items, dense kid
// ascending with the item, so c > max(X) compares alike) can still be in a
// rule; every row is cut to them and each entry packed into 8 bytes:
//   x = kid, y = first | last << 16  (itemset indexes of the row, < 65536)
// one load per lane per entry (the entry's support check is the alive bitmap).
__global__ __launch_bounds__(kBlock) void k_rows_pack(const uint32_t* __restrict__ row_off,
                                                      const uint32_t* __restrict__ item,
                                                      const uint32_t* __restrict__ first,
                                                      const uint32_t* __restrict__ last,
                                                      const uint32_t* __restrict__ kid_of, uint64_t N,
                                                      uint32_t* __restrict__ cnt, uint32_t* __restrict__ maxpos,
                                                      const uint64_t* __restrict__ off, uint2* __restrict__ out) {
    const uint64_t wstride = (uint64_t(gridDim.x) * blockDim.x) >> 6;
    uint32_t mp = 0;
    for (uint64_t r = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; r < N; r += wstride) {
        const uint32_t rb = row_off[r], re = row_off[r + 1];
        uint64_t o = off ? off[r] : 0;
        uint32_t n = 0;
        for (uint32_t e0 = rb; e0 < re; e0 += 64) {
            const uint32_t e = e0 + lane_id();
            const uint32_t k = e < re ? kid_of[item[e]] : kNone;
            const bool keep = k != kNone;
            const uint64_t b = ballot(keep);
            if (keep) {
                const uint32_t la = last[e];
                mp = max(mp, la);
                if (off) out[o + uint32_t(__popcll(b & lanemask_lt()))] = make_uint2(k, first[e] | (la << 16));
            }
            o += uint32_t(__popcll(b));
            n += uint32_t(__popcll(b));
        }
        if (!off && lane_id() == 0) cnt[r] = n;
    }
    if (!off) {
        mp = wave_max(mp);
        if (lane_id() == 0 && mp) atomicMax(maxpos, mp);
    }
}

// alive[w], 2 bits per kid (16 kids per word): code 1 when kid 16w + j still
// has support >= the launch minsup t, else 0 (t only rises, so a dead kid
// never comes back; run when t changes).  k_exp_rows marks X / Y on its copy.
__global__ __launch_bounds__(kBlock) void k_alive(const uint32_t* __restrict__ ksup, uint32_t K, uint32_t t,
                                                  uint32_t* __restrict__ alive) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= (K + 15) / 16) return;
    uint32_t v = 0;
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t k = w * 16 + j;
        if (k < K && ksup[k] >= t) v |= 1u << (2 * j);
    }
    alive[w] = v;
}

// Expansions on the bitmap path (no device-scope atomics per
// entry): k_exp_domain ANDs each rule's |X|+|Y| item bitmaps once and
// compacts the sids holding X u Y into a per-slot domain list; k_exp_rows
// counts the expandL / expandR candidates of the domain rows into LDS
// histograms, one dense partial row per block; k_expand_reduce sums them.
#ifndef FSM_TSR_XBLOCK
#define FSM_TSR_XBLOCK 512
#endif
constexpr int kXBlock = FSM_TSR_XBLOCK;     // threads of an expansion block
constexpr uint32_t kExpWin = 2 * kXBlock;   // sids per LDS window (two per thread in the length scan)
#ifndef FSM_TSR_EPT
#define FSM_TSR_EPT 8
#endif
constexpr int kEpt = FSM_TSR_EPT;           // row entries per lane per chunk (registers)
constexpr uint32_t kChunkEnt = uint32_t(kXBlock) * kEpt;  // entries of one flat chunk
constexpr uint32_t kPassKids = 4096;        // kids per LDS histogram pass (2 x 16 KiB)
constexpr uint32_t kMaxKids = 65536;        // bitmap path: kept items (kid codes 16 KiB of LDS)

// |sids(X u {c})| memo (bitmap path): open addressing over uint4 entries (64-bit key, the
// count), written by k_dl, read by k_expand_reduce of later launches.  The key is the item
// set's identity, not a hash of it: (id(X) + 1) << 32 | c, with id(X) the host's interned id
// of the item set X (Replay::XIntern), so two different sets never share a key.  An entry is
// written once (key by CAS, then the count in one 8-byte store with a written flag) and every
// count is final, so a reader sees either a miss or the exact count.
struct DlMemo {
    uint4* tab;     // nullptr: no memo
    uint32_t mask;  // entries - 1 (a power of two)
};
constexpr uint32_t kMemoProbe = 8;
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t memo_key(uint32_t xid, uint32_t c) { return (uint64_t(xid) + 1ull) << 32 | c; }
__device__ __forceinline__ uint32_t memo_slot(const DlMemo& m, uint64_t key) { return uint32_t(mix64(key)) & m.mask; }
__device__ __forceinline__ uint32_t memo_find(const DlMemo& m, uint64_t key) {
    uint32_t h = memo_slot(m, key);
    for (uint32_t k = 0; k < kMemoProbe; ++k, h = (h + 1) & m.mask) {
        const uint4 e = m.tab[h];
        const uint64_t ek = uint64_t(e.x) | (uint64_t(e.y) << 32);
        if (ek == 0) return 0u;
        if (ek == key) return e.z ? e.w : 0u;  // (z = 0: claimed, count not yet written)
    }
    return 0u;
}
__device__ __forceinline__ void memo_put(const DlMemo& m, uint64_t key, uint32_t v) {
    uint32_t h = memo_slot(m, key);
    for (uint32_t k = 0; k < kMemoProbe; ++k, h = (h + 1) & m.mask) {
        unsigned long long* kp = reinterpret_cast<unsigned long long*>(&m.tab[h].x);
        const unsigned long long old = atomicCAS(kp, 0ull, (unsigned long long)key);
        if (old == 0ull || old == key) {
            *reinterpret_cast<unsigned long long*>(&m.tab[h].z) = 1ull | (uint64_t(v) << 32);
            return;
        }
    }
}

struct ExpGeo {       // kernel view of one launch's geometry
    uint32_t K, KP;   // kept items, kids per pass
    uint32_t nblk;    // expansion blocks of the launch (partial rows per pass)
    uint32_t t;       // launch minsup
};

// the bumps of one candidate entry (kid c alive and not in X u Y; first |
// last << 16) of a row where X => Y holds (firstX fX < lastY lY): expandL when
// c > max X and c occurs before lastY; expandR when c > max Y and c occurs
// after firstX; only kids of this pass [kid_lo, kid_lo + KP)
__device__ __forceinline__ void bump(uint32_t c, uint32_t fl, uint32_t fX, uint32_t lY, bool, bool, uint32_t maxX,
                                     uint32_t maxY, uint32_t doL, uint32_t doR, uint32_t kid_lo, uint32_t KP,
                                     uint32_t* hL, uint32_t* hR) {
    const uint32_t rel = c - kid_lo;
    if (rel >= KP) return;
    if (doL && c > maxX && (fl & 0xFFFFu) < lY) atomicAdd(&hL[rel], 1u);
    if (doR && c > maxY && (fl >> 16) > fX) atomicAdd(&hR[rel], 1u);
}

// Rank directory of the kept items' sid bitmaps: rdir[k * NW4 + g] = the sids below
// 128 g holding kid k's item (exclusive prefix popcount, one entry per 4-word group).
// One block per kid.
__global__ __launch_bounds__(kBlock) void k_rank_dir(const uint32_t* __restrict__ bm, uint32_t NW,
                                                     const uint32_t* __restrict__ kept, uint32_t* __restrict__ rdir) {
    __shared__ uint32_t wsum[kBlock / 64];
    const uint32_t k = blockIdx.x, NW4 = NW / 4u;
    const uint4* row = reinterpret_cast<const uint4*>(bm + uint64_t(kept[k]) * NW);
    uint32_t* out = rdir + uint64_t(k) * NW4;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (uint32_t g0 = 0; g0 < NW4; g0 += blockDim.x) {
        const uint32_t g = g0 + threadIdx.x;
        uint32_t c = 0;
        if (g < NW4) {
            const uint4 v = row[g];
            c = uint32_t(__popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w));
        }
        const uint32_t inc = wave_incl_scan(c);
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint32_t before = 0, tot = 0;
        for (uint32_t w = 0; w < kBlock / 64; ++w) {
            before += w < wv ? wsum[w] : 0u;
            tot += wsum[w];
        }
        if (g < NW4) out[g] = carry + before + inc - c;
        carry += tot;
        __syncthreads();  // wsum is rewritten next round
    }
}

// rank of sid in one item's sid bitmap (the sids below it holding the item): the
// item's rank directory entry + the popcounts of its words before sid
__device__ __forceinline__ uint32_t bm_rank(const uint32_t* __restrict__ bmrow, const uint32_t* __restrict__ rd,
                                            uint32_t sid) {
    const uint32_t g = sid >> 7, wi = (sid >> 5) & 3u, bit = sid & 31u;
    const uint4 v = reinterpret_cast<const uint4*>(bmrow)[g];
    uint32_t r = rd[g];
    r += wi > 0u ? uint32_t(__popc(v.x)) : 0u;
    r += wi > 1u ? uint32_t(__popc(v.y)) : 0u;
    r += wi > 2u ? uint32_t(__popc(v.z)) : 0u;
    const uint32_t cw = wi == 0u ? v.x : (wi == 1u ? v.y : (wi == 2u ? v.z : v.w));
    return r + uint32_t(__popc(cw & ((1u << bit) - 1u)));
}

// The kept rows' vertical entries: for the entry of kid k in packed row s,
// vfl[kvoff[k] + rank of s in k's bitmap] = (first | last << 16, its position in
// the row), so a sid's entry of any kid is two loads away (bm_rank, vfl).  One
// thread per row.
__global__ __launch_bounds__(kBlock) void k_vfl(const uint32_t* __restrict__ k_off, const uint2* __restrict__ ent,
                                                uint32_t N, const uint32_t* __restrict__ bm, uint32_t NW,
                                                const uint32_t* __restrict__ kept, const uint32_t* __restrict__ rdir,
                                                const uint32_t* __restrict__ kvoff, uint2* __restrict__ vfl) {
    const uint32_t NW4 = NW / 4u;
    for (uint32_t sid = blockIdx.x * blockDim.x + threadIdx.x; sid < N; sid += gridDim.x * blockDim.x) {
        const uint32_t rs = k_off[sid], re = k_off[sid + 1];
        for (uint32_t e = rs; e < re; ++e) {
            const uint2 v = ent[e];
            const uint32_t r = bm_rank(bm + uint64_t(kept[v.x]) * NW, rdir + uint64_t(v.x) * NW4, sid);
            vfl[kvoff[v.x] + r] = make_uint2(v.y, e - rs);
        }
    }
}

// Domain of rule slot k (grid.y): its |X|+|Y| item bitmaps ANDed over this
// block's kDomWords words (4 consecutive words per thread, 16-byte operand
// loads, 8 operands in flight), the set sids compacted into the slot's domain
// list at dom_off[k] (one cursor atomic per block: ExpCtl::nsid).  Every pass of
// the row kernel reads this list; the bitmaps are ANDed once per rule.
constexpr uint32_t kDomThreads = 256;
constexpr uint32_t kDomWords = 4 * kDomThreads;  // bitmap words per domain block

// List mode (Side::lmode, chosen on the host when the rarest item's sid list is shorter than
// a quarter of a bitmap's words): the slot's blocks split that list, every sid is probed in
// the other items' bitmaps (one 4-byte read each, L2-resident) and the survivors compacted
// as above: |L| x |X u Y| probes instead of |X u Y| whole-bitmap operands.
__global__ __launch_bounds__(kDomThreads) void k_exp_domain(const Side* __restrict__ sides,
                                                            const uint32_t* __restrict__ bm, uint32_t NW,
                                                            const uint64_t* __restrict__ dom_off,
                                                            uint32_t* __restrict__ dom, ExpCtl* __restrict__ ctlb,
                                                            const uint64_t* __restrict__ vert_off,
                                                            const uint32_t* __restrict__ vert_sid) {
    __shared__ uint32_t sIt[2 * kMaxSide];
    __shared__ uint32_t wsum[kDomThreads / 64];
    __shared__ uint32_t b_base;
    const uint32_t k = blockIdx.y;
    const Side& side = sides[k];
    if (side.lmode == 2) return;  // the domain is the parent's kept rows (k_exp_rows reads them)
    const uint32_t nxy = side.nx + side.ny;
    for (uint32_t q = threadIdx.x; q < nxy; q += blockDim.x) sIt[q] = q < side.nx ? side.X[q] : side.Y[q - side.nx];
    __syncthreads();
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    uint32_t* out = dom + dom_off[k];
    if (side.lmode) {
        const uint32_t drv = side.drv;
        const uint64_t l0 = vert_off[drv], l1 = vert_off[drv + 1];
        const uint64_t per = (l1 - l0 + gridDim.x - 1) / gridDim.x;
        const uint64_t a = l0 + per * blockIdx.x, z = min(l1, a + per);
        for (uint64_t r0 = a; r0 < z; r0 += blockDim.x) {  // block-uniform rounds
            const uint64_t q = r0 + threadIdx.x;
            bool keep = false;
            uint32_t sid = 0;
            if (q < z) {
                sid = vert_sid[q];
                keep = true;
                for (uint32_t t = 0; t < nxy && keep; ++t) {
                    const uint32_t it = sIt[t];
                    if (it != drv) keep = (bm[uint64_t(it) * NW + (sid >> 5)] >> (sid & 31u)) & 1u;
                }
            }
            const uint64_t bal = ballot(keep);
            if (lane == 0) wsum[wv] = uint32_t(__popcll(bal));
            __syncthreads();
            if (threadIdx.x == 0) {
                uint32_t tot = 0;
                for (uint32_t w = 0; w < kDomThreads / 64; ++w) tot += wsum[w];
                b_base = tot ? atomicAdd(&ctlb[k].nsid, tot) : 0u;
            }
            __syncthreads();
            if (keep) {
                uint32_t p = b_base + uint32_t(__popcll(bal & lanemask_lt()));
                for (uint32_t w = 0; w < wv; ++w) p += wsum[w];
                out[p] = sid;
            }
            __syncthreads();  // wsum / b_base are rewritten next round
        }
        return;
    }
    const uint32_t w = blockIdx.x * kDomWords + 4 * threadIdx.x;  // NW is a multiple of 4
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (w < NW) {
        v = make_uint4(~0u, ~0u, ~0u, ~0u);
        for (uint32_t k0 = 0; k0 < nxy; k0 += 8) {
            uint4 o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                o[j] = k0 + j < nxy ? *reinterpret_cast<const uint4*>(bm + uint64_t(sIt[k0 + j]) * NW + w)
                                    : make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                v.x &= o[j].x;
                v.y &= o[j].y;
                v.z &= o[j].z;
                v.w &= o[j].w;
            }
            if (!(v.x | v.y | v.z | v.w)) break;
        }
    }
    const uint32_t cnt = uint32_t(__popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w));
    const uint32_t incl = wave_incl_scan(cnt);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t q = 0; q < kDomThreads / 64; ++q) tot += wsum[q];
        b_base = tot ? atomicAdd(&ctlb[k].nsid, tot) : 0u;
    }
    __syncthreads();
    if (!cnt) return;
    uint32_t p = b_base + incl - cnt;
    for (uint32_t q = 0; q < wv; ++q) p += wsum[q];
    const uint32_t ww[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int h = 0; h < 4; ++h)
        for (uint32_t m = ww[h]; m; m &= m - 1u) out[p++] = (w + uint32_t(h)) * 32u + uint32_t(__builtin_ctz(m));
}

// A domain sid's firstX (max over X of the item's first itemset) and lastY (min over
// Y of the last), and the row positions of max X and max Y (the sides' last items),
// from the kept items' vertical entries: rank of the sid in the item's bitmap (rank
// directory + popcounts) -> vfl.  Two dependent loads per item, the items' loads in
// flight together.
struct DomProbe {
    const uint32_t* bm;
    uint32_t NW, NW4;
    const uint32_t* rdir;
    const uint32_t* kvoff;
    const uint2* vfl;
    __device__ __forceinline__ bool operator()(uint32_t sid, const uint32_t* sIt, const uint32_t* sKid, uint32_t nx,
                                               uint32_t nxy, uint32_t& fl, uint32_t& pX, uint32_t& pY) const {
        uint32_t fX = 0, lY = 0xFFFFu;
        pX = pY = 0;
        for (uint32_t t0 = 0; t0 < nxy; t0 += 4) {
            uint2 v[4];
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t t = t0 + u;
                if (t < nxy) {
                    const uint32_t kk = sKid[t];
                    const uint32_t r = bm_rank(bm + uint64_t(sIt[t]) * NW, rdir + uint64_t(kk) * NW4, sid);
                    v[u] = vfl[kvoff[kk] + r];
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t t = t0 + u;
                if (t >= nxy) break;
                if (t < nx) fX = max(fX, v[u].x & 0xFFFFu); else lY = min(lY, v[u].x >> 16);
                if (t == nx - 1u) pX = v[u].y;
                if (t == nxy - 1u) pY = v[u].y;
            }
        }
        fl = fX | (lY << 16);
        return fX < lY;
    }
};

// The rows of slot b's domain (k_exp_domain's list of row suffixes, this block's
// share of it) counted into LDS histograms of the kid range [kid_lo, kid_lo + KP),
// pass = blockIdx.y.  Windows of kExpWin domain rows: their (start, length,
// firstX | lastY) entries are loaded coalesced and the lengths scanned; the
// window's rows are then walked FLAT: chunks of whole rows holding at most
// kChunkEnt entries are spread over every lane of the block (each wave a
// contiguous stretch of the chunk, lane-interleaved: one coalesced 8-byte load
// per lane per step, kEpt steps per lane in registers), so a 2,000-entry row is
// 4 steps of 8 waves instead of one wave's serial chain of dependent loads, and
// an 8-entry row does not leave 56 lanes idle.  A lane finds its row from the
// step's row-start mask: the rows starting inside the step flag their offsets in
// a wave-private LDS word array, one ballot turns the flags into a 64-bit mask
// and mbcnt counts the starts up to the lane.  Each kid's role comes from one
// 2-bit code (dead, candidate, in X, in Y; ctab) behind a 64-bit bloom of X u Y;
// the candidates are bumped straight from the registers (firstX / lastY come with
// the row: no first walk, no barrier).  Each block writes its whole histogram as
// one dense partial row (plain coalesced stores); k_expand_reduce sums a slot's
// rows.
__device__ __forceinline__ uint32_t kid_code(const uint32_t* ctab, uint32_t c) {
    return (ctab[c >> 4] >> ((c & 15u) * 2u)) & 3u;
}

__global__ __launch_bounds__(kXBlock) void k_exp_rows(const Side* __restrict__ sides,
                                                      const uint64_t* __restrict__ blk_off, uint32_t nslot,
                                                      const uint64_t* __restrict__ dom_off,
                                                      const uint32_t* __restrict__ dom,
                                                      const uint32_t* __restrict__ row_off,
                                                      const uint2* __restrict__ ent,
                                                      const uint32_t* __restrict__ kid_of,
                                                      const uint32_t* __restrict__ alive, ExpGeo geo,
                                                      uint32_t* __restrict__ part, ExpCtl* __restrict__ ctlb,
                                                      uint32_t* __restrict__ ndlw, DomProbe probe, uint4* arena) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dsm[];  // hist L [KP] | hist R [KP] | ctab
    // window rows: x = first flat entry (exclusive scan of the lengths), y = row start in
    // `ent` minus x (u32 wrap: the ent index of flat entry q is y + q)
    __shared__ uint2 rowv[kExpWin + 1];
    __shared__ uint32_t sfl[kExpWin];                // per row: firstX | lastY << 16
    __shared__ unsigned long long s_bloom;
    __shared__ uint32_t wflag[kXBlock / 64][64];     // per wave: row-start flags of the current step (tags)
    __shared__ uint32_t sXY[2 * kMaxSide];           // X then Y, as kids
    __shared__ uint32_t sItm[2 * kMaxSide];          // X then Y, as items
    __shared__ uint32_t wsum[kXBlock / 64], wcnt[kXBlock / 64];
    __shared__ uint32_t s_kbase;                     // the window's first kept row (pass 0)
    const uint32_t KP = geo.KP, pass = blockIdx.y, kid_lo = pass * KP;
    uint32_t* hL = dsm;
    uint32_t* hR = dsm + KP;
    uint32_t* ctab = dsm + 2 * KP;  // 2 bits per kid: 0 dead, 1 candidate, 2 in X, 3 in Y
    // slot of this block: the last b with blk_off[b] <= blockIdx.x (blocks per slot sized by its domain)
    uint32_t b = 0;
    for (uint32_t step = kMaxBatch / 2; step > 0; step >>= 1)
        if (b + step < nslot && blk_off[b + step] <= blockIdx.x) b += step;
    const uint32_t bx = uint32_t(blockIdx.x - blk_off[b]), nbx = uint32_t(blk_off[b + 1] - blk_off[b]);
    const Side& side = sides[b];
    ExpCtl* ctl = ctlb + b;
    // k_expand_reduce (next on the stream) appends the k_dl work list
    if (blockIdx.x == 0 && pass == 0 && threadIdx.x == 0) *ndlw = 0u;
    const uint32_t nx = side.nx, ny = side.ny, nxy = nx + ny;
    const uint32_t doL = side.doL, doR = side.doR;
    const uint32_t lane = lane_id();
    const uint32_t wv = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    for (uint32_t k = threadIdx.x; k < 2 * KP; k += blockDim.x) dsm[k] = 0;
    for (uint32_t k = threadIdx.x; k < (geo.K + 15) / 16; k += blockDim.x) ctab[k] = alive[k];
    for (uint32_t k = threadIdx.x; k < nxy; k += blockDim.x) {
        const uint32_t it = k < nx ? side.X[k] : side.Y[k - nx];
        sItm[k] = it;
        sXY[k] = kid_of[it];
    }
    wflag[wv][lane] = 0;
    // this block's share of the slot's domain: the sids of the bitmap AND (k_exp_domain), or the
    // parent rule's kept rows (lmode 2)
    const bool pmode = side.lmode == 2;
    const uint32_t nd = pmode ? side.pn : ctl->nsid;
    const uint32_t d0 = uint32_t(uint64_t(nd) * bx / nbx), d1 = uint32_t(uint64_t(nd) * (bx + 1) / nbx);
    const uint32_t* dl = dom + dom_off[b];
    const uint4* dlp = arena + (pmode ? side.pl : 0ull);  // (arena: read here, written below; no restrict)
    const bool keep = side.ko != kNoList;
    uint4* kp = arena + (keep ? side.ko : 0ull);  // the rule's kept rows (for its children)
    // a row's candidates lie past min(max X, max Y) (sides ascend by item): its position is max X's
    // when max X is the smaller (or only X extends), else max Y's
    const bool use_px = doL && (!doR || side.maxX < side.maxY);
    const uint32_t pkid = pmode ? kid_of[side.pc] : 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nxy; k += blockDim.x) {  // X -> code 2, Y -> code 3
        const uint32_t c = sXY[k], sh = (c & 15u) * 2u;
        atomicAnd(&ctab[c >> 4], ~(3u << sh));
        atomicOr(&ctab[c >> 4], (k < nx ? 2u : 3u) << sh);
    }
    if (threadIdx.x == 0) {  // bit (c & 63) of every kid c of X u Y: most entries skip the ctab read
        unsigned long long bl = 0;
        for (uint32_t k = 0; k < nxy; ++k) bl |= 1ull << (sXY[k] & 63u);
        s_bloom = bl;
    }
    const uint32_t maxX = sXY[nx - 1], maxY = sXY[nxy - 1];  // sides ascend by item, so by kid
    uint32_t my_ent = 0;   // row entries walked by this block (thread 0)
    uint32_t my_full = 0, my_hold = 0;  // pass 0: the domain rows' entries, the rows where the rule holds
    uint32_t tag = 0;      // this wave's step tags in wflag
    // the domain rows start past min(max X, max Y) already; a later pass starts at its kid_lo
    const uint32_t mlo = kid_lo == 0 ? 0u : kid_lo - 1u;
    for (uint32_t win = d0; win < d1; win += kExpWin) {
        const uint32_t n0 = min(kExpWin, d1 - win);
        uint32_t n;  // the window's rows where X => Y holds (block-uniform)
        {   // the window's sids probed (2t, 2t + 1 per thread): the rows where X => Y holds with a
            // non-empty suffix past mlo, compacted, with the exclusive scan of the suffix lengths.
            // A parent-list row probes only the added item: X => Y held there for the parent, the
            // child holds where the item is present and keeps first X before last Y
            const uint32_t j = 2 * threadIdx.x;
            uint32_t st[2] = {0u, 0u}, ln[2] = {0u, 0u}, fv[2] = {0u, 0u}, ok[2] = {0u, 0u};
            uint4 kv[2];
#pragma unroll
            for (uint32_t u = 0; u < 2; ++u) {
                if (j + u >= n0) continue;
                uint32_t sid, f = 0, pX = 0, pY = 0;
                bool hold;
                if (pmode) {
                    const uint4 pe = dlp[win + j + u];  // (sid, firstX | lastY << 16, pos max X, pos max Y)
                    sid = pe.x;
                    const uint32_t* bmc = probe.bm + uint64_t(side.pc) * probe.NW;
                    hold = (bmc[sid >> 5] >> (sid & 31u)) & 1u;
                    if (hold) {
                        const uint32_t r = bm_rank(bmc, probe.rdir + uint64_t(pkid) * probe.NW4, sid);
                        const uint2 v = probe.vfl[probe.kvoff[pkid] + r];
                        uint32_t fX = pe.y & 0xFFFFu, lY = pe.y >> 16;
                        pX = pe.z;
                        pY = pe.w;
                        if (side.pleft) {
                            fX = max(fX, v.x & 0xFFFFu);
                            pX = v.y;
                        } else {
                            lY = min(lY, v.x >> 16);
                            pY = v.y;
                        }
                        f = fX | (lY << 16);
                        hold = fX < lY;
                    }
                } else {
                    sid = dl[win + j + u];
                    hold = probe(sid, sItm, sXY, nx, nxy, f, pX, pY);
                }
                if (!hold) continue;
                const uint32_t rs = row_off[sid], rl = row_off[sid + 1] - rs;
                if (pass == 0) my_full += rl;  // (SURVEY basis: the rows where the rule holds, whole)
                const uint32_t pm = use_px ? pX : pY;
                if (pm + 1u < rl) {
                    ok[u] = 1u;
                    st[u] = rs + pm + 1u;
                    ln[u] = rl - pm - 1u;
                    fv[u] = f;
                    kv[u] = make_uint4(sid, f, pX, pY);
                }
            }
            const uint32_t c = ok[0] + ok[1], pr = ln[0] + ln[1];
            const uint32_t cinc = wave_incl_scan(c), inc = wave_incl_scan(pr);
            if (lane == 63) {
                wsum[wv] = inc;
                wcnt[wv] = cinc;
            }
            __syncthreads();  // (also: the previous window's LDS and the ctab codes are ready)
            uint32_t bb = 0, tt = 0, cb = 0, ct = 0;
            for (uint32_t k = 0; k < wpb; ++k) {
                bb += k < wv ? wsum[k] : 0u;
                tt += wsum[k];
                cb += k < wv ? wcnt[k] : 0u;
                ct += wcnt[k];
            }
            uint32_t ex = bb + inc - pr, ci = cb + cinc - c;
            const uint32_t ci0 = ci;
#pragma unroll
            for (uint32_t u = 0; u < 2; ++u) {
                if (!ok[u]) continue;
                rowv[ci] = make_uint2(ex, st[u] - ex);
                sfl[ci] = fv[u];
                ex += ln[u];
                ++ci;
            }
            if (threadIdx.x == 0) {
                rowv[ct] = make_uint2(tt, 0u);
                if (pass == 0) {
                    my_ent += tt;
                    my_hold += ct;
                    s_kbase = ct ? atomicAdd(&ctl->nkeep, ct) : 0u;
                }
            }
            n = ct;
            if (pass == 0 && keep) {  // the kept rows, for the rule's children (s_kbase: barrier)
                __syncthreads();
                uint32_t kc = s_kbase + ci0;  // (more than kb: the host drops the list)
#pragma unroll
                for (uint32_t u = 0; u < 2; ++u)
                    if (ok[u] && kc < side.kb) kp[kc++] = kv[u];
            }
        }
        __syncthreads();
        // an entry's kid code: 1 (a candidate) when its bloom bit is clear (not in X u Y;
        // whether the kid is still alive does not matter: a dead kid's count stays below
        // t, so k_expand_reduce drops it), else the exact code from ctab
        const uint64_t bloom = s_bloom;
        auto code_of = [&](uint32_t c) -> uint32_t { return ((bloom >> (c & 63u)) & 1ull) ? kid_code(ctab, c) : 1u; };
        // chunks of whole rows [j0, j1) with at most kChunkEnt entries (block-uniform loop).
        // Every domain row suffix holds an entry, so at most 64 rows start inside a step.
        for (uint32_t j0 = 0; j0 < n;) {
            const uint32_t E0 = rowv[j0].x;
            uint32_t j1 = j0;  // the last j in [j0, n] with start(j) - E0 <= kChunkEnt
            for (uint32_t hi = n; j1 < hi;) {
                const uint32_t mid = (j1 + hi + 1) >> 1;
                if (rowv[mid].x - E0 <= kChunkEnt) j1 = mid; else hi = mid - 1;
            }
            if (j1 == j0) {
                // one row longer than a chunk: the block walks it
                const uint32_t rs = rowv[j0].y + E0, len = rowv[j0 + 1].x - E0;
                const uint32_t fl = sfl[j0], fX = fl & 0xFFFFu, lY = fl >> 16;
                for (uint32_t q = threadIdx.x; q < len; q += blockDim.x) {
                    const uint2 e = ent[rs + q];
                    if (e.x > mlo && code_of(e.x) == 1u)
                        bump(e.x, e.y, fX, lY, false, false, maxX, maxY, doL, doR, kid_lo, KP, hL, hR);
                }
                ++j0;
                continue;
            }
            const uint32_t Tc = rowv[j1].x - E0;
            const uint32_t sw = (Tc + wpb * 64 - 1) / (wpb * 64) * 64;  // entries per wave (<= 64 kEpt)
            const uint32_t qa = E0 + wv * sw, qz = min(E0 + Tc, qa + sw);
            if (qa < qz) {
                // the wave's first row: the last j in [j0, j1) with start(j) <= qa (wave-uniform)
                uint32_t ja = j0;
                for (uint32_t hi = j1 - 1; ja < hi;) {
                    const uint32_t mid = (ja + hi + 1) >> 1;
                    if (rowv[mid].x <= qa) ja = mid; else hi = mid - 1;
                }
                uint32_t idx[kEpt], ej[kEpt];
                // the row of each entry from the step's row-start mask
#pragma unroll
                for (int u = 0; u < kEpt; ++u) {
                    const uint32_t q0 = qa + 64u * uint32_t(u);  // wave-uniform
                    idx[u] = kNone;
                    ej[u] = 0;
                    if (q0 < qz) {
                        const uint32_t jl = ja + 1u + lane;  // the rows after ja (non-empty: <= 64 start in the step)
                        const uint2 rl = jl < j1 ? rowv[jl] : make_uint2(0xFFFFFFFFu, 0u);
                        const uint32_t pp = rl.x - q0;  // row jl starts pp entries into the step (>= 1)
                        ++tag;
                        if (jl < j1 && pp - 1u < 63u) wflag[wv][pp] = tag;  // a start inside the step
                        const uint64_t nxt = ballot(jl < j1 && pp - 1u < 64u);  // starts in (q0, q0 + 64]
                        __builtin_amdgcn_wave_barrier();
                        const uint64_t m = ballot(wflag[wv][lane] == tag);
                        // row of lane l = ja + starts at offsets 1..l (lane r - 1 holds row ja + r)
                        const uint32_t r = uint32_t(__builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u))) +
                                           uint32_t((m >> lane) & 1ull);
                        const uint32_t ya = rowv[ja].y;
                        const uint32_t ys = uint32_t(__shfl(int(rl.y), int(r == 0u ? 0u : r - 1u), 64));
                        const uint32_t ab = r == 0u ? ya : ys;
                        if (q0 + lane < qz) {
                            idx[u] = ab + q0 + lane;
                            ej[u] = ja + r;
                        }
                        ja += uint32_t(__popcll(nxt));
                    }
                }
                uint2 e[kEpt];
#pragma unroll
                for (int u = 0; u < kEpt; ++u) e[u] = idx[u] != kNone ? ent[idx[u]] : make_uint2(0u, 0u);
#pragma unroll
                for (int u = 0; u < kEpt; ++u) {
                    if (idx[u] == kNone || e[u].x <= mlo || code_of(e[u].x) != 1u) continue;
                    const uint32_t fl = sfl[ej[u]];
                    bump(e[u].x, e[u].y, fl & 0xFFFFu, fl >> 16, false, false, maxX, maxY, doL, doR, kid_lo, KP,
                         hL, hR);
                }
            }
            j0 = j1;  // the next chunk's rows are disjoint
        }
    }
    __syncthreads();
    // the block's histograms -> its partial rows [L | R] (k_expand_reduce sums a slot's).  No kid at
    // or below min(max X, max Y) is ever counted (candidates lie past it): only the kids above it
    // are written, and the reduce reads no others
    uint32_t* prow = part + (uint64_t(pass) * geo.nblk + blockIdx.x) * 2 * KP;
    const uint32_t lo_abs = min(maxX, maxY) + 1u;
    const uint32_t klo = lo_abs > kid_lo ? min(lo_abs - kid_lo, KP) : 0u;
    for (uint32_t k = klo + threadIdx.x; k < KP; k += blockDim.x) {
        prow[k] = hL[k];
        prow[KP + k] = hR[k];
    }
    if (pass == 0 && threadIdx.x == 0) {
        if (my_ent) atomicAdd(&ctl->nwalk, my_ent);
        if (my_hold) atomicAdd(&ctl->nhold, my_hold);
    }
    if (pass == 0) {
        for (int d = 32; d > 0; d >>= 1) my_full += uint32_t(__shfl_xor(int(my_full), d, 64));
        if (lane == 0 && my_full) atomicAdd(&ctl->nent, my_full);
    }
}

// Sum each slot's partial rows per kid and keep the counts >= t: block x of
// (slot, pass) owns the kid range [x q, (x + 1) q) of the pass (q = ceil(KP /
// gridDim.x)) and writes its kept records IN KID ORDER from that range's start
// (block-ordered ballot compaction), with the count in rcnt, so the host takes
// every slot's records in item order without sorting.  Left extensions are
// queued for k_dl.  grid = (blocks per slot, slots, kid passes).
__global__ __launch_bounds__(kBlock) void k_expand_reduce(const uint32_t* __restrict__ part,
                                                          const uint64_t* __restrict__ blk_off, ExpGeo geo,
                                                          const uint32_t* __restrict__ kept,
                                                          ExpCtl* __restrict__ ctlb, ExpRec* __restrict__ outb,
                                                          uint32_t cap, uint4* __restrict__ dlw,
                                                          uint32_t* __restrict__ ndlw, uint32_t* __restrict__ rcnt,
                                                          const Side* __restrict__ sides, DlMemo memo) {
    __shared__ uint32_t wsum[kBlock / 64];
    const uint32_t b = blockIdx.y, pass = blockIdx.z, KP = geo.KP, kid_lo = pass * KP;
    // kids at or below min(max X, max Y) are never counted (k_exp_rows writes none of them)
    const uint32_t lo_abs = sides[b].klo;
    const uint64_t r0 = blk_off[b], r1 = blk_off[b + 1];
    const uint32_t q = (KP + gridDim.x - 1) / gridDim.x;
    const uint32_t c0 = blockIdx.x * q, c1 = min(KP, c0 + q);
    ExpRec* out = outb + uint64_t(b) * cap + kid_lo + c0;  // this range's records, from its start
    const uint32_t* rows = part + uint64_t(pass) * geo.nblk * 2 * KP;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    uint32_t n = 0;  // records written by this block (block-uniform)
    for (uint32_t cb = c0; cb < c1; cb += blockDim.x) {
        const uint32_t c = cb + threadIdx.x;
        uint32_t tl = 0, tr = 0;
        bool keep = false;
        if (c < c1 && kid_lo + c < geo.K && kid_lo + c >= lo_abs) {
            for (uint64_t r = r0; r < r1; ++r) {
                tl += rows[r * 2 * KP + c];
                tr += rows[r * 2 * KP + KP + c];
            }
            keep = tl >= geo.t || tr >= geo.t;
        }
        const uint64_t bal = ballot(keep);
        if (lane == 0) wsum[wv] = uint32_t(__popcll(bal));
        __syncthreads();
        uint32_t at = n, tot = 0;
        for (uint32_t k = 0; k < blockDim.x / 64; ++k) {
            at += k < wv ? wsum[k] : 0u;
            tot += wsum[k];
        }
        if (keep) {
            const uint32_t idx = at + uint32_t(__popcll(bal & lanemask_lt()));
            const uint32_t it = kept[kid_lo + c];
            // |sids(X u {c})| of a left extension: from the memo, else from k_dl
            uint32_t dl = 0;
            if (tl >= geo.t && memo.tab) dl = memo_find(memo, memo_key(sides[b].xid, it));
            out[idx] = ExpRec{it, tl, dl, tr};
            if (tl >= geo.t && !dl) dlw[atomicAdd(ndlw, 1u)] = make_uint4(b, it, kid_lo + c0 + idx, 0u);
        }
        n += tot;
        __syncthreads();  // wsum is rewritten next round
    }
    if (threadIdx.x == 0) {
        rcnt[(uint64_t(b) * gridDim.z + pass) * gridDim.x + blockIdx.x] = n;
        if (n) atomicAdd(&ctlb[b].nout, n);
    }
}

// |sids(X u {c})| for the kept left-extension candidates: AND + popcount
// A candidate c with fewer sids than bitmap words is counted over its own
// sid list (vertical list of c: one X-bitmap bit test per sid, the X bitmaps
// stay cache resident) instead of ANDing whole bitmaps.
__global__ __launch_bounds__(kBlock) void k_dl(const Side* __restrict__ sides, const uint32_t* __restrict__ bm,
                                               uint32_t NW, const uint64_t* __restrict__ vert_off,
                                               const uint32_t* __restrict__ vert_sid, const uint4* __restrict__ dlw,
                                               const uint32_t* __restrict__ ndlw, ExpRec* __restrict__ outb,
                                               uint32_t cap, ExpCtl* __restrict__ ctlb, ExpHdr* __restrict__ hdrb,
                                               uint32_t nslot, DlMemo memo) {
    __shared__ uint32_t red[kBlock / 64];
    if (blockIdx.x == 0) publish_slots(ctlb, hdrb, nslot);
    const uint32_t n = *ndlw;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint4 wk = dlw[i];
        const Side& side = sides[wk.x];
        uint32_t acc = 0;
        const uint64_t v0 = vert_off[wk.y], v1 = vert_off[wk.y + 1];
        const uint32_t nx = side.nx;
        // latency-bound (a few hundred KiB per candidate): kDlUnroll independent
        // steps per thread, every load of a round issued before any is used
        if (v1 - v0 < NW) {
            for (uint64_t q0 = v0 + threadIdx.x; q0 < v1; q0 += uint64_t(blockDim.x) * kDlUnroll) {
                uint32_t sid[kDlUnroll];
#pragma unroll
                for (int u = 0; u < kDlUnroll; ++u) {
                    const uint64_t q = q0 + uint64_t(u) * blockDim.x;
                    sid[u] = q < v1 ? vert_sid[q] : 0xFFFFFFFFu;
                }
                bool all[kDlUnroll];
#pragma unroll
                for (int u = 0; u < kDlUnroll; ++u) all[u] = sid[u] != 0xFFFFFFFFu;
                for (uint32_t k = 0; k < nx; ++k) {
                    const uint32_t* row = bm + uint64_t(side.X[k]) * NW;
                    uint32_t wv[kDlUnroll];
#pragma unroll
                    for (int u = 0; u < kDlUnroll; ++u) wv[u] = all[u] ? row[sid[u] >> 5] : 0u;
#pragma unroll
                    for (int u = 0; u < kDlUnroll; ++u) all[u] = all[u] && ((wv[u] >> (sid[u] & 31u)) & 1u);
                }
#pragma unroll
                for (int u = 0; u < kDlUnroll; ++u) acc += all[u] ? 1u : 0u;
            }
        } else {
            const uint32_t* rc = bm + uint64_t(wk.y) * NW;
            for (uint32_t w0 = threadIdx.x; w0 < NW; w0 += blockDim.x * kDlUnroll) {
                uint32_t v[kDlUnroll];
#pragma unroll
                for (int u = 0; u < kDlUnroll; ++u) {
                    const uint32_t w = w0 + uint32_t(u) * blockDim.x;
                    v[u] = w < NW ? rc[w] : 0u;
                }
                for (uint32_t k = 0; k < nx; ++k) {
                    const uint32_t* row = bm + uint64_t(side.X[k]) * NW;
                    uint32_t o[kDlUnroll];
#pragma unroll
                    for (int u = 0; u < kDlUnroll; ++u) {
                        const uint32_t w = w0 + uint32_t(u) * blockDim.x;
                        o[u] = w < NW ? row[w] : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < kDlUnroll; ++u) v[u] &= o[u];
                }
#pragma unroll
                for (int u = 0; u < kDlUnroll; ++u) acc += uint32_t(__popc(v[u]));
            }
        }
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) acc += uint32_t(__shfl_xor(int(acc), d, 64));
        if (lane_id() == 0) red[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (uint32_t k = 0; k < blockDim.x / 64; ++k) tot += red[k];
            outb[uint64_t(wk.x) * cap + wk.z].dl = tot;
            if (memo.tab && tot) memo_put(memo, memo_key(side.xid, wk.y), tot);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------ host replay
// Rules live in an arena (stable addresses, no per-rule heap vectors); their
// items sit in one shared pool, X then Y.  k1 / k2 hold the comparator's
// leading keys inline so heap sifts touch no rule object unless they tie.
struct Rule {
    uint64_t k1 = 0;   // sup << 32 | |X| << 16 | |Y|
    uint64_t k2 = 0;   // X[0] << 32 | (|X| > 1 ? X[1] : Y[0])
    double conf = 0;
    uint32_t sup = 0;
    uint32_t nX = 0;   // |sids(X)|
    uint32_t* it = nullptr;  // X at it[0, nx), Y at it[nx, nx + ny) (RuleStore's item chunks)
    uint16_t nx = 0, ny = 0;
    bool expandLR = false;
    bool dropped = false;  // a speculated child its parent's commit did not register
    int8_t inset = -1;     // replay: the launch set expanding it (results not yet taken in), or -1
    bool pleft = false;    // derived by adding pc to its parent's X (else to Y)
    bool spec = false;     // made by child speculation
    int32_t res = -1;      // replay: its expansion results (slot of the result pool), or -1
    uint32_t ln = 0, pn = 0, pc = 0;
    uint64_t loff = kNoList;   // its kept domain rows in the arena (ln of them), after its expansion
    uint64_t ploff = kNoList;  // its parent's (pn of them): its own domain is a subset of those rows
    uint32_t xid = 0;          // its item set X, interned (XIntern); kNone until first needed
    uint32_t pxid = 0;         // a left extension's parent X (X = X(parent) + its last item)
};

// The item sets X of the rules, interned: the |sids(X u {c})| memo's exact keys (DlMemo).  A
// single item is its own id; X u {c} gets the id of the pair (id(X), c), numbered from U up.
// A left extension only adds an item above every item of X (TopSeqRules' expandLeft
// candidates), so a set has exactly one chain of prefixes and one id whatever
// rule it appears in.
struct XIntern {
    uint32_t next = 0;
    std::vector<uint64_t> key;
    std::vector<uint32_t> val;
    size_t used = 0;
    void init(uint32_t U) {
        next = U;
        key.assign(size_t(1) << 16, 0ull);
        val.assign(key.size(), 0u);
        used = 0;
    }
    uint32_t get(uint32_t xid, uint32_t c) {
        const uint64_t k = (uint64_t(xid) + 1ull) << 32 | c;
        size_t m = key.size() - 1, h = size_t(mix64(k)) & m;
        for (; key[h]; h = (h + 1) & m)
            if (key[h] == k) return val[h];
        if (next >= 0xFFFFFFFEu) throw Error(FSM_ELIMIT, "TSR: more than 2^32 distinct rule antecedents");
        key[h] = k;
        val[h] = next;
        if (++used * 2 > key.size()) grow();
        return next++;
    }

  private:
    void grow() {
        std::vector<uint64_t> ok(key.size() * 2, 0ull);
        std::vector<uint32_t> ov(ok.size(), 0u);
        ok.swap(key);
        ov.swap(val);
        const size_t m = key.size() - 1;
        for (size_t q = 0; q < ok.size(); ++q)
            if (ok[q]) {
                size_t h = size_t(mix64(ok[q])) & m;
                while (key[h]) h = (h + 1) & m;
                key[h] = ok[q];
                val[h] = ov[q];
            }
    }
};

// Rules and their items in large chunks that never move (a c4 replay makes millions
// of rules: no per-rule allocation, no copy of a growing pool)
struct RuleStore {
    static constexpr size_t kRuleChunk = size_t(1) << 16, kItemChunk = size_t(1) << 22;
    std::vector<std::unique_ptr<Rule[]>> rule_chunks;
    std::vector<std::unique_ptr<uint32_t[]>> item_chunks;
    size_t n_rules = 0, item_used = kItemChunk;
    size_t size() const { return n_rules; }
    Rule& new_rule() {
        if (n_rules % kRuleChunk == 0) rule_chunks.emplace_back(new Rule[kRuleChunk]);
        Rule& r = rule_chunks.back()[n_rules % kRuleChunk];
        r = Rule{};
        ++n_rules;
        return r;
    }
    uint32_t* new_items(size_t n) {  // n <= 2 * kMaxSide
        if (item_used + n > kItemChunk) {
            item_chunks.emplace_back(new uint32_t[kItemChunk]);
            item_used = 0;
        }
        uint32_t* p = item_chunks.back().get() + item_used;
        item_used += n;
        return p;
    }
    const uint32_t* X(const Rule* r) const { return r->it; }
    const uint32_t* Y(const Rule* r) const { return r->it + r->nx; }
};

// RuleG.compareTo [EXT, recalled; SURVEY A.3]
int rule_cmp(const RuleStore& st, const Rule* a, const Rule* b) {
    if (a == b) return 0;
    if (a->k1 != b->k1) return a->k1 < b->k1 ? -1 : 1;  // support, |X|, |Y|
    // (int)(conf_a - conf_b): always 0 here (both in (0, 1]), kept for fidelity
    const int c4 = int(a->conf - b->conf);
    if (c4) return c4;
    if (a->k2 != b->k2) return a->k2 < b->k2 ? -1 : 1;  // X[0], then X[1] or Y[0]
    const uint32_t *xa = st.X(a), *xb = st.X(b);
    for (uint32_t k = 0; k < a->nx; ++k)
        if (xa[k] != xb[k]) return xa[k] < xb[k] ? -1 : 1;
    const uint32_t *ya = st.Y(a), *yb = st.Y(b);
    for (uint32_t k = 0; k < a->ny; ++k)
        if (ya[k] != yb[k]) return ya[k] < yb[k] ? -1 : 1;
    return 0;
}

// heap entry with the leading keys inline (k1 then k2 decide almost every sift)
struct HeapEnt {
    uint64_t k1, k2;
    Rule* r;
};

struct Replay {
    int32_t k;
    double minconf;
    uint32_t minsup = 1;
    RuleStore st;
    struct MinFirst {  // std::priority_queue puts the "largest" on top
        const RuleStore* st;
        bool operator()(const HeapEnt& a, const HeapEnt& b) const {
            if (a.k1 != b.k1) return a.k1 > b.k1;
            if (a.k2 != b.k2) return a.k2 > b.k2;
            return rule_cmp(*st, a.r, b.r) > 0;
        }
    };
    struct MaxFirst {
        const RuleStore* st;
        bool operator()(const HeapEnt& a, const HeapEnt& b) const {
            if (a.k1 != b.k1) return a.k1 < b.k1;
            if (a.k2 != b.k2) return a.k2 < b.k2;  // conf key between them is always 0 (see rule_cmp)
            return rule_cmp(*st, a.r, b.r) < 0;
        }
    };
    // candidates: one bucket per support value (the comparator's first key), so
    // the buckets below minsup (never expandable: minsup only rises) are freed as
    // it rises.  A bucket is an unsorted append-only array until it first becomes
    // the top: it is then sorted once (ascending: the maximum at the back, popped
    // in O(1) with sequential memory), and later arrivals into it go to a small
    // side heap.  A pop takes the larger of the sorted back and the side heap's
    // top: the same order as one heap, the comparator being a total order.
    // (Round 3's 4-ary heap per bucket measured 2-4 % slower on c4 and was retired in round 5.)
    struct CandQueue {
        struct Bucket {
            std::vector<HeapEnt> v;     // unsorted, or sorted ascending (sorted = true)
            std::vector<HeapEnt> side;  // sorted buckets: later arrivals, a binary max-heap
            bool sorted = false;
            bool empty() const { return v.empty() && side.empty(); }
        };
        std::vector<Bucket> bucket;
        std::vector<uint64_t> occ;  // bit s: bucket[s] non-empty (the next lower bucket is a word scan away)
        uint32_t top_sup = 0, floor = 0;  // buckets < floor are dropped
        size_t n = 0;
        size_t n_sorted = 0, n_popped = 0;  // entries sorted, and popped (verbose)
        MaxFirst cmp;
        explicit CandQueue(MaxFirst c) : cmp(c) {}
        bool empty() const { return n == 0; }
        size_t size() const { return n; }
        void push(const HeapEnt& e) {
            const uint32_t sp = uint32_t(e.k1 >> 32);
            if (sp < floor) return;  // dead on arrival (cannot happen: callers register sup >= minsup)
            if (sp >= bucket.size()) {
                bucket.resize(size_t(sp) + 1);
                occ.resize(size_t(sp) / 64 + 1, 0);
            }
            Bucket& b = bucket[sp];
            if (b.sorted) {
                b.side.push_back(e);
                std::push_heap(b.side.begin(), b.side.end(), cmp);
            } else {
                b.v.push_back(e);
            }
            occ[sp >> 6] |= 1ull << (sp & 63u);
            if (n == 0 || sp > top_sup) top_sup = sp;
            ++n;
        }
        Bucket& settle() {  // n > 0: move top_sup down to the highest non-empty bucket (sorted)
            if (bucket[top_sup].empty()) {
                size_t w = top_sup >> 6;
                uint64_t m = occ[w] & ((top_sup & 63u) ? ((1ull << (top_sup & 63u)) - 1ull) : 0ull);
                while (!m) m = occ[--w];
                top_sup = uint32_t(w * 64 + 63 - size_t(__builtin_clzll(m)));
            }
            Bucket& b = bucket[top_sup];
            if (!b.sorted) {
                n_sorted += b.v.size();
                std::sort(b.v.begin(), b.v.end(), cmp);  // (a parallel merge sort on the host pool measured no faster at c4)
                b.sorted = true;
            }
            return b;
        }
        // in a sorted bucket: the side heap's top is the maximum
        bool side_first(const Bucket& b) const { return !b.side.empty() && (b.v.empty() || cmp(b.v.back(), b.side.front())); }
        const HeapEnt& top() {
            Bucket& b = settle();
            return side_first(b) ? b.side.front() : b.v.back();
        }
        void pop() {
            Bucket& b = settle();
            ++n_popped;
            if (side_first(b)) {
                std::pop_heap(b.side.begin(), b.side.end(), cmp);
                b.side.pop_back();
            } else {
                b.v.pop_back();
            }
            if (b.empty()) {
                occ[top_sup >> 6] &= ~(1ull << (top_sup & 63u));
                std::vector<HeapEnt>().swap(b.v);
                std::vector<HeapEnt>().swap(b.side);
                b.sorted = false;
            }
            --n;
        }
        void drop_below(uint32_t ms) {
            for (; floor < ms && floor < bucket.size(); ++floor) {
                Bucket& b = bucket[floor];
                n -= b.v.size() + b.side.size();
                std::vector<HeapEnt>().swap(b.v);
                std::vector<HeapEnt>().swap(b.side);
                b.sorted = false;
                occ[floor >> 6] &= ~(1ull << (floor & 63u));
            }
            if (floor < ms) floor = ms;
        }
    };
    std::priority_queue<HeapEnt, std::vector<HeapEnt>, MinFirst> krules;
    CandQueue cand;
    XIntern xin;

    Replay(int32_t k_, double mc) : k(k_), minconf(mc), krules(MinFirst{&st}), cand(MaxFirst{&st}) {}

    // X = X(src) + ax, Y = Y(src) + ay (src == nullptr: X = {ax}, Y = {ay})
    Rule* derive(const Rule* src, uint32_t ax, uint32_t ay, uint32_t sup, uint32_t nX) {
        const uint32_t nx0 = src ? src->nx : 0u, ny0 = src ? src->ny : 0u;
        const uint32_t mx = nx0 + (ax != kNone), my = ny0 + (ay != kNone);
        if (mx >= uint32_t(kMaxSide) || my >= uint32_t(kMaxSide))
            throw Error(FSM_ELIMIT, "TSR: rule side exceeds " + std::to_string(kMaxSide - 1) + " items");
        Rule& r = st.new_rule();
        uint32_t* d = st.new_items(mx + my);
        r.it = d;
        const uint32_t* si = src ? src->it : nullptr;
        for (uint32_t q = 0; q < nx0; ++q) *d++ = si[q];
        if (ax != kNone) *d++ = ax;
        for (uint32_t q = 0; q < ny0; ++q) *d++ = si[nx0 + q];
        if (ay != kNone) *d++ = ay;
        r.nx = uint16_t(mx);
        r.ny = uint16_t(my);
        r.sup = sup;
        r.nX = nX;
        r.conf = double(sup) / double(nX);
        const uint32_t* x = st.X(&r);
        r.k1 = uint64_t(sup) << 32 | uint64_t(mx) << 16 | uint64_t(my);
        r.k2 = uint64_t(x[0]) << 32 | (mx > 1 ? x[1] : x[mx]);
        // a left extension's X is interned when the rule is first launched (most derived rules
        // never are); a right extension shares its parent's X
        r.xid = !src ? ax : (ax != kNone ? kNone : src->xid);
        r.pxid = src ? src->xid : 0u;
        if (src && src->loff != kNoList) {  // the parent's kept rows: the child's domain probes only pc there
            r.ploff = src->loff;
            r.pn = src->ln;
            r.pc = ax != kNone ? ax : ay;
            r.pleft = ax != kNone;
        }
        return &r;
    }
    // AlgoTopSeqRules.save
    void save(Rule* r) {
        krules.push(HeapEnt{r->k1, r->k2, r});
        if (int64_t(krules.size()) > k) {
            if (r->sup > minsup) {
                do {
                    if (krules.empty()) break;
                    krules.pop();
                } while (int64_t(krules.size()) > k);
            }
            minsup = krules.top().r->sup;
            cand.drop_below(minsup);
        }
    }
    void reg(Rule* r, bool lr) {
        r->expandLR = lr;
        cand.push(HeapEnt{r->k1, r->k2, r});
    }
};

}  // namespace

void tsr_upload(fsm_ctx* ctx, fsm_db* db) {
    const FlatTsr& f = db->tsr;
    hipStream_t s = ctx->stream;
    auto d = std::make_unique<TsrDevDB>();
    d->N = f.total;
    d->E = int64_t(f.ent_item.size());
    d->U = int64_t(f.item_val.size());
    d->row_off.alloc(f.row_off.size() * 4);
    d->item.alloc(size_t(std::max<int64_t>(d->E, 1)) * 4);
    d->first.alloc(size_t(std::max<int64_t>(d->E, 1)) * 4);
    d->last.alloc(size_t(std::max<int64_t>(d->E, 1)) * 4);
    FSM_HIP(hipMemcpyAsync(d->row_off.p, f.row_off.data(), f.row_off.size() * 4, hipMemcpyHostToDevice, s));
    if (d->E) {
        FSM_HIP(hipMemcpyAsync(d->item.p, f.ent_item.data(), size_t(d->E) * 4, hipMemcpyHostToDevice, s));
        FSM_HIP(hipMemcpyAsync(d->first.p, f.ent_first.data(), size_t(d->E) * 4, hipMemcpyHostToDevice, s));
        FSM_HIP(hipMemcpyAsync(d->last.p, f.ent_last.data(), size_t(d->E) * 4, hipMemcpyHostToDevice, s));
    }
    tsr_finish(ctx, d.get());
    db->tsr_dev = d.release();
}

// The vertical transpose (item -> sids), the sid bitmaps and the item
// supports from the horizontal rows already in HBM (host upload or K0).
void tsr_finish(fsm_ctx* ctx, TsrDevDB* d) {
    hipStream_t s = ctx->stream;
    // vertical transpose on the device (K0)
    DevBuf cnt(size_t(std::max<int64_t>(d->U, 1)) * 4), cursor(size_t(std::max<int64_t>(d->U, 1)) * 4);
    d->vert_off.alloc(size_t(d->U + 1) * 8);
    d->vert_sid.alloc(size_t(std::max<int64_t>(d->E, 1)) * 4);
    d->vert_item.alloc(size_t(std::max<int64_t>(d->E, 1)) * 4);
    FSM_HIP(hipMemsetAsync(cnt.p, 0, size_t(d->U) * 4, s));
    FSM_HIP(hipMemsetAsync(cursor.p, 0, size_t(d->U) * 4, s));
    if (d->E) {
        const unsigned g = unsigned(std::min<int64_t>((d->E + kBlock - 1) / kBlock, 8192));
        hipLaunchKernelGGL(k_vcount, dim3(g), dim3(kBlock), 0, s, d->item.as<uint32_t>(), uint64_t(d->E),
                           cnt.as<uint32_t>());
        FSM_LAUNCHED("k_vcount", s);
    }
    scan_exclusive(cnt.as<uint32_t>(), d->vert_off.as<uint64_t>(), size_t(d->U), s);
    if (d->N) {
        hipLaunchKernelGGL(k_vscatter, dim3(unsigned((d->N + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                           d->row_off.as<uint32_t>(), d->item.as<uint32_t>(), uint64_t(d->N),
                           d->vert_off.as<uint64_t>(), cursor.as<uint32_t>(), d->vert_sid.as<uint32_t>(),
                           d->vert_item.as<uint32_t>());
        FSM_LAUNCHED("k_vscatter", s);
    }
    // sid bitmaps for the expansion domain (skipped when they would take more
    // than a quarter of the free HBM; FSM_TSR_BITMAP=0 forces the list path)
    d->NW = uint32_t((d->N + 127) / 128 * 4);  // a multiple of 4 words: k_exp_domain reads 16-byte words
    const uint64_t bm_bytes = uint64_t(d->U) * d->NW * 4;
    size_t free_b = 0, total_b = 0;
    FSM_HIP(hipMemGetInfo(&free_b, &total_b));
    const char* bm_env = std::getenv("FSM_TSR_BITMAP");
    if (d->E && bm_bytes <= free_b / (4 * uint64_t(ctx->dev_share)) && !(bm_env && bm_env[0] == '0')) {
        d->bm.alloc(bm_bytes);
        FSM_HIP(hipMemsetAsync(d->bm.p, 0, bm_bytes, s));
        const unsigned g = unsigned(std::min<int64_t>((d->E + kBlock - 1) / kBlock, 8192));
        hipLaunchKernelGGL(k_bitmap_build, dim3(g), dim3(kBlock), 0, s, d->vert_sid.as<uint32_t>(),
                           d->vert_item.as<uint32_t>(), uint64_t(d->E), d->NW, d->bm.as<uint32_t>());
        FSM_LAUNCHED("k_bitmap_build", s);
    }
    d->sup.resize(size_t(d->U));
    if (d->U) FSM_HIP(hipMemcpyAsync(d->sup.data(), cnt.p, size_t(d->U) * 4, hipMemcpyDeviceToHost, s));
    FSM_HIP(hipStreamSynchronize(s));
}

void tsr_release(fsm_db* db) {
    delete db->tsr_dev;
    db->tsr_dev = nullptr;
}

void tsr_mine(fsm_ctx* ctx, fsm_db* db, int32_t k, double minconf, fsm_rules** out) {
    const double t0 = now_ms();
    TsrDevDB* d = db->tsr_dev;
    hipStream_t s = ctx->stream;
    const uint32_t U = uint32_t(d->U);
    Replay rp{k, minconf};
    rp.xin.init(U);
    std::vector<uint64_t> voff(size_t(U) + 1);
    FSM_HIP(hipMemcpyAsync(voff.data(), d->vert_off.p, (size_t(U) + 1) * 8, hipMemcpyDeviceToHost, s));
    DevBuf d_sup(size_t(std::max<uint32_t>(U, 1)) * 4);
    FSM_HIP(hipMemcpyAsync(d_sup.p, d->sup.data(), size_t(U) * 4, hipMemcpyHostToDevice, s));
    FSM_HIP(hipStreamSynchronize(s));
    const std::vector<uint32_t>& sup = d->sup;

    // ---------------- pair phase (i ascending, j > i; IJ then JI)
    // nranks > 1: each rank counts the pairs of its own sequence range; the candidate
    // keys are exchanged and their partial counts summed.  The
    // expansions then run on every rank alike (replicated, no exchange).  A failure
    // on one rank is agreed on before each collective, so no peer is left blocked.
    Comm* comm = ctx->comm;
    const bool shard = comm && comm->nranks() > 1;
    Agreement agr;
    agr.comm = shard ? comm : nullptr;
    agr.what = "TSR";
    const int R = shard ? comm->nranks() : 1;
    const uint32_t slo = shard ? uint32_t(uint64_t(d->N) * uint64_t(comm->rank()) / uint64_t(R)) : 0u;
    const uint32_t shi = shard ? uint32_t(uint64_t(d->N) * uint64_t(comm->rank() + 1) / uint64_t(R))
                               : uint32_t(d->N);
    uint64_t rp_pair_exchanged = 0;  // union keys exchanged (verbose)
    uint32_t nb_items = 16;
    // the batch grows while a batch's candidate records stay below pair_recs and
    // shrinks above 4 x pair_recs (FSM_TSR_PAIR_RECS lowers it: test hook for the
    // sharded batch agreement)
    const uint64_t pair_recs = [] {
        const char* v = std::getenv("FSM_TSR_PAIR_RECS");
        return v ? std::clamp<uint64_t>(std::strtoull(v, nullptr, 10), 1, uint64_t(1) << 30) : uint64_t(1) << 20;
    }();
    const uint64_t scr_cap_items = std::max<uint64_t>(1, (uint64_t(256) << 20) / (uint64_t(std::max<uint32_t>(U, 1)) * 8));
    DevBuf scr;
    uint64_t scr_items = 0;
    std::vector<PairRec> recs;
    for (uint32_t a = 0; a < U;) {
        const uint32_t t = rp.minsup;
        const uint32_t nb = uint32_t(std::min<uint64_t>({uint64_t(nb_items), uint64_t(U - a), scr_cap_items}));
        const uint32_t b = a + nb;
        // compaction threshold: t, or ceil(t / R) for a rank's partial counts (a pair whose
        // total reaches t has a partial >= t / R on some rank)
        const uint32_t tq = shard ? (t + uint32_t(R) - 1) / uint32_t(R) : t;
        const unsigned grid = unsigned((uint64_t(nb) * 64 + kBlock - 1) / kBlock);
        std::vector<uint64_t> hoff(size_t(nb) + 1, 0);
        std::vector<PairRec> mine;
        uint64_t nrec = 0;
        // this rank's counts of the batch (rank-local work: deferred on failure when sharded)
        agr.run([&] {
            if (shard) agr.maybe_inject("pairs");
            if (scr_items < nb) {
                scr.alloc(uint64_t(nb) * U * 8);
                FSM_HIP(hipMemsetAsync(scr.p, 0, uint64_t(nb) * U * 8, s));
                scr_items = nb;
            }
            const uint64_t v0 = voff[a], v1 = voff[b];
            if (v1 > v0) {
                hipLaunchKernelGGL(k_pairs, dim3(unsigned((v1 - v0 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                                   d->vert_sid.as<uint32_t>(), d->vert_item.as<uint32_t>(), v0, v1, a, U, t, slo, shi,
                                   d_sup.as<uint32_t>(), d->row_off.as<uint32_t>(), d->item.as<uint32_t>(),
                                   d->first.as<uint32_t>(), d->last.as<uint32_t>(), scr.as<uint32_t>());
                FSM_LAUNCHED("k_pairs", s);
            }
            DevBuf rowcnt(size_t(nb) * 4 + 4), rowoff((size_t(nb) + 1) * 8);
            hipLaunchKernelGGL(k_pairs_compact, dim3(grid), dim3(kBlock), 0, s, scr.as<uint32_t>(), a, nb, U, tq,
                               rowcnt.as<uint32_t>(), rowoff.as<uint64_t>(), (PairRec*)nullptr, 0);
            FSM_LAUNCHED("k_pairs_compact", s);
            scan_exclusive(rowcnt.as<uint32_t>(), rowoff.as<uint64_t>(), nb, s);
            FSM_HIP(hipMemcpyAsync(hoff.data(), rowoff.p, (size_t(nb) + 1) * 8, hipMemcpyDeviceToHost, s));
            FSM_HIP(hipStreamSynchronize(s));
            nrec = hoff[nb];
            DevBuf d_recs(std::max<uint64_t>(nrec, 1) * sizeof(PairRec));
            // unsharded: the compaction also re-zeroes the counters it visits; sharded: the
            // counters are read again for the union's partials
            hipLaunchKernelGGL(k_pairs_compact, dim3(grid), dim3(kBlock), 0, s, scr.as<uint32_t>(), a, nb, U, tq,
                               rowcnt.as<uint32_t>(), rowoff.as<uint64_t>(), d_recs.as<PairRec>(), shard ? 0 : 1);
            FSM_LAUNCHED("k_pairs_compact", s);
            std::vector<PairRec>& dst = shard ? mine : recs;
            dst.resize(nrec);
            if (nrec) FSM_HIP(hipMemcpyAsync(dst.data(), d_recs.p, nrec * sizeof(PairRec), hipMemcpyDeviceToHost, s));
            FSM_HIP(hipStreamSynchronize(s));
        });
        uint64_t nadapt = nrec;  // drives the next batch size (must be alike on every rank)
        if (shard) {
            // candidate keys of this rank -> union over ranks -> every rank's partials of
            // the union summed -> the exact counts, kept at t like the one-rank compaction
            agr.agree(s);
            std::vector<uint8_t> blob(mine.size() * 8);
            for (size_t q = 0; q < mine.size(); ++q) {
                std::memcpy(blob.data() + q * 8, &mine[q].i, 4);
                std::memcpy(blob.data() + q * 8 + 4, &mine[q].j, 4);
            }
            std::vector<size_t> sizes;
            const std::vector<uint8_t> all = comm->gather_blobs(blob, sizes, s);
            std::vector<uint2> keys(all.size() / 8);
            for (size_t q = 0; q < keys.size(); ++q) std::memcpy(&keys[q], all.data() + q * 8, 8);
            std::sort(keys.begin(), keys.end(),
                      [](const uint2& x, const uint2& y) { return x.x != y.x ? x.x < y.x : x.y < y.y; });
            keys.erase(std::unique(keys.begin(), keys.end(),
                                   [](const uint2& x, const uint2& y) { return x.x == y.x && x.y == y.y; }),
                       keys.end());
            std::vector<uint32_t> part(keys.size() * 2, 0u);
            agr.run([&] {
                for (const uint2& kk : keys)  // every rank batched [a, b) alike
                    if (kk.x < a || kk.x >= b || kk.y >= U)
                        throw Error(FSM_EDEVICE, "TSR sharded pair phase: exchanged key outside the batch");
                if (!keys.empty()) {
                    DevBuf d_keys(keys.size() * 8), d_part(keys.size() * 8);
                    FSM_HIP(hipMemcpyAsync(d_keys.p, keys.data(), keys.size() * 8, hipMemcpyHostToDevice, s));
                    hipLaunchKernelGGL(k_pairs_gather, dim3(unsigned((keys.size() + kBlock - 1) / kBlock)),
                                       dim3(kBlock), 0, s, scr.as<uint32_t>(), a, U, d_keys.as<uint2>(),
                                       uint32_t(keys.size()), d_part.as<uint32_t>());
                    FSM_LAUNCHED("k_pairs_gather", s);
                    FSM_HIP(hipMemcpyAsync(part.data(), d_part.p, keys.size() * 8, hipMemcpyDeviceToHost, s));
                }
                FSM_HIP(hipMemsetAsync(scr.p, 0, uint64_t(nb) * U * 8, s));
                FSM_HIP(hipStreamSynchronize(s));
            });
            agr.agree(s);
            comm->host_allreduce_u32(part.data(), part.size(), s);
            recs.clear();
            std::fill(hoff.begin(), hoff.end(), 0);
            for (size_t q = 0; q < keys.size(); ++q) {
                const uint32_t ij = part[2 * q], ji = part[2 * q + 1];
                if (ij < t && ji < t) continue;
                recs.push_back(PairRec{keys[q].x, keys[q].y, ij, ji});
                hoff[keys[q].x - a + 1] += 1;
            }
            for (uint32_t g = 0; g < nb; ++g) hoff[g + 1] += hoff[g];
            rp_pair_exchanged += keys.size();
            nadapt = keys.size();  // the union: the same number on every rank
        }
        for (uint32_t g = 0; g < nb; ++g) {
            const uint32_t i = a + g;
            if (sup[i] < rp.minsup) continue;
            for (uint64_t q = hoff[g]; q < hoff[g + 1]; ++q) {
                const PairRec& pr = recs[q];
                const uint32_t j = pr.j;
                if (sup[j] < rp.minsup) continue;
                if (pr.ij >= rp.minsup) {
                    Rule* r = rp.derive(nullptr, i, j, pr.ij, sup[i]);
                    if (r->conf >= minconf) rp.save(r);
                    rp.reg(r, true);
                }
                if (pr.ji >= rp.minsup) {
                    Rule* r = rp.derive(nullptr, j, i, pr.ji, sup[j]);
                    if (r->conf >= minconf) rp.save(r);
                    rp.reg(r, true);
                }
            }
        }
        if (nadapt < pair_recs) nb_items = std::min<uint32_t>(nb_items * 2, 4096);
        else if (nadapt > 4 * pair_recs && nb_items > 1) nb_items /= 2;
        a = b;
    }
    scr.release();
    // The expansions see only the items that can still be in a rule: support >=
    // the pair phase's minsup, which only rises from here (K "kept" items).
    std::vector<uint32_t> kept_items;
    for (uint32_t c = 0; c < U; ++c)
        if (sup[c] >= rp.minsup) kept_items.push_back(c);
    const uint32_t K = uint32_t(kept_items.size());
    const uint64_t N = uint64_t(d->N);
    // bitmap path: sid bitmaps built, K <= kMaxKids, itemset indexes < 2^16 (packed rows);
    // FSM_TSR_MAX_KIDS / FSM_TSR_MAX_POS lower both caps (test hooks: the list path, taken up
    // front or after the rows were packed)
    const uint32_t max_kids = [] {
        const char* v = std::getenv("FSM_TSR_MAX_KIDS");
        return v ? std::min<uint32_t>(uint32_t(std::strtoul(v, nullptr, 10)), kMaxKids) : kMaxKids;
    }();
    const uint32_t max_pos = [] {
        const char* v = std::getenv("FSM_TSR_MAX_POS");
        return v ? std::min<uint32_t>(uint32_t(std::strtoul(v, nullptr, 10)), 0xFFFFu) : 0xFFFFu;
    }();
    bool use_bm = d->bm.p != nullptr && K > 0 && K <= max_kids;
    std::vector<uint32_t> h_kid_of;  // bitmap path: item -> kid (host copy)
    DevBuf k_off, k_item, k_first, k_last, k_sup;  // list path rows (SoA)
    DevBuf k_ent, d_kidof, d_kept, d_ksup;  // bitmap path rows (packed) and kid tables
    DevBuf d_rdir, d_kvoff, d_vfl;          // bitmap path: rank directories and vertical entries of the kids
    uint64_t E2 = 0;
    const unsigned rows_grid = unsigned(std::min<uint64_t>((N * 64 + kBlock - 1) / kBlock, 65536));
    if (use_bm) {
        std::vector<uint32_t>& kid_of = h_kid_of;
        kid_of.assign(U, kNone);
        std::vector<uint32_t> ksup(K);
        for (uint32_t q = 0; q < K; ++q) {
            kid_of[kept_items[q]] = q;
            ksup[q] = sup[kept_items[q]];
        }
        d_kidof.alloc(size_t(std::max<uint32_t>(U, 1)) * 4);
        d_kept.alloc(size_t(K) * 4);
        d_ksup.alloc(size_t(K) * 4);
        FSM_HIP(hipMemcpyAsync(d_kidof.p, kid_of.data(), size_t(U) * 4, hipMemcpyHostToDevice, s));
        FSM_HIP(hipMemcpyAsync(d_kept.p, kept_items.data(), size_t(K) * 4, hipMemcpyHostToDevice, s));
        FSM_HIP(hipMemcpyAsync(d_ksup.p, ksup.data(), size_t(K) * 4, hipMemcpyHostToDevice, s));
        DevBuf rc(std::max<uint64_t>(N, 1) * 4), off64((N + 1) * 8), mpos(4);
        FSM_HIP(hipMemsetAsync(mpos.p, 0, 4, s));
        if (N) {
            hipLaunchKernelGGL(k_rows_pack, dim3(rows_grid), dim3(kBlock), 0, s, d->row_off.as<uint32_t>(),
                               d->item.as<uint32_t>(), d->first.as<uint32_t>(), d->last.as<uint32_t>(),
                               d_kidof.as<uint32_t>(), N, rc.as<uint32_t>(), mpos.as<uint32_t>(),
                               (const uint64_t*)nullptr, (uint2*)nullptr);
            FSM_LAUNCHED("k_rows_pack", s);
        }
        scan_exclusive(rc.as<uint32_t>(), off64.as<uint64_t>(), N, s);
        uint32_t maxpos = 0;
        FSM_HIP(hipMemcpyAsync(&E2, off64.as<uint64_t>() + N, 8, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipMemcpyAsync(&maxpos, mpos.p, 4, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
        if (maxpos > max_pos || E2 >= kNone) {
            use_bm = false;  // an itemset index past 2^16: the list path takes it
        } else {
            k_off.alloc((N + 1) * 4);
            k_ent.alloc(std::max<uint64_t>(E2, 1) * 8);
            hipLaunchKernelGGL(k_off32, dim3(unsigned(std::min<uint64_t>((N + 256) / 256, 4096))), dim3(256), 0, s,
                               off64.as<uint64_t>(), N, k_off.as<uint32_t>());
            FSM_LAUNCHED("k_off32", s);
            if (N) {
                hipLaunchKernelGGL(k_rows_pack, dim3(rows_grid), dim3(kBlock), 0, s, d->row_off.as<uint32_t>(),
                                   d->item.as<uint32_t>(), d->first.as<uint32_t>(), d->last.as<uint32_t>(),
                                   d_kidof.as<uint32_t>(), N, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                   off64.as<uint64_t>(), k_ent.as<uint2>());
                FSM_LAUNCHED("k_rows_pack", s);
            }
            // the kept items' rank directories and vertical entries (k_exp_domain's probes)
            std::vector<uint32_t> kvoff(size_t(K) + 1, 0);
            for (uint32_t q = 0; q < K; ++q) kvoff[q + 1] = kvoff[q] + ksup[q];
            if (kvoff[K] != E2) throw Error(FSM_EDEVICE, "TSR: kept row entries differ from the kept supports");
            d_kvoff.alloc((size_t(K) + 1) * 4);
            FSM_HIP(hipMemcpyAsync(d_kvoff.p, kvoff.data(), (size_t(K) + 1) * 4, hipMemcpyHostToDevice, s));
            d_rdir.alloc(std::max<size_t>(size_t(K) * (d->NW / 4) * 4, 4));
            hipLaunchKernelGGL(k_rank_dir, dim3(K), dim3(kBlock), 0, s, d->bm.as<uint32_t>(), d->NW,
                               d_kept.as<uint32_t>(), d_rdir.as<uint32_t>());
            FSM_LAUNCHED("k_rank_dir", s);
            d_vfl.alloc(std::max<uint64_t>(E2, 1) * 8);
            if (N) {
                hipLaunchKernelGGL(k_vfl, dim3(unsigned(std::min<uint64_t>((N + kBlock - 1) / kBlock, 65536))),
                                   dim3(kBlock), 0, s, k_off.as<uint32_t>(), k_ent.as<uint2>(), uint32_t(N),
                                   d->bm.as<uint32_t>(), d->NW, d_kept.as<uint32_t>(), d_rdir.as<uint32_t>(),
                                   d_kvoff.as<uint32_t>(), d_vfl.as<uint2>());
                FSM_LAUNCHED("k_vfl", s);
            }
            FSM_HIP(hipStreamSynchronize(s));
        }
    }
    if (!use_bm) {  // list path: rows restricted to the kept items, SoA with each entry's item support
        DevBuf rc(std::max<uint64_t>(N, 1) * 4), off64((N + 1) * 8);
        if (N) {
            hipLaunchKernelGGL(k_rows_keep, dim3(rows_grid), dim3(kBlock), 0, s, d->row_off.as<uint32_t>(),
                               d->item.as<uint32_t>(), d->first.as<uint32_t>(), d->last.as<uint32_t>(),
                               d_sup.as<uint32_t>(), rp.minsup, N, rc.as<uint32_t>(), (const uint64_t*)nullptr,
                               (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr);
            FSM_LAUNCHED("k_rows_keep", s);
        }
        scan_exclusive(rc.as<uint32_t>(), off64.as<uint64_t>(), N, s);
        FSM_HIP(hipMemcpyAsync(&E2, off64.as<uint64_t>() + N, 8, hipMemcpyDeviceToHost, s));
        FSM_HIP(hipStreamSynchronize(s));
        k_off.alloc((N + 1) * 4);
        k_item.alloc(std::max<uint64_t>(E2, 1) * 4);
        k_first.alloc(std::max<uint64_t>(E2, 1) * 4);
        k_last.alloc(std::max<uint64_t>(E2, 1) * 4);
        k_sup.alloc(std::max<uint64_t>(E2, 1) * 4);
        hipLaunchKernelGGL(k_off32, dim3(unsigned(std::min<uint64_t>((N + 256) / 256, 4096))), dim3(256), 0, s,
                           off64.as<uint64_t>(), N, k_off.as<uint32_t>());
        FSM_LAUNCHED("k_off32", s);
        if (N) {
            hipLaunchKernelGGL(k_rows_keep, dim3(rows_grid), dim3(kBlock), 0, s, d->row_off.as<uint32_t>(),
                               d->item.as<uint32_t>(), d->first.as<uint32_t>(), d->last.as<uint32_t>(),
                               d_sup.as<uint32_t>(), rp.minsup, N, (uint32_t*)nullptr, off64.as<uint64_t>(),
                               k_item.as<uint32_t>(), k_first.as<uint32_t>(), k_last.as<uint32_t>(),
                               k_sup.as<uint32_t>());
            FSM_LAUNCHED("k_rows_keep", s);
        }
        FSM_HIP(hipStreamSynchronize(s));
    }
    const double t1 = now_ms();
    if (ctx->opts.verbose)
        std::fprintf(stderr, "[fsm tsr] pair phase %.0f ms: minsup %u, candidates %zu, rules %zu, kept items %u, "
                     "row entries %llu, %s path (ranks %d, keys exchanged %llu)\n",
                     t1 - t0, rp.minsup, rp.cand.size(), rp.krules.size(), K, (unsigned long long)E2,
                     use_bm ? "bitmap" : "list", R, (unsigned long long)rp_pair_exchanged);

    // ---------------- expansions
    // Batched speculation, committed in the exact sequential order: the next
    // kExpBatch candidates (in heap order) are expanded together on the GPU;
    // they are committed one by one while each is still the heap maximum; when
    // a newly registered rule outranks the next one, the rest go back to the
    // heap with their results cached (results are minsup-independent supersets,
    // re-filtered against the current minsup at commit), so no expansion is
    // computed twice and the outcome equals the one-at-a-time replay.
    // Rules per launch (FSM_TSR_BATCH overrides, for tuning).  Wide batches halve the launches
    // (round trips) where supports are coarse: at c4 (pair-phase minsup in the hundreds) every
    // speculated rule is committed, and 768 rules per launch take 12,973 launches down to 7,179
    // (2.76 -> 2.39 s).  Where supports are a few units (the 5K prefix ends at minsup 2) a wide
    // batch's lowest rules sit at the threshold, their speculated children mostly fall below the
    // rising minsup (1.45M speculated, 0.22M committed) and the launches multiply (2.6K -> 15K):
    // those mines keep kExpBatch.
    const uint32_t B = [&] {
        const char* v = std::getenv("FSM_TSR_BATCH");
        if (v) return uint32_t(std::clamp<long>(std::strtol(v, nullptr, 10), 1, kMaxBatch));
        return uint32_t(rp.minsup >= kWideMinsup ? kExpBatchWide : kExpBatch);
    }();
    const uint64_t SU = uint64_t(B) * std::max<uint32_t>(U, 1);
    const size_t kSidesB = B * sizeof(Side), kOffB = (B + 1) * 8;
    // records per slot: at most one per candidate item (bitmap path: the kept items)
    const uint32_t ecap = use_bm ? std::max<uint32_t>(K, 1) : std::max<uint32_t>(U, 1);
    // bitmap path geometry: LDS histogram passes of KP kids; dense partial rows of
    // 2 * KP counters per expansion block, at most max_blocks blocks per launch
    const uint32_t pass_kids = [] {  // FSM_TSR_PASS_KIDS lowers the pass width (test hook: several passes)
        const char* v = std::getenv("FSM_TSR_PASS_KIDS");
        return v ? std::clamp<uint32_t>(uint32_t(std::strtoul(v, nullptr, 10)), 1, kPassKids) : kPassKids;
    }();
    const uint32_t KP = use_bm ? std::min<uint32_t>(K, pass_kids) : 0u;
    const uint32_t P = use_bm ? (K + KP - 1) / KP : 0u;
    const uint64_t row_bytes = uint64_t(P) * 2 * KP * 4;
    const uint64_t part_mb = [] {  // FSM_TSR_PART_MB: partial-row budget per launch (tuning)
        const char* v = std::getenv("FSM_TSR_PART_MB");
        return v ? std::clamp<uint64_t>(std::strtoull(v, nullptr, 10), 1, 4096) : uint64_t(32);
    }();
    const uint64_t part_budget = std::max<uint64_t>(part_mb << 20, uint64_t(B) * row_bytes);
    const uint64_t max_blocks = use_bm ? part_budget / row_bytes : 0;
    const size_t xlds = use_bm ? (size_t(2) * KP + (K + 15) / 16) * 4 : 0;
    // Two sets of launch buffers, so the GPU runs one launch while the host commits
    // the results of the previous one.  A set holds the rule descriptors (pinned
    // stage + device copy, one H2D copy per launch), the per-slot control blocks,
    // the histograms (list path: per-slot HBM arrays; bitmap path: per-block partial
    // rows and the domain lists), the results (mapped pinned host memory, at most
    // ecap records per slot) and its own events (completion, per-kernel timing).
    const TsrGrid grid;
    // Sharded TSR (nranks > 1, bitmap path): each launch's rule slots are split over the
    // ranks and the slots' results all-gathered once per launch (finish); the replay
    // stays replicated and deterministic.  FSM_TSR_SHARD=0 replicates the expansions.
    // FSM_TSR_DOMAIN=bitmap keeps every domain on the whole-bitmap AND (tests, A/B)
    const int dom_mode = [] {  // 0 auto (by the rarest item's list length), 1 every slot bitmap, 2 every slot list
        const char* v = std::getenv("FSM_TSR_DOMAIN");
        return !v ? 0 : (!std::strcmp(v, "bitmap") ? 1 : (!std::strcmp(v, "list") ? 2 : 0));
    }();
    const bool shard_exp = shard && use_bm && [] {
        const char* v = std::getenv("FSM_TSR_SHARD");
        return !(v && v[0] == '0');
    }();
    // Kept-row lists (bitmap path, unsharded): an expansion keeps the rows where its rule holds
    // with a non-empty suffix (sid, firstX | lastY, max X / max Y positions) in a per-mine device
    // arena; a child rule's domain is then its parent's list with only the added item probed
    // (a child holds only where its parent does).  Rules whose parent list did not fit the arena
    // probe the whole bitmap AND.  FSM_TSR_PLIST=0 turns the lists off.
    // A launch is sharded only when its expected domain (sum of 2 sup + 1 over its rules) reaches
    // FSM_TSR_SHARD_MIN (default 256K sids: about 60 us of kernels at c4, the break-even of a
    // per-launch gather); smaller launches run replicated on every rank (no gather), so the many
    // small speculation launches of a c4-sized mine cost no exchange
    const uint64_t shard_min = [] {
        const char* v = std::getenv("FSM_TSR_SHARD_MIN");
        return v ? std::strtoull(v, nullptr, 10) : uint64_t(1) << 18;
    }();
    // (the lists are rank-local: a rank keeps the lists of the slots it expanded, a child of
    // another rank's slot probes the bitmaps; the counts are the same either way)
    const bool plist = use_bm && [] {
        const char* v = std::getenv("FSM_TSR_PLIST");
        return !(v && v[0] == '0');
    }();
    // The arena is a ring: a launch writes its rules' lists (each at most the rule's support)
    // at the head, at most acap / (4 nsets) entries (else it keeps none); a child reads its
    // parent's list only while it lies within acap / 2 of the head.  A launch may stay in
    // flight (its set not yet finished by the replay) while later launches advance the head,
    // so each set records the oldest ring position it reads or writes (ExpSet::amin), and a
    // launch that would overwrite that position finishes the set first (launch()).
    DevBuf arena;
    uint64_t acap = 0;   // arena entries (16 B)
    uint64_t ahead = 0;  // the ring's head (entries written, monotonic; a list's position mod acap)
    if (plist) {
        size_t fr = 0, tot = 0;
        FSM_HIP(hipMemGetInfo(&fr, &tot));
        // lists for about the whole mine: the rows where a rule holds summed over the expansions
        // reach a few thousand per sequence (c4: 2.0 G entries)
        acap = std::min<uint64_t>({fr / (4 * uint64_t(ctx->dev_share)), uint64_t(64) << 30,
                                   std::max<uint64_t>(uint64_t(64) << 20, uint64_t(d->NW) * 32 * 4096 * sizeof(uint4))}) /
               sizeof(uint4);
        if (const char* v = std::getenv("FSM_TSR_ARENA_MB"))  // (fractions of a MiB: tests)
            acap = uint64_t(std::strtod(v, nullptr) * double(1u << 20)) / sizeof(uint4);
        if (acap) arena.alloc(acap * sizeof(uint4));
    }
    // a child reads its parent's list while it lies within this many entries of the head
    // (16/16: while no later write has reached it yet): acap / 2 by default, which keeps every
    // list a launch in flight reads clear of the later launches' writes;
    // FSM_TSR_PLIST_WINDOW=<sixteenths of the ring> (tests: 16 makes the in-flight guard below
    // fire, its waits counted in fsm_stats.tsr_ring_waits)
    const uint64_t plist_window = [&] {
        const char* v = std::getenv("FSM_TSR_PLIST_WINDOW");
        return acap / 16 * uint64_t(v ? std::clamp(std::atoi(v), 1, 16) : 8);
    }();
    // |sids(X u {c})| memo (bitmap path; FSM_TSR_DLMEMO=0 turns it off): zeroed once per mine
    DevBuf memo_buf;
    DlMemo memo{nullptr, 0u};
    if (use_bm && [] { const char* v = std::getenv("FSM_TSR_DLMEMO"); return !(v && v[0] == '0'); }()) {
        // 2^24 entries (256 MiB); FSM_TSR_DLMEMO_LOG2 (tests: a tiny table fills, probes run out)
        const char* lv = std::getenv("FSM_TSR_DLMEMO_LOG2");
        const uint32_t ent = 1u << (lv ? std::clamp(std::atoi(lv), 4, 28) : 24);
        memo_buf.alloc(size_t(ent) * sizeof(uint4));
        FSM_HIP(hipMemsetAsync(memo_buf.p, 0, size_t(ent) * sizeof(uint4), s));
        FSM_HIP(hipStreamSynchronize(s));  // (the launches run on the sets' own streams)
        memo = DlMemo{memo_buf.as<uint4>(), ent - 1u};
    }
    struct ExpSet {
        DevBuf TL, DL, TR, seen, list, ctl, d_stage, d_dlw, d_ndlw, part, dom;
        std::unique_ptr<PinnedBuf> stage, pin;
        Side* h_sides = nullptr;
        uint64_t *h_drv = nullptr, *h_wave = nullptr;
        Side* d_sides = nullptr;
        uint64_t *d_drv = nullptr, *d_wave = nullptr;
        ExpHdr *h_hdr = nullptr, *d_hdr = nullptr;
        ExpRec *h_rec = nullptr, *d_rec = nullptr;
        uint32_t *h_rcnt = nullptr, *d_rcnt = nullptr;  // bitmap path: records per reduce block
        std::vector<Rule*> batch;
        std::vector<char> drv_in_x;
        std::vector<uint64_t> kmono;  // bitmap path: each slot's kept-row list (ring position; kNoList: none)
        uint64_t amin = kNoList;      // the oldest ring position the launch reads or writes (kNoList: none)
        bool sharded = false;         // this launch's slots split over the ranks (results gathered)
        uint32_t la = 0, lz = 0;  // slot sharding: this rank's slots [la, lz) of the batch (else all)
        hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};  // 0-4 timing, 5 done
        // the set's own stream: the two sets' launches are independent, so the GPU runs
        // one set's kernels while the other's are in flight
        hipStream_t st = nullptr;
        bool own_stream = false;
        DevBuf alive;          // kid codes for alive_t (each set its own: k_alive never races a launch)
        uint32_t alive_t = 0;  // minsup the set's kid codes were built for
        bool timed = false, busy = false;
        int depth = 0;        // speculation depth of the batch (0: heap batch)
        int64_t seq = 0;      // launch number (the older busy set finishes first)
        uint64_t blocks = 0;  // expansion blocks of the launch
        ~ExpSet() {  // (unwinding: the launch may still be running on buffers about to be freed)
            if (busy && ev[5]) (void)hipEventSynchronize(ev[5]);
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
            if (own_stream && st) {
                (void)hipStreamSynchronize(st);
                (void)hipStreamDestroy(st);
            }
        }
    };
    const int nsets = [] {  // launch sets in flight (FSM_TSR_SETS, 2-4)
        const char* v = std::getenv("FSM_TSR_SETS");
        return v ? std::clamp(std::atoi(v), 2, 4) : kExpSets;
    }();
    std::unique_ptr<ExpSet[]> xs_own(new ExpSet[nsets]);
    ExpSet* const xs = xs_own.get();
    for (int xi = 0; xi < nsets; ++xi) {
        ExpSet& x = xs[xi];
        FSM_HIP(hipStreamCreateWithFlags(&x.st, hipStreamNonBlocking));
        x.own_stream = true;
        if (use_bm) x.alive.alloc(size_t((K + 15) / 16) * 4);
        x.ctl.alloc(B * sizeof(ExpCtl));
        FSM_HIP(hipMemsetAsync(x.ctl.p, 0, B * sizeof(ExpCtl), s));
        if (use_bm) {
            x.part.alloc(max_blocks * row_bytes);
            x.d_dlw.alloc(uint64_t(B) * ecap * sizeof(uint4));
        } else {
            x.TL.alloc(SU * 4);
            x.DL.alloc(SU * 4);
            x.TR.alloc(SU * 4);
            x.seen.alloc(SU * 4);
            x.list.alloc(SU * 4);
            FSM_HIP(hipMemsetAsync(x.TL.p, 0, SU * 4, s));
            FSM_HIP(hipMemsetAsync(x.DL.p, 0, SU * 4, s));
            FSM_HIP(hipMemsetAsync(x.TR.p, 0, SU * 4, s));
            FSM_HIP(hipMemsetAsync(x.seen.p, 0, SU * 4, s));
        }
        x.stage = std::make_unique<PinnedBuf>(kSidesB + 2 * kOffB);
        x.d_stage.alloc(kSidesB + 2 * kOffB);
        // [drv offsets | wave offsets | sides]: a launch copies the offsets and its nb sides
        x.h_drv = static_cast<uint64_t*>(x.stage->host);
        x.h_wave = x.h_drv + (B + 1);
        x.h_sides = reinterpret_cast<Side*>(static_cast<char*>(x.stage->host) + 2 * kOffB);
        x.d_drv = x.d_stage.as<uint64_t>();
        x.d_wave = x.d_drv + (B + 1);
        x.d_sides = reinterpret_cast<Side*>(x.d_stage.as<char>() + 2 * kOffB);
        x.d_ndlw.alloc(16);
        // [headers | records, ecap per slot | bitmap path: reduce region counts, B x P x collect]
        const size_t nrc = use_bm ? size_t(B) * P * grid.collect : 0;
        x.pin = std::make_unique<PinnedBuf>(B * sizeof(ExpHdr) + B * size_t(ecap) * sizeof(ExpRec) + nrc * 4);
        x.h_hdr = static_cast<ExpHdr*>(x.pin->host);
        x.h_rec = reinterpret_cast<ExpRec*>(x.h_hdr + B);
        x.h_rcnt = reinterpret_cast<uint32_t*>(x.h_rec + size_t(B) * ecap);
        x.d_hdr = static_cast<ExpHdr*>(x.pin->dev);
        x.d_rec = reinterpret_cast<ExpRec*>(x.d_hdr + B);
        x.d_rcnt = reinterpret_cast<uint32_t*>(x.d_rec + size_t(B) * ecap);
        for (int q = 0; q < 5; ++q) FSM_HIP(hipEventCreate(&x.ev[q]));
        FSM_HIP(hipEventCreateWithFlags(&x.ev[5], hipEventDisableTiming));
    }
    FSM_HIP(hipStreamSynchronize(s));  // the DB, kid tables and set buffers are ready for the set streams
    // Expansion results of rules not yet committed: slots of a pool (Rule::res; a deque,
    // so slots never move; released slots keep their vectors' capacity for the next
    // rule).  Rules in flight carry their launch set in Rule::inset.
    struct ExpResult {
        std::vector<ExpRec> recs;
        std::vector<Rule*> preL, preR;  // children created (and expanded) ahead of the commit, by record
        Rule* owner = nullptr;
    };
    std::deque<ExpResult> res_pool;
    std::vector<int32_t> res_free;
    size_t res_live = 0;
    auto res_get = [&](Rule* r) -> ExpResult& {
        if (r->res < 0) {
            if (res_free.empty()) {
                res_free.push_back(int32_t(res_pool.size()));
                res_pool.emplace_back();
            }
            r->res = res_free.back();
            res_free.pop_back();
            res_pool[size_t(r->res)].owner = r;
            ++res_live;
        }
        return res_pool[size_t(r->res)];
    };
    auto res_release = [&](Rule* r) {
        ExpResult& e = res_pool[size_t(r->res)];
        e.recs.clear();
        e.preL.clear();
        e.preR.clear();
        e.owner = nullptr;
        res_free.push_back(r->res);
        r->res = -1;
        --res_live;
    };
    std::vector<std::pair<std::vector<Rule*>, int>> spec_todo;  // finished launches whose children to speculate
    // speculated rules committed, and dropped at their parent's commit (verbose)
    int64_t spec_hit = 0, spec_waste = 0;
    int64_t expansions = 0, launches = 0, spec_pushback = 0, gpu_rules = 0;
    double wait_ms = 0;  // host time blocked on the GPU in the expansion loop
    double last_log_ms = now_ms();  // verbose progress line every 20 s
    double prep_ms = 0, post_ms = 0, commit_ms = 0, pop_ms = 0;  // host time split (verbose summary)
    double fill_ms = 0;  // launch prep: descriptor fill (the rest is the HIP calls)

    const uint64_t exp_spb = [] {  // bitmap path: target domain sids per expansion block (FSM_TSR_SPB, tuning)
        const char* v = std::getenv("FSM_TSR_SPB");
        return v ? std::clamp<uint64_t>(std::strtoull(v, nullptr, 10), 1, 1u << 20) : uint64_t(kExpSpb);
    }();
    const uint64_t pl_spb = [] {  // parent-list rows per row block (one probe each: cheaper than a domain sid)
        const char* v = std::getenv("FSM_TSR_PLSPB");
        return v ? std::clamp<uint64_t>(std::strtoull(v, nullptr, 10), 1, 1u << 20) : uint64_t(kExpSpb);
    }();
    // per-kernel device time: every 16th launch records one set of events and reads
    // them back when it finishes (ctx->kstats rows); FSM_TSR_TIME_EVERY=n times every n-th
    // (1: every launch, the bench's roofline mine)
    const int64_t time_every = [] {
        const char* v = std::getenv("FSM_TSR_TIME_EVERY");
        return v ? std::clamp<int64_t>(std::strtoll(v, nullptr, 10), 1, 1 << 20) : int64_t(16);
    }();
    struct Seg {
        double ms = 0;  // over the timed launches
        int64_t n = 0, timed = 0, bytes = 0, survey = 0;  // survey: SURVEY §8(d) TSR units
    } seg[4];  // bitmap path: domain, rows, reduce, k_dl; list path: expansion, -, collect, k_publish
    const char* seg_name[4] = {use_bm ? "k_exp_domain" : "k_expand", use_bm ? "k_exp_rows" : "",
                               use_bm ? "k_expand_reduce" : "k_expand_collect", use_bm ? "k_dl" : "k_publish"};
    int64_t exp_domain = 0, exp_entries = 0, exp_bitmap_bytes = 0, exp_part_bytes = 0;
    int64_t exp_hold = 0, exp_walk = 0;  // domain rows where the rule holds, row entries walked (verbose)
    int64_t exp_plist = 0;               // expansions whose domain came from the parent's kept rows (verbose)
    int64_t ring_waits = 0;              // launches in flight finished early to free their ring positions
    int64_t seq_next = 0;
    // Take in the results of set x (waits for its launch): records sorted into the
    // cache, and its batch queued for child speculation.
    auto finish = [&](ExpSet& x) {
        const double tw0 = now_ms();
        FSM_HIP(hipEventSynchronize(x.ev[5]));
        const double tw1 = now_ms();
        wait_ms += tw1 - tw0;
        x.busy = false;
        for (int q = 0; q < 4; ++q) {
            float ms = 0;
            if (x.timed && hipEventElapsedTime(&ms, x.ev[q], x.ev[q + 1]) == hipSuccess) {
                seg[q].ms += ms;
                seg[q].timed += 1;
            }
            seg[q].n += 1;
        }
        const uint32_t nb = x.lz - x.la;  // the slots expanded here (slot sharding: this rank's share)
        if (use_bm && nb) {
            exp_part_bytes += int64_t(x.blocks * row_bytes);
            seg[1].bytes += int64_t(x.blocks * row_bytes);  // the partial rows the row kernel writes
        }
        uint64_t nout_all = 0;
        ctx->stats.rank_units += int64_t(nb);
        for (uint32_t k = 0; k < nb; ++k) {
            Rule* r = x.batch[x.la + k];
            const ExpHdr h = x.h_hdr[k];
            nout_all += h.nout;
            if (use_bm) {
                // own bytes: domain = the |X|+|Y| bitmap operands + 4 B written per domain sid;
                // rows = per domain sid its id and row bounds (12 B) and |X u Y| probes (rank
                // directory 4 B + bitmap words 16 B + vertical entry 8 B), or per parent row 16 B
                // and one probe (plist), + 8 B per entry walked + 16 B per kept row written
                const bool pm = x.h_sides[k].lmode == 2;
                const uint64_t bmb = pm ? 0ull : uint64_t(r->nx + r->ny) * d->NW * 4;
                const uint64_t ndom = pm ? r->pn : h.nsid;
                exp_domain += ndom;
                exp_entries += h.nent;
                exp_hold += h.nhold;
                exp_walk += h.nwalk;
                exp_plist += pm ? 1 : 0;
                exp_bitmap_bytes += int64_t(bmb);
                seg[0].bytes += int64_t(bmb + 4ull * (pm ? 0ull : h.nsid));
                seg[1].bytes += int64_t(8ull * h.nwalk + (pm ? 44ull : 12ull + 28ull * (r->nx + r->ny)) * ndom +
                                        (x.kmono[k] != kNoList ? 16ull * h.ln : 0ull));
                // SURVEY: N/8 B per sid-bitmap operand; 4 B token + 4 B first/last per position of
                // every sequence where the rule holds (the reference scans each of them whole)
                seg[0].survey += int64_t(bmb);
                seg[1].survey += int64_t(8ull * h.nent);
                // the rule's kept rows (more than its support: the list was cut, none kept)
                r->loff = x.kmono[k] != kNoList && h.ln <= x.h_sides[k].kb ? x.kmono[k] : kNoList;
                r->ln = h.ln;
            }
            if (h.nout > ecap) throw Error(FSM_ELIMIT, "TSR: expansion candidate buffer overflow");
            if (!use_bm && x.drv_in_x[k] && h.nx != r->nX)
                throw Error(FSM_EDEVICE, "TSR: |sids(X)| mismatch in expansion (" + std::to_string(h.nx) + " vs " +
                                             std::to_string(r->nX) + ")");
            r->inset = -1;
            if (r->dropped) continue;  // a speculated child its parent's commit did not register
            ExpResult& res = res_get(r);
            const ExpRec* rec = x.h_rec + size_t(k) * ecap;
            if (use_bm) {  // the reduce blocks' kid ranges, in kid (= item) order
                res.recs.clear();
                res.recs.reserve(h.nout);
                const uint32_t* rc = x.h_rcnt + size_t(k) * P * grid.collect;
                const uint32_t q = (KP + grid.collect - 1) / grid.collect;
                for (uint32_t p = 0; p < P; ++p)
                    for (uint32_t g = 0; g < grid.collect; ++g) {
                        const ExpRec* r0 = rec + size_t(p) * KP + size_t(g) * q;
                        res.recs.insert(res.recs.end(), r0, r0 + rc[p * grid.collect + g]);
                    }
            } else {
                res.recs.assign(rec, rec + h.nout);
                std::sort(res.recs.begin(), res.recs.end(), [](const ExpRec& a, const ExpRec& c) { return a.c < c.c; });
            }
        }
        if (x.sharded) {
            // every rank's slots: (nsid, nent, nrec, records) per slot of its share, gathered
            // once per launch (the failure agreement rides along); the replay then goes on
            // alike on every rank
            std::vector<uint8_t> mine;
            auto put = [&](const void* p, size_t n) {
                const uint8_t* b = static_cast<const uint8_t*>(p);
                mine.insert(mine.end(), b, b + n);
            };
            for (uint32_t k = 0; k < nb; ++k) {
                Rule* r = x.batch[x.la + k];
                const ExpHdr h = x.h_hdr[k];
                const uint32_t nrec = r->dropped || r->res < 0 ? 0u : uint32_t(res_pool[size_t(r->res)].recs.size());
                const uint32_t hd[3] = {h.nsid, h.nent, nrec};
                put(hd, sizeof(hd));
                if (nrec) put(res_pool[size_t(r->res)].recs.data(), nrec * sizeof(ExpRec));
            }
            std::vector<size_t> sizes;
            const std::vector<uint8_t> all = comm->gather_blobs(mine, sizes, s, &agr);
            // the ranks' blobs hold their contiguous slot ranges, in rank and slot order
            size_t at = 0;
            uint32_t k = 0;
            for (int q = 0; q < R; ++q) {
                const size_t end = at + sizes[size_t(q)];
                for (; k < x.batch.size() && at < end; ++k) {
                    uint32_t hd[3];
                    std::memcpy(hd, all.data() + at, sizeof(hd));
                    at += sizeof(hd);
                    Rule* r = x.batch[k];
                    if (q != comm->rank()) {
                        exp_domain += hd[0];
                        exp_entries += hd[1];
                        r->inset = -1;
                        if (!r->dropped) {
                            ExpResult& res = res_get(r);
                            res.recs.resize(hd[2]);
                            if (hd[2]) std::memcpy(res.recs.data(), all.data() + at, hd[2] * sizeof(ExpRec));
                        }
                    }
                    at += size_t(hd[2]) * sizeof(ExpRec);
                }
            }
            if (at != all.size()) throw Error(FSM_EDEVICE, "TSR: sharded expansion results out of step");
        }
        seg[2].bytes += int64_t(nout_all * sizeof(ExpRec));
        x.timed = false;
        spec_todo.emplace_back(std::move(x.batch), x.depth);
        x.batch.clear();
        post_ms += now_ms() - tw1;
    };
    // expand `batch` on a free set (finishing the older busy one first when both are
    // busy): enqueue the launch and return; finish() takes the results in
    auto launch = [&](const std::vector<Rule*>& batch, int depth) {
        ExpSet* xp = nullptr;
        for (int xi = 0; xi < nsets && !xp; ++xi)
            if (!xs[xi].busy) xp = &xs[xi];
        if (!xp) {  // every set busy: the oldest launch finishes first
            xp = &xs[0];
            for (int xi = 1; xi < nsets; ++xi)
                if (xs[xi].seq < xp->seq) xp = &xs[xi];
            finish(*xp);
        }
        ExpSet& x = *xp;
        const double tl0 = now_ms();
        x.batch = batch;
        x.depth = depth;
        x.seq = seq_next++;
        for (Rule* r : batch) {
            r->inset = int8_t(xp - xs);
            // every rule of the batch (not only this rank's slots): its children's X ids derive from it
            if (r->xid == kNone) r->xid = rp.xin.get(r->pxid, rp.st.X(r)[r->nx - 1]);
        }
        // slot sharding: this rank expands only its contiguous share of the batch, split so
        // that the shares' expected domains (about twice each rule's support) are equal
        x.la = 0;
        x.lz = uint32_t(batch.size());
        x.sharded = false;
        uint64_t tot = 0;
        if (shard_exp)
            for (Rule* r : batch) tot += 2ull * r->sup + 1;
        if (shard_exp && tot >= shard_min) {
            x.sharded = true;
            const uint64_t lo = tot * uint64_t(comm->rank()) / uint64_t(R), hi = tot * uint64_t(comm->rank() + 1) / uint64_t(R);
            uint64_t acc = 0;
            x.la = x.lz = uint32_t(batch.size());
            for (uint32_t k = 0; k < batch.size(); ++k) {  // slot k belongs to the rank whose range holds its start
                if (acc >= lo && x.la == batch.size()) x.la = k;
                if (acc >= hi) { x.lz = k; break; }
                acc += 2ull * batch[k]->sup + 1;
            }
            if (x.lz < x.la) x.lz = x.la;
        }
        const uint32_t nb = x.lz - x.la;  // slots launched here
        const Rule* const* bp = batch.data() + x.la;
        gpu_rules += nb;
        // descriptors written in place into the set's pinned stage (only the used items:
        // the kernels read X[0, nx) and Y[0, ny))
        uint64_t* drv_off = x.h_drv;
        uint64_t* wave_off = x.h_wave;
        drv_off[0] = wave_off[0] = 0;
        x.drv_in_x.assign(nb, 1);
        for (uint32_t k = 0; k < nb; ++k) {
            const Rule* r = bp[k];
            const uint32_t *rx = rp.st.X(r), *ry = rp.st.Y(r);
            Side& sd = x.h_sides[k];
            sd.nx = r->nx;
            sd.ny = r->ny;
            sd.doL = r->expandLR;
            sd.doR = 1;
            sd.maxX = rx[r->nx - 1];
            sd.maxY = ry[r->ny - 1];
            std::copy(rx, rx + r->nx, sd.X);
            std::copy(ry, ry + r->ny, sd.Y);
            sd.pc = sd.pleft = sd.pn = sd.kb = 0;
            sd.pl = 0;
            sd.ko = kNoList;
            sd.xid = r->xid;  // (the memo key of its left extensions)
            sd.klo = use_bm ? std::min(h_kid_of[rx[r->nx - 1]], h_kid_of[ry[r->ny - 1]]) + 1u : 0u;
            if (use_bm && plist && r->ploff != kNoList && r->ploff + plist_window >= ahead) {
                // the parent's kept rows (still in the ring) are the domain: only the added item is
                // probed there
                wave_off[k + 1] = wave_off[k] + std::clamp<uint64_t>((uint64_t(r->pn) + pl_spb - 1) / pl_spb, 1,
                                                                     grid.expand);
                drv_off[k + 1] = drv_off[k];
                sd.drv = 0;
                sd.lmode = 2;
                sd.pc = r->pc;
                sd.pleft = r->pleft ? 1u : 0u;
                sd.pn = r->pn;
                sd.pl = r->ploff % acap;
            } else if (use_bm) {
                // bitmap path: row blocks sized by the expected domain (about twice the rule's
                // support: sids holding X u Y in either order), exp_spb sids per block; the
                // domain list holds at most the support of the rarest item of X u Y
                wave_off[k + 1] = wave_off[k] + std::clamp<uint64_t>((2ull * r->sup + exp_spb - 1) / exp_spb, 1,
                                                                     grid.expand);
                uint32_t cap = kNone, drv = rx[0];
                for (uint32_t q = 0; q < r->nx; ++q) if (sup[rx[q]] < cap) { cap = sup[rx[q]]; drv = rx[q]; }
                for (uint32_t q = 0; q < r->ny; ++q) if (sup[ry[q]] < cap) { cap = sup[ry[q]]; drv = ry[q]; }
                drv_off[k + 1] = drv_off[k] + cap;
                sd.drv = drv;
                sd.lmode = dom_mode == 2 || (dom_mode == 0 && uint64_t(cap) * 4 < d->NW) ? 1u : 0u;
            } else {
                // list path: one wave per sid of the driver list: the rarest item of X
                // (expandL needs all of sids(X)), else of X u Y
                uint32_t drv = rx[0];
                for (uint32_t q = 0; q < r->nx; ++q) if (sup[rx[q]] < sup[drv]) drv = rx[q];
                if (!r->expandLR)
                    for (uint32_t q = 0; q < r->ny; ++q) if (sup[ry[q]] < sup[drv]) { drv = ry[q]; x.drv_in_x[k] = 0; }
                drv_off[k] = voff[drv];
                wave_off[k + 1] = wave_off[k] + (voff[drv + 1] - voff[drv]);
            }
        }
        x.kmono.assign(nb, kNoList);
        x.amin = kNoList;
        for (uint32_t k = 0; k < nb; ++k)
            if (x.h_sides[k].lmode == 2) x.amin = std::min(x.amin, bp[k]->ploff);
        if (plist && acap) {  // the slots' kept-row lists at the ring's head, each at most the rule's support
            uint64_t need = 0;
            for (uint32_t k = 0; k < nb; ++k) need += bp[k]->sup;
            // (the head skips to the ring's start when a list would wrap)
            const uint64_t at = ahead % acap + need > acap ? ahead + acap - ahead % acap : ahead;
            // a launch never overwrites the parent lists its own slots read (x.amin): it keeps
            // no lists then (only a parent window wider than the default can come this close)
            const bool own_ok = x.amin == kNoList || x.amin + acap >= at + need;
            if (need && need <= acap / (4 * uint64_t(nsets)) && own_ok) {
                ahead = at;
                // positions below ahead + need - acap are overwritten now: a set still in flight
                // that reads or writes one of them is finished first (its results are taken in)
                for (int xi = 0; xi < nsets; ++xi) {
                    ExpSet& o = xs[xi];
                    if (&o != &x && o.busy && o.amin != kNoList && o.amin + acap < ahead + need) {
                        // its kernels completed is all the ring needs (its results are taken in at
                        // their turn: a finish here would be a rank-local collective when sharded)
                        FSM_HIP(hipEventSynchronize(o.ev[5]));
                        o.amin = kNoList;
                        ++ring_waits;
                    }
                }
                x.amin = std::min(x.amin, ahead);
                for (uint32_t k = 0; k < nb; ++k) {
                    x.h_sides[k].ko = ahead % acap;
                    x.h_sides[k].kb = bp[k]->sup;
                    x.kmono[k] = ahead;
                    ahead += bp[k]->sup;
                }
            }
        }
        if (use_bm && wave_off[nb] > max_blocks) {
            // partial rows over budget: the budget is shared in proportion to the slots'
            // expected domains (the launch lasts as long as its largest slot's blocks), at
            // least one block each
            const uint64_t tot = wave_off[nb];
            uint64_t prev = 0;  // the original prefix at k
            for (uint32_t k = 0; k < nb; ++k) {
                const uint64_t n0 = wave_off[k + 1] - prev;
                prev = wave_off[k + 1];
                wave_off[k + 1] = wave_off[k] + std::max<uint64_t>(1, n0 * (max_blocks - nb) / tot);
            }
        }
        x.blocks = wave_off[nb];
        if (use_bm && x.dom.bytes < drv_off[nb] * 4)
            x.dom.alloc(std::max<uint64_t>(drv_off[nb] * 4 * 5 / 4, uint64_t(1) << 20));
        fill_ms += now_ms() - tl0;
        hipStream_t s = x.st;  // (shadows the context stream for this launch)
        // the descriptors by a copy kernel on the set's stream (reading the mapped staging over PCIe:
        // an SDMA copy would cost the launch's first kernel a cross-engine wait)
        static_assert(sizeof(Side) % 4 == 0, "Side: whole words");
        copy_from_mapped(x.d_stage.p, x.stage->dev, 2 * kOffB + size_t(nb) * sizeof(Side), s);
        x.timed = nb && launches % time_every == 0;  // every 16th launch is timed (events cost host time)
        const ExpGeo geo{K, KP, uint32_t(wave_off[nb]), rp.minsup};
        if (nb) {  // (a rank may get no slot of a small sharded batch)
            if (use_bm && x.alive_t != rp.minsup) {  // minsup rose: the kids below it stop counting
                hipLaunchKernelGGL(k_alive, dim3(unsigned(((K + 15) / 16 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                                   d_ksup.as<uint32_t>(), K, rp.minsup, x.alive.as<uint32_t>());
                FSM_LAUNCHED("k_alive", s);
                x.alive_t = rp.minsup;
            }
            if (x.timed) FSM_HIP(hipEventRecord(x.ev[0], s));
            bool any_dom = false;  // (every slot on its parent's kept rows: no domain kernel)
            for (uint32_t k = 0; k < nb && !any_dom; ++k) any_dom = x.h_sides[k].lmode != 2;
            if (use_bm) {
                if (any_dom) {
                    hipLaunchKernelGGL(k_exp_domain, dim3((d->NW + kDomWords - 1) / kDomWords, nb), dim3(kDomThreads),
                                       0, s, x.d_sides, d->bm.as<uint32_t>(), d->NW, x.d_drv, x.dom.as<uint32_t>(),
                                       x.ctl.as<ExpCtl>(), d->vert_off.as<uint64_t>(), d->vert_sid.as<uint32_t>());
                    FSM_LAUNCHED("k_exp_domain", s);
                }
                if (x.timed) FSM_HIP(hipEventRecord(x.ev[1], s));
                hipLaunchKernelGGL(k_exp_rows, dim3(unsigned(wave_off[nb]), P), dim3(kXBlock), xlds, s, x.d_sides,
                                   x.d_wave, nb, x.d_drv, x.dom.as<uint32_t>(), k_off.as<uint32_t>(), k_ent.as<uint2>(),
                                   d_kidof.as<uint32_t>(), x.alive.as<uint32_t>(), geo, x.part.as<uint32_t>(),
                                   x.ctl.as<ExpCtl>(), x.d_ndlw.as<uint32_t>(),
                                   DomProbe{d->bm.as<uint32_t>(), d->NW, d->NW / 4, d_rdir.as<uint32_t>(),
                                            d_kvoff.as<uint32_t>(), d_vfl.as<uint2>()},
                                   arena.as<uint4>());
                FSM_LAUNCHED("k_exp_rows", s);
                if (x.timed) FSM_HIP(hipEventRecord(x.ev[2], s));
                hipLaunchKernelGGL(k_expand_reduce, dim3(grid.collect, nb, P), dim3(kBlock), 0, s, x.part.as<uint32_t>(),
                                   x.d_wave, geo, d_kept.as<uint32_t>(), x.ctl.as<ExpCtl>(), x.d_rec, ecap,
                                   x.d_dlw.as<uint4>(), x.d_ndlw.as<uint32_t>(), x.d_rcnt, x.d_sides, memo);
                FSM_LAUNCHED("k_expand_reduce", s);
                if (x.timed) FSM_HIP(hipEventRecord(x.ev[3], s));
                hipLaunchKernelGGL(k_dl, dim3(grid.dl), dim3(kBlock), 0, s, x.d_sides, d->bm.as<uint32_t>(),
                                   d->NW, d->vert_off.as<uint64_t>(), d->vert_sid.as<uint32_t>(), x.d_dlw.as<uint4>(),
                                   x.d_ndlw.as<uint32_t>(), x.d_rec, ecap, x.ctl.as<ExpCtl>(), x.d_hdr, nb, memo);
                FSM_LAUNCHED("k_dl", s);
            } else {
                const uint64_t waves = wave_off[nb];
                if (waves) {
                    hipLaunchKernelGGL(k_expand, dim3(unsigned((waves * 64 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                                       x.d_sides, x.d_drv, x.d_wave, nb,
                                       d->vert_sid.as<uint32_t>(), k_off.as<uint32_t>(), k_item.as<uint32_t>(),
                                       k_first.as<uint32_t>(), k_last.as<uint32_t>(), U, x.TL.as<uint32_t>(),
                                       x.DL.as<uint32_t>(), x.TR.as<uint32_t>(), x.seen.as<uint32_t>(),
                                       x.list.as<uint32_t>(), x.ctl.as<ExpCtl>(), d_sup.as<uint32_t>(), rp.minsup);
                    FSM_LAUNCHED("k_expand", s);
                }
                if (x.timed) FSM_HIP(hipEventRecord(x.ev[1], s));
                if (x.timed) FSM_HIP(hipEventRecord(x.ev[2], s));
                hipLaunchKernelGGL(k_expand_collect, dim3(grid.collect, nb), dim3(kBlock), 0, s, x.TL.as<uint32_t>(),
                                   x.DL.as<uint32_t>(), x.TR.as<uint32_t>(), x.seen.as<uint32_t>(), x.list.as<uint32_t>(),
                                   x.ctl.as<ExpCtl>(), U, rp.minsup, x.d_rec, ecap);
                FSM_LAUNCHED("k_expand_collect", s);
                if (x.timed) FSM_HIP(hipEventRecord(x.ev[3], s));
                hipLaunchKernelGGL(k_publish, dim3(1), dim3(kBlock), 0, s, x.ctl.as<ExpCtl>(), x.d_hdr, nb);
                FSM_LAUNCHED("k_publish", s);
            }
        }
        if (x.timed) FSM_HIP(hipEventRecord(x.ev[4], s));
        FSM_HIP(hipEventRecord(x.ev[5], s));
        x.busy = true;
        ++launches;
        prep_ms += now_ms() - tl0;
    };
    // Speculated rules wait in `pending` (ordered like the heap, results
    // cached or in flight) instead of going back to the heap: the next rule to
    // commit is always the larger of the heap top and the pending front, which
    // is exactly the one-at-a-time order; new rules only ever enter the heap.
    // The rules of one batch pop leave the heap in its order, so `pending` is a
    // merge of sorted runs (one per pop loop): a small heap of runs keyed by their
    // fronts, no per-rule tree node.
    struct PendingRuns {
        const RuleStore* st;
        struct Run {
            std::vector<Rule*> v;  // largest first
            size_t h = 0;          // front
        };
        std::vector<Run> runs;
        std::vector<int> free_ids, heap;  // heap: live runs, the largest front on top
        bool front_less(int a, int b) const {
            return rule_cmp(*st, runs[size_t(a)].v[runs[size_t(a)].h], runs[size_t(b)].v[runs[size_t(b)].h]) < 0;
        }
        bool empty() const { return heap.empty(); }
        Rule* front() const { return runs[size_t(heap[0])].v[runs[size_t(heap[0])].h]; }
        void pop() {
            auto cmp = [this](int a, int b) { return front_less(a, b); };
            const int id = heap[0];
            std::pop_heap(heap.begin(), heap.end(), cmp);
            heap.pop_back();
            Run& r = runs[size_t(id)];
            if (++r.h < r.v.size()) {
                heap.push_back(id);
                std::push_heap(heap.begin(), heap.end(), cmp);
            } else {
                r.v.clear();
                r.h = 0;
                free_ids.push_back(id);
            }
        }
        void add(std::vector<Rule*>& v) {  // v: in heap pop order; taken over (left empty)
            if (v.empty()) return;
            int id;
            if (free_ids.empty()) {
                id = int(runs.size());
                runs.emplace_back();
            } else {
                id = free_ids.back();
                free_ids.pop_back();
            }
            runs[size_t(id)].v.swap(v);
            runs[size_t(id)].h = 0;
            v.clear();
            heap.push_back(id);
            std::push_heap(heap.begin(), heap.end(), [this](int a, int b) { return front_less(a, b); });
        }
        uint32_t min_sup() const {  // support of the smallest pending rule (the runs' backs)
            uint32_t m = 0xFFFFFFFFu;
            for (int id : heap) m = std::min(m, runs[size_t(id)].v.back()->sup);
            return m;
        }
    };
    PendingRuns pending{&rp.st, {}, {}, {}};
    std::vector<Rule*> popped;  // one pop loop's rules (a run of `pending`)
    // a speculated child that its parent's commit did not register: drop its
    // results (cached, or marked so that an in-flight launch's are discarded) and,
    // recursively, those of its own speculated children
    std::function<void(Rule*)> drop_spec = [&](Rule* x) {
        x->dropped = true;
        spec_waste += x->spec;
        if (x->res < 0) return;
        std::vector<Rule*> kids;
        {
            const ExpResult& e = res_pool[size_t(x->res)];
            for (Rule* c : e.preL) if (c) kids.push_back(c);
            for (Rule* c : e.preR) if (c) kids.push_back(c);
        }
        res_release(x);
        for (Rule* c : kids) drop_spec(c);
    };
    auto commit = [&](Rule* r, ExpResult& res) {
        const std::vector<ExpRec>& er = res.recs;
        const bool pre = !res.preL.empty();
        expansions += r->expandLR ? 2 : 1;
        if (ctx->opts.verbose && now_ms() - last_log_ms > 20000.0 && (last_log_ms = now_ms()) > 0)
            std::fprintf(stderr, "[fsm tsr] %lld expansions, minsup %u, candidates %zu, rules %zu, %.0f ms\n",
                         (long long)expansions, rp.minsup, rp.cand.size(), rp.krules.size(), now_ms() - t0);
        if (r->expandLR) {  // expandL: X u {c} => Y
            for (size_t i = 0; i < er.size(); ++i) {
                const ExpRec& e = er[i];
                Rule* sp = pre ? res.preL[i] : nullptr;
                if (e.tl == 0 || e.tl < rp.minsup) {
                    if (sp) drop_spec(sp);
                    continue;
                }
                Rule* nr = sp ? sp : rp.derive(r, e.c, kNone, e.tl, e.dl);
                if (nr->conf >= minconf) rp.save(nr);
                rp.reg(nr, true);
            }
        }
        for (size_t i = 0; i < er.size(); ++i) {  // expandR: X => Y u {c}
            const ExpRec& e = er[i];
            Rule* sp = pre ? res.preR[i] : nullptr;
            if (e.tr == 0 || e.tr < rp.minsup) {
                if (sp) drop_spec(sp);
                continue;
            }
            Rule* nr = sp ? sp : rp.derive(r, kNone, e.c, e.tr, r->nX);
            if (nr->conf >= minconf) rp.save(nr);
            rp.reg(nr, false);
        }
    };

    // Child speculation: when a launch finishes, the children of its rules that
    // rank at or above the lowest pending rule (sup >= T) are the ones whose
    // registration would force the next launch (a fresh rule outranking the
    // pending front).  They are created now, exactly as their parent's commit
    // would create them, and expanded in a follow-up launch (a few levels deep)
    // while the host commits; the commit then registers the pre-built rule
    // (results cached or in flight) instead of deriving it again.
    int64_t spec_made = 0, spec_launches = 0;
    int spec_depth = kSpecDepth, spec_max = kSpecMax * int(B);  // FSM_TSR_SPEC="depth,max" (tuning; "0" disables)
    double spec_frac = 1.0;  // FSM_TSR_SPEC_FRAC: speculate children with sup >= frac * T (tuning)
    if (const char* v = std::getenv("FSM_TSR_SPEC_FRAC")) {
        const double f = std::atof(v);
        if (f > 0.0 && f <= 1.0) spec_frac = f;
    }
    if (const char* v = std::getenv("FSM_TSR_SPEC")) {
        int a = 0, b2 = 0;
        if (std::sscanf(v, "%d,%d", &a, &b2) == 2 && a >= 0 && a <= 64 && b2 > 0 && b2 <= 4096) {
            spec_depth = a;
            spec_max = b2;
        }
    }
    const bool spec_on = [] { const char* v = std::getenv("FSM_TSR_SPEC"); return !(v && v[0] == '0'); }();
    // the next level of one finished launch's batch
    auto speculate = [&](const std::vector<Rule*>& level, int depth) {
        if (!spec_on || depth >= spec_depth || level.empty()) return;
        uint32_t T = 0xFFFFFFFFu;
        for (Rule* x : level) T = std::min(T, x->sup);
        if (!pending.empty()) T = std::min(T, pending.min_sup());
        T = std::max(uint32_t(double(T) * spec_frac), rp.minsup);
        std::vector<Rule*> next;
        for (Rule* x : level) {
            if (x->res < 0) continue;  // committed already, or dropped
            ExpResult& res = res_pool[size_t(x->res)];
            const size_t n = res.recs.size();
            res.preL.assign(n, nullptr);
            res.preR.assign(n, nullptr);
            for (size_t i = 0; i < n && next.size() < size_t(spec_max); ++i) {
                const ExpRec& e = res.recs[i];
                if (x->expandLR && e.tl >= T) {
                    Rule* c = rp.derive(x, e.c, kNone, e.tl, e.dl);
                    c->expandLR = true;
                    c->spec = true;
                    res.preL[i] = c;
                    next.push_back(c);
                }
                if (e.tr >= T && next.size() < size_t(spec_max)) {
                    Rule* c = rp.derive(x, kNone, e.c, e.tr, x->nX);
                    c->expandLR = false;
                    c->spec = true;
                    res.preR[i] = c;
                    next.push_back(c);
                }
            }
        }
        spec_made += int64_t(next.size());
        for (size_t a = 0; a < next.size(); a += size_t(B)) {
            const std::vector<Rule*> part(next.begin() + a, next.begin() + std::min(next.size(), a + size_t(B)));
            launch(part, depth + 1);
            ++spec_launches;
        }
    };

    std::vector<Rule*> batch;
    size_t sweep_at = size_t(1) << 16;
    for (;;) {
        // children of finished launches first (their launches overlap the commits below)
        while (!spec_todo.empty()) {
            std::vector<std::pair<std::vector<Rule*>, int>> todo;
            todo.swap(spec_todo);
            for (auto& [lvl, dp] : todo) speculate(lvl, dp);
        }
        const bool have_h = !rp.cand.empty(), have_p = !pending.empty();
        if (!have_h && !have_p) break;
        const bool from_p = have_p && (!have_h || rule_cmp(rp.st, pending.front(), rp.cand.top().r) > 0);
        Rule* r = from_p ? pending.front() : rp.cand.top().r;
        if (r->sup < rp.minsup) break;
        if (r->res < 0 && r->inset >= 0) {  // expanding on the GPU: take its launch in, then decide again
            finish(xs[r->inset]);
            continue;
        }
        if (r->res >= 0) {  // results at hand: commit now
            if (from_p) pending.pop();
            else rp.cand.pop();
            // (the host-time split is taken only when verbose: a clock read costs as much as a commit)
            const double tc0 = ctx->opts.verbose ? now_ms() : 0.0;
            commit(r, res_pool[size_t(r->res)]);
            spec_hit += r->spec;
            if (r->res >= 0) res_release(r);
            if (ctx->opts.verbose) commit_ms += now_ms() - tc0;
            if (res_live > sweep_at) {  // results of rules now below minsup can never be committed
                for (ExpResult& e : res_pool)
                    if (e.owner && e.owner->sup < rp.minsup) res_release(e.owner);
                sweep_at = std::max<size_t>(2 * res_live, 1u << 16);
            }
            continue;
        }
        if (from_p) throw Error(FSM_EDEVICE, "TSR: a pending rule has neither results nor a launch");
        // r (neither cached nor in flight) and the next heap rules are expanded together
        const double tp0 = now_ms();
        batch.clear();
        popped.clear();
        while (batch.size() < size_t(B) && !rp.cand.empty() && uint32_t(rp.cand.top().k1 >> 32) >= rp.minsup) {
            Rule* x = rp.cand.top().r;
            rp.cand.pop();
            popped.push_back(x);
            if (x->res < 0 && x->inset < 0) batch.push_back(x);  // else already expanded by speculation
        }
        pending.add(popped);
        pop_ms += now_ms() - tp0;
        launch(batch, 0);
        spec_pushback += int64_t(batch.size()) - 1;
    }
    for (int xi = 0; xi < nsets; ++xi)  // speculation still in flight when the replay ended
        if (xs[xi].busy) finish(xs[xi]);
    ctx->stats.tsr_ring_waits = ring_waits;
    if (ctx->opts.verbose)
        std::fprintf(stderr,
                     "[fsm tsr] expansions %lld in %lld launches (%lld rules expanded, %lld pushed back), %.0f ms waiting on the "
                     "GPU; host: %.0f ms launch prep (%.0f descriptors), %.0f ms result intake, %.0f ms commit, %.0f ms batch pops; %zu rules "
                     "made\n",
                     (long long)expansions, (long long)launches, (long long)gpu_rules, (long long)spec_pushback, wait_ms,
                     prep_ms, fill_ms, post_ms, commit_ms, pop_ms, rp.st.size());
    if (ctx->opts.verbose)
        std::fprintf(stderr, "[fsm tsr] child speculation: %lld rules in %lld launches (%lld committed, %lld dropped); partial rows %.1f MB; domain sids "
                     "%lld (row entries %lld), rows where the rule holds %lld, row entries walked %lld; "
                     "rules on their parent's kept rows %lld (ring: %llu entries written, %lld early finishes); candidates sorted %zu, popped %zu\n",
                     (long long)spec_made, (long long)spec_launches, (long long)spec_hit, (long long)spec_waste, double(exp_part_bytes) / 1e6, (long long)exp_domain,
                     (long long)exp_entries, (long long)exp_hold, (long long)exp_walk, (long long)exp_plist,
                     (unsigned long long)ahead, (long long)ring_waits, rp.cand.n_sorted, rp.cand.n_popped);
    // ---------------- result = kRules
    std::vector<const Rule*> res;
    while (!rp.krules.empty()) {
        res.push_back(rp.krules.top().r);
        rp.krules.pop();
    }
    auto* o = static_cast<fsm_rules*>(std::calloc(1, sizeof(fsm_rules)));
    if (!o) throw Error(FSM_ENOMEM, "calloc failed");
    const size_t n = res.size();
    o->n = int64_t(n);
    o->total = d->N;
    o->final_minsup = int32_t(rp.minsup);
    size_t na = 0, nc = 0;
    for (const Rule* r : res) { na += r->nx; nc += r->ny; }
    o->support = static_cast<int32_t*>(std::malloc(std::max<size_t>(n, 1) * 4));
    o->confidence = static_cast<double*>(std::malloc(std::max<size_t>(n, 1) * 8));
    o->ante_off = static_cast<int64_t*>(std::malloc((n + 1) * 8));
    o->cons_off = static_cast<int64_t*>(std::malloc((n + 1) * 8));
    o->ante = static_cast<int32_t*>(std::malloc(std::max<size_t>(na, 1) * 4));
    o->cons = static_cast<int32_t*>(std::malloc(std::max<size_t>(nc, 1) * 4));
    if (!o->support || !o->confidence || !o->ante_off || !o->cons_off || !o->ante || !o->cons) {
        fsm_rules_free(o);
        throw Error(FSM_ENOMEM, "malloc failed");
    }
    o->ante_off[0] = o->cons_off[0] = 0;
    for (size_t q = 0; q < n; ++q) {
        const Rule* r = res[q];
        o->support[q] = int32_t(r->sup);
        o->confidence[q] = r->conf;
        const uint32_t *rx = rp.st.X(r), *ry = rp.st.Y(r);
        for (uint32_t x = 0; x < r->nx; ++x) o->ante[o->ante_off[q] + int64_t(x)] = db->tsr.item_val[rx[x]];
        for (uint32_t x = 0; x < r->ny; ++x) o->cons[o->cons_off[q] + int64_t(x)] = db->tsr.item_val[ry[x]];
        o->ante_off[q + 1] = o->ante_off[q] + int64_t(r->nx);
        o->cons_off[q + 1] = o->cons_off[q] + int64_t(r->ny);
    }
    ctx->kstats.clear();
    for (int q = 0; q < 4; ++q) {
        if (!seg_name[q][0]) continue;
        fsm_kernel_stat k{};
        std::snprintf(k.name, sizeof(k.name), "%s", seg_name[q]);
        k.launches = seg[q].n;
        k.ms = seg[q].timed ? seg[q].ms * double(seg[q].n) / double(seg[q].timed) : 0.0;  // sampled, scaled
        k.alg_bytes = seg[q].bytes;
        k.survey_bytes = seg[q].survey;
        ctx->kstats.push_back(k);
    }
    ctx->stats.exp_domain = exp_domain;
    ctx->stats.exp_entries = exp_entries;
    ctx->stats.exp_bitmap_bytes = exp_bitmap_bytes;
    ctx->stats.expansions = expansions;
    ctx->stats.rules = int64_t(n);
    ctx->stats.ms_f2 = t1 - t0;          // pair phase
    ctx->stats.ms_lattice = now_ms() - t1;  // expansions
    ctx->stats.ms_count_kernel = wait_ms;   // of which: waiting for the expansion kernels
    ctx->stats.count_launches = launches;
    ctx->stats.ms_mine = now_ms() - t0;
    *out = o;
}

}  // namespace fsm
