// fsm_api.cpp — the extern "C" boundary (include/fsm.h).  Every entry point
// catches everything: no C++ exception crosses the ABI, failures come back as
// FSM_E* codes with the message in fsm_last_error (the Scala shim turns them
// into java.lang.Exception so TrainActor records FAILURE, TrainActor.scala:65-67).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>

#include "comm.h"
#include "dev_db.h"
#include "device_util.h"
#include "fsm_internal.h"
#include "host_pool.h"

using fsm::Error;

namespace {

thread_local std::string g_err;  // errors before a context exists

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

int make_db(fsm_ctx* ctx, int32_t mode, const fsm::Source& src, fsm_db** out) {
    if (!ctx || !out) return fail(ctx, FSM_EINVAL, "null argument");
    *out = nullptr;
    if (src.n < 0 || (src.n > 0 && !src.sids)) return fail(ctx, FSM_EINVAL, "bad record arrays");
    if (mode != FSM_MODE_SPADE && mode != FSM_MODE_TSR) return fail(ctx, FSM_EINVAL, "mode must be SPADE(0) or TSR(1)");
    fsm_db* db = new (std::nothrow) fsm_db();
    if (!db) return fail(ctx, FSM_ENOMEM, "host allocation failed");
    db->ctx = ctx;
    db->mode = mode;
    const int rc = guarded(ctx, [&] {
        FSM_HIP(hipSetDevice(ctx->opts.device));
        ctx->stats.k0_device = 0;
        if (fsm::k0_build(ctx, mode, src, db)) return;  // K0 on the GPU (token input)
        const double t0 = fsm::now_ms();
        if (mode == FSM_MODE_SPADE) fsm::flatten_spade(src, db->spade);
        else fsm::flatten_tsr(src, db->tsr);
        const double t1 = fsm::now_ms();
        if (mode == FSM_MODE_SPADE) fsm::spade_upload(ctx, db);
        else fsm::tsr_upload(ctx, db);
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
    if (!opts || opts->nranks < 2) return fail(nullptr, FSM_EINVAL, "selftest needs nranks >= 2");
    return guarded(nullptr, [&] {
        if (!opts->host_comm) FSM_HIP(hipSetDevice(opts->device));
        auto comm = fsm::make_comm(*opts);
        const uint32_t N = uint32_t(opts->nranks), r = uint32_t(opts->rank);
        std::vector<uint32_t> v(1000);
        for (uint32_t i = 0; i < v.size(); ++i) v[i] = r + i;
        comm->host_allreduce_u32(v.data(), v.size(), nullptr);
        for (uint32_t i = 0; i < v.size(); ++i)
            if (v[i] != N * i + N * (N - 1) / 2) throw Error(FSM_ECOMM, "selftest: all-reduce mismatch");
        std::vector<uint8_t> mine(size_t(r) * 3 + 1);
        for (size_t j = 0; j < mine.size(); ++j) mine[j] = uint8_t(r * 7 + j);
        std::vector<size_t> sizes;
        // (the work-stealing counter of the claim test below is reset before this gather, which
        // also agrees on whether every rank has the shared counters)
        const int64_t key = comm->next_key();
        comm->reset_counter(key);
        uint32_t ex = comm->has_fetch_add() ? 1u : 0u;
        const std::vector<uint8_t> all = comm->gather_blobs(mine, sizes, nullptr, nullptr, &ex, 1);
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
                const int64_t old = comm->fetch_add(key, int64_t(r) + 1);
                if (old < 0) throw Error(FSM_ECOMM, "selftest: fetch_add failed");
                if (old >= kUnits) break;
                for (int64_t u = old; u < std::min<int64_t>(old + r + 1, kUnits); ++u) {
                    const uint16_t v16 = uint16_t(u);
                    got.push_back(uint8_t(v16 & 0xFF));
                    got.push_back(uint8_t(v16 >> 8));
                }
            }
            std::vector<size_t> csz;
            const std::vector<uint8_t> claimed = comm->gather_blobs(got, csz, nullptr);
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
    });
}

int fsm_ctx_create(const fsm_opts* opts, fsm_ctx** out) {
    if (!out) return FSM_EINVAL;
    *out = nullptr;
    fsm_ctx* ctx = new (std::nothrow) fsm_ctx();
    if (!ctx) return fail(nullptr, FSM_ENOMEM, "host allocation failed");
    if (opts) ctx->opts = *opts;
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
        ctx->comm = fsm::make_comm(ctx->opts).release();
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

void fsm_ctx_destroy(fsm_ctx* ctx) {
    if (!ctx) return;
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

void fsm_patterns_free(fsm_patterns* p) {
    if (!p) return;
    std::free(p->support);
    std::free(p->pat_off);
    std::free(p->set_off);
    std::free(p->items);
    std::free(p);
}

void fsm_rules_free(fsm_rules* r) {
    if (!r) return;
    std::free(r->support);
    std::free(r->confidence);
    std::free(r->ante_off);
    std::free(r->ante);
    std::free(r->cons_off);
    std::free(r->cons);
    std::free(r);
}

}  // extern "C"
