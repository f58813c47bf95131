/*
 * fsm.h — C ABI of the MI355X spark-fsm engine (libfsm.so).
 *
 * This is the drop-in boundary for the two hot-path entry points of the
 * reference (paths relative to /root/reference/src/main/scala/de/kp/spark/fsm):
 *
 *   SPADE.extractRDDPatterns(dataset: RDD[(Int,String)], support: Double,
 *                            dfs: Boolean = true, stats: Boolean = true)
 *       : List[de.kp.core.spade.Pattern]                       SPADE.scala:36
 *     -> fsm_db_from_spmf(ctx, FSM_MODE_SPADE, ...) + fsm_spade_mine(...)
 *
 *   TSR.extractRDDRules(dataset: RDD[(Int,String)], k: Int, minconf: Double)
 *       : List[de.kp.core.tsr.Rule]                            TSR.scala:31
 *     -> fsm_db_from_spmf(ctx, FSM_MODE_TSR, ...) + fsm_tsr_mine(...)
 *
 * The JVM side collects the RDD once (sids + SPMF lines) and hands plain
 * arrays across; see INTEGRATION.md for the JNI binding.  No C++ exception
 * crosses this boundary: every entry point returns 0 on success or a nonzero
 * FSM_E* code, with a message in fsm_last_error(ctx).  Parse errors that make
 * the reference throw (SPADE.scala:161-168,194; TSR.scala:41,135) return
 * FSM_EPARSE, which the Scala shim rethrows as a java.lang.Exception so that
 * TrainActor (TrainActor.scala:65-67) records FAILURE exactly as today.
 *
 * Ownership: input arrays are borrowed for the duration of the call; result
 * objects are owned by the library until freed.  Threading: calls block; a
 * context owns its HIP stream and device buffers; distinct contexts may be
 * used from distinct threads (the reference runs concurrent requests on one
 * SparkContext, RequestContext.scala:30).
 */
#ifndef SPARK_FSM_AMD_FSM_H
#define SPARK_FSM_AMD_FSM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSM_ABI_VERSION 7

/* status codes */
#define FSM_OK 0
#define FSM_EINVAL 1    /* invalid argument (null pointer, k < 1, bad mode, ...) */
#define FSM_EPARSE 2    /* input the reference would throw on (SPADE.scala:161-194, TSR.scala:41-135) */
#define FSM_EDEVICE 3   /* HIP runtime / kernel failure, or no usable gfx950 device */
#define FSM_ENOMEM 4    /* host or device allocation failed */
#define FSM_ECOMM 5     /* RCCL failure (multi-GPU) */
#define FSM_ELIMIT 6    /* input exceeds an engine limit (e.g. > 65536 eids per sequence) */

typedef struct fsm_ctx fsm_ctx;
typedef struct fsm_db fsm_db;

typedef enum { FSM_MODE_SPADE = 0, FSM_MODE_TSR = 1 } fsm_mode;

/* Host-side collectives, an alternative to RCCL for nranks > 1 (several ranks
 * on one GPU, or any host transport).  The first two are called collectively by
 * every rank with the same sizes and return 0 on success.  Buffers are host memory.
 *   allreduce_u32: buf[0..n) <- element-wise sum over ranks (in place)
 *   allgather:     recv[r*bytes .. (r+1)*bytes) <- rank r's send[0..bytes)
 *   fetch_add:     (optional, NULL = none) NOT collective: atomically adds inc to
 *                  the shared counter `key` (0 before its first add) and returns
 *                  its previous value, or -1 on failure.  The work-stealing claim of
 *                  the sharded SPADE lattice; without it the ranks
 *                  split the classes by a static plan.  Keys are never reused.  */
typedef struct {
    void* user;
    int (*allreduce_u32)(void* user, uint32_t* buf, int64_t n);
    int (*allgather)(void* user, const void* send, void* recv, int64_t bytes);
    int64_t (*fetch_add)(void* user, int64_t key, int64_t inc);
} fsm_host_comm;

#define FSM_MAX_DEVICES 16

/* Device selection (1, 2, 4 or 8 GPUs).  Two ways to shard a mine:
 *  - in-process (the drop-in's way: SPADE.scala:132-133 and TSR.scala:102-103 run on
 *    one driver thread): ndevices > 1 makes ONE context that drives ndevices ranks,
 *    rank r on HIP device devices[r] with its own stream, pool and DB replica, one host
 *    thread per rank, collectives through host memory inside the library.  Every call
 *    on the context is one call for the caller; the result is the whole mine's.  A
 *    device may repeat (several ranks on one GPU);
 *  - one process per GPU (torch.distributed launches): nranks > 1, rank, and RCCL over
 *    unique_id or host_comm callbacks; each process gets the complete result.
 * ndevices <= 1 with nranks <= 1 is the single-GPU context on `device`. */
typedef struct {
    int32_t device;          /* local HIP device ordinal (ndevices <= 1) */
    int32_t nranks;          /* 1: single GPU; >1: sharded over ranks, one process per GPU */
    int32_t rank;            /* this process's rank in [0, nranks) */
    int32_t verbose;         /* 1: per-level trace on stderr */
    uint8_t unique_id[128];  /* RCCL unique id (fsm_comm_unique_id on rank 0), nranks > 1 */
    int64_t mem_budget;      /* device bytes for lattice frontier slabs; 0 = 1/2 of free HBM (divided
                                among the in-process ranks that share a device) */
    const fsm_host_comm* host_comm; /* nranks > 1: NULL = RCCL over unique_id, else these callbacks
                                       (must outlive the context) */
    int32_t ndevices;        /* > 1: in-process ranks on devices[0..ndevices) (nranks must be <= 1).
                                The DB is parsed once (rank 0) and copied device to device to the
                                other ranks.  A call waits at most FSM_COMM_TIMEOUT_S (default 300)
                                for a rank, then returns FSM_ECOMM */
    int32_t devices[FSM_MAX_DEVICES]; /* HIP ordinals of the in-process ranks */
} fsm_opts;

/* SPADE result: the patterns of List[Pattern] in CSR form.  Pattern p has
 * itemsets set_off[pat_off[p]] .. set_off[pat_off[p+1]]; itemset s has items
 * items[set_off[s]] .. items[set_off[s+1]] in ascending order.  Pattern order is
 * the engine's discovery order (the reference's is also discovery order). */
typedef struct {
    int64_t n;
    int32_t* support;        /* absolute support (#sequence ids) */
    int64_t* pat_off;        /* [n+1] */
    int64_t* set_off;        /* [n_sets+1] */
    int32_t* items;          /* [n_items] */
    int64_t n_sets;
    int64_t n_items;
    int64_t total;           /* sequences.count() of the input (SPADE.scala:46) */
    int32_t minsup;          /* absolute threshold max(1, ceil(support*total)) */
} fsm_patterns;

/* TSR result: the rules of List[Rule] (getItemset1/getItemset2,
 * getAbsoluteSupport, getConfidence, TSRActor.scala:55-59). */
typedef struct {
    int64_t n;
    int32_t* support;        /* getAbsoluteSupport */
    double* confidence;      /* getConfidence */
    int64_t* ante_off;       /* [n+1] */
    int32_t* ante;           /* getItemset1 */
    int64_t* cons_off;       /* [n+1] */
    int32_t* cons;           /* getItemset2 */
    int64_t total;           /* number of input sequences (TSRActor.scala:52) */
    int32_t final_minsup;
} fsm_rules;

/* Replaces algorithm.printStatistics() (SPADE.scala:136). */
typedef struct {
    int64_t joins;              /* candidate id-list joins per SURVEY A.2 (incl. infrequent) */
    int64_t patterns;           /* frequent patterns found */
    int64_t classes;            /* prefix equivalence classes processed */
    int64_t batches;            /* class batches (kernel rounds) */
    int64_t entries;            /* class-row entries streamed by the count kernel */
    int64_t bytes_join_equiv;   /* sum 12*(|Li|+|Lj|) + 12*|Lout| */
    int64_t bytes_streamed;     /* bytes the count+emit kernels read/write once per entry */
    int64_t expansions;         /* TSR: expandL + expandR evaluations */
    int64_t rules;              /* TSR: rules returned */
    double ms_flatten;          /* host parse + flatten (fsm_db_*) */
    double ms_upload;           /* host -> HBM copy of the flattened DB */
    double ms_f1;               /* SPADE: F1 histogram + root row filter */
    double ms_f2;               /* SPADE: root pair-count matrix (F2) */
    double ms_lattice;          /* SPADE: class batches below the root */
    double ms_mine;             /* whole fsm_*_mine call */
    double ms_count_kernel;     /* device time of the class pair-count kernel */
    double ms_emit_kernel;      /* device time of the child-row emission kernel */
    int64_t count_launches;
    int64_t mask_words;         /* W: u64 words per eid mask of this DB */
    int64_t bytes_count_alg;    /* count kernel algorithmic bytes: entries * (12 + 8W) */
    double ms_gpu_wait;         /* SPADE: host time blocked on the stream during F1/F2/lattice */
    double ms_output;           /* SPADE: host build of the pattern CSR */
    int64_t joins_root;         /* SPADE: A.2 candidate joins of the root class, F^2 + F(F-1)/2 (part of joins) */
    int64_t root_keys;          /* SPADE: non-empty (sequence, frequent-item pair) joins the root F2 counted */
    int64_t pair_tests;         /* SPADE: (entry, partner) join tests executed by the class count kernels */
    int64_t root_entries;       /* SPADE: (frequent item, sequence) entries of the root class (F2 input) */
    int64_t k0_device;          /* 1: the last fsm_db_* built the DB on the GPU (K0), 0: host flatten + upload */
    int64_t exp_domain;         /* TSR: sids expanded over (sum over expansions of |sids(X u Y)|) */
    int64_t exp_entries;        /* TSR: row entries read by the expansions */
    int64_t exp_bitmap_bytes;   /* TSR: sid-bitmap operand bytes ANDed by the expansions */
    /* this rank's own share of a sharded mine (not summed over ranks) */
    int64_t rank_claims;        /* SPADE: work units (first-level classes / sub-classes) this rank claimed */
    int64_t rank_root_owned;    /* SPADE: root entries this rank joined as the owner (F2 keys + root emit) */
    int64_t rank_root_slab;     /* SPADE: root entries this rank wrote to a root slab (0: DB-direct root) */
    int64_t rank_units;         /* TSR: expansion rule slots this rank counted */
    /* DB build (kept across mines) */
    int64_t db_parses;          /* passes over the caller's input of the last fsm_db_* (1; a group's DB is
                                   parsed once on rank 0, every other rank copies the resident arrays) */
    int64_t db_replicas;        /* group DBs: rank replicas made by device-to-device copy */
    int64_t tsr_ring_waits;     /* TSR: launches in flight finished early to free their kept-row ring
                                   positions before a later launch overwrote them */
} fsm_stats;

/* Per-kernel device time of the last fsm_*_mine call (HIP events on the
 * context's stream) with the kernel's algorithmic bytes: the
 * numbers bench.py's roofline is computed from. */
typedef struct {
    char name[40];
    int64_t launches;
    int64_t alg_bytes;          /* algorithmic HBM bytes over all launches (the kernel's own layout) */
    double ms;                  /* summed device time over all launches */
    int64_t survey_bytes;       /* the same work priced in SURVEY §8(d) units (12-B (sid, mask) id-list
                                   entries for SPADE, 8 B per scanned position for TSR); 0 = not priced */
} fsm_kernel_stat;

int fsm_abi_version(void);
/* RCCL unique id for fsm_opts.unique_id (call on rank 0, broadcast the bytes). */
int fsm_comm_unique_id(uint8_t out[128]);
/* Multi-GPU work plan (pure host, deterministic): largest-first assignment of
 * n work units with estimated volumes to the least-loaded of nranks ranks.
 * The engine shards SPADE's first-level prefix classes with it. */
int fsm_shard_plan(const uint64_t* volume, int64_t n, int32_t nranks, int32_t* owner);
/* Collective self-test of the nranks > 1 plumbing (all-reduce, all-gather of
 * ragged blobs, the work-stealing counter) on the context-free transport of opts;
 * no GPU compute when opts->host_comm is set.  With opts->ndevices > 1 the test runs
 * the in-process transport on ndevices host threads (no GPU at all).  0 = every rank
 * saw the expected data. */
int fsm_comm_selftest(const fsm_opts* opts);

int fsm_ctx_create(const fsm_opts* opts, fsm_ctx** out);
void fsm_ctx_destroy(fsm_ctx* ctx);
const char* fsm_last_error(const fsm_ctx* ctx);
int fsm_get_stats(const fsm_ctx* ctx, fsm_stats* out);
/* Copies up to max entries; *n = number available. */
int fsm_get_kernel_stats(const fsm_ctx* ctx, fsm_kernel_stat* out, int32_t max, int32_t* n);

/* Flatten an SPMF-format dataset (one line per sequence id, as produced by
 * SPMFHandler.sequence2SPMF) once and upload it to HBM.  mode selects the
 * reference parser: SPADE.scala:145-212 or TSR.scala:41,109-143. */
int fsm_db_from_spmf(fsm_ctx* ctx, int32_t mode, const int32_t* sids, const char* const* lines,
                     const int64_t* lens, int64_t n, fsm_db** out);
/* Pre-tokenized variant: sequence r has tokens tokens[seq_off[r] .. seq_off[r+1]]
 * where -1 ends an itemset, -2 ends the sequence, other values are items
 * (implicit timestamps 1,2,3,...). */
int fsm_db_from_tokens(fsm_ctx* ctx, int32_t mode, const int32_t* sids, const int64_t* seq_off,
                       const int64_t* tokens, int64_t n, fsm_db** out);
void fsm_db_free(fsm_db* db);

/* Host copy of a flattened DB as it sits in HBM (verification and debugging:
 * the device-built DB is compared byte for byte with the host flatten's).
 * SPADE: rows = distinct sequence ids, item = dense ids (ascending value
 * order, item_val maps them back), mask = mask_words u64 eid bits per entry.
 * TSR: rows = sequences, first / last = itemset indexes.  Library-owned until
 * fsm_db_image_free. */
typedef struct {
    int32_t mode;
    int32_t mask_words;
    int64_t rows;
    int64_t entries;
    int64_t items;
    int64_t max_occ;            /* SPADE: closed item tokens of the longest row */
    uint32_t* row_off;          /* [rows+1] */
    uint32_t* item;             /* [entries] */
    uint64_t* mask;             /* SPADE: [entries * mask_words] */
    uint32_t* first;            /* TSR: [entries] */
    uint32_t* last;             /* TSR: [entries] */
    int32_t* item_val;          /* [items] */
} fsm_db_image;
int fsm_db_export(fsm_ctx* ctx, const fsm_db* db, fsm_db_image** out);
void fsm_db_image_free(fsm_db_image* img);

/* Native input conversion (util/SPMFBuilder.scala:27-198): a whole input file
 * image in one of the builder's formats -> the token arrays of
 * fsm_db_from_tokens (sid, seq_off, tokens; every item its own itemset as the
 * builder writes it, -1 / -2 separators), numbered 0, 1, 2 ... in file order
 * like SPMFBuilder.index, keeping the first `limit` sequences (take(limit):
 * 0 keeps none; < 0 keeps all, an extension).
 * FSM_FMT_INDEXED reads the builder's own "idx|sequence" output.  Malformed
 * input returns FSM_EPARSE (message in fsm_last_error(NULL)). */
#define FSM_FMT_SPMF 0
#define FSM_FMT_INDEXED 1
#define FSM_FMT_BMS 2
#define FSM_FMT_CSV 3
#define FSM_FMT_KOSARAK 4
#define FSM_FMT_SNAKE 5
typedef struct {
    int64_t n;                  /* sequences */
    int32_t* sids;              /* [n] */
    int64_t* seq_off;           /* [n+1] */
    int64_t* tokens;            /* [n_tokens] */
    int64_t n_tokens;
} fsm_token_db;
int fsm_ingest(int32_t format, const char* data, int64_t len, int64_t limit, fsm_token_db** out);
void fsm_token_db_free(fsm_token_db* t);

int fsm_spade_mine(fsm_ctx* ctx, fsm_db* db, double support, int32_t dfs, fsm_patterns** out);
void fsm_patterns_free(fsm_patterns* p);

int fsm_tsr_mine(fsm_ctx* ctx, fsm_db* db, int32_t k, double minconf, fsm_rules** out);
void fsm_rules_free(fsm_rules* r);

/* Result persistence (SPADEActor.scala:47-68, TSRActor.scala:52-71): the
 * mined CSR rendered in bulk as the documents the actors hand to their sinks.
 *   fsm_patterns_serialize: one SPMF serialize() line per pattern,
 *     "i j -1 k -1 | support\n" (SPADE.scala:111-122 / GpuPattern.serialize)
 *   fsm_patterns_json: json4s write(Patterns(List[Pattern(support, itemsets)]))
 *   fsm_rules_json: json4s write(Rules(List[Rule(antecedent, consequent,
 *     support, total, confidence)])), confidence as java.lang.Double.toString
 * *out is NUL-terminated, *len excludes the NUL; free with fsm_buffer_free.
 * Errors: fsm_last_error(NULL). */
int fsm_patterns_serialize(const fsm_patterns* p, char** out, int64_t* len);
int fsm_patterns_json(const fsm_patterns* p, char** out, int64_t* len);
int fsm_rules_json(const fsm_rules* r, char** out, int64_t* len);
void fsm_buffer_free(char* p);

/* Rule queries (FSMQuestor.scala:46-98, get:antecedent / get:consequent):
 * side 0 = antecedent, 1 = consequent; writes the indexes (ascending) of the
 * rules whose side's items all occur in items[0..n) to out_idx (capacity
 * r->n) and their count to *n_out. */
int fsm_rules_query(const fsm_rules* r, int32_t side, const int32_t* items, int64_t n, int64_t* out_idx,
                    int64_t* n_out);

#ifdef __cplusplus
}
#endif
#endif
