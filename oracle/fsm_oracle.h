/*
 * fsm_oracle.h — CPU restatement of spark-fsm's hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline. The product (libfsm.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" against the reference. The reference keeps
 * the mining arithmetic in the unvendored modules de.kp.core.spade /
 * de.kp.core.tsr (SPADE.scala:24, TSR.scala:24; no version pinned, absent
 * from pom.xml:27-116), has no tests and no fixtures, and
 * no JVM exists in this image. This restatement is pinned instead against the
 * published definitions by an independent brute-force enumerator
 * (oracle/brute.py) on the committed fixtures under tests/golden/.
 *
 * Semantics restated (file:line in /root/reference/src/main/scala/de/kp/spark/fsm):
 *   SPADE parse        SPADE.scala:145-212   (split(" "), <t> timestamps, -1/-2)
 *   SPADE F1 + filter  SPADE.scala:53-126    (distinct-sid support, ceil(support*total))
 *   SPADE lattice      SPADE.scala:132-135   [EXT: SpadeAlgorithm — Zaki 2001 definitions]
 *   TSR parse          TSR.scala:41,109-143  (all tokens toInt, -1 closes itemset)
 *   TSR vertical       TSR.scala:52-94       (first/last itemset index per (item,sid))
 *   TSR mining         TSR.scala:102-105     [EXT: TopSeqRules control flow, SURVEY A.3]
 */
#ifndef FSM_ORACLE_H
#define FSM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int64_t  n;          /* number of patterns */
    int32_t* support;    /* [n] */
    int64_t* pat_off;    /* [n+1] offsets into set_off */
    int64_t* set_off;    /* [n_sets+1] offsets into items */
    int32_t* items;      /* [n_items] */
    int64_t  n_sets;
    int64_t  n_items;
    int64_t  joins;      /* candidate joins evaluated (SURVEY A.2 unit) */
    int32_t  minsup;     /* absolute threshold used */
    int32_t  complete;   /* 0 if a time limit stopped the lattice early */
    double   seconds;    /* wall time of F1 build + lattice (after parse) */
    double   seconds_f1; /* of which the F1 vertical build + filter */
} oracle_patterns;

typedef struct {
    int64_t  n;
    int32_t* support;    /* [n] absolute support */
    double*  confidence; /* [n] */
    int64_t* ante_off;   /* [n+1] */
    int32_t* ante;       /* antecedent items */
    int64_t* cons_off;   /* [n+1] */
    int32_t* cons;       /* consequent items */
    int64_t  total;      /* number of input sequences */
    int64_t  expansions; /* expandL/expandR calls */
    int32_t  final_minsup;
    int32_t  complete;   /* 0 if a time limit stopped the mining early */
    double   seconds;    /* wall time of the pair phase + expansions (after parse and Vertical build) */
    int64_t  pairs;      /* item pairs (i < j, both >= minsup) evaluated in the pair phase */
} oracle_rules;

/* Returns 0 on success; on failure returns nonzero and writes a message to err. */
int oracle_spade(const int32_t* sids, const char* const* lines, const int64_t* lens, int64_t n,
                 double support, oracle_patterns** out, char* err, int errlen);
void oracle_patterns_free(oracle_patterns* p);
int oracle_spade_tokens(const int64_t* seq_off, const int64_t* tokens, int64_t n, double support,
                        double time_limit_s, oracle_patterns** out, char* err, int errlen);
/* Same, first-level classes mined by nthreads OpenMP threads (CPU baseline mode ii). */
int oracle_spade_tokens_mt(const int64_t* seq_off, const int64_t* tokens, int64_t n, double support,
                           double time_limit_s, int nthreads, oracle_patterns** out, char* err, int errlen);
/* only the first-level classes of rank % stride == 0 (bench.py's sampled CPU baseline) */
int oracle_spade_tokens_sample(const int64_t* seq_off, const int64_t* tokens, int64_t n, double support,
                               double time_limit_s, int nthreads, int64_t stride, oracle_patterns** out, char* err,
                               int errlen);

int oracle_tsr(const int32_t* sids, const char* const* lines, const int64_t* lens, int64_t n,
               int32_t k, double minconf, oracle_rules** out, char* err, int errlen);
int oracle_tsr_timed(const int32_t* sids, const char* const* lines, const int64_t* lens, int64_t n,
                     int32_t k, double minconf, double time_limit_s, oracle_rules** out, char* err, int errlen);
void oracle_rules_free(oracle_rules* r);

/* Every valid rule (conf >= minconf) with support >= t, by definition at a fixed
 * threshold (oracle/tsr_exhaustive.c; seed subtrees on nthreads OpenMP threads).
 * expansions = rule nodes with sup >= t visited, pairs = seed pairs, final_minsup = t. */
int oracle_tsr_all(const int64_t* seq_off, const int64_t* tokens, int64_t n, int32_t t, double minconf,
                   int nthreads, oracle_rules** out, char* err, int errlen);

/* Definitional point checks over a token stream (-1 / -2 separators). */
int64_t oracle_pattern_support(const int64_t* seq_off, const int64_t* tokens, int64_t n,
                               const int32_t* items, const int64_t* set_off, int64_t nsets);
void oracle_rule_support(const int64_t* seq_off, const int64_t* tokens, int64_t n, const int32_t* X,
                         int64_t nx, const int32_t* Y, int64_t ny, int64_t* sup_out, int64_t* nx_out);

#ifdef __cplusplus
}
#endif
#endif
