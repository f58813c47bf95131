/*
 * fsm_oracle.c — CPU restatement of spark-fsm's hot path (SPADE + TopSeqRules).
 *
 * TEST INFRASTRUCTURE ONLY (see fsm_oracle.h for the rules of use and for the
 * parity status: "parity unpinned" vs the reference, pinned to the published
 * definitions by oracle/brute.py). Deliberately simple and single-threaded:
 * it mirrors the reference's one-driver-thread mining (SPADE.scala:106,132-133;
 * TSR.scala:94,102-103) and doubles as the "port" CPU baseline in bench.py.
 *
 * Data structures follow the reference algorithms, not the GPU engine:
 *   SPADE: vertical id-lists of (sid, eid-bitmask) joined pairwise inside each
 *          prefix equivalence class, DFS (SpadeAlgorithm(support, dfs=true)).
 *   TSR:   per-rule tid sets + first/last occurrence arrays, horizontal
 *          position scans in expandL/expandR (SPMF TopSeqRules control flow).
 */
#define _POSIX_C_SOURCE 200809L
#include "fsm_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ utils */
#define VEC(T) struct { T* a; int64_t n, cap; }
#define VPUSH(v, x)                                                            \
    do {                                                                       \
        if ((v).n == (v).cap) {                                                \
            (v).cap = (v).cap ? 2 * (v).cap : 16;                              \
            (v).a = realloc((v).a, (size_t)(v).cap * sizeof(*(v).a));          \
        }                                                                      \
        (v).a[(v).n++] = (x);                                                  \
    } while (0)
#define VFREE(v) do { free((v).a); (v).a = NULL; (v).n = (v).cap = 0; } while (0)

static void set_err(char* err, int errlen, const char* fmt, ...) {
    if (!err || errlen <= 0) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err, (size_t)errlen, fmt, ap);
    va_end(ap);
}

typedef struct { const char* p; int64_t n; } tok_t;
typedef VEC(tok_t) tokvec;

/* java.lang.String.split(" ") with limit 0: split on every single space, drop
 * trailing empty strings; an input with no match is returned whole (so ""
 * yields [""] and " " yields []).  SPADE.scala:151, TSR.scala:41,111. */
static void java_split_space(const char* s, int64_t len, tokvec* out) {
    out->n = 0;
    if (len == 0) {
        tok_t t = {s, 0};
        VPUSH(*out, t);
        return;
    }
    int64_t start = 0;
    for (int64_t i = 0; i <= len; i++) {
        if (i == len || s[i] == ' ') {
            tok_t t = {s + start, i - start};
            VPUSH(*out, t);
            start = i + 1;
        }
    }
    while (out->n > 0 && out->a[out->n - 1].n == 0) out->n--;
}

/* Long.parseLong / Integer.parseInt (radix 10, ASCII digits). */
static int parse_java_long(const char* p, int64_t n, int64_t* out) {
    if (n <= 0) return -1;
    int neg = 0;
    int64_t i = 0;
    if (p[0] == '-' || p[0] == '+') {
        neg = p[0] == '-';
        i = 1;
        if (n == 1) return -1;
    }
    uint64_t lim = neg ? (uint64_t)INT64_MAX + 1u : (uint64_t)INT64_MAX;
    uint64_t v = 0;
    for (; i < n; i++) {
        char c = p[i];
        if (c < '0' || c > '9') return -1;
        uint64_t d = (uint64_t)(c - '0');
        if (v > (lim - d) / 10u) return -1;
        v = v * 10u + d;
    }
    *out = neg ? (int64_t)(0u - v) : (int64_t)v;
    return 0;
}

static int parse_java_int(const char* p, int64_t n, int32_t* out) {
    int64_t v;
    if (n <= 0) return -1;
    if (parse_java_long(p, n, &v)) return -1;
    if (v < INT32_MIN || v > INT32_MAX) return -1;
    *out = (int32_t)v;
    return 0;
}

static int tok_eq(tok_t t, const char* lit) {
    int64_t l = (int64_t)strlen(lit);
    return t.n == l && memcmp(t.p, lit, (size_t)l) == 0;
}

static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

static int64_t lower_bound_i32(const int32_t* a, int64_t n, int32_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* ============================================================== SPADE === */

typedef struct { int32_t sid, item, ts; } reg_t; /* one registerBit(sid, ts) for item */
typedef VEC(reg_t) regvec;
typedef VEC(int32_t) i32vec;

/* SPADE.newSequence (SPADE.scala:145-212) + the seqOp registrations
 * (SPADE.scala:53-102): emits one reg_t per item of every CLOSED itemset. */
static int spade_parse_line(int32_t sid, const char* s, int64_t len, tokvec* toks, regvec* regs,
                            i32vec* cur, char* err, int errlen) {
    java_split_space(s, len, toks);
    int64_t ts_state = -1;      /* `var timestamp:Long = -1` (:153) */
    int64_t cur_ts = 0;         /* Itemset default timestamp [EXT; assumed 0] */
    cur->n = 0;
    for (int64_t t = 0; t < toks->n; t++) {
        tok_t tk = toks->a[t];
        if (tk.n == 0) {        /* "".codePointAt(0) throws (:161) */
            set_err(err, errlen, "SPADE parse: empty token in sequence sid=%d "
                    "(StringIndexOutOfBoundsException at SPADE.scala:161)", sid);
            return -1;
        }
        if (tk.p[0] == '<') {   /* timestamp token (:161-169) */
            int64_t v;
            if (tk.n < 2 || parse_java_long(tk.p + 1, tk.n - 2, &v)) {
                set_err(err, errlen, "SPADE parse: bad timestamp token '%.*s' sid=%d "
                        "(SPADE.scala:166-168)", (int)(tk.n > 40 ? 40 : tk.n), tk.p, sid);
                return -1;
            }
            ts_state = v;
            cur_ts = v;
        } else if (tok_eq(tk, "-1")) { /* end of itemset (:171-183) */
            int64_t next = (int64_t)((uint64_t)cur_ts + 1u);
            for (int64_t i = 0; i < cur->n; i++) {
                int32_t ts32 = (int32_t)(uint32_t)(uint64_t)cur_ts; /* timestamp.toInt (:74,:90) */
                if (ts32 < 0) {
                    set_err(err, errlen, "SPADE: negative timestamp %d for sid=%d "
                            "(IDListBitmap.registerBit, SPADE.scala:74,90)", ts32, sid);
                    return -1;
                }
                reg_t r = {sid, cur->a[i], ts32};
                VPUSH(*regs, r);
            }
            cur->n = 0;
            cur_ts = next;
            ts_state = (int64_t)((uint64_t)ts_state + 1u);
        } else if (tok_eq(tk, "-2")) { /* end of sequence: no-op (:185-188) */
        } else {                       /* item (:190-205) */
            int32_t item;
            if (parse_java_int(tk.p, tk.n, &item)) {
                set_err(err, errlen, "SPADE parse: bad item token '%.*s' sid=%d "
                        "(NumberFormatException at SPADE.scala:194)", (int)(tk.n > 40 ? 40 : tk.n), tk.p, sid);
                return -1;
            }
            VPUSH(*cur, item);
            if (ts_state < 0) {
                ts_state = 1;
                cur_ts = 1;
            }
        }
    }
    /* items after the last "-1" are never added to the sequence */
    return 0;
}

static int cmp_reg(const void* a, const void* b) {
    const reg_t* x = a;
    const reg_t* y = b;
    if (x->sid != y->sid) return x->sid < y->sid ? -1 : 1;
    if (x->ts != y->ts) return x->ts < y->ts ? -1 : 1;
    if (x->item != y->item) return x->item < y->item ? -1 : 1;
    return 0;
}

typedef struct { int64_t n, cap; int32_t* sid; uint64_t* mask; } ilist; /* mask: n*W words */

enum { SEQ = 0, ITEMSET = 1 };

typedef struct { int32_t parent, item, type, support; } pnode;
typedef VEC(pnode) nodevec;

typedef struct {
    int32_t node;
    int32_t item;
    int32_t type;
    ilist L;
} member;
typedef VEC(member) membervec;

typedef struct {
    int W;
    int32_t minsup;
    int64_t joins;
    nodevec nodes;
    double deadline;   /* CLOCK_MONOTONIC seconds; 0 = none */
    int stopped;
} spade_ctx;

static double mono_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void ilist_push(ilist* l, int W, int32_t sid, const uint64_t* m) {
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 16;
        l->sid = realloc(l->sid, (size_t)l->cap * sizeof(int32_t));
        l->mask = realloc(l->mask, (size_t)l->cap * (size_t)W * sizeof(uint64_t));
    }
    l->sid[l->n] = sid;
    memcpy(l->mask + (size_t)l->n * W, m, (size_t)W * sizeof(uint64_t));
    l->n++;
}

static void ilist_free(ilist* l) {
    free(l->sid);
    free(l->mask);
    memset(l, 0, sizeof(*l));
}

static int first_bit(const uint64_t* m, int W) {
    for (int w = 0; w < W; w++)
        if (m[w]) return w * 64 + __builtin_ctzll(m[w]);
    return -1;
}

/* IDListBitmap join [EXT]: sid merge; temporal keeps the bits of b strictly
 * after the first bit of a (P x -> y), equality keeps a & b (P (x y)). */
static void join(const ilist* a, const ilist* b, int W, int temporal, ilist* out) {
    int64_t i = 0, j = 0;
    uint64_t res[1024]; /* W <= 1024: 65,536 distinct timestamps per sequence */
    out->n = 0;
    while (i < a->n && j < b->n) {
        int32_t sa = a->sid[i], sb = b->sid[j];
        if (sa < sb) { i++; continue; }
        if (sb < sa) { j++; continue; }
        const uint64_t* ma = a->mask + (size_t)i * W;
        const uint64_t* mb = b->mask + (size_t)j * W;
        uint64_t any = 0;
        if (temporal) {
            int lo = first_bit(ma, W);
            int lw = lo >> 6, lb = lo & 63;
            for (int w = 0; w < W; w++) {
                uint64_t v = mb[w];
                if (w < lw) v = 0;
                else if (w == lw) v = (lb == 63) ? 0 : (v & (~0ull << (lb + 1)));
                res[w] = v;
                any |= v;
            }
        } else {
            for (int w = 0; w < W; w++) {
                res[w] = ma[w] & mb[w];
                any |= res[w];
            }
        }
        if (any) ilist_push(out, W, sa, res);
        i++;
        j++;
    }
}

static void try_candidate(spade_ctx* c, const member* mi, const member* mj, int temporal,
                          membervec* child) {
    member m;
    memset(&m, 0, sizeof(m));
    if (c->stopped) return;
    if (c->deadline > 0 && (c->joins & 255) == 0 && mono_s() > c->deadline) {
        c->stopped = 1;
        return;
    }
    c->joins++;
    join(&mi->L, &mj->L, c->W, temporal, &m.L);
    if (m.L.n >= c->minsup) {
        pnode nd = {mi->node, mj->item, temporal ? SEQ : ITEMSET, (int32_t)m.L.n};
        m.node = (int32_t)c->nodes.n;
        m.item = mj->item;
        m.type = nd.type;
        VPUSH(c->nodes, nd);
        VPUSH(*child, m);
    } else {
        ilist_free(&m.L);
    }
}

/* Equivalence-class DFS (SURVEY.md Appendix A.2 candidate rules). */
static void process_class(spade_ctx* c, member* m, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        membervec child = {0};
        for (int64_t j = 0; j < n; j++) {
            if (m[i].type == SEQ && m[j].type == SEQ) {
                try_candidate(c, &m[i], &m[j], 1, &child);          /* P->x->y   */
                if (m[j].item > m[i].item)
                    try_candidate(c, &m[i], &m[j], 0, &child);      /* P->(x y)  */
            } else if (m[i].type == ITEMSET && m[j].type == ITEMSET) {
                if (m[j].item > m[i].item)
                    try_candidate(c, &m[i], &m[j], 0, &child);      /* P(x y)    */
            } else if (m[i].type == ITEMSET && m[j].type == SEQ) {
                try_candidate(c, &m[i], &m[j], 1, &child);          /* P x -> y  */
            }
        }
        if (child.n && !c->stopped) process_class(c, child.a, child.n);
        for (int64_t k = 0; k < child.n; k++) ilist_free(&child.a[k].L);
        VFREE(child);
    }
}

static oracle_patterns* build_patterns(const nodevec* nodes) {
    oracle_patterns* p = calloc(1, sizeof(*p));
    int64_t n = nodes->n;
    p->n = n;
    p->support = malloc((size_t)(n ? n : 1) * sizeof(int32_t));
    p->pat_off = malloc((size_t)(n + 1) * sizeof(int64_t));
    i32vec items = {0};
    VEC(int64_t) set_off = {0};
    i32vec path = {0};
    i32vec ptype = {0};
    VPUSH(set_off, 0);
    p->pat_off[0] = 0;
    for (int64_t k = 0; k < n; k++) {
        path.n = ptype.n = 0;
        for (int32_t q = (int32_t)k; q >= 0; q = nodes->a[q].parent) {
            VPUSH(path, nodes->a[q].item);
            VPUSH(ptype, nodes->a[q].type);
        }
        /* walk root -> leaf; a SEQ node opens a new itemset */
        for (int64_t t = path.n - 1; t >= 0; t--) {
            if (ptype.a[t] == SEQ && t != path.n - 1) VPUSH(set_off, items.n);
            VPUSH(items, path.a[t]);
        }
        VPUSH(set_off, items.n);
        p->support[k] = nodes->a[k].support;
        p->pat_off[k + 1] = set_off.n - 1;
    }
    p->items = items.a;
    p->n_items = items.n;
    p->set_off = set_off.a;
    p->n_sets = set_off.n - 1;
    VFREE(path);
    VFREE(ptype);
    return p;
}

static int spade_core(regvec* regs, int64_t n, double support, double time_limit_s, int nthreads, int64_t stride,
                      oracle_patterns** out, char* err, int errlen);

int oracle_spade(const int32_t* sids, const char* const* lines, const int64_t* lens, int64_t n,
                 double support, oracle_patterns** out, char* err, int errlen) {
    *out = NULL;
    regvec regs = {0};
    tokvec toks = {0};
    i32vec cur = {0};
    int rc = 0;
    for (int64_t r = 0; r < n; r++) {
        if (sids[r] < 0) {
            set_err(err, errlen, "SPADE: negative sequence id %d (IDListBitmap sid index)", sids[r]);
            rc = -1;
            goto done;
        }
        if (spade_parse_line(sids[r], lines[r], lens[r], &toks, &regs, &cur, err, errlen)) {
            rc = -1;
            goto done;
        }
    }
    rc = spade_core(&regs, n, support, 0.0, 1, 1, out, err, errlen);
done:
    VFREE(regs);
    VFREE(toks);
    VFREE(cur);
    return rc;
}

/* Token-stream front end (sid = record index, implicit timestamps 1,2,3..);
 * time_limit_s > 0 stops the lattice after that many seconds (bounded CPU
 * baseline sample: joins done / seconds). */
int oracle_spade_tokens(const int64_t* seq_off, const int64_t* tokens, int64_t n, double support,
                        double time_limit_s, oracle_patterns** out, char* err, int errlen) {
    return oracle_spade_tokens_mt(seq_off, tokens, n, support, time_limit_s, 1, out, err, errlen);
}

/* All-cores variant (SURVEY.md §8d CPU mode ii): the first-level classes [x]
 * are independent DFS roots, processed by nthreads OpenMP threads (dynamic
 * schedule, one class per grab).  Each class's nodes are renumbered after the
 * root nodes in class order, so a complete run returns exactly the pattern
 * list of the sequential DFS. */
/* Class-stride sample (bench.py's CPU baseline): only the first-level classes
 * [x] with rank(x) % stride == 0 are mined (their root joins and their whole
 * subtrees), so the joins/s of a bounded run is an unbiased sample of every
 * depth of the lattice rather than its first classes only.  stride 1 = the
 * complete mine. */
int oracle_spade_tokens_sample(const int64_t* seq_off, const int64_t* tokens, int64_t n, double support,
                               double time_limit_s, int nthreads, int64_t stride, oracle_patterns** out, char* err,
                               int errlen) {
    *out = NULL;
    regvec regs = {0};
    for (int64_t r = 0; r < n; r++) {
        /* items of closed itemsets only */
        int64_t lastm = -1;
        for (int64_t q = seq_off[r]; q < seq_off[r + 1]; q++) if (tokens[q] == -1) lastm = q;
        int32_t ts = 1;
        for (int64_t q = seq_off[r]; q < lastm; q++) {
            int64_t t = tokens[q];
            if (t == -1) { ts++; continue; }
            if (t == -2) continue;
            reg_t rg = {(int32_t)r, (int32_t)t, ts};
            VPUSH(regs, rg);
        }
    }
    int rc = spade_core(&regs, n, support, time_limit_s, nthreads < 1 ? 1 : nthreads, stride < 1 ? 1 : stride, out,
                        err, errlen);
    VFREE(regs);
    return rc;
}

int oracle_spade_tokens_mt(const int64_t* seq_off, const int64_t* tokens, int64_t n, double support,
                           double time_limit_s, int nthreads, oracle_patterns** out, char* err, int errlen) {
    return oracle_spade_tokens_sample(seq_off, tokens, n, support, time_limit_s, nthreads, 1, out, err, errlen);
}

/* Top level of process_class with one OpenMP task per first-level class.
 * Task i owns a private ctx whose node table starts with copies of the root
 * nodes (so parents < nroot are root nodes), then the merge appends each
 * task's own nodes in i order, remapping parents. */
static void process_root_mt(spade_ctx* c, member* m, int64_t n, int nthreads, int64_t stride) {
    const int64_t nroot = c->nodes.n;
    spade_ctx* tc = calloc((size_t)(n ? n : 1), sizeof(spade_ctx));
    volatile int stop = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (int64_t i = 0; i < n; i++) {
        spade_ctx* t = &tc[i];
        t->W = c->W;
        t->minsup = c->minsup;
        t->deadline = c->deadline;
        if (stop) { t->stopped = 1; continue; }
        if (i % stride != 0) continue;  /* class-stride sample */
        for (int64_t k = 0; k < nroot; k++) VPUSH(t->nodes, c->nodes.a[k]);
        membervec child = {0};
        for (int64_t j = 0; j < n; j++) {  /* root members are all SEQ (P = {}) */
            try_candidate(t, &m[i], &m[j], 1, &child);
            if (m[j].item > m[i].item) try_candidate(t, &m[i], &m[j], 0, &child);
        }
        if (child.n && !t->stopped) process_class(t, child.a, child.n);
        for (int64_t k = 0; k < child.n; k++) ilist_free(&child.a[k].L);
        VFREE(child);
        if (t->stopped) stop = 1;
    }
    for (int64_t i = 0; i < n; i++) {
        spade_ctx* t = &tc[i];
        const int64_t base = c->nodes.n;
        for (int64_t k = nroot; k < t->nodes.n; k++) {
            pnode nd = t->nodes.a[k];
            if (nd.parent >= nroot) nd.parent = (int32_t)(base + (nd.parent - nroot));
            VPUSH(c->nodes, nd);
        }
        c->joins += t->joins;
        if (t->stopped) c->stopped = 1;
        VFREE(t->nodes);
    }
    free(tc);
}

static int spade_core(regvec* regsp, int64_t n, double support, double time_limit_s, int nthreads, int64_t stride,
                      oracle_patterns** out, char* err, int errlen) {
    regvec regs = *regsp;
    int rc = 0;
    {
        spade_ctx c;
        memset(&c, 0, sizeof(c));
        const double t_start = mono_s();
        if (time_limit_s > 0) c.deadline = t_start + time_limit_s;
        /* minsupp = Math.ceil(support * total) (SPADE.scala:113); the lattice
         * needs at least one occurrence, so the absolute threshold is >= 1. */
        double ms = ceil(support * (double)n);
        int empty = !(ms == ms) || ms > (double)INT32_MAX;
        c.minsup = empty ? INT32_MAX : (ms < 1.0 ? 1 : (int32_t)ms);

        qsort(regs.a, (size_t)regs.n, sizeof(reg_t), cmp_reg);
        regsp->a = regs.a; /* (sorted in place) */
        /* dense sid index + eid rank per sid; W = words per eid mask */
        int64_t nreg = regs.n;
        int32_t* eid = malloc((size_t)(nreg ? nreg : 1) * sizeof(int32_t));
        int32_t* sidx = malloc((size_t)(nreg ? nreg : 1) * sizeof(int32_t));
        int32_t nsid = 0, maxE = 0;
        for (int64_t a = 0; a < nreg;) {
            int64_t b = a;
            while (b < nreg && regs.a[b].sid == regs.a[a].sid) b++;
            int32_t e = -1, last_ts = 0;
            for (int64_t q = a; q < b; q++) {
                if (q == a || regs.a[q].ts != last_ts) e++;
                last_ts = regs.a[q].ts;
                eid[q] = e;
                sidx[q] = nsid;
            }
            if (e + 1 > maxE) maxE = e + 1;
            nsid++;
            a = b;
        }
        int W = (maxE + 63) / 64;
        if (W < 1) W = 1;
        if (W > 1024) {
            set_err(err, errlen, "SPADE oracle: sequence with %d distinct timestamps exceeds 65536", maxE);
            free(eid);
            free(sidx);
            rc = -1;
            goto done;
        }
        c.W = W;
        /* items -> dense, ascending by value */
        int32_t* uitems = malloc((size_t)(nreg ? nreg : 1) * sizeof(int32_t));
        for (int64_t q = 0; q < nreg; q++) uitems[q] = regs.a[q].item;
        qsort(uitems, (size_t)nreg, sizeof(int32_t), cmp_i32);
        int64_t nitems = 0;
        for (int64_t q = 0; q < nreg; q++)
            if (q == 0 || uitems[q] != uitems[q - 1]) uitems[nitems++] = uitems[q];
        ilist* vert = calloc((size_t)(nitems ? nitems : 1), sizeof(ilist));
        uint64_t m[1024];
        /* F1 vertical build (SPADE.scala:53-106): one id-list per distinct item */
        for (int64_t a = 0; a < nreg;) {
            int64_t b = a;
            while (b < nreg && regs.a[b].sid == regs.a[a].sid) b++;
            /* per item within this sid: OR the eid bits (regs sorted by ts) */
            for (int64_t q = a; q < b; q++) {
                int64_t it = lower_bound_i32(uitems, nitems, regs.a[q].item);
                ilist* L = &vert[it];
                if (L->n > 0 && L->sid[L->n - 1] == sidx[q]) {
                    L->mask[(size_t)(L->n - 1) * W + (eid[q] >> 6)] |= 1ull << (eid[q] & 63);
                } else {
                    memset(m, 0, sizeof(uint64_t) * (size_t)W);
                    m[eid[q] >> 6] |= 1ull << (eid[q] & 63);
                    ilist_push(L, W, sidx[q], m);
                }
            }
            a = b;
        }
        /* F1 filter (SPADE.scala:113-126): support = distinct sids */
        membervec root = {0};
        for (int64_t it = 0; it < nitems; it++) {
            if (vert[it].n >= c.minsup && !empty) {
                member mm;
                memset(&mm, 0, sizeof(mm));
                pnode nd = {-1, uitems[it], SEQ, (int32_t)vert[it].n};
                mm.node = (int32_t)c.nodes.n;
                mm.item = uitems[it];
                mm.type = SEQ;
                mm.L = vert[it];
                VPUSH(c.nodes, nd);
                VPUSH(root, mm);
            } else {
                ilist_free(&vert[it]);
            }
        }
        free(vert);
        const double t_f1 = mono_s() - t_start;
        if (nthreads > 1 || stride > 1) process_root_mt(&c, root.a, root.n, nthreads, stride);
        else process_class(&c, root.a, root.n);
        for (int64_t k = 0; k < root.n; k++) ilist_free(&root.a[k].L);
        VFREE(root);
        oracle_patterns* p = build_patterns(&c.nodes);
        p->joins = c.joins;
        p->minsup = c.minsup;
        p->complete = !c.stopped;
        p->seconds = mono_s() - t_start;
        p->seconds_f1 = t_f1;
        *out = p;
        VFREE(c.nodes);
        free(uitems);
        free(eid);
        free(sidx);
    }
done:
    return rc;
}

void oracle_patterns_free(oracle_patterns* p) {
    if (!p) return;
    free(p->support);
    free(p->pat_off);
    free(p->set_off);
    free(p->items);
    free(p);
}

/* ================================================================ TSR === */

/* (sid, position) arrays sorted by sid, shared between rules by refcount. */
typedef struct {
    int refs;
    int64_t n;
    int32_t* sid;
    int32_t* pos;
} tidpos;

static tidpos* tidpos_new(int64_t cap) {
    tidpos* t = calloc(1, sizeof(tidpos));
    t->refs = 1;
    t->sid = malloc((size_t)(cap ? cap : 1) * sizeof(int32_t));
    t->pos = malloc((size_t)(cap ? cap : 1) * sizeof(int32_t));
    return t;
}
static void tidpos_release(tidpos* t) {
    if (t && --t->refs == 0) {
        free(t->sid);
        free(t->pos);
        free(t);
    }
}

/* A rule carries only its items, support and confidence while it waits in the
 * candidate heap; its tid state (I, J, common) is built from the items'
 * first / last lists when it is expanded and released right after (memory
 * follows the live candidates, not their tid sets: the 100K-sequence Kosarak
 * prefix registers ~10^8 candidates while minsup is still low). */
typedef struct rule {
    int32_t* X;       /* X and Y live in the same allocation, after the struct */
    int32_t nx;
    int32_t* Y;
    int32_t ny;
    int32_t sup;
    double conf;
    int expandLR;
    tidpos* I;        /* sids(X) with firstX (occurencesIfirst), while expanded */
    tidpos* J;        /* sids(Y) with lastY  (occurencesJlast), while expanded  */
    int32_t* common;  /* tidsIJ, sorted, while expanded */
    int64_t ncommon;
    int in_k;         /* still referenced by kRules */
    int in_cand;      /* still referenced by candidates */
} rule;

/* RuleG.compareTo [EXT, recalled]: support, |X|, |Y|, (int)(conf diff),
 * then X and Y lexicographically. */
static int rule_cmp(const rule* a, const rule* b) {
    if (a == b) return 0;
    if (a->sup != b->sup) return a->sup < b->sup ? -1 : 1;
    if (a->nx != b->nx) return a->nx < b->nx ? -1 : 1;
    if (a->ny != b->ny) return a->ny < b->ny ? -1 : 1;
    int c4 = (int)(a->conf - b->conf);
    if (c4) return c4;
    for (int i = 0; i < a->nx; i++)
        if (a->X[i] != b->X[i]) return a->X[i] < b->X[i] ? -1 : 1;
    for (int i = 0; i < a->ny; i++)
        if (a->Y[i] != b->Y[i]) return a->Y[i] < b->Y[i] ? -1 : 1;
    return 0;
}

typedef struct { rule** a; int64_t n, cap; int max; } heap; /* max=1: max-heap */

static int heap_before(const heap* h, const rule* x, const rule* y) {
    int c = rule_cmp(x, y);
    return h->max ? c > 0 : c < 0;
}
static void heap_push(heap* h, rule* r) {
    if (h->n == h->cap) {
        h->cap = h->cap ? 2 * h->cap : 64;
        h->a = realloc(h->a, (size_t)h->cap * sizeof(rule*));
    }
    int64_t i = h->n++;
    h->a[i] = r;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (!heap_before(h, h->a[i], h->a[p])) break;
        rule* t = h->a[i]; h->a[i] = h->a[p]; h->a[p] = t;
        i = p;
    }
}
static rule* heap_pop(heap* h) {
    if (!h->n) return NULL;
    rule* top = h->a[0];
    h->a[0] = h->a[--h->n];
    int64_t i = 0;
    for (;;) {
        int64_t l = 2 * i + 1, r = l + 1, b = i;
        if (l < h->n && heap_before(h, h->a[l], h->a[b])) b = l;
        if (r < h->n && heap_before(h, h->a[r], h->a[b])) b = r;
        if (b == i) break;
        rule* t = h->a[i]; h->a[i] = h->a[b]; h->a[b] = t;
        i = b;
    }
    return top;
}

typedef struct {
    int32_t k;
    double minconf;
    int32_t minsup;             /* minsuppRelative */
    int64_t nitems;             /* dense item count */
    int32_t* item_val;          /* dense -> item value (ascending) */
    tidpos** first;             /* per dense item: (sid, first index) */
    tidpos** last;              /* per dense item: (sid, last index)  */
    /* horizontal sequences: seq s -> itemsets -> dense items */
    int64_t nseq;
    int64_t* set_off;           /* [nseq+1] into itemset table */
    int64_t* item_off;          /* [nsets+1] into items */
    int32_t* items;             /* dense item ids */
    heap krules, cand;
    int64_t purge_at;           /* candidate count that triggers the next purge */
    int64_t expansions;
    /* scratch for expansions */
    int32_t* cnt_last_tid;
    i32vec* tids_of;
    i32vec touched;
} tsr_ctx;

static void rule_release_state(rule* r) {
    tidpos_release(r->I);
    tidpos_release(r->J);
    free(r->common);
    r->I = r->J = NULL;
    r->common = NULL;
}

/* A rule is freed as soon as neither kRules nor the candidates (nor the
 * expansion in progress, which holds in_cand) reference it: memory then
 * follows the live rules, not every rule ever made (the 100K-sequence
 * Kosarak prefix makes ~10^8 of them while minsup is still low). */
static void rule_maybe_free(rule* r) {
    if (r->in_k || r->in_cand) return;
    rule_release_state(r);
    free(r);
}

/* Candidates with sup < minsup can never be expanded (the expansion loop
 * stops at the first such pop, and minsup only rises), so dropping them
 * changes nothing: the remaining pop order is the comparator's total order. */
static void tsr_purge(tsr_ctx* c) {
    heap old = c->cand;
    c->cand.a = NULL;
    c->cand.n = c->cand.cap = 0;
    for (int64_t q = 0; q < old.n; q++) {
        rule* r = old.a[q];
        if (r->sup >= c->minsup) {
            heap_push(&c->cand, r);
        } else {
            r->in_cand = 0;
            rule_maybe_free(r);
        }
    }
    free(old.a);
    c->purge_at = 2 * c->cand.n > (1 << 20) ? 2 * c->cand.n : (1 << 20);
}

/* AlgoTopSeqRules.save [EXT, SURVEY A.3] */
static void tsr_save(tsr_ctx* c, rule* r) {
    heap_push(&c->krules, r);
    r->in_k = 1;
    if (c->krules.n > c->k) {
        if (r->sup > c->minsup) {
            do {
                rule* lower = heap_pop(&c->krules);
                if (!lower) break;
                lower->in_k = 0;
                if (lower != r) rule_maybe_free(lower);  /* r itself is registered next */
            } while (c->krules.n > c->k);
        }
        c->minsup = c->krules.a[0]->sup;
    }
}

static void tsr_register(tsr_ctx* c, rule* r, int lr) {
    r->expandLR = lr;
    r->in_cand = 1;
    heap_push(&c->cand, r);
    if (c->cand.n > c->purge_at) tsr_purge(c);
}

static rule* rule_new(tsr_ctx* c, const int32_t* X, int32_t nx, int32_t xadd, const int32_t* Y,
                      int32_t ny, int32_t yadd) {
    (void)c;
    const int32_t mx = nx + (xadd >= 0), my = ny + (yadd >= 0);
    rule* r = calloc(1, sizeof(rule) + (size_t)(mx + my) * sizeof(int32_t));
    r->nx = mx;
    r->ny = my;
    r->X = (int32_t*)(r + 1);
    r->Y = r->X + mx;
    memcpy(r->X, X, (size_t)nx * sizeof(int32_t));
    memcpy(r->Y, Y, (size_t)ny * sizeof(int32_t));
    if (xadd >= 0) r->X[nx] = xadd;
    if (yadd >= 0) r->Y[ny] = yadd;
    return r;
}

/* position lookup in a (sid,pos) array; returns -1 if absent */
static int32_t tp_get(const tidpos* t, int32_t sid) {
    int64_t i = lower_bound_i32(t->sid, t->n, sid);
    return (i < t->n && t->sid[i] == sid) ? t->pos[i] : -1;
}

static void scan_reset(tsr_ctx* c) {
    for (int64_t q = 0; q < c->touched.n; q++) {
        int32_t it = c->touched.a[q];
        c->tids_of[it].n = 0;
        c->cnt_last_tid[it] = -1;
    }
    c->touched.n = 0;
}

static void scan_add(tsr_ctx* c, int32_t it, int32_t tid) {
    if (c->cnt_last_tid[it] == tid) return;  /* HashSet semantics per c */
    if (c->tids_of[it].n == 0) VPUSH(c->touched, it);
    c->cnt_last_tid[it] = tid;
    VPUSH(c->tids_of[it], tid);
}

/* containsLEXPlus(itemset, c): true if c in itemset or some element > c. */
static int contains_lex_plus(const int32_t* s, int32_t n, int32_t c) {
    for (int32_t i = 0; i < n; i++)
        if (s[i] >= c) return 1;
    return 0;
}
/* containsLEX(itemset, c): true if c in itemset (sorted). */
static int contains_lex(const int32_t* s, int32_t n, int32_t c) {
    for (int32_t i = 0; i < n; i++) {
        if (s[i] == c) return 1;
        if (s[i] > c) return 0;
    }
    return 0;
}

/* tidsIJ of a pair-phase rule, made when the rule is first expanded (the pair
 * phase keeps no per-rule sid lists: at minsup 1 there are ~10^8 such rules on
 * the 100K-sequence Kosarak prefix): the sids of I (sids(X), firstX) and J
 * (sids(Y), lastY) with firstX < lastY, ascending. */
/* sids(S) with the max (first lists) or min (last lists) position over the items of S */
static tidpos* tid_intersect(tidpos* const* lists, const int32_t* S, int32_t n, int take_max) {
    tidpos* acc = lists[S[0]];
    if (n == 1) {
        acc->refs++;
        return acc;
    }
    tidpos* cur = NULL;
    for (int32_t k = 1; k < n; k++) {
        const tidpos* o = lists[S[k]];
        tidpos* nx = tidpos_new(acc->n < o->n ? acc->n : o->n);
        nx->n = 0;
        int64_t a = 0, b = 0;
        while (a < acc->n && b < o->n) {
            if (acc->sid[a] < o->sid[b]) a++;
            else if (o->sid[b] < acc->sid[a]) b++;
            else {
                nx->sid[nx->n] = acc->sid[a];
                nx->pos[nx->n] = take_max ? (acc->pos[a] > o->pos[b] ? acc->pos[a] : o->pos[b])
                                          : (acc->pos[a] < o->pos[b] ? acc->pos[a] : o->pos[b]);
                nx->n++;
                a++;
                b++;
            }
        }
        tidpos_release(cur);
        cur = acc = nx;
    }
    return cur;
}

/* I = sids(X) with firstX, J = sids(Y) with lastY (from the items' lists), and
 * common = tidsIJ: the sids of both with firstX < lastY, ascending. */
static void ensure_state(tsr_ctx* c, rule* r) {
    if (!r->I) r->I = tid_intersect(c->first, r->X, r->nx, 1);
    if (!r->J) r->J = tid_intersect(c->last, r->Y, r->ny, 0);
    if (r->common) return;
    const tidpos *I = r->I, *J = r->J;
    r->common = malloc((size_t)(I->n < J->n ? I->n : J->n) * sizeof(int32_t) + 4);
    r->ncommon = 0;
    int64_t a = 0, b = 0;
    while (a < I->n && b < J->n) {
        if (I->sid[a] < J->sid[b]) a++;
        else if (J->sid[b] < I->sid[a]) b++;
        else {
            if (I->pos[a] < J->pos[b]) r->common[r->ncommon++] = I->sid[a];
            a++;
            b++;
        }
    }
}

/* expandL: rules X U {c} => Y, c > max(X), c not in Y, c before lastY(s). */
static void tsr_expand_left(tsr_ctx* c, rule* r) {
    c->expansions++;
    ensure_state(c, r);
    scan_reset(c);
    for (int64_t q = 0; q < r->ncommon; q++) {
        int32_t tid = r->common[q];
        int32_t end = tp_get(r->J, tid);
        for (int64_t k = c->set_off[tid]; k < c->set_off[tid] + end; k++)
            for (int64_t m = c->item_off[k]; m < c->item_off[k + 1]; m++) {
                int32_t it = c->items[m];
                if (contains_lex_plus(r->X, r->nx, it) || contains_lex(r->Y, r->ny, it)) continue;
                scan_add(c, it, tid);
            }
    }
    qsort(c->touched.a, (size_t)c->touched.n, sizeof(int32_t), cmp_i32);
    for (int64_t q = 0; q < c->touched.n; q++) {
        int32_t it = c->touched.a[q];
        i32vec* tl = &c->tids_of[it];
        if (tl->n < c->minsup) continue;
        /* |tidsIC| = |sids(X) ∩ sids(c)| (the child's tid state is rebuilt if it is expanded) */
        const tidpos* fc = c->first[it];
        int64_t a = 0, b = 0, nI2 = 0;
        while (a < r->I->n && b < fc->n) {
            if (r->I->sid[a] < fc->sid[b]) a++;
            else if (fc->sid[b] < r->I->sid[a]) b++;
            else {
                nI2++;
                a++;
                b++;
            }
        }
        rule* nr = rule_new(c, r->X, r->nx, it, r->Y, r->ny, -1);
        nr->sup = (int32_t)tl->n;
        nr->conf = (double)tl->n / (double)nI2;
        if (nr->conf >= c->minconf) tsr_save(c, nr);
        tsr_register(c, nr, 1);
    }
}

/* expandR: rules X => Y U {c}, c > max(Y), c not in X, c after firstX(s). */
static void tsr_expand_right(tsr_ctx* c, rule* r) {
    c->expansions++;
    ensure_state(c, r);
    scan_reset(c);
    for (int64_t q = 0; q < r->ncommon; q++) {
        int32_t tid = r->common[q];
        int32_t first = tp_get(r->I, tid);
        for (int64_t k = c->set_off[tid] + first + 1; k < c->set_off[tid + 1]; k++)
            for (int64_t m = c->item_off[k]; m < c->item_off[k + 1]; m++) {
                int32_t it = c->items[m];
                if (contains_lex(r->X, r->nx, it) || contains_lex_plus(r->Y, r->ny, it)) continue;
                scan_add(c, it, tid);
            }
    }
    qsort(c->touched.a, (size_t)c->touched.n, sizeof(int32_t), cmp_i32);
    for (int64_t q = 0; q < c->touched.n; q++) {
        int32_t it = c->touched.a[q];
        i32vec* tl = &c->tids_of[it];
        if (tl->n < c->minsup) continue;
        /* X => Y u {c}: conf over |sids(X)| (tid state rebuilt if it is expanded) */
        rule* nr = rule_new(c, r->X, r->nx, -1, r->Y, r->ny, it);
        nr->sup = (int32_t)tl->n;
        nr->conf = (double)tl->n / (double)r->I->n;
        if (nr->conf >= c->minconf) tsr_save(c, nr);
        tsr_register(c, nr, 0);
    }
}

int oracle_tsr(const int32_t* sids, const char* const* lines, const int64_t* lens, int64_t n,
               int32_t k, double minconf, oracle_rules** out, char* err, int errlen) {
    return oracle_tsr_timed(sids, lines, lens, n, k, minconf, 0.0, out, err, errlen);
}

/* time_limit_s > 0 stops after that many seconds of mining (bounded CPU
 * baseline): the result is then partial, complete = 0. */
int oracle_tsr_timed(const int32_t* sids, const char* const* lines, const int64_t* lens, int64_t n,
                     int32_t k, double minconf, double time_limit_s, oracle_rules** out, char* err, int errlen) {
    *out = NULL;
    int complete = 1;
    double t_start = 0.0;
    if (k < 1) {
        set_err(err, errlen, "TSR: k must be >= 1 (got %d)", k);
        return -1;
    }
    tokvec toks = {0};
    i32vec vals = {0};                 /* item value per stored item */
    VEC(int64_t) set_off = {0};        /* per sequence: first itemset index */
    VEC(int64_t) item_off = {0};       /* per itemset: first item index */
    int any_item = 0;
    int rc = 0;
    VPUSH(item_off, 0);
    for (int64_t r = 0; r < n; r++) {
        if (sids[r] != (int32_t)r) {
            set_err(err, errlen, "TSR: sequence ids must be dense 0..N-1 in input order "
                    "(TSR.scala:95,103 index sequences by sid); record %lld has sid %d",
                    (long long)r, sids[r]);
            rc = -1;
            goto done;
        }
        java_split_space(lines[r], lens[r], &toks);
        /* TSR.scala:41 — every token goes through toInt */
        for (int64_t t = 0; t < toks.n; t++) {
            int32_t v;
            if (parse_java_int(toks.a[t].p, toks.a[t].n, &v)) {
                set_err(err, errlen, "TSR parse: bad token '%.*s' in sid=%d (NumberFormatException "
                        "at TSR.scala:41)", (int)(toks.a[t].n > 40 ? 40 : toks.a[t].n), toks.a[t].p, sids[r]);
                rc = -1;
                goto done;
            }
            if (v > -1) any_item = 1;
        }
        /* TSR.newSequence (TSR.scala:109-143) */
        VPUSH(set_off, item_off.n - 1);
        for (int64_t t = 0; t < toks.n; t++) {
            tok_t tk = toks.a[t];
            if (tok_eq(tk, "-1")) {
                VPUSH(item_off, vals.n);
            } else if (tok_eq(tk, "-2")) {
            } else {
                int32_t v = 0;
                parse_java_int(tk.p, tk.n, &v);
                VPUSH(vals, v);
            }
        }
        /* drop items after the last -1 */
        vals.n = item_off.a[item_off.n - 1];
        /* a negative item of a closed itemset indexes the Vertical arrays (TSR.scala:63-75):
           ArrayIndexOutOfBounds; one in the dropped trailing itemset is never used */
        for (int64_t q = item_off.a[set_off.a[set_off.n - 1]]; q < vals.n; q++)
            if (vals.a[q] < 0) {
                set_err(err, errlen, "TSR: negative item %d in sid=%d (Vertical array index)", vals.a[q], sids[r]);
                rc = -1;
                goto done;
            }
    }
    VPUSH(set_off, item_off.n - 1);
    if (!any_item) {
        set_err(err, errlen, "TSR: no items in dataset (empty.max at TSR.scala:43)");
        rc = -1;
        goto done;
    }
    {
        tsr_ctx c;
        memset(&c, 0, sizeof(c));
        c.k = k;
        c.minconf = minconf;
        c.minsup = 1;
        c.krules.max = 0;
        c.cand.max = 1;
        c.purge_at = 1 << 20;
        c.nseq = n;
        c.set_off = set_off.a;
        c.item_off = item_off.a;
        int64_t nvals = vals.n;
        /* dense item ids, ascending by value */
        int32_t* u = malloc((size_t)(nvals ? nvals : 1) * sizeof(int32_t));
        memcpy(u, vals.a, (size_t)nvals * sizeof(int32_t));
        qsort(u, (size_t)nvals, sizeof(int32_t), cmp_i32);
        int64_t nu = 0;
        for (int64_t q = 0; q < nvals; q++)
            if (q == 0 || u[q] != u[q - 1]) u[nu++] = u[q];
        c.nitems = nu;
        c.item_val = u;
        c.items = malloc((size_t)(nvals ? nvals : 1) * sizeof(int32_t));
        for (int64_t q = 0; q < nvals; q++) c.items[q] = (int32_t)lower_bound_i32(u, nu, vals.a[q]);
        /* Vertical: first/last itemset index per (item, sid)  (TSR.scala:52-94) */
        c.first = calloc((size_t)(nu ? nu : 1), sizeof(tidpos*));
        c.last = calloc((size_t)(nu ? nu : 1), sizeof(tidpos*));
        int64_t* cnt = calloc((size_t)(nu ? nu : 1), sizeof(int64_t));
        int32_t* seen = malloc((size_t)(nu ? nu : 1) * sizeof(int32_t));
        for (int64_t q = 0; q < nu; q++) seen[q] = -1;
        for (int64_t s = 0; s < n; s++)
            for (int64_t q = c.item_off[c.set_off[s]]; q < c.item_off[c.set_off[s + 1]]; q++)
                if (seen[c.items[q]] != s) { seen[c.items[q]] = (int32_t)s; cnt[c.items[q]]++; }
        for (int64_t q = 0; q < nu; q++) {
            c.first[q] = tidpos_new(cnt[q]);
            c.last[q] = tidpos_new(cnt[q]);
        }
        for (int64_t s = 0; s < n; s++)
            for (int64_t ks = c.set_off[s]; ks < c.set_off[s + 1]; ks++) {
                int32_t j = (int32_t)(ks - c.set_off[s]);
                for (int64_t q = c.item_off[ks]; q < c.item_off[ks + 1]; q++) {
                    int32_t it = c.items[q];
                    tidpos* f = c.first[it];
                    tidpos* l = c.last[it];
                    if (f->n == 0 || f->sid[f->n - 1] != (int32_t)s) {
                        f->sid[f->n] = (int32_t)s; f->pos[f->n] = j; f->n++;
                        l->sid[l->n] = (int32_t)s; l->pos[l->n] = j; l->n++;
                    } else {
                        l->pos[l->n - 1] = j;
                    }
                }
            }
        free(cnt);
        free(seen);
        c.cnt_last_tid = malloc((size_t)(nu ? nu : 1) * sizeof(int32_t));
        for (int64_t q = 0; q < nu; q++) c.cnt_last_tid[q] = -1;
        c.tids_of = calloc((size_t)(nu ? nu : 1), sizeof(i32vec));

        /* Pair phase: i ascending, j > i; IJ then JI. */
        t_start = mono_s();
        const double deadline = time_limit_s > 0 ? t_start + time_limit_s : 0.0;
        int64_t pairs = 0;
        for (int64_t i = 0; i < nu && complete; i++) {
            if (deadline > 0 && mono_s() > deadline) { complete = 0; break; }
            const tidpos* fi = c.first[i];
            const tidpos* li = c.last[i];
            if (fi->n < c.minsup) continue;
            for (int64_t j = i + 1; j < nu; j++) {
                const tidpos* fj = c.first[j];
                const tidpos* lj = c.last[j];
                if (fj->n < c.minsup) continue;
                pairs++;
                int64_t a = 0, b = 0, nij = 0, nji = 0;
                while (a < fi->n && b < fj->n) {
                    if (fi->sid[a] < fj->sid[b]) a++;
                    else if (fj->sid[b] < fi->sid[a]) b++;
                    else {
                        nij += fi->pos[a] < lj->pos[b];
                        nji += fj->pos[b] < li->pos[a];
                        a++;
                        b++;
                    }
                }
                int32_t xi = (int32_t)i, xj = (int32_t)j;
                if (nij >= c.minsup) {
                    rule* r = rule_new(&c, &xi, 1, -1, &xj, 1, -1);
                    r->sup = (int32_t)nij;
                    r->conf = (double)nij / (double)fi->n;
                    r->I = c.first[i]; r->I->refs++;
                    r->J = c.last[j]; r->J->refs++;
                    /* tidsIJ: made by ensure_common if r is ever expanded */
                    if (r->conf >= c.minconf) tsr_save(&c, r);
                    tsr_register(&c, r, 1);
                }
                if (nji >= c.minsup) {
                    rule* r = rule_new(&c, &xj, 1, -1, &xi, 1, -1);
                    r->sup = (int32_t)nji;
                    r->conf = (double)nji / (double)fj->n;
                    r->I = c.first[j]; r->I->refs++;
                    r->J = c.last[i]; r->J->refs++;
                    /* tidsJI: likewise */
                    if (r->conf >= c.minconf) tsr_save(&c, r);
                    tsr_register(&c, r, 1);
                }
            }
        }
        /* Expansion loop */
        while (complete && c.cand.n > 0) {
            if (deadline > 0 && mono_s() > deadline) { complete = 0; break; }
            rule* r = heap_pop(&c.cand);  /* in_cand stays set while r is expanded */
            if (r->sup < c.minsup) {
                r->in_cand = 0;
                rule_maybe_free(r);
                break;
            }
            if (r->expandLR) {
                tsr_expand_left(&c, r);
                tsr_expand_right(&c, r);
            } else {
                tsr_expand_right(&c, r);
            }
            r->in_cand = 0;
            rule_release_state(r);
            rule_maybe_free(r);
        }
        /* result = kRules */
        oracle_rules* o = calloc(1, sizeof(*o));
        int64_t nr = c.krules.n;
        o->n = nr;
        o->total = n;
        o->expansions = c.expansions;
        o->final_minsup = c.minsup;
        o->complete = complete;
        o->seconds = mono_s() - t_start;
        o->pairs = pairs;
        o->support = malloc((size_t)(nr ? nr : 1) * sizeof(int32_t));
        o->confidence = malloc((size_t)(nr ? nr : 1) * sizeof(double));
        o->ante_off = malloc((size_t)(nr + 1) * sizeof(int64_t));
        o->cons_off = malloc((size_t)(nr + 1) * sizeof(int64_t));
        int64_t na = 0, nc = 0;
        for (int64_t q = 0; q < nr; q++) { na += c.krules.a[q]->nx; nc += c.krules.a[q]->ny; }
        o->ante = malloc((size_t)(na ? na : 1) * sizeof(int32_t));
        o->cons = malloc((size_t)(nc ? nc : 1) * sizeof(int32_t));
        o->ante_off[0] = o->cons_off[0] = 0;
        for (int64_t q = 0; q < nr; q++) {
            rule* r = c.krules.a[q];
            o->support[q] = r->sup;
            o->confidence[q] = r->conf;
            for (int32_t t = 0; t < r->nx; t++) o->ante[o->ante_off[q] + t] = c.item_val[r->X[t]];
            for (int32_t t = 0; t < r->ny; t++) o->cons[o->cons_off[q] + t] = c.item_val[r->Y[t]];
            o->ante_off[q + 1] = o->ante_off[q] + r->nx;
            o->cons_off[q + 1] = o->cons_off[q] + r->ny;
        }
        *out = o;
        /* cleanup */
        for (int64_t q = 0; q < c.krules.n; q++) {
            c.krules.a[q]->in_k = 0;
            rule_maybe_free(c.krules.a[q]);
        }
        for (int64_t q = 0; q < c.cand.n; q++) {
            c.cand.a[q]->in_cand = 0;
            rule_maybe_free(c.cand.a[q]);
        }
        for (int64_t q = 0; q < nu; q++) {
            tidpos_release(c.first[q]);
            tidpos_release(c.last[q]);
            VFREE(c.tids_of[q]);
        }
        free(c.first);
        free(c.last);
        free(c.tids_of);
        free(c.cnt_last_tid);
        VFREE(c.touched);
        free(c.krules.a);
        free(c.cand.a);
        free(c.items);
        free(u);
    }
done:
    VFREE(toks);
    VFREE(vals);
    VFREE(set_off);
    VFREE(item_off);
    return rc;
}

void oracle_rules_free(oracle_rules* r) {
    if (!r) return;
    free(r->support);
    free(r->confidence);
    free(r->ante_off);
    free(r->ante);
    free(r->cons_off);
    free(r->cons);
    free(r);
}

/* ======================================================= point checkers ===
 * Definitional support of ONE pattern / ONE rule over a token stream
 * (-1 ends an itemset, -2 ends a sequence; implicit timestamps, one record per
 * sid).  Used by the full-size property tests (sampled patterns / rules). */

static int itemset_contains(const int64_t* set, int64_t n, const int32_t* need, int64_t m) {
    for (int64_t a = 0; a < m; a++) {
        int found = 0;
        for (int64_t b = 0; b < n; b++)
            if (set[b] == need[a]) { found = 1; break; }
        if (!found) return 0;
    }
    return 1;
}

int64_t oracle_pattern_support(const int64_t* seq_off, const int64_t* tokens, int64_t n,
                               const int32_t* items, const int64_t* set_off, int64_t nsets) {
    int64_t sup = 0;
    for (int64_t s = 0; s < n; s++) {
        int64_t k = 0; /* next pattern itemset to match (greedy earliest) */
        int64_t a = seq_off[s];
        while (a < seq_off[s + 1] && k < nsets) {
            int64_t b = a;
            while (b < seq_off[s + 1] && tokens[b] != -1) b++;
            if (b >= seq_off[s + 1] || tokens[b] != -1) break; /* unterminated: dropped */
            if (itemset_contains(tokens + a, b - a, items + set_off[k], set_off[k + 1] - set_off[k])) k++;
            a = b + 1;
        }
        if (k == nsets) sup++;
    }
    return sup;
}

/* X => Y: sup = #{s : X,Y present, max first_x < min last_y}; nX = |sids(X)|.
 * Positions are 0-based itemset indexes (TSR.scala:57-79). */
void oracle_rule_support(const int64_t* seq_off, const int64_t* tokens, int64_t n, const int32_t* X,
                         int64_t nx, const int32_t* Y, int64_t ny, int64_t* sup_out, int64_t* nx_out) {
    int64_t sup = 0, cx = 0;
    int32_t fbuf[256], lbuf[256];
    for (int64_t s = 0; s < n; s++) {
        for (int64_t q = 0; q < nx; q++) fbuf[q] = -1;
        for (int64_t q = 0; q < ny; q++) lbuf[q] = -1;
        int32_t pos = 0;
        int64_t a = seq_off[s];
        int64_t end = seq_off[s + 1];
        /* find the last -1 : items after it are dropped */
        int64_t lastm = -1;
        for (int64_t b = a; b < end; b++) if (tokens[b] == -1) lastm = b;
        for (int64_t b = a; b < lastm; b++) {
            int64_t t = tokens[b];
            if (t == -1) { pos++; continue; }
            if (t == -2) continue;
            for (int64_t q = 0; q < nx; q++) if (X[q] == t && fbuf[q] < 0) fbuf[q] = pos;
            for (int64_t q = 0; q < ny; q++) if (Y[q] == t) lbuf[q] = pos;
        }
        int okx = 1, oky = 1;
        int32_t fX = -1, lY = 0x7FFFFFFF;
        for (int64_t q = 0; q < nx; q++) { if (fbuf[q] < 0) okx = 0; else if (fbuf[q] > fX) fX = fbuf[q]; }
        for (int64_t q = 0; q < ny; q++) { if (lbuf[q] < 0) oky = 0; else if (lbuf[q] < lY) lY = lbuf[q]; }
        if (okx) cx++;
        if (okx && oky && fX < lY) sup++;
    }
    *sup_out = sup;
    *nx_out = cx;
}
