/*
 * fsmgen.c — seeded synthetic sequence-database generators.
 *
 *  gen_quest   IBM-Quest-shaped (Agrawal & Srikant 1995, restated from the
 *              paper's description): N_I potentially large itemsets (size
 *              ~Poisson(I), items correlated with the previous itemset,
 *              exponential weights, corruption ~N(0.75,0.1)), N_S potentially
 *              large sequences (length ~Poisson(S), itemsets drawn by weight),
 *              customer sequences of ~Poisson(C) transactions of ~Poisson(T)
 *              items filled with corrupted large sequences.
 *  gen_zipf    single-item-itemset click / word streams (Kosarak, BIBLE, SIGN
 *              shapes): Zipf(s) item popularity, log-normal lengths clipped to
 *              [1, max_len], a Markov "successor" link so sequential rules with
 *              real confidence exist, optional distinct-items-per-sequence.
 *
 * Output is the token stream of fsm_db_from_tokens: per sequence the items,
 * -1 after each itemset, -2 at the end.  Deterministic for a given seed
 * (own xoshiro256** PRNG).  Tool code: used by tests and bench.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t s[4]; } rng_t;

static uint64_t splitmix(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t* r, uint64_t seed) {
    for (int i = 0; i < 4; i++) r->s[i] = splitmix(&seed);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static uint64_t next_u64(rng_t* r) {
    uint64_t* s = r->s;
    uint64_t res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static double uni(rng_t* r) { return (double)(next_u64(r) >> 11) * (1.0 / 9007199254740992.0); }
static int64_t below(rng_t* r, int64_t n) { return (int64_t)(uni(r) * (double)n); }
static double expo(rng_t* r, double mean) { return -mean * log(1.0 - uni(r)); }
static double normal(rng_t* r, double mu, double sd) {
    double u1 = uni(r), u2 = uni(r);
    if (u1 < 1e-300) u1 = 1e-300;
    return mu + sd * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}
static int64_t poisson(rng_t* r, double lam) {
    if (lam <= 0) return 0;
    if (lam > 30) {
        double v = normal(r, lam, sqrt(lam));
        return v < 0 ? 0 : (int64_t)(v + 0.5);
    }
    double L = exp(-lam), p = 1.0;
    int64_t k = 0;
    do { k++; p *= uni(r); } while (p > L);
    return k - 1;
}
/* index from a cumulative weight table */
static int64_t pick(rng_t* r, const double* cum, int64_t n) {
    double x = uni(r) * cum[n - 1];
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (cum[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

typedef struct { int64_t* a; int64_t n, cap; } i64v;
static void push(i64v* v, int64_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 1024;
        v->a = realloc(v->a, (size_t)v->cap * sizeof(int64_t));
    }
    v->a[v->n++] = x;
}

static int cmp_i64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

void gen_free(void* p) { free(p); }

int gen_quest(uint64_t seed, int64_t D, double C, double T, double S, double I, int32_t NS, int32_t NI,
              int32_t N, int64_t** seq_off_out, int64_t** tokens_out, int64_t* ntok_out) {
    rng_t r;
    rng_seed(&r, seed);
    /* potentially large itemsets */
    int64_t* is_off = malloc((size_t)(NI + 1) * sizeof(int64_t));
    i64v is_items = {0};
    double* is_cum = malloc((size_t)NI * sizeof(double));
    double* is_cor = malloc((size_t)NI * sizeof(double));
    is_off[0] = 0;
    double acc = 0;
    for (int32_t k = 0; k < NI; k++) {
        int64_t sz = poisson(&r, I - 1.0) + 1; /* size >= 1, mean I */
        int64_t from_prev = 0;
        if (k > 0) {
            double frac = expo(&r, 0.5);
            if (frac > 1) frac = 1;
            int64_t plen = is_off[k] - is_off[k - 1];
            from_prev = (int64_t)(frac * (double)sz + 0.5);
            if (from_prev > plen) from_prev = plen;
        }
        int64_t base = is_items.n;
        for (int64_t q = 0; q < from_prev; q++) push(&is_items, is_items.a[is_off[k - 1] + below(&r, is_off[k] - is_off[k - 1])]);
        while (is_items.n - base < sz) push(&is_items, below(&r, N) + 1);
        /* dedup within the itemset */
        qsort(is_items.a + base, (size_t)(is_items.n - base), sizeof(int64_t), cmp_i64);
        int64_t w = base;
        for (int64_t q = base; q < is_items.n; q++)
            if (q == base || is_items.a[q] != is_items.a[q - 1]) is_items.a[w++] = is_items.a[q];
        is_items.n = w;
        is_off[k + 1] = is_items.n;
        acc += expo(&r, 1.0);
        is_cum[k] = acc;
        double c = normal(&r, 0.75, 0.1);
        is_cor[k] = c < 0 ? 0 : (c > 1 ? 1 : c);
    }
    /* potentially large sequences */
    int64_t* ls_off = malloc((size_t)(NS + 1) * sizeof(int64_t));
    i64v ls_sets = {0};
    double* ls_cum = malloc((size_t)NS * sizeof(double));
    double* ls_cor = malloc((size_t)NS * sizeof(double));
    ls_off[0] = 0;
    acc = 0;
    for (int32_t k = 0; k < NS; k++) {
        int64_t len = poisson(&r, S - 1.0) + 1;
        int64_t from_prev = 0;
        if (k > 0) {
            double frac = expo(&r, 0.5);
            if (frac > 1) frac = 1;
            int64_t plen = ls_off[k] - ls_off[k - 1];
            from_prev = (int64_t)(frac * (double)len + 0.5);
            if (from_prev > plen) from_prev = plen;
        }
        for (int64_t q = 0; q < len; q++) {
            if (q < from_prev) push(&ls_sets, ls_sets.a[ls_off[k - 1] + q]);
            else push(&ls_sets, pick(&r, is_cum, NI));
        }
        ls_off[k + 1] = ls_sets.n;
        acc += expo(&r, 1.0);
        ls_cum[k] = acc;
        double c = normal(&r, 0.75, 0.1);
        ls_cor[k] = c < 0 ? 0 : (c > 1 ? 1 : c);
    }
    /* customer sequences */
    int64_t* seq_off = malloc((size_t)(D + 1) * sizeof(int64_t));
    i64v tok = {0};
    i64v* trans = NULL;
    int64_t tcap = 0;
    i64v buf = {0};
    seq_off[0] = 0;
    for (int64_t d = 0; d < D; d++) {
        int64_t nt = poisson(&r, C);
        if (nt < 1) nt = 1;
        if (nt > tcap) {
            trans = realloc(trans, (size_t)nt * sizeof(i64v));
            for (int64_t q = tcap; q < nt; q++) memset(&trans[q], 0, sizeof(i64v));
            tcap = nt;
        }
        int64_t target = 0;
        for (int64_t q = 0; q < nt; q++) {
            trans[q].n = 0;
            int64_t ts = poisson(&r, T);
            target += ts < 1 ? 1 : ts;
        }
        int64_t placed = 0, guard = 0;
        while (placed < target && guard++ < 64) {
            int64_t ls = pick(&r, ls_cum, NS);
            int64_t len = ls_off[ls + 1] - ls_off[ls];
            int64_t use = len < nt ? len : nt;
            /* increasing transaction slots for the sequence's first `use` itemsets */
            int64_t pos[64];
            if (use > 64) use = 64;
            for (int64_t q = 0; q < use; q++) pos[q] = below(&r, nt);
            qsort(pos, (size_t)use, sizeof(int64_t), cmp_i64);
            for (int64_t q = 1; q < use; q++)
                if (pos[q] <= pos[q - 1]) pos[q] = pos[q - 1] + 1;
            while (use > 0 && pos[use - 1] >= nt) use--;
            for (int64_t q = 0; q < use; q++) {
                int64_t is = ls_sets.a[ls_off[ls] + q];
                for (int64_t x = is_off[is]; x < is_off[is + 1]; x++) {
                    /* corruption: drop items while uniform < c (itemset level) */
                    if (uni(&r) < is_cor[is] * 0.5) continue;
                    push(&trans[pos[q]], is_items.a[x]);
                    placed++;
                }
            }
            if (uni(&r) < ls_cor[ls] * 0.1) break;
        }
        /* fill remaining budget with noise items */
        while (placed < target) {
            push(&trans[below(&r, nt)], below(&r, N) + 1);
            placed++;
        }
        for (int64_t q = 0; q < nt; q++) {
            if (!trans[q].n) continue;
            buf.n = 0;
            for (int64_t x = 0; x < trans[q].n; x++) push(&buf, trans[q].a[x]);
            qsort(buf.a, (size_t)buf.n, sizeof(int64_t), cmp_i64);
            for (int64_t x = 0; x < buf.n; x++)
                if (x == 0 || buf.a[x] != buf.a[x - 1]) push(&tok, buf.a[x]);
            push(&tok, -1);
        }
        push(&tok, -2);
        seq_off[d + 1] = tok.n;
    }
    for (int64_t q = 0; q < tcap; q++) free(trans[q].a);
    free(trans);
    free(buf.a);
    free(is_off); free(is_items.a); free(is_cum); free(is_cor);
    free(ls_off); free(ls_sets.a); free(ls_cum); free(ls_cor);
    *seq_off_out = seq_off;
    *tokens_out = tok.a;
    *ntok_out = tok.n;
    return 0;
}

int gen_zipf(uint64_t seed, int64_t D, int32_t nitems, double zipf_s, double mean_len, double sigma,
             int64_t max_len, double p_succ, int32_t distinct, int64_t** seq_off_out, int64_t** tokens_out,
             int64_t* ntok_out) {
    rng_t r;
    rng_seed(&r, seed);
    double* cum = malloc((size_t)nitems * sizeof(double));
    double acc = 0;
    for (int32_t k = 0; k < nitems; k++) {
        acc += 1.0 / pow((double)(k + 1), zipf_s);
        cum[k] = acc;
    }
    /* item ids: a fixed random permutation of popularity ranks, 1-based */
    int64_t* perm = malloc((size_t)nitems * sizeof(int64_t));
    for (int32_t k = 0; k < nitems; k++) perm[k] = k + 1;
    for (int32_t k = nitems - 1; k > 0; k--) {
        int64_t j = below(&r, k + 1), t = perm[k];
        perm[k] = perm[j];
        perm[j] = t;
    }
    /* successor link: each rank points at a (popular-biased) rank */
    int64_t* succ = malloc((size_t)nitems * sizeof(int64_t));
    for (int32_t k = 0; k < nitems; k++) succ[k] = pick(&r, cum, nitems);
    double mu = log(mean_len) - 0.5 * sigma * sigma;
    int64_t* seq_off = malloc((size_t)(D + 1) * sizeof(int64_t));
    i64v tok = {0};
    char* seen = calloc((size_t)nitems, 1);
    i64v used = {0};
    seq_off[0] = 0;
    for (int64_t d = 0; d < D; d++) {
        double l = exp(normal(&r, mu, sigma));
        int64_t len = (int64_t)(l + 0.5);
        if (len < 1) len = 1;
        if (len > max_len) len = max_len;
        if (distinct && len > nitems / 2) len = nitems / 2 > 0 ? nitems / 2 : 1;
        int64_t prev = -1;
        used.n = 0;
        for (int64_t q = 0, tries = 0; q < len && tries < 8 * len + 64; tries++) {
            int64_t rk = (prev >= 0 && uni(&r) < p_succ) ? succ[prev] : pick(&r, cum, nitems);
            if (distinct) {
                if (seen[rk]) { prev = -1; continue; }
                seen[rk] = 1;
                push(&used, rk);
            }
            push(&tok, perm[rk]);
            push(&tok, -1);
            prev = rk;
            q++;
        }
        for (int64_t q = 0; q < used.n; q++) seen[used.a[q]] = 0;
        push(&tok, -2);
        seq_off[d + 1] = tok.n;
    }
    free(cum); free(perm); free(succ); free(seen); free(used.a);
    *seq_off_out = seq_off;
    *tokens_out = tok.a;
    *ntok_out = tok.n;
    return 0;
}
