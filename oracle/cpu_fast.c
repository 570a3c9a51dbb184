/*
 * cpu_fast.c — optimized, multi-threaded CPU evaluator of the placement rules:
 * the CPU baseline that bench.py times beside the GPU (cpu_baseline legs at
 * 1 thread, 2 threads -- the reference manager's 2-CPU limit,
 * config/components/manager/manager.yaml:94-100 -- and every core of the
 * box's share). TEST INFRASTRUCTURE ONLY: called by bench.py's cpu_baseline
 * leg and by tests/ (which check it bit-exact against cpu_ref.c); never
 * linked or imported by the product package jobset_amd/.
 *
 * Rules: exactly cpu_ref.c's (see its header for the rules and their
 * reference anchors; parity status there). What is different is only how
 * they are evaluated:
 *   prepare (untimed; the engine's topology/class upload is untimed too):
 *     class digests with invariant-divisor constants, per-thread row ranges
 *     cut at leaf boundaries and balanced by rows, the hierarchy's parent and
 *     child tables;
 *   tally: each thread, per class, runs straight vectorisable passes over its
 *     rows (fit by multiply-high division per resource, label AND-compare per
 *     word, taint AND) into a row buffer, then sums the buffer per leaf;
 *   feasibility: one bit per domain per class, threads split the classes'
 *     words;
 *   assignment: one thread (the greedy is sequential), per-class cursors over
 *     the bit words (ctz), taken marks of ancestors (parent chain) and
 *     descendants (bit ranges).
 * Threads come from a persistent pthread pool woken by a generation counter.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "jspo.h"

#define MAXT 64
#define MAXC 64
#define DIV_IDENT 0xFFFFFFFFu

typedef struct jspf_ctx jspf_ctx;
typedef void (*phase_fn)(jspf_ctx*, int);
typedef struct {
    jspf_ctx* x;
    int id;
} worker_arg;

struct jspf_ctx {
    /* pool */
    int T;
    pthread_t th[MAXT];
    worker_arg args[MAXT];
    atomic_int gen;
    atomic_int finished;
    atomic_int quit;
    phase_fn phase;
    /* problem */
    const jspo_problem* p;
    uint32_t K, L, N, W, R, C, D[MAXL];
    uint64_t req[MAXC][4], mask[MAXC][4];
    uint32_t tolinv[MAXC], pods[MAXC], level[MAXC], res[MAXC][4], magic[MAXC][4], shift[MAXC][4];
    uint32_t lbeg[MAXT + 1];        /* thread t owns leaves [lbeg[t], lbeg[t+1]) */
    uint32_t* vbuf[MAXT];           /* per-thread row buffer */
    uint32_t* fl[MAXL];             /* first_leaf per level (identity materialised) */
    int32_t* par[MAXL];             /* par[k][d]: level k-1 domain of level-k domain d */
    uint32_t* cs[MAXL];             /* cs[k][d]: first level-(k+1) domain of level-k domain d */
    uint32_t woff[MAXC + 1], toff[MAXL + 1];
    uint32_t* cap;                  /* [C][L] */
    uint32_t* occ;                  /* [L] */
    uint64_t* feas;                 /* [woff[C]] */
    uint64_t* taken;                /* [toff[K]] */
};

/* ---------------------------------------------------------------- pool */
static void* worker(void* arg) {
    jspf_ctx* x = ((worker_arg*)arg)->x;
    const int me = ((worker_arg*)arg)->id;
    int seen = 0;
    for (;;) {
        int g;
        unsigned spins = 0;
        while ((g = atomic_load_explicit(&x->gen, memory_order_acquire)) == seen) {
            if (atomic_load_explicit(&x->quit, memory_order_relaxed)) return NULL;
            if (++spins > 4096) {
                sched_yield();
                spins = 0;
            } else {
                __builtin_ia32_pause();
            }
        }
        seen = g;
        if (atomic_load_explicit(&x->quit, memory_order_relaxed)) return NULL;
        x->phase(x, me);
        atomic_fetch_add_explicit(&x->finished, 1, memory_order_acq_rel);
    }
}

static void run_phase(jspf_ctx* x, phase_fn fn) {
    if (x->T == 1) {
        fn(x, 0);
        return;
    }
    x->phase = fn;
    atomic_store_explicit(&x->finished, 0, memory_order_relaxed);
    atomic_fetch_add_explicit(&x->gen, 1, memory_order_acq_rel);
    fn(x, 0);
    while (atomic_load_explicit(&x->finished, memory_order_acquire) < x->T - 1) __builtin_ia32_pause();
}

/* ---------------------------------------------------------------- helpers */
static void divisor_magic(uint32_t d, uint32_t* magic, uint32_t* shift) {
    *magic = 0;
    *shift = DIV_IDENT;
    if (d <= 1) return;
    uint32_t L = 31 - (uint32_t)__builtin_clz(d);
    if ((d & (d - 1)) == 0) {
        *shift = L - 1;
        return;
    }
    const uint64_t num = 1ull << (32 + L);
    uint64_t m = num / d;
    const uint64_t rem = num % d;
    m = (m + m) & 0xFFFFFFFFull;
    if (rem + rem >= d) m = (m + 1) & 0xFFFFFFFFull;
    *magic = (uint32_t)((1 + m) & 0xFFFFFFFFull);
    *shift = L;
}

static void set_bit(uint64_t* t, uint32_t d) { t[d >> 6] |= 1ull << (d & 63); }

static void set_range(uint64_t* t, uint32_t lo, uint32_t hi) {
    while (lo < hi) {
        const uint32_t w = lo >> 6, b = lo & 63;
        const uint32_t n = (hi - lo) < (64 - b) ? (hi - lo) : (64 - b);
        t[w] |= (n == 64) ? ~0ull : (((1ull << n) - 1) << b);
        lo += n;
    }
}

/* ---------------------------------------------------------------- tally (per thread) */
static void tally_phase(jspf_ctx* x, int t) {
    const jspo_problem* p = x->p;
    const uint32_t l0 = x->lbeg[t], l1 = x->lbeg[t + 1];
    if (l0 >= l1) return;
    const uint32_t* ls = p->leaf_start;
    const uint32_t r0 = ls[l0], r1 = ls[l1], n = r1 - r0, N = x->N, L = x->L;
    uint32_t* restrict v = x->vbuf[t];
    for (uint32_t c = 0; c < x->C; ++c) {
        const uint32_t pods = x->pods[c];
        for (uint32_t i = 0; i < n; ++i) v[i] = pods;
        for (uint32_t r = 0; r < x->R; ++r) {
            const uint32_t rq = x->res[c][r];
            if (rq == 0) continue;
            const uint32_t* restrict f = p->free_res + (size_t)r * N + r0;
            if (x->shift[c][r] == DIV_IDENT) {
                for (uint32_t i = 0; i < n; ++i) v[i] = f[i] < v[i] ? f[i] : v[i];
            } else {
                const uint32_t mg = x->magic[c][r], sh = x->shift[c][r];
                for (uint32_t i = 0; i < n; ++i) {
                    const uint32_t a = f[i], h = (uint32_t)(((uint64_t)a * mg) >> 32);
                    const uint32_t q = (((a - h) >> 1) + h) >> sh;
                    v[i] = q < v[i] ? q : v[i];
                }
            }
        }
        for (uint32_t w = 0; w < x->W; ++w) {
            const uint64_t mk = x->mask[c][w], rq = x->req[c][w];
            if (mk == 0) continue;
            const uint64_t* restrict lab = p->labels + (size_t)w * N + r0;
            for (uint32_t i = 0; i < n; ++i) v[i] = (lab[i] & mk) == rq ? v[i] : 0u;
        }
        {
            const uint32_t ti = x->tolinv[c];
            const uint32_t* restrict tn = p->taints + r0;
            for (uint32_t i = 0; i < n; ++i) v[i] = (tn[i] & ti) == 0 ? v[i] : 0u;
        }
        uint32_t* restrict cp = x->cap + (size_t)c * L;
        for (uint32_t l = l0; l < l1; ++l) {
            uint32_t s = 0;
            for (uint32_t i = ls[l] - r0; i < ls[l + 1] - r0; ++i) s += v[i];
            cp[l] = s;
        }
    }
    const int32_t* ex = p->excl;
    for (uint32_t l = l0; l < l1; ++l) {
        uint32_t o = 0;
        for (uint32_t i = ls[l]; i < ls[l + 1]; ++i) o += ex[i] != -1;
        x->occ[l] = o;
    }
}

/* ---------------------------------------------------------------- feasibility (threads split words) */
static void feas_phase(jspf_ctx* x, int t) {
    const uint32_t total = x->woff[x->C];
    const uint32_t w0 = (uint32_t)(((uint64_t)total * t) / x->T), w1 = (uint32_t)(((uint64_t)total * (t + 1)) / x->T);
    uint32_t c = 0;
    for (uint32_t gw = w0; gw < w1; ++gw) {
        while (x->woff[c + 1] <= gw) ++c;
        const uint32_t k = x->level[c], D = x->D[k], pods = x->pods[c];
        const uint32_t* cp = x->cap + (size_t)c * x->L;
        const uint32_t* fl = x->fl[k];
        uint64_t word = 0;
        const uint32_t d0 = (gw - x->woff[c]) * 64;
        for (uint32_t b = 0; b < 64 && d0 + b < D; ++b) {
            const uint32_t d = d0 + b;
            uint64_t s = 0, o = 0;
            for (uint32_t leaf = fl[d]; leaf < fl[d + 1]; ++leaf) {
                s += cp[leaf];
                o += x->occ[leaf];
            }
            if (s >= pods && o == 0) word |= 1ull << b;
        }
        x->feas[gw] = word;
    }
}

/* ---------------------------------------------------------------- assignment (one thread) */
static int assign_all(jspf_ctx* x, int32_t* assign) {
    const jspo_problem* p = x->p;
    const uint32_t K = x->K;
    uint32_t cur[MAXC];
    memset(cur, 0, sizeof cur);
    memset(x->taken, 0, sizeof(uint64_t) * x->toff[K]);
    int placed = 0;
    for (uint32_t j = 0; j < p->n_jobs; ++j) {
        const uint32_t c = p->job_class[j], k = x->level[c], D = x->D[k], nw = (D + 63) >> 6;
        const uint64_t* F = x->feas + x->woff[c];
        uint64_t* Tk = x->taken + x->toff[k];
        uint32_t w = cur[c] >> 6;
        uint64_t bits = 0;
        if (w < nw) bits = F[w] & ~Tk[w] & (~0ull << (cur[c] & 63));
        while (bits == 0 && ++w < nw) bits = F[w] & ~Tk[w];
        if (bits == 0) {
            assign[j] = -1;
            cur[c] = D;
            continue;
        }
        const uint32_t d = w * 64 + (uint32_t)__builtin_ctzll(bits);
        assign[j] = (int32_t)d;
        cur[c] = d + 1;
        ++placed;
        if (x->fl[k][d] == x->fl[k][d + 1]) continue; /* empty domain intersects nothing (never feasible) */
        Tk[d >> 6] |= 1ull << (d & 63);
        uint32_t dd = d;
        for (int kk = (int)k - 1; kk >= 0; --kk) {
            dd = (uint32_t)x->par[kk + 1][dd];
            set_bit(x->taken + x->toff[kk], dd);
        }
        uint32_t lo = d, hi = d + 1;
        for (uint32_t kk = k + 1; kk < K; ++kk) {
            lo = x->cs[kk - 1][lo];
            hi = x->cs[kk - 1][hi];
            set_range(x->taken + x->toff[kk], lo, hi);
        }
    }
    return placed;
}

/* ---------------------------------------------------------------- API */
jspf_ctx* jspf_create(int threads) {
    if (threads < 1) threads = 1;
    if (threads > MAXT) threads = MAXT;
    jspf_ctx* x = (jspf_ctx*)calloc(1, sizeof(jspf_ctx));
    if (!x) return NULL;
    x->T = threads;
    atomic_init(&x->gen, 0);
    atomic_init(&x->finished, 0);
    atomic_init(&x->quit, 0);
    for (int t = 1; t < threads; ++t) {
        x->args[t].x = x;
        x->args[t].id = t;
        if (pthread_create(&x->th[t], NULL, worker, &x->args[t]) != 0) {
            x->T = t;
            break;
        }
    }
    return x;
}

static void free_problem(jspf_ctx* x) {
    for (int t = 0; t < MAXT; ++t) {
        free(x->vbuf[t]);
        x->vbuf[t] = NULL;
    }
    for (int k = 0; k < MAXL; ++k) {
        free(x->fl[k]);
        free(x->par[k]);
        free(x->cs[k]);
        x->fl[k] = NULL;
        x->par[k] = NULL;
        x->cs[k] = NULL;
    }
    free(x->cap);
    free(x->occ);
    free(x->feas);
    free(x->taken);
    x->cap = x->occ = NULL;
    x->feas = x->taken = NULL;
}

void jspf_destroy(jspf_ctx* x) {
    if (!x) return;
    atomic_store(&x->quit, 1);
    atomic_fetch_add(&x->gen, 1);
    for (int t = 1; t < x->T; ++t) pthread_join(x->th[t], NULL);
    free_problem(x);
    free(x);
}

int jspf_threads(const jspf_ctx* x) { return x ? x->T : 0; }

/* Untimed preparation of a snapshot + classes (the problem must outlive the
 * following jspf_run calls). Returns 0 or -1 (allocation / limits). */
int jspf_prepare(jspf_ctx* x, const jspo_problem* p) {
    free_problem(x);
    x->p = p;
    x->K = p->n_levels;
    x->L = p->n_domains[x->K - 1];
    x->N = p->n_nodes;
    x->W = p->W;
    x->R = p->R;
    x->C = p->n_classes;
    if (x->C > MAXC || x->K < 1 || x->K > MAXL) return -1;
    for (uint32_t k = 0; k < x->K; ++k) {
        x->D[k] = p->n_domains[k];
        x->fl[k] = (uint32_t*)malloc(sizeof(uint32_t) * (x->D[k] + 1));
        if (!x->fl[k]) return -1;
        for (uint32_t d = 0; d <= x->D[k]; ++d)
            x->fl[k][d] = (k + 1 == x->K || !p->first_leaf[k]) ? d : p->first_leaf[k][d];
    }
    for (uint32_t k = 0; k < x->K; ++k) {
        if (k + 1 < x->K) { /* child start of each level-k domain at level k+1 */
            x->cs[k] = (uint32_t*)malloc(sizeof(uint32_t) * (x->D[k] + 1));
            if (!x->cs[k]) return -1;
            uint32_t j = 0;
            for (uint32_t d = 0; d <= x->D[k]; ++d) {
                while (j < x->D[k + 1] + 1 && x->fl[k + 1][j] < x->fl[k][d]) ++j;
                x->cs[k][d] = j;
            }
        }
        if (k >= 1) { /* parent at level k-1: last level-(k-1) domain starting at or before d's first leaf */
            x->par[k] = (int32_t*)malloc(sizeof(int32_t) * (x->D[k] + 1));
            if (!x->par[k]) return -1;
            uint32_t j = 0;
            for (uint32_t d = 0; d < x->D[k]; ++d) {
                while (j + 1 < x->D[k - 1] && x->fl[k - 1][j + 1] <= x->fl[k][d]) ++j;
                x->par[k][d] = (int32_t)j;
            }
        }
    }
    for (uint32_t c = 0; c < x->C; ++c) {
        for (int w = 0; w < 4; ++w) {
            x->req[c][w] = p->cls_req[4 * c + w];
            x->mask[c][w] = p->cls_req[4 * c + w] | p->cls_forbid[4 * c + w];
        }
        x->tolinv[c] = ~p->cls_tol[c];
        x->pods[c] = p->cls_pods[c];
        x->level[c] = p->cls_level[c];
        for (int r = 0; r < 4; ++r) {
            x->res[c][r] = p->cls_res[4 * c + r];
            divisor_magic(x->res[c][r], &x->magic[c][r], &x->shift[c][r]);
        }
        x->woff[c + 1] = x->woff[c] + (x->D[x->level[c]] + 63) / 64;
    }
    x->toff[0] = 0;
    for (uint32_t k = 0; k < x->K; ++k) x->toff[k + 1] = x->toff[k] + (x->D[k] + 63) / 64;
    /* thread row ranges at leaf boundaries, balanced by rows */
    const uint32_t* ls = p->leaf_start;
    x->lbeg[0] = 0;
    for (int t = 1; t < x->T; ++t) {
        const uint64_t target = (uint64_t)x->N * (uint64_t)t / (uint64_t)x->T;
        uint32_t l = x->lbeg[t - 1];
        while (l < x->L && ls[l] < target) ++l;
        x->lbeg[t] = l;
    }
    x->lbeg[x->T] = x->L;
    for (int t = 0; t < x->T; ++t) {
        const uint32_t rows = ls[x->lbeg[t + 1]] - ls[x->lbeg[t]];
        x->vbuf[t] = (uint32_t*)malloc(sizeof(uint32_t) * (rows + 1));
        if (!x->vbuf[t]) return -1;
    }
    x->cap = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)x->C * x->L + 1));
    x->occ = (uint32_t*)malloc(sizeof(uint32_t) * (x->L + 1));
    x->feas = (uint64_t*)malloc(sizeof(uint64_t) * (x->woff[x->C] + 1));
    x->taken = (uint64_t*)malloc(sizeof(uint64_t) * (x->toff[x->K] + 1));
    if (!x->cap || !x->occ || !x->feas || !x->taken) return -1;
    return 0;
}

/* One placement of the prepared problem (tally, feasibility, assignment).
 * cap_out / occ_out may be NULL. Returns the number of placed jobs. */
int jspf_run(jspf_ctx* x, int32_t* assign, uint32_t* cap_out, uint32_t* occ_out) {
    run_phase(x, tally_phase);
    run_phase(x, feas_phase);
    const int placed = assign_all(x, assign);
    if (cap_out) memcpy(cap_out, x->cap, sizeof(uint32_t) * (size_t)x->C * x->L);
    if (occ_out) memcpy(occ_out, x->occ, sizeof(uint32_t) * x->L);
    return placed;
}

/* Timed loops (the bench's CPU legs, timed in C like the engine's
 * jsp_place_loop, so that no Python call overhead sits in either figure):
 * `iters` placements back to back; with rows (nrows > 0), row rows[i % nrows]
 * of the taint column rewritten before each (a watch event's one-row patch,
 * the same write the engine's patched step makes). Returns the wall time in
 * microseconds. */
#include <time.h>
static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e6 + (double)ts.tv_nsec * 1e-3;
}

double jspf_run_loop(jspf_ctx* x, int32_t* assign, uint32_t iters, const uint32_t* rows, uint32_t nrows) {
    uint32_t* taints = (uint32_t*)x->p->taints;
    const double t0 = now_us();
    for (uint32_t i = 0; i < iters; ++i) {
        if (nrows > 0) {
            const uint32_t r = rows[i % nrows];
            __atomic_store_n(taints + r, __atomic_load_n(taints + r, __ATOMIC_RELAXED), __ATOMIC_RELEASE);
        }
        (void)jspf_run(x, assign, NULL, NULL);
    }
    return now_us() - t0;
}

/* The cold recovery timed in C, like the engine's jsp_recovery_loop: per
 * trial the idle period (slept, or spun when spin != 0), a one-row write of
 * vals[k] into the taint column (the watch event's patch), the gap, then one
 * placement. out_us[3t] = the write, [3t+1] = the placement, [3t+2] = the gap
 * as it passed. */
static void wait_us(double us, int spin) {
    if (us <= 0.0) return;
    if (spin) {
        const double end = now_us() + us;
        while (now_us() < end) {
        }
        return;
    }
    struct timespec ts;
    ts.tv_sec = (time_t)(us / 1e6);
    ts.tv_nsec = (long)((us - (double)ts.tv_sec * 1e6) * 1e3);
    while (nanosleep(&ts, &ts) != 0) {
    }
}

void jspf_recovery_loop(jspf_ctx* x, int32_t* assign, uint32_t trials, double idle_us, double gap_us, int spin,
                        const uint32_t* rows, const uint32_t* vals, uint32_t nrows, double* out_us) {
    uint32_t* taints = (uint32_t*)x->p->taints;
    for (uint32_t t = 0; t < trials; ++t) {
        wait_us(idle_us, spin);
        const uint32_t k = nrows ? t % nrows : 0u;
        const double t0 = now_us();
        if (nrows) __atomic_store_n(taints + rows[k], vals[k], __ATOMIC_RELEASE);
        const double t1 = now_us();
        wait_us(gap_us, spin);
        const double t2 = now_us();
        (void)jspf_run(x, assign, NULL, NULL);
        const double t3 = now_us();
        out_us[3 * t] = t1 - t0;
        out_us[3 * t + 1] = t3 - t2;
        out_us[3 * t + 2] = t2 - t1;
    }
}
