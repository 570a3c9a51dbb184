/*
 * cpu_ref.c — CPU restatement (parity ORACLE) of the exclusive-topology
 * placement rules. TEST INFRASTRUCTURE ONLY: linked by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the checker /
 * CPU baseline; never by the product path (jobset_amd/).
 *
 * Parity status:
 *   - The reference has no placement algorithm: JobSet only injects the
 *     leader's required podAffinity `job-key In [own]` and podAntiAffinity
 *     `job-key Exists, NotIn [own]` on topologyKey
 *     (pkg/webhooks/pod_mutating_webhook.go:95-135) and pins followers to the
 *     leader's domain (:137-171). The choice of domain is made by
 *     kube-scheduler, which is not in /root/reference nor in go.mod
 *     (go.mod:5-25) and breaks ties at random.
 *   - This file therefore restates the constraints as the deterministic
 *     rules A7/A8 of SURVEY.md §8a (defined by this build). The predicate
 *     semantics (label selector, taint/toleration, resource fit) are a
 *     documented simplification of kube-scheduler's: PARITY UNPINNED against
 *     any reference fixture; they are pinned by the invariants I1-I4
 *      that tests/ check on every output.
 *
 * Rules (one node row n, one class c):
 *   pred(c,n)  = AND_w (labels[w][n] & req[c][w]) == req[c][w]      (nodeSelector)
 *              && AND_w (labels[w][n] & forbid[c][w]) == 0            (NotIn / DoesNotExist)
 *              && (taints[n] & ~tol[c]) == 0                          (NoSchedule/NoExecute)
 *   cap(c,n)   = pred ? min(pods[c], min_{r: req_res[c][r] > 0} floor(free[r][n] / req_res[c][r])) : 0
 *   occ(leaf)  = #rows of the leaf with excl != -1   (covered by another job's
 *                exclusive domain: the symmetric required anti-affinity of an
 *                existing leader, pod_mutating_webhook.go:119-134)
 *   capsum(c,d), occsum(d) = sums over the leaves of domain d at level[c]
 *   feasible(c,d) = capsum(c,d) >= pods[c] && occsum(d) == 0
 *   Jobs in global order (globalJobIndex, jobset_controller.go:1056-1065):
 *     assign[j] = lowest d at level[c_j] with feasible(c_j,d) and d not taken;
 *     -1 if none. Taking d marks taken every domain, at every level, whose
 *     leaf range intersects d's (anti-affinity in both directions: one job
 *     per domain, I2).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "jspo.h"

static uint32_t fl(const jspo_problem* p, uint32_t k, uint32_t d) {
    if (k == p->n_levels - 1 || p->first_leaf[k] == NULL) return d;
    return p->first_leaf[k][d];
}

/* per-(class, leaf) capacity and per-leaf occupancy */
int jspo_tally(const jspo_problem* p, uint32_t* cap /*[C][L]*/, uint32_t* occ /*[L]*/) {
    const uint32_t L = p->n_domains[p->n_levels - 1];
    const uint32_t N = p->n_nodes;
    for (uint32_t c = 0; c < p->n_classes; ++c) {
        const uint64_t* req = p->cls_req + 4 * c;
        const uint64_t* fb = p->cls_forbid + 4 * c;
        const uint32_t tol = p->cls_tol[c];
        const uint32_t pods = p->cls_pods[c];
        const uint32_t* rr = p->cls_res + 4 * c;
        for (uint32_t leaf = 0; leaf < L; ++leaf) {
            uint32_t sum = 0;
            for (uint32_t n = p->leaf_start[leaf]; n < p->leaf_start[leaf + 1]; ++n) {
                int ok = 1;
                for (uint32_t w = 0; w < p->W; ++w) {
                    uint64_t lab = p->labels[(size_t)w * N + n];
                    if ((lab & req[w]) != req[w] || (lab & fb[w]) != 0) ok = 0;
                }
                if ((p->taints[n] & ~tol) != 0) ok = 0;
                if (!ok) continue;
                uint32_t k = pods;
                for (uint32_t r = 0; r < p->R; ++r) {
                    if (rr[r] == 0) continue;
                    uint32_t q = p->free_res[(size_t)r * N + n] / rr[r];
                    if (q < k) k = q;
                }
                sum += k;
            }
            cap[(size_t)c * L + leaf] = sum;
        }
    }
    for (uint32_t leaf = 0; leaf < L; ++leaf) {
        uint32_t o = 0;
        for (uint32_t n = p->leaf_start[leaf]; n < p->leaf_start[leaf + 1]; ++n) o += (p->excl[n] != -1);
        occ[leaf] = o;
    }
    return 0;
}

/* Assignment from per-(class, leaf) capacities and per-leaf occupancy (the
 * multi-GPU path assigns from all-reduced tallies). Returns the number of
 * placed jobs or a negative value on allocation failure. */
int jspo_assign(const jspo_problem* p, const uint32_t* cap, const uint32_t* occ, int32_t* assign) {
    const uint32_t K = p->n_levels;
    const uint32_t L = p->n_domains[K - 1];
    const uint32_t C = p->n_classes;
    uint8_t* feas[64];
    uint8_t* taken[MAXL];
    uint32_t cursor[64];
    int placed = 0;
    /* feasibility per class at its level */
    for (uint32_t c = 0; c < C; ++c) {
        uint32_t k = p->cls_level[c];
        uint32_t D = p->n_domains[k];
        feas[c] = (uint8_t*)calloc(D + 1, 1);
        if (!feas[c]) return -1;
        cursor[c] = 0;
        for (uint32_t d = 0; d < D; ++d) {
            uint64_t cs = 0, os = 0;
            for (uint32_t leaf = fl(p, k, d); leaf < fl(p, k, d + 1); ++leaf) {
                cs += cap[(size_t)c * L + leaf];
                os += occ[leaf];
            }
            feas[c][d] = (cs >= p->cls_pods[c] && os == 0);
        }
    }
    for (uint32_t k = 0; k < K; ++k) {
        taken[k] = (uint8_t*)calloc(p->n_domains[k] + 1, 1);
        if (!taken[k]) return -1;
    }
    /* Greedy in global job order. The per-class cursor only skips domains
     * that are infeasible for the class or already taken; both stay so for
     * the rest of the call, so the lowest available domain never lies behind
     * it. */
    for (uint32_t j = 0; j < p->n_jobs; ++j) {
        uint32_t c = p->job_class[j];
        uint32_t k = p->cls_level[c];
        uint32_t D = p->n_domains[k];
        uint32_t d = cursor[c];
        while (d < D && !(feas[c][d] && !taken[k][d])) ++d;
        cursor[c] = d;
        if (d == D) { assign[j] = -1; continue; }
        assign[j] = (int32_t)d;
        ++placed;
        uint32_t a = fl(p, k, d), b = fl(p, k, d + 1);
        for (uint32_t k2 = 0; k2 < K; ++k2) {
            /* first domain of level k2 whose leaf range ends after a */
            uint32_t lo = 0, hi = p->n_domains[k2];
            while (lo < hi) {
                uint32_t mid = (lo + hi) / 2;
                if (fl(p, k2, mid + 1) > a) hi = mid; else lo = mid + 1;
            }
            for (uint32_t d2 = lo; d2 < p->n_domains[k2] && fl(p, k2, d2) < b; ++d2) {
                uint32_t a2 = fl(p, k2, d2), b2 = fl(p, k2, d2 + 1);
                uint32_t l2 = a > a2 ? a : a2, h2 = b < b2 ? b : b2;
                if (l2 < h2) taken[k2][d2] = 1;
            }
        }
    }
    for (uint32_t c = 0; c < C; ++c) free(feas[c]);
    for (uint32_t k = 0; k < K; ++k) free(taken[k]);
    (void)L;
    return placed;
}

/* Full placement. cap/occ may be NULL. Returns the number of placed jobs or
 * a negative value on allocation failure. */
int jspo_place(const jspo_problem* p, int32_t* assign, uint32_t* cap_out, uint32_t* occ_out) {
    const uint32_t L = p->n_domains[p->n_levels - 1];
    const uint32_t C = p->n_classes;
    uint32_t* cap = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)C * L + 1));
    uint32_t* occ = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)L + 1));
    if (!cap || !occ) return -1;
    jspo_tally(p, cap, occ);
    int placed = jspo_assign(p, cap, occ, assign);
    if (cap_out) memcpy(cap_out, cap, sizeof(uint32_t) * (size_t)C * L);
    if (occ_out) memcpy(occ_out, occ, sizeof(uint32_t) * L);
    free(cap);
    free(occ);
    return placed;
}
