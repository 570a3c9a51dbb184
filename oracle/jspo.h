/* jspo.h — problem layout shared by the CPU restatements of the placement
 * rules (cpu_ref.c: the parity oracle; cpu_fast.c: the optimized, threaded
 * CPU baseline). TEST INFRASTRUCTURE ONLY (see cpu_ref.c). */
#ifndef JSPO_H
#define JSPO_H
#include <stdint.h>

#define MAXL 4

typedef struct jspo_problem {
    uint32_t n_levels;
    uint32_t n_domains[MAXL];
    const uint32_t* first_leaf[MAXL]; /* [D_k+1]; level K-1 may be NULL (identity) */
    uint32_t n_nodes;
    const uint32_t* leaf_start;       /* [L+1] */
    uint32_t W;
    const uint64_t* labels;           /* [W][N] */
    const uint32_t* taints;           /* [N] */
    uint32_t R;
    const uint32_t* free_res;         /* [R][N] */
    const int32_t* excl;              /* [N] */
    uint32_t n_classes;
    const uint64_t* cls_req;          /* [C][4] */
    const uint64_t* cls_forbid;       /* [C][4] */
    const uint32_t* cls_tol;          /* [C] */
    const uint32_t* cls_level;        /* [C] */
    const uint32_t* cls_pods;         /* [C] */
    const uint32_t* cls_res;          /* [C][4] */
    uint32_t n_jobs;
    const uint32_t* job_class;        /* [J] */
} jspo_problem;

#endif
