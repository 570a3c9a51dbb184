/*
 * jsplace.h — C ABI of the MI355X exclusive-topology placement engine.
 *
 * This is the drop-in boundary for JobSet's exclusive-placement path
 * (SURVEY.md §8b). Every entry point takes plain pointers and sizes; no Go,
 * torch or HIP types cross it (device pointers and streams are passed as
 * void* / uintptr-sized handles). Return value: 0 on success, a negative
 * JSP_E* code on failure; the message is available from jsp_last_error()
 * (thread-local). Nothing aborts or throws across the ABI.
 *
 * Which reference interface each entry point replaces (file:line under the
 * reference tree, danielvegamyhre/jobset @ 2024-10-08):
 *
 *  jsp_engine_create / jsp_engine_create_multi / jsp_engine_destroy
 *      Constructed beside NewPodReconciler / NewPodWebhook in main.go:168,186
 *      and injected into them (there is no engine in the reference: the domain
 *      is chosen by kube-scheduler); the device-set form is
 *      the manager process's handle over several GPUs.
 *  jsp_topology_upload / jsp_snapshot_upload / jsp_snapshot_patch
 *      Replace the per-pod cached Node Get of topologyFromPod
 *      (pkg/webhooks/pod_mutating_webhook.go:173-194) and leaderPodTopology
 *      (pkg/controllers/pod_controller.go:242-263) with one resident snapshot
 *      of the node informer cache (RBAC nodes get/list/watch,
 *      config/components/rbac/role.yaml:16-23).
 *  jsp_place / jsp_place_device (= jsp_tally_device + jsp_assign_device)
 *      The placement decision that the leader's exclusive affinity terms
 *      (setExclusiveAffinities, pod_mutating_webhook.go:95-135) delegate to
 *      kube-scheduler, evaluated for every child Job of a JobSet at first
 *      admission and at full recreate (failurePolicyRecreateAll,
 *      pkg/controllers/failure_policy.go:155-175 -> reconcile,
 *      pkg/controllers/jobset_controller.go:172-176, 523-551).
 *      Job order = globalJobIndex (jobset_controller.go:1056-1065).
 *  jsp_resolve_leader_domains
 *      Batched form of setNodeSelector/topologyFromPod
 *      (pod_mutating_webhook.go:137-194): leader node row -> domain id at the
 *      job's topology level (the follower nodeSelector value).
 *  jsp_audit_placements
 *      Batched form of validatePodPlacements / leaderPodTopology /
 *      followerPodTopology (pod_controller.go:172-277).
 *
 * Threading: one engine is not re-entrant; calls on one engine are
 * serialised by an internal mutex (the Go wrapper also holds one).
 *
 * Stream ordering: uploads, patches, jsp_place and the webhook batches run on
 * the engine's own stream and return after it has finished; the *_device
 * entry points enqueue on the caller's stream and return at once -- except
 * where the walk runs on the host (ABI v7, jsp_stats.fused 7 and 8: the
 * multi-class / multi-level shapes the GPU level walker does not take, 256 to
 * 65536 jobs): there the call waits for its own kernels' answer (the stream's
 * earlier work first), walks, and returns with the assign[] copy enqueued on
 * the stream behind them (it waits for the walk's release, so no launch
 * separates the walk from the copy). Every call
 * is ordered after all work the engine enqueued earlier, on whatever stream
 * (the first call on a different stream waits on an event of the previous
 * one), so a patch after a jsp_place_device never races its tally.
 *
 * Kernel-side failures: every wait inside a launch is bounded -- the
 * single-class compaction's look-back, the pipelined batch walk's wait for an
 * earlier batch, the one-launch level walk's expanders' wait for the walker.
 * A wait that gives up writes the launch's tag to an error word and leaves
 * that launch's assign[] invalid. jsp_place reports it (JSP_EHIP) before it
 * returns; the device path reports it from jsp_engine_check (which waits for
 * the engine's work) or, once visible, from the next call on the engine. No
 * timeout returns JSP_OK with a stale assign[].
 *
 * Environment: JSP_SERVICE=0 (no resident service) / =parked, JSP_SERVICE_IDLE_MS
 * (its idle exit, default 50), JSP_RCCL_LIB (device sets) are the operational
 * switches; JSP_TEST_HOOKS is for tests only (jsp_engine.cc TestHooks).
 *
 * This header is the product boundary: every entry point in it is one the Go
 * binding calls (tests/test_abi.py checks the two agree).
 * The bench's and probes' entry points -- C-timed loops, dispatch-timed
 * kernels, the host-link floor, phase clocks, shape selection -- are a
 * separate symbol set, jspb_*, declared in jsplace_bench.h (ABI v7).
 */
#ifndef JSPLACE_H
#define JSPLACE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JSP_ABI_VERSION 7

#define JSP_MAX_LEVELS 4      /* topology levels, 0 = coarsest (zone) .. K-1 = finest (rack) */
#define JSP_MAX_LABEL_WORDS 4 /* 256 interned (key,value) label bits */
#define JSP_MAX_RES 4         /* cpu-milli, memory-MiB, gpu, pods (any 4 the host chooses) */
#define JSP_MAX_CLASSES 64

/* error codes */
#define JSP_OK 0
#define JSP_EINVAL -1   /* bad argument / malformed snapshot */
#define JSP_EHIP -2     /* HIP runtime error (includes: no GPU) */
#define JSP_ENOMEM -3   /* device or host allocation failed */
#define JSP_ESTATE -4   /* call order: no topology / snapshot / classes yet */
#define JSP_ERANGE -5   /* problem exceeds an engine limit (message says which) */

typedef struct jsp_engine jsp_engine;

/* Global domain hierarchy; identical on every shard. Level K-1 domains are the
 * "leaves". Domain ids at each level are dense 0..D_k-1 and ordered so that
 * each domain covers a contiguous leaf range [first_leaf[k][d], first_leaf[k][d+1]).
 * Nesting is required: every level-k boundary is also a level-(k+1) boundary. */
typedef struct jsp_topology {
    uint32_t n_levels;                           /* K, 1..JSP_MAX_LEVELS */
    uint32_t n_domains[JSP_MAX_LEVELS];          /* D_k */
    const uint32_t* first_leaf[JSP_MAX_LEVELS];  /* [D_k+1]; entry K-1 ignored (identity) */
} jsp_topology;

/* Node rows held by this engine (one shard), sorted by leaf domain.
 * Column layout is SoA so every column streams coalesced from HBM. */
typedef struct jsp_nodes {
    uint32_t n_nodes;          /* N rows */
    uint32_t leaf_begin;       /* global id of the first leaf held here */
    uint32_t n_leaves;         /* leaves held here: [leaf_begin, leaf_begin+n_leaves) */
    const uint32_t* leaf_start;/* [n_leaves+1] row offsets (0 .. N) */
    uint32_t n_label_words;    /* W, 1..JSP_MAX_LABEL_WORDS */
    const uint64_t* labels;    /* [W][N] interned (key,value) label bits */
    const uint32_t* taints;    /* [N] interned NoSchedule/NoExecute taint bits */
    uint32_t n_res;            /* R, 1..JSP_MAX_RES */
    const uint32_t* free_res;  /* [R][N] allocatable minus requested */
    const int32_t* excl_owner; /* [N] id of the exclusive job whose domain covers the
                                  row (existing placements), -1 = none */
} jsp_nodes;

/* One requirement class: jobs are deduplicated into classes on the host. */
typedef struct jsp_job_class {
    uint64_t req_labels[JSP_MAX_LABEL_WORDS];    /* bits that must be set (nodeSelector) */
    uint64_t forbid_labels[JSP_MAX_LABEL_WORDS]; /* bits that must be clear (NotIn/DoesNotExist) */
    uint32_t tolerated_taints;                   /* taint bits this class tolerates */
    uint32_t level;                              /* topology level of its exclusive-topology key */
    uint32_t pods;                               /* pods per job (parallelism), >= 1 */
    uint32_t req_res[JSP_MAX_RES];               /* per-pod request per resource, 0 = none */
} jsp_job_class;

typedef struct jsp_stats {
    uint32_t jobs;             /* J */
    uint32_t placed;           /* assign[j] != -1 */
    uint32_t runs;             /* replicated-job runs the assignment walked */
    uint32_t fused;            /* launch shape: 0 tally->feas->assign, 1 fused tail, 2 one-class compaction,
                                  3 one-class compaction answered by the resident service,
                                  4 (unused since ABI v6: the fused resident kernel was retired),
                                  5 split service: resident tiles + the walk on the host,
                                  6 device set: shard tallies combined (RCCL / on-device add), then assign,
                                  7 (ABI v7) tally + feasibility on the GPU, the walk on the host: every
                                    shape the GPU level walker does not take (several levels, or more
                                    than 32 runs), up to 65536 jobs -- launch path and device paths
                                    (jspb_set_fused OFF keeps the GPU walkers: shape 0),
                                  8 (ABI v7) the split service's tiles launched for this one request, the
                                    walk on the host: the launch path and the device paths of every shape
                                    the split service takes, when no tallies are requested */
    double wall_us;            /* host wall time of the call */
} jsp_stats;

/* Engine metrics (ABI v7; SURVEY.md §5 "engine histograms"): what a
 * Prometheus exporter in the Go manager publishes beside the reference's
 * jobset_failed_total / jobset_completed_total counters
 * (pkg/metrics/metrics.go:24-38). Always on, per engine, cheap (a few adds
 * per call under a lock of their own).
 *
 * A log2 histogram: bucket 0 counts values below lo, bucket i (1..30) values
 * in [lo * 2^(i-1), lo * 2^i), bucket 31 the rest. Counts are per bucket (not
 * cumulative: an exporter sums them up for its `le` boundaries lo * 2^i). */
#define JSP_HIST_BUCKETS 32
typedef struct jsp_hist {
    uint64_t count;
    double sum;
    double max;
    uint64_t bucket[JSP_HIST_BUCKETS];
} jsp_hist;

#define JSP_HIST_LO_US 0.5     /* lo of the latency histograms (us): bucket 30 ends at ~537 s */
#define JSP_HIST_LO_JOBS 1.0   /* lo of the batch-size histogram */

typedef struct jsp_metrics {
    jsp_hist place_us;         /* jsp_place / jsp_place_jobs: host wall per call, us (failed calls too) */
    jsp_hist patch_us;         /* jsp_snapshot_patch: host wall per call, us */
    jsp_hist batch_jobs;       /* jobs per successful jsp_place call */
    jsp_hist device_us;        /* device time per placement, us: the resident service's in-kernel request
                                  time, or a single-launch placement's kernel events. Recorded only while
                                  device timing is on (jsplace_bench.h jspb_set_timing): the stamps and
                                  events cost ~1 us per call */
    uint64_t placed;           /* jobs given a domain */
    uint64_t unplaceable;      /* jobs answered -1 */
    uint64_t place_errors;     /* jsp_place calls that returned an error */
    uint64_t patch_errors;     /* jsp_snapshot_patch calls that returned an error */
    uint64_t svc_calls;        /* placements the resident service answered (stats.fused 3 or 5) */
    uint64_t svc_starts;       /* resident service launches (first use, after uploads, idle exits, wakes) */
    uint64_t svc_fallbacks;    /* placements the service could not answer (answered on the launch path) */
} jsp_metrics;

/* jsp_engine_set_service modes. With AUTO, a host-API jsp_place of the
 * one-class compaction shape or of a multi-class / multi-level shape whose
 * tiles fit the GPU at once (no tallies requested) is answered by a resident
 * service kernel: one workgroup per tile stays on the
 * GPU, a dispatcher workgroup polls a request word in pinned host memory, and
 * assign[] goes back into pinned memory -- no launch per placement. It is started by the first such
 * jsp_place, stopped by every upload, jsp_engine_set_service/set_fused and
 * jsp_engine_destroy, and leaves by itself after JSP_SERVICE_IDLE_MS
 * (default 50 ms) without a request; jsp_place restarts it when needed, and
 * so does a jsp_snapshot_patch after a placement it answered (the deletions of
 * a recovery patch the snapshot before the recreate places it).
 * While it runs, a device-wide synchronize (hipDeviceSynchronize,
 * torch.cuda.synchronize) waits for it to leave: call
 * jsp_engine_service_stop first (which also keeps patches from restarting it
 * until the next jsp_place it answers). */
#define JSP_SERVICE_OFF 0
#define JSP_SERVICE_AUTO 1     /* default: the multi-class / multi-level shapes are answered by the split
                                  service -- resident tiles tally and hand back per-domain feasibility,
                                  the host walks (stats.fused = 5) */
#define JSP_SERVICE_PARKED 2   /* AUTO without the idle exit (ABI v6): the service stays on the GPU
                                  between requests however long the gap -- a dedicated GPU, where a
                                  recovery hours after the last placement finds it polling (the
                                  GPU analogue of a CPU pool whose threads spin). It leaves on
                                  jsp_engine_service_stop, an upload, a mode change or destroy;
                                  a device-wide synchronize needs the stop first. JSP_SERVICE=parked
                                  in the environment selects it. Freeing device memory waits for
                                  every kernel on the device as well: with several engines on one
                                  GPU, stop a parked service before another engine's destroy or
                                  re-upload (whose frees would otherwise wait for it). */

/* ---- lifecycle ---- */
int jsp_abi_version(void);
const char* jsp_last_error(void);
int jsp_device_count(int* out);
int jsp_engine_create(int device_id, jsp_engine** out);
/* A device-set engine: one handle over n_devices shard engines (device_ids
 * may repeat: several shards on one GPU). The snapshot given to
 * jsp_snapshot_upload (whole: leaves 0..L) is split by whole level-0 domains
 * into row-balanced shards; jsp_place tallies every shard on its device,
 * SUM-combines the per-(class, leaf) tallies -- one RCCL all-reduce over the
 * distinct devices (ncclCommInitAll in this process; librccl.so.1 is loaded
 * at run time), an on-device add between shards that share a device -- and
 * runs feasibility + assignment on device_ids[0]. Results are bit-identical
 * to a single-device engine (integer sums). Uploads, patches, jsp_place /
 * jsp_place_jobs, jsp_resolve_leader_domains, jsp_audit_placements and the
 * settings work as on a single engine; the *_device entry points return
 * JSP_ESTATE (the device buffers span devices). stats.fused = 6.
 * Replaces, for the Go manager's one process (main.go:161-190), the
 * per-rank torch.distributed step of jobset_amd/distributed.py. */
int jsp_engine_create_multi(const int* device_ids, int n_devices, jsp_engine** out);
/* shards of a device-set engine and its distinct devices (1 and 1 for a
 * single-device engine) */
int jsp_engine_shards(jsp_engine* e, int* shards, int* devices);
void jsp_engine_destroy(jsp_engine* e);

/* ---- snapshot ---- */
int jsp_topology_upload(jsp_engine* e, const jsp_topology* topo);
int jsp_snapshot_upload(jsp_engine* e, const jsp_nodes* nodes);
/* Overwrite n rows (ids in `rows`, local to this shard) of the resident
 * snapshot. delta columns are [W][n], [n], [R][n], [n] (NULL: column
 * unchanged); structure (leaf ranges) is unchanged. The call copies the delta
 * into pinned staging and returns without waiting for the device (ABI v5);
 * every later call sees the patched rows. Who applies it:
 *  - the resident service, when it is up: its dispatcher workgroup reads the
 *    staged delta (up to 4096 rows in one host-link round trip) and writes the
 *    rows; no launch. The patch is posted at once, so it lands during the gap
 *    before the next request, and a request that finds it not yet taken
 *    carries it again (writing a staged delta twice writes the same values);
 *    a dispatcher that never takes it (bounded wait) is stopped and the patch
 *    kernel applies it;
 *  - after the service left, while it is armed (the last jsp_place was
 *    answered by it): a patch is the first sign of a recovery, so the engine's
 *    waker thread restarts the service and posts the patch, followed by a
 *    warm-up request without jobs, off the caller's thread;
 *  - otherwise a patch kernel on the engine stream.
 * Later launches wait for its completion word (or are stream-ordered after
 * the patch kernel); uploads and jsp_engine_sync apply pending patches first. */
int jsp_snapshot_patch(jsp_engine* e, const uint32_t* rows, uint32_t n,
                       const uint64_t* labels, const uint32_t* taints,
                       const uint32_t* free_res, const int32_t* excl_owner);
int jsp_classes_upload(jsp_engine* e, const jsp_job_class* classes, uint32_t n_classes);

/* ---- placement (host buffers; includes H2D of the runs and D2H of results) ----
 * Jobs arrive as replicated-job runs in global order: run i is run_len[i]
 * consecutive jobs of class run_class[i] (one ReplicatedJob with
 * rjob.Replicas children, jobset_controller.go:638-649; global job index =
 * globalJobIndex, :1056-1065). n_jobs = sum of run_len.
 * assign_out [n_jobs]: domain id at the job's class level, -1 = unplaceable.
 * tally_out (nullable) [C][n_leaves_total]: per-(class, leaf) pod capacity.
 * occ_out (nullable) [n_leaves_total]: rows covered by other exclusive jobs. */
int jsp_place(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
              int32_t* assign_out, uint32_t* tally_out, uint32_t* occ_out, jsp_stats* stats);
/* Same with one class id per job (run-length encoded on the host). */
int jsp_place_jobs(jsp_engine* e, const uint32_t* job_class, uint32_t n_jobs,
                   int32_t* assign_out, uint32_t* tally_out, uint32_t* occ_out, jsp_stats* stats);

/* ---- placement (device-resident buffers) ----
 * `stream` is a hipStream_t used as given: NULL = the HIP null stream (torch's
 * default stream), jsp_engine_stream(e) = the engine's own stream.
 * d_cap [C][ld] and d_occ [ld] with ld >= total leaves; a shard writes only
 * columns [leaf_begin, leaf_begin+n_leaves) so the caller can SUM-all-reduce
 * zero-initialised buffers across shards before jsp_assign_device.
 * d_run_class / d_run_len [n_runs] as for jsp_place; n_jobs = their sum. */
int jsp_tally_device(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld,
                     void* stream);
int jsp_assign_device(jsp_engine* e, const uint32_t* d_cap, const uint32_t* d_occ,
                      uint32_t ld, const uint32_t* d_run_class, const uint32_t* d_run_len,
                      uint32_t n_runs, uint32_t n_jobs, int32_t* d_assign, void* stream);
int jsp_place_device(jsp_engine* e, const uint32_t* d_run_class, const uint32_t* d_run_len,
                     uint32_t n_runs, uint32_t n_jobs, int32_t* d_assign, void* stream);

/* ---- follower pinning and audit (batched webhook / PodReconciler work) ----
 * jsp_resolve_leader_domains: for each job, the domain (at `levels[i]`) of
 * the node row its leader is bound to; -1 when the row is -1 (leader not
 * bound / node unknown). Host buffers.
 * jsp_audit_placements: for each job i, followers [follower_off[i],
 * follower_off[i+1]) carry the interned domain id their nodeSelector names
 * (-1 = selector missing); bad_out[i] = number of followers whose domain
 * differs from the domain of leader_rows[i] at levels[i], or 0xFFFFFFFF when
 * the leader row is -1 (leader node unknown). */
int jsp_resolve_leader_domains(jsp_engine* e, const int32_t* leader_rows,
                               const uint32_t* levels, uint32_t n, int32_t* domain_out);
int jsp_audit_placements(jsp_engine* e, const int32_t* leader_rows, const uint32_t* levels,
                         const uint32_t* follower_off, const int32_t* follower_domains,
                         uint32_t n_jobs, uint32_t* bad_out);

/* ---- resident service, metrics, synchronisation ---- */
int jsp_engine_set_service(jsp_engine* e, int mode);
/* Stops the resident service (if running) and waits (bounded: 2 s, then
 * JSP_EHIP and the service stays off until the next upload) for its
 * workgroups to leave. */
int jsp_engine_service_stop(jsp_engine* e);
/* The engine's metrics since creation or the last reset (jsp_metrics). */
int jsp_engine_get_metrics(jsp_engine* e, jsp_metrics* out, int reset);
/* The engine's own stream (a caller may pass it to the *_device calls). */
void* jsp_engine_stream(jsp_engine* e);
/* Waits for every patch and launch the engine has issued. */
int jsp_engine_sync(jsp_engine* e);
/* Waits for every launch the engine has enqueued (on any stream) and returns
 * JSP_EHIP if one of them failed on the device (see "Kernel-side failures"). */
int jsp_engine_check(jsp_engine* e);

#ifdef __cplusplus
}
#endif
#endif /* JSPLACE_H */
