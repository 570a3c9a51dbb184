/*
 * jsplace_bench.h -- the measurement and diagnostic symbol set of
 * libjsplace.so (prefix jspb_, ABI v7). Not part of the product boundary
 * (include/jsplace.h): no Go caller binds these. bench.py, the GPU tests and
 * the probes under tools/ use them to time the product entry points from C
 * (no interpreter between calls), to time kernels by events on their own
 * dispatch packets, to read the resident service's device stamps, and to
 * force a launch shape.
 */
#ifndef JSPLACE_BENCH_H
#define JSPLACE_BENCH_H

#include "jsplace.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Phase clocks of the engine's calls (sums since the last reset). The host
 * phases are always accumulated; the device ones (HIP events, service
 * stamps) only while jspb_set_timing(e, 1). */
typedef struct jsp_timing {
    uint64_t calls;            /* timed placements (or tallies) since last reset */
    double tally_ms;           /* summed HIP-event time of the tally kernel */
    double feas_ms;            /* summed HIP-event time of the feasibility-bitmap kernel */
    double assign_ms;          /* summed HIP-event time of the assignment kernel */
    double fused_ms;           /* summed HIP-event time of single-launch placements (fused / compaction) */
    uint64_t fused_calls;      /* placements that ran as a single launch */
    /* host-API placements (jsp_place), host wall clock, always accumulated */
    uint64_t host_calls;
    double host_prep_us;       /* entry to launch: checks, run list into the pinned staging buffer */
    double host_launch_us;     /* the kernel launch call(s) */
    double host_wait_us;       /* launch return to completion seen (completion words or stream sync) */
    double host_post_us;       /* assign[] (and tallies) out, stats; the split service: its host walk (inside wait) */
    /* resident service (jsp_engine_set_service) */
    uint64_t svc_calls;        /* jsp_place calls it answered */
    uint64_t svc_starts;       /* service launches (first use, after uploads, idle exits, restarts) */
    double svc_us;             /* summed in-kernel request time (first tile saw the request -> last tile
                                  done, 100 MHz device clock); accumulated while timing is on */
    uint64_t svc_fallbacks;    /* jsp_place calls the service could not answer (its grid does not fit the
                                  CUs, it left twice, or a request failed on the device): answered by the
                                  launch path instead. When its grid cannot be co-resident the service stays
                                  off until the next upload; otherwise the next call starts it again */
    double svc_ready_us;       /* host time spent waiting for a (re)started service's dispatcher to poll */
    double svc_pre_us;         /* service-answered jsp_place: entry of the service path to the request post
                                  (a queued wake, settling the previous request, patch bookkeeping) (ABI v6) */
    double svc_answer_us;      /* ... the request post to the answer's last entry seen (ABI v6) */
    double svc_first_us;       /* ... the request post to its first answer entry seen (compaction service) */
    /* jsp_snapshot_patch (ABI v5), host wall clock, always accumulated */
    uint64_t patches;          /* patch calls with at least one row */
    double patch_us;           /* their host time (a waker-thread restart is not in it) */
    double wake_us;            /* host time (re)starting the service for a coming recovery, wherever it ran */
    /* the split tiles launched for one request (stats.fused 8, ABI v7), host wall clock */
    uint64_t oneshot_calls;
    double oneshot_launch_us;  /* entry to the launch's return */
    double oneshot_wait_us;    /* ... to every tile's lines seen */
    double oneshot_walk_us;    /* ... the host walk and (device paths) the assign[] copy launch */
    double oneshot_stage_us;   /* the part of oneshot_launch_us before the launch call (staging slot, set-up) */
} jsp_timing;

/* jspb_set_fused modes */
#define JSP_FUSED_OFF 0       /* always tally -> feas -> assign (three launches) */
#define JSP_FUSED_AUTO 1      /* one launch when possible (default): the single-class compaction
                                 for one leaf-level class, the fused tail for small snapshots */

/* jspb_set_fused modes: which launch shape the launch path takes */
#define JSP_FUSED_OFF 0       /* always tally -> feas -> assign (three launches) */
#define JSP_FUSED_AUTO 1      /* one launch when possible (default): the single-class compaction
                                 for one leaf-level class, the fused tail for small snapshots */

/* ---- C-timed loops of the product calls ---- */
/* `iters` jsp_place calls back to back, timed in C (ABI v6): what a cgo
 * caller's loop sees, with no interpreter between the calls (the bench's
 * host-API steps). With n_patch > 0, each call is preceded by a one-row
 * jsp_snapshot_patch of the taint column (row patch_rows[i % n_patch] set to
 * patch_taints[i % n_patch]: a watch event between recoveries). out_us[0]
 * total wall, [1] median and [2] p99 per step, microseconds; assign_out holds
 * the last call's answer. */
int jspb_place_loop(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                   int32_t* assign_out, uint32_t iters, const uint32_t* patch_rows, const uint32_t* patch_taints,
                   uint32_t n_patch, double* out_us);
/* The realistic recovery timed in C (ABI v6), `trials` times: the idle period
 * (idle_us, slept -- or spun when spin != 0), a one-row taint patch
 * (patch_rows[t % n_patch] := patch_taints[t % n_patch]; the failed job's
 * node back to schedulable), the gap (gap_us: the reconciler's round trips
 * between the deletions and the recreate), then jsp_place. out_us[3t] = the
 * patch call, [3t+1] = the place call, [3t+2] = the gap as it passed (us). */
int jspb_recovery_loop(jsp_engine* e, const uint32_t* run_class, const uint32_t* run_len, uint32_t n_runs,
                      int32_t* assign_out, uint32_t trials, double idle_us, double gap_us, int spin,
                      const uint32_t* patch_rows, const uint32_t* patch_taints, uint32_t n_patch, double* out_us);
/* ---- shapes, device timing, clocks ---- */
int jspb_set_fused(jsp_engine* e, int mode);
/* With timing on: the last service request's 100 MHz device-clock stamps, 8
 * per tile (0 request seen, 1 after the acquire, 2 tallied, 3 feasible count
 * scanned, 4 look-back done, 5 assign[] drained; 6-7 unused). Copies up to
 * cap/8 tiles; *n_tiles = how many (0 when no timed request is held). When
 * cap leaves room for one more row after all the tiles, it receives the
 * dispatcher's {0 request seen in the mailbox, 1 bell rung} (ABI v6). */
int jspb_service_clock(jsp_engine* e, uint32_t* out, uint32_t cap, uint32_t* n_tiles);
/* Device time of `iters` back-to-back steps on the engine stream (the bench's
 * kernel-time legs): each step carries a start event on its first dispatch and
 * a stop event on its last (hipExtLaunchKernel: the dispatch packets' own
 * timestamps, as a kernel trace reports them, with no host submit time between
 * them). d_scrub (nullable): a device buffer larger than the caches, read
 * (never written) before every step, so each step starts cold.
 * out_us[0] = median, out_us[1] = mean per step, in microseconds.
 * jspb_tally_device_timed: the tally of jsp_tally_device.
 * jspb_place_device_timed: the whole placement of jsp_place_device. */
int jspb_tally_device_timed(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, uint32_t iters,
                           const void* d_scrub, size_t scrub_bytes, double* out_us);
int jspb_place_device_timed(jsp_engine* e, const uint32_t* d_run_class, const uint32_t* d_run_len, uint32_t n_runs,
                           uint32_t n_jobs, int32_t* d_assign, uint32_t iters, const void* d_scrub,
                           size_t scrub_bytes, double* out_us);
/* The host-link floor (ABI v6): `iters` host -> device -> host round trips
 * through pinned memory with the resident service's polling (four device
 * waves a quarter of a round trip apart poll a request word; the first to
 * see request i writes an ack the host spins on). out_us[0] median, [1]
 * p99, [2] mean, microseconds. Every host-API request pays this at least
 * once; the bench reports it beside the host-API latency. */
int jspb_link_floor(jsp_engine* e, uint32_t iters, double* out_us);
/* The tally's in-kernel span (ABI v6): `iters` back-to-back launches of the
 * one-tile wave tally with per-wave stamps of the device's 100 MHz clock
 * (every wave's start, and its end once its stores drained); per launch the
 * span from the first wave's start to the last wave's end -- a third measure
 * beside the dispatch-packet events and a kernel trace, with no tracer and no
 * dispatch overhead in it. out_us[0] median, [1] mean; out_us[2] the median
 * dispatch-event time of an empty one-workgroup launch (the fixed cost events
 * on the dispatch packets add to a kernel's own span); out_us[3] the launches'
 * period by the same clock (first wave of the first launch to first wave of
 * the last, per launch: execution plus the gap dispatch leaves between
 * back-to-back launches). JSP_ESTATE when the snapshot's tally runs another
 * shape. */
int jspb_tally_device_spans(jsp_engine* e, uint32_t* d_cap, uint32_t* d_occ, uint32_t ld, uint32_t iters,
                           double* out_us);
int jspb_set_timing(jsp_engine* e, int enable);
int jspb_get_timing(jsp_engine* e, jsp_timing* out, int reset);


#ifdef __cplusplus
}
#endif
#endif /* JSPLACE_BENCH_H */
