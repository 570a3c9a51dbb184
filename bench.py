#!/usr/bin/env python3
"""Benchmark of the MI355X exclusive-topology placement engine.

Metric (BASELINE.json): exclusive-topology placements/sec at 15k nodes; p99
recovery placement latency. Workload (`value`): config 2 -- a 15,000-node /
1,000-rack post-delete snapshot and a full-JobSet recovery of 990 jobs x 15
pods. One step = one `jsp_place` call through the C ABI, as
the recovery path makes it: the run list goes host -> device, the engine
tallies, decides feasibility and assigns all 990 jobs, and assign[] comes
back to the caller's host buffer (placements/sec = J_placed /
wall time of jsp_place including H2D and D2H). The snapshot is resident (its
upload is the "post-delete snapshot ready" point and is not timed).
`kernel_only_*` is the same placement from device-resident runs to a
device-resident assign[] (no host round trip).

`--gpus N` (torchrun, one rank per GPU): config 2 has ~0.4 MB of rows and does
not shard usefully, so ranks run independent replicas (weak scaling, no
data-path collective, SURVEY.md §8e "replicas only"); value = all ranks'
placements / max-over-ranks time. The sharded path of config 4 (1M nodes,
node dimension split over the ranks, per-leaf tallies SUM-all-reduced by RCCL)
is reported beside it under "cfg4_1M".

Roofline: the dominant kernel's average duration comes from two HIP events
recorded on the launch stream around K back-to-back launches; its algorithmic
bytes are DESIGN.md §4's. `traffic` is the PMC-measured HBM bytes per launch
of the same kernel from the committed rocprofv3 passes under profiles/
(FETCH_SIZE x 2 for gfx950's wide-load halving + WRITE_SIZE, per
MI355X_MICROARCH.md "HBM"), or null when no pass for it is committed.

CPU baseline: oracle/cpu_fast.c, an optimized threaded evaluator of the same
rules (bit-exact with the oracle), timed on this host at 1 thread, 2 threads
(the reference manager's 2-CPU limit) and every core of the box's share.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md "Chip-level parameters")
SHAPES = {0: "three launches (tally -> feas -> assign + expand)", 1: "fused single launch",
          2: "single-class compaction, one launch",
          3: "single-class compaction answered by the resident service (no launch per placement)",
          4: "fused shape answered by the resident service (no launch per placement)"}
KERNEL = {0: "tally_kernel", 1: "place_fused_kernel", 2: "place_compact_kernel", 3: "place_compact_kernel",
          4: "place_fused_kernel"}


def tally_bytes(p) -> int:
    """Algorithmic bytes of one tally launch: every node row read once
    (labels 8W + taints 4 + free 4R + excl 4 B), leaf offsets read,
    per-(class, leaf) capacities and per-leaf occupancy written once."""
    n = p.nodes
    row = 8 * n.n_label_words + 4 + 4 * n.n_res + 4
    L = n.n_leaves
    return n.n_nodes * row + 4 * (L + 1) + 4 * len(p.classes) * L + 4 * L


def compact_bytes(p) -> int:
    """Algorithmic bytes of one compaction launch (one leaf-level class): the
    rows and leaf offsets read once, assign[] written once (the per-leaf
    tallies stay in LDS)."""
    n = p.nodes
    row = 8 * n.n_label_words + 4 + 4 * n.n_res + 4
    return n.n_nodes * row + 4 * (n.n_leaves + 1) + 4 * p.n_jobs


def placement_tail_bytes(p) -> int:
    """Algorithmic bytes of the feasibility + assignment tail: tallies read
    back once, one 64-bit bitmap word per 64 domains per class, runs read,
    assign[] written."""
    L = p.topology.n_leaves
    C = len(p.classes)
    words = sum((p.topology.n_domains[c.level] + 63) // 64 for c in p.classes)
    n_runs = int((np.diff(p.job_class.astype(np.int64)) != 0).sum()) + (1 if p.n_jobs else 0)
    return 4 * (C + 1) * L + 8 * words + 8 * n_runs + 4 * p.n_jobs


def pmc_traffic(kernel: str, cfg: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    passes (latest round under profiles/): FETCH_SIZE (KiB, x2 on gfx950) +
    WRITE_SIZE (KiB), averaged over that kernel's dispatches."""
    def avg(path):
        vals = []
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if name.startswith("void "):
                    name = name[5:]
                if name.startswith("jsp::"):
                    name = name[5:]
                if name.startswith(kernel):
                    vals.append(float(row["Counter_Value"]))
        return sum(vals) / len(vals) if vals else None
    dirs = []
    for r in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")), reverse=True):
        dirs += [os.path.join(r, sub) for sub in ("final", "mid", "baseline", "")]  # newest evidence first
    for d in dirs:
        fp, wp = os.path.join(d, f"pmc_fetch_cfg{cfg}.csv"), os.path.join(d, f"pmc_write_cfg{cfg}.csv")
        if os.path.exists(fp) and os.path.exists(wp):
            fa, wa = avg(fp), avg(wp)
            if fa is not None and wa is not None:
                return {"bytes": round((2 * fa + wa) * 1024), "source": os.path.relpath(d, ROOT)}
    return None


def trace_avg_us(kernel: str):
    """Median duration (µs) of `kernel` in the newest committed rocprofv3
    kernel-trace summary under profiles/ (this bench run under the profiler),
    taken at the grid size with the most dispatches (the timed cfg2 loop):
    the cross-check of the event-timed average, which also counts the gap
    between back-to-back launches."""
    for r in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")), reverse=True):
        for sub in ("final", "mid", "baseline"):
            f = os.path.join(r, sub, "summary.txt")
            if not os.path.exists(f):
                continue
            best = None
            for line in open(f):
                t = line.split()
                if not t or not t[0].startswith(kernel) or "median_ns=" not in line:
                    continue
                n = int(line.split("n=")[1].split()[0])
                med = int(line.split("median_ns=")[1].split()[0])
                if best is None or n > best[0]:
                    best = (n, med)
            if best:
                return round(best[1] / 1e3, 3), os.path.relpath(f, ROOT)
    return None, None


def event_loop_us(fn, k: int, stream) -> float:
    """Average µs per call of `fn` over k back-to-back calls, HIP events on
    the launch stream around the whole loop."""
    import torch
    s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.default_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(k):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / k


def cold_us(fn, k: int, stream, scrub) -> float:
    """Median µs of one call of `fn` with cold caches: before each call a
    512 MiB buffer is read and written on the same stream, which evicts the
    256 MiB Infinity Cache and every XCD's L2; HIP events bracket the call."""
    import torch
    s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.default_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    with torch.cuda.stream(s):
        for _ in range(k):
            scrub.add_(1)
            a.record(s)
            fn()
            b.record(s)
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def cpu_threads() -> int:
    """Threads of this host's share: OMP_NUM_THREADS (the GPU box sets it to
    its per-GPU CPU share; os.cpu_count() there reports the whole machine),
    bounded by the affinity mask."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp))) if omp and omp.isdigit() else aff


def time_cpu(fc, seconds: float):
    """µs per placement of the prepared FastCPU over a bounded sample."""
    fc.run()
    n, t0 = 0, time.perf_counter()
    while True:
        fc.run()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return dt * 1e6 / n, n, dt


def host_api_latency(eng, p, trials: int, trial_fn=None):
    """Host-API wall of jsp_place (µs): over `trials` seeded trial snapshots
    when trial_fn is given (upload untimed: "post-delete snapshot ready" ->
    "assign[] returned"), else repeated calls on the resident snapshot."""
    from jobset_amd.snapshot import job_runs
    lat = []
    if trial_fn is not None:
        for t in range(trials):
            pt = trial_fn(t)
            eng.upload_snapshot(pt.nodes)
            call = eng.host_placer(*job_runs(pt.job_class))
            t0 = time.perf_counter()
            call()
            lat.append((time.perf_counter() - t0) * 1e6)
        eng.upload_snapshot(p.nodes)
    else:
        call = eng.host_placer(*job_runs(p.job_class))
        for _ in range(10):
            call()
        for _ in range(trials):
            t0 = time.perf_counter()
            call()
            lat.append((time.perf_counter() - t0) * 1e6)
    lat.sort()
    pct = lambda q: round(lat[min(len(lat) - 1, int(q * len(lat)))], 1)  # noqa: E731
    return {"p50_us": pct(0.50), "p99_us": pct(0.99), "n": len(lat)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--trials", type=int, default=1000, help="recovery-latency trials (p99) on config 2")
    ap.add_argument("--cpu-seconds", type=float, default=9.0, help="bounded CPU-baseline sample (all legs)")
    ap.add_argument("--no-cfg4", action="store_true", help="skip the 1M-node sharded leg")
    ap.add_argument("--no-configs", action="store_true", help="skip the per-config (1, 3, 5) lines")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from jobset_amd import synth
    from jobset_amd.distributed import ShardedPlacement, barrier, max_over_ranks
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs

    stream = torch.cuda.current_stream().cuda_stream
    eng = Engine(local)

    def device_step(p):
        rc_np, rl_np = job_runs(p.job_class)
        rc = torch.from_numpy(rc_np.astype(np.int32)).cuda()
        rl = torch.from_numpy(rl_np.astype(np.int32)).cuda()
        out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")

        def step():
            eng.place_device(rc.data_ptr(), rl.data_ptr(), rc_np.shape[0], p.n_jobs, out.data_ptr(), stream)
        return step, out

    # ------------------------------------------------ config 2: host-API placements/s (value)
    p = synth.config2()
    eng.load(p)
    J = p.n_jobs
    shape = eng.place(p.job_class).fused
    call = eng.host_placer(*job_runs(p.job_class))
    for _ in range(args.warmup):
        call()
    # The resident service (shape 3) stays on the GPU between calls, and a
    # device-wide synchronize waits for it to leave: it is stopped right
    # before each synchronize, and its restart by the first timed call and
    # its stop after the last are inside the timed region.
    eng.service_stop()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call()
    eng.service_stop()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    placed = int((call.assign >= 0).sum())
    value = placed * args.steps * world / elapsed

    # the service's own clock: per request, first tile saw it -> last tile's
    # assign[] drained (100 MHz device stamps, timing on; not the timed loop)
    svc = None
    if shape == 3:
        eng.set_timing(True)
        for _ in range(args.warmup):
            call()
        eng.timing(reset=True)
        for _ in range(args.steps):
            call()
        ts = eng.timing(reset=True)
        eng.set_timing(False)
        eng.service_stop()
        req_us = ts.svc_us / max(ts.svc_calls, 1)
        svc = {"request_us_device": round(req_us, 3),
               "achieved_gbs": round(compact_bytes(p) / (req_us * 1e-6) / 1e9, 2),
               "calls": int(ts.svc_calls),
               "note": "device time of one request inside the resident kernel (stamps on, which add "
                       "~0.5-1 us); the host-API wall adds the host-link hand-offs"}

    # ------------------------------------------------ config 2: kernel-only (device-resident runs and assign)
    step, out = device_step(p)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    el_dev = max_over_ranks(time.perf_counter() - t0, world)
    assert int((out[:J].cpu().numpy() >= 0).sum()) == placed

    # dominant kernel: the step's single launch (compaction / fused), else the
    # tally. With the resident service (shape 3) the same tile code runs inside
    # the persistent kernel, which HIP events cannot bracket per request: the
    # roofline is the launch-path compaction kernel's, the service's own
    # per-request device time is under "service".
    if shape in (1, 2, 3, 4):
        dom_us = event_loop_us(step, args.steps, stream)
        tb = compact_bytes(p) if shape in (2, 3) else tally_bytes(p) + placement_tail_bytes(p)
    else:
        cap = torch.empty((len(p.classes) + 1, p.topology.n_leaves), dtype=torch.int32, device="cuda")
        dom_us = event_loop_us(lambda: eng.tally_device(cap.data_ptr(), cap[-1].data_ptr(), p.topology.n_leaves,
                                                        stream), args.steps, stream)
        tb = tally_bytes(p)
    eng.check()
    achieved = tb / (dom_us * 1e-6) / 1e9
    # the same kernel's dispatch-only duration from the committed rocprofv3 trace of this bench (cfg2 grid)
    tr_us, tr_src = trace_avg_us(KERNEL[shape])
    traffic = pmc_traffic(KERNEL[shape], 2)

    # ------------------------------------------------ p50/p99 recovery latency (host API, trial snapshots)
    lat2 = host_api_latency(eng, p, args.trials, synth.config2) if rank == 0 and args.trials > 0 else None
    eng.service_stop()

    # ------------------------------------------------ CPU baseline (rank 0, N=1 only): optimized evaluator
    cpu = None
    T = cpu_threads()
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from oracle import oracle as O
        legs = []
        for th in sorted({1, 2, T}):
            fc = O.FastCPU(th)
            fc.prepare(p)
            a, _, _, pl = fc.run()
            assert np.array_equal(a, call.assign), "CPU evaluator differs from the engine"
            us, n, dt = time_cpu(fc, args.cpu_seconds / 3)
            fc.close()
            legs.append({"threads": th, "us_per_placement": round(us, 2),
                         "placements_per_s": round(pl / (us * 1e-6), 1), "runs": n, "seconds": round(dt, 2)})
        best = legs[-1]
        cpu = {"value": best["placements_per_s"], "unit": "placements/s", "cores": best["threads"], "kind": "port",
               "nproc": os.cpu_count(), "threads_share": T,
               "sample": f"config 2 placed {best['runs']} times in {best['seconds']} s by oracle/cpu_fast.c "
                         f"({best['threads']} threads, -O3 AVX2, same snapshot and rules, bit-exact with the "
                         f"engine); legs at 1/2/{T} threads below",
               "legs": legs}

    # ------------------------------------------------ configs 1, 3, 5 (one GPU)
    configs = None
    if rank == 0 and not args.no_configs:
        configs = {}
        for cfg in (1, 3, 5):
            pc = synth.CONFIGS[cfg]()
            eng.load(pc)
            r = eng.place(pc.job_class)
            st, _ = device_step(pc)
            for _ in range(5):
                st()
            us = event_loop_us(st, 50, stream)
            eng.check()
            line = {"nodes": pc.nodes.n_nodes, "jobs": pc.n_jobs, "classes": len(pc.classes),
                    "levels": pc.topology.n_levels, "placed": r.placed, "shape": SHAPES[r.fused],
                    "kernel_us_per_placement": round(us, 2),
                    "kernel_placements_per_s": round(r.placed / (us * 1e-6), 1),
                    "host_api_resident": host_api_latency(eng, pc, 200)}
            if cfg in (3, 5):
                line["host_api_recovery_trials"] = host_api_latency(eng, pc, 200, synth.CONFIGS[cfg])
            eng.service_stop()
            if world == 1 and args.cpu_seconds > 0:
                from oracle import oracle as O
                for th in sorted({1, T}):
                    fc = O.FastCPU(th)
                    fc.prepare(pc)
                    us_c, _, _ = time_cpu(fc, min(0.5, args.cpu_seconds / 10))
                    fc.close()
                    line[f"cpu_fast_{th}t_us_per_placement"] = round(us_c, 1)
            configs[f"cfg{cfg}"] = line
        eng.load(p)

    # ------------------------------------------------ config 4: 1M nodes, sharded over the ranks
    cfg4 = None
    if not args.no_cfg4:
        p4 = synth.config4()
        sp = ShardedPlacement(Engine(local) if world > 1 else eng, p4, rank, world, stream)
        for _ in range(max(2, args.warmup // 4)):
            sp.step()
        torch.cuda.synchronize()
        barrier(world)
        steps4 = max(10, args.steps // 4)
        t0 = time.perf_counter()
        for _ in range(steps4):
            sp.step()
        torch.cuda.synchronize()
        barrier(world)
        el4 = max_over_ranks(time.perf_counter() - t0, world)
        placed4 = sp.placed()
        sp.engine.set_timing(True)
        for _ in range(steps4):
            sp.step()
        torch.cuda.synchronize()
        t4 = sp.engine.timing(reset=True)
        sp.engine.set_timing(False)
        n4 = max(t4.calls - t4.fused_calls, 1)
        # tally alone, back to back, events around the loop
        C4, L4 = len(p4.classes), p4.topology.n_leaves
        cap4 = torch.zeros((C4 + 1, L4), dtype=torch.int32, device="cuda")
        tally_us = event_loop_us(lambda: sp.engine.tally_device(cap4.data_ptr(), cap4[-1].data_ptr(), L4, stream),
                                 steps4, stream)
        tb4 = tally_bytes(p4) if world == 1 else sp.shard_tally_bytes()
        scrub = torch.zeros(128 << 20, dtype=torch.int32, device="cuda")  # 512 MiB
        tally_cold = cold_us(lambda: sp.engine.tally_device(cap4.data_ptr(), cap4[-1].data_ptr(), L4, stream),
                             20, stream, scrub)
        copy_ceiling = None
        if world == 1:  # achievable streaming rate: a cold copy of the same byte count
            src = torch.empty(tb4 // 2 // 16 * 4, dtype=torch.int32, device="cuda").fill_(1)
            dst = torch.empty_like(src)
            cu = cold_us(lambda: dst.copy_(src), 20, stream, scrub)
            copy_ceiling = {"bytes": 2 * src.numel() * 4, "cold_us": round(cu, 2),
                            "cold_gbs": round(2 * src.numel() * 4 / (cu * 1e-6) / 1e9, 1)}
            del src, dst
        del scrub
        sp.engine.check()
        cfg4 = {"workload": "cfg4: 1,048,576 nodes / 50,000 racks, 40,000 jobs x 16 pods, C=4",
                "placements_per_s": round(placed4 * steps4 / el4, 1), "ms_per_step": round(el4 * 1e3 / steps4, 4),
                "placed": placed4, "tally_us": round(tally_us, 2),
                "tally_gbs": round(tb4 / (tally_us * 1e-6) / 1e9, 1),
                "tally_frac": round(tb4 / (tally_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "tally_cold_us": round(tally_cold, 2),
                "tally_cold_gbs": round(tb4 / (tally_cold * 1e-6) / 1e9, 1),
                "tally_cold_frac": round(tb4 / (tally_cold * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "copy_ceiling_same_bytes": copy_ceiling,
                "tally_traffic": pmc_traffic("tally_kernel", 4) if world == 1 else None,
                "feas_us": round(t4.feas_ms * 1e3 / n4, 2),
                "assign_expand_us": round(t4.assign_ms * 1e3 / n4, 2),
                "allreduce_us": sp.allreduce_us(), "shards": world}

    if rank == 0:
        line = {
            "metric": "exclusive-topology placements/sec at 15k nodes; p99 recovery placement latency",
            "value": round(value, 1),
            "unit": "placements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "cfg2: 15k-node / 1k-rack post-delete snapshot, full-JobSet recovery; one step "
                                   "= one host-API jsp_place (run list in, assign[] back in the caller's host buffer)",
                       "nodes": p.nodes.n_nodes, "domains": p.topology.n_leaves, "jobs": J,
                       "pods_per_job": p.classes[0].pods, "classes": len(p.classes),
                       "shape": SHAPES[shape], "parallelism": f"replicas{world}"},
            "kernel_only_placements_per_s": round(placed * args.steps * world / el_dev, 1),
            "kernel_only_us_per_step": round(el_dev * 1e6 / args.steps, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic["bytes"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "kernel": KERNEL[shape], "bytes_per_launch": tb, "avg_us": round(dom_us, 3),
                         "trace_median_us": tr_us, "trace_source": tr_src,
                         "note": "latency-bound: one launch moving 0.43 MB; see DESIGN.md §8"},
            "service": svc,
            "p50_recovery_us": lat2["p50_us"] if lat2 else None,
            "p99_recovery_us": lat2["p99_us"] if lat2 else None,
            "recovery_trials": lat2["n"] if lat2 else 0,
            "cpu_baseline": cpu,
            "configs": configs,
            "cfg4_1M": cfg4,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
