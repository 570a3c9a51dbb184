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
`kernel_only` is the same placement from device-resident runs to a
device-resident assign[] (no host round trip).

p99 recovery latency (`p99_recovery_us`): the realistic, cold recovery
(failures are hours apart): the caller's thread sleeps past the resident
service's idle exit, a watch event patches one row, and after the
reconciler's round trip (1 ms) the recreate calls jsp_place; timed = the
patch call + the place call, >= 1000 trials issued and timed in C
(jspb_recovery_loop). Gaps 0 and 10 ms and the parked service are reported
beside it, each next to the CPU evaluator's same recovery at equal sample
size. The bench sets JSP_SERVICE_IDLE_MS=30 (unless given) so that a trial
sleeps only 35 ms and 1000 trials fit the run; a 10 ms gap stays inside the
idle limit's half, so the service stays up across it as with the default 50.

`--gpus N` (torchrun, one rank per GPU): config 2 has ~0.4 MB of rows and does
not shard usefully, so ranks run independent replicas (weak scaling, no
data-path collective, SURVEY.md §8e "replicas only"); value = all ranks'
placements / max-over-ranks time. The sharded path of config 4 (1M nodes,
node dimension split over the ranks, per-leaf tallies SUM-all-reduced by RCCL)
is reported beside it under "cfg4".

Roofline: the dominant kernel's average duration comes from events on the
dispatch packets of K back-to-back launches on the launch stream; its
algorithmic bytes are DESIGN.md §4's. `traffic` is the PMC-measured HBM bytes
per launch of the same kernel from the committed rocprofv3 passes under
profiles/ (FETCH_SIZE x 2 for gfx950's wide-load halving + WRITE_SIZE, per
MI355X_MICROARCH.md "HBM"), or null when no pass for it is committed.

CPU baseline: oracle/cpu_fast.c, an optimized threaded evaluator of the same
rules (bit-exact with the oracle), timed on this host at 1 thread, 2 threads
(the reference manager's 2-CPU limit) and every core of the box's share.

Prints ONE compact JSON line on rank 0 (build_line; tests/test_bench_line.py
keeps it under the driver's 8 KB tail). Every measured figure, with its
context, goes to the detail file (--detail-out, default
gpurun_out/bench_detail.json); DESIGN.md §8 defines each field.
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
METRIC = "exclusive-topology placements/sec at 15k nodes; p99 recovery placement latency"
LINE_MAX_BYTES = 6144  # the driver keeps the last 8 KB of stdout+stderr; leave room for stderr
SHAPES = {0: "three launches", 1: "fused single launch", 2: "one-class compaction, one launch",
          3: "compaction service (resident)", 5: "split service (resident tiles, host walk)",
          7: "tally + feasibility launches, host walk", 8: "split tiles launched once, host walk"}
KERNEL = {0: "tally_kernel", 1: "place_fused_kernel", 2: "place_compact_kernel", 3: "place_compact_kernel",
          4: "place_fused_kernel", 5: "place_fused_kernel", 7: "tally_kernel", 8: "place_split_service_kernel"}
# cold recovery: the gap between the patch and the place (ms) -> share of --cold-trials
COLD_GAPS = {1.0: 1.0, 0.0: 0.1, 10.0: 0.1}
COLD_SLEEP_EXTRA_MS = 5.0  # a trial sleeps the idle limit plus this (the service has left)
COLD_WARM = 2  # untimed trials before each cold leg, GPU and CPU alike


_T0 = time.perf_counter()
_PROGRESS = True  # rank 0 only (set in main)


def progress(msg: str) -> None:
    """One short line on stderr per phase: the run's progress (a silent run of
    minutes reads as hung to a watchdog), before the one JSON line on stdout."""
    if _PROGRESS:
        print(f"bench: {msg} ({time.perf_counter() - _T0:.0f} s)", file=sys.stderr, flush=True)


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


def evidence_dirs():
    """Committed profile directories, newest evidence first: the one named in
    profiles/LATEST (written by the profiling script of the final tree), then
    every profiles/r*/<run>/ by round (descending) and file time."""
    out = []
    latest = os.path.join(ROOT, "profiles", "LATEST")
    if os.path.exists(latest):  # a path under profiles/ (scripts/collect_profiles.sh writes it)
        d = os.path.join(ROOT, "profiles", open(latest).read().strip())
        if os.path.isdir(d):
            out.append(d)
    for r in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")), reverse=True):
        subs = [d for d in glob.glob(os.path.join(r, "*")) if os.path.isdir(d)]
        subs.sort(key=lambda d: max((os.path.getmtime(f) for f in glob.glob(os.path.join(d, "*"))), default=0.0),
                  reverse=True)
        out += [d for d in subs + [r] if d not in out]
    return out


def latest_dir():
    """The evidence directory profiles/LATEST names (None when absent)."""
    f = os.path.join(ROOT, "profiles", "LATEST")
    return os.path.join(ROOT, "profiles", open(f).read().strip()) if os.path.exists(f) else None


def pmc_traffic(kernel, cfg: int):
    """HBM bytes per launch of `kernel` (a name prefix or a tuple of them) from
    the committed rocprofv3 PMC passes (latest round under profiles/):
    FETCH_SIZE (KiB, x2 on gfx950) + WRITE_SIZE (KiB), averaged over that
    kernel's dispatches."""
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
    for d in evidence_dirs():
        fp, wp = os.path.join(d, f"pmc_fetch_cfg{cfg}.csv"), os.path.join(d, f"pmc_write_cfg{cfg}.csv")
        if os.path.exists(fp) and os.path.exists(wp):
            fa, wa = avg(fp), avg(wp)
            if fa is not None and wa is not None:
                return {"bytes": round((2 * fa + wa) * 1024), "source": os.path.relpath(d, ROOT),
                        "latest": d == latest_dir()}
    return None


def trace_avg_us(kernel: str):
    """Median duration (µs) of `kernel` in the newest committed rocprofv3
    kernel-trace summary under profiles/ (this bench run under the profiler),
    taken at the grid size with the most dispatches (the timed cfg2 loop):
    the cross-check of the event-timed average."""
    for d in evidence_dirs():
        f = os.path.join(d, "summary.txt")
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


def cold_us(fn, k: int, stream, scrub, dirty: bool = False) -> float:
    """Median µs of one call of `fn` with cold caches: before each call a
    512 MiB buffer is read on the same stream (a sum: no lines dirtied), which
    evicts the 256 MiB Infinity Cache and every XCD's L2; HIP events bracket
    the call. dirty=True reads and writes it instead (add_)."""
    import torch
    s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.default_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    with torch.cuda.stream(s):
        for _ in range(k):
            if dirty:
                scrub.add_(1)
            else:
                scrub.sum()
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
    """µs per placement of the prepared FastCPU over a bounded sample, the
    placements timed in C (jspf_run_loop, batches of 64) like the GPU's
    host-API loop (jspb_place_loop): no interpreter between the calls."""
    fc.run()
    n, tot = 0, 0.0
    while tot < seconds * 1e6:
        tot += fc.run_loop(64)
        n += 64
    return tot / n, n, tot * 1e-6


def _pct(lat, q):
    return round(lat[min(len(lat) - 1, int(q * len(lat)))], 2)


def pcts(lat):
    lat = sorted(lat)
    return {"p50_us": _pct(lat, 0.50), "p95_us": _pct(lat, 0.95), "p99_us": _pct(lat, 0.99),
            "max_us": round(lat[-1], 2), "n": len(lat)}


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
    return pcts(lat)


def settled_place(eng, job_class):
    """Place until the engine answers in its resident shape: the first call
    after the service (re)starts is answered on the launch path while the
    service comes up."""
    for _ in range(4):
        r = eng.place(job_class)
        if r.fused in (3, 4, 5):
            break
    return r


def cold_plan(trials: int, gaps=COLD_GAPS):
    """Trials per gap: the 1 ms gap (the headline's) gets all of `trials`,
    the others a tenth (at least 20)."""
    return {g: max(20, int(round(trials * share))) if share < 1.0 else trials for g, share in gaps.items()} \
        if trials > 0 else {}


def _recovery_rows(p, trials: int, gap: float):
    rows = np.array([(t * 7919 + int(gap * 13)) % max(p.nodes.n_nodes, 1) for t in range(trials)], dtype=np.uint32)
    return rows, np.ascontiguousarray(p.nodes.taints[rows], dtype=np.uint32)  # same values: the snapshot is unchanged


def _recovery_line(out):
    tot = out[:, 0] + out[:, 1]
    line = pcts(tot.tolist())
    pa, pl = pcts(out[:, 0].tolist()), pcts(out[:, 1].tolist())
    line.update({"patch_p50_us": pa["p50_us"], "patch_p99_us": pa["p99_us"],
                 "place_p50_us": pl["p50_us"], "place_p99_us": pl["p99_us"],
                 "gap_ms_p50": round(float(np.median(out[:, 2])) * 1e-3, 3)})
    return line


def cold_recovery_latency(eng, p, plan, idle_ms: float):
    """The realistic recovery (failures are hours apart,
    keps/262-ConfigurableFailurePolicy/README.md:232-234): the resident
    service has idle-exited (the caller sleeps past JSP_SERVICE_IDLE_MS), a
    watch event patches one row (the failed job's node back to schedulable),
    then the recreate calls jsp_place. Timed: the patch call plus the place
    call. Between them a gap: 0 (the place right behind the patch) or the time
    the reconciler needs before it recreates -- the deletions that produce the
    patches are foreground deletes whose completion triggers the recreate
    (pkg/controllers/jobset_controller.go:553-576, 698-709), at least one
    API-server round trip (1 and 10 ms here); the gap itself is not counted.
    The trials run in C (jspb_recovery_loop: sleep, patch, gap, place, each
    call timed by the library's clock), as a cgo caller would make them."""
    from jobset_amd.snapshot import job_runs
    if not plan:
        return None
    call = eng.host_placer(*job_runs(p.job_class))
    call()
    out = {}
    for gap, trials in plan.items():
        progress(f"cold recovery ({p.name}), gap {gap:g} ms, {trials} trials")
        rows, vals = _recovery_rows(p, trials, gap)
        # COLD_WARM untimed trials first (as the CPU leg): the leg's first
        # trial after a mode change or another leg is not a recovery's
        call.recovery(COLD_WARM, (idle_ms + COLD_SLEEP_EXTRA_MS) * 1e3, gap * 1e3, rows[:COLD_WARM], vals[:COLD_WARM])
        eng.timing(reset=True)
        res = call.recovery(trials, (idle_ms + COLD_SLEEP_EXTRA_MS) * 1e3, gap * 1e3, rows, vals)
        t = eng.timing(reset=True)
        line = _recovery_line(res)
        line["answered_by_service"] = int(t.svc_calls)
        out[f"gap_{gap:g}ms"] = line
    return out


def cpu_cold_recovery(p, plan, threads, idle_ms: float):
    """The same recovery on the CPU evaluator, like for like with the GPU legs
    and, like them, timed in C (jspf_recovery_loop): after the same idle
    sleep, the same one-row patch (written into the evaluator's columns), the
    same gap (slept), then one placement; timed = patch + placement, the gap
    excluded. The widest leg (the box's share: the CPU's best median) runs the
    GPU leg's number of trials, so the two p99s are order statistics of equal
    samples; narrower legs run a fifth as many (context). (The evaluator's
    pool threads spin between placements -- cpu_fast.c worker -- so its
    multi-thread legs start with hot workers: a CPU-favouring baseline.)"""
    from oracle import oracle as O
    out = {}
    for gap, trials in plan.items():
        legs = {}
        for th in threads:
            progress(f"CPU cold recovery ({p.name}), gap {gap:g} ms, {th} threads")
            fc = O.FastCPU(th)
            fc.prepare(p)
            fc.run()
            n = trials if th == max(threads) else max(20, trials // 5)
            rows, vals = _recovery_rows(p, n, gap)
            fc.recovery_loop(COLD_WARM, (idle_ms + COLD_SLEEP_EXTRA_MS) * 1e3, gap * 1e3, rows[:COLD_WARM],
                             vals[:COLD_WARM])  # untimed, as the GPU leg's
            res = fc.recovery_loop(n, (idle_ms + COLD_SLEEP_EXTRA_MS) * 1e3, gap * 1e3, rows, vals)
            fc.close()
            legs[f"{th}t"] = pcts((res[:, 0] + res[:, 1]).tolist())
        out[f"gap_{gap:g}ms"] = legs
    return out


def cold_vs_cpu(cold, cpu):
    """Per gap: the GPU cold p50/p95/p99 beside the best like-for-like CPU
    leg's (the leg with the best median, at the GPU leg's sample size)."""
    out = {}
    for g, legs in cpu.items():
        if g not in cold:
            continue
        name, best = min(legs.items(), key=lambda kv: kv[1]["p50_us"])
        out[g] = {"gpu_p50_us": cold[g]["p50_us"], "gpu_p95_us": cold[g]["p95_us"], "gpu_p99_us": cold[g]["p99_us"],
                  "gpu_n": cold[g]["n"], "best_cpu_leg": name, "cpu_p50_us": best["p50_us"],
                  "cpu_p95_us": best["p95_us"], "cpu_p99_us": best["p99_us"], "cpu_n": best["n"]}
    return out


def cpu_patched_step(p, threads, seconds: float):
    """The CPU counterpart of patched_step_us: one row written into the
    evaluator's columns, then one placement, back to back (µs per step)."""
    from oracle import oracle as O
    out = {}
    for th in threads:
        fc = O.FastCPU(th)
        fc.prepare(p)
        fc.run()
        rows = np.array([(i * 7919) % max(p.nodes.n_nodes, 1) for i in range(16)], dtype=np.uint32)
        n, tot = 0, 0.0
        while tot < seconds * 1e6:
            tot += fc.run_loop(64, rows)  # timed in C, like the GPU leg
            n += 64
        out[f"{th}t"] = round(tot / n, 2)
        fc.close()
    return out


def patched_step_us(eng, p, steps: int):
    """Host-API steps with one row patched before each placement (a watch
    event between recoveries): the patch rides in the next request
    (micro-patch) and the resident tiles apply it before they answer. µs per
    (patch + place), timed in C (jspb_place_loop with patch rows)."""
    from jobset_amd.snapshot import job_runs
    call = eng.host_placer(*job_runs(p.job_class))
    rows = np.array([(i * 7919) % p.nodes.n_nodes for i in range(16)], dtype=np.uint32)
    taints = np.ascontiguousarray(p.nodes.taints[rows], dtype=np.uint32)
    call.loop(20, rows, taints)
    tot, med, p99 = call.loop(steps, rows, taints)
    return {"mean_us": round(tot / steps, 3), "p50_us": round(med, 2), "p99_us": round(p99, 2)}


def cpu_legs(p, ref_assign, threads, seconds_total: float, placed: int):
    """cpu_fast.c placing `p` at each thread count (bit-exact with the
    engine's answer), each leg timed in C over a bounded sample."""
    from oracle import oracle as O
    legs = []
    for th in threads:
        fc = O.FastCPU(th)
        fc.prepare(p)
        a = fc.run()[0]
        assert np.array_equal(a, ref_assign), "CPU evaluator differs from the engine"
        us, n, dt = time_cpu(fc, seconds_total / len(threads))
        fc.close()
        legs.append({"threads": th, "us_per_placement": round(us, 2),
                     "placements_per_s": round(placed / (us * 1e-6), 1), "runs": n, "seconds": round(dt, 2)})
    return legs


def device_set_leg(p4, ref_assign, steps: int):
    """cfg4 through jsp_engine_create_multi over every visible GPU of this
    process (RCCL all-reduce between distinct devices; ids {0, 0} on a
    one-GPU box: two shards and the on-device add). Host-API step time and
    bit-exactness against the single-device engine's answer."""
    import torch
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    n_dev = torch.cuda.device_count()
    ids = list(range(n_dev)) if n_dev > 1 else [0, 0]
    try:
        with Engine(devices=ids) as ds:
            ds.load(p4)
            call = ds.host_placer(*job_runs(p4.job_class))
            for _ in range(3):
                call()
            us = call.loop(steps)[0] / steps  # timed in C (jspb_place_loop), like the single-device leg
            sh, nd = ds.shards()
            exact = bool(np.array_equal(call.assign, ref_assign))
            return {"device_ids": ids, "shards": sh, "devices": nd, "us_per_step": round(us, 1),
                    "placed": int((call.assign >= 0).sum()),
                    "placements_per_s": round(int((call.assign >= 0).sum()) / (us * 1e-6), 1),
                    "bit_exact_vs_single_device": exact, "steps": steps}
    except Exception as ex:  # noqa: BLE001 -- reported in the line, never hidden
        return {"device_ids": ids, "error": str(ex)[:200]}


def relaunch_with_torchrun(n: int) -> int:
    """Run this bench under torchrun with n ranks (one per GPU) as a child
    process; returns its exit code. Only called before anything touches the
    GPU, and the parent never replaces itself (no exec)."""
    import socket
    import subprocess
    try:
        import torch
        n_dev = torch.cuda.device_count()  # does not initialise the GPU
    except Exception:  # noqa: BLE001
        n_dev = 0
    if n > n_dev:
        print(f"bench.py: --gpus {n} but this box has {n_dev} GPU(s)", file=sys.stderr)
        return 2
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def bind_to_gpu_node(device: int):
    """Run this rank's threads on the CPUs of its GPU's NUMA node (the
    numactl --cpunodebind a latency-bound deployment uses; Kubernetes' topology
    manager gives a GPU pod the same with its single-numa-node policy): every
    host-API call polls pinned host memory the GPU writes, and a thread on the
    other socket pays the cross-socket coherence on each line. The CPU
    baseline legs run under the same binding."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return {"bound": False, "why": "hipDeviceGetPCIBusId failed"}
        bdf = buf.value.decode().lower()
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
    except (OSError, ValueError) as ex:
        return {"bound": False, "why": str(ex)}
    if node < 0:
        return {"bound": False, "gpu": bdf, "why": "no NUMA node reported"}
    allowed = os.sched_getaffinity(0)
    local = set()
    for c in allowed:
        g = glob.glob(f"/sys/devices/system/cpu/cpu{c}/node*")
        if g and int(os.path.basename(g[0])[4:]) == node:
            local.add(c)
    if not local:
        return {"bound": False, "gpu": bdf, "gpu_numa_node": node, "why": "none of the allowed CPUs is on that node"}
    os.sched_setaffinity(0, local)
    return {"bound": True, "gpu": bdf, "gpu_numa_node": node, "cpus": len(local), "of_allowed": len(allowed)}


# ----------------------------------------------------------------------------- the printed line

def _r(x, nd=2):
    return None if x is None else round(float(x), nd)


def _cold_row(v):
    """[gpu p50, p95, p99, n, cpu p50, p95, p99, n] (µs) of one gap."""
    return [v["gpu_p50_us"], v["gpu_p95_us"], v["gpu_p99_us"], v["gpu_n"],
            v["cpu_p50_us"], v["cpu_p95_us"], v["cpu_p99_us"], v["cpu_n"]]


def _cold_rows(vs):
    return {g.replace("gap_", ""): _cold_row(v) for g, v in (vs or {}).items()} or None


def build_line(d: dict) -> dict:
    """The one JSON line the driver parses, from the bench's detail dict:
    numbers only (DESIGN.md §8 defines every field), so that it stays under
    LINE_MAX_BYTES whatever the measured values."""
    c2 = d["cfg2"]
    line = {
        "metric": METRIC, "value": c2["value"], "unit": "placements/s", "n_gpus": d["world"],
        "steps": d["steps"], "warmup": d["warmup"], "ms_per_step": c2["ms_per_step"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": "cfg2: 15k-node/1k-rack post-delete snapshot, full-JobSet recovery; one step = "
                               "one host-API jsp_place (run list in, assign[] back in host memory)",
                   "nodes": c2["nodes"], "domains": c2["domains"], "jobs": c2["jobs"],
                   "pods_per_job": c2["pods_per_job"], "classes": c2["classes"],
                   "shape": c2["shape"], "parallelism": f"replicas{d['world']}"},
        "host_api_us": {"p50": c2.get("loop_p50_us"), "p99": c2.get("loop_p99_us")},
        "kernel_only": {"placements_per_s": c2.get("kernel_only_placements_per_s"),
                        "us_per_step": c2.get("kernel_only_us_per_step")},
    }
    rf = c2.get("roofline")
    if rf:
        line["roofline"] = {"bound": "hbm", "achieved": rf["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": rf["frac"], "traffic": rf.get("traffic"), "kernel": rf["kernel"],
                            "bytes": rf["bytes"], "avg_us": rf["avg_us"], "trace_median_us": rf.get("trace_median_us")}
    cpu = c2.get("cpu")
    if cpu:
        line["cpu_baseline"] = {"value": cpu["value"], "unit": "placements/s", "cores": cpu["cores"], "kind": "port",
                                "sample": cpu["sample"],
                                "legs_us": {str(x["threads"]): x["us_per_placement"] for x in cpu["legs"]}}
        line["gpu_over_best_cpu"] = cpu.get("gpu_over_best_cpu")
    cold = d.get("cold2") or {}
    vs = cold.get("vs_cpu")
    head = (vs or {}).get("gap_1ms") or {}
    g1 = (cold.get("gpu") or {}).get("gap_1ms")
    if g1:
        line["p50_recovery_us"] = g1["p50_us"]
        line["p99_recovery_us"] = g1["p99_us"]
        line["recovery_trials"] = g1["n"]
        line["recovery_leg"] = "cold: idle-exited service, 1-row patch, 1 ms gap, jsp_place; patch+place, timed in C"
        if head:
            line["p99_recovery_cpu_us"] = head["cpu_p99_us"]
            line["p50_recovery_cpu_us"] = head["cpu_p50_us"]
    warm = c2.get("warm_trials")
    if warm:
        line["p99_recovery_warm_us"] = warm["p99_us"]
    if vs:
        line["cold_cols"] = "gpu p50,p95,p99,n | best cpu p50,p95,p99,n (us)"
        line["cold_recovery"] = _cold_rows(vs)
    parked = d.get("cold2_parked")
    if parked:
        line["cold_recovery_parked"] = _cold_rows(parked.get("vs_cpu"))
    ps = c2.get("patched")
    if ps:
        line["patched_step_us"] = {"gpu": ps["mean_us"], "gpu_p99": ps["p99_us"], "cpu_best": c2.get("cpu_patched_best_us")}
    line["link_floor_us"] = c2.get("link_floor_p50_us")
    line["service_request_us_device"] = c2.get("service_request_us_device")
    for name in ("cfg1", "cfg3", "cfg5"):
        c = (d.get("configs") or {}).get(name)
        if not c:
            continue
        e = {"host_p50_us": c["host_api_resident"]["p50_us"], "host_p99_us": c["host_api_resident"]["p99_us"],
             "kernel_only_us": c["kernel_us"], "kernel_loop_us": c.get("kernel_loop_us"),
             "kernel_frac": c["kernel_frac"], "placed": c["placed"], "jobs": c["jobs"]}
        if "cpu_us" in c:
            e["cpu_us"] = c["cpu_us"]
        if c.get("cold_vs_cpu"):
            e["cold"] = _cold_rows(c["cold_vs_cpu"])
        if c.get("service_frac") is not None:
            e["service_frac"] = c["service_frac"]
        line[name] = e
    c4 = d.get("cfg4")
    if c4:
        e = {k: c4.get(k) for k in ("placements_per_s", "host_api_us", "kernel_only_us", "kernel_only_placements_per_s",
                                    "tally_us", "tally_frac", "tally_cold_us", "tally_cold_frac", "copy_cold_us",
                                    "tally_traffic", "allreduce_us", "shards", "placed")}
        cpu4 = c4.get("cpu_baseline")
        if cpu4:
            e["cpu_best_us"] = cpu4["best_us"]
            e["cpu_cores"] = cpu4["cores"]
            e["gpu_over_best_cpu"] = cpu4["gpu_over_best_cpu"]
        ds = c4.get("device_set")
        if ds:
            e["device_set"] = {"us": ds.get("us_per_step"), "shards": ds.get("shards"), "devices": ds.get("devices"),
                               "exact": ds.get("bit_exact_vs_single_device"), "error": ds.get("error")}
        line["cfg4"] = e
    line["host_binding"] = {k: d.get("binding", {}).get(k) for k in ("bound", "gpu_numa_node", "cpus")}
    line["detail"] = d.get("detail_path")
    return line


def emit(line: dict) -> str:
    s = json.dumps(line, separators=(",", ":"))
    if len(s) > LINE_MAX_BYTES:  # never print a line the driver cannot parse: drop the per-config blocks first
        for k in ("cfg1", "cfg5", "cfg3", "cold_recovery_parked", "cfg4"):
            line.pop(k, None)
            s = json.dumps(line, separators=(",", ":"))
            if len(s) <= LINE_MAX_BYTES:
                break
    return s


# ----------------------------------------------------------------------------- measurement

def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--trials", type=int, default=200, help="warm recovery trials (trial snapshots, upload untimed)")
    ap.add_argument("--cpu-seconds", type=float, default=9.0, help="bounded CPU-baseline sample (all legs)")
    ap.add_argument("--cold-trials", type=int, default=1000,
                    help="cold recovery trials on config 2 at the 1 ms gap (a tenth at 0 and 10 ms, and on 3 and 5)")
    ap.add_argument("--no-cfg4", action="store_true", help="skip the 1M-node sharded leg")
    ap.add_argument("--no-configs", action="store_true", help="skip the per-config (1, 3, 5) lines")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="where the full measurement record goes ('' = nowhere)")
    args = ap.parse_args()

    # --gpus N is the job's rank count. Without a launcher (no WORLD_SIZE) and
    # N > 1, this process starts torchrun with N ranks as a child -- before any
    # GPU call -- and exits with its code; a launcher whose world size differs
    # from N, or more ranks than GPUs, is an error, never a silent 1-GPU run.
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if env_world is None and args.gpus > 1:
        sys.exit(relaunch_with_torchrun(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
    # the resident service's idle exit: short enough that a cold trial (sleep
    # past it) costs 35 ms, long enough that a 10 ms gap stays within its half
    os.environ.setdefault("JSP_SERVICE_IDLE_MS", "30")
    idle_ms = float(os.environ["JSP_SERVICE_IDLE_MS"])

    import torch
    import torch.distributed as dist

    n_dev = torch.cuda.device_count()  # counting does not initialise the GPU
    if args.gpus > n_dev:
        sys.exit(f"bench.py: --gpus {args.gpus} but this box has {n_dev} GPU(s)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    global _PROGRESS
    _PROGRESS = rank == 0
    progress(f"start: {world} rank(s), steps {args.steps}, warmup {args.warmup}")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from jobset_amd import synth
    from jobset_amd.distributed import ShardedPlacement, barrier, max_over_ranks
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs

    d = {"world": world, "steps": args.steps, "warmup": args.warmup, "idle_ms": idle_ms}
    d["binding"] = bind_to_gpu_node(local)  # before the engine allocates its pinned buffers and threads
    stream = torch.cuda.current_stream().cuda_stream
    eng = Engine(local)
    T = cpu_threads()
    do_cpu = rank == 0 and world == 1 and args.cpu_seconds > 0

    def device_step(p):
        rc_np, rl_np = job_runs(p.job_class)
        rc = torch.from_numpy(rc_np.astype(np.int32)).cuda()
        rl = torch.from_numpy(rl_np.astype(np.int32)).cuda()
        out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")

        def step():
            eng.place_device(rc.data_ptr(), rl.data_ptr(), rc_np.shape[0], p.n_jobs, out.data_ptr(), stream)
        step.keep = (rc, rl)
        step.rc, step.rl, step.n_runs = rc, rl, rc_np.shape[0]
        return step, out

    # ------------------------------------------------ config 2: host-API placements/s (value)
    progress("config 2: host-API placements/s")
    p = synth.config2()
    eng.load(p)
    J = p.n_jobs
    shape = settled_place(eng, p.job_class).fused
    call = eng.host_placer(*job_runs(p.job_class))
    for _ in range(args.warmup):
        call()
    # The resident service stays on the GPU between calls, and a device-wide
    # synchronize waits for it to leave: it is stopped right before each
    # synchronize. One untimed call after the opening synchronize restarts it
    # (the steady state of back-to-back placements; its cold start is measured
    # apart, "cold_recovery"); its stop after the last timed call is inside
    # the timed region.
    eng.service_stop()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    call()
    eng.timing(reset=True)
    t0 = time.perf_counter()
    # the K timed jsp_place calls, issued from C (jspb_place_loop) as a cgo
    # caller's loop would: no interpreter between them
    _, loop_p50, loop_p99 = call.loop(args.steps)
    eng.service_stop()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    tphase = eng.timing(reset=True)
    placed = int((call.assign >= 0).sum())
    value = placed * args.steps * world / elapsed
    c2 = {"value": round(value, 1), "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
          "nodes": p.nodes.n_nodes, "domains": p.topology.n_leaves, "jobs": J, "placed": placed,
          "pods_per_job": p.classes[0].pods, "classes": len(p.classes), "shape": SHAPES.get(shape, str(shape)),
          "loop_p50_us": round(loop_p50, 3), "loop_p99_us": round(loop_p99, 3),
          "library_us_per_call": round((tphase.host_prep_us + tphase.host_wait_us) / max(int(tphase.host_calls), 1), 3),
          "svc_calls": int(tphase.svc_calls)}
    d["cfg2"] = c2

    # the service's own clock: per request, first tile saw it -> last tile's
    # answer drained (100 MHz device stamps, timing on; not the timed loop)
    if shape == 3:
        eng.set_timing(True)
        for _ in range(args.warmup):
            call()
        eng.timing(reset=True)
        for _ in range(max(args.steps, 200)):
            call()
        ts = eng.timing(reset=True)
        eng.set_timing(False)
        eng.service_stop()
        req_us = ts.svc_us / max(ts.svc_calls, 1)
        c2["service_request_us_device"] = round(req_us, 3)
        c2["service_achieved_gbs"] = round(compact_bytes(p) / (req_us * 1e-6) / 1e9, 2)
        # one row patched before each call: the patch rides in the request
        c2["patched"] = patched_step_us(eng, p, max(200, args.steps * 5))
    eng.service_stop()
    if rank == 0:
        floor = eng.link_floor(2000)
        c2["link_floor_p50_us"], c2["link_floor_p99_us"] = round(floor[0], 2), round(floor[1], 2)

    # ------------------------------------------------ config 2: kernel-only (device-resident runs and assign)
    progress("config 2: kernel-only")
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
    c2["kernel_only_placements_per_s"] = round(placed * args.steps * world / el_dev, 1)
    c2["kernel_only_us_per_step"] = round(el_dev * 1e6 / args.steps, 3)

    # dominant kernel: the step's single launch (compaction / fused), else the
    # tally. The resident service runs the same tile code inside the
    # persistent kernel, which HIP events cannot bracket per request: the
    # roofline is the launch-path compaction kernel's, timed by events on the
    # dispatch packets of back-to-back launches (jspb_place_device_timed).
    n_dev_iters = max(200, args.steps)
    if shape in (1, 2, 3, 4):
        dom_med, dom_us = eng.place_device_timed(step.rc.data_ptr(), step.rl.data_ptr(), step.n_runs, J,
                                                 out.data_ptr(), n_dev_iters)
        tb = compact_bytes(p) if shape in (2, 3) else tally_bytes(p) + placement_tail_bytes(p)
    else:
        cap = torch.empty((len(p.classes) + 1, p.topology.n_leaves), dtype=torch.int32, device="cuda")
        dom_med, dom_us = eng.tally_device_timed(cap.data_ptr(), cap[-1].data_ptr(), p.topology.n_leaves, n_dev_iters)
        tb = tally_bytes(p)
    eng.check()
    achieved = tb / (dom_us * 1e-6) / 1e9
    tr_us, tr_src = trace_avg_us(KERNEL[shape])
    traffic = pmc_traffic(KERNEL[shape], 2)
    c2["roofline"] = {"kernel": KERNEL[shape], "bytes": tb, "avg_us": round(dom_us, 3), "median_us": round(dom_med, 3),
                      "achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 5),
                      "traffic": traffic["bytes"] if traffic else None,
                      "traffic_source": traffic["source"] if traffic else None,
                      "trace_median_us": tr_us, "trace_source": tr_src}

    # ------------------------------------------------ recovery latency (rank 0)
    progress("config 2: recovery latency")
    if rank == 0 and args.trials > 0:
        c2["warm_trials"] = host_api_latency(eng, p, args.trials, synth.config2)
    plan2 = cold_plan(args.cold_trials) if rank == 0 else {}
    if plan2:
        cold = {"gpu": cold_recovery_latency(eng, p, plan2, idle_ms)}
        eng.service_stop()
        if do_cpu:
            cold["cpu"] = cpu_cold_recovery(p, plan2, sorted({2, T}), idle_ms)
            cold["vs_cpu"] = cold_vs_cpu(cold["gpu"], cold["cpu"])
        d["cold2"] = cold
        # the same recovery with the service parked (JSP_SERVICE_PARKED: no
        # idle exit, a dedicated GPU -- the GPU side of the CPU pool's
        # spinning threads): the 1 ms gap at the headline's sample size (its
        # p99 beside the CPU leg's at equal n), no gap at the short gaps'
        plan_p = {1.0: args.cold_trials, 0.0: max(20, args.cold_trials // 10)}
        eng.set_service(True, parked=True)
        settled_place(eng, p.job_class)
        gp = cold_recovery_latency(eng, p, plan_p, idle_ms)
        eng.service_stop()
        eng.set_service(True)
        parked = {"gpu": gp}
        if "cpu" in cold:
            parked["vs_cpu"] = cold_vs_cpu(gp, {g: v for g, v in cold["cpu"].items() if g in gp})
        d["cold2_parked"] = parked

    # ------------------------------------------------ CPU baseline (rank 0, N=1 only): optimized evaluator
    progress("config 2: CPU baseline legs")
    if do_cpu:
        legs = cpu_legs(p, call.assign, sorted({1, 2, T}), args.cpu_seconds, placed)
        best = max(legs, key=lambda x: x["placements_per_s"])  # the fastest leg is the baseline
        c2["cpu"] = {"value": best["placements_per_s"], "cores": best["threads"], "legs": legs,
                     "sample": f"cfg2 placed {best['runs']}x in {best['seconds']} s by oracle/cpu_fast.c "
                               f"({best['threads']} threads, fastest of 1/2/{T}; bit-exact with the engine)",
                     "gpu_over_best_cpu": round(value / best["placements_per_s"], 3)}
        if "patched" in c2:
            legs_p = cpu_patched_step(p, sorted({2, T}), min(2.0, args.cpu_seconds / 6))
            c2["cpu_patched_legs_us"] = legs_p
            c2["cpu_patched_best_us"] = min(legs_p.values())

    # ------------------------------------------------ configs 1, 3, 5 (one GPU)
    progress("configs 1, 3, 5")
    if rank == 0 and not args.no_configs:
        configs = {}
        for cfg in (1, 3, 5):
            progress(f"config {cfg}")
            pc = synth.CONFIGS[cfg]()
            eng.load(pc)
            r = settled_place(eng, pc.job_class)
            st, out_c = device_step(pc)
            for _ in range(5):
                st()
            loop_us = event_loop_us(st, 200, stream)  # ctypes-issued calls back to back, events around the loop
            # the device path's own step: first dispatch start -> last dispatch end (jspb_place_device_timed)
            us = eng.place_device_timed(st.rc.data_ptr(), st.rl.data_ptr(), st.n_runs, pc.n_jobs, out_c.data_ptr(), 200)[0]
            eng.check()
            # the device path's launch shape (no service there): what the launch path reports
            eng.set_service(False)
            dev_shape = eng.place(pc.job_class).fused
            eng.set_service(True)
            r = settled_place(eng, pc.job_class)
            kb = compact_bytes(pc) if dev_shape == 2 else tally_bytes(pc) if dev_shape == 8 else \
                tally_bytes(pc) + placement_tail_bytes(pc)
            line = {"nodes": pc.nodes.n_nodes, "jobs": pc.n_jobs, "classes": len(pc.classes),
                    "levels": pc.topology.n_levels, "placed": r.placed, "shape": SHAPES.get(r.fused, str(r.fused)),
                    "kernel_us": round(us, 2), "kernel_loop_us": round(loop_us, 2),
                    "kernel_shape": SHAPES.get(dev_shape, str(dev_shape)),
                    "kernel_kernel": KERNEL.get(dev_shape), "kernel_bytes": kb,
                    "kernel_frac": round(kb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
                    "host_api_resident": host_api_latency(eng, pc, 200)}
            if r.fused in (3, 5):
                eng.set_timing(True)
                cl = eng.host_placer(*job_runs(pc.job_class))
                for _ in range(20):
                    cl()
                eng.timing(reset=True)
                for _ in range(200):
                    cl()
                tsv = eng.timing(reset=True)
                eng.set_timing(False)
                dev_us = tsv.svc_us / max(tsv.svc_calls, 1)
                sb = compact_bytes(pc) if r.fused == 3 else tally_bytes(pc)
                line["service_request_us_device"] = round(dev_us, 3)
                line["service_bytes"] = sb
                line["service_frac"] = round(sb / (dev_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
            if cfg in (3, 5):
                line["host_api_recovery_trials"] = host_api_latency(eng, pc, 100, synth.CONFIGS[cfg])
                plan = cold_plan(max(20, args.cold_trials // 10), {1.0: 1.0, 10.0: 1.0, 0.0: 0.5})
                line["cold"] = cold_recovery_latency(eng, pc, plan, idle_ms)
                if line["cold"] is not None and do_cpu:
                    line["cold_cpu"] = cpu_cold_recovery(pc, plan, [T], idle_ms)
                    line["cold_vs_cpu"] = cold_vs_cpu(line["cold"], line["cold_cpu"])
            eng.service_stop()
            if do_cpu:
                from oracle import oracle as O
                for th in sorted({1, T}):
                    fc = O.FastCPU(th)
                    fc.prepare(pc)
                    us_c, _, _ = time_cpu(fc, min(0.5, args.cpu_seconds / 10))
                    fc.close()
                    line[f"cpu_{th}t_us"] = round(us_c, 2)
                line["cpu_us"] = {"1t": line["cpu_1t_us"], f"{T}t": line[f"cpu_{T}t_us"]}
            configs[f"cfg{cfg}"] = line
        d["configs"] = configs
        eng.load(p)

    # ------------------------------------------------ config 4: 1M nodes, sharded over the ranks
    progress("config 4")
    if not args.no_cfg4:
        p4 = synth.config4()
        sp = ShardedPlacement(Engine(local) if world > 1 else eng, p4, rank, world, stream)
        for _ in range(max(2, args.warmup // 4)):
            sp.step()
        torch.cuda.synchronize()
        barrier(world)
        steps4 = max(50, args.steps // 4)
        t0 = time.perf_counter()
        for _ in range(steps4):
            sp.step()
        torch.cuda.synchronize()
        barrier(world)
        el4 = max_over_ranks(time.perf_counter() - t0, world)
        placed4 = sp.placed()
        a4 = sp.assign()
        C4, L4 = len(p4.classes), p4.topology.n_leaves
        cap4 = torch.zeros((C4 + 1, L4), dtype=torch.int32, device="cuda")
        tally_fn = lambda: sp.engine.tally_device(cap4.data_ptr(), cap4[-1].data_ptr(), L4, stream)  # noqa: E731
        for _ in range(10):  # untimed: the first launches into a new output buffer pay its first touch
            tally_fn()
        # the kernel's own time: events on the dispatch packets of back-to-back
        # launches on the engine stream (jspb_tally_device_timed)
        tally_med, tally_us = sp.engine.tally_device_timed(cap4.data_ptr(), cap4[-1].data_ptr(), L4, 200)
        try:
            span_med, span_mean, empty_us, period_us = sp.engine.tally_device_spans(cap4.data_ptr(), cap4[-1].data_ptr(),
                                                                                    L4, 200)
        except Exception:  # noqa: BLE001 -- another tally shape (sharded ranks): no span
            span_med = span_mean = empty_us = period_us = None
        tb4 = tally_bytes(p4) if world == 1 else sp.shard_tally_bytes()
        scrub = torch.zeros(128 << 20, dtype=torch.int32, device="cuda")  # 512 MiB
        tally_cold, _ = sp.engine.tally_device_timed(cap4.data_ptr(), cap4[-1].data_ptr(), L4, 20,
                                                     scrub.data_ptr(), scrub.numel() * 4)
        c4 = {"workload": "cfg4: 1,048,576 nodes / 50,000 racks, 40,000 jobs x 16 pods, C=4", "placed": placed4,
              "shards": world, "kernel_only_us": round(el4 * 1e6 / steps4, 2),
              "kernel_only_placements_per_s": round(placed4 * steps4 / el4, 1),
              "tally_us": round(tally_us, 2), "tally_median_us": round(tally_med, 2),
              "tally_frac": round(tb4 / (tally_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
              "tally_span_us": _r(span_mean), "tally_period_us": _r(period_us), "tally_empty_launch_us": _r(empty_us),
              "tally_cold_us": round(tally_cold, 2),
              "tally_cold_frac": round(tb4 / (tally_cold * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
              "tally_bytes": tb4, "allreduce_us": sp.allreduce_us()}
        if world == 1:
            # the whole single-GPU step on the device (first dispatch -> last), warm and cold
            sw = eng.place_device_timed(sp.rc.data_ptr(), sp.rl.data_ptr(), sp.n_runs, p4.n_jobs, sp.out.data_ptr(), 100)
            sc = eng.place_device_timed(sp.rc.data_ptr(), sp.rl.data_ptr(), sp.n_runs, p4.n_jobs, sp.out.data_ptr(), 20,
                                        scrub.data_ptr(), scrub.numel() * 4)
            c4["step_device_us"] = round(sw[0], 2)
            c4["step_device_cold_us"] = round(sc[0], 2)
            # placements/s through the host API (run list in, assign[] back in host memory)
            call4 = eng.host_placer(*job_runs(p4.job_class))
            for _ in range(5):
                call4()
            tot4, med4, _ = call4.loop(steps4)  # timed in C (jspb_place_loop)
            host4 = tot4 / steps4
            assert np.array_equal(call4.assign, a4), "host API differs from the device path on cfg4"
            c4["host_api_us"] = round(host4, 2)
            c4["host_api_p50_us"] = round(med4, 2)
            c4["placements_per_s"] = round(placed4 / (host4 * 1e-6), 1)
            src = torch.empty(tb4 // 2 // 16 * 4, dtype=torch.int32, device="cuda").fill_(1)
            dst = torch.empty_like(src)
            c4["copy_cold_us"] = round(cold_us(lambda: dst.copy_(src), 20, stream, scrub), 2)
            del src, dst
            c4["tally_traffic"] = (pmc_traffic(("tally_wave",), 4) or {}).get("bytes")
        else:  # the sharded step through torch.distributed (device-resident runs and assign[])
            c4["placements_per_s"] = c4["kernel_only_placements_per_s"]
        del scrub
        sp.engine.check()
        if do_cpu:
            progress("config 4: CPU legs")
            legs4 = cpu_legs(p4, a4, sorted({1, 2, T}), max(1.5, args.cpu_seconds / 2), placed4)
            best4 = max(legs4, key=lambda x: x["placements_per_s"])
            c4["cpu_baseline"] = {"value": best4["placements_per_s"], "cores": best4["threads"],
                                  "best_us": best4["us_per_placement"], "legs": legs4,
                                  "gpu_over_best_cpu": round(c4["placements_per_s"] / best4["placements_per_s"], 2)}
        # the device-set engine inside the C ABI (what the Go manager's one
        # process would drive, main.go:161-190): rank 0 opens every visible GPU
        # (ids {0, 0} on a one-GPU box: two shards, on-device add)
        barrier(world)
        # (one process only: under torchrun the ranks' own process group and
        # engines hold the GPUs, and the device set's RCCL would sit beside it)
        if rank == 0 and world == 1 and os.environ.get("JSP_BENCH_DEVICE_SET", "1") != "0":
            progress("config 4: device set")
            c4["device_set"] = device_set_leg(p4, a4, max(20, args.steps))
            torch.cuda.set_device(local)  # the rank's own device for the barrier (the library restores it too)
        barrier(world)
        d["cfg4"] = c4

    if rank == 0:
        if args.detail_out:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(args.detail_out)), exist_ok=True)
                with open(args.detail_out, "w") as f:
                    json.dump(d, f, indent=1)
                d["detail_path"] = args.detail_out
            except OSError:
                d["detail_path"] = None
        print(emit(build_line(d)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
