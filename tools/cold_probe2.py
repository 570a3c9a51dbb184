"""Cold recovery phases (diagnostic): after the service idle-exited, a
one-row patch and a place, with a gap between them; per series the patch
call, the place call and the sum (host wall, medians and p99), with the
patch waking the service (default) or not (JSP_SVC_WAKE=0 in a child run)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
e = Engine(0)
p = synth.config2()
e.load(p)
call = e.host_placer(*job_runs(p.job_class))
call()
wake = os.environ.get("JSP_SVC_WAKE", "1")
series = [(m, 0.06, g) for m in ("1", "0") for g in (0.0, 0.001, 0.01)] + [(m, 0.002, g) for g in (0.0, 0.001) for m in ("1", "2", "0")] * 2
for mode, idle, gap in series:
    os.environ["JSP_SVC_PATCH"] = mode  # read per call (in-process A/B: 1 carried, 2 posted, 0 patch kernel)
    pa, pl, starts, wk = [], [], [], []
    for t in range(trials):
        row = np.array([(t * 7919) % p.nodes.n_nodes], dtype=np.uint32)
        patch = e.host_patcher(row, taints=p.nodes.taints[row])
        time.sleep(idle)
        e.timing(reset=True)
        t0 = time.perf_counter()
        patch()
        t1 = time.perf_counter()
        if gap:
            time.sleep(gap)
        t2 = time.perf_counter()
        call()
        t3 = time.perf_counter()
        pa.append((t1 - t0) * 1e6)
        pl.append((t3 - t2) * 1e6)
        tm = e.timing(reset=True)
        starts.append(tm.svc_starts)
        wk.append(tm.wake_us)
    pa, pl = np.array(pa), np.array(pl)
    print(f"wake={wake} svc_patch={mode} idle {idle * 1e3:g} ms gap {gap * 1e3:g} ms: patch p50 {np.median(pa):.1f} p99 {np.percentile(pa, 99):.1f} | "
          f"place p50 {np.median(pl):.1f} p99 {np.percentile(pl, 99):.1f} | wake (in patch) p50 {np.median(wk):.1f} | "
          f"starts/trial {np.mean(starts):.2f}",
          flush=True)
e.service_stop()
