"""Cold recovery, phase by phase (diagnostic): after the
service idle-exited, a one-row patch (which wakes the service) and, after a
gap, two placements back to back. Idle time and gap are slept (the host core
may drop into a deep idle state) or spun (the host core stays busy). Per
series: the patch call, the first placement split into the library's service
path before the request post (svc_pre: a queued wake, settling the warm-up
request, patch bookkeeping) and from the post to the answer (svc_answer), the
Python/ctypes remainder, and the second (warm) placement. The library is the
product one, or another build through JSP_LIB_PATH (tools/bin/ab_inlinewake:
the wake inside the patch call); a third argument "parked" keeps the
service on the GPU through the idle period (JSP_SERVICE_PARKED)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402


def wait(seconds, spin):
    if not spin:
        time.sleep(seconds)
        return
    end = time.perf_counter() + seconds
    while time.perf_counter() < end:
        pass


trials = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
parked = len(sys.argv) > 3 and sys.argv[3] == "parked"  # JSP_SERVICE_PARKED: no idle exit
tag = os.path.basename(os.path.dirname(os.environ.get("JSP_LIB_PATH", ""))) or ("parked" if parked else "product")
e = Engine(0)
if parked:
    e.set_service(True, parked=True)
p = synth.CONFIGS[cfg]()
e.load(p)
call = e.host_placer(*job_runs(p.job_class))
for _ in range(3):
    call()
series = [(False, g) for g in (0.0, 0.001, 0.01)] + [(True, 0.001)]
f = lambda v: f"p50 {np.median(v):5.1f} p99 {np.percentile(v, 99):5.1f}"  # noqa: E731
for spin, gap in series:
    pa, p1, p2, pre, ans, rest = [], [], [], [], [], []
    for t in range(trials):
        row = np.array([(t * 7919) % p.nodes.n_nodes], dtype=np.uint32)
        patch = e.host_patcher(row, taints=p.nodes.taints[row])
        wait(0.06, spin)
        t0 = time.perf_counter()
        patch()
        t1 = time.perf_counter()
        if gap:
            wait(gap, spin)
        e.timing(reset=True)
        t2 = time.perf_counter()
        call()
        t3 = time.perf_counter()
        tm = e.timing(reset=True)
        call()
        t4 = time.perf_counter()
        pa.append((t1 - t0) * 1e6)
        p1.append((t3 - t2) * 1e6)
        p2.append((t4 - t3) * 1e6)
        pre.append(tm.svc_pre_us)
        ans.append(tm.svc_answer_us)
        rest.append((t3 - t2) * 1e6 - tm.svc_pre_us - tm.svc_answer_us)
    tot = np.array(pa) + np.array(p1)
    print(f"cfg{cfg} {tag:12s} {'spin ' if spin else 'sleep'} gap {gap * 1e3:4g} ms: patch {f(pa)} | place1 {f(p1)} "
          f"[svc_pre {f(pre)}; svc_answer {f(ans)}; outside {f(rest)}] | place2 {f(p2)} | patch+place1 {f(tot)}",
          flush=True)
e.service_stop()
