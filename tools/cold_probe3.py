"""Cold recovery, host side vs GPU side (diagnostic): after
the service idle-exited, a one-row patch (which wakes the service) and,
after a gap, two placements back to back. The idle time and the gap are
either slept (the host core may drop into a deep idle state, as it does for
the CPU evaluator's cold leg) or spun (the host core stays busy, as a
manager deleting pods would be). Per series: patch call, first and second
place (host wall), and the first place's split into host work before the
wait and the wait for the service (jsp_timing)."""
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
e = Engine(0)
p = synth.config2()
e.load(p)
call = e.host_placer(*job_runs(p.job_class))
call()
series = [(w, False, False, g) for w in ("1", "0") for g in (0.0, 0.001, 0.01)] + \
    [(w, True, True, g) for w in ("1", "0") for g in (0.0, 0.001)]
if len(sys.argv) > 2:  # only the slept series (A/B of the waker's spin across processes)
    series = [(w, False, False, g) for w in ("1",) for g in (0.001, 0.01)]
for waker, idle_spin, gap_spin, gap in series:
    os.environ["JSP_SVC_WAKER"] = waker  # read per call (in-process A/B: 0 = the patch call restarts the service)
    if True:
        pa, p1, p2, prep, wt = [], [], [], [], []
        for t in range(trials):
            row = np.array([(t * 7919) % p.nodes.n_nodes], dtype=np.uint32)
            patch = e.host_patcher(row, taints=p.nodes.taints[row])
            wait(0.06, idle_spin)
            e.timing(reset=True)
            t0 = time.perf_counter()
            patch()
            t1 = time.perf_counter()
            if gap:
                wait(gap, gap_spin)
            t2 = time.perf_counter()
            call()
            t3 = time.perf_counter()
            tm = e.timing(reset=True)
            call()
            t4 = time.perf_counter()
            pa.append((t1 - t0) * 1e6)
            p1.append((t3 - t2) * 1e6)
            p2.append((t4 - t3) * 1e6)
            prep.append(tm.host_prep_us)
            wt.append(tm.host_wait_us)
        f = lambda v: f"p50 {np.median(v):.1f} p99 {np.percentile(v, 99):.1f}"  # noqa: E731
        print(f"waker={os.environ['JSP_SVC_WAKER']} idle {'spin ' if idle_spin else 'sleep'} gap {gap * 1e3:g} ms {'spin ' if gap_spin else 'sleep'}: "
              f"patch {f(pa)} | place1 {f(p1)} (prep p50 {np.median(prep):.1f}, wait p50 {np.median(wt):.1f}) | "
              f"place2 {f(p2)}", flush=True)
e.service_stop()
