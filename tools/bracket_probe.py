"""What the timed region's closing bracket costs (diagnostic): after K
C-timed jsp_place calls, the service stop, then torch.cuda.synchronize twice
(bench.py's bracket; a one-rank barrier is a no-op). Medians over reps."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
e = Engine(0)
p = synth.config2()
e.load(p)
call = e.host_placer(*job_runs(p.job_class))
for _ in range(20):
    call()
loop, stop, s1, s2, start = [], [], [], [], []
for _ in range(reps):
    e.service_stop()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    call()  # restarts the service
    t1 = time.perf_counter()
    tot, _, _ = call.loop(20)
    t2 = time.perf_counter()
    e.service_stop()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    start.append((t1 - t0) * 1e6)
    loop.append((t2 - t1) * 1e6)
    stop.append((t3 - t2) * 1e6)
    s1.append((t4 - t3) * 1e6)
    s2.append((t5 - t4) * 1e6)
m = lambda v: f"{np.median(v):7.1f}"  # noqa: E731
print(f"restart call {m(start)} us | 20 C-timed calls {m(loop)} us | stop {m(stop)} us | sync1 {m(s1)} us | "
      f"sync2 {m(s2)} us", flush=True)
e.close()
