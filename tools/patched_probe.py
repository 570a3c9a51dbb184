"""Patched steps (diagnostic): host-API placements of cfg2
back to back with k one-row patches before each (k = 0: the resident step;
k = 1: a watch event between recoveries; k = 15: a whole job's nodes, one
watch event each), and the same with one 50-row patch. µs per (patches +
place), p50 over the steps, and the library's service phases."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
e = Engine(0)
p = synth.config2()
e.load(p)
call = e.host_placer(*job_runs(p.job_class))
for _ in range(20):
    call()
N = p.nodes.n_nodes
for k, width in ((0, 1), (1, 1), (2, 1), (15, 1), (1, 50)):
    pats = []
    for i in range(16 * max(k, 1)):
        rows = np.array([((i * 7919) + j * 31) % N for j in range(width)], dtype=np.uint32)
        pats.append(e.host_patcher(rows, taints=p.nodes.taints[rows]))
    lat = []
    e.timing(reset=True)
    for s in range(steps):
        t0 = time.perf_counter()
        for j in range(k):
            pats[(s * k + j) % len(pats)]()
        call()
        lat.append((time.perf_counter() - t0) * 1e6)
    tm = e.timing(reset=True)
    lat = np.array(lat[20:])
    print(f"cfg2 patches {k} x {width} row(s): p50 {np.median(lat):.2f} p99 {np.percentile(lat, 99):.2f} us | "
          f"svc_pre {tm.svc_pre_us / max(tm.svc_calls, 1):.2f} svc_answer {tm.svc_answer_us / max(tm.svc_calls, 1):.2f} "
          f"patch call {tm.patch_us / max(tm.patches, 1):.2f} us", flush=True)
e.service_stop()
