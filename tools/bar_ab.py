"""Host API with the service's request line in pinned host memory (default)
or in device memory written through the BAR (JSP_SVC_BAR=1), interleaved in
one process (diagnostic; the mode is read at each service start). Per round
and mode: cfg1/cfg2/cfg3/cfg5 host-API p50 / p99 over 400 calls, answers
checked against the first call."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
e = Engine(0)
for cfg in (1, 2, 3, 5):
    p = synth.CONFIGS[cfg]()
    e.load(p)
    call = e.host_placer(*job_runs(p.job_class))
    call()
    ref = call.assign.copy()
    res = {"0": [], "1": []}
    for r in range(rounds):
        for mode in ("0", "1"):
            os.environ["JSP_SVC_BAR"] = mode
            e.service_stop()
            for _ in range(50):
                call()
            w = []
            for _ in range(400):
                t0 = time.perf_counter()
                st = call()
                w.append((time.perf_counter() - t0) * 1e6)
            assert np.array_equal(call.assign, ref), f"cfg{cfg} mode {mode}: answer differs"
            res[mode].append((np.median(w), np.percentile(w, 99), st.fused))
    for mode in ("0", "1"):
        a = np.array([(x[0], x[1]) for x in res[mode]])
        print(f"cfg{cfg} bar={mode}: p50 {' '.join(f'{x:.2f}' for x in a[:, 0])} | p99 "
              f"{' '.join(f'{x:.2f}' for x in a[:, 1])} | shape {res[mode][-1][2]}", flush=True)
e.service_stop()
