#!/usr/bin/env python3
"""Diagnostic: what the bench's closing bracket costs on cfg2 (host API through
the resident service): jsp_engine_service_stop, then torch.cuda.synchronize(),
each timed on the host after a warm call, against a bare synchronize with
nothing running and against one warm call. Median / p90 over 50 rounds (us)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    p = synth.config2()
    eng = Engine(0)
    eng.load(p)
    call = eng.host_placer(*job_runs(p.job_class))
    for _ in range(50):
        call()
    rows = {"call": [], "stop": [], "sync_after_stop": [], "bare_sync": [], "restart_call": []}
    for _ in range(50):
        for _ in range(5):
            call()
        t0 = time.perf_counter()
        call()
        t1 = time.perf_counter()
        eng.service_stop()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        call()
        t5 = time.perf_counter()
        for k, a, b in (("call", t0, t1), ("stop", t1, t2), ("sync_after_stop", t2, t3), ("bare_sync", t3, t4),
                        ("restart_call", t4, t5)):
            rows[k].append((b - a) * 1e6)
    for k, v in rows.items():
        v = np.sort(np.array(v))
        print(f"{k:16s} p50 {np.median(v):8.1f} us  p90 {v[int(0.9 * len(v))]:8.1f} us")


if __name__ == "__main__":
    main()
