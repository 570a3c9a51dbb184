#!/usr/bin/env python3
"""What a cold host-API placement pays after the GPU sat idle (diagnostic).

For idle gaps of 0.1 / 1 / 5 / 20 / 60 / 200 ms before each call, medians
over trials of:
  torch_empty   a 1-element torch op + synchronize (a launch's floor after idling)
  launch_cfg2   jsp_place on config 2 with the resident service off (launch path)
  service_cfg2  jsp_place with the service on (default: a gap past
                JSP_SERVICE_IDLE_MS / 2 restarts it; the launch path answers
                that call and the service is launched after it)
Prints one JSON line per series."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GAPS_MS = (0.1, 1.0, 5.0, 20.0, 60.0, 200.0)


def series(name, fn, trials):
    out = {}
    for g in GAPS_MS:
        ts = []
        for _ in range(trials):
            time.sleep(g * 1e-3)
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e6)
        ts.sort()
        out[f"{g:g}ms"] = {"p50": round(ts[len(ts) // 2], 1), "max": round(ts[-1], 1)}
    print(json.dumps({name: out}), flush=True)


def main():
    import torch
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    x = torch.zeros(1, device="cuda")

    def empty():
        x.add_(1)
        torch.cuda.synchronize()
    for _ in range(20):
        empty()
    series("torch_empty", empty, trials)
    p = synth.config2()
    eng = Engine(0)
    eng.load(p)
    call = eng.host_placer(*job_runs(p.job_class))
    eng.set_service(False)
    for _ in range(20):
        call()
    series("launch_cfg2", call, trials)
    eng.set_service(True)
    for _ in range(20):
        call()
    series("service_cfg2", call, trials)
    eng.service_stop()


if __name__ == "__main__":
    main()
