#!/usr/bin/env python3
"""A/B of the call-entry prefetch of the engine's lines (jsp_engine.cc
warm_engine; test hook warm=0 turns it off) on the realistic cold recovery
of cfg2: sleep 60 ms, one-row patch, gap, jsp_place, timed in C
(jspb_recovery_loop), default and parked service. Alternating blocks per
variant; p50 / p95 / p99 of patch + place, and the patch and place p50.
Diagnostic only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    p = synth.config2()
    res = {}
    for rep in range(reps):
        for hooks in ("", "warm=0"):
            os.environ["JSP_TEST_HOOKS"] = hooks
            eng = Engine(0)
            eng.load(p)
            call = eng.host_placer(*job_runs(p.job_class))
            for parked in (False, True):
                eng.set_service(True, parked=parked)
                call()
                for gap in (1.0, 10.0):
                    rows = np.array([(t * 7919 + rep) % p.nodes.n_nodes for t in range(trials)], dtype=np.uint32)
                    out = call.recovery(trials, 60_000.0, gap * 1e3, rows, p.nodes.taints[rows])
                    res.setdefault((hooks or "warm=1", parked, gap), []).append(out)
                eng.service_stop()
            eng.set_service(True)
            eng.close()
    for k in sorted(res):
        o = np.concatenate(res[k])
        tot = o[:, 0] + o[:, 1]
        q = lambda v, x: float(np.percentile(v, x))  # noqa: E731
        print(f"{k[0]:7s} {'parked ' if k[1] else 'default'} gap {k[2]:4.0f} ms: p50 {q(tot, 50):6.2f} p95 {q(tot, 95):6.2f} "
              f"p99 {q(tot, 99):6.2f} | patch p50 {q(o[:, 0], 50):5.2f} p95 {q(o[:, 0], 95):5.2f} | place p50 "
              f"{q(o[:, 1], 50):5.2f} p95 {q(o[:, 1], 95):5.2f} (n {len(tot)})", flush=True)


if __name__ == "__main__":
    main()
