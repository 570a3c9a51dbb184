#!/usr/bin/env python3
"""Interleaved in-process A/B of a resident-service switch read at each
service start: JSP_SVC_ROW_CACHE (the tiles' LDS row cache, default) or
JSP_SVC_EARLY (python tools/ab_rowcache.py ROUNDS early: the compaction answer
read from its tagged entries). For cfg2, cfg3, cfg5, ROUNDS alternations of
300 host-API calls with the switch on and off (the service is restarted at
each switch). Prints per variant the median of the per-round p50 and p99
(µs). Diagnostic only."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    var_env = "JSP_SVC_EARLY" if len(sys.argv) > 2 and sys.argv[2] == "early" else "JSP_SVC_ROW_CACHE"
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    from oracle import oracle as O
    eng = Engine(0)
    out = {}
    for cfg in ((1, 2) if var_env == "JSP_SVC_EARLY" else (2, 3, 5)):
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        a = O.place_c(p)[0]
        call = eng.host_placer(*job_runs(p.job_class))
        res = {"on": [], "off": []}
        for r in range(rounds):
            for var in (("on", "off") if r % 2 == 0 else ("off", "on")):
                os.environ[var_env] = "1" if var == "on" else "0"
                eng.service_stop()
                for _ in range(30):
                    call()
                lat = []
                for _ in range(300):
                    t0 = time.perf_counter()
                    call()
                    lat.append((time.perf_counter() - t0) * 1e6)
                assert np.array_equal(call.assign, a)
                lat.sort()
                res[var].append((lat[150], lat[297]))
        out[f"cfg{cfg}"] = {v: {"p50": round(float(np.median([x[0] for x in res[v]])), 2),
                                "p99": round(float(np.median([x[1] for x in res[v]])), 2)} for v in res}
        print(json.dumps({f"cfg{cfg}": out[f"cfg{cfg}"]}), flush=True)
    eng.service_stop()


if __name__ == "__main__":
    main()
