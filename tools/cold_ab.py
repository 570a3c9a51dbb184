#!/usr/bin/env python3
"""Cold recovery A/B on one box (diagnostic): cfg2, gap 1 ms, timed in C --
the default service (waker sleeping 200 us between polls), the waker spinning
(test hook waker_spin=1: a host core kept awake, as the CPU evaluator's pool
threads are), the parked service, and the 16-thread CPU evaluator; each
variant `trials` trials per round, rounds alternating. Usage:
cold_ab.py [trials] [rounds]. Run with JSP_SERVICE_IDLE_MS=30."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(a):
    return "/".join(f"{np.percentile(a, q):.2f}" for q in (50, 95, 99))


def main():
    import torch
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    from oracle import oracle as O
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    idle = float(os.environ.get("JSP_SERVICE_IDLE_MS", "30"))
    torch.cuda.init()
    p = synth.config2()
    rows = np.array([(i * 7919) % p.nodes.n_nodes for i in range(trials)], dtype=np.uint32)
    vals = np.ascontiguousarray(p.nodes.taints[rows], dtype=np.uint32)
    engines = {}
    variants = os.environ.get("COLD_AB_VARIANTS", "default,waker_spin,parked").split(",")
    hooks_of = {"default": None, "waker_spin": "waker_spin=1", "poll50": "waker_poll_us=50",
                "poll20": "waker_poll_us=20", "parked": None}
    for label, hooks in ((v, hooks_of[v]) for v in variants):
        if hooks:
            os.environ["JSP_TEST_HOOKS"] = hooks
        e = Engine(0)
        os.environ.pop("JSP_TEST_HOOKS", None)
        e.load(p)
        if label == "parked":
            e.set_service(True, parked=True)
        c = e.host_placer(*job_runs(p.job_class))
        for _ in range(5):
            c()
        engines[label] = (e, c)
    res = {k: [] for k in list(engines) + ["cpu16"]}
    for r in range(rounds):
        for label, (e, c) in engines.items():
            print(f"round {r} {label}", file=sys.stderr, flush=True)
            c.recovery(2, (idle + 5) * 1e3, 1e3, rows[:2], vals[:2])
            out = c.recovery(trials, (idle + 5) * 1e3, 1e3, rows, vals)
            res[label].append(out)
        print(f"round {r} cpu16", file=sys.stderr, flush=True)
        fc = O.FastCPU(16)
        fc.prepare(p)
        fc.run()
        fc.recovery_loop(2, (idle + 5) * 1e3, 1e3, rows[:2], vals[:2])
        res["cpu16"].append(fc.recovery_loop(trials, (idle + 5) * 1e3, 1e3, rows, vals))
        fc.close()
    for label, outs in res.items():
        a = np.concatenate(outs)
        tot = a[:, 0] + a[:, 1]
        print(f"{label:10s} n={a.shape[0]}: total p50/p95/p99 {pct(tot)} | patch {pct(a[:, 0])} | place {pct(a[:, 1])}",
              flush=True)
    # every service stops before any engine is destroyed: an engine's frees
    # wait for every kernel on the device, another engine's parked service too
    for e, _ in engines.values():
        e.service_stop()
    for e, _ in engines.values():
        e.close()


if __name__ == "__main__":
    main()
