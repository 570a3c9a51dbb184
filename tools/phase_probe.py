#!/usr/bin/env python3
"""Where the host-API time goes (diagnostic): the library's phase clocks
(jspb_get_timing) per call, warm (back-to-back calls) and cold (the
recovery loop: sleep past the idle exit, one-row patch, gap, place), on
configs 2, 3, 5; and cfg4's host-API step split into prep / launch / wait /
post beside its device step. Run with JSP_SERVICE_IDLE_MS=30."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FIELDS = ("host_prep_us", "host_launch_us", "host_wait_us", "host_post_us", "svc_pre_us", "svc_answer_us",
          "svc_first_us", "svc_ready_us", "patch_us", "wake_us")


def per_call(t, n):
    return " ".join(f"{f[:-3]}={getattr(t, f) / max(n, 1):.2f}" for f in FIELDS) + \
        f" svc_calls={t.svc_calls} starts={t.svc_starts} fallbacks={t.svc_fallbacks}"


def main():
    import torch
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    torch.cuda.init()
    idle = float(os.environ.get("JSP_SERVICE_IDLE_MS", "50"))
    eng = Engine(0)
    for cfg in (2, 3, 5):
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        call = eng.host_placer(*job_runs(p.job_class))
        for _ in range(50):
            call()
        eng.timing(reset=True)
        tot, med, p99 = call.loop(500)
        t = eng.timing(reset=True)
        print(f"cfg{cfg} warm: p50 {med:.2f} p99 {p99:.2f} | {per_call(t, t.host_calls)}", flush=True)
        for gap in (0.0, 1.0, 10.0):
            rows = np.array([(i * 7919) % p.nodes.n_nodes for i in range(40)], dtype=np.uint32)
            vals = np.ascontiguousarray(p.nodes.taints[rows], dtype=np.uint32)
            eng.timing(reset=True)
            res = call.recovery(40, (idle + 5) * 1e3, gap * 1e3, rows, vals)
            t = eng.timing(reset=True)
            pa, pl = np.median(res[:, 0]), np.median(res[:, 1])
            print(f"cfg{cfg} cold gap {gap:g} ms: patch p50 {pa:.2f} place p50 {pl:.2f} "
                  f"(p90 {np.percentile(res[:, 1], 90):.2f}) | {per_call(t, t.host_calls)}", flush=True)
        eng.service_stop()
    p4 = synth.config4()
    eng.load(p4)
    call = eng.host_placer(*job_runs(p4.job_class))
    for _ in range(5):
        call()
    eng.timing(reset=True)
    tot, med, _ = call.loop(50)
    t = eng.timing(reset=True)
    rc, rl = job_runs(p4.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(p4.n_jobs, dtype=torch.int32, device="cuda")
    dmed, _ = eng.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p4.n_jobs, out.data_ptr(), 50)
    print(f"cfg4 host API: mean {tot / 50:.2f} p50 {med:.2f} | device step {dmed:.2f} | {per_call(t, t.host_calls)}",
          flush=True)


if __name__ == "__main__":
    main()
