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
        if cfg == 2:
            # raw per-trial (patch, place) at gap 1 ms: default service, parked,
            # and the gap spun instead of slept (a caller whose core stays awake)
            out_dir = os.environ.get("PHASE_OUT", ".")
            for label, parked, spin in (("default", False, False), ("default_condvar_waker", False, False),
                                        ("parked", True, False)):
                if label == "default_condvar_waker":  # A/B: the waker on its condition variable only
                    os.environ["JSP_TEST_HOOKS"] = "waker_poll_us=0"
                    e2 = Engine(0)
                    del os.environ["JSP_TEST_HOOKS"]
                    e2.load(p)
                    c2 = e2.host_placer(*job_runs(p.job_class))
                    for _ in range(5):
                        c2()
                    rows = np.array([(i * 7919) % p.nodes.n_nodes for i in range(300)], dtype=np.uint32)
                    vals = np.ascontiguousarray(p.nodes.taints[rows], dtype=np.uint32)
                    res = c2.recovery(300, (idle + 5) * 1e3, 1e3, rows, vals)
                    e2.service_stop()
                    e2.close()
                    tot = res[:, 0] + res[:, 1]
                    q = lambda a, x: np.percentile(a, x)  # noqa: E731
                    print(f"cfg2 cold gap 1 ms {label}: total p50/p95/p99 {q(tot, 50):.2f}/{q(tot, 95):.2f}/"
                          f"{q(tot, 99):.2f} | patch {q(res[:, 0], 50):.2f}/{q(res[:, 0], 95):.2f}/"
                          f"{q(res[:, 0], 99):.2f} | place {q(res[:, 1], 50):.2f}/{q(res[:, 1], 95):.2f}/"
                          f"{q(res[:, 1], 99):.2f}", flush=True)
                    np.savetxt(os.path.join(out_dir, f"cold_cfg2_{label}.csv"), res, delimiter=",", fmt="%.3f",
                               header="patch_us,place_us,gap_us")
                    continue
                if parked:
                    eng.set_service(True, parked=True)
                    call()
                    call()
                rows = np.array([(i * 7919) % p.nodes.n_nodes for i in range(300)], dtype=np.uint32)
                vals = np.ascontiguousarray(p.nodes.taints[rows], dtype=np.uint32)
                res = call.recovery(300, (idle + 5) * 1e3, 1e3, rows, vals, spin=spin)
                np.savetxt(os.path.join(out_dir, f"cold_cfg2_{label}.csv"), res, delimiter=",", fmt="%.3f",
                           header="patch_us,place_us,gap_us")
                tot = res[:, 0] + res[:, 1]
                q = lambda a, x: np.percentile(a, x)  # noqa: E731
                print(f"cfg2 cold gap 1 ms {label}: total p50/p95/p99 {q(tot, 50):.2f}/{q(tot, 95):.2f}/"
                      f"{q(tot, 99):.2f} | patch {q(res[:, 0], 50):.2f}/{q(res[:, 0], 95):.2f}/{q(res[:, 0], 99):.2f}"
                      f" | place {q(res[:, 1], 50):.2f}/{q(res[:, 1], 95):.2f}/{q(res[:, 1], 99):.2f}", flush=True)
                if parked:
                    eng.service_stop()
                    eng.set_service(True)
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
    # the same device step with assign[] in pinned host memory (what the host API writes)
    pin = torch.empty(p4.n_jobs, dtype=torch.int32, pin_memory=True)
    pmed, _ = eng.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p4.n_jobs, pin.data_ptr(), 50)
    print(f"cfg4 device step with assign[] in pinned host memory: {pmed:.2f} us", flush=True)
    # device paths of the multi-level shapes (cfg3, cfg5): host walk after the GPU feasibility
    s = torch.cuda.current_stream().cuda_stream
    for cfg in (3, 5):
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        eng.set_service(False)
        shape = eng.place(p.job_class).fused
        eng.set_service(True)
        rc, rl = job_runs(p.job_class)
        rct = torch.from_numpy(rc.astype(np.int32)).cuda()
        rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
        out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
        for _ in range(20):
            eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), s)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), s)
        b.record()
        b.synchronize()
        loop = a.elapsed_time(b) * 1e3 / 200
        dmed, _ = eng.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 100)
        eng.set_fused(False)
        fmed, _ = eng.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 100)
        eng.set_fused(True)
        eng.timing(reset=True)
        for _ in range(100):
            eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), s)
        eng.check()
        t = eng.timing(reset=True)
        n = max(t.calls, 1)
        o = max(t.oneshot_calls, 1)
        print(f"cfg{cfg} device path (shape {shape}): event loop {loop:.2f} us/step, dispatch-timed {dmed:.2f} | "
              f"GPU walk (three launches) {fmed:.2f} | events per call: tally {t.tally_ms * 1e3 / n:.2f} "
              f"feas {t.feas_ms * 1e3 / n:.2f} walk+copy {t.assign_ms * 1e3 / n:.2f} | split launch host phases: "
              f"launch {t.oneshot_launch_us / o:.2f} (stage {t.oneshot_stage_us / o:.2f}) wait "
              f"{t.oneshot_wait_us / o:.2f} walk+copy {t.oneshot_walk_us / o:.2f} (calls {t.oneshot_calls})",
              flush=True)


if __name__ == "__main__":
    main()
