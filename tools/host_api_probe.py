#!/usr/bin/env python3
"""Host-API latency of jsp_place on configs 1, 2, 3, 5 (same resident
snapshot, repeated pre-bound calls), split into the library's host phases
(jsp_timing.host_*), next to the device-resident step. Diagnostic only."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    torch.cuda.init()
    eng = Engine(0)
    for cfg, fused in ((1, True), (2, True), (3, True), (5, True), (5, False), (3, False)):
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        eng.set_fused(fused)
        call = eng.host_placer(*job_runs(p.job_class))
        for _ in range(50):
            call()
        eng.timing(reset=True)
        wall = []
        for _ in range(1000):
            t0 = time.perf_counter()
            call()
            wall.append((time.perf_counter() - t0) * 1e6)
        t = eng.timing(reset=True)
        n = max(t.host_calls, 1)
        wall.sort()
        rc, rl = job_runs(p.job_class)
        rct = torch.from_numpy(rc.astype(np.int32)).cuda()
        rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
        out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        dev = []
        for i in range(300):
            t0 = time.perf_counter()
            eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), s)
            torch.cuda.synchronize()
            if i >= 20:
                dev.append((time.perf_counter() - t0) * 1e6)
        dev.sort()
        eng.set_fused(True)
        print(f"cfg{cfg}{'' if fused else ' (three launches)'}: host API p50 {wall[500]:.1f} us p99 {wall[990]:.1f} | lib phases (mean us): prep "
              f"{t.host_prep_us / n:.2f} launch {t.host_launch_us / n:.2f} wait {t.host_wait_us / n:.2f} post "
              f"{t.host_post_us / n:.2f} | device path + stream sync p50 {dev[len(dev) // 2]:.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
