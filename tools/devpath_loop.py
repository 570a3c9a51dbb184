#!/usr/bin/env python3
"""Device path and host API of the multi-level shapes (diagnostic): per
config, jsp_place_device dispatch-timed (jspb_place_device_timed) and by an
event loop of back-to-back calls on the caller's stream, and the host API's
per-call p50 through the resident service (C loop), `reps` times each.
Usage: devpath_loop.py [cfgs] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    cfgs = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [5, 3]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    torch.cuda.init()
    s = torch.cuda.current_stream().cuda_stream
    eng = Engine(0)
    for cfg in cfgs:
        p = synth.CONFIGS[cfg]()
        rc, rl = job_runs(p.job_class)
        rct = torch.from_numpy(rc.astype(np.int32)).cuda()
        rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
        out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
        eng.load(p)
        for rep in range(reps):
            eng.set_service(False)
            shape = eng.place(p.job_class).fused
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
            dmed, _ = eng.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 200)
            eng.set_service(True)
            call = eng.host_placer(rc, rl)
            for _ in range(50):
                call()
            _, hmed, _ = call.loop(500)
            eng.service_stop()
            print(f"cfg{cfg} rep{rep}: device path shape {shape} dispatch-timed {dmed:.2f} us, event loop {loop:.2f} us"
                  f" | host API (service) p50 {hmed:.2f} us", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
