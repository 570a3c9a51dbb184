#!/usr/bin/env python3
"""Per-kernel time breakdown of every config in both launch shapes (HIP
events from the engine's own timing hooks), for finding which kernel of a
placement to work on next. Usage: breakdown.py [cfg ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    cfgs = [int(x) for x in sys.argv[1:]] or [1, 2, 3, 4, 5]
    eng = Engine(0)
    for cfg in cfgs:
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        rc, rl = job_runs(p.job_class)
        rct = torch.from_numpy(rc.astype(np.int32)).cuda()
        rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
        out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
        for fused in (True, False):
            eng.set_fused(fused)
            for _ in range(5):
                eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
            torch.cuda.synchronize()
            eng.set_timing(True)
            n = 30
            for _ in range(n):
                eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
            torch.cuda.synchronize()
            t = eng.timing(reset=True)
            eng.set_timing(False)
            k = max(t.calls, 1)
            print(f"cfg{cfg} fused={int(fused)} runs={rc.shape[0]} jobs={p.n_jobs} "
                  f"placed={int((out[:p.n_jobs].cpu().numpy() >= 0).sum())}: "
                  f"single={t.fused_ms * 1e3 / k:.2f} tally={t.tally_ms * 1e3 / k:.2f} "
                  f"feas={t.feas_ms * 1e3 / k:.2f} assign={t.assign_ms * 1e3 / k:.2f} us/placement", flush=True)
        eng.set_fused(True)


if __name__ == "__main__":
    main()
