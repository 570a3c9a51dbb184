"""Device path (jsp_place_device: runs and assign[] device-resident) per
config, the fused one-launch shape against the three-launch step (tally ->
feasibility -> walk), bit-exact against the oracle (diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402
from oracle import oracle as O  # noqa: E402

e = Engine(0)
e.set_service(False)
for cfg in (3, 5, 2):
    p = synth.CONFIGS[cfg]()
    e.load(p)
    ref = O.place_c(p)[0]
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
    for fused in (True, False):
        e.set_fused(fused)
        e.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 10)
        med, mean = e.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 200)
        e.check()
        ok = np.array_equal(out[:p.n_jobs].cpu().numpy(), ref)
        print(f"cfg{cfg} fused={int(fused)} shape={e.place(p.job_class).fused}: device step median {med:.2f} us "
              f"mean {mean:.2f} us exact={ok}", flush=True)
    e.set_fused(True)
e.close()
