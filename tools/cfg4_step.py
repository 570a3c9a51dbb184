"""cfg4 device steps for a kernel trace (diagnostic): 50 device-path
placements (tally with folded feasibility -> level walk -> expand) and 50
sharded-harness steps (tally -> feasibility -> walk), bit-exact checked;
prints the dispatch-timed step medians."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402
from oracle import oracle as O  # noqa: E402

p = synth.config4()
e = Engine(0)
e.load(p)
a = O.place_c(p)[0]
rc, rl = job_runs(p.job_class)
rct = torch.from_numpy(rc.astype(np.int32)).cuda()
rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
med, mean = e.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 50)
e.check()
assert np.array_equal(out.cpu().numpy(), a)
print(f"device step: median {med:.2f} us mean {mean:.2f} us", flush=True)
L = p.topology.n_leaves
cap = torch.zeros((len(p.classes) + 1, L), dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(50):
    e.tally_device(cap.data_ptr(), cap[-1].data_ptr(), L, s)
    e.assign_device(cap.data_ptr(), cap[-1].data_ptr(), L, rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs,
                    out.data_ptr(), s)
torch.cuda.synchronize()
assert np.array_equal(out.cpu().numpy(), a)
print("harness steps bit-exact", flush=True)
