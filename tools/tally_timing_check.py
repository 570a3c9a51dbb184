"""The cfg4 tally's device time two ways in one process (diagnostic, DESIGN.md
§9): events on the dispatch packets of K back-to-back launches inside the
library (jspb_tally_device_timed, what bench.py reports) -- run it under
rocprofv3 --kernel-trace --stats and compare with the trace's own durations
of the same launches. Also the folded-feasibility step's tally (the host API
and jsp_place_device path) for its grid size."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 400
e = Engine(0)
p = synth.config4()
e.load(p)
C, L = len(p.classes), p.topology.n_leaves
cap = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
for _ in range(3):
    med, mean = e.tally_device_timed(cap.data_ptr(), cap[-1].data_ptr(), L, iters)
    print(f"tally (jsp_tally_device): dispatch events median {med:.3f} us mean {mean:.3f} us over {iters}", flush=True)
rc, rl = job_runs(p.job_class)
rct = torch.from_numpy(rc.astype(np.int32)).cuda()
rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
a = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
med, mean = e.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, a.data_ptr(), iters // 4)
print(f"step (jsp_place_device, folded tally): dispatch events median {med:.3f} us mean {mean:.3f} us", flush=True)
e.close()
