"""Row-pass stamps of the resident compaction service (diagnostic; A/B build
tools/bin/ab_fine, -DJSP_AB_FINESTAMP): per request, tile 0's slots
seen(0) bcast(1) chunk-loop start(2) class record read(3) first scan(4) row
pass barrier(6) leaf pass barrier(7) drained(5), us from seen; medians."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

e = Engine(0)
for cfg in (1, 2):
    p = synth.CONFIGS[cfg]()
    e.load(p)
    e.set_timing(True)
    call = e.host_placer(*job_runs(p.job_class))
    rows = []
    for i in range(400):
        call()
        c = e.service_clock().astype(np.int64)
        if i >= 20:
            rows.append(c[0] - c[0, 0])
    m = np.median(np.array(rows), axis=0) * 0.01
    print(f"cfg{cfg} tile0: " + " ".join(f"{n} {m[k]:.2f}" for n, k in (("bcast", 1), ("loop", 2), ("class", 3),
                                                                     ("scan0", 4), ("rowpass", 6), ("leafpass", 7),
                                                                     ("drained", 5))), flush=True)
    e.set_timing(False)
    e.service_stop()
