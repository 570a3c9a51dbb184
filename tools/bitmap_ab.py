"""Compaction service answer forms, interleaved A/B in one process
(diagnostic): tile bitmaps expanded on the host (default) vs per-job entries
after the tiles' look-back (test hook svc_entries=1). Host-API calls timed in
C (jspb_place_loop); the host's post -> first / last answer split from
jsp_timing (svc_first_us / svc_answer_us)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402
from oracle import oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
iters = 2000
for cfg in (2, 1):
    p = synth.CONFIGS[cfg]()
    ref = O.place_c(p)[0]
    res = {"bitmap": [], "entries": []}
    for r in range(reps):
        for form in ("bitmap", "entries"):
            os.environ["JSP_TEST_HOOKS"] = "svc_entries=1" if form == "entries" else ""
            e = Engine(0)
            e.load(p)
            call = e.host_placer(*job_runs(p.job_class))
            for _ in range(50):
                call()
            e.timing(reset=True)
            tot, p50, p99 = call.loop(iters)
            t = e.timing(reset=True)
            assert np.array_equal(call.assign, ref), form
            n = max(int(t.svc_calls), 1)
            res[form].append((p50, p99, t.svc_first_us / n, t.svc_answer_us / n, tot / iters))
            e.close()
    os.environ.pop("JSP_TEST_HOOKS", None)
    for form, v in res.items():
        a = np.array(v)
        print(f"cfg{cfg} {form:8s}: per call p50 {np.median(a[:, 0]):.2f} us p99 {np.median(a[:, 1]):.2f} mean "
              f"{np.median(a[:, 4]):.2f} | post->first {np.median(a[:, 2]):.2f} ->last {np.median(a[:, 3]):.2f} "
              f"(runs: {' '.join(f'{x:.2f}' for x in a[:, 0])})", flush=True)
