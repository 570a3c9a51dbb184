"""Effective shader clock of the resident service's request (diagnostic, A/B
build tools/bin/ab_clk with -DJSP_AB_CLKFREQ: stamp slots 6/7 carry s_memtime
at slots 1/2). Prints per-phase medians (us) and the clock (MHz)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

ab = os.environ.get("JSP_LIB_PATH", "")
e = Engine(0)
for cfg in (1, 2):
    p = synth.CONFIGS[cfg]()
    e.load(p)
    e.set_timing(True)
    call = e.host_placer(*job_runs(p.job_class))
    for gap, xcd, res in ((0.0, "1", "1"), (0.0, "1", "0"), (0.0, "0", "1"), (0.0, "0", "0"), (0.001, "1", "1")):
        os.environ["JSP_SVC_XCD"] = xcd  # read at the service's start
        os.environ["JSP_SVC_RESIDENT"] = res
        e.service_stop()
        rows = []
        for i in range(300):
            if gap:
                time.sleep(gap)
            call()
            c = e.service_clock().astype(np.int64)
            if i >= 20:
                rows.append(c)
        ph = []
        fq = []
        for c in rows:
            ref = c[:, 0].min()
            ph.append([(c[:, k].max() - ref) * 0.01 for k in (1, 2, 3, 4, 5)])
            if "ab_clk" in ab:
                dm = (c[:, 7] - c[:, 6]) & 0xFFFFFFFF
                dr = (c[:, 2] - c[:, 1]) * 0.01
                fq.append(float(np.median(dm / np.maximum(dr, 1e-3))))
        m = np.median(np.array(ph), axis=0)
        walls = []
        for i in range(300):
            t0 = time.perf_counter()
            e.set_timing(False) if i == 0 else None
            call()
            walls.append((time.perf_counter() - t0) * 1e6)
        e.set_timing(True)
        line = f"cfg{cfg} xcd={xcd} resident={res} gap {gap * 1e3:g} ms: wall(timing off) p50 {np.median(walls[20:]):.2f} us | bcast {m[0]:.2f} tallied {m[1]:.2f} scanned {m[2]:.2f} lookback {m[3]:.2f} drained {m[4]:.2f} us"
        if fq:
            line += f" | row+leaf pass clock {np.median(fq):.0f} MHz"
        print(line, flush=True)
    e.set_timing(False)
    e.service_stop()
