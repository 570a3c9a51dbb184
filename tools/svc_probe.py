#!/usr/bin/env python3
"""Where a resident-service placement's time goes: per host-API
call, the host wall time beside the service's 100 MHz device stamps (timing
on): request seen -> acquire -> tallied -> scanned -> looked back -> assign[]
drained, each phase taken at its slowest tile relative to the first tile that
saw the request. Diagnostic only."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (one HIP runtime)
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    eng = Engine(0)
    fl = eng.link_floor(2000)
    print(f"host-link floor (jspb_link_floor): p50 {fl[0]:.2f} us p99 {fl[1]:.2f}", flush=True)
    cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2]
    for cfg in cfgs:
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        call = eng.host_placer(*job_runs(p.job_class))
        for timed, patched in ((False, False), (True, False), (False, True), (True, True)):
            eng.set_timing(timed)
            for _ in range(100):
                call()
            walls, phases, hops = [], [], []
            for r in range(reps):
                if patched:  # one row rewritten with its own values: the tiles reload their rows
                    row = np.array([(r * 7919) % p.nodes.n_nodes], dtype=np.uint32)
                    eng.patch_rows(row, taints=p.nodes.taints[row])
                eng.timing(reset=True)
                t0 = time.perf_counter()
                call()
                walls.append((time.perf_counter() - t0) * 1e6)
                tm = eng.timing(reset=True)
                if timed:
                    c, d = eng.service_clock_rows()
                    c, d = c.astype(np.int64), d.astype(np.int64)
                    ref = c[:, 0].min()
                    # the dispatcher's row: request seen in the mailbox, bell rung (relative to the first tile)
                    ds = (d[0] - ref) * 10 if d[0] else 0
                    dr = (d[1] - ref) * 10 if d[1] else 0
                    phases.append([ds, dr] + [(c[:, k].max() - ref) * 10 for k in (0, 1, 6, 7, 2, 3, 4, 5)])
                    if d[0] and tm.svc_first_us > 0:
                        # host: post -> first / last answer entry; device: the
                        # dispatcher saw the request -> tile 0 / the last tile
                        # drained. The difference is the two host-link hops.
                        dev_first = (int(c[0, 5]) - int(d[0])) * 1e-2
                        dev_last = (int(c[:, 5].max()) - int(d[0])) * 1e-2
                        hops.append([tm.svc_first_us, tm.svc_answer_us, dev_first, dev_last,
                                     tm.svc_first_us - dev_first, tm.svc_answer_us - dev_last])
            w = np.array(walls)
            line = f"cfg{cfg} timing={'on ' if timed else 'off'} patched={int(patched)}: wall p50 {np.median(w):.2f} us p99 {np.percentile(w, 99):.2f}"
            if timed:
                ph = np.median(np.array(phases), axis=0)
                line += " | device (ns from first tile seeing the request, slowest tile): " + " ".join(
                    f"{n} {v:.0f}" for n, v in zip(("disp_seen", "disp_rung", "seen", "bcast", "rowpass", "leafpass",
                                                     "tally", "scan", "lookback", "drained"), ph))
            print(line, flush=True)
            if hops:
                h = np.median(np.array(hops), axis=0)
                print(f"    host post->first entry {h[0]:.2f} us, ->last {h[1]:.2f} | device seen->tile0 drained {h[2]:.2f}, "
                      f"->last drained {h[3]:.2f} | hops (host - device): first {h[4]:.2f}, last {h[5]:.2f} us "
                      f"(floor {fl[0]:.2f})", flush=True)
        eng.set_timing(False)
    eng.close()


if __name__ == "__main__":
    main()
