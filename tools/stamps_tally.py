#!/usr/bin/env python3
"""Per-wave timeline of the wave-tile tally (cfg4, 1M rows) from the
diagnostic build (make diag): 100 MHz s_memrealtime stamps per wave at
0 entry, 1 class staging + tile descriptors ready (after the barrier),
2 first tile evaluated (its rows arrived), 3 the second tile's rows drained
(waits for every load in flight), 4 second tile evaluated (so 4 - 3 is one
tile's evaluation alone), 5 last tile's stores issued. Two tiles per wave
need JSP_TALLY_WPS <= 2 (the default).
Warm (back-to-back launches) and cold (512 MiB read-only scrub before the
launch). Prints percentiles over waves of each stamp relative to the
launch's first entry stamp (ns), medians over repetitions."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("JSP_LIB_PATH", os.path.join(ROOT, "tools", "diag", "libjsplace.so"))
os.environ.setdefault("JSP_TALLY_WPS", "2")  # two tiles per wave (stamps 3 and 4 need a second tile),
os.environ.setdefault("JSP_TALLY_ONE", "0")  # on the double-buffered kernel (the one-tile kernel has no stamps)


def main():
    import torch
    from jobset_amd import native, synth
    from jobset_amd.engine import Engine
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = native.lib()
    lib.jsp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    p = synth.config4()
    eng = Engine(0)
    eng.load(p)
    C, L = len(p.classes), p.topology.n_leaves
    cap = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    fn = lambda: eng.tally_device(cap.data_ptr(), cap[-1].data_ptr(), L, stream)  # noqa: E731
    scrub = torch.zeros(128 << 20, dtype=torch.int32, device="cuda")
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    for mode in ("warm", "cold"):
        res = []
        for _ in range(reps):
            lib.jsp_debug_clear()
            torch.cuda.synchronize()
            if mode == "warm":
                for _ in range(3):
                    fn()
            else:
                scrub.sum()
                fn()
            torch.cuda.synchronize()
            lib.jsp_debug_stamps(buf.ctypes.data, buf.shape[0])
            full = buf.reshape(4096, 8).astype(np.int64)
            full = full[(full[:, 0] != 0) & (full[:, 4] != 0)]
            st = full[:, :6]
            t0 = st[:, 0].min()
            rel = (st - t0) * 10
            ev = (st[:, 4] - st[:, 3]) * 10
            mhz = (full[:, 7] - full[:, 6]) / np.maximum(st[:, 4] - st[:, 3], 1) * 100.0  # shader clock, MHz
            res.append([np.percentile(rel[:, k], q) for k in range(6) for q in (0, 50, 90, 100)] +
                       [np.percentile(ev, q) for q in (0, 50, 90, 100)] +
                       [np.percentile(mhz, q) for q in (0, 50, 90, 100)])
        m = np.median(np.array(res), axis=0).reshape(8, 4)
        print(f"{mode}: waves with two tiles {st.shape[0]}")
        for k, name in enumerate(("entry", "staged", "tile 1 done", "tile 2 rows", "tile 2 done", "end",
                                  "tile 2 eval", "clock MHz")):
            print(f"  {name:12s} min {m[k,0]:7.0f}  p50 {m[k,1]:7.0f}  p90 {m[k,2]:7.0f}  max {m[k,3]:7.0f}"
                  f"{' ns' if k < 7 else ''}")


if __name__ == "__main__":
    main()
