#!/usr/bin/env python3
"""Per-wave timeline of the wave-tile tally (cfg4, 1M rows) from the
diagnostic build (make diag): 100 MHz s_memrealtime stamps per wave at
0 entry, 1 class staging + tile descriptors ready (after the barrier),
2 first tile evaluated (its rows arrived), 3 last tile's stores issued.
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
            st = buf.reshape(4096, 8)[:, :4].astype(np.int64)
            st = st[st[:, 0] != 0]
            t0 = st[:, 0].min()
            rel = (st - t0) * 10
            res.append([np.percentile(rel[:, k], q) for k in range(4) for q in (0, 50, 90, 100)])
        m = np.median(np.array(res), axis=0).reshape(4, 4)
        print(f"{mode}: waves {st.shape[0]}")
        for k, name in enumerate(("entry", "staged", "first tile", "end")):
            print(f"  {name:10s} min {m[k,0]:7.0f}  p50 {m[k,1]:7.0f}  p90 {m[k,2]:7.0f}  max {m[k,3]:7.0f} ns")


if __name__ == "__main__":
    main()
