#!/usr/bin/env python3
"""Phase timeline of the single-launch compaction kernel from the diagnostic
build (make diag): per workgroup, 100 MHz s_memrealtime stamps at
0 entry, 1 first barrier (row loads + LDS staging), 2 tally done,
3 feasible-count scan, 4 look-back done, 5 end; inside the tally 6 row pass
done, 7 leaf pass done. Prints the median over
launches of each phase's start relative to the launch's first stamp (ns)."""
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
    from jobset_amd.snapshot import job_runs
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    b2b = int(sys.argv[3]) if len(sys.argv) > 3 else 1  # launches per sample: >1 = back-to-back (GPU busy)
    lib = native.lib()
    lib.jsp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    p = synth.CONFIGS[cfg]()
    eng = Engine(0)
    eng.load(p)
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    rows = []
    for i in range(reps):
        lib.jsp_debug_clear()
        torch.cuda.synchronize()
        for _ in range(b2b):  # the stamps keep the last launch's times
            eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
        torch.cuda.synchronize()
        lib.jsp_debug_stamps(buf.ctypes.data, buf.shape[0])
        st = buf.reshape(4096, 8)
        used = st[:, 0] != 0
        st = st[used].astype(np.int64)
        t0 = st[:, 0].min()
        rows.append(((st[:, :8] - t0) * 10))  # ns
    arr = np.stack(rows[5:])  # [reps, blocks, 6]
    med = np.median(arr, axis=0)
    print(f"cfg{cfg} ({b2b} back-to-back launches per sample): {med.shape[0]} workgroups; phase start (ns, median over {arr.shape[0]} launches)")
    cols = [0, 1, 6, 7, 2, 3, 4, 5]
    print("phase:          entry  barrier1  rowpass  leafpass  tallied  scanned  lookback  end")
    for b in range(min(med.shape[0], 24)):
        print(f"  wg {b:4d}: " + "  ".join(f"{med[b][c]:8.0f}" for c in cols))
    print("  max     : " + "  ".join(f"{med.max(axis=0)[c]:8.0f}" for c in cols))
    for q in (10, 50, 90):
        print(f"  p{q:<2d} wgs : " + "  ".join(f"{np.percentile(med[:, c], q):8.0f}" for c in cols))
    late = np.nonzero(med[:, 0] > 2000)[0]
    print(f"  {late.size} workgroups enter > 2 us after the first: {late[:40].tolist()}")
    if late.size:
        print(f"  their entry (ns): {med[late[:40], 0].astype(int).tolist()}")
    # per-workgroup phase durations (tally launch: entry -> barrier1 -> rowpass -> leafpass -> end)
    d = lambda a, b: np.median(med[:, b] - med[:, a])
    print(f"  median wg durations (ns): to-barrier1 {d(0, 1):.0f}  rowpass {d(1, 6):.0f}  "
          f"leafpass {d(6, 7):.0f}  write-out {d(7, 5):.0f}  total {d(0, 5):.0f}")


if __name__ == "__main__":
    main()
