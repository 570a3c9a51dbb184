#!/usr/bin/env python3
"""Diagnostic (make diag): phase timeline of assign_kernel at a config in the
three-launch shape: stamps at entry, after staging, after each run (up to
5), end — ns relative to entry, median over launches."""
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
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = native.lib()
    lib.jsp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    p = synth.CONFIGS[cfg]()
    eng = Engine(0)
    eng.load(p)
    eng.set_fused(False)
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    rows = []
    for i in range(reps):
        lib.jsp_debug_clear()
        torch.cuda.synchronize()
        for _ in range(3):
            eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
        torch.cuda.synchronize()
        lib.jsp_debug_stamps(buf.ctypes.data, buf.shape[0])
        st = buf.reshape(4096, 8)[4000:4009].astype(np.int64)
        rows.append((st - st[0, 0]) * 10)
    med = np.median(np.stack(rows[3:]), axis=0)
    print(f"cfg{cfg} assign_kernel ({rc.shape[0]} runs): [entry, staged, .., end]; then per long run of class c<8: "
          f"start, scanned, window published, walked, copied out (last step), end (ns)")
    print("  kernel: " + "  ".join(f"{x:8.0f}" for x in med[0]))
    for t in range(8):
        if buf.reshape(4096, 8)[4001 + t, 0] != 0:
            print(f"  class {t}: " + "  ".join(f"{x:8.0f}" for x in med[1 + t][:6]))


if __name__ == "__main__":
    main()
