#!/usr/bin/env python3
"""Diagnostic (make diag): timeline of the assignment walk at a config —
kernel entry/staged/end (row 4000) and, per block of 64 runs of the
register-resident walker, stamps at runs 0, 16, 32, 48 and the block end
(rows 4010+). ns relative to the kernel's first stamp, median over launches.
Usage: stamps_walk.py cfg fused(0/1) reps"""
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
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    fused = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lib = native.lib()
    lib.jsp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    p = synth.CONFIGS[cfg]()
    eng = Engine(0)
    eng.load(p)
    eng.set_fused(bool(fused))
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    rows, clk = [], []
    for i in range(reps):
        lib.jsp_debug_clear()
        torch.cuda.synchronize()
        eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
        torch.cuda.synchronize()
        lib.jsp_debug_stamps(buf.ctypes.data, buf.shape[0])
        st = buf.reshape(4096, 8).astype(np.int64)
        rt = st[:4090]  # real-time stamps (row 4090 mixes in shader-clock values)
        nz = rt[rt != 0]
        t0 = nz.min() if nz.size else 0
        sel = np.concatenate([st[4000:4050], st[0:64]])  # walk rows, then tally tiles 0..63
        rows.append(np.where(sel != 0, (sel - t0) * 10, -1))
        r = st[4090]
        if r[0] and r[2]:
            clk.append((r[2] - r[0]) / ((r[3] - r[1]) * 10.0))  # shader cycles per ns = GHz
    med = np.median(np.stack(rows[3:]), axis=0)
    print(f"cfg{cfg} fused={fused} runs={rc.shape[0]}: ns from the launch's first stamp; "
          f"effective shader clock over the walk {np.median(clk) if clk else float('nan'):.2f} GHz")
    for r in range(50):
        if (med[r] >= 0).any():
            print(f"  row {4000 + r}: " + "  ".join(f"{x:8.0f}" for x in med[r]))
    print("  tally tiles (0 entry, 1 staged, 6 row pass, 7 leaf pass, 5 published):")
    for r in range(50, 114):
        if (med[r] >= 0).any():
            print(f"  tile {r - 50:4d}: " + "  ".join(f"{med[r][i]:8.0f}" for i in (0, 1, 6, 7, 5)))


if __name__ == "__main__":
    main()
