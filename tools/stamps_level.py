#!/usr/bin/env python3
"""Diagnostic (tools/bin/diag stamp build): phase timeline of
assign_level_kernel on cfg4 through the device path: entry, staged, after
runs 1..5, end -- ns relative to entry, median over launches."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("JSP_LIB_PATH", os.path.join(ROOT, "tools", "bin", "diag", "libjsplace.so"))


def main():
    import torch
    from jobset_amd import native, synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = native.lib()
    lib.jsp_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    p = synth.config4()
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
        eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
        torch.cuda.synchronize()
        lib.jsp_debug_stamps(buf.ctypes.data, buf.shape[0])
        b = buf.reshape(4096, 8)
        st = b[4050].astype(np.int64)
        sub = b[4051].astype(np.int64)
        rows.append(np.concatenate([(st - st[0]) * 10, (sub - st[0]) * 10]))
    med = np.median(np.stack(rows[3:]), axis=0)
    print("assign_level_kernel cfg4 (ns from entry): staged {:.0f} | runs {} | end {:.0f}".format(
        med[1], " ".join(f"{x:.0f}" for x in med[2:6]), med[7]), flush=True)
    print("  per run: scan done {} | records issued {}".format(
        " ".join(f"{x:.0f}" for x in med[8:12]), " ".join(f"{x:.0f}" for x in med[12:16])), flush=True)


if __name__ == "__main__":
    main()
