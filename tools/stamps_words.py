#!/usr/bin/env python3
"""Diagnostic (make diag): per-word cost of the register walker's first four
batches at a config -- shader cycles from word start to the end of the job
chain and to the end of the word, jobs visited and domains taken. Rows
4020 + 4*batch + word of the stamp buffer (s_memtime cycles), medians over
launches. Usage: stamps_words.py cfg fused reps"""
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
    cfg, fused, reps = (int(x) for x in (sys.argv[1:4] + ["5", "1", "20"][len(sys.argv) - 1:]))
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
    rows = []
    for _ in range(reps):
        lib.jsp_debug_clear()
        torch.cuda.synchronize()
        eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
        torch.cuda.synchronize()
        lib.jsp_debug_stamps(buf.ctypes.data, buf.shape[0])
        rows.append(buf.reshape(4096, 8)[4020:4036].astype(np.int64).copy())
    a = np.stack(rows[3:])
    print(f"cfg{cfg} fused={fused}: per word of batches 1-4 (last tile): cycles chain / word, visits, taken")
    for r in range(16):
        x = a[:, r]
        if (x[:, 0] == 0).all():
            continue
        chain = np.median(x[:, 1] - x[:, 0])
        word = np.median(x[:, 2] - x[:, 0])
        print(f"  batch {r // 4 + 1} word {r % 4}: chain {chain:7.0f}  word {word:7.0f}  visits {int(np.median(x[:, 3])):3d}"
              f"  taken {int(np.median(x[:, 4])):3d}  cycles/visit {chain / max(1, np.median(x[:, 3])):6.1f}")


if __name__ == "__main__":
    main()
