#!/usr/bin/env python3
"""Profiling driver: run one config's placement `--steps` times on cuda:0
(device-resident runs API), for rocprofv3 kernel traces / PMC passes."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--fused", type=int, default=1)
    args = ap.parse_args()
    import torch
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    p = synth.CONFIGS[args.cfg]()
    eng = Engine(0)
    eng.load(p)
    eng.set_fused(bool(args.fused))
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
    for _ in range(args.steps):
        eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 0)
    torch.cuda.synchronize()
    print(f"cfg{args.cfg}: placed {int((out.cpu().numpy() >= 0).sum())}/{p.n_jobs}")


if __name__ == "__main__":
    main()
