#!/usr/bin/env python3
"""Host walk of the split service (jsp_walk.cc) timed on the CPU alone: the
tiles' answer lines emulated from the oracle (tests/test_host_walk.py), then
HostWalk::place() on one set-up walker, repeated; mean ns per place and per
feasibility build. Runs anywhere (no GPU). Diagnostic only."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from jobset_amd import native, synth
    from jobset_amd.snapshot import job_runs
    from oracle import oracle as O
    import test_host_walk as T
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [3, 5]
    # WALK_LIB: another build of jsp_walk.cc with the same entry (A/B)
    lib = ctypes.CDLL(os.environ["WALK_LIB"]) if os.environ.get("WALK_LIB") else native.lib()
    f = lib.jspi_walk_bench
    f.restype = ctypes.c_int
    for cfg in cfgs:
        p = synth.CONFIGS[cfg]()
        a, cap, occ = O.place_c(p)
        slots, blocks, groups, cpg = T.emulate_tiles(p, cap, occ)
        topo = p.topology
        K = topo.n_levels
        D = np.array(topo.n_domains + [0] * (4 - K), dtype=np.uint32)
        fls = [np.ascontiguousarray(topo.first_leaf[k], dtype=np.uint32) for k in range(K)]
        flp = (ctypes.c_void_p * 4)(*([x.ctypes.data for x in fls] + [None] * (4 - K)))
        lv = np.array([c.level for c in p.classes], dtype=np.uint32)
        pods = np.array([c.pods for c in p.classes], dtype=np.uint32)
        b0 = np.array(blocks[0], dtype=np.uint32)
        b1 = np.array(blocks[1], dtype=np.uint32)
        rc, rl = job_runs(p.job_class)
        rc = np.ascontiguousarray(rc, dtype=np.uint32)
        rl = np.ascontiguousarray(rl, dtype=np.uint32)
        assign = np.full(max(p.n_jobs, 1), -7, dtype=np.int32)
        out = np.zeros(2, dtype=np.float64)
        vp = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        placed = f(ctypes.c_uint32(K), vp(D), flp, ctypes.c_uint32(len(p.classes)), vp(lv), vp(pods),
                   ctypes.c_uint32(len(b0)), vp(b0), vp(b1), ctypes.c_uint32(groups), ctypes.c_uint32(cpg), vp(slots),
                   vp(rc), vp(rl), ctypes.c_uint32(rc.shape[0]), vp(assign), ctypes.c_uint32(iters), vp(out))
        ok = np.array_equal(assign[:p.n_jobs], a)
        print(f"cfg{cfg}: K {K} D {list(topo.n_domains)} classes {len(p.classes)} runs {rc.shape[0]} jobs {p.n_jobs} "
              f"placed {placed} exact {ok} | place {out[0] / 1e3:.3f} us, feasibility build {out[1] / 1e3:.3f} us",
              flush=True)


if __name__ == "__main__":
    main()
