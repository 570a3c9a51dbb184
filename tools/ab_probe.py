#!/usr/bin/env python3
"""A/B probes on cuda:0 (diagnostic only, not the bench). Each variant runs in
its own child process because the engine reads its tuning variables once.

  python tools/ab_probe.py tally     cfg4 tally: block kernel vs wave-tile kernel
                                     (waves per SIMD 1/2/3/4), warm (200 back-to-back
                                     launches, HIP events) and cold (512 MiB scrub
                                     before each of 20 launches), bit-exact vs oracle
  python tools/ab_probe.py mark      device path (jsp_place_device) per-call host and
                                     GPU time with each caller-stream marker
  python tools/ab_probe.py step      cfg4 three-launch step (place_device) GPU time
                                     per call with 1/4/16/64 records per expand wave, or staged stores
  python tools/ab_probe.py one KEY   one variant (the child side)
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

AB = os.path.join(ROOT, "tools", "ablib")  # A/B builds (make tools/ablib/<name>/libjsplace.so)
TALLY = {"one": {}, "wave2": {"JSP_TALLY_ONE": "0", "JSP_TALLY_WPS": "2"},
         "wave4": {"JSP_TALLY_ONE": "0", "JSP_TALLY_WPS": "4"}, "block": {"JSP_TALLY_BLOCK": "1"},
         "one_b": {}, "wave4_b": {"JSP_TALLY_ONE": "0", "JSP_TALLY_WPS": "4"},
         # diagnostic build: descriptors from the tile index (wrong sums, exact false): the cost of the dependent load
         "fakedesc": {"JSP_LIB_PATH": os.path.join(AB, "fakedesc", "libjsplace.so")}, "one_c": {},
         "fakedesc_b": {"JSP_LIB_PATH": os.path.join(AB, "fakedesc", "libjsplace.so")}}
# a variant can also load another build of the library: {"JSP_LIB_PATH": os.path.join(AB, name, "libjsplace.so")}
# (make tools/ablib/<name>/libjsplace.so with AB_FLAGS_<name> in the Makefile)
SVC = {"svc_default": {}, "svc_split_compact": {"JSP_SPLIT_COMPACT": "1"},
       "svc_rows508": {"JSP_BLOCK_ROWS": "508"}, "svc_rows252": {"JSP_BLOCK_ROWS": "252"},
       "svc_split_rows252": {"JSP_SPLIT_COMPACT": "1", "JSP_BLOCK_ROWS": "252"},
       "svc_cold_launch": {"JSP_COLD_LAUNCH": "1"}}
SVC2 = {"svc_default_1": {}, "svc_no_row_cache_1": {"JSP_SVC_ROW_CACHE": "0"},
        "svc_default_2": {}, "svc_no_row_cache_2": {"JSP_SVC_ROW_CACHE": "0"},
        "svc_default_3": {}, "svc_no_row_cache_3": {"JSP_SVC_ROW_CACHE": "0"}}
STEP = {"rpw1": {"JSP_EXPAND_RPW": "1"}, "rpw4": {"JSP_EXPAND_RPW": "4"}, "rpw16": {"JSP_EXPAND_RPW": "16"},
        "rpw64": {"JSP_EXPAND_RPW": "64"}, "staged": {"JSP_ASSIGN_RECORDS": "0"}, "rpw16_b": {"JSP_EXPAND_RPW": "16"},
        "staged_b": {"JSP_ASSIGN_RECORDS": "0"}}
MARK = {"launch_stop": {}, "record": {"JSP_STREAM_MARK": "record"}, "event_sys": {"JSP_EVENT_FLAGS": "sys"}, "event_dev": {"JSP_EVENT_FLAGS": "dev"},
        "event_nofence": {"JSP_EVENT_FLAGS": "nofence"}, "value": {"JSP_STREAM_MARK": "value"},
        "none": {"JSP_STREAM_MARK": "none"}}


def child_tally():
    import numpy as np
    import torch

    import bench
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from oracle import oracle as O
    p = synth.config4()
    eng = Engine(0)
    eng.load(p)
    stream = torch.cuda.current_stream().cuda_stream
    C, L = len(p.classes), p.topology.n_leaves
    cap = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
    fn = lambda: eng.tally_device(cap.data_ptr(), cap[-1].data_ptr(), L, stream)  # noqa: E731
    fn()
    eng.check()
    _, ocap, oocc = O.place_c(p)
    got = cap.cpu().numpy().astype(np.uint32)
    exact = bool(np.array_equal(got[:C], ocap) and np.array_equal(got[C], oocc))
    for _ in range(10):
        fn()
    warm = bench.event_loop_us(fn, 200, stream)
    scrub = torch.zeros(128 << 20, dtype=torch.int32, device="cuda")
    cold = bench.cold_us(fn, 20, stream, scrub)
    cold_dirty = bench.cold_us(fn, 20, stream, scrub, dirty=True)
    eng.check()
    tb = bench.tally_bytes(p)
    return {"exact": exact, "warm_us": round(warm, 2), "cold_us": round(cold, 2), "cold_dirty_us": round(cold_dirty, 2),
            "warm_frac": round(tb / warm / 1e3 / 8000, 4), "cold_frac": round(tb / cold / 1e3 / 8000, 4)}


def child_mark():
    import numpy as np
    import torch

    import bench
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    out = {}
    eng = Engine(0)
    stream = torch.cuda.current_stream().cuda_stream
    for cfg in (1, 2):
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        rc, rl = job_runs(p.job_class)
        rct = torch.from_numpy(rc.astype(np.int32)).cuda()
        rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
        o = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
        fn = lambda: eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs,  # noqa: E731
                                      o.data_ptr(), stream)
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(1000):
            fn()
        host = (time.perf_counter() - t0) * 1e6 / 1000
        torch.cuda.synchronize()
        gpu = bench.event_loop_us(fn, 1000, stream)
        eng.check()
        out[f"cfg{cfg}"] = {"host_us_per_call": round(host, 2), "gpu_us_per_call": round(gpu, 2)}
    return out


def child_step():
    """cfg4 device path (tally -> feas -> assign -> expand) GPU time per call
    over 500 back-to-back calls, bit-exact vs the oracle."""
    import numpy as np
    import torch

    import bench
    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    from oracle import oracle as O
    p = synth.config4()
    eng = Engine(0)
    eng.load(p)
    stream = torch.cuda.current_stream().cuda_stream
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    o = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
    fn = lambda: eng.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs,  # noqa: E731
                                  o.data_ptr(), stream)
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    exact = bool(np.array_equal(o.cpu().numpy(), O.place_c(p)[0]))
    gpu = bench.event_loop_us(fn, 500, stream)
    eng.check()
    return {"exact": exact, "gpu_us_per_call": round(gpu, 2)}


def child_svc():
    """Host-API jsp_place p50/p99 (resident service) on cfg1/2/3/5, 1000 calls
    each, plus 40 cold calls (the service idle-exited, a row patched)."""
    import numpy as np

    from jobset_amd import synth
    from jobset_amd.engine import Engine
    from jobset_amd.snapshot import job_runs
    from oracle import oracle as O
    out = {}
    eng = Engine(0)
    for cfg in (1, 2, 3, 5):
        p = synth.CONFIGS[cfg]()
        eng.load(p)
        a = O.place_c(p)[0]
        call = eng.host_placer(*job_runs(p.job_class))
        for _ in range(20):
            call()
        assert np.array_equal(call.assign, a)
        lat = []
        for _ in range(1000):
            t0 = time.perf_counter()
            st = call()
            lat.append((time.perf_counter() - t0) * 1e6)
        shape = int(st.fused)
        assert np.array_equal(call.assign, a)
        cold = []
        row = np.zeros(1, dtype=np.uint32)
        for t in range(40):
            time.sleep(0.06)
            row[0] = (t * 7919) % p.nodes.n_nodes
            eng.patch_rows(row, taints=p.nodes.taints[row])
            t0 = time.perf_counter()
            call()
            cold.append((time.perf_counter() - t0) * 1e6)
        assert np.array_equal(call.assign, a)
        lat.sort()
        cold.sort()
        out[f"cfg{cfg}"] = {"shape": shape, "p50": round(lat[500], 2), "p99": round(lat[990], 2),
                            "cold_p50": round(cold[20], 1), "cold_max": round(cold[-1], 1)}
    return out


def main():
    mode = sys.argv[1]
    if mode == "one":
        key = sys.argv[2]
        for d in (TALLY, SVC, SVC2, MARK, STEP):  # the variant's environment (also when run directly, e.g. under rocprofv3)
            os.environ.update(d.get(key, {}))
        res = (child_tally() if key in TALLY else child_svc() if key in SVC or key in SVC2
               else child_step() if key in STEP else child_mark())
        print(json.dumps({key: res}), flush=True)
        return
    variants = {"tally": TALLY, "svc": SVC, "svc2": SVC2, "step": STEP}.get(mode, MARK)
    for key, env in variants.items():
        e = dict(os.environ)
        e.update(env)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "one", key], env=e, capture_output=True,
                           text=True, timeout=240)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        print(line[-1] if line else json.dumps({key: {"rc": r.returncode, "err": r.stderr[-400:]}}), flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
