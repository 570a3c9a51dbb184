"""The line bench.py prints must stay parseable by the driver, which keeps only
the last 8 KB of the run's stdout and stderr (a 21 KB line left
BENCH_r05 with `parsed: null`). build_line() is the function bench.py prints
through; here it runs on a stubbed detail dict with every block present and
every number at a worst-case width."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


X = 123456789.123  # worst-case width of any measured number


def _pc(n=1000):
    return {"p50_us": X, "p95_us": X, "p99_us": X, "max_us": X, "n": n}


def _vs(n=1000):
    return {"gpu_p50_us": X, "gpu_p95_us": X, "gpu_p99_us": X, "gpu_n": n, "best_cpu_leg": "16t",
            "cpu_p50_us": X, "cpu_p95_us": X, "cpu_p99_us": X, "cpu_n": n}


def stub_detail(b):
    gaps = [f"gap_{g:g}ms" for g in b.COLD_GAPS]
    legs = [{"threads": t, "us_per_placement": X, "placements_per_s": X, "runs": 99999, "seconds": X}
            for t in (1, 2, 16)]
    c2 = {"value": X, "ms_per_step": X, "nodes": 15000, "domains": 1000, "jobs": 990, "placed": 990,
          "pods_per_job": 15, "classes": 1, "shape": b.SHAPES[5], "loop_p50_us": X, "loop_p99_us": X,
          "kernel_only_placements_per_s": X, "kernel_only_us_per_step": X,
          "roofline": {"kernel": "place_compact_kernel", "bytes": 427964, "avg_us": X, "median_us": X,
                       "achieved": X, "frac": X, "traffic": 494000, "traffic_source": "profiles/r06/e1",
                       "trace_median_us": X, "trace_source": "profiles/r06/e1/summary.txt"},
          "cpu": {"value": X, "cores": 16, "legs": legs, "gpu_over_best_cpu": X,
                  "sample": "cfg2 placed 99999x in 3.0 s by oracle/cpu_fast.c (16 threads, fastest of 1/2/16; "
                            "bit-exact with the engine)"},
          "warm_trials": _pc(200), "patched": {"mean_us": X, "p50_us": X, "p99_us": X}, "cpu_patched_best_us": X,
          "link_floor_p50_us": X, "service_request_us_device": X}
    cfg = {"nodes": 40960, "jobs": 64, "placed": 64, "kernel_us": X, "kernel_loop_us": X, "kernel_frac": X,
           "service_frac": X,
           "host_api_resident": _pc(200), "cpu_us": {"1t": X, "16t": X},
           "cold_vs_cpu": {g: _vs(100) for g in gaps}}
    c4 = {k: X for k in ("placements_per_s", "host_api_us", "kernel_only_us", "kernel_only_placements_per_s",
                         "tally_us", "tally_frac", "tally_cold_us", "tally_cold_frac", "copy_cold_us",
                         "tally_traffic", "allreduce_us")}
    c4.update({"shards": 8, "placed": 31115,
               "cpu_baseline": {"best_us": X, "cores": 16, "gpu_over_best_cpu": X},
               "device_set": {"us_per_step": X, "shards": 8, "devices": 8, "bit_exact_vs_single_device": True,
                              "error": None}})
    return {"world": 8, "steps": 2000, "warmup": 200, "cfg2": c2,
            "cold2": {"gpu": {g: _pc() for g in gaps}, "vs_cpu": {g: _vs() for g in gaps}},
            "cold2_parked": {"vs_cpu": {g: _vs(100) for g in gaps}},
            "configs": {"cfg1": dict(cfg), "cfg3": dict(cfg), "cfg5": dict(cfg)}, "cfg4": c4,
            "binding": {"bound": True, "gpu_numa_node": 1, "cpus": 16},
            "detail_path": "gpurun_out/bench_detail.json"}


def test_line_fits_the_driver_tail():
    b = _bench()
    s = b.emit(b.build_line(stub_detail(b)))
    assert len(s) <= b.LINE_MAX_BYTES <= 8192 - 1024, len(s)
    line = json.loads(s)
    # every block survives at worst-case widths (emit drops none)
    for k in ("cfg1", "cfg3", "cfg5", "cfg4", "cold_recovery_parked"):
        assert k in line, k


def test_line_carries_the_contract_fields():
    b = _bench()
    line = json.loads(b.emit(b.build_line(stub_detail(b))))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "p99_recovery_us",
              "p50_recovery_us", "cold_recovery", "patched_step_us"):
        assert k in line, k
    assert line["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert set(line["roofline"]) >= {"bound", "achieved", "peak", "unit", "frac", "traffic"}
    assert set(line["cpu_baseline"]) >= {"value", "unit", "cores", "kind", "sample"}
    assert line["cpu_baseline"]["kind"] in ("port", "reference")
    # the headline p99 is the cold recovery's at the 1 ms gap, beside the CPU's
    assert line["recovery_trials"] == 1000 and "p99_recovery_cpu_us" in line
    assert set(line["cold_recovery"]) == {"0ms", "1ms", "10ms"}
    assert all(len(v) == 8 for v in line["cold_recovery"].values())


def test_line_has_no_prose_notes():
    """Only the fixed labels (workload, cold_cols, recovery_leg, shape,
    sample) are strings longer than a word; nothing named *note*."""
    b = _bench()
    s = b.emit(b.build_line(stub_detail(b)))
    assert "note" not in s

    def strings(x):
        if isinstance(x, dict):
            for v in x.values():
                yield from strings(v)
        elif isinstance(x, list):
            for v in x:
                yield from strings(v)
        elif isinstance(x, str):
            yield x
    assert sum(len(t) for t in strings(json.loads(s))) < 1200
