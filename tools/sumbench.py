"""Print the headline fields of bench.py JSON lines (diagnostic)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"== {f}")
    print(" value", d["value"], "ms", d["ms_per_step"], "p50", d.get("host_api_step_p50_us"), "p99",
          d.get("host_api_step_p99_us"), "py", d.get("python_loop_us_per_step"), "binding", d.get("host_binding"))
    cb = d["cpu_baseline"]
    print(" cpu", cb["value"], cb["gpu_over_best_cpu"], [(l["threads"], l["us_per_placement"]) for l in cb["legs"]])
    print(" patched", d["patched_step_us"], "cpu", d["cpu_patched_step"]["legs_us"], d["cpu_patched_step"]["gpu_over_best_cpu"])
    print(" bd", {k: v for k, v in (d.get("host_api_breakdown") or {}).items() if k != "note"})
    print(" floor", d.get("host_link_floor_us"), "svc dev", (d.get("service") or {}).get("request_us_device"))
    print(" warm p50/p99", d["p50_recovery_us"], d["p99_recovery_us"])
    for k in ("cold_recovery", "cold_recovery_parked"):
        c = d.get(k) or {}
        for g, v in c.get("vs_cpu", {}).items():
            print(" ", k, g, {kk: v[kk] for kk in ("gpu_p50_us", "gpu_p99_us", "best_cpu_p50_us", "best_cpu_p99_us")})
    for cn, l in (d.get("configs") or {}).items():
        print(" ", cn, l["host_api_resident"], (l.get("service_roofline") or {}).get("request_us_device"),
              "cpu1/16", l.get("cpu_fast_1t_us_per_placement"), l.get("cpu_fast_16t_us_per_placement"))
        for g, v in ((l.get("host_api_cold_recovery") or {}).get("vs_cpu") or {}).items():
            print("    ", g, {kk: v[kk] for kk in ("gpu_p50_us", "gpu_p99_us", "best_cpu_p50_us", "best_cpu_p99_us")})
    c4 = d.get("cfg4_1M") or {}
    if c4:
        print(" cfg4", {k: c4.get(k) for k in ("placements_per_s", "tally_us", "tally_span_us", "tally_empty_launch_event_us",
                                              "host_api_step_us", "tally_cold_us")},
              (c4.get("step_device") or {}).get("warm_median_us"), (c4.get("device_set") or {}).get("us_per_step"),
              (c4.get("cpu_baseline") or {}).get("gpu_over_best_cpu"))
    r = d["roofline"]
    print(" roofline", {k: r[k] for k in ("achieved", "frac", "avg_us", "median_us", "trace_median_us", "traffic")})
