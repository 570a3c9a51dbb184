"""Back-to-back host-API placements against placements with a gap (test
hook loop_gap_ns: jspb_place_loop spins between calls), cfg2 (diagnostic):
per-call time without the gap, and the library's request post -> first /
last answer line. A post -> first that shrinks as the gap grows means the
service was not ready for a request right behind the previous answer."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

extra = sys.argv[1] if len(sys.argv) > 1 else ""
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
p = synth.CONFIGS[cfg]()
print(f"cfg{cfg}", end=" ")
print(f"hooks: {extra or '-'}; floor", end=" ", flush=True)
for gap in (0, 1000, 3000, 6000, 10000, 0):
    os.environ["JSP_TEST_HOOKS"] = ",".join(x for x in (extra, f"loop_gap_ns={gap}") if x)
    e = Engine(0)
    if gap == 0 and extra == "":
        pass
    e.load(p)
    call = e.host_placer(*job_runs(p.job_class))
    for _ in range(50):
        call()
    e.timing(reset=True)
    tot, p50, p99 = call.loop(2000)
    t = e.timing(reset=True)
    n = max(int(t.svc_calls), 1)
    print(f"\n  gap {gap:5d} ns: per call (gap excluded) p50 {p50:.2f} us | post->first {t.svc_first_us / n:.2f} "
          f"->last {t.svc_answer_us / n:.2f} | svc_pre {t.svc_pre_us / n:.2f}", end="", flush=True)
    e.close()
print(flush=True)
