"""Split-service host-API calls (cfg3, cfg5) timed in C (jspb_place_loop), with
the library's phase clocks per call: entry -> request post (svc_pre), post ->
answer complete incl. the host walk (svc_answer), the walk's share
(host_post), and the host-link floor. Diagnostic."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402

if len(sys.argv) > 1:
    os.environ["JSP_TEST_HOOKS"] = sys.argv[1]
e = Engine(0)
fl = e.link_floor(2000)
print(f"floor p50 {fl[0]:.2f} us", flush=True)
for cfg in (3, 5, 2):
    p = synth.CONFIGS[cfg]()
    e.load(p)
    call = e.host_placer(*job_runs(p.job_class))
    for _ in range(50):
        call()
    e.timing(reset=True)
    tot, p50, p99 = call.loop(2000)
    t = e.timing(reset=True)
    n = max(int(t.svc_calls), 1)
    print(f"cfg{cfg}: per call p50 {p50:.2f} p99 {p99:.2f} us | svc_pre {t.svc_pre_us / n:.2f} svc_answer "
          f"{t.svc_answer_us / n:.2f} (walk {t.host_post_us / n:.2f}) | calls {n}", flush=True)
e.close()
