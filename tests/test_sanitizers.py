"""The host mirror (jobset_amd/csrc/host: webhook, reconciler, planner, JSON)
and the C oracles under AddressSanitizer + UndefinedBehaviorSanitizer (host
code only): `make sanitize` builds them (Makefile, oracle/Makefile), and the
host-parity, ingestion and oracle suites run against those builds in a child
process with libasan preloaded. Any report aborts the child."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs g++ and hipcc")
def test_host_and_oracle_suites_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-j8", "sanitize"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    assert asan and ubsan
    env = dict(os.environ, LD_PRELOAD=f"{asan}:{ubsan}", ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               JSP_LIB_PATH=os.path.join(ROOT, "build/asan/libjsplace.so"),
               JSPO_LIB_PATH=os.path.join(ROOT, "oracle/sanitize/libjsp_oracle.so"),
               JSPF_LIB_PATH=os.path.join(ROOT, "oracle/sanitize/libjsp_cpufast.so"), JSP_UNDER_SANITIZER="1")
    probe = ("import jobset_amd.native as n, oracle.oracle as o; n.lib(); o.fast_lib(); m=open('/proc/self/maps').read();"
             "print(int('asan/libjsplace.so' in m and 'sanitize/libjsp_cpufast.so' in m and 'libasan' in m))")
    r = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.stdout.strip().endswith("1"), r.stdout + r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        "tests/test_host_parity.py", "tests/test_ingest.py", "tests/test_oracle.py",
                        "tests/test_concurrency.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
