"""Host-API placement time against where the host thread runs (diagnostic):
the GPU's NUMA node (its PCI device's numa_node), the CPUs this process may
use per node, then for the thread bound to each node in turn: the host-link
floor and cfg2 per-call time (C loop), each on a fresh engine."""
import ctypes
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from jobset_amd import synth  # noqa: E402
from jobset_amd.engine import Engine  # noqa: E402
from jobset_amd.snapshot import job_runs  # noqa: E402


def cpu_node(c):
    g = glob.glob(f"/sys/devices/system/cpu/cpu{c}/node*")
    return int(os.path.basename(g[0])[4:]) if g else -1


hip = ctypes.CDLL("libamdhip64.so")
buf = ctypes.create_string_buffer(64)
hip.hipDeviceGetPCIBusId(buf, 64, 0)
bdf = buf.value.decode().lower()
try:
    gnode = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
except OSError:
    gnode = -1
allowed = sorted(os.sched_getaffinity(0))
nodes = {}
for c in allowed:
    nodes.setdefault(cpu_node(c), []).append(c)
print(f"GPU {bdf} numa_node {gnode}; allowed CPUs per node: { {n: len(v) for n, v in nodes.items()} }", flush=True)
libc = ctypes.CDLL("libc.so.6")
p = synth.config2()
for rep in range(2):
    for n, cpus in sorted(nodes.items()):
        os.sched_setaffinity(0, cpus)
        e = Engine(0)
        e.load(p)
        call = e.host_placer(*job_runs(p.job_class))
        for _ in range(50):
            call()
        fl = e.link_floor(2000)
        tot, p50, p99 = call.loop(2000)
        t = e.timing(reset=True)
        print(f"  rep {rep} thread on node {n} (cpu {libc.sched_getcpu()}): floor p50 {fl[0]:.2f} us | cfg2 per call "
              f"p50 {p50:.2f} p99 {p99:.2f} us", flush=True)
        e.close()
os.sched_setaffinity(0, allowed)
