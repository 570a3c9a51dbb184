"""Concurrent callers.

The reference serves the pod webhook concurrently -- one handler goroutine per
AdmissionReview (pkg/webhooks/pod_mutating_webhook.go:45-51, :64) -- and the
recreate path fans its API calls out with ParallelizeUntil(..., 50, ...)
(pkg/controllers/jobset_controller.go:526-530). An engine shared by those
callers sees placements, watch-event patches and the webhook / reconciler
batches from many threads at once, while its own waker thread restarts the
resident service after idle exits.

GPU: 8 host threads on one engine (resident service AUTO, which idles out
and is woken by patches, and PARKED) interleave jsp_place,
jsp_snapshot_patch, jsp_resolve_leader_domains and jsp_audit_placements.
Patches are serialised through a version counter the test owns (a
reader/writer lock: placements of version v run while no patch is in
flight), and every answer is checked bit-exactly against oracle/cpu_ref.c on
the snapshot of the version it was issued against. Every wait is bounded.

CPU: the host mirror (jsk_call: webhook Default / ValidateCreate, the
leader PodReconciler, child-Job construction) from 8 threads on one shared
cache while a writer thread mutates it, each answer equal to the
single-threaded one. tests/test_sanitizers.py runs this file under ASan +
UBSan, and a ThreadSanitizer build of the host mirror
(test_host_mirror_under_tsan) runs the same calls.
"""
import copy
import dataclasses
import os
import random
import shutil
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from jobset_amd import host, synth
from jobset_amd.snapshot import job_runs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JOIN_S = 120.0  # bound on every thread of a test


class VersionLock:
    """Readers (placements, batches) share the current snapshot version;
    the writer (a patch) waits for them to leave and bumps the version.
    Writer preference, bounded waits."""

    def __init__(self):
        self.cv = threading.Condition()
        self.readers = 0
        self.writing = False
        self.waiting = 0
        self.version = 0

    def read(self):
        with self.cv:
            assert self.cv.wait_for(lambda: not self.writing and self.waiting == 0, timeout=JOIN_S)
            self.readers += 1
            return self.version

    def done_read(self):
        with self.cv:
            self.readers -= 1
            self.cv.notify_all()

    def write(self):
        with self.cv:
            self.waiting += 1
            assert self.cv.wait_for(lambda: not self.writing and self.readers == 0, timeout=JOIN_S)
            self.waiting -= 1
            self.writing = True

    def done_write(self):
        with self.cv:
            self.writing = False
            self.version += 1
            self.cv.notify_all()


def _run_threads(targets):
    errors = []

    def wrap(fn):
        def run():
            try:
                fn()
            except BaseException as ex:  # noqa: BLE001 -- surfaced below
                errors.append(ex)
        return run
    ts = [threading.Thread(target=wrap(f), daemon=True) for f in targets]
    for t in ts:
        t.start()
    deadline = time.monotonic() + JOIN_S
    for t in ts:
        t.join(max(0.0, deadline - time.monotonic()))
    alive = [t for t in ts if t.is_alive()]
    assert not alive, f"{len(alive)} threads did not finish within {JOIN_S} s"
    if errors:
        raise errors[0]


def _untolerated_bit(p):
    tol = 0
    for c in p.classes:
        tol |= c.tolerated_taints
    for b in range(31, -1, -1):
        if not (tol >> b) & 1:
            return 1 << b
    raise AssertionError("every taint bit is tolerated")


def _versions(p, n_versions: int):
    """Cumulative one-row patches: version v has the first v rows tainted
    with a bit no class tolerates -- each row the first node of the domain
    the oracle's answer for version v-1 gave job v-1 -- so every patch moves
    the answer. Returns (rows, taint values, expected assign per version)."""
    from oracle import oracle as O
    bit = _untolerated_bit(p)
    leaf_start = np.asarray(p.nodes.leaf_start, dtype=np.int64)
    taints = np.array(p.nodes.taints, dtype=np.uint32)
    cur = p
    expected = [O.place_c(cur)[0]]
    rows, vals = [], []
    for v in range(n_versions):
        a = expected[-1]
        j = int(np.flatnonzero(a >= 0)[v % max(1, int((a >= 0).sum()))])
        lvl = p.classes[int(p.job_class[j])].level
        leaf = int(np.asarray(p.topology.first_leaf[lvl])[a[j]]) if lvl + 1 < p.topology.n_levels else int(a[j])
        r = int(leaf_start[leaf])
        taints = taints.copy()
        taints[r] |= bit
        rows.append(r)
        vals.append(int(taints[r]))
        cur = dataclasses.replace(cur, nodes=dataclasses.replace(cur.nodes, taints=taints))
        expected.append(O.place_c(cur)[0])
    return np.array(rows, dtype=np.uint32), np.array(vals, dtype=np.uint32), expected


def _resolve_expect(p, rows, levels):
    leaf_of_row = p.nodes.leaf_of_row()
    out = []
    for r, k in zip(rows, levels):
        if r < 0:
            out.append(-1)
            continue
        leaf = int(leaf_of_row[r])
        out.append(leaf if k + 1 == p.topology.n_levels else int(p.topology.parent_of_leaf(int(k))[leaf]))
    return np.array(out, dtype=np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["auto", "parked"])
@pytest.mark.parametrize("cfg", [2, 5])
def test_concurrent_callers_one_engine(engine, cfg, mode):
    p = synth.CONFIGS[cfg]()
    engine.load(p)
    engine.set_fused(True)
    engine.set_service(True, parked=(mode == "parked"))
    n_versions = 6
    rows, vals, expected = _versions(p, n_versions)
    rc, rl = job_runs(p.job_class)
    lock = VersionLock()
    results = []  # (version, assign) -- appended under the GIL
    rng_seed = 1000 * cfg + (mode == "parked")
    K = p.topology.n_levels
    N = p.nodes.n_nodes
    before = engine.metrics(reset=True)  # noqa: F841 -- reset

    def placer(tid):
        rng = random.Random(rng_seed + tid)
        for it in range(40):
            # gaps: back to back, a reconciler's round trip, and (AUTO) past
            # the idle exit so that patches and placements meet a service
            # that left and is woken by the waker thread
            time.sleep(rng.choice([0.0, 0.0, 0.0005, 0.002, 0.01, 0.07 if it % 10 == 3 else 0.0]))
            v = lock.read()
            try:
                r = engine.place_runs(rc, rl)
            finally:
                lock.done_read()
            results.append((v, r.assign.copy()))

    def patcher():
        rng = random.Random(rng_seed + 99)
        for i in range(n_versions):
            time.sleep(rng.choice([0.001, 0.005, 0.02, 0.08]))
            lock.write()
            try:
                engine.patch_rows(rows[i:i + 1], taints=vals[i:i + 1])
            finally:
                lock.done_write()

    def batcher(tid):
        rng = random.Random(rng_seed + 50 + tid)
        for _ in range(30):
            n = rng.randint(1, 64)
            lr = np.array([rng.randrange(-1, N) for _ in range(n)], dtype=np.int32)
            lv = np.array([rng.randrange(K) for _ in range(n)], dtype=np.uint32)
            exp = _resolve_expect(p, lr, lv)
            got = engine.resolve_leader_domains(lr, lv)
            np.testing.assert_array_equal(got, exp)
            # audit: two followers per job, the second one wrong for odd jobs
            fd = np.stack([exp, np.where(np.arange(n) % 2 == 1, exp + 1, exp)], axis=1).reshape(-1).astype(np.int32)
            off = np.arange(0, 2 * n + 1, 2, dtype=np.uint32)
            bad = engine.audit_placements(lr, lv, off, fd)
            want = np.where(lr < 0, 0xFFFFFFFF, np.where(np.arange(n) % 2 == 1, 1, 0)).astype(np.uint32)
            np.testing.assert_array_equal(bad, want)
            time.sleep(rng.choice([0.0, 0.001, 0.01]))

    try:
        _run_threads([lambda t=t: placer(t) for t in range(5)] + [patcher] +
                     [lambda t=t: batcher(t) for t in range(2)])
        assert lock.version == n_versions
        assert len(results) == 5 * 40
        seen = set()
        for v, a in results:
            seen.add(v)
            np.testing.assert_array_equal(a, expected[v], err_msg=f"cfg{cfg} {mode}: version {v}")
        assert len(seen) >= 2, seen  # the placements met more than one snapshot version
        # after everything, the engine answers the final version
        np.testing.assert_array_equal(engine.place_runs(rc, rl).assign, expected[-1])
        m = engine.metrics()
        assert m.place_us.count == 5 * 40 + 1 and m.place_errors == 0 and m.patch_errors == 0
        assert m.patch_us.count == n_versions
        assert m.batch_jobs.count == m.place_us.count and m.placed + m.unplaceable == m.place_us.count * p.n_jobs
    finally:
        engine.service_stop()
        engine.set_service(True)


# ---------------------------------------------------------------------------- host mirror (CPU)
JOBSET, RJOB, JOBIDX, JOBKEY = ("jobset.sigs.k8s.io/jobset-name", "jobset.sigs.k8s.io/replicatedjob-name",
                                "jobset.sigs.k8s.io/job-index", "jobset.sigs.k8s.io/job-key")
EXCL = "alpha.jobset.sigs.k8s.io/exclusive-topology"
COMPLETION = "batch.kubernetes.io/job-completion-index"


def _pod(name, ns, labels, ann, node, owner):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": ns, "labels": labels, "annotations": ann,
                      "ownerReferences": [{"kind": "Job", "name": "-".join(name.split("-")[:-2]), "uid": owner,
                                           "controller": True}]},
         "spec": {"containers": [{"name": "c"}]}}
    if node:
        p["spec"]["nodeName"] = node
    return p


def _host_world(n_jobs=24, followers=3):
    """A cache with n_jobs bound leaders on racked nodes, and the calls of
    their followers' admission: (cache, work items [(method, request)])."""
    c = host.Cache()
    items = []
    for j in range(n_jobs):
        job = f"js-rj-{j}"
        key = host.jobHashKey("default", job)
        lab = {JOBSET: "js", RJOB: "rj", JOBIDX: str(j), JOBKEY: key}
        ann = {**lab, EXCL: "rack"}
        node = f"node-{j}"
        c.add_node({"metadata": {"name": node, "labels": {"rack": f"rack-{j // 2}" if j % 5 else "x"}}})
        if j % 7 == 3:
            c.add_node({"metadata": {"name": node, "labels": {"zone": "z"}}})  # lacks the rack label
        leader = _pod(f"{job}-0-abcde", "default", lab, {**ann, COMPLETION: "0"}, node, f"uid-{j}")
        c.add_pod(leader)
        items.append(("webhooks.Default", {"pod": leader}))
        for i in range(1, followers + 1):
            f = _pod(f"{job}-{i}-fghij", "default", lab, {**ann, COMPLETION: str(i)}, None, f"uid-{j}")
            items.append(("webhooks.Default", {"pod": f}))
            g = copy.deepcopy(f)
            g["spec"]["nodeSelector"] = {"rack": f"rack-{j // 2}"}
            items.append(("webhooks.ValidateCreate", {"pod": g}))
            if i == 1:
                items.append(("webhooks.ValidateCreate", {"pod": f}))
        items.append(("controllers.Reconcile", {"namespace": "default", "name": f"{job}-0-abcde",
                                                "now": "2024-10-08T00:00:00Z"}))
        items.append(("controllers.jobHashKey", {"ns": "default", "jobName": job}))
        items.append(("placement.GenPodName", {"jobSet": "js", "replicatedJob": "rj", "jobIndex": str(j),
                                               "podIndex": "0"}))
    return c, items


def _call(c, method, req):
    r = dict(req)
    if method.startswith(("webhooks.", "controllers.Reconcile")):
        r["cache"] = c.id
    return host.call(method, **r)


def test_host_mirror_concurrent_callers():
    c, items = _host_world()
    expected = [_call(c, m, r) for m, r in items]
    stop = threading.Event()

    def caller(tid):
        rng = random.Random(tid)
        order = list(range(len(items))) * 3
        rng.shuffle(order)
        for i in order:
            got = _call(c, *items[i])
            assert got == expected[i], (items[i][0], got, expected[i])

    def writer():
        # unrelated objects come and go (another namespace, other nodes)
        k = 0
        while not stop.is_set() and k < 2000:
            name = f"other-{k % 17}-0-zzzzz"
            c.add_pod(_pod(name, "other", {JOBSET: "o"}, {COMPLETION: "0"}, None, "uid-o"))
            c.add_node({"metadata": {"name": f"spare-{k % 5}", "labels": {"rack": "spare"}}})
            c.remove_pod("other", name)
            k += 1

    w = threading.Thread(target=writer, daemon=True)
    w.start()
    try:
        _run_threads([lambda t=t: caller(t) for t in range(8)])
    finally:
        stop.set()
        w.join(JOIN_S)
    assert not w.is_alive()


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs g++ and hipcc")
def test_host_mirror_under_tsan():
    """The host mirror built with -fsanitize=thread (Makefile `tsan`), the
    concurrent-callers test above run against it with libtsan preloaded: any
    data race report fails the child."""
    if os.environ.get("JSP_UNDER_SANITIZER"):
        pytest.skip("already inside a sanitizer run")
    r = subprocess.run(["make", "-s", "-j8", "tsan"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    tsan = subprocess.run(["g++", "-print-file-name=libtsan.so"], capture_output=True, text=True).stdout.strip()
    assert os.path.isabs(tsan) and os.path.exists(tsan)
    env = dict(os.environ, LD_PRELOAD=tsan, TSAN_OPTIONS="halt_on_error=1:exitcode=66:report_signal_unsafe=0",
               JSP_LIB_PATH=os.path.join(ROOT, "build/tsan/libjsplace.so"), JSP_UNDER_SANITIZER="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        "tests/test_concurrency.py::test_host_mirror_concurrent_callers"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout[-3000:] + r.stderr[-3000:]
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, out
    probe = subprocess.run([sys.executable, "-c", "import jobset_amd.native as n; n.lib(); "
                            "print(int('tsan/libjsplace.so' in open('/proc/self/maps').read()))"],
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert probe.stdout.strip().endswith("1"), probe.stdout + probe.stderr[-2000:]
