"""GPU tests of the engine wired into the reference's seams (SURVEY.md §8a A5,
A9, A10 and §8f rows 1-4): the planner ingests informer-cache Node / Pod
objects into the resident snapshot, places JobSets' child Jobs through
jsp_place, serves the webhook's follower topology and the PodReconciler's
audit from the snapshot (batched), and labels node pools for the
node-selector strategy. Results are compared with the oracle on the same
snapshot and, for the webhook / reconciler, with the reference's Node-Get
path byte for byte."""
import copy
import json
import os

import numpy as np
import pytest

from jobset_amd import host, synth
from jobset_amd.engine import Engine
from jobset_amd.native import JspStats, check
from oracle import oracle as O

import k8s_fixtures as K

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))
EXCL = "alpha.jobset.sigs.k8s.io/exclusive-topology"
JOBSET = "jobset.sigs.k8s.io/jobset-name"
RJOB = "jobset.sigs.k8s.io/replicatedjob-name"
JOBIDX = "jobset.sigs.k8s.io/job-index"
JOBKEY = "jobset.sigs.k8s.io/job-key"
RESTARTS = "jobset.sigs.k8s.io/restart-attempt"
COMPLETION = "batch.kubernetes.io/job-completion-index"
NSJOB = "alpha.jobset.sigs.k8s.io/namespaced-job"
NOSCHED = "alpha.jobset.sigs.k8s.io/no-schedule"
POOL = "cloud.google.com/gke-nodepool"
RES = ["cpu", "memory", "amd.com/gpu"]


def node(name, labels, taints=(), unschedulable=False, gpus=8):
    spec = {"taints": list(taints)}
    if unschedulable:
        spec["unschedulable"] = True
    return {"metadata": {"name": name, "labels": labels}, "spec": spec,
            "status": {"allocatable": {"cpu": "192", "memory": "1536000Mi", "amd.com/gpu": str(gpus)}}}


def engine_tallies(engine, cols, n_classes, job_class):
    """jsp_place with tally output on the engine's resident snapshot + classes."""
    L = len(cols["leafStart"]) - 1
    assign = np.empty(max(len(job_class), 1), dtype=np.int32)
    cap = np.empty((max(n_classes, 1), max(L, 1)), dtype=np.uint32)
    occ = np.empty(max(L, 1), dtype=np.uint32)
    jc = np.ascontiguousarray(job_class, dtype=np.uint32)
    st = JspStats()
    import ctypes
    check(engine._lib.jsp_place_jobs(engine._h, jc.ctypes.data, jc.shape[0], assign.ctypes.data, cap.ctypes.data,
                                     occ.ctypes.data, ctypes.byref(st)))
    return assign[:len(job_class)], cap[:n_classes, :L], occ[:L]


def planned(c, jobs):
    r, e = c.plan(jobs)
    assert e is None, e
    return r


# ------------------------------------------------------------------ ingestion + engine vs oracle
@pytest.mark.parametrize("seed", range(12))
def test_planner_places_like_oracle(engine, seed):
    """Node / Pod / Job objects of a random snapshot -> planner -> engine; the
    oracle on the planner's own snapshot and classes gives the same assign[],
    and the same placements by domain value as the original problem."""
    p = synth.random_problem(seed, max_nodes=3000, max_leaves=120)
    c = host.Cache()
    K.load_cache(c, p)
    c.planner_new(engine, [K.level_key(k) for k in range(p.topology.n_levels)], K.res_names(p.nodes.n_res))
    r = planned(c, K.job_objects(p))
    cols = c.planner_columns()
    q = K.problem_from_planner(p, cols, r)
    a_q = O.place_c(q)[0]
    got = np.array([j["domainId"] for j in r["jobs"]], dtype=np.int32)
    np.testing.assert_array_equal(got, a_q)
    vals = {k: v for k, v in enumerate(cols["domainValues"])}
    assert K.assign_values(p, O.place_c(p)[0]) == [j["domain"] for j in r["jobs"]]
    assert K.assign_values(q, got, vals) == [j["domain"] for j in r["jobs"]]


def exclusive_placement_jobset():
    """examples/simple/exclusive-placement.yaml as an object (restated: the
    reference tree is not on the GPU box)."""
    return {"metadata": {"name": "exclusive-placement", "annotations": {EXCL: POOL}},
            "spec": {"failurePolicy": {"maxRestarts": 3}, "network": {},
                     "replicatedJobs": [{"name": "workers", "replicas": 3, "template": {"spec": {
                         "parallelism": 3, "completions": 3, "backoffLimit": 10, "template": {"spec": {
                             "containers": [{"name": "sleep", "image": "busybox", "command": ["sleep"],
                                             "args": ["1000s"]}]}}}}}]},
            "status": {"restarts": 0}}


def pool_cluster(c, pools=4, per=3):
    for i in range(pools):
        for n in range(per):
            c.add_node(node(f"gke-pool-{i}-node-{n}", {POOL: f"pool-{i}", "kubernetes.io/os": "linux",
                                                       "kubernetes.io/hostname": f"gke-pool-{i}-node-{n}"}))


def test_config1_from_node_objects(engine):
    """examples/simple/exclusive-placement.yaml (the JobSet object of the
    reference's example, tests/golden/reference_vectors.json) on 4 node pools
    x 3 nodes: the engine reproduces synth.config1()'s assign / cap / occ."""
    js = exclusive_placement_jobset()
    c = host.Cache()
    pool_cluster(c)
    c.planner_new(engine, [POOL], RES)
    jobs = []
    for rj in js["spec"]["replicatedJobs"]:
        jobs += host.constructJobsFromTemplate(js, rj, {})
    r = planned(c, jobs)
    assert [j["domain"] for j in r["jobs"]] == ["pool-0", "pool-1", "pool-2"] and r["unplaceable"] == []
    cols = c.planner_columns()
    a, cap, occ = engine_tallies(engine, cols, len(r["classes"]), r["jobClass"])
    p1 = synth.config1()
    a1, cap1, occ1 = O.place_c(p1)
    np.testing.assert_array_equal(a, a1)
    np.testing.assert_array_equal(cap, cap1)
    np.testing.assert_array_equal(occ, occ1)


def rack_cluster(c, zones=2, racks=4, per=4, gpus=8):
    for z in range(zones):
        for r in range(racks):
            for n in range(per):
                name = f"z{z}-r{r}-n{n}"
                c.add_node(node(name, {"zone": f"zone-{z}", "rack": f"zone-{z}-rack-{r}",
                                       "kubernetes.io/hostname": name}, gpus=gpus))


def gpu_job_set(name, replicas=3, parallelism=4, key="rack", restarts=0):
    return {"metadata": {"name": name, "namespace": "default", "annotations": {EXCL: key}},
            "spec": {"replicatedJobs": [{"name": "workers", "replicas": replicas, "template": {
                "spec": {"parallelism": parallelism, "completions": parallelism, "template": {"spec": {
                    "containers": [{"name": "train", "resources": {"requests": {"amd.com/gpu": "8"}}}]}}}}}],
                "network": {}},
            "status": {"restarts": restarts}}


def bind_job_pods(c, job, nodes, phase="Running"):
    """The Job controller + scheduler outcome: one pod per node, bound."""
    pods = []
    for i, nn in enumerate(nodes):
        md = job["spec"]["template"]["metadata"]
        pods.append({"metadata": {"name": f"{job['metadata']['name']}-{i}-abcde", "namespace": "default",
                                  "labels": dict(md["labels"]),
                                  "annotations": {**md["annotations"], COMPLETION: str(i)},
                                  "ownerReferences": [{"uid": f"uid-{job['metadata']['name']}", "kind": "Job",
                                                       "controller": True}]},
                     "spec": {"nodeName": nn, **copy.deepcopy(job["spec"]["template"]["spec"])},
                     "status": {"phase": phase}})
    for p in pods:
        c.add_pod(p)
    return pods


def test_patch_event_matches_reingest(engine):
    """Watch events that keep the snapshot's structure (a node gains a taint
    already in the dictionary, a pod binds and takes GPUs) go to the engine as
    a row patch; the placement then equals a fresh full ingest of the same
    objects."""
    c = host.Cache()
    rack_cluster(c)
    c.add_node(node("z1-r3-n3", {"zone": "zone-1", "rack": "zone-1-rack-3", "kubernetes.io/hostname": "z1-r3-n3"},
                    taints=[{"key": "maintenance", "value": "", "effect": "NoSchedule"}]))
    c.planner_new(engine, ["zone", "rack"], RES)
    js = gpu_job_set("train", replicas=6)
    jobs = host.constructJobsFromTemplate(js, js["spec"]["replicatedJobs"][0], {})
    planned(c, jobs)
    assert c.planner_sync()["upload"] == "none"
    # events
    c.add_node(node("z0-r1-n2", {"zone": "zone-0", "rack": "zone-0-rack-1", "kubernetes.io/hostname": "z0-r1-n2"},
                    taints=[{"key": "maintenance", "value": "", "effect": "NoSchedule"}]))
    other = gpu_job_set("other", replicas=1, parallelism=1)
    ojob = host.constructJobsFromTemplate(other, other["spec"]["replicatedJobs"][0], {})[0]
    bind_job_pods(c, ojob, ["z0-r2-n0"])
    st = c.planner_sync()
    assert st["upload"] == "patch" and st["patchedRows"] == 5  # the tainted row + the held rack's 4 rows
    r = planned(c, jobs)
    cols = c.planner_columns()
    got = engine_tallies(engine, cols, len(r["classes"]), r["jobClass"])
    fresh_engine = Engine(0)
    try:
        f = host.Cache()
        rack_cluster(f)
        for n in ("z1-r3-n3", "z0-r1-n2"):
            f.add_node(node(n, {"zone": f"zone-{n[1]}", "rack": f"zone-{n[1]}-rack-{n[4]}",
                                "kubernetes.io/hostname": n},
                            taints=[{"key": "maintenance", "value": "", "effect": "NoSchedule"}]))
        bind_job_pods(f, ojob, ["z0-r2-n0"])
        f.planner_new(fresh_engine, ["zone", "rack"], RES)
        rf = planned(f, jobs)
        assert f.planner_columns() == cols
        want = engine_tallies(fresh_engine, cols, len(rf["classes"]), rf["jobClass"])
    finally:
        fresh_engine.close()
    for x, y in zip(got, want):
        np.testing.assert_array_equal(x, y)
    # racks with the tainted node / the exclusive pod are skipped: 0-1 (taint), 0-2 (other's pod)
    assert [j["domain"] for j in r["jobs"]] == ["zone-0-rack-0", "zone-0-rack-3", "zone-1-rack-0", "zone-1-rack-1",
                                                "zone-1-rack-2", None]


def test_recreate_path_consults_engine(engine):
    """A10: fail -> restart -> recreate. failurePolicyRecreateAll bumps
    restarts; while the old attempt's Jobs are listed, reconcileRecreate
    deletes and creates nothing; once they and their pods are gone (watch
    Deleted events) it constructs the new attempt's Jobs unchanged and places
    them on the post-delete snapshot -- the engine's assign[] equals the
    oracle's on that snapshot."""
    c = host.Cache()
    rack_cluster(c)
    c.planner_new(engine, ["zone", "rack"], RES)
    js = gpu_job_set("train", replicas=3)
    rj = js["spec"]["replicatedJobs"][0]
    jobs = host.constructJobsFromTemplate(js, rj, {})
    plan0 = planned(c, jobs)
    assert [j["domain"] for j in plan0["jobs"]] == ["zone-0-rack-0", "zone-0-rack-1", "zone-0-rack-2"]
    pods = []
    for job, pj in zip(jobs, plan0["jobs"]):
        z, r = pj["domain"][5], pj["domain"][-1]
        pods += bind_job_pods(c, job, [f"z{z}-r{r}-n{n}" for n in range(4)])
    # another tenant holds zone-0-rack-3; job 1 fails
    other = gpu_job_set("other", replicas=1, parallelism=1)
    bind_job_pods(c, host.constructJobsFromTemplate(other, other["spec"]["replicatedJobs"][0], {})[0], ["z0-r3-n0"])
    jobs[1]["status"] = {"conditions": [{"type": "Failed", "status": "True"}]}
    owned, err = host.getChildJobs(js, jobs)
    assert err is None and [j["metadata"]["name"] for j in owned["failed"]] == ["train-workers-1"]
    js1 = host.failurePolicyRecreateAll(js, True)
    out, err = c.reconcileRecreate(js1, jobs)
    assert err is None and out["delete"] == ["train-workers-0", "train-workers-1", "train-workers-2"]
    assert out["create"] == [] and out["plan"] is None
    # Foreground deletion: pods, then Jobs, leave the cache; a node of rack 0 goes unschedulable
    for p in pods:
        c.remove_pod(p["metadata"]["namespace"], p["metadata"]["name"])
    c.add_node(node("z0-r0-n1", {"zone": "zone-0", "rack": "zone-0-rack-0", "kubernetes.io/hostname": "z0-r0-n1"},
                    unschedulable=True))
    out, err = c.reconcileRecreate(js1, [])
    assert err is None and out["delete"] == [] and "planError" not in out
    create = out["create"]
    assert [j["metadata"]["labels"][RESTARTS] for j in create] == ["1", "1", "1"]
    assert create == host.constructJobsFromTemplate(js1, js1["spec"]["replicatedJobs"][0], {})  # Jobs unchanged
    plan = out["plan"]
    cols = c.planner_columns()
    q = K.problem_from_planner(synth.config1(), cols, plan)
    a_q, cap_q, occ_q = O.place_c(q)
    np.testing.assert_array_equal(np.array([j["domainId"] for j in plan["jobs"]], dtype=np.int32), a_q)
    # rack 0 has an unschedulable node (3 of 4 GPUs nodes left), rack 3 is held: 1, 2, then zone 1
    assert [j["domain"] for j in plan["jobs"]] == ["zone-0-rack-1", "zone-0-rack-2", "zone-1-rack-0"]
    a, cap, occ = engine_tallies(engine, cols, len(plan["classes"]), plan["jobClass"])
    np.testing.assert_array_equal(cap, cap_q)
    np.testing.assert_array_equal(occ, occ_q)


def webhook_pods(ns, js, idx, owner, key, leader_node, n=3):
    job = f"{js}-w-{idx}"
    jkey = host.jobHashKey(ns, job)
    lab = {JOBSET: js, RJOB: "w", JOBIDX: str(idx), JOBKEY: jkey}
    ann = {**lab, EXCL: key}
    pods = []
    for i in range(n):
        pods.append({"metadata": {"name": f"{job}-{i}-abcde", "namespace": ns, "labels": dict(lab),
                                  "annotations": {**ann, COMPLETION: str(i)},
                                  "ownerReferences": [{"uid": owner, "kind": "Job", "controller": True}]},
                     "spec": {"nodeName": leader_node} if i == 0 else {}})
    return pods


def test_batched_follower_resolution_and_audit(engine):
    """§8f rows 2-3: DefaultBatch resolves every follower of a JobSet with one
    engine call and mutates each exactly as the reference's per-pod Default on
    a Node-Get cache; Reconcile audits a leader's whole job with one engine
    call; mismatches and missing selectors give the reference's first error."""
    plain, bound = host.Cache(), host.Cache()
    for c in (plain, bound):
        rack_cluster(c)
    bound.planner_new(engine, ["zone", "rack"], RES)
    bound.planner_sync()
    leaders = ["z0-r1-n2", "z1-r3-n0", "z0-r0-n0", "z1-r2-n3"]
    keys = ["rack", "zone", "rack", "kubernetes.io/hostname"]  # the last is not an engine level
    all_pods = [webhook_pods("default", "js", i, f"u{i}", keys[i], leaders[i]) for i in range(4)]
    followers = []
    for pods in all_pods:
        for c in (plain, bound):
            c.add_pod(pods[0])
        followers += pods[1:]
    before = bound.stats()
    got = bound.DefaultBatch(followers)
    after = bound.stats()
    want = [plain.Default(f) for f in followers]
    assert got == [(p, e) for p, e in want]
    assert after["engineCalls"] - before["engineCalls"] == 1        # one call for the engine-held followers
    assert after["nodeGets"] - before["nodeGets"] == 2              # the hostname-key followers: Node Gets
    assert {tuple(p["spec"]["nodeSelector"].items()) for p, _ in got} >= {(("rack", "zone-0-rack-1"),)}
    for (p, _) in got:
        for c in (plain, bound):
            c.add_pod(p)
    for i, pods in enumerate(all_pods):
        name = pods[0]["metadata"]["name"]
        b0 = bound.stats()
        assert bound.Reconcile("default", name) == plain.Reconcile("default", name) is None
        b1 = bound.stats()
        if keys[i] != "kubernetes.io/hostname":
            assert b1["engineCalls"] - b0["engineCalls"] == 1 and b1["nodeGets"] == b0["nodeGets"]
    # a follower pinned elsewhere, then one without the selector: identical errors
    bad = copy.deepcopy([p for p, _ in got][0])
    bad["spec"]["nodeSelector"] = {"rack": "zone-1-rack-3"}
    for c in (plain, bound):
        c.add_pod(bad)
    name = all_pods[0][0]["metadata"]["name"]
    e = plain.Reconcile("default", name)
    assert e == 'follower topology "zone-1-rack-3" != leader topology "zone-0-rack-1"'
    assert bound.Reconcile("default", name) == e
    nosel = copy.deepcopy(bad)
    del nosel["spec"]["nodeSelector"]
    for c in (plain, bound):
        c.add_pod(nosel)
    e = plain.Reconcile("default", name)
    assert e is not None and "nodeSelector is nil" in e and bound.Reconcile("default", name) == e


def test_engine_bound_topology_boundary_cases(engine):
    """A5 edge cases stay the reference's with an engine bound: a node without
    the topology label -> its error; a key that is not an engine level -> the
    Node's label (Node Get); an unknown node -> "" and no error."""
    plain, bound = host.Cache(), host.Cache()
    for c in (plain, bound):
        rack_cluster(c)
        c.add_node(node("lonely", {"zone": "zone-0", "kubernetes.io/hostname": "lonely"}))  # no rack label
    bound.planner_new(engine, ["zone", "rack"], RES)
    st = bound.planner_sync()
    assert st["skippedNodes"] == ["lonely"]
    cases = [("lonely", "rack"), ("lonely", "zone"), ("z0-r2-n1", "kubernetes.io/hostname"),
             ("no-such-node", "rack"), ("z1-r1-n1", "rack"), ("z1-r1-n1", "zone")]
    for i, (nn, key) in enumerate(cases):
        pods = webhook_pods("default", f"b{i}", 0, f"u{i}", key, nn)
        for c in (plain, bound):
            c.add_pod(pods[0])
        assert bound.Default(pods[1]) == plain.Default(pods[1]), (nn, key)
    m, e = bound.Default(webhook_pods("default", "b0", 0, "u0", "rack", "lonely")[1])
    assert e == "node does not have topology label: rack"
    m, e = bound.Default(webhook_pods("default", "b3", 0, "u3", "rack", "no-such-node")[1])
    assert e is None and m["spec"]["nodeSelector"] == {"rack": ""}


def test_node_events_after_sync_take_node_get_path(engine):
    """After a sync, a Node removed or relabelled in the cache must not be
    answered from the (now stale) snapshot: the reference's live Node Get
    gives "" + nil for a removed node and the new label value for a
    relabelled one (pod_mutating_webhook.go:173-194, pod_controller.go:242-263).
    Default, DefaultBatch and Reconcile stay identical to the Node-Get cache
    until the next sync, which serves from the engine again."""
    plain, bound = host.Cache(), host.Cache()
    for c in (plain, bound):
        rack_cluster(c)
    bound.planner_new(engine, ["zone", "rack"], RES)
    bound.planner_sync()
    leaders = ["z0-r1-n2", "z1-r3-n0", "z0-r0-n0"]
    all_pods = [webhook_pods("default", "ev", i, f"u{i}", "rack", leaders[i]) for i in range(3)]
    for pods in all_pods:
        for c in (plain, bound):
            c.add_pod(pods[0])
    # events after the sync: leader 0's node is deleted, leader 1's node moves rack
    moved = node("z1-r3-n0", {"zone": "zone-1", "rack": "zone-1-rack-9", "kubernetes.io/hostname": "z1-r3-n0"})
    for c in (plain, bound):
        c.remove_node("z0-r1-n2")
        c.add_node(moved)
    followers = [p for pods in all_pods for p in pods[1:]]
    want = [plain.Default(f) for f in followers]
    assert [bound.Default(f) for f in followers] == want
    assert bound.DefaultBatch(followers) == want
    assert want[0][0]["spec"]["nodeSelector"] == {"rack": ""}
    assert want[2][0]["spec"]["nodeSelector"] == {"rack": "zone-1-rack-9"}
    for (p, _) in want:
        for c in (plain, bound):
            c.add_pod(p)
    for pods in all_pods:
        name = pods[0]["metadata"]["name"]
        assert bound.Reconcile("default", name) == plain.Reconcile("default", name)
    # the next sync brings the snapshot up to date: engine answers, same mutations
    bound.planner_sync()
    b0 = bound.stats()
    assert bound.DefaultBatch(followers[4:]) == want[4:]
    assert bound.stats()["engineCalls"] - b0["engineCalls"] == 1


def test_label_nodes_is_deterministic(engine):
    """§8f row 4: the node-selector strategy's node patches from the engine's
    lowest-index assignment, replacing label_nodes.py's set-order mapping
    (hack/label_nodes/label_nodes.py:115-120). Job names are
    generate_namespaced_jobs' (:99-112, golden vector); patch bodies are the
    script's (:65-80)."""
    js = exclusive_placement_jobset()
    c = host.Cache()
    pool_cluster(c, pools=4)
    # pool-1 is tainted for another tenant (not tolerated): skipped
    for n in range(3):
        c.add_node(node(f"gke-pool-1-node-{n}", {POOL: "pool-1", "kubernetes.io/os": "linux"},
                        taints=[{"key": "tenant", "value": "b", "effect": "NoSchedule"}]))
    c.planner_new(engine, [POOL], RES)
    r, err = c.labelNodes(js)
    assert err is None
    names = GOLD["generateNamespacedJobs"]["want"]
    assert r["mapping"] == {names[0]: "pool-0", names[1]: "pool-2", names[2]: "pool-3"}
    assert r["unplaceable"] == []
    body = lambda job: {"metadata": {"labels": {NSJOB: job}},  # noqa: E731
                        "spec": {"taints": [{"key": NOSCHED, "value": "true", "effect": "NoSchedule"}]}}
    want = [{"node": f"gke-pool-{p}-node-{n}", "body": body(names[j])} for j, p in enumerate((0, 2, 3))
            for n in range(3)]
    assert r["patches"] == want
    assert c.labelNodes(js)[0] == r  # deterministic
