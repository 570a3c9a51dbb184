"""Parity of the host-side mirror (include/jsk_host.h) with the reference's own
unit tests, replayed from tests/golden/reference_vectors.json (each vector
cites the reference test file:line it was transcribed from), plus the webhook
and reconciler behaviours SURVEY.md §8a rows A4-A6/A9/A11 list, which no
reference test covers (pod_mutating_webhook.go has no _test file) — those are
checked against the reference code's control flow as cited."""
import copy
import json
import os

import pytest

from jobset_amd import host

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))

JOBSET = "jobset.sigs.k8s.io/jobset-name"
RJOB = "jobset.sigs.k8s.io/replicatedjob-name"
JOBIDX = "jobset.sigs.k8s.io/job-index"
JOBKEY = "jobset.sigs.k8s.io/job-key"
GIDX = "jobset.sigs.k8s.io/job-global-index"
REPL = "jobset.sigs.k8s.io/replicatedjob-replicas"
RESTARTS = "jobset.sigs.k8s.io/restart-attempt"
EXCL = "alpha.jobset.sigs.k8s.io/exclusive-topology"
NSS = "alpha.jobset.sigs.k8s.io/node-selector"
NSJOB = "alpha.jobset.sigs.k8s.io/namespaced-job"
NOSCHED = "alpha.jobset.sigs.k8s.io/no-schedule"
COMPLETION = "batch.kubernetes.io/job-completion-index"


def make_pod(name, ns="default", labels=None, annotations=None, node=None, owner=None, node_selector=None,
             has_node_selector=False):
    p = {"metadata": {"name": name, "namespace": ns, "labels": dict(labels or {}),
                      "annotations": dict(annotations or {})}, "spec": {}}
    if node:
        p["spec"]["nodeName"] = node
    if owner:
        p["metadata"]["ownerReferences"] = [{"uid": owner, "kind": "Job", "controller": True}]
    if node_selector is not None or has_node_selector:
        p["spec"]["nodeSelector"] = node_selector
    return p


# ------------------------------------------------------------------ golden vectors
@pytest.mark.parametrize("c", GOLD["jobHashKey"]["cases"], ids=lambda c: c["jobName"] or "empty")
def test_job_hash_key(c):
    assert host.jobHashKey(c["ns"], c["jobName"]) == c["want"]


@pytest.mark.parametrize("c", GOLD["sha1Hash"]["cases"], ids=lambda c: str(len(c["s"])))
def test_sha1(c):
    assert host.sha1Hash(c["s"]) == c["want"]


@pytest.mark.parametrize("c", GOLD["genLeaderPodName"]["cases"], ids=lambda c: c["desc"])
def test_leader_pod_name(c):
    got, err = host.genLeaderPodName(make_pod("pod", labels=c["labels"]))
    if c.get("wantErr"):
        assert err
    else:
        assert err is None and got == c["want"]


@pytest.mark.parametrize("c", GOLD["podsOwnedBySameJob"]["cases"], ids=lambda c: c["name"])
def test_pods_owned_by_same_job(c):
    leader = make_pod(c["leader"][0], owner=c["leader"][1] or None)
    follower = make_pod(c["follower"][0], owner=c["follower"][1] or None)
    assert host.podsOwnedBySameJob(leader, follower) == c["want"]


@pytest.mark.parametrize("c", GOLD["globalJobIndex"]["cases"], ids=lambda c: c["name"])
def test_global_job_index(c):
    js = {"spec": {"replicatedJobs": [{"name": n, "replicas": r} for n, r in c["rjobs"]]}}
    assert host.globalJobIndex(js, c["replicatedJob"], c["jobIdx"]) == c["want"]


def _placement_pods(g, c):
    ann = {JOBSET: "test-jobset", JOBIDX: "0", JOBKEY: g["jobKey"], EXCL: g["topologyKey"]}
    lab = {JOBSET: "test-jobset", RJOB: "replicated-job-1", JOBIDX: "0", JOBKEY: g["jobKey"]}
    leader = make_pod("test-jobset-replicated-job-1-test-job-0-0", labels=lab,
                      annotations={**ann, COMPLETION: "0"}, node="test-node")
    follower = make_pod("test-jobset-replicated-job-1-test-job-0-1", labels=lab, annotations={**ann, COMPLETION: "1"},
                        node_selector=c["followerNodeSelector"], has_node_selector=c["followerNodeSelector"] is not None)
    return leader, follower


@pytest.mark.parametrize("c", GOLD["validatePodPlacements"]["cases"], ids=lambda c: c["name"])
def test_validate_pod_placements(c):
    g = GOLD["validatePodPlacements"]
    leader, follower = _placement_pods(g, c)
    cache = host.Cache()
    if c["nodeLabels"] is not None:
        cache.add_node({"metadata": {"name": "test-node", "labels": c["nodeLabels"]}})
    if c.get("forceClientErr"):
        cache.inject("get/Node", c["forceClientErr"])
    matched, err = cache.validatePodPlacements(leader, [leader, follower])
    assert err == c["wantErr"]
    assert matched == c["wantMatched"]


@pytest.mark.parametrize("c", GOLD["deleteFollowerPods"]["cases"], ids=lambda c: c["name"])
def test_delete_follower_pods(c):
    leader = make_pod("test-jobset-replicated-job-1-test-job-0-0", annotations={COMPLETION: "0"}, node="test-node")
    follower = make_pod("test-jobset-replicated-job-1-test-job-0-1", annotations={COMPLETION: "1"})
    if c["followerCondition"]:
        follower["status"] = {"conditions": [{"type": "DisruptionTarget", "status": c["followerCondition"],
                                              "reason": "ExclusivePlacementViolation",
                                              "message": "Pod violated JobSet exclusive placement policy"}]}
    cache = host.Cache()
    cache.add_pod(leader)
    cache.add_pod(follower)
    if c.get("forceClientErr"):
        cache.inject("update/Pod", c["forceClientErr"])
        cache.inject("delete/Pod", c["forceClientErr"])
    err = cache.deleteFollowerPods([leader, follower])
    assert err == c.get("wantErr")
    assert len(cache.stats()["deleted"]) == c["wantDeleted"]


@pytest.mark.parametrize("c", GOLD["constructJobsFromTemplate"]["cases"], ids=lambda c: c["name"])
def test_construct_jobs_exclusive(c):
    """TestConstructJobsFromTemplate exclusive / node-selector cases: labels,
    annotations (A1 precedence), nodeSelector + toleration of the
    node-selector strategy, suspend, on both the Job and its pod template."""
    js = {"metadata": {"name": "test-jobset", "namespace": "default", "annotations": c["jobSetAnnotations"]},
          "spec": {"replicatedJobs": [], "network": {}}}
    for name, replicas, ann in c["rjobs"]:
        js["spec"]["replicatedJobs"].append({"name": name, "replicas": replicas, "template": {
            "metadata": {"name": "test-job", "namespace": "default", "annotations": ann or None},
            "spec": {"template": {"spec": {}}}}})
    got = []
    for rj in js["spec"]["replicatedJobs"]:
        got += host.constructJobsFromTemplate(js, rj, {})
    assert [j["metadata"]["name"] for j in got] == [w["name"] for w in c["want"]]
    for gidx, (job, w) in enumerate(zip(got, c["want"])):
        rj = "replicated-job-A" if "-A-" in w["name"] else "replicated-job-B"
        want_labels = {JOBSET: "test-jobset", RJOB: rj, REPL: "1", JOBIDX: "0", RESTARTS: "0",
                       JOBKEY: w["jobKey"], GIDX: str(gidx)}
        want_ann = dict(want_labels)
        if w["topology"]:
            want_ann[EXCL] = w["topology"]
            if w["nss"]:
                want_ann[NSS] = "true"
        for md in (job["metadata"], job["spec"]["template"]["metadata"]):
            assert md["labels"] == want_labels
            assert md["annotations"] == want_ann
        ps = job["spec"]["template"]["spec"]
        if w["nss"]:
            assert ps["nodeSelector"] == {NSJOB: w["namespacedJob"]}
            assert ps["tolerations"] == [{"key": NOSCHED, "operator": "Exists", "effect": "NoSchedule"}]
        else:
            assert "nodeSelector" not in ps and "tolerations" not in ps
        assert job["spec"]["suspend"] is False


def test_generate_namespaced_jobs():
    g = GOLD["generateNamespacedJobs"]
    assert host.generateNamespacedJobs(g["jobSet"]) == g["want"]
    for j, want in zip(range(3), g["want"]):
        assert host.namespacedJobName("default", host.GenJobName("exclusive-placement", "workers", j)) == want


# ------------------------------------------------------------------ placement utilities (placement.go:14-28)
def test_names_and_leader():
    assert host.GenJobName("js", "rj", 7) == "js-rj-7"
    assert host.GenPodName("js", "rj", "7", "0") == "js-rj-7-0"
    assert host.IsLeaderPod(make_pod("p", annotations={COMPLETION: "0"}))
    assert not host.IsLeaderPod(make_pod("p", annotations={COMPLETION: "1"}))
    assert not host.IsLeaderPod(make_pod("p"))


@pytest.mark.parametrize("name,want,err", [
    ("js-rj-0-0-abcde", "js-rj-0-0", None), ("my-js-rj-1-2-x1y2z", "my-js-rj-1-2", None),
    ("js-rj-0-abcde", None, "invalid pod name: js-rj-0-abcde"), ("", None, "invalid pod name: ")])
def test_remove_pod_name_suffix(name, want, err):
    got, e = host.removePodNameSuffix(name)
    assert e == err
    if want:
        assert got == want


def test_pod_indexes_only_for_exclusive_pods():
    """SetupPodIndexes, pod_controller.go:75-106 (A11)."""
    p = make_pod("js-rj-0-0-abcde", labels={JOBKEY: "k"}, annotations={EXCL: "rack"})
    assert host.podIndexes(p) == {"podName": ["js-rj-0-0"], "podJobKey": ["k"]}
    p2 = make_pod("js-rj-0-0-abcde", labels={JOBKEY: "k"})
    assert host.podIndexes(p2) == {"podName": [], "podJobKey": []}


def test_pod_predicate():
    """Leader ∧ scheduled ∧ exclusive ∧ not deleting (pod_controller.go:66-71)."""
    base = make_pod("p", annotations={COMPLETION: "0", EXCL: "rack"}, node="n1")
    assert host.podPredicate(base)
    assert not host.podPredicate(make_pod("p", annotations={COMPLETION: "0", EXCL: "rack"}))
    d = copy.deepcopy(base)
    d["metadata"]["deletionTimestamp"] = "2024-10-08T00:00:00Z"
    assert not host.podPredicate(d)


# ------------------------------------------------------------------ webhook (A4-A6)
def _job_pods(ns="default", js="js", rj="rj", idx=0, owner="uid-1", topo="rack", leader_node="node-a", n=3,
              extra_ann=None):
    job = f"{js}-{rj}-{idx}"
    key = host.jobHashKey(ns, job)
    lab = {JOBSET: js, RJOB: rj, JOBIDX: str(idx), JOBKEY: key}
    ann = {JOBSET: js, RJOB: rj, JOBIDX: str(idx), JOBKEY: key, EXCL: topo, **(extra_ann or {})}
    pods = []
    for i in range(n):
        pods.append(make_pod(f"{job}-{i}-abcde", ns=ns, labels=lab, annotations={**ann, COMPLETION: str(i)},
                             node=leader_node if i == 0 else None, owner=owner))
    return key, pods


def test_default_leader_gets_exclusive_affinities():
    """setExclusiveAffinities, pod_mutating_webhook.go:95-135 (A4): exactly two
    terms, in order, NamespaceSelector {} (all namespaces), appended."""
    key, pods = _job_pods()
    got, err = host.Cache().Default(pods[0])
    assert err is None
    aff = got["spec"]["affinity"]
    assert aff["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"] == [{
        "labelSelector": {"matchExpressions": [{"key": JOBKEY, "operator": "In", "values": [key]}]},
        "topologyKey": "rack", "namespaceSelector": {}}]
    assert aff["podAntiAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"] == [{
        "labelSelector": {"matchExpressions": [{"key": JOBKEY, "operator": "Exists"},
                                               {"key": JOBKEY, "operator": "NotIn", "values": [key]}]},
        "topologyKey": "rack", "namespaceSelector": {}}]
    again = host.setExclusiveAffinities(got)  # appends, never dedupes
    assert len(again["spec"]["affinity"]["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"]) == 2


def test_default_skips_non_exclusive_and_node_selector_strategy():
    _, pods = _job_pods(extra_ann={NSS: "true"})
    got, err = host.Cache().Default(pods[0])
    assert err is None and "affinity" not in got["spec"]
    p = make_pod("x", annotations={COMPLETION: "0"})
    assert host.Cache().Default(p) == (p, None)


def test_default_follower_pinned_to_leader_domain():
    """setNodeSelector, pod_mutating_webhook.go:137-171 (A5)."""
    _, pods = _job_pods()
    c = host.Cache()
    c.add_pod(pods[0])
    c.add_node({"metadata": {"name": "node-a", "labels": {"rack": "rack-7"}}})
    got, err = c.Default(pods[1])
    assert err is None and got["spec"]["nodeSelector"] == {"rack": "rack-7"}


def test_default_follower_edge_cases():
    _, pods = _job_pods()
    # leader lookup fails (no leader in the index) -> no mutation, no error (:140-145)
    got, err = host.Cache().Default(pods[1])
    assert err is None and "nodeSelector" not in got["spec"]
    # leader unbound -> no mutation (:148-151)
    _, unbound = _job_pods(leader_node=None)
    c = host.Cache()
    c.add_pod(unbound[0])
    got, err = c.Default(unbound[1])
    assert err is None and "nodeSelector" not in got["spec"]
    # node NotFound -> value "" with nil error (:181-186 -> :169)
    c = host.Cache()
    c.add_pod(pods[0])
    got, err = c.Default(pods[1])
    assert err is None and got["spec"]["nodeSelector"] == {"rack": ""}
    # node lacks the topology label -> error (:189-192)
    c.add_node({"metadata": {"name": "node-a", "labels": {"zone": "z"}}})
    got, err = c.Default(pods[1])
    assert err == "node does not have topology label: rack"
    # stale index entry from the previous restart: owner UID differs -> no mutation (A5 race guard)
    _, old = _job_pods(owner="uid-old")
    c = host.Cache()
    c.add_pod(old[0])
    c.add_node({"metadata": {"name": "node-a", "labels": {"rack": "rack-7"}}})
    got, err = c.Default(pods[1])
    assert err is None and "nodeSelector" not in got["spec"]


def test_validate_create():
    """ValidateCreate, pod_admission_webhook.go:24-67 (A6)."""
    _, pods = _job_pods()
    c = host.Cache()
    assert c.ValidateCreate(make_pod("not-a-jobset-pod")) is None
    assert c.ValidateCreate(pods[0]) is None  # leaders pass
    assert c.ValidateCreate(pods[1]) == "follower pod node selector not set"
    f = copy.deepcopy(pods[1])
    f["spec"]["nodeSelector"] = {"zone": "z"}
    assert c.ValidateCreate(f) == ("follower pod node selector for topology domain not found. "
                                   "missing selector: rack")
    f["spec"]["nodeSelector"] = {"rack": "rack-7"}
    assert c.ValidateCreate(f) == ("expected 1 leader pod (js-rj-0-0), but got 0. this is an expected, "
                                   "transient error")
    _, unbound = _job_pods(leader_node=None)
    c.add_pod(unbound[0])
    assert c.ValidateCreate(f) == ("leader pod not yet scheduled, not creating follower pod. this is an "
                                   "expected, transient error")
    c2 = host.Cache()
    c2.add_pod(pods[0])
    assert c2.ValidateCreate(f) is None
    _, nss = _job_pods(extra_ann={NSS: "true"})
    assert host.Cache().ValidateCreate(nss[1]) is None


# ------------------------------------------------------------------ PodReconciler (A9) + recreate (A10)
def test_reconcile_mismatch_is_error_not_delete():
    """Reconcile returns on validatePodPlacements' error before its !valid
    branch (pod_controller.go:148-155): a mismatch requeues, nothing is deleted."""
    _, pods = _job_pods()
    c = host.Cache()
    c.add_node({"metadata": {"name": "node-a", "labels": {"rack": "rack-7"}}})
    leader, f1, f2 = pods
    f1["spec"]["nodeSelector"] = {"rack": "rack-7"}
    f2["spec"]["nodeSelector"] = {"rack": "rack-9"}
    for p in (leader, f1, f2):
        c.add_pod(p)
    assert c.Reconcile("default", leader["metadata"]["name"]) == ('follower topology "rack-9" != leader '
                                                                  'topology "rack-7"')
    assert c.stats()["deleted"] == []
    f2["spec"]["nodeSelector"] = {"rack": "rack-7"}
    c.add_pod(f2)
    assert c.Reconcile("default", leader["metadata"]["name"]) is None
    assert c.Reconcile("default", "gone") is None  # NotFound is ignored
    nokey = make_pod("x-y-0-0-abcde", annotations={COMPLETION: "0", EXCL: "rack"}, node="node-a")
    c.add_pod(nokey)
    assert c.Reconcile("default", "x-y-0-0-abcde") == 'job key label not found on leader pod: "x-y-0-0-abcde"'


def test_update_pod_condition():
    """updatePodCondition, pod_controller.go:309-327."""
    cond = {"type": "DisruptionTarget", "status": "True", "reason": "r", "message": "m"}
    changed, p = host.updatePodCondition(make_pod("p"), cond)
    assert changed and p["status"]["conditions"] == [cond]
    changed, p = host.updatePodCondition(p, cond)
    assert not changed
    changed, p = host.updatePodCondition(p, {**cond, "status": "False"})
    assert changed and p["status"]["conditions"][0]["status"] == "False"
    changed, _ = host.updatePodCondition(make_pod("q"), {**cond, "status": "False"})
    assert not changed


def test_recreate_all_flow():
    """Full-JobSet recovery (A10): failurePolicyRecreateAll bumps restarts
    (failure_policy.go:155-175); getChildJobs moves older attempts to delete
    (jobset_controller.go:281-290); shouldCreateJob refuses while the old Job
    is still listed (:698-709), then the new attempt is constructed with the
    new restart-attempt label."""
    js = {"metadata": {"name": "js", "namespace": "default", "annotations": {EXCL: "rack"}},
          "spec": {"replicatedJobs": [{"name": "rj", "replicas": 2, "template": {"spec": {"template": {}}}}],
                   "network": {}},
          "status": {"restarts": 0}}
    jobs = host.constructJobsFromTemplate(js, js["spec"]["replicatedJobs"][0], {})
    assert [j["metadata"]["labels"][RESTARTS] for j in jobs] == ["0", "0"]
    jobs[1]["status"] = {"conditions": [{"type": "Failed", "status": "True"}]}
    owned, err = host.getChildJobs(js, jobs)
    assert err is None and [j["metadata"]["name"] for j in owned["failed"]] == ["js-rj-1"]
    js2 = host.failurePolicyRecreateAll(js, True)
    assert js2["status"]["restarts"] == 1 and js2["status"]["restartsCountTowardsMax"] == 1
    owned, err = host.getChildJobs(js2, jobs)
    assert err is None and len(owned["delete"]) == 2 and owned["active"] == []
    assert not host.shouldCreateJob("js-rj-0", owned)
    assert host.constructJobsFromTemplate(js2, js2["spec"]["replicatedJobs"][0], owned) == []
    new = host.constructJobsFromTemplate(js2, js2["spec"]["replicatedJobs"][0], {})
    assert [j["metadata"]["labels"][RESTARTS] for j in new] == ["1", "1"]
    assert new[0]["metadata"]["labels"][JOBKEY] == jobs[0]["metadata"]["labels"][JOBKEY]  # same job key
    bad = [dict(jobs[0], metadata={**jobs[0]["metadata"], "labels": {RESTARTS: "x"}})]
    _, err = host.getChildJobs(js2, bad)
    assert err == 'strconv.Atoi: parsing "x": invalid syntax'
    js3 = host.failurePolicyRecreateAll(js2, False)
    assert js3["status"]["restarts"] == 2 and js3["status"]["restartsCountTowardsMax"] == 1


def test_label_and_annotate_precedence_and_coordinator():
    """A1: ReplicatedJob-level exclusive annotation overrides JobSet-level;
    node-selector flag comes only from the level that set the key."""
    js = {"metadata": {"name": "js", "namespace": "ns", "annotations": {EXCL: "zone", NSS: "true"}},
          "spec": {"replicatedJobs": [{"name": "a", "replicas": 1,
                                       "template": {"metadata": {"annotations": {EXCL: "rack"}}}}],
                   "network": {"subdomain": "sd"},
                   "coordinator": {"replicatedJob": "a", "jobIndex": 0, "podIndex": 0}}}
    job = host.constructJob(js, js["spec"]["replicatedJobs"][0], 0)
    ann = job["metadata"]["annotations"]
    assert ann[EXCL] == "rack" and ann[NSS] == "true"  # NSS from the JobSet level, key overridden
    assert ann["jobset.sigs.k8s.io/coordinator"] == "js-a-0-0.sd"


def test_bad_method_and_json():
    with pytest.raises(host.HostCallError):
        host.call("no.such.method")
