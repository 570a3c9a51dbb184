"""CPU tests of snapshot ingestion (jobset_amd/csrc/host/placement.cc, SURVEY.md
§8f row 1) with a host-only planner (no engine): Kubernetes Node / bound Pod /
Job objects -> the engine's SoA snapshot and requirement classes. The
restated objects of a synthetic problem (tests/k8s_fixtures.py) must give the
oracle the same placements (by domain value) and the same per-leaf
capacities and occupancy as the problem itself."""
import numpy as np
import pytest

from jobset_amd import host, synth
from oracle import oracle as O

import k8s_fixtures as K


def ingest(p):
    c = host.Cache()
    K.load_cache(c, p)
    c.planner_new(None, [K.level_key(k) for k in range(p.topology.n_levels)], K.res_names(p.nodes.n_res))
    enc = c.planner_encode(K.job_objects(p))
    cols = c.planner_columns()
    return c, cols, enc


def check_equivalent(p):
    c, cols, enc = ingest(p)
    q = K.problem_from_planner(p, cols, enc)
    a, cap, occ = O.place_c(p)
    b, cap2, occ2 = O.place_c(q)
    vals = {k: v for k, v in enumerate(cols["domainValues"])}
    assert K.assign_values(p, a) == K.assign_values(q, b, vals)
    # per-leaf tallies of the leaves that have nodes, for the classes jobs use
    # (planner class i = the class of the first job encoded as i)
    orig = {}
    for jc, pc in zip(p.job_class.tolist(), enc["jobClass"]):
        orig.setdefault(pc, jc)
    leaf_of = {v: i for i, v in enumerate(K.leaf_values(p))}
    for j, v in enumerate(cols["domainValues"][-1]):
        for pc, oc in orig.items():
            assert cap2[pc, j] == cap[oc, leaf_of[v]]
        assert occ2[j] == occ[leaf_of[v]]
    return cols


@pytest.mark.parametrize("seed", range(30))
def test_ingest_random_problem(seed):
    check_equivalent(synth.random_problem(seed, max_nodes=1500, max_leaves=80))


@pytest.mark.parametrize("cfg", [1, 2, 5])
def test_ingest_configs(cfg):
    cols = check_equivalent(synth.CONFIGS[cfg]())
    assert len(cols["rows"]) == synth.CONFIGS[cfg]().nodes.n_nodes


def test_dictionaries_sorted_and_deterministic():
    """Bits are ranks in the sorted predicate / taint dictionaries, whatever
    the order objects arrived in."""
    p = synth.random_problem(7, max_nodes=500, max_leaves=30)
    nodes, pods = K.node_objects(p)
    out = []
    for order in (1, -1):
        c = host.Cache()
        for n in nodes[::order]:
            c.add_node(n)
        for q in pods[::order]:
            c.add_pod(q)
        c.planner_new(None, [K.level_key(k) for k in range(p.topology.n_levels)], K.res_names(p.nodes.n_res))
        c.planner_encode(K.job_objects(p))
        out.append(c.planner_columns())
    assert out[0] == out[1]
    keys = [(x["key"], x["op"], x["values"]) for x in out[0]["predicates"]]
    assert keys == sorted(keys)
    assert [t["key"] for t in out[0]["taintKeys"]] == sorted(t["key"] for t in out[0]["taintKeys"])


def node(name, labels, taints=(), alloc=None, unschedulable=False):
    spec = {"taints": list(taints)}
    if unschedulable:
        spec["unschedulable"] = True
    return {"metadata": {"name": name, "labels": labels}, "spec": spec,
            "status": {"allocatable": alloc or {"cpu": "96", "memory": "1536000Mi", "amd.com/gpu": "8"}}}


def job(name, key, spec, parallelism=1, rj="w"):
    return {"metadata": {"name": name, "namespace": "default",
                         "labels": {K.RJOB: rj}, "annotations": {K.EXCL: key}},
            "spec": {"parallelism": parallelism, "template": {"spec": spec}}}


def test_selector_operators_and_taint_semantics():
    """In with several values, NotIn, Exists, DoesNotExist, Gt/Lt as node-label
    predicates; tolerations by kube's ToleratesTaint; spec.unschedulable as the
    node.kubernetes.io/unschedulable:NoSchedule taint; PreferNoSchedule ignored."""
    c = host.Cache()
    c.add_node(node("a", {"rack": "r1", "gpu": "mi355x", "gen": "4"}))
    c.add_node(node("b", {"rack": "r2", "gpu": "mi300x", "gen": "3", "spot": "true"}))
    c.add_node(node("c", {"rack": "r3", "gpu": "mi355x", "gen": "5"},
                    taints=[{"key": "dedicated", "value": "ml", "effect": "NoSchedule"},
                            {"key": "soft", "value": "", "effect": "PreferNoSchedule"}]))
    c.add_node(node("d", {"rack": "r4", "gpu": "mi355x", "gen": "5"}, unschedulable=True))
    c.planner_new(None, ["rack"], ["cpu", "memory", "amd.com/gpu"])
    aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [{
        "matchExpressions": [{"key": "gpu", "operator": "In", "values": ["mi355x", "mi300x"]},
                             {"key": "spot", "operator": "DoesNotExist"},
                             {"key": "gen", "operator": "Gt", "values": ["3"]}]}]}}}
    specs = [{"affinity": aff},
             {"affinity": aff, "tolerations": [{"key": "dedicated", "operator": "Equal", "value": "ml"}]},
             {"affinity": aff, "tolerations": [{"operator": "Exists"}]},
             {"nodeSelector": {"gpu": "mi300x"}}]
    jobs = [job(f"j{i}", "rack", s, rj=f"rj{i}") for i, s in enumerate(specs)]
    enc = c.planner_encode(jobs)
    cols = c.planner_columns()
    q = K.problem_from_planner(synth.config1(), cols, enc)
    cap, occ = O.place_c(q)[1:]
    feasible = (cap > 0)  # one pod per job, no requests: node-level predicate result
    # rows a, b, c, d (sorted by rack)
    np.testing.assert_array_equal(feasible, [[True, False, False, False],    # c tainted, d unschedulable, b spot
                                             [True, False, True, False],     # tolerates dedicated=ml
                                             [True, False, True, True],      # tolerates everything
                                             [False, True, False, False]])   # nodeSelector gpu=mi300x
    assert [t["key"] for t in cols["taintKeys"]] == ["dedicated", "node.kubernetes.io/unschedulable"]


def test_resources_requests_and_quantities():
    """allocatable - requests of bound non-terminal pods, per resource unit:
    cpu millicores (requests round up), memory MiB, others whole units; the
    effective request is max(sum of containers, max of init containers)."""
    c = host.Cache()
    c.add_node(node("a", {"rack": "r1"}, alloc={"cpu": "95500m", "memory": "1.5Ti", "amd.com/gpu": "8"}))
    pod = {"metadata": {"name": "p", "namespace": "x"},
           "spec": {"nodeName": "a",
                    "containers": [{"name": "a", "resources": {"requests": {"cpu": "1.2", "memory": "1Gi"}}},
                                   {"name": "b", "resources": {"requests": {"cpu": "300m", "amd.com/gpu": "2"}}}],
                    "initContainers": [{"name": "i", "resources": {"requests": {"cpu": "4", "memory": "100M"}}}]},
           "status": {"phase": "Running"}}
    done = {"metadata": {"name": "q", "namespace": "x"},
            "spec": {"nodeName": "a", "containers": [{"name": "a", "resources": {"requests": {"cpu": "90"}}}]},
            "status": {"phase": "Succeeded"}}
    c.add_pod(pod)
    c.add_pod(done)
    c.planner_new(None, ["rack"], ["cpu", "memory", "amd.com/gpu"])
    cols = c.planner_columns()
    # cpu: 95500 - max(1200 + 300, 4000) = 91500; memory: 1.5 TiB = 1572864 MiB - max(1024, ceil(95.37)) = 1571840
    assert cols["free"] == [[91500, 1571840, 6]]
    c.remove_pod("x", "p")
    assert c.planner_columns()["free"] == [[95500, 1572864, 8]]


def test_non_nested_keys_and_skipped_nodes():
    c = host.Cache()
    c.add_node(node("a", {"zone": "z1", "rack": "r1"}))
    c.add_node(node("b", {"zone": "z2", "rack": "r1"}))  # rack r1 under two zones
    c.add_node(node("c", {"zone": "z2"}))                # no rack label: not in the snapshot
    c.planner_new(None, ["zone", "rack"], ["cpu"])
    with pytest.raises(host.HostCallError, match="spans several zone domains"):
        c.planner_sync()
    c.remove_node("b")
    st = c.planner_sync()
    assert st["skippedNodes"] == ["c"] and st["rows"] == 1


def test_unsupported_selectors_are_errors():
    c = host.Cache()
    c.add_node(node("a", {"rack": "r1"}))
    c.planner_new(None, ["rack"], ["cpu"])
    two_terms = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": "x", "operator": "Exists"}]},
        {"matchExpressions": [{"key": "y", "operator": "Exists"}]}]}}}
    with pytest.raises(host.HostCallError, match="ORed terms"):
        c.planner_encode([job("j", "rack", {"affinity": two_terms})])
    with pytest.raises(host.HostCallError, match="not one of the engine's topology keys"):
        c.planner_encode([job("j", "zone", {})])


def test_reconcile_recreate_without_engine():
    """controllers.reconcileRecreate's Job side (no planner bound): old attempt
    listed -> delete only; gone -> the new attempt's Jobs, unchanged."""
    js = {"metadata": {"name": "train", "namespace": "default", "annotations": {
        "alpha.jobset.sigs.k8s.io/exclusive-topology": "rack"}},
        "spec": {"network": {}, "replicatedJobs": [
            {"name": "a", "replicas": 2, "template": {"spec": {"parallelism": 2, "template": {"spec": {}}}}},
            {"name": "b", "replicas": 1, "template": {"spec": {"parallelism": 1, "template": {"spec": {}}}}}]},
        "status": {"restarts": 0}}
    c = host.Cache()
    jobs = sum((host.constructJobsFromTemplate(js, rj, {}) for rj in js["spec"]["replicatedJobs"]), [])
    js1 = host.failurePolicyRecreateAll(js, True)
    out, err = c.reconcileRecreate(js1, jobs)
    assert err is None and out["delete"] == ["train-a-0", "train-a-1", "train-b-0"] and out["create"] == []
    out, err = c.reconcileRecreate(js1, [])
    want = sum((host.constructJobsFromTemplate(js1, rj, {}) for rj in js1["spec"]["replicatedJobs"]), [])
    assert err is None and out["delete"] == [] and out["create"] == want and out["plan"] is None
    assert [j["metadata"]["labels"]["jobset.sigs.k8s.io/restart-attempt"] for j in want] == ["1", "1", "1"]
