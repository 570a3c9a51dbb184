"""Kubernetes-object fixtures for the ingestion tests: a synthetic Problem
(jobset_amd.synth) restated as the Node, bound Pod and child Job objects an
informer cache would hold, such that ingesting them reproduces the problem.

  label bit b        -> node label  b<bbb>="1"; a class's required bit -> its
                        nodeSelector, a forbidden bit -> matchExpressions NotIn ["1"]
  taint bit t        -> node taint  t<tt>:NoSchedule; a tolerated bit -> toleration
                        {key: t<tt>, operator: Exists, effect: NoSchedule}
  free[r]            -> status.allocatable r<r> (a non-cpu/memory name: whole units)
  excl (a domain)    -> one bound pod on a node of that domain carrying the
                        exclusive-topology annotation at that level and a job-key
  domain d, level k  -> node label level-<k>="<k>-<d:06d>" (sorted = id order)

Domains without nodes do not exist as Kubernetes objects; they are never
feasible, so placements compare by domain value.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from jobset_amd.snapshot import Problem

EXCL = "alpha.jobset.sigs.k8s.io/exclusive-topology"
JOBKEY = "jobset.sigs.k8s.io/job-key"
RJOB = "jobset.sigs.k8s.io/replicatedjob-name"


def level_key(k: int) -> str:
    return f"level-{k}"


def domain_value(k: int, d: int) -> str:
    return f"{k}-{d:06d}"


def res_names(R: int) -> List[str]:
    return [f"r{r}" for r in range(R)]


def node_objects(p: Problem) -> Tuple[List[dict], List[dict]]:
    topo, nodes = p.topology, p.nodes
    K, N, W, R = topo.n_levels, nodes.n_nodes, nodes.n_label_words, nodes.n_res
    leaf = nodes.leaf_of_row()
    dom = [topo.parent_of_leaf(k)[leaf] if N else np.zeros(0, dtype=np.int64) for k in range(K)]
    out, pods = [], []
    for i in range(N):
        lab = {level_key(k): domain_value(k, int(dom[k][i])) for k in range(K)}
        for w in range(W):
            x = int(nodes.labels[w, i])
            while x:
                b = (x & -x).bit_length() - 1
                x &= x - 1
                lab[f"b{64 * w + b:03d}"] = "1"
        taints = [{"key": f"t{t:02d}", "value": "", "effect": "NoSchedule"}
                  for t in range(32) if (int(nodes.taints[i]) >> t) & 1]
        alloc = {res_names(R)[r]: str(int(nodes.free[r, i])) for r in range(R)}
        out.append({"metadata": {"name": f"n{i:08d}", "labels": lab},
                    "spec": {"taints": taints}, "status": {"allocatable": alloc}})
    # exclusive occupancy: the covered rows are whole leaves (excl marks whole
    # domains); one marker pod per covered leaf, exclusive at the leaf level
    for l in range(nodes.n_leaves):
        a, e = int(nodes.leaf_start[l]), int(nodes.leaf_start[l + 1])
        if a < e and (nodes.excl[a:e] != -1).all():
            pods.append({"metadata": {"name": f"owner-{l}", "namespace": "other",
                                      "labels": {JOBKEY: f"key-{int(nodes.excl[a])}"},
                                      "annotations": {EXCL: level_key(K - 1)}},
                         "spec": {"nodeName": f"n{a:08d}", "containers": [{"name": "c"}]},
                         "status": {"phase": "Running"}})
        elif a < e and (nodes.excl[a:e] != -1).any():
            raise ValueError("excl does not cover whole leaves")
    return out, pods


def job_objects(p: Problem) -> List[dict]:
    """One child Job per problem job, in global order; class c = replicatedJob class<c>."""
    W, R = p.nodes.n_label_words, p.nodes.n_res
    templates = []
    for jc in p.classes:
        req, fb = jc.words(4)
        sel, exprs = {}, []
        for w in range(W):
            for b in range(64):
                if (req[w] >> b) & 1:
                    sel[f"b{64 * w + b:03d}"] = "1"
                if (fb[w] >> b) & 1:
                    exprs.append({"key": f"b{64 * w + b:03d}", "operator": "NotIn", "values": ["1"]})
        spec = {"containers": [{"name": "c", "resources": {"requests": {
            res_names(R)[r]: str(v) for r, v in enumerate(jc.res()[:R]) if v > 0}}}]}
        if sel:
            spec["nodeSelector"] = sel
        if exprs:
            spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchExpressions": exprs}]}}}
        tol = [{"key": f"t{t:02d}", "operator": "Exists", "effect": "NoSchedule"}
               for t in range(32) if (jc.tolerated_taints >> t) & 1]
        if tol:
            spec["tolerations"] = tol
        templates.append((jc.level, jc.pods, spec))
    jobs = []
    for j, c in enumerate(p.job_class.tolist()):
        level, pods, spec = templates[c]
        jobs.append({"metadata": {"name": f"job-{j:06d}", "namespace": "default",
                                  "labels": {RJOB: f"class{c}"}, "annotations": {EXCL: level_key(level)}},
                     "spec": {"parallelism": pods, "template": {"spec": spec}}})
    return jobs


def load_cache(cache, p: Problem) -> None:
    nodes, pods = node_objects(p)
    for n in nodes:
        cache.add_node(n)
    for q in pods:
        cache.add_pod(q)


def problem_from_planner(p: Problem, cols: dict, enc: dict) -> Problem:
    """The Problem the planner's snapshot and encoded classes describe."""
    from jobset_amd.snapshot import JobClass, Nodes, Topology
    K = len(cols["firstLeaf"])
    fl = [np.array(x, dtype=np.uint32) for x in cols["firstLeaf"]]
    topo = Topology(level_keys=[level_key(k) for k in range(K)], n_domains=[len(x) - 1 for x in fl], first_leaf=fl,
                    domain_values=cols["domainValues"])
    N = len(cols["rows"])
    W = len(cols["labels"][0]) if N else 1
    labels = np.array([[int(cols["labels"][i][w], 16) for i in range(N)] for w in range(W)], dtype=np.uint64)
    nodes = Nodes(leaf_start=np.array(cols["leafStart"], dtype=np.uint32), labels=labels.reshape(W, N),
                  taints=np.array(cols["taints"], dtype=np.uint32),
                  free=np.array(cols["free"], dtype=np.uint32).T.reshape(-1, N) if N else np.zeros((p.nodes.n_res, 0),
                                                                                                    dtype=np.uint32),
                  excl=np.array(cols["excl"], dtype=np.int32))
    classes = [JobClass(req_labels=tuple(int(x, 16) for x in c["reqLabels"]),
                        forbid_labels=tuple(int(x, 16) for x in c["forbidLabels"]),
                        tolerated_taints=c["toleratedTaints"], level=c["level"], pods=c["pods"],
                        req_res=tuple(c["reqRes"])) for c in enc["classes"]]
    return Problem(topology=topo, nodes=nodes, classes=classes,
                   job_class=np.array(enc["jobClass"], dtype=np.uint32))


def leaf_values(p: Problem) -> List[str]:
    K = p.topology.n_levels
    return [domain_value(K - 1, d) for d in range(p.topology.n_leaves)]


def assign_values(p: Problem, assign: np.ndarray, values: Dict[int, List[str]] = None) -> List:
    """Placements as domain values (None = unplaceable)."""
    out = []
    for j, d in enumerate(assign.tolist()):
        if d < 0:
            out.append(None)
        else:
            lvl = p.classes[int(p.job_class[j])].level
            out.append(values[lvl][d] if values is not None else domain_value(lvl, d))
    return out
