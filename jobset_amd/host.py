"""Python face of the host-side mirror (include/jsk_host.h): the reference's
pod webhook, leader PodReconciler, child-Job construction and placement
utilities, with the Go function names. Each call goes through the C ABI into
jobset_amd/csrc/host/jobset_host.cc; objects are Kubernetes JSON dicts.
"""
from __future__ import annotations

import ctypes
import json
from typing import Any, Dict, List, Optional, Tuple

from . import native

_bound = False


def _lib():
    global _bound
    lib = native.lib()
    if not _bound:
        lib.jsk_call.restype = ctypes.c_int
        lib.jsk_call.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        lib.jsk_free.restype = None
        lib.jsk_free.argtypes = [ctypes.c_void_p]
        _bound = True
    return lib


class HostCallError(RuntimeError):
    pass


def call(method: str, **req: Any) -> Tuple[Any, Optional[str]]:
    """Returns (result, go_error_text_or_None)."""
    lib = _lib()
    out = ctypes.c_void_p()
    rc = lib.jsk_call(method.encode(), json.dumps(req).encode(), ctypes.byref(out))
    try:
        text = ctypes.string_at(out.value).decode() if out.value else "{}"
    finally:
        if out.value:
            lib.jsk_free(out.value)
    resp = json.loads(text)
    if rc != 0:
        raise HostCallError(resp.get("error", f"jsk_call rc={rc}"))
    return resp.get("result"), resp.get("error")


# ---------------------------------------------------------------- stateless helpers
def GenJobName(js: str, rjob: str, idx: int) -> str:
    return call("placement.GenJobName", jsName=js, rjobName=rjob, jobIndex=idx)[0]


def GenPodName(js: str, rjob: str, job_idx: str, pod_idx: str) -> str:
    return call("placement.GenPodName", jobSet=js, replicatedJob=rjob, jobIndex=job_idx, podIndex=pod_idx)[0]


def IsLeaderPod(pod: dict) -> bool:
    return call("placement.IsLeaderPod", pod=pod)[0]


def jobHashKey(ns: str, job: str) -> str:
    return call("controllers.jobHashKey", ns=ns, jobName=job)[0]


def sha1Hash(s: str) -> str:
    return call("controllers.sha1Hash", s=s)[0]


def namespacedJobName(ns: str, job: str) -> str:
    return call("controllers.namespacedJobName", ns=ns, jobName=job)[0]


def globalJobIndex(js: dict, rjob: str, idx: int) -> str:
    return call("controllers.globalJobIndex", jobSet=js, replicatedJob=rjob, jobIdx=idx)[0]


def removePodNameSuffix(name: str):
    return call("controllers.removePodNameSuffix", podName=name)


def constructJob(js: dict, rjob: dict, idx: int) -> dict:
    return call("controllers.constructJob", jobSet=js, replicatedJob=rjob, jobIdx=idx)[0]


def constructJobsFromTemplate(js: dict, rjob: dict, owned: Optional[dict] = None) -> List[dict]:
    return call("controllers.constructJobsFromTemplate", jobSet=js, replicatedJob=rjob, ownedJobs=owned or {})[0]


def shouldCreateJob(name: str, owned: dict) -> bool:
    return call("controllers.shouldCreateJob", jobName=name, ownedJobs=owned)[0]


def getChildJobs(js: dict, jobs: List[dict]):
    return call("controllers.getChildJobs", jobSet=js, jobs=jobs)


def failurePolicyRecreateAll(js: dict, should_count: bool) -> dict:
    return call("controllers.failurePolicyRecreateAll", jobSet=js, shouldCountTowardsMax=should_count)[0]


def followerPodTopology(pod: dict, key: str):
    return call("controllers.followerPodTopology", pod=pod, topologyKey=key)


def updatePodCondition(pod: dict, cond: dict):
    r = call("controllers.updatePodCondition", pod=pod, condition=cond)[0]
    return r["changed"], r["pod"]


def podIndexes(pod: dict) -> Dict[str, List[str]]:
    return call("controllers.podIndexes", pod=pod)[0]


def podPredicate(pod: dict) -> bool:
    return call("controllers.podPredicate", pod=pod)[0]


def genLeaderPodName(pod: dict):
    return call("webhooks.genLeaderPodName", pod=pod)


def podsOwnedBySameJob(leader: dict, follower: dict) -> Optional[str]:
    return call("webhooks.podsOwnedBySameJob", leaderPod=leader, followerPod=follower)[1]


def setExclusiveAffinities(pod: dict) -> dict:
    return call("webhooks.setExclusiveAffinities", pod=pod)[0]


def generateNamespacedJobs(js: dict) -> List[str]:
    return call("hack.generateNamespacedJobs", jobSet=js)[0]


# ---------------------------------------------------------------- cached client + webhook/reconciler
class Cache:
    """The controller-runtime cached client the webhook and reconciler read
    (pods with the podName / podJobKey field indexes, nodes), with
    injectable errors like the reference tests' interceptor.Funcs."""

    def __init__(self):
        self.id = call("cache.new")[0]

    def close(self):
        if self.id is not None:
            call("cache.free", cache=self.id)
            self.id = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_pod(self, pod: dict):
        call("cache.add", cache=self.id, kind="Pod", object=pod)

    def add_node(self, node: dict):
        call("cache.add", cache=self.id, kind="Node", object=node)

    def inject(self, what: str, error: Optional[str]):
        """what: "get/Node", "get/Pod", "list/Pod", "update/Pod" (status), "delete/Pod"."""
        call("cache.inject", cache=self.id, what=what, error=error)

    def stats(self) -> dict:
        return call("cache.stats", cache=self.id)[0]

    def bind_engine(self, engine, node_rows: Dict[str, int], level_keys: List[str], domain_values: List[List[str]]):
        """Answer topologyFromPod from the engine's resident snapshot."""
        call("cache.bindEngine", cache=self.id, engine=engine._h.value, nodeRows=node_rows, levelKeys=level_keys,
             domainValues=domain_values)

    # webhook (pkg/webhooks)
    def Default(self, pod: dict):
        return call("webhooks.Default", cache=self.id, pod=pod)

    def ValidateCreate(self, pod: dict) -> Optional[str]:
        return call("webhooks.ValidateCreate", cache=self.id, pod=pod)[1]

    def leaderPodForFollower(self, pod: dict):
        return call("webhooks.leaderPodForFollower", cache=self.id, pod=pod)

    # PodReconciler (pkg/controllers/pod_controller.go)
    def validatePodPlacements(self, leader: dict, pods: List[dict]):
        return call("controllers.validatePodPlacements", cache=self.id, leaderPod=leader, podList=pods)

    def deleteFollowerPods(self, pods: List[dict], now: str = "2024-10-08T00:00:00Z") -> Optional[str]:
        return call("controllers.deleteFollowerPods", cache=self.id, pods=pods, now=now)[1]

    def Reconcile(self, ns: str, name: str, now: str = "2024-10-08T00:00:00Z") -> Optional[str]:
        return call("controllers.Reconcile", cache=self.id, namespace=ns, name=name, now=now)[1]

    def remove_pod(self, ns: str, name: str):
        call("cache.remove", cache=self.id, kind="Pod", namespace=ns, name=name)

    def remove_node(self, name: str):
        call("cache.remove", cache=self.id, kind="Node", name=name)

    # placement planner (jobset_amd/csrc/host/placement.h): the engine's snapshot
    # built from this cache's Node / Pod objects
    def planner_new(self, engine, level_keys: List[str], resources: List[str]):
        """engine=None: a host-only planner (ingestion without uploads)."""
        call("planner.new", cache=self.id, engine=engine._h.value if engine is not None else 0,
             levelKeys=level_keys, resources=resources)

    def _ok(self, method: str, **req):
        r, e = call(method, cache=self.id, **req)
        if e is not None:
            raise HostCallError(e)
        return r

    def planner_sync(self) -> dict:
        return self._ok("planner.sync")

    def planner_columns(self) -> dict:
        return self._ok("planner.columns")

    def planner_encode(self, jobs: List[dict]) -> dict:
        return self._ok("planner.encode", jobs=jobs)

    def plan(self, jobs: List[dict]):
        return call("planner.plan", cache=self.id, jobs=jobs)

    def reconcileRecreate(self, js: dict, jobs: List[dict]):
        return call("controllers.reconcileRecreate", cache=self.id, jobSet=js, jobs=jobs)

    def labelNodes(self, js: dict):
        return call("hack.labelNodes", cache=self.id, jobSet=js)

    def DefaultBatch(self, pods: List[dict]) -> List[Tuple[dict, Optional[str]]]:
        r = call("webhooks.DefaultBatch", cache=self.id, pods=pods)[0]
        return [(x["pod"], x["error"]) for x in r]
