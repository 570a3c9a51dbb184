"""Cluster-snapshot data model of the exclusive-placement engine.

The engine sees the node informer cache as an in-memory snapshot (SURVEY.md
§8a rows A5/A8): nodes sorted by their finest topology domain (the "leaf",
e.g. a rack) so that every domain at every level is a contiguous row range,
with SoA columns that stream coalesced from HBM:

  labels  uint64 [W, N]   interned (key, value) node-label bits
  taints  uint32 [N]      interned NoSchedule / NoExecute taint bits
  free    uint32 [R, N]   allocatable - requested, per resource
  excl    int32  [N]      id of the exclusive job whose domain covers the row, -1 none

Job requirement classes (a deduplicated {nodeSelector, required node affinity,
tolerations, per-pod request, pods/job, topologyKey} tuple) carry bit masks
over the same dictionaries. The dictionaries are sorted, so the bit assignment
is deterministic (SURVEY.md §7 "String->bit encoding").

Reference anchors: the topologyKey is the value of the exclusive-topology
annotation (api/jobset/v1alpha2/jobset_types.go:41) copied onto every Job and
pod template by labelAndAnnotateObject (pkg/controllers/jobset_controller.go:
751-766); a domain value is node.Labels[topologyKey]
(pkg/webhooks/pod_mutating_webhook.go:189, pkg/controllers/pod_controller.go:258).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

MAX_LEVELS = 4
MAX_LABEL_WORDS = 4
MAX_RES = 4
MAX_CLASSES = 64

TAINT_EFFECTS = ("NoSchedule", "NoExecute")  # PreferNoSchedule is a soft preference: not a predicate


@dataclass
class Topology:
    """Nested domain hierarchy, level 0 = coarsest .. K-1 = finest ("leaf")."""

    level_keys: List[str]
    n_domains: List[int]
    # first_leaf[k]: uint32 [D_k + 1] leaf range of each level-k domain; the
    # finest level is the identity range.
    first_leaf: List[np.ndarray]
    # Label values of each domain per level (node.Labels[level_keys[k]]).
    domain_values: Optional[List[List[str]]] = None

    @property
    def n_levels(self) -> int:
        return len(self.level_keys)

    @property
    def n_leaves(self) -> int:
        return self.n_domains[-1]

    def validate(self) -> None:
        K = self.n_levels
        if not 1 <= K <= MAX_LEVELS:
            raise ValueError(f"n_levels {K} out of range")
        L = self.n_leaves
        for k in range(K):
            fl = np.asarray(self.first_leaf[k], dtype=np.uint32)
            if fl.shape != (self.n_domains[k] + 1,):
                raise ValueError(f"first_leaf[{k}] has shape {fl.shape}")
            if fl[0] != 0 or fl[-1] != L or np.any(np.diff(fl.astype(np.int64)) < 0):
                raise ValueError(f"first_leaf[{k}] is not a monotone cover of the leaves")
        for k in range(K - 1):
            if not np.all(np.isin(self.first_leaf[k], self.first_leaf[k + 1])):
                raise ValueError(f"level {k} is not nested in level {k + 1}")

    def parent_of_leaf(self, level: int) -> np.ndarray:
        """Domain id at `level` containing each leaf (int64 [L])."""
        fl = np.asarray(self.first_leaf[level], dtype=np.int64)
        leaves = np.arange(self.n_leaves, dtype=np.int64)
        return np.searchsorted(fl, leaves, side="right") - 1

    def domain_value(self, level: int, d: int) -> str:
        if self.domain_values is not None:
            return self.domain_values[level][d]
        return default_domain_value(self.level_keys[level], d)


def default_domain_value(key: str, d: int) -> str:
    stem = key.rsplit("/", 1)[-1]
    return f"{stem}-{d:05d}"


@dataclass
class Nodes:
    """Node rows of one shard, sorted by leaf domain."""

    leaf_start: np.ndarray          # uint32 [n_leaves + 1]
    labels: np.ndarray              # uint64 [W, N]
    taints: np.ndarray              # uint32 [N]
    free: np.ndarray                # uint32 [R, N]
    excl: np.ndarray                # int32  [N]
    leaf_begin: int = 0
    node_names: Optional[List[str]] = None

    @property
    def n_nodes(self) -> int:
        return int(self.taints.shape[0])

    @property
    def n_leaves(self) -> int:
        return int(self.leaf_start.shape[0] - 1)

    @property
    def n_label_words(self) -> int:
        return int(self.labels.shape[0])

    @property
    def n_res(self) -> int:
        return int(self.free.shape[0])

    def validate(self) -> None:
        N = self.n_nodes
        ls = self.leaf_start
        if ls.dtype != np.uint32 or ls[0] != 0 or ls[-1] != N or np.any(np.diff(ls.astype(np.int64)) < 0):
            raise ValueError("leaf_start is not a monotone uint32 cover of the rows")
        if self.labels.dtype != np.uint64 or self.labels.shape[1] != N or not 1 <= self.labels.shape[0] <= MAX_LABEL_WORDS:
            raise ValueError("labels must be uint64 [W, N], 1 <= W <= 4")
        if self.taints.dtype != np.uint32 or self.free.dtype != np.uint32 or self.excl.dtype != np.int32:
            raise ValueError("taints/free/excl dtypes must be uint32/uint32/int32")
        if self.free.shape[1] != N or not 1 <= self.free.shape[0] <= MAX_RES:
            raise ValueError("free must be uint32 [R, N], 1 <= R <= 4")

    def leaf_of_row(self) -> np.ndarray:
        """Global leaf id of every row (int64 [N])."""
        counts = np.diff(self.leaf_start.astype(np.int64))
        return np.repeat(np.arange(self.n_leaves, dtype=np.int64) + self.leaf_begin, counts)


@dataclass
class JobClass:
    """One requirement class (see module docstring)."""

    req_labels: Tuple[int, ...] = (0,)
    forbid_labels: Tuple[int, ...] = (0,)
    tolerated_taints: int = 0
    level: int = 0
    pods: int = 1
    req_res: Tuple[int, ...] = (0,)

    def words(self, W: int) -> Tuple[List[int], List[int]]:
        req = list(self.req_labels) + [0] * (MAX_LABEL_WORDS - len(self.req_labels))
        fb = list(self.forbid_labels) + [0] * (MAX_LABEL_WORDS - len(self.forbid_labels))
        return req[:MAX_LABEL_WORDS], fb[:MAX_LABEL_WORDS]

    def res(self) -> List[int]:
        r = list(self.req_res) + [0] * (MAX_RES - len(self.req_res))
        return r[:MAX_RES]


@dataclass
class Problem:
    """A placement call: snapshot + classes + jobs in global order."""

    topology: Topology
    nodes: Nodes
    classes: List[JobClass]
    job_class: np.ndarray                     # uint32 [J]
    name: str = ""
    job_names: Optional[List[str]] = None     # namespaced job names, global order
    meta: Dict[str, object] = field(default_factory=dict)

    @property
    def n_jobs(self) -> int:
        return int(self.job_class.shape[0])


class Dictionary:
    """Sorted, deterministic interning of string tuples to bit positions."""

    def __init__(self, items: Sequence[Tuple[str, ...]], capacity: int):
        uniq = sorted(set(items))
        if len(uniq) > capacity:
            raise ValueError(f"{len(uniq)} distinct entries exceed capacity {capacity}")
        self.items = uniq
        self.bit: Dict[Tuple[str, ...], int] = {t: i for i, t in enumerate(uniq)}

    def mask_words(self, items: Sequence[Tuple[str, ...]], W: int) -> List[int]:
        words = [0] * W
        for t in items:
            b = self.bit[t]
            words[b >> 6] |= 1 << (b & 63)
        return words


def job_runs(job_class: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Run-length encode a per-job class list into replicated-job runs
    (run_class, run_len), preserving the global job order."""
    jc = np.asarray(job_class, dtype=np.uint32)
    if jc.shape[0] == 0:
        return np.zeros(0, dtype=np.uint32), np.zeros(0, dtype=np.uint32)
    starts = np.concatenate([[0], np.nonzero(jc[1:] != jc[:-1])[0] + 1])
    lens = np.diff(np.concatenate([starts, [jc.shape[0]]]))
    return jc[starts].astype(np.uint32), lens.astype(np.uint32)


def shard_problem(p: Problem, rank: int, world: int) -> Nodes:
    """Domain-aligned node shard for `rank`: level-0 domains are
    split into `world` contiguous groups of about equal row count, so every
    domain at every level lives wholly on one shard."""
    topo, nodes = p.topology, p.nodes
    fl0 = np.asarray(topo.first_leaf[0], dtype=np.int64)
    rows_at = nodes.leaf_start.astype(np.int64)[fl0]          # row offset of each level-0 boundary
    N = nodes.n_nodes
    cuts = [0]
    for r in range(1, world):
        target = N * r // world
        i = int(np.searchsorted(rows_at, target, side="left"))
        i = min(max(i, cuts[-1]), len(fl0) - 1)
        cuts.append(i)
    cuts.append(len(fl0) - 1)
    z0, z1 = cuts[rank], cuts[rank + 1]
    l0, l1 = int(fl0[z0]), int(fl0[z1])
    r0, r1 = int(nodes.leaf_start[l0]), int(nodes.leaf_start[l1])
    return Nodes(
        leaf_start=(nodes.leaf_start[l0:l1 + 1].astype(np.int64) - r0).astype(np.uint32),
        labels=np.ascontiguousarray(nodes.labels[:, r0:r1]),
        taints=np.ascontiguousarray(nodes.taints[r0:r1]),
        free=np.ascontiguousarray(nodes.free[:, r0:r1]),
        excl=np.ascontiguousarray(nodes.excl[r0:r1]),
        leaf_begin=l0,
    )
