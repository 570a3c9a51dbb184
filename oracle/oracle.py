"""Parity oracle for the exclusive-placement engine — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline. The product package
(jobset_amd/) never imports it and fails loudly without its HIP library.

Two independent restatements of the placement rules documented in
oracle/cpu_ref.c:
  place_c   — the C restatement (oracle/libjsp_oracle.so), O(N*C + J + C*D)
  place_py  — a literal pure-Python loop (O(J*D) greedy), small cases only
plus the invariant checker applied to every output.

Parity status: the domain-choice rule is defined by this build (the
reference delegates it to kube-scheduler, absent here); the predicate
semantics are PARITY UNPINNED against reference fixtures and pinned by
invariants — see DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("JSPO_LIB_PATH") or os.path.join(_HERE, "libjsp_oracle.so")
_lib = None

sys.path.insert(0, os.path.dirname(_HERE))
from jobset_amd.snapshot import Problem  # noqa: E402  (data model only: no engine code)


class _Problem(ctypes.Structure):
    _fields_ = [
        ("n_levels", ctypes.c_uint32),
        ("n_domains", ctypes.c_uint32 * 4),
        ("first_leaf", ctypes.c_void_p * 4),
        ("n_nodes", ctypes.c_uint32),
        ("leaf_start", ctypes.c_void_p),
        ("W", ctypes.c_uint32),
        ("labels", ctypes.c_void_p),
        ("taints", ctypes.c_void_p),
        ("R", ctypes.c_uint32),
        ("free_res", ctypes.c_void_p),
        ("excl", ctypes.c_void_p),
        ("n_classes", ctypes.c_uint32),
        ("cls_req", ctypes.c_void_p),
        ("cls_forbid", ctypes.c_void_p),
        ("cls_tol", ctypes.c_void_p),
        ("cls_level", ctypes.c_void_p),
        ("cls_pods", ctypes.c_void_p),
        ("cls_res", ctypes.c_void_p),
        ("n_jobs", ctypes.c_uint32),
        ("job_class", ctypes.c_void_p),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
                os.path.join(_HERE, "cpu_ref.c")):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.jspo_place.restype = ctypes.c_int
        _lib.jspo_place.argtypes = [ctypes.POINTER(_Problem), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.jspo_tally.restype = ctypes.c_int
        _lib.jspo_tally.argtypes = [ctypes.POINTER(_Problem), ctypes.c_void_p, ctypes.c_void_p]
        _lib.jspo_assign.restype = ctypes.c_int
        _lib.jspo_assign.argtypes = [ctypes.POINTER(_Problem), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class PackedProblem:
    """Keeps the numpy buffers alive for the ctypes struct."""

    def __init__(self, p: Problem):
        topo, nodes = p.topology, p.nodes
        if nodes.leaf_begin != 0 or nodes.n_leaves != topo.n_leaves:
            raise ValueError("oracle needs the full (unsharded) snapshot")
        C = len(p.classes)
        self.keep = []
        st = _Problem()
        st.n_levels = topo.n_levels
        for k in range(topo.n_levels):
            st.n_domains[k] = topo.n_domains[k]
            fl = np.ascontiguousarray(topo.first_leaf[k], dtype=np.uint32)
            self.keep.append(fl)
            st.first_leaf[k] = _ptr(fl)
        arrs = dict(
            leaf_start=np.ascontiguousarray(nodes.leaf_start, dtype=np.uint32),
            labels=np.ascontiguousarray(nodes.labels, dtype=np.uint64),
            taints=np.ascontiguousarray(nodes.taints, dtype=np.uint32),
            free_res=np.ascontiguousarray(nodes.free, dtype=np.uint32),
            excl=np.ascontiguousarray(nodes.excl, dtype=np.int32),
            cls_req=np.zeros((C, 4), dtype=np.uint64),
            cls_forbid=np.zeros((C, 4), dtype=np.uint64),
            cls_tol=np.zeros(C, dtype=np.uint32),
            cls_level=np.zeros(C, dtype=np.uint32),
            cls_pods=np.zeros(C, dtype=np.uint32),
            cls_res=np.zeros((C, 4), dtype=np.uint32),
            job_class=np.ascontiguousarray(p.job_class, dtype=np.uint32),
        )
        for c, jc in enumerate(p.classes):
            req, fb = jc.words(4)
            arrs["cls_req"][c] = req
            arrs["cls_forbid"][c] = fb
            arrs["cls_tol"][c] = jc.tolerated_taints
            arrs["cls_level"][c] = jc.level
            arrs["cls_pods"][c] = jc.pods
            arrs["cls_res"][c] = jc.res()
            if jc.pods < 1 or jc.level >= topo.n_levels:
                raise ValueError(f"class {c}: pods must be >= 1 and level < K")
        if np.any(arrs["job_class"] >= C):
            raise ValueError("job_class out of range")
        for k, a in arrs.items():
            self.keep.append(a)
            setattr(st, k, _ptr(a))
        self.arrs = arrs  # the evaluator reads these in place: writing one patches its snapshot
        st.n_nodes = nodes.n_nodes
        st.W = nodes.n_label_words
        st.R = nodes.n_res
        st.n_classes = C
        st.n_jobs = p.n_jobs
        self.st = st
        self.C, self.L, self.J = C, topo.n_leaves, p.n_jobs


def place_c(p: Problem, packed: Optional[PackedProblem] = None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    pk = packed or PackedProblem(p)
    assign = np.empty(max(pk.J, 1), dtype=np.int32)
    cap = np.empty((pk.C, max(pk.L, 1)), dtype=np.uint32)
    occ = np.empty(max(pk.L, 1), dtype=np.uint32)
    rc = lib().jspo_place(ctypes.byref(pk.st), _ptr(assign), _ptr(cap), _ptr(occ))
    if rc < 0:
        raise MemoryError("oracle allocation failed")
    return assign[:pk.J], cap[:, :pk.L], occ[:pk.L]


def tally_nodes(topology_leaves: int, nodes, classes) -> Tuple[np.ndarray, np.ndarray]:
    """Per-(class, leaf) capacity and per-leaf occupancy of a (possibly
    sharded) node set: the tally half of the rules, for the shard tests."""
    from jobset_amd.snapshot import Problem, Topology
    L = nodes.n_leaves
    topo = Topology(level_keys=["leaf"], n_domains=[L], first_leaf=[np.arange(L + 1, dtype=np.uint32)])
    flat = [type(c)(req_labels=c.req_labels, forbid_labels=c.forbid_labels, tolerated_taints=c.tolerated_taints,
                    level=0, pods=c.pods, req_res=c.req_res) for c in classes]
    from jobset_amd.snapshot import Nodes
    n0 = Nodes(leaf_start=nodes.leaf_start, labels=nodes.labels, taints=nodes.taints, free=nodes.free,
               excl=nodes.excl, leaf_begin=0)
    pk = PackedProblem(Problem(topology=topo, nodes=n0, classes=flat, job_class=np.zeros(0, dtype=np.uint32)))
    cap = np.empty((pk.C, max(L, 1)), dtype=np.uint32)
    occ = np.empty(max(L, 1), dtype=np.uint32)
    lib().jspo_tally(ctypes.byref(pk.st), _ptr(cap), _ptr(occ))
    return cap[:, :L], occ[:L]


def assign_from_tallies(p: Problem, cap: np.ndarray, occ: np.ndarray) -> np.ndarray:
    pk = PackedProblem(p)
    cap = np.ascontiguousarray(cap, dtype=np.uint32)
    occ = np.ascontiguousarray(occ, dtype=np.uint32)
    assign = np.empty(max(pk.J, 1), dtype=np.int32)
    if lib().jspo_assign(ctypes.byref(pk.st), _ptr(cap), _ptr(occ), _ptr(assign)) < 0:
        raise MemoryError("oracle allocation failed")
    return assign[:pk.J]


# ------------------------------------------------------------------ optimized threaded CPU evaluator
_FAST_PATH = os.environ.get("JSPF_LIB_PATH") or os.path.join(_HERE, "libjsp_cpufast.so")
_fast = None


def fast_lib():
    """oracle/libjsp_cpufast.so (cpu_fast.c): the CPU baseline bench.py times;
    bit-exact with place_c (tests/test_oracle.py)."""
    global _fast
    if _fast is None:
        if not os.path.exists(_FAST_PATH) or os.path.getmtime(_FAST_PATH) < os.path.getmtime(
                os.path.join(_HERE, "cpu_fast.c")):
            build()
        f = ctypes.CDLL(_FAST_PATH)
        f.jspf_create.restype = ctypes.c_void_p
        f.jspf_create.argtypes = [ctypes.c_int]
        f.jspf_destroy.restype = None
        f.jspf_destroy.argtypes = [ctypes.c_void_p]
        f.jspf_threads.restype = ctypes.c_int
        f.jspf_threads.argtypes = [ctypes.c_void_p]
        f.jspf_prepare.restype = ctypes.c_int
        f.jspf_prepare.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Problem)]
        f.jspf_run.restype = ctypes.c_int
        f.jspf_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        f.jspf_run_loop.restype = ctypes.c_double
        f.jspf_run_loop.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        f.jspf_recovery_loop.restype = None
        f.jspf_recovery_loop.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_void_p]
        _fast = f
    return _fast


class FastCPU:
    """The optimized evaluator on `threads` host threads (a persistent pool).
    prepare() is the untimed upload; run() one timed placement."""

    def __init__(self, threads: int = 1):
        self.lib = fast_lib()
        self.h = self.lib.jspf_create(int(threads))
        if not self.h:
            raise MemoryError("jspf_create failed")
        self.threads = self.lib.jspf_threads(self.h)
        self.pk: Optional[PackedProblem] = None

    def prepare(self, p: Problem) -> None:
        self.pk = PackedProblem(p)
        if self.lib.jspf_prepare(self.h, ctypes.byref(self.pk.st)) != 0:
            raise MemoryError("jspf_prepare failed")
        self.assign = np.empty(max(self.pk.J, 1), dtype=np.int32)

    def patch_taints(self, rows: np.ndarray, taints: np.ndarray) -> None:
        """A watch event's row patch, as the engine gets it through
        jsp_snapshot_patch: the evaluator reads the packed columns in place."""
        self.pk.arrs["taints"][rows] = taints

    def run(self, want_tally: bool = False):
        pk = self.pk
        cap = np.empty((pk.C, max(pk.L, 1)), dtype=np.uint32) if want_tally else None
        occ = np.empty(max(pk.L, 1), dtype=np.uint32) if want_tally else None
        placed = self.lib.jspf_run(self.h, _ptr(self.assign), None if cap is None else _ptr(cap),
                                   None if occ is None else _ptr(occ))
        return (self.assign[:pk.J], None if cap is None else cap[:, :pk.L], None if occ is None else occ[:pk.L],
                placed)

    def run_loop(self, iters: int, rows: Optional[np.ndarray] = None) -> float:
        """`iters` placements back to back, timed in C (µs in total); with
        rows, one of them rewritten in the taint column before each."""
        r = None if rows is None else np.ascontiguousarray(rows, dtype=np.uint32)
        return float(self.lib.jspf_run_loop(self.h, _ptr(self.assign), int(iters), None if r is None else _ptr(r),
                                            0 if r is None else int(r.shape[0])))

    def recovery_loop(self, trials: int, idle_us: float, gap_us: float, rows: np.ndarray, vals: np.ndarray,
                      spin: bool = False) -> np.ndarray:
        """The cold recovery timed in C (jspf_recovery_loop): per trial the
        idle wait, a one-row taint write, the gap, one placement. Returns
        [trials, 3] µs: write, placement, gap."""
        r = np.ascontiguousarray(rows, dtype=np.uint32)
        v = np.ascontiguousarray(vals, dtype=np.uint32)
        out = np.zeros((int(trials), 3), dtype=np.float64)
        self.lib.jspf_recovery_loop(self.h, _ptr(self.assign), int(trials), float(idle_us), float(gap_us),
                                    1 if spin else 0, _ptr(r), _ptr(v), int(r.shape[0]), _ptr(out))
        return out

    def close(self) -> None:
        if self.h:
            self.lib.jspf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ pure Python
def place_py(p: Problem) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Literal restatement for small cases: per-node loops and an O(J*D) greedy
    with no cursor, written independently of cpu_ref.c."""
    topo, nodes = p.topology, p.nodes
    K, L, N = topo.n_levels, topo.n_leaves, nodes.n_nodes
    W, R = nodes.n_label_words, nodes.n_res
    labels = [[int(x) for x in nodes.labels[w]] for w in range(W)]
    taints = [int(x) for x in nodes.taints]
    free = [[int(x) for x in nodes.free[r]] for r in range(R)]
    ls = [int(x) for x in nodes.leaf_start]
    C = len(p.classes)
    cap = np.zeros((C, L), dtype=np.uint32)
    occ = np.zeros(L, dtype=np.uint32)
    for leaf in range(L):
        occ[leaf] = sum(1 for n in range(ls[leaf], ls[leaf + 1]) if int(nodes.excl[n]) != -1)
    for c, jc in enumerate(p.classes):
        req, fb = jc.words(4)
        res = jc.res()
        for leaf in range(L):
            tot = 0
            for n in range(ls[leaf], ls[leaf + 1]):
                if any((labels[w][n] & req[w]) != req[w] or (labels[w][n] & fb[w]) for w in range(W)):
                    continue
                if taints[n] & ~jc.tolerated_taints & 0xFFFFFFFF:
                    continue
                fits = [free[r][n] // res[r] for r in range(R) if res[r] > 0]
                tot += min([jc.pods] + fits)
            cap[c, leaf] = tot

    def leaf_range(k, d):
        fl = topo.first_leaf[k]
        return int(fl[d]), int(fl[d + 1])

    taken = [set() for _ in range(K)]
    assign = np.full(p.n_jobs, -1, dtype=np.int32)
    for j in range(p.n_jobs):
        jc = p.classes[int(p.job_class[j])]
        c = int(p.job_class[j])
        k = jc.level
        for d in range(topo.n_domains[k]):
            if d in taken[k]:
                continue
            a, b = leaf_range(k, d)
            if int(cap[c, a:b].astype(np.int64).sum()) >= jc.pods and int(occ[a:b].sum()) == 0:
                assign[j] = d
                for k2 in range(K):
                    for d2 in range(topo.n_domains[k2]):
                        a2, b2 = leaf_range(k2, d2)
                        if max(a, a2) < min(b, b2):
                            taken[k2].add(d2)
                break
    return assign, cap, occ


# ------------------------------------------------------------------ invariants
def check_invariants(p: Problem, assign: np.ndarray, cap: np.ndarray, occ: np.ndarray) -> None:
    """SURVEY.md §8c I1/I2 on a placement, plus greedy maximality:
    - every placed job's domain has capacity for all its pods and no foreign
      exclusive occupancy (I1: all pods fit in one domain);
    - the leaf ranges of placed jobs are pairwise disjoint (I2);
    - an unplaced job had no feasible domain disjoint from all earlier ones."""
    topo = p.topology
    used = np.zeros(topo.n_leaves, dtype=bool)
    for j in range(p.n_jobs):
        c = int(p.job_class[j])
        jc = p.classes[c]
        fl = topo.first_leaf[jc.level]
        d = int(assign[j])
        if d >= 0:
            a, b = int(fl[d]), int(fl[d + 1])
            assert int(cap[c, a:b].astype(np.int64).sum()) >= jc.pods, f"job {j}: domain {d} lacks capacity"
            assert int(occ[a:b].sum()) == 0, f"job {j}: domain {d} is covered by another exclusive job"
            assert not used[a:b].any(), f"job {j}: domain {d} overlaps an earlier job (I2)"
            used[a:b] = True
        else:
            for dd in range(topo.n_domains[jc.level]):
                a, b = int(fl[dd]), int(fl[dd + 1])
                if a < b and not used[a:b].any() and int(occ[a:b].sum()) == 0 and \
                        int(cap[c, a:b].astype(np.int64).sum()) >= jc.pods:
                    raise AssertionError(f"job {j} unplaced although domain {dd} was feasible")
