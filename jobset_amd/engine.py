"""Python host mirror of the engine interface the Go `pkg/placement` package
exposes: `Engine.place(problem) -> assign[]`.

In the reference the domain for each child Job is chosen by kube-scheduler
from the leader's exclusive affinity terms (pkg/webhooks/
pod_mutating_webhook.go:95-135); this engine computes it deterministically for
all Jobs of a JobSet at once, at first admission and at full recreate
(pkg/controllers/failure_policy.go:155-175). Every call goes through the C ABI
of include/jsplace.h into the gfx950 kernels; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import native
from .native import JspJobClass, JspNodes, JspStats, JspTiming, JspTopology, check
from .snapshot import JobClass, Nodes, Problem, Topology, job_runs


def _p(a: Optional[np.ndarray]) -> Optional[int]:
    return None if a is None else a.ctypes.data


@dataclass
class PlaceResult:
    assign: np.ndarray           # int32 [J], domain id at the job's class level, -1 unplaceable
    cap: Optional[np.ndarray]    # uint32 [C, L] per-(class, leaf) pod capacity
    occ: Optional[np.ndarray]    # uint32 [L] rows covered by other exclusive jobs
    placed: int
    runs: int
    wall_us: float
    fused: int = 0               # launch shape: 0 three launches, 1 fused tail, 2 one-class compaction, 3/4 the resident service (compaction / fused), 5 the split service (host walk)


class Engine:
    """One engine per GPU (device id = local rank), or -- with `devices`, a
    list of device ids (repeats allowed) -- one device-set engine over several
    shards (jsp_engine_create_multi)."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        self._lib = native.lib()
        h = ctypes.c_void_p()
        if devices is not None:
            ids = (ctypes.c_int * len(devices))(*devices)
            check(self._lib.jsp_engine_create_multi(ids, len(devices), ctypes.byref(h)))
            device = int(devices[0]) if len(devices) else 0
        else:
            check(self._lib.jsp_engine_create(device, ctypes.byref(h)))
        self._h = h
        self.device = device
        self._keep: List[object] = []
        self.topology: Optional[Topology] = None
        self.nodes: Optional[Nodes] = None
        self.n_classes = 0

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.jsp_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---------------------------------------------------------------- snapshot
    def upload_topology(self, topo: Topology) -> None:
        t = JspTopology()
        t.n_levels = topo.n_levels
        keep = []
        for k in range(topo.n_levels):
            t.n_domains[k] = topo.n_domains[k]
            fl = np.ascontiguousarray(topo.first_leaf[k], dtype=np.uint32)
            keep.append(fl)
            t.first_leaf[k] = fl.ctypes.data
        check(self._lib.jsp_topology_upload(self._h, ctypes.byref(t)))
        self.topology = topo
        self.nodes = None
        self.n_classes = 0

    def upload_snapshot(self, nodes: Nodes) -> None:
        cols = dict(
            leaf_start=np.ascontiguousarray(nodes.leaf_start, dtype=np.uint32),
            labels=np.ascontiguousarray(nodes.labels, dtype=np.uint64),
            taints=np.ascontiguousarray(nodes.taints, dtype=np.uint32),
            free=np.ascontiguousarray(nodes.free, dtype=np.uint32),
            excl=np.ascontiguousarray(nodes.excl, dtype=np.int32),
        )
        n = JspNodes()
        n.n_nodes = nodes.n_nodes
        n.leaf_begin = nodes.leaf_begin
        n.n_leaves = nodes.n_leaves
        n.leaf_start = _p(cols["leaf_start"])
        n.n_label_words = cols["labels"].shape[0]
        n.labels = _p(cols["labels"])
        n.taints = _p(cols["taints"])
        n.n_res = cols["free"].shape[0]
        n.free_res = _p(cols["free"])
        n.excl_owner = _p(cols["excl"])
        check(self._lib.jsp_snapshot_upload(self._h, ctypes.byref(n)))
        self.nodes = nodes

    def patch_rows(self, rows: np.ndarray, labels: Optional[np.ndarray] = None, taints: Optional[np.ndarray] = None,
                   free: Optional[np.ndarray] = None, excl: Optional[np.ndarray] = None) -> None:
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        arrs = [None if a is None else np.ascontiguousarray(a, dtype=dt)
                for a, dt in ((labels, np.uint64), (taints, np.uint32), (free, np.uint32), (excl, np.int32))]
        check(self._lib.jsp_snapshot_patch(self._h, _p(rows), rows.shape[0], *[_p(a) for a in arrs]))

    def upload_classes(self, classes: Sequence[JobClass]) -> None:
        arr = (JspJobClass * max(len(classes), 1))()
        for i, jc in enumerate(classes):
            req, fb = jc.words(4)
            for w in range(4):
                arr[i].req_labels[w] = req[w] & ((1 << 64) - 1)
                arr[i].forbid_labels[w] = fb[w] & ((1 << 64) - 1)
            arr[i].tolerated_taints = jc.tolerated_taints & 0xFFFFFFFF
            arr[i].level = jc.level
            arr[i].pods = jc.pods
            for r, v in enumerate(jc.res()):
                arr[i].req_res[r] = v
        check(self._lib.jsp_classes_upload(self._h, arr, len(classes)))
        self.n_classes = len(classes)

    def load(self, p: Problem, nodes: Optional[Nodes] = None) -> None:
        self.upload_topology(p.topology)
        self.upload_snapshot(nodes if nodes is not None else p.nodes)
        self.upload_classes(p.classes)

    # ---------------------------------------------------------------- placement
    def place_runs(self, run_class: np.ndarray, run_len: np.ndarray, want_tally: bool = False) -> PlaceResult:
        """Jobs as replicated-job runs in global order: run i = run_len[i] jobs of
        class run_class[i] (a ReplicatedJob's replicas share one template)."""
        rc = np.ascontiguousarray(run_class, dtype=np.uint32)
        rl = np.ascontiguousarray(run_len, dtype=np.uint32)
        J = int(rl.astype(np.int64).sum())
        L = self.topology.n_leaves if self.topology is not None else 0
        assign = np.empty(max(J, 1), dtype=np.int32)
        cap = np.empty((max(self.n_classes, 1), max(L, 1)), dtype=np.uint32) if want_tally else None
        occ = np.empty(max(L, 1), dtype=np.uint32) if want_tally else None
        st = JspStats()
        check(self._lib.jsp_place(self._h, _p(rc), _p(rl), rc.shape[0], _p(assign), _p(cap), _p(occ),
                                  ctypes.byref(st)))
        return PlaceResult(assign=assign[:J], cap=None if cap is None else cap[:self.n_classes, :L],
                           occ=None if occ is None else occ[:L], placed=st.placed, runs=st.runs,
                           wall_us=st.wall_us, fused=int(st.fused))

    def place(self, job_class: np.ndarray, want_tally: bool = False) -> PlaceResult:
        """One class id per job (global order); run-length encoded in the library."""
        jc = np.ascontiguousarray(job_class, dtype=np.uint32)
        J = jc.shape[0]
        L = self.topology.n_leaves if self.topology is not None else 0
        assign = np.empty(max(J, 1), dtype=np.int32)
        cap = np.empty((max(self.n_classes, 1), max(L, 1)), dtype=np.uint32) if want_tally else None
        occ = np.empty(max(L, 1), dtype=np.uint32) if want_tally else None
        st = JspStats()
        check(self._lib.jsp_place_jobs(self._h, _p(jc), J, _p(assign), _p(cap), _p(occ), ctypes.byref(st)))
        return PlaceResult(assign=assign[:J], cap=None if cap is None else cap[:self.n_classes, :L],
                           occ=None if occ is None else occ[:L], placed=st.placed, runs=st.runs,
                           wall_us=st.wall_us, fused=int(st.fused))

    def host_placer(self, run_class: np.ndarray, run_len: np.ndarray):
        """A pre-bound jsp_place call for one run list (host buffers allocated
        once): what a caller that places the same JobSet repeatedly -- the
        recovery path, the benchmark -- binds. Returns a callable; its
        `.assign` array and `.stats` struct hold the last call's results."""
        rc = np.ascontiguousarray(run_class, dtype=np.uint32)
        rl = np.ascontiguousarray(run_len, dtype=np.uint32)
        J = int(rl.astype(np.int64).sum())
        assign = np.empty(max(J, 1), dtype=np.int32)
        st = JspStats()
        fn = self._lib.jsp_place
        args = (self._h, rc.ctypes.data, rl.ctypes.data, rc.shape[0], assign.ctypes.data, None, None,
                ctypes.byref(st))

        def call() -> JspStats:
            r = fn(*args)
            if r:
                check(r)
            return st
        loop_out = np.zeros(3, dtype=np.float64)

        def recovery(trials: int, idle_us: float, gap_us: float, patch_rows: np.ndarray, patch_taints: np.ndarray,
                     spin: bool = False) -> np.ndarray:
            """The cold recovery timed in C (jspb_recovery_loop): per trial the
            idle wait, a one-row patch, the gap, jsp_place. [trials, 3] µs:
            patch call, place call, gap."""
            pr = np.ascontiguousarray(patch_rows, dtype=np.uint32)
            pt = np.ascontiguousarray(patch_taints, dtype=np.uint32)
            out = np.zeros((int(trials), 3), dtype=np.float64)
            check(self._lib.jspb_recovery_loop(self._h, rc.ctypes.data, rl.ctypes.data, rc.shape[0], assign.ctypes.data,
                                              int(trials), float(idle_us), float(gap_us), 1 if spin else 0, _p(pr),
                                              _p(pt), int(pr.shape[0]), out.ctypes.data))
            return out

        def loop(iters: int, patch_rows: Optional[np.ndarray] = None,
                 patch_taints: Optional[np.ndarray] = None) -> Tuple[float, float, float]:
            """`iters` calls back to back timed in C (jspb_place_loop), each
            after a one-row taint patch when rows are given: total, median and
            p99 per step, microseconds."""
            pr = None if patch_rows is None else np.ascontiguousarray(patch_rows, dtype=np.uint32)
            pt = None if patch_taints is None else np.ascontiguousarray(patch_taints, dtype=np.uint32)
            check(self._lib.jspb_place_loop(self._h, rc.ctypes.data, rl.ctypes.data, rc.shape[0], assign.ctypes.data,
                                           int(iters), _p(pr), _p(pt), 0 if pr is None else int(pr.shape[0]),
                                           loop_out.ctypes.data))
            return float(loop_out[0]), float(loop_out[1]), float(loop_out[2])
        call.assign = assign[:J]
        call.stats = st
        call.loop = loop
        call.recovery = recovery
        call.keep = (rc, rl, assign, loop_out)
        return call

    def host_patcher(self, rows: np.ndarray, labels: Optional[np.ndarray] = None,
                     taints: Optional[np.ndarray] = None, free: Optional[np.ndarray] = None,
                     excl: Optional[np.ndarray] = None):
        """A pre-bound jsp_snapshot_patch for one delta (arrays converted once):
        what a watch-event handler that patches the same rows repeatedly binds
        (the bench's recovery legs). Returns a callable."""
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        arrs = [None if a is None else np.ascontiguousarray(a, dtype=dt)
                for a, dt in ((labels, np.uint64), (taints, np.uint32), (free, np.uint32), (excl, np.int32))]
        fn = self._lib.jsp_snapshot_patch
        args = (self._h, rows.ctypes.data, rows.shape[0], *[_p(a) for a in arrs])

        def call() -> None:
            r = fn(*args)
            if r:
                check(r)
        call.keep = (rows, arrs)
        return call

    def shards(self) -> Tuple[int, int]:
        """(shards, distinct devices) of this engine (1, 1 unless a device set)."""
        a, b = ctypes.c_int(0), ctypes.c_int(0)
        check(self._lib.jsp_engine_shards(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def check(self) -> None:
        """jsp_engine_check: wait for the engine's launches, raise if one failed."""
        check(self._lib.jsp_engine_check(self._h))

    def place_device(self, d_run_class: int, d_run_len: int, n_runs: int, n_jobs: int, d_assign: int,
                     stream: Optional[int] = None) -> None:
        check(self._lib.jsp_place_device(self._h, d_run_class, d_run_len, n_runs, n_jobs, d_assign, stream))

    def tally_device(self, d_cap: int, d_occ: int, ld: int, stream: Optional[int] = None) -> None:
        check(self._lib.jsp_tally_device(self._h, d_cap, d_occ, ld, stream))

    def assign_device(self, d_cap: int, d_occ: int, ld: int, d_run_class: int, d_run_len: int, n_runs: int,
                      n_jobs: int, d_assign: int, stream: Optional[int] = None) -> None:
        check(self._lib.jsp_assign_device(self._h, d_cap, d_occ, ld, d_run_class, d_run_len, n_runs, n_jobs,
                                          d_assign, stream))

    def tally_device_timed(self, d_cap: int, d_occ: int, ld: int, iters: int, scrub: int = 0,
                           scrub_bytes: int = 0) -> Tuple[float, float]:
        """(median, mean) device µs of `iters` back-to-back tallies on the
        engine stream, timed by events on the dispatches themselves
        (jspb_tally_device_timed); with a scrub buffer, each one cold."""
        out = np.zeros(2, dtype=np.float64)
        check(self._lib.jspb_tally_device_timed(self._h, d_cap, d_occ, ld, iters, scrub or None, scrub_bytes,
                                               _p(out)))
        return float(out[0]), float(out[1])

    def place_device_timed(self, d_run_class: int, d_run_len: int, n_runs: int, n_jobs: int, d_assign: int,
                           iters: int, scrub: int = 0, scrub_bytes: int = 0) -> Tuple[float, float]:
        """(median, mean) device µs of `iters` back-to-back device-path
        placements (first dispatch start -> last dispatch end each;
        jspb_place_device_timed); with a scrub buffer, each one cold."""
        out = np.zeros(2, dtype=np.float64)
        check(self._lib.jspb_place_device_timed(self._h, d_run_class, d_run_len, n_runs, n_jobs, d_assign, iters,
                                               scrub or None, scrub_bytes, _p(out)))
        return float(out[0]), float(out[1])

    def tally_device_spans(self, d_cap: int, d_occ: int, ld: int,
                           iters: int) -> Tuple[float, float, float, float]:
        """In-kernel span of the one-tile wave tally (first wave start -> last
        wave end, device clock; jspb_tally_device_spans): (median, mean) us,
        the dispatch-event time of an empty one-workgroup launch, and the
        back-to-back launches' period by the kernels' own clock."""
        out = np.zeros(4, dtype=np.float64)
        check(self._lib.jspb_tally_device_spans(self._h, d_cap, d_occ, ld, int(iters), _p(out)))
        return float(out[0]), float(out[1]), float(out[2]), float(out[3])

    def link_floor(self, iters: int = 2000) -> Tuple[float, float, float]:
        """Host -> device -> host round trip through pinned memory with the
        resident service's polling (jspb_link_floor): (p50, p99, mean) us."""
        out = np.zeros(3, dtype=np.float64)
        check(self._lib.jspb_link_floor(self._h, int(iters), _p(out)))
        return float(out[0]), float(out[1]), float(out[2])

    def set_fused(self, enable: bool) -> None:
        check(self._lib.jspb_set_fused(self._h, native.JSP_FUSED_AUTO if enable else native.JSP_FUSED_OFF))

    def set_service(self, enable: bool, parked: bool = False) -> None:
        """Resident placement service for host-API placements
        (jsp_engine_set_service; on by default). parked: it never idles out
        (JSP_SERVICE_PARKED, a dedicated GPU)."""
        mode = (native.JSP_SERVICE_PARKED if parked else native.JSP_SERVICE_AUTO) if enable else native.JSP_SERVICE_OFF
        check(self._lib.jsp_engine_set_service(self._h, mode))

    def service_stop(self) -> None:
        """Stop the resident service now (before a device-wide synchronize)."""
        check(self._lib.jsp_engine_service_stop(self._h))

    def service_clock(self) -> np.ndarray:
        """The last timed service request's per-tile 100 MHz stamps [tiles, 8]
        (jspb_service_clock); empty when none is held."""
        return self.service_clock_rows()[0]

    def service_clock_rows(self) -> Tuple[np.ndarray, np.ndarray]:
        """(the tiles' stamps [tiles, 8], the dispatcher's row [8]: 0 request
        seen in the mailbox, 1 bell rung) of the last timed service request."""
        out = np.zeros(257 * 8, dtype=np.uint32)
        n = ctypes.c_uint32(0)
        check(self._lib.jspb_service_clock(self._h, _p(out), out.shape[0], ctypes.byref(n)))
        k = n.value
        return out[:k * 8].reshape(k, 8), out[k * 8:(k + 1) * 8]

    # ---------------------------------------------------------------- webhook / reconciler batches
    def resolve_leader_domains(self, leader_rows: np.ndarray, levels: np.ndarray) -> np.ndarray:
        rows = np.ascontiguousarray(leader_rows, dtype=np.int32)
        lv = np.ascontiguousarray(levels, dtype=np.uint32)
        out = np.empty(max(rows.shape[0], 1), dtype=np.int32)
        check(self._lib.jsp_resolve_leader_domains(self._h, _p(rows), _p(lv), rows.shape[0], _p(out)))
        return out[:rows.shape[0]]

    def audit_placements(self, leader_rows: np.ndarray, levels: np.ndarray, follower_off: np.ndarray,
                         follower_domains: np.ndarray) -> np.ndarray:
        rows = np.ascontiguousarray(leader_rows, dtype=np.int32)
        lv = np.ascontiguousarray(levels, dtype=np.uint32)
        off = np.ascontiguousarray(follower_off, dtype=np.uint32)
        fd = np.ascontiguousarray(follower_domains, dtype=np.int32)
        out = np.empty(max(rows.shape[0], 1), dtype=np.uint32)
        check(self._lib.jsp_audit_placements(self._h, _p(rows), _p(lv), _p(off), _p(fd) if fd.size else None,
                                             rows.shape[0], _p(out)))
        return out[:rows.shape[0]]

    # ---------------------------------------------------------------- metrics (jsp_engine_get_metrics)
    def metrics(self, reset: bool = False) -> native.JspMetrics:
        """The engine's histograms and counters (jsplace.h jsp_metrics)."""
        m = native.JspMetrics()
        check(self._lib.jsp_engine_get_metrics(self._h, ctypes.byref(m), 1 if reset else 0))
        return m

    # ---------------------------------------------------------------- instrumentation (jsplace_bench.h)
    def set_timing(self, enable: bool) -> None:
        check(self._lib.jspb_set_timing(self._h, 1 if enable else 0))

    def timing(self, reset: bool = True) -> JspTiming:
        t = JspTiming()
        check(self._lib.jspb_get_timing(self._h, ctypes.byref(t), 1 if reset else 0))
        return t

    @property
    def stream(self) -> int:
        return self._lib.jsp_engine_stream(self._h) or 0

    def sync(self) -> None:
        check(self._lib.jsp_engine_sync(self._h))
