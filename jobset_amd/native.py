"""ctypes binding of include/jsplace.h (the engine's C ABI).

The shared library is built in-tree (`make` or __graft_entry__.build()) as
jobset_amd/libjsplace.so. There is no fallback: if the library or a GPU is
missing, engine construction raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# JSP_LIB_PATH selects another build of the same library (tools/stamps.py
# loads the -DJSP_STAMPS diagnostic build); the default is the in-tree product.
LIB_PATH = os.environ.get("JSP_LIB_PATH") or os.path.join(_HERE, "libjsplace.so")

JSP_OK, JSP_EINVAL, JSP_EHIP, JSP_ENOMEM, JSP_ESTATE, JSP_ERANGE = 0, -1, -2, -3, -4, -5
ERROR_NAMES = {JSP_EINVAL: "JSP_EINVAL", JSP_EHIP: "JSP_EHIP", JSP_ENOMEM: "JSP_ENOMEM",
               JSP_ESTATE: "JSP_ESTATE", JSP_ERANGE: "JSP_ERANGE"}

MAX_LEVELS, MAX_LABEL_WORDS, MAX_RES = 4, 4, 4

u32, i32, u64, vp = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_void_p


class JspTopology(ctypes.Structure):
    _fields_ = [("n_levels", u32), ("n_domains", u32 * MAX_LEVELS), ("first_leaf", vp * MAX_LEVELS)]


class JspNodes(ctypes.Structure):
    _fields_ = [("n_nodes", u32), ("leaf_begin", u32), ("n_leaves", u32), ("leaf_start", vp),
                ("n_label_words", u32), ("labels", vp), ("taints", vp), ("n_res", u32),
                ("free_res", vp), ("excl_owner", vp)]


class JspJobClass(ctypes.Structure):
    _fields_ = [("req_labels", u64 * MAX_LABEL_WORDS), ("forbid_labels", u64 * MAX_LABEL_WORDS),
                ("tolerated_taints", u32), ("level", u32), ("pods", u32), ("req_res", u32 * MAX_RES)]


class JspStats(ctypes.Structure):
    _fields_ = [("jobs", u32), ("placed", u32), ("runs", u32), ("fused", u32), ("wall_us", ctypes.c_double)]


class JspTiming(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("tally_ms", ctypes.c_double), ("feas_ms", ctypes.c_double),
                ("assign_ms", ctypes.c_double), ("fused_ms", ctypes.c_double), ("fused_calls", ctypes.c_uint64),
                ("host_calls", ctypes.c_uint64), ("host_prep_us", ctypes.c_double),
                ("host_launch_us", ctypes.c_double), ("host_wait_us", ctypes.c_double),
                ("host_post_us", ctypes.c_double), ("svc_calls", ctypes.c_uint64), ("svc_starts", ctypes.c_uint64),
                ("svc_us", ctypes.c_double), ("svc_fallbacks", ctypes.c_uint64),
                ("svc_ready_us", ctypes.c_double), ("svc_pre_us", ctypes.c_double),
                ("svc_answer_us", ctypes.c_double), ("svc_first_us", ctypes.c_double), ("patches", ctypes.c_uint64), ("patch_us", ctypes.c_double),
                ("wake_us", ctypes.c_double), ("oneshot_calls", ctypes.c_uint64), ("oneshot_launch_us", ctypes.c_double),
                ("oneshot_wait_us", ctypes.c_double), ("oneshot_walk_us", ctypes.c_double),
                ("oneshot_stage_us", ctypes.c_double)]


HIST_BUCKETS = 32
HIST_LO_US, HIST_LO_JOBS = 0.5, 1.0


class JspHist(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("sum", ctypes.c_double), ("max", ctypes.c_double),
                ("bucket", ctypes.c_uint64 * HIST_BUCKETS)]

    def upper_bounds(self, lo: float):
        """`le` of each bucket (the last one +inf), as a Prometheus exporter
        would publish them."""
        return [lo * 2.0 ** i for i in range(HIST_BUCKETS - 1)] + [float("inf")]

    def quantile(self, q: float, lo: float) -> float:
        """Upper bound of the bucket holding the q-quantile."""
        target, acc = q * self.count, 0
        for ub, n in zip(self.upper_bounds(lo), self.bucket):
            acc += n
            if acc >= target and acc > 0:
                return ub
        return float("inf")


class JspMetrics(ctypes.Structure):
    _fields_ = [("place_us", JspHist), ("patch_us", JspHist), ("batch_jobs", JspHist), ("device_us", JspHist),
                ("placed", ctypes.c_uint64), ("unplaceable", ctypes.c_uint64), ("place_errors", ctypes.c_uint64),
                ("patch_errors", ctypes.c_uint64), ("svc_calls", ctypes.c_uint64), ("svc_starts", ctypes.c_uint64),
                ("svc_fallbacks", ctypes.c_uint64)]


JSP_FUSED_OFF, JSP_FUSED_AUTO = 0, 1
JSP_SERVICE_OFF, JSP_SERVICE_AUTO, JSP_SERVICE_PARKED = 0, 1, 2


# (name, restype, argtypes) — every entry point declared in include/jsplace.h
# (the product boundary) and, after it, include/jsplace_bench.h (jspb_*: the
# bench's and probes' symbol set)
SIGNATURES = [
    ("jsp_abi_version", ctypes.c_int, []),
    ("jsp_last_error", ctypes.c_char_p, []),
    ("jsp_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("jsp_engine_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
    ("jsp_engine_create_multi", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(vp)]),
    ("jsp_engine_shards", ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("jsp_engine_destroy", None, [vp]),
    ("jsp_topology_upload", ctypes.c_int, [vp, ctypes.POINTER(JspTopology)]),
    ("jsp_snapshot_upload", ctypes.c_int, [vp, ctypes.POINTER(JspNodes)]),
    ("jsp_snapshot_patch", ctypes.c_int, [vp, vp, u32, vp, vp, vp, vp]),
    ("jsp_classes_upload", ctypes.c_int, [vp, ctypes.POINTER(JspJobClass), u32]),
    ("jsp_place", ctypes.c_int, [vp, vp, vp, u32, vp, vp, vp, ctypes.POINTER(JspStats)]),
    ("jsp_place_jobs", ctypes.c_int, [vp, vp, u32, vp, vp, vp, ctypes.POINTER(JspStats)]),
    ("jsp_tally_device", ctypes.c_int, [vp, vp, vp, u32, vp]),
    ("jsp_assign_device", ctypes.c_int, [vp, vp, vp, u32, vp, vp, u32, u32, vp, vp]),
    ("jsp_place_device", ctypes.c_int, [vp, vp, vp, u32, u32, vp, vp]),
    ("jsp_resolve_leader_domains", ctypes.c_int, [vp, vp, vp, u32, vp]),
    ("jsp_audit_placements", ctypes.c_int, [vp, vp, vp, vp, vp, u32, vp]),
    ("jsp_engine_set_service", ctypes.c_int, [vp, ctypes.c_int]),
    ("jsp_engine_service_stop", ctypes.c_int, [vp]),
    ("jsp_engine_get_metrics", ctypes.c_int, [vp, ctypes.POINTER(JspMetrics), ctypes.c_int]),
    ("jsp_engine_stream", vp, [vp]),
    ("jsp_engine_sync", ctypes.c_int, [vp]),
    ("jsp_engine_check", ctypes.c_int, [vp]),
    # jsplace_bench.h
    ("jspb_place_loop", ctypes.c_int, [vp, vp, vp, u32, vp, u32, vp, vp, u32, vp]),
    ("jspb_recovery_loop", ctypes.c_int, [vp, vp, vp, u32, vp, u32, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                         vp, vp, u32, vp]),
    ("jspb_set_fused", ctypes.c_int, [vp, ctypes.c_int]),
    ("jspb_service_clock", ctypes.c_int, [vp, vp, u32, vp]),
    ("jspb_tally_device_timed", ctypes.c_int, [vp, vp, vp, u32, u32, vp, ctypes.c_size_t, vp]),
    ("jspb_place_device_timed", ctypes.c_int, [vp, vp, vp, u32, u32, vp, u32, vp, ctypes.c_size_t, vp]),
    ("jspb_link_floor", ctypes.c_int, [vp, u32, vp]),
    ("jspb_tally_device_spans", ctypes.c_int, [vp, vp, vp, u32, u32, vp]),
    ("jspb_set_timing", ctypes.c_int, [vp, ctypes.c_int]),
    ("jspb_get_timing", ctypes.c_int, [vp, ctypes.POINTER(JspTiming), ctypes.c_int]),
]

_lib = None


class JspError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {message}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load libjsplace.so. Raises (no fallback) when it has not been built."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: when torch is installed its bundled
        # libamdhip64 must be the one libjsplace.so binds to (same SONAME), or
        # torch cannot initialise the GPU afterwards and the stream / device
        # pointers handed across (bench.py, distributed.py) would belong to
        # another runtime. Load it first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make` or __graft_entry__.build()")
        l = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def check(rc: int) -> None:
    if rc != JSP_OK:
        msg = lib().jsp_last_error()
        raise JspError(rc, msg.decode() if msg else "")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().jsp_device_count(ctypes.byref(n))
    return n.value if rc == JSP_OK else 0
