"""Resident placement service (jsp_engine_set_service): host-API
placements of the one-class compaction shape answered by the persistent
kernel through the pinned request word. Bit-exact against the oracle and the
launch path, across repeated requests, job counts that outgrow the output
buffer, snapshot re-uploads and patches, idle exits and explicit stops."""
import dataclasses
import time

import numpy as np
import pytest

from jobset_amd import synth
from jobset_amd.snapshot import job_runs
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture
def svc_engine(engine):
    engine.set_service(True)
    engine.set_fused(True)
    yield engine
    engine.service_stop()


def warm(engine, job_class):
    """The first host-API call after the service (re)starts -- an upload, an
    idle exit, a geometry change -- is answered on the launch path while the
    new service comes up (DESIGN.md §4.3 cold start); place until a resident
    shape answers (at most a few calls). Returns that answer."""
    for _ in range(4):
        got = engine.place(job_class)
        if got.fused in (3, 4, 5):
            return got
    return got


def one_leaf_class(p):
    """The problem reduced to its first class moved to the leaf level (the
    compaction shape the service answers)."""
    K = p.topology.n_levels
    p.classes = [dataclasses.replace(p.classes[0], level=K - 1)]
    p.job_class = np.zeros(p.n_jobs, dtype=np.uint32)
    return p


def test_service_configs_repeated(svc_engine):
    """cfg1 and cfg2 (the headline), 200 requests each on one service."""
    svc_engine.timing(reset=True)
    for cfg in (1, 2):
        p = synth.CONFIGS[cfg]()
        svc_engine.load(p)
        a = O.place_c(p)[0]
        warm(svc_engine, p.job_class)
        call = svc_engine.host_placer(*job_runs(p.job_class))
        for _ in range(200):
            st = call()
            assert st.fused == 3
            np.testing.assert_array_equal(call.assign, a)
            assert st.placed == int((a >= 0).sum())
    t = svc_engine.timing(reset=True)
    assert 400 <= t.svc_calls <= 402
    assert 2 <= t.svc_starts <= 4  # one per upload (+ a rare idle restart)


@pytest.mark.parametrize("seed", range(40))
def test_service_random_parity(svc_engine, seed):
    """Ragged random snapshots (empty and 1-node leaves, 1-3 levels, W/R 1..4,
    occupancy) with one leaf-level class: service == oracle == launch path."""
    p = one_leaf_class(synth.random_problem(seed))
    svc_engine.load(p)
    a, cap, occ = O.place_c(p)
    np.testing.assert_array_equal(warm(svc_engine, p.job_class).assign, a)
    for _ in range(3):
        got = svc_engine.place(p.job_class)
        assert got.fused == 3
        np.testing.assert_array_equal(got.assign, a)
        assert got.placed == int((a >= 0).sum())
    ref = svc_engine.place(p.job_class, want_tally=True)  # launch path (tallies requested)
    assert ref.fused == 2
    np.testing.assert_array_equal(ref.assign, a)
    np.testing.assert_array_equal(ref.cap, cap)


def test_service_job_counts_and_growth(svc_engine):
    """J = 0, 1, more jobs than feasible racks, and a J beyond the service's
    output capacity (restart with a larger pinned buffer: that call is
    answered on the launch path, the next by the new service)."""
    p = synth.config2()
    svc_engine.load(p)
    warm(svc_engine, p.job_class)
    for J in (0, 1, 990, 1500, 5000, 7000, 3, 0):
        p.job_class = np.zeros(J, dtype=np.uint32)
        a = O.place_c(p)[0]
        for _ in range(2):
            got = svc_engine.place(p.job_class)
            assert got.assign.shape == (J,)
            np.testing.assert_array_equal(got.assign, a)
        assert got.fused == 3


def test_service_patch_and_reupload(svc_engine):
    """Patches (no restart: the service is idle between requests and the patch
    is synchronous) and re-uploads (restart on new buffers) are both seen."""
    p = synth.config2()
    svc_engine.load(p)
    np.testing.assert_array_equal(warm(svc_engine, p.job_class).assign, O.place_c(p)[0])
    svc_engine.timing(reset=True)
    rng = np.random.default_rng(7)
    for step in range(10):
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=50, replace=False)).astype(np.uint32)
        taints = rng.integers(0, 2, size=50).astype(np.uint32)
        svc_engine.patch_rows(rows, taints=taints)
        p.nodes.taints[rows] = taints
        got = svc_engine.place(p.job_class)
        # the service, or the launch path if the oracle's host time between
        # requests outlasted half the idle limit (a cold start: DESIGN.md §4.3)
        assert got.fused in (2, 3)
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
    t = svc_engine.timing(reset=True)
    assert t.svc_starts <= 10 - t.svc_calls + 1  # patches restart nothing; only idle gaps do
    for t in range(5):  # recovery trials: a new post-delete snapshot each
        q = synth.config2(trial=t)
        svc_engine.load(q)
        got = svc_engine.place(q.job_class)  # the service restarted at the upload's end
        assert got.fused == 3
        np.testing.assert_array_equal(got.assign, O.place_c(q)[0])
    assert svc_engine.timing(reset=True).svc_starts == 5


def test_service_idle_exit_and_stop(svc_engine):
    """After an idle gap the service has left (or is about to): the host
    restarts it and the answer is unchanged. An explicit stop, a device-wide
    synchronize, and the launch path in between all keep working."""
    import torch
    p = synth.config2()
    svc_engine.load(p)
    a = O.place_c(p)[0]
    svc_engine.timing(reset=True)
    for gap in (0.0, 0.03, 0.2, 0.0):
        time.sleep(gap)
        np.testing.assert_array_equal(svc_engine.place(p.job_class).assign, a)
    assert svc_engine.timing(reset=True).svc_starts >= 2
    svc_engine.service_stop()
    torch.cuda.synchronize()  # nothing resident: returns at once
    np.testing.assert_array_equal(svc_engine.place(p.job_class).assign, a)
    t0 = time.perf_counter()
    torch.cuda.synchronize()  # waits for the service's idle exit (JSP_SERVICE_IDLE_MS, 50 ms)
    assert time.perf_counter() - t0 < 5.0
    np.testing.assert_array_equal(svc_engine.place(p.job_class).assign, a)


def test_service_off_equals_on(svc_engine):
    p = synth.config2(trial=3)
    svc_engine.load(p)
    on = warm(svc_engine, p.job_class)
    svc_engine.set_service(False)
    off = svc_engine.place(p.job_class)
    svc_engine.set_service(True)
    assert on.fused == 3 and off.fused == 2
    np.testing.assert_array_equal(on.assign, off.assign)


def test_service_timing_stamps(svc_engine):
    """With timing on, every request's in-kernel time (first tile saw it ->
    last tile done, 100 MHz device clock) is accumulated and is below the
    host wall time of the call."""
    p = synth.config2()
    svc_engine.load(p)
    svc_engine.set_timing(True)
    try:
        warm(svc_engine, p.job_class)  # timing on restarts the service (stamps on)
        call = svc_engine.host_placer(*job_runs(p.job_class))
        svc_engine.timing(reset=True)
        walls = []
        for _ in range(100):
            t0 = time.perf_counter()
            call()
            walls.append((time.perf_counter() - t0) * 1e6)
        t = svc_engine.timing(reset=True)
    finally:
        svc_engine.set_timing(False)
    assert t.svc_calls == 100
    per = t.svc_us / t.svc_calls
    assert 0.0 < per < float(np.median(walls))


def test_service_after_device_path_and_patch(svc_engine):
    """A device-path placement (caller's stream, other CUs' L1s fill with the
    old rows), then a patch, then a service request: the service sees the
    patched rows (its acquire drops stale L1 lines; L2 is coherent)."""
    import torch
    p = synth.config2()
    svc_engine.load(p)
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    rng = np.random.default_rng(11)
    for step in range(40):
        np.testing.assert_array_equal(warm(svc_engine, p.job_class).assign, O.place_c(p)[0])
        for _ in range(4):
            svc_engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(),
                                    side.cuda_stream)
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=200, replace=False)).astype(np.uint32)
        free = rng.integers(0, 4000, size=(p.nodes.free.shape[0], 200)).astype(np.uint32)
        svc_engine.patch_rows(rows, free=free)
        p.nodes.free[:, rows] = free
        # the patch leaves the service running (its staging grows without a
        # free while the service is resident: no stall), so the service answers
        got = svc_engine.place(p.job_class)
        assert got.fused == 3
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
    svc_engine.check()


def test_service_early_answer_then_patch_and_varying_jobs(svc_engine):
    """The compaction service answers from its seq-tagged assign[] entries and
    returns before the tiles' done words; tiles past the J-th feasible leaf may
    still be tallying then. A patch right after such an answer -- of the rows
    of the LAST tiles -- and requests whose J alternates (1, fewer than the
    feasible racks, all of them, more than the racks: the -1 tail) must all
    equal the oracle on the snapshot as patched so far."""
    p = synth.config2()
    svc_engine.load(p)
    warm(svc_engine, p.job_class)
    rng = np.random.default_rng(5)
    n = p.nodes.n_nodes
    for step in range(60):
        J = [1, 300, 990, 1500][step % 4]
        jc = np.zeros(J, dtype=np.uint32)
        got = svc_engine.place(jc)
        np.testing.assert_array_equal(got.assign, O.place_c(dataclasses.replace(p, job_class=jc))[0])
        assert got.placed == int((got.assign >= 0).sum())
        if step % 3 == 0:  # right after the early answer: rows of the last tiles
            rows = np.sort(rng.choice(np.arange(n - 2000, n), size=50, replace=False)).astype(np.uint32)
            taints = rng.integers(0, 2, size=50).astype(np.uint32)
            svc_engine.patch_rows(rows, taints=taints)
            p.nodes.taints[rows] = taints
    svc_engine.check()


# ---------------------------------------------------------------- multi-class shapes (cfg3, cfg5)
# The split service: resident tiles hand back per-domain feasibility, the
# host walks (stats.fused 5).


@pytest.mark.parametrize("cfg", [3, 5])
def test_fused_service_configs(svc_engine, cfg):
    """The multi-class shape resident: several classes / levels, 100 requests
    each."""
    p = synth.CONFIGS[cfg]()
    svc_engine.load(p)
    a = O.place_c(p)[0]
    warm(svc_engine, p.job_class)
    call = svc_engine.host_placer(*job_runs(p.job_class))
    for _ in range(100):
        st = call()
        assert st.fused == 5
        np.testing.assert_array_equal(call.assign, a)
        assert st.placed == int((a >= 0).sum())
    rc, rl = job_runs(p.job_class)
    assert st.runs == rc.shape[0]


@pytest.mark.parametrize("seed", range(40))
def test_fused_service_random_parity(svc_engine, seed):
    """Ragged random snapshots in their own shape (a resident service when the
    snapshot is small enough), the job order changing between requests."""
    p = synth.random_problem(seed)
    svc_engine.load(p)
    a = O.place_c(p)[0]
    for _ in range(3):
        got = svc_engine.place(p.job_class)
        np.testing.assert_array_equal(got.assign, a)
    rng = np.random.default_rng(seed)
    q = dataclasses.replace(p, job_class=rng.permutation(p.job_class))
    got = svc_engine.place(q.job_class)
    np.testing.assert_array_equal(got.assign, O.place_c(q)[0])
    ref = svc_engine.place(p.job_class, want_tally=True)  # launch path (tallies requested)
    np.testing.assert_array_equal(ref.assign, a)


@pytest.mark.parametrize("seed", range(12))
def test_split_tiles_reuse_staged_words(svc_engine, seed):
    """Round 6: a resident split tile stages its class records, leaf starts
    and per-upper-level ancestor words in LDS at its first request and reuses
    them. Four-level ragged snapshots with classes at every level (several per
    level: the words are shared per level), requests with and without rows
    patched in between (dirty rows reload, the staged words stay), every answer
    against the oracle of the snapshot as patched."""
    p = synth.random_problem(7300 + seed, max_nodes=12_000, max_levels=4, max_leaves=600, max_jobs=400)
    K = p.topology.n_levels
    for i, c in enumerate(p.classes):  # spread the classes over the levels
        c.level = i % K
    svc_engine.load(p)
    rng = np.random.default_rng(seed)
    call = svc_engine.host_placer(*job_runs(p.job_class))
    call()
    shapes = set()
    for step in range(6):
        if step in (2, 4):
            rows = np.sort(rng.choice(p.nodes.n_nodes, size=min(3, p.nodes.n_nodes), replace=False)).astype(np.uint32)
            taints = rng.integers(0, 4, size=rows.shape[0]).astype(np.uint32)
            svc_engine.patch_rows(rows, taints=taints)
            p.nodes.taints[rows] = taints
        st = call()
        shapes.add(st.fused)
        np.testing.assert_array_equal(call.assign, O.place_c(p)[0], err_msg=f"seed {seed} step {step}")
    assert shapes <= {0, 1, 2, 3, 5, 7, 8}, shapes  # (the split service when the tiles fit: fused 5)


def test_fused_service_patch_and_device_path(svc_engine):
    """cfg5 resident while device-path launches (their own tally buffers) and
    patches interleave with its requests."""
    import torch
    p = synth.config5()
    svc_engine.load(p)
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    rng = np.random.default_rng(5)
    warm(svc_engine, p.job_class)
    for step in range(20):
        got = svc_engine.place(p.job_class)
        assert got.fused == 5
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
        svc_engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(),
                                side.cuda_stream)
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=64, replace=False)).astype(np.uint32)
        taints = (rng.integers(0, 2, size=64) << rng.integers(0, 4, size=64)).astype(np.uint32)
        svc_engine.patch_rows(rows, taints=taints)
        p.nodes.taints[rows] = taints
    svc_engine.check()


def test_two_engines_with_services(svc_engine):
    """Two engines on one GPU, each with its own resident service (compaction
    on one, split on the other), requests interleaved; destroying one while
    its service runs leaves the other answering."""
    from jobset_amd.engine import Engine
    p2, q5 = synth.config2(), synth.config5()
    a2, a5 = O.place_c(p2)[0], O.place_c(q5)[0]
    svc_engine.load(p2)
    e2 = Engine(0)
    try:
        e2.load(q5)
        warm(svc_engine, p2.job_class)
        warm(e2, q5.job_class)
        for _ in range(50):
            g2 = svc_engine.place(p2.job_class)
            g5 = e2.place(q5.job_class)
            assert g2.fused == 3 and g5.fused == 5
            np.testing.assert_array_equal(g2.assign, a2)
            np.testing.assert_array_equal(g5.assign, a5)
    finally:
        e2.close()  # its service is running: destroy stops it
    for _ in range(10):
        np.testing.assert_array_equal(svc_engine.place(p2.job_class).assign, a2)


def test_service_request_numbers_across_2_pow_30(monkeypatch):
    """The compaction tiles tag their look-back granules with the request
    number's low 30 bits: requests must never share a tag with the request
    before them across 2^30. A service started at 2^30 - 3 answers
    every request bit-exactly through the wrap."""
    from jobset_amd.engine import Engine
    monkeypatch.setenv("JSP_TEST_HOOKS", f"seq0={(1 << 30) - 3}")
    e = Engine(0)
    try:
        p = synth.config2()
        e.load(p)
        a = O.place_c(p)[0]
        warm(e, p.job_class)
        call = e.host_placer(*job_runs(p.job_class))
        for _ in range(12):
            st = call()
            assert st.fused == 3
            np.testing.assert_array_equal(call.assign, a)
        rng = np.random.default_rng(3)
        for _ in range(4):  # the answers change between requests: stale granules would show
            rows = np.sort(rng.choice(p.nodes.n_nodes, size=40, replace=False)).astype(np.uint32)
            t = rng.integers(0, 2, size=40).astype(np.uint32)
            e.patch_rows(rows, taints=t)
            p.nodes.taints[rows] = t
            got = e.place(p.job_class)
            np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
    finally:
        e.close()


def test_service_that_cannot_fit_falls_back(monkeypatch):
    """Every workgroup of a service grid must be co-resident. On a GPU (or a
    partition) with too few CUs for the grid -- the cu_limit hook stands in for
    one -- the service is not started: the call is answered by the launch
    path (same assign[]), counted once in jsp_timing.svc_fallbacks, and the
    engine stays on the launch path until the next upload."""
    from jobset_amd.engine import Engine
    monkeypatch.setenv("JSP_TEST_HOOKS", "cu_limit=2")  # read at engine creation
    e = Engine(0)
    try:
        for cfg in (2, 5):
            p = synth.CONFIGS[cfg]()
            e.load(p)
            a = O.place_c(p)[0]
            e.timing(reset=True)
            for _ in range(5):
                got = e.place(p.job_class)
                assert got.fused in (1, 2, 7, 8)  # launch shapes only
                np.testing.assert_array_equal(got.assign, a)
            assert e.timing(reset=True).svc_fallbacks == 1
    finally:
        e.close()
    monkeypatch.delenv("JSP_TEST_HOOKS")
    e = Engine(0)  # no limit: the same snapshot is served by the service
    try:
        p = synth.config2()
        e.load(p)
        got = warm(e, p.job_class)
        assert got.fused == 3 and e.timing(reset=True).svc_fallbacks == 0
    finally:
        e.close()


def test_patch_wakes_the_service(svc_engine):
    """A patch after the service idle-exited starts it again without waiting
    (the deletions of a recovery patch the snapshot before the recreate
    places it): the next place finds it up and starts nothing. After an
    explicit stop a patch starts nothing until a place is answered by it."""
    p = synth.config2()
    svc_engine.load(p)
    a = O.place_c(p)[0]
    assert warm(svc_engine, p.job_class).fused == 3
    row = np.array([123], dtype=np.uint32)
    patch = svc_engine.host_patcher(row, taints=p.nodes.taints[row])
    for gap in (0.0, 0.002, 0.02):
        svc_engine.timing(reset=True)
        time.sleep(0.08)  # past JSP_SERVICE_IDLE_MS: the service has left
        patch()
        # woken by the patch: the waker thread restarts it (poll briefly)
        for _ in range(200):
            if svc_engine.timing(reset=False).svc_starts == 1:
                break
            time.sleep(0.0005)
        assert svc_engine.timing(reset=False).svc_starts == 1
        time.sleep(gap)
        got = svc_engine.place(p.job_class)
        t = svc_engine.timing(reset=True)
        assert got.fused == 3 and t.svc_starts == 1 and t.svc_calls == 1
        np.testing.assert_array_equal(got.assign, a)
    svc_engine.service_stop()  # disarmed
    svc_engine.timing(reset=True)
    patch()
    assert svc_engine.timing(reset=False).svc_starts == 0
    got = svc_engine.place(p.job_class)
    assert got.fused == 3 and svc_engine.timing(reset=True).svc_starts == 1
    np.testing.assert_array_equal(got.assign, a)


@pytest.mark.parametrize("then", ["place", "patch_again", "upload", "tally_launch", "stop", "sync"])
def test_wake_then_any_reader(svc_engine, then):
    """A recovery's first patch after the service left is held back and the
    waker thread restarts the service and posts it. Whatever comes next --
    the placement, a second patch right behind it, a re-upload, a launch
    with tallies, an explicit stop, a sync -- finds the patched rows,
    bit-exact, at once or after the sleep the waker may still be in."""
    p = synth.config2()
    svc_engine.load(p)
    assert warm(svc_engine, p.job_class).fused == 3
    rng = np.random.default_rng(len(then))
    R = p.nodes.free.shape[0]
    for gap in (0.0, 0.003):
        time.sleep(0.08)  # past JSP_SERVICE_IDLE_MS: the service has left
        n = int(rng.integers(1, 40))
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=n, replace=False)).astype(np.uint32)
        free = rng.integers(0, 200_000, size=(R, n)).astype(np.uint32)
        excl = np.where(rng.random(n) < 0.2, 5, -1).astype(np.int32)
        svc_engine.patch_rows(rows, free=free, excl=excl)
        p.nodes.free[:, rows] = free
        p.nodes.excl[rows] = excl
        time.sleep(gap)
        if then == "patch_again":
            taints = rng.integers(0, 2, size=n).astype(np.uint32)
            svc_engine.patch_rows(rows, taints=taints)
            p.nodes.taints[rows] = taints
        elif then == "upload":
            svc_engine.load(p)
        elif then == "stop":
            svc_engine.service_stop()
        elif then == "sync":
            svc_engine.sync()
        a, cap, occ = O.place_c(p)
        if then == "tally_launch":
            got = svc_engine.place(p.job_class, want_tally=True)
            np.testing.assert_array_equal(got.cap, cap)
            np.testing.assert_array_equal(got.occ, occ)
        else:
            got = svc_engine.place(p.job_class)
            assert got.fused == 3
        np.testing.assert_array_equal(got.assign, a)


@pytest.mark.parametrize("n", [1, 255, 256, 257, 4095, 4096, 4097, 5000, 14999])
def test_async_patch_sizes_then_place(svc_engine, n):
    """The patch kernel reads the delta from pinned memory and its last
    workgroup publishes the completion word the next service request waits
    for: every column, 1 to ~all rows (one to 59 workgroups), placed at once
    behind the patch -- bit-exact, answered by the service, and no call
    stalls on a buffer that grew while the service was resident."""
    p = synth.config2()
    svc_engine.load(p)
    assert warm(svc_engine, p.job_class).fused == 3
    rng = np.random.default_rng(n)
    for _ in range(3):
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=n, replace=False)).astype(np.uint32)
        W, R = p.nodes.labels.shape[0], p.nodes.free.shape[0]
        lab = p.nodes.labels[:, rows].copy()
        lab ^= (rng.integers(0, 2, size=lab.shape).astype(np.uint64) << np.uint64(rng.integers(0, 3)))
        taints = rng.integers(0, 2, size=n).astype(np.uint32)
        free = rng.integers(0, 200_000, size=(R, n)).astype(np.uint32)
        excl = np.where(rng.random(n) < 0.01, 7, -1).astype(np.int32)
        t0 = time.perf_counter()
        svc_engine.patch_rows(rows, labels=lab, taints=taints, free=free, excl=excl)
        got = svc_engine.place(p.job_class)
        wall = time.perf_counter() - t0
        p.nodes.labels[:, rows] = lab
        p.nodes.taints[rows] = taints
        p.nodes.free[:, rows] = free
        p.nodes.excl[rows] = excl
        assert got.fused == 3
        assert wall < 0.02, f"patch + place took {wall * 1e3:.1f} ms"
        a, cap, occ = O.place_c(p)
        np.testing.assert_array_equal(got.assign, a)
    full = svc_engine.place(p.job_class, want_tally=True)  # launch path, tallies out: the patched columns
    a, cap, occ = O.place_c(p)
    np.testing.assert_array_equal(full.cap, cap)
    np.testing.assert_array_equal(full.occ, occ)


@pytest.mark.gpu
@pytest.mark.parametrize("rep", range(3))
@pytest.mark.parametrize("then", ["place", "tally_launch", "stop", "patch_again", "shared_rows"])
def test_patch_applied_by_the_dispatcher(svc_engine, rep, then):
    """A patch while the service is up is applied by its dispatcher: posted
    at once and carried again by a request that finds it not yet applied.
    Whatever reads the rows next -- the service's next request, a launch
    (tallies out), a service stop, another patch (of the same rows) -- sees
    every patched column, bit-exact."""
    p = synth.config2()
    svc_engine.load(p)
    assert warm(svc_engine, p.job_class).fused == 3
    rng = np.random.default_rng(rep * 10 + len(then))
    R = p.nodes.free.shape[0]
    rows0 = None
    for k in range(3):
        n = int(rng.integers(1, 3000))
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=n, replace=False)).astype(np.uint32)
        if then == "shared_rows" and rows0 is not None:
            rows = rows0
            n = rows.shape[0]
        rows0 = rows
        taints = rng.integers(0, 2, size=n).astype(np.uint32)
        free = rng.integers(0, 200_000, size=(R, n)).astype(np.uint32)
        svc_engine.patch_rows(rows, taints=taints, free=free)
        p.nodes.taints[rows] = taints
        p.nodes.free[:, rows] = free
        if then in ("patch_again", "shared_rows"):
            excl = np.where(rng.random(n) < 0.05, 3, -1).astype(np.int32)
            svc_engine.patch_rows(rows, excl=excl)
            p.nodes.excl[rows] = excl
        a, cap, occ = O.place_c(p)
        if then == "tally_launch":
            got = svc_engine.place(p.job_class, want_tally=True)
            np.testing.assert_array_equal(got.cap, cap)
            np.testing.assert_array_equal(got.occ, occ)
        elif then == "stop":
            svc_engine.service_stop()
            got = svc_engine.place(p.job_class)
        else:
            got = svc_engine.place(p.job_class)
            assert got.fused == 3
        np.testing.assert_array_equal(got.assign, a)
    got = svc_engine.place(p.job_class, want_tally=True)
    a, cap, occ = O.place_c(p)
    np.testing.assert_array_equal(got.assign, a)
    np.testing.assert_array_equal(got.cap, cap)


def test_no_stall_when_buffers_grow_under_the_service(svc_engine):
    """Batched follower resolution / audits whose scratch outgrows its
    buffers while the service is resident: the old buffers wait for the
    service to stop instead of a free that waits for the service to leave."""
    p = synth.config2()
    svc_engine.load(p)
    a = warm(svc_engine, p.job_class).assign
    svc_engine.timing(reset=True)
    for n in (10, 1000, 20_000, 200_000):
        rows = (np.arange(n, dtype=np.int64) * 7919 % p.nodes.n_nodes).astype(np.int32)
        lv = np.zeros(n, dtype=np.uint32)
        t0 = time.perf_counter()
        dom = svc_engine.resolve_leader_domains(rows, lv)
        assert time.perf_counter() - t0 < 0.02
        assert dom.shape[0] == n
        got = svc_engine.place(p.job_class)
        assert got.fused == 3
        np.testing.assert_array_equal(got.assign, a)
    assert svc_engine.timing(reset=True).svc_starts == 0


@pytest.mark.parametrize("hooks", ["", "svc_xcd=0", "block_chunks=2", "svc_xcd=0,block_chunks=2", "svc_entries=1",
                                   "svc_xcd=0,svc_entries=1", "block_chunks=2,svc_entries=1"])
def test_service_colocated_and_spread(monkeypatch, hooks):
    """The compaction service co-located on one XCD (plain bell and granule
    stores when every workgroup votes the same XCC id) and spread over the
    chip (write-through, as a partition mode would place it), with the
    tiles' rows held in registers (one chunk per tile) or reloaded per
    request (two-chunk tiles): the same answers, across requests, patches
    and J."""
    from jobset_amd.engine import Engine
    monkeypatch.setenv("JSP_TEST_HOOKS", hooks)
    svc_engine = Engine(0)
    p = synth.config2()
    svc_engine.load(p)
    rng = np.random.default_rng(len(hooks) + 3)
    for step in range(30):
        J = [990, 1, 500, 1200][step % 4]
        jc = np.zeros(J, dtype=np.uint32)
        got = svc_engine.place(jc)
        assert got.fused in (3,) or step == 0
        np.testing.assert_array_equal(got.assign, O.place_c(dataclasses.replace(p, job_class=jc))[0])
        if step % 5 == 4:
            rows = np.sort(rng.choice(p.nodes.n_nodes, size=64, replace=False)).astype(np.uint32)
            taints = rng.integers(0, 2, size=64).astype(np.uint32)
            svc_engine.patch_rows(rows, taints=taints)
            p.nodes.taints[rows] = taints
    svc_engine.check()
    svc_engine.close()


@pytest.mark.parametrize("idle", [False, True])
def test_wider_snapshot_then_inline_patch(svc_engine, idle):
    """a snapshot upload that widens W and R (after the
    armed service idled out, or while it runs), then small patches staged in
    the service's inline buffer, then placements. The inline staging is sized
    for the new W/R at the upload itself (the service is stopped there and no
    patch is pending), so a staged delta is never lost to a reallocation or
    read from freed memory: bit-exact with the oracle."""
    p = synth.config2()  # W = 1, R = 3
    svc_engine.load(p)
    assert warm(svc_engine, p.job_class).fused == 3
    if idle:
        time.sleep(0.08)  # past JSP_SERVICE_IDLE_MS: the service left, still armed
    N = p.nodes.n_nodes
    wide = dataclasses.replace(
        p.nodes,
        labels=np.vstack([p.nodes.labels, np.zeros((3, N), dtype=np.uint64)]),
        free=np.vstack([p.nodes.free, np.full((1, N), 1 << 20, dtype=np.uint32)]))
    q = dataclasses.replace(p, nodes=wide)
    svc_engine.upload_snapshot(q.nodes)
    rng = np.random.default_rng(9 + int(idle))
    for step in range(6):
        if idle and step == 3:
            time.sleep(0.08)
        n = int(rng.integers(1, 30))
        rows = np.sort(rng.choice(N, size=n, replace=False)).astype(np.uint32)
        lab = q.nodes.labels[:, rows].copy()
        lab[3] = rng.integers(0, 1 << 40, size=n).astype(np.uint64)  # a word no class reads
        free = rng.integers(0, 200_000, size=(4, n)).astype(np.uint32)
        taints = rng.integers(0, 2, size=n).astype(np.uint32)
        svc_engine.patch_rows(rows, labels=lab, taints=taints, free=free)
        q.nodes.labels[:, rows] = lab
        q.nodes.free[:, rows] = free
        q.nodes.taints[rows] = taints
        got = svc_engine.place(q.job_class)
        np.testing.assert_array_equal(got.assign, O.place_c(q)[0])
    svc_engine.check()


@pytest.mark.parametrize("then", ["place", "place_twice", "tally_launch", "stop", "sync", "upload", "big_patch"])
@pytest.mark.parametrize("cfg", [2, 5])
def test_micro_patches_ride_in_the_request(svc_engine, cfg, then):
    """Patches of a few rows while the service is up ride in the next
    request's line (no staging read, no request of their own): consecutive
    patches of the same columns merge (a row patched twice keeps the last
    values), a patch of other columns or a larger one sends the held one
    first, and whatever reads the rows next -- the next request, a launch
    with tallies, a stop, a sync, an upload -- sees every patched column,
    bit-exact."""
    p = synth.CONFIGS[cfg]()
    svc_engine.load(p)
    assert warm(svc_engine, p.job_class).fused in (3, 5)
    rng = np.random.default_rng(cfg * 100 + len(then))
    N, R = p.nodes.n_nodes, p.nodes.free.shape[0]
    for step in range(8):
        k = int(rng.integers(1, 4))
        hot = int(rng.integers(0, N))
        for _ in range(k):  # a few watch events, one row each (one row twice)
            row = np.array([hot if rng.random() < 0.3 else int(rng.integers(0, N))], dtype=np.uint32)
            if step % 3 == 2:
                t = rng.integers(0, 2, size=1).astype(np.uint32)
                svc_engine.patch_rows(row, taints=t)
                p.nodes.taints[row] = t
            else:
                f = rng.integers(0, 200_000, size=(R, 1)).astype(np.uint32)
                ex = np.where(rng.random(1) < 0.2, 4, -1).astype(np.int32)
                svc_engine.patch_rows(row, free=f, excl=ex)
                p.nodes.free[:, row] = f
                p.nodes.excl[row] = ex
        if then == "big_patch":
            rows = np.sort(rng.choice(N, size=50, replace=False)).astype(np.uint32)
            t = rng.integers(0, 2, size=50).astype(np.uint32)
            svc_engine.patch_rows(rows, taints=t)
            p.nodes.taints[rows] = t
        a, cap, occ = O.place_c(p)
        if then == "tally_launch":
            got = svc_engine.place(p.job_class, want_tally=True)
            np.testing.assert_array_equal(got.cap, cap)
            np.testing.assert_array_equal(got.occ, occ)
        elif then == "stop":
            svc_engine.service_stop()
            got = svc_engine.place(p.job_class)
        elif then == "sync":
            svc_engine.sync()
            got = svc_engine.place(p.job_class)
        elif then == "upload":
            svc_engine.upload_snapshot(p.nodes)
            got = svc_engine.place(p.job_class)
        else:
            got = svc_engine.place(p.job_class)
            if then == "place_twice":
                np.testing.assert_array_equal(got.assign, a)
                got = svc_engine.place(p.job_class)
        np.testing.assert_array_equal(got.assign, a)
    got = svc_engine.place(p.job_class, want_tally=True)
    a, cap, occ = O.place_c(p)
    np.testing.assert_array_equal(got.assign, a)
    np.testing.assert_array_equal(got.cap, cap)
    np.testing.assert_array_equal(got.occ, occ)


@pytest.mark.parametrize("cols", ["labels", "all"])
def test_micro_patch_rows_from_the_microbox(svc_engine, cols):
    """A one-row micro-patch carried by the next request of the co-located
    resident service reaches its tiles through the dispatcher's microbox
    (their rows stay in registers): label words copied from another row (the
    row's feasibility flips), or every column at once; rows at the ends of
    the snapshot and of the tiles' 4-row groups; bit-exact after each place."""
    p = synth.config2()
    svc_engine.load(p)
    assert warm(svc_engine, p.job_class).fused in (3, 5)
    rng = np.random.default_rng(7 if cols == "labels" else 8)
    N, R = p.nodes.n_nodes, p.nodes.free.shape[0]
    picks = [0, 1, 3, 4, N - 1, N - 2] + [int(x) for x in rng.integers(0, N, size=10)]
    for i, r in enumerate(picks):
        row = np.array([r], dtype=np.uint32)
        src = int(rng.integers(0, N))
        lab = p.nodes.labels[:, [src]].copy()
        if cols == "labels":
            svc_engine.patch_rows(row, labels=lab)
        else:
            f = rng.integers(0, 200_000, size=(R, 1)).astype(np.uint32)
            t = rng.integers(0, 2, size=1).astype(np.uint32)
            ex = np.where(rng.random(1) < 0.3, 2, -1).astype(np.int32)
            svc_engine.patch_rows(row, labels=lab, taints=t, free=f, excl=ex)
            p.nodes.free[:, row] = f
            p.nodes.taints[row] = t
            p.nodes.excl[row] = ex
        p.nodes.labels[:, row] = lab
        got = svc_engine.place(p.job_class)
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
        if i % 4 == 3:  # a request without a patch keeps the registers
            np.testing.assert_array_equal(svc_engine.place(p.job_class).assign, O.place_c(p)[0])
    got = svc_engine.place(p.job_class, want_tally=True)
    a, cap, occ = O.place_c(p)
    np.testing.assert_array_equal(got.assign, a)
    np.testing.assert_array_equal(got.cap, cap)
    np.testing.assert_array_equal(got.occ, occ)


@pytest.mark.parametrize("pair", [(0, -1), (-1, -2), (0, 1)])
def test_micro_patch_two_rows_at_the_ends(svc_engine, pair):
    """Two rows in one micro-patch (the most a request line carries at W=1,
    R=3): the snapshot's first and last rows, the last two, the first two --
    as one patch call, and as two calls that merge into one held
    micro-patch. Row 0 and row N-1 are where the round-5 aperture fault's
    row-id word (k == 0) sat; bit-exact after each place."""
    p = synth.config2()
    svc_engine.load(p)
    assert warm(svc_engine, p.job_class).fused == 3
    N = p.nodes.n_nodes
    rows = np.array([r % N for r in pair], dtype=np.uint32)
    for k, how in enumerate(("one call", "two calls", "one call")):
        lab = p.nodes.labels[:, [(7 * k + 5) % N, (11 * k + 3) % N]].copy()
        t = np.array([k & 1, (k + 1) & 1], dtype=np.uint32)
        if how == "one call":
            svc_engine.patch_rows(rows, labels=lab, taints=t)
        else:
            svc_engine.patch_rows(rows[:1], labels=lab[:, :1], taints=t[:1])
            svc_engine.patch_rows(rows[1:], labels=lab[:, 1:], taints=t[1:])
        p.nodes.labels[:, rows] = lab
        p.nodes.taints[rows] = t
        got = svc_engine.place(p.job_class)
        assert got.fused == 3
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0], err_msg=f"{how} {pair}")
    a, cap, occ = O.place_c(p)
    got = svc_engine.place(p.job_class, want_tally=True)
    np.testing.assert_array_equal(got.assign, a)
    np.testing.assert_array_equal(got.cap, cap)


def test_microbox_wait_that_gives_up_is_reported(svc_engine, monkeypatch):
    """a resident tile whose wait for the request's
    micro-patch rows gives up must not answer from the registers it holds.
    micro_spins=0 makes every microbox wait give up: the tiles write no answer
    line but the service's error word, the host stops the service and answers
    the call on the launch path from the rows in memory (the dispatcher wrote
    the patch through before its completion word) -- the right answer,
    counted as a service fallback, never a stale one. The next request starts
    a fresh service; bit-exact throughout."""
    p = synth.config2()
    monkeypatch.setenv("JSP_TEST_HOOKS", "micro_spins=0")
    try:
        svc_engine.load(p)  # hooks are read at upload
        assert warm(svc_engine, p.job_class).fused == 3
        a0 = O.place_c(p)[0]
        np.testing.assert_array_equal(svc_engine.place(p.job_class).assign, a0)
        for k in range(3):
            # a row of a placed rack made infeasible (an untolerated taint)
            r = int(p.nodes.leaf_start[int(a0[3 + 5 * k])])
            t = np.array([p.nodes.taints[r] | (1 << 31)], dtype=np.uint32)
            svc_engine.metrics(reset=True)
            svc_engine.patch_rows(np.array([r], dtype=np.uint32), taints=t)
            p.nodes.taints[r] = t[0]
            want = O.place_c(p)[0]
            got = svc_engine.place(p.job_class)
            np.testing.assert_array_equal(got.assign, want)
            assert got.fused not in (3, 5)  # the launch path answered it
            m = svc_engine.metrics()
            assert m.svc_fallbacks == 1 and m.place_errors == 0
            got = warm(svc_engine, p.job_class)  # a fresh service, rows from memory
            assert got.fused == 3
            np.testing.assert_array_equal(got.assign, want)
            a0 = want
    finally:
        monkeypatch.delenv("JSP_TEST_HOOKS")
        svc_engine.load(p)


@pytest.mark.parametrize("cfg", [2, 5])
def test_parked_service_survives_idle_gaps(svc_engine, cfg):
    """JSP_SERVICE_PARKED: no idle exit. Gaps of several idle limits, a
    one-row patch before each place (it rides in the request), an upload
    (the service restarts parked), then a stop and a device-wide synchronize
    that returns at once. Bit-exact against the oracle throughout."""
    import torch
    p = synth.CONFIGS[cfg]()
    try:
        svc_engine.set_service(True, parked=True)
        svc_engine.load(p)
        np.testing.assert_array_equal(warm(svc_engine, p.job_class).assign, O.place_c(p)[0])
        svc_engine.timing(reset=True)
        rng = np.random.default_rng(cfg)
        for gap in (0.12, 0.2, 0.0, 0.15):
            time.sleep(gap)
            row = np.array([rng.integers(0, p.nodes.n_nodes)], dtype=np.uint32)
            val = np.array([rng.integers(0, 4)], dtype=np.uint32)
            svc_engine.patch_rows(row, taints=val)
            p.nodes.taints[row] = val
            got = svc_engine.place(p.job_class)
            assert got.fused in (3, 5)
            np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
        t = svc_engine.timing(reset=True)
        assert t.svc_starts == 0, "a parked service never idles out"
        assert t.svc_calls == 4
        q = synth.CONFIGS[cfg](trial=1)
        svc_engine.load(q)
        time.sleep(0.12)
        got = svc_engine.place(q.job_class)
        assert got.fused in (3, 5)
        np.testing.assert_array_equal(got.assign, O.place_c(q)[0])
        svc_engine.service_stop()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 1.0
    finally:
        svc_engine.service_stop()
        svc_engine.set_service(True)


@pytest.mark.parametrize("parked", [False, True])
def test_recovery_loop_answers_exactly(svc_engine, parked):
    """jspb_recovery_loop (the bench's C-timed cold recovery): idle sleeps past
    the idle limit, one-row patches with the rows' own values, gaps; every
    call succeeds, the last answer is the oracle's, and each trial's three
    times are sane."""
    p = synth.config2()
    try:
        svc_engine.set_service(True, parked=parked)
        svc_engine.load(p)
        call = svc_engine.host_placer(*job_runs(p.job_class))
        call()
        rows = np.array([(t * 7919) % p.nodes.n_nodes for t in range(4)], dtype=np.uint32)
        out = call.recovery(4, 70_000.0, 1_000.0, rows, p.nodes.taints[rows])
        np.testing.assert_array_equal(call.assign, O.place_c(p)[0])
        assert out.shape == (4, 3) and (out[:, :2] > 0).all() and (out[:, 2] >= 900.0).all()
    finally:
        svc_engine.service_stop()
        svc_engine.set_service(True)


@pytest.mark.parametrize("rep", range(2))
def test_patch_kernel_after_dispatcher_patches(svc_engine, rep):
    """The round-4 red run (`snapshot patch 7 ended without its completion
    word`): patches the dispatcher applies must not advance the
    patch kernel's completion target. Dispatcher-applied, micro, waker-applied
    and patch-kernel patches alternate on one engine -- with the service up,
    idle-exited, switched off, and patched right at half the idle limit (the
    posted-versus-idle-exit edge) -- and every later reader sees every patch."""
    p = synth.config2()
    svc_engine.load(p)
    rng = np.random.default_rng(100 + rep)
    warm(svc_engine, p.job_class)
    for step in range(12):
        mode = step % 4
        if mode == 1:
            time.sleep(0.08)  # idle-exited: the waker restarts it
        elif mode == 2:
            svc_engine.set_service(False)  # the patch kernel applies the next patch
        elif mode == 3:
            time.sleep(0.025)  # at half the idle limit: posted, or handed to the patch kernel
        n = int(rng.choice([1, 3, 300, 5000]))
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=n, replace=False)).astype(np.uint32)
        taints = rng.integers(0, 2, size=n).astype(np.uint32)
        svc_engine.patch_rows(rows, taints=taints)
        p.nodes.taints[rows] = taints
        got = svc_engine.place(p.job_class)
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
        if mode == 2:
            svc_engine.set_service(True)
    svc_engine.sync()
