"""GPU parity tests: the HIP engine (through the C ABI) against the CPU oracle,
bit-exact on assign[], the per-(class, leaf) tallies and the occupancy
counts, on BASELINE.json configs 1-5 and on ragged random snapshots; plus the
invariants of SURVEY.md §8c and the edge cases of the reference's own tests
(empty inputs, unplaceable jobs, maximum sizes)."""
import os

import numpy as np
import pytest

from jobset_amd import synth
from jobset_amd.engine import Engine
from jobset_amd.native import JSP_EINVAL, JSP_ERANGE, JSP_ESTATE, JspError
from jobset_amd.snapshot import JobClass, Nodes, Problem, Topology, shard_problem
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["fused", "three-launch"])
def any_engine(request, engine):
    """The session engine in both launch shapes (fused single launch where the
    snapshot allows it, and tally -> feas -> assign)."""
    engine.set_fused(request.param == "fused")
    yield engine
    engine.set_fused(True)


def run_both(engine: Engine, p: Problem):
    engine.load(p)
    got = engine.place(p.job_class, want_tally=True)
    a, cap, occ = O.place_c(p)
    return got, a, cap, occ


def assert_same(got, a, cap, occ):
    np.testing.assert_array_equal(got.occ, occ)
    np.testing.assert_array_equal(got.cap, cap)
    np.testing.assert_array_equal(got.assign, a)
    assert got.placed == int((a >= 0).sum())


@pytest.mark.parametrize("cfg", [1, 2, 3, 5])
def test_config_parity(any_engine, cfg):
    p = synth.CONFIGS[cfg]()
    got, a, cap, occ = run_both(any_engine, p)
    assert_same(got, a, cap, occ)
    O.check_invariants(p, got.assign, got.cap, got.occ)


def test_config4_1M_parity(engine):
    p = synth.config4()
    got, a, cap, occ = run_both(engine, p)
    assert_same(got, a, cap, occ)
    # size-independent property: every placed job's domain is distinct (I2)
    placed = got.assign[got.assign >= 0]
    assert np.unique(placed).shape[0] == placed.shape[0]


def test_config2_expected_shape(engine):
    """cfg2 mirrors the 290 pods/s recovery: 990 jobs onto the 990 healthy racks."""
    p = synth.config2()
    engine.load(p)
    got = engine.place(p.job_class)
    healthy = np.setdiff1d(np.arange(1000), p.meta["bad_racks"])
    np.testing.assert_array_equal(got.assign, healthy)


@pytest.mark.parametrize("seed", range(120))
def test_random_parity(any_engine, seed):
    p = synth.random_problem(seed)
    got, a, cap, occ = run_both(any_engine, p)
    assert_same(got, a, cap, occ)


@pytest.mark.parametrize("seed", range(8))
def test_random_parity_large(engine, seed):
    p = synth.random_problem(1000 + seed, max_nodes=400_000, max_jobs=30_000, max_leaves=20_000)
    got, a, cap, occ = run_both(engine, p)
    assert_same(got, a, cap, occ)


@pytest.mark.parametrize("chunks", [2, 3, 8])
@pytest.mark.parametrize("seed", range(6))
def test_multichunk_workgroups_parity(any_engine, monkeypatch, chunks, seed):
    """Workgroups owning several 1024-row chunks (the next chunk's rows are
    prefetched while one is evaluated): ragged leaves straddle chunk borders;
    every launch shape, incl. the fused tail and the single-class compaction."""
    monkeypatch.setenv("JSP_TEST_HOOKS", f"block_chunks={chunks}")  # read at snapshot upload
    p = synth.random_problem(3000 + seed, max_nodes=60_000, max_leaves=3000)
    got, a, cap, occ = run_both(any_engine, p)
    assert_same(got, a, cap, occ)
    p.classes = [p.classes[0]]
    p.classes[0].level = p.topology.n_levels - 1
    p.job_class = np.zeros(min(p.n_jobs, 500), dtype=np.uint32)
    got, a, cap, occ = run_both(any_engine, p)
    assert_same(got, a, cap, occ)


@pytest.mark.parametrize("seed", range(24))
def test_deep_interleaved_walk_parity(any_engine, seed):
    """Up to 4 nested levels, many interleaved short runs and some long ones:
    the register-resident walker's lazy ancestor marking (flushed when a
    coarser job or a long run needs it) must equal the eager rule."""
    p = synth.random_problem(5000 + seed, max_nodes=20_000, max_levels=4, max_leaves=1500,
                             max_jobs=1200)
    got, a, cap, occ = run_both(any_engine, p)
    assert_same(got, a, cap, occ)
    O.check_invariants(p, got.assign, got.cap, got.occ)


def test_trials_parity(engine):
    """Recovery trials (seed = 2*1000 + trial) as timed by bench.py's p99 leg."""
    for t in range(20):
        p = synth.config2(trial=t)
        got, a, cap, occ = run_both(engine, p)
        assert_same(got, a, cap, occ)
        assert got.fused


def test_fused_repeat_and_ticket(engine):
    """The fused launch's last-arriver ticket survives many launches and
    snapshot changes (block counts change between snapshots)."""
    for cfg in (2, 1, 5, 2):
        p = synth.CONFIGS[cfg]()
        engine.load(p)
        a = O.place_c(p)[0]
        for _ in range(25):
            got = engine.place(p.job_class)
            np.testing.assert_array_equal(got.assign, a)
            assert got.fused


@pytest.mark.parametrize("jobs", [0, 1, 39_000, 60_000])
def test_compaction_many_tiles(engine, jobs):
    """One leaf-level class over 1M nodes: the single-launch compaction with a
    look-back across ~1000 workgroups (multiple 64-tile windows), incl. more
    jobs than feasible racks (the tail of assign[] must be -1)."""
    p = synth.config4()
    p.classes = [p.classes[0]]
    p.job_class = np.zeros(jobs, dtype=np.uint32)
    engine.load(p)
    for _ in range(3):  # the epoch scheme across repeated launches
        got = engine.place(p.job_class, want_tally=True)
        assert got.fused == 2
        a, cap, occ = O.place_c(p)
        assert_same(got, a, cap, occ)


def test_runs_api_equals_job_api(engine):
    from jobset_amd.snapshot import job_runs
    p = synth.config5()
    engine.load(p)
    rc, rl = job_runs(p.job_class)
    got = engine.place_runs(rc, rl)
    np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
    assert got.runs == rc.shape[0]


def _tiny(n_leaves=3, per=2, K=1):
    topo = Topology(level_keys=["k"], n_domains=[n_leaves], first_leaf=[np.arange(n_leaves + 1, dtype=np.uint32)])
    N = n_leaves * per
    nodes = Nodes(leaf_start=(np.arange(n_leaves + 1) * per).astype(np.uint32),
                  labels=np.ones((1, N), dtype=np.uint64), taints=np.zeros(N, dtype=np.uint32),
                  free=np.full((1, N), 10, dtype=np.uint32), excl=np.full(N, -1, dtype=np.int32))
    return topo, nodes


def test_zero_jobs(engine):
    topo, nodes = _tiny()
    p = Problem(topology=topo, nodes=nodes, classes=[JobClass(pods=1)], job_class=np.zeros(0, dtype=np.uint32))
    got, a, cap, occ = run_both(engine, p)
    assert got.assign.shape == (0,)
    np.testing.assert_array_equal(got.cap, cap)


def test_more_jobs_than_domains(engine):
    topo, nodes = _tiny(n_leaves=3)
    p = Problem(topology=topo, nodes=nodes, classes=[JobClass(pods=2, req_res=(5,))],
                job_class=np.zeros(7, dtype=np.uint32))
    got, a, cap, occ = run_both(engine, p)
    assert_same(got, a, cap, occ)
    np.testing.assert_array_equal(got.assign, [0, 1, 2, -1, -1, -1, -1])


def test_all_infeasible(engine):
    topo, nodes = _tiny()
    p = Problem(topology=topo, nodes=nodes, classes=[JobClass(req_labels=(2,), pods=1)],
                job_class=np.zeros(4, dtype=np.uint32))
    got, a, cap, occ = run_both(engine, p)
    assert (got.assign == -1).all()
    assert_same(got, a, cap, occ)


def test_empty_leaves_and_zero_rows(engine):
    topo = Topology(level_keys=["z", "r"], n_domains=[2, 5],
                    first_leaf=[np.array([0, 3, 5], dtype=np.uint32), np.arange(6, dtype=np.uint32)])
    ls = np.array([0, 0, 4, 4, 4, 9], dtype=np.uint32)  # leaves 0, 2, 3 are empty
    N = 9
    nodes = Nodes(leaf_start=ls, labels=np.ones((1, N), dtype=np.uint64), taints=np.zeros(N, dtype=np.uint32),
                  free=np.full((2, N), 7, dtype=np.uint32), excl=np.full(N, -1, dtype=np.int32))
    classes = [JobClass(pods=4, level=1, req_res=(7, 1)), JobClass(pods=9, level=0, req_res=(7, 0))]
    p = Problem(topology=topo, nodes=nodes, classes=classes, job_class=np.array([1, 0, 0, 1, 0], dtype=np.uint32))
    got, a, cap, occ = run_both(engine, p)
    assert_same(got, a, cap, occ)


def test_max_levels_words_resources(engine):
    """K = 4 nested levels, W = 4 label words, R = 4 resources, 64 classes."""
    rng = np.random.default_rng(7)
    L = 256
    fl3 = np.arange(L + 1, dtype=np.uint32)
    fl2 = np.arange(0, L + 1, 4, dtype=np.uint32)
    fl1 = np.arange(0, L + 1, 16, dtype=np.uint32)
    fl0 = np.arange(0, L + 1, 64, dtype=np.uint32)
    topo = Topology(level_keys=["a", "b", "c", "d"], n_domains=[4, 16, 64, 256], first_leaf=[fl0, fl1, fl2, fl3])
    sizes = rng.integers(0, 9, L)
    ls = np.zeros(L + 1, dtype=np.uint32)
    np.cumsum(sizes, out=ls[1:])
    N = int(ls[-1])
    labels = rng.integers(0, 2**63, (4, N), dtype=np.uint64) | rng.integers(0, 2**63, (4, N), dtype=np.uint64)
    nodes = Nodes(leaf_start=ls, labels=labels, taints=rng.integers(0, 4, N).astype(np.uint32),
                  free=rng.integers(0, 100, (4, N)).astype(np.uint32),
                  excl=np.where(rng.random(N) < 0.02, 5, -1).astype(np.int32))
    classes = [JobClass(req_labels=tuple(int(x) for x in (rng.integers(0, 2**63, 4) & rng.integers(0, 2**63, 4)
                                                            & rng.integers(0, 2**63, 4))),
                        tolerated_taints=int(rng.integers(0, 4)), level=int(rng.integers(0, 4)),
                        pods=int(rng.integers(1, 40)), req_res=tuple(int(x) for x in rng.integers(0, 30, 4)))
               for _ in range(64)]
    p = Problem(topology=topo, nodes=nodes, classes=classes,
                job_class=rng.integers(0, 64, 500).astype(np.uint32))
    got, a, cap, occ = run_both(engine, p)
    assert_same(got, a, cap, occ)


def test_exact_division_boundaries(engine):
    """fit_count must equal floor(free/req) for every 32-bit value, incl. values
    that break a float quotient (2^24+1, 2^32-1)."""
    vals = np.array([0, 1, 2, 3, 7, 8, 9, 1 << 24, (1 << 24) + 1, (1 << 24) - 1, 123456789, (1 << 31) - 1,
                     1 << 31, (1 << 32) - 1, 999_999_937, 4_000_000_000], dtype=np.uint64)
    reqs = [1, 2, 3, 7, 1000, 4097, (1 << 20) + 3, 65521, 4_000_000_001, (1 << 32) - 1]
    N = vals.shape[0]
    topo = Topology(level_keys=["k"], n_domains=[N], first_leaf=[np.arange(N + 1, dtype=np.uint32)])
    nodes = Nodes(leaf_start=np.arange(N + 1, dtype=np.uint32), labels=np.zeros((1, N), dtype=np.uint64),
                  taints=np.zeros(N, dtype=np.uint32), free=vals.astype(np.uint32)[None, :],
                  excl=np.full(N, -1, dtype=np.int32))
    classes = [JobClass(pods=1 << 22, req_res=(r,)) for r in reqs]
    p = Problem(topology=topo, nodes=nodes, classes=classes, job_class=np.zeros(0, dtype=np.uint32))
    got, a, cap, occ = run_both(engine, p)
    exp = np.minimum(vals[None, :] // np.array(reqs, dtype=np.uint64)[:, None], 1 << 22).astype(np.uint32)
    np.testing.assert_array_equal(got.cap, exp)
    np.testing.assert_array_equal(cap, exp)


def test_exact_division_boundaries(engine):
    """floor(free/req) at the 2^31 edge and for divisors up to 2^32-1, and
    after a patch brings values >= 2^31 in (the f64 reciprocal path covers
    every u32 dividend; the multiply-high form it replaced needed a 2^31 bound
    for its 2-op variant)."""
    rng = np.random.default_rng(31)
    vals = np.concatenate([np.array([0, 1, 2, 3, (1 << 31) - 1, (1 << 31) - 2, 1 << 30, (1 << 24) + 1,
                                     123456789, 999_999_937, 96_000, 1_024_000], dtype=np.uint64),
                           rng.integers(0, 1 << 31, size=52, dtype=np.uint64)])
    reqs = [2, 3, 7, 1000, 1024, 4097, 24_000, 200_000, (1 << 20) + 3, 65521, 1 << 30, (1 << 31) - 1,
            (1 << 31) + 1, 4_000_000_001, (1 << 32) - 1]
    N = vals.shape[0]
    topo = Topology(level_keys=["k"], n_domains=[N], first_leaf=[np.arange(N + 1, dtype=np.uint32)])
    nodes = Nodes(leaf_start=np.arange(N + 1, dtype=np.uint32), labels=np.zeros((1, N), dtype=np.uint64),
                  taints=np.zeros(N, dtype=np.uint32), free=vals.astype(np.uint32)[None, :],
                  excl=np.full(N, -1, dtype=np.int32))
    classes = [JobClass(pods=1 << 22, req_res=(r,)) for r in reqs]
    p = Problem(topology=topo, nodes=nodes, classes=classes, job_class=np.zeros(0, dtype=np.uint32))
    got, a, cap, occ = run_both(engine, p)
    exp = np.minimum(vals[None, :] // np.array(reqs, dtype=np.uint64)[:, None], 1 << 22).astype(np.uint32)
    np.testing.assert_array_equal(got.cap, exp)
    np.testing.assert_array_equal(cap, exp)
    big = np.array([(1 << 32) - 1, 1 << 31, 3_000_000_001], dtype=np.uint64)
    rows = np.array([0, 5, 9], dtype=np.uint32)
    engine.patch_rows(rows, free=big.astype(np.uint32)[None, :])
    vals[rows] = big
    got = engine.place(p.job_class, want_tally=True)
    exp = np.minimum(vals[None, :] // np.array(reqs, dtype=np.uint64)[:, None], 1 << 22).astype(np.uint32)
    np.testing.assert_array_equal(got.cap, exp)


def test_f64_division_exact(engine):
    """floor(free / req) through fl(double(free) * rcp(req)) truncated to u32
    equals the integer quotient at every edge: free = k*req - 1, k*req,
    k*req + 1 up to 2^32 - 1, for divisors from 2 to 2^32 - 1 (DESIGN.md
    §4.1) -- on the launch shapes (fused and three-launch tallies) and the
    device tally."""
    import torch
    rng = np.random.default_rng(64)
    reqs = [2, 3, 7, 10, 1000, 1024, 4097, 24_000, 200_000, (1 << 20) + 3, 65521, 1 << 30, (1 << 31) - 1,
            (1 << 31) + 1, 4_000_000_001, (1 << 32) - 1]
    M = (1 << 32) - 1
    vals = [0, 1, 2, M, M - 1, 1 << 31, (1 << 31) - 1]
    for d in reqs:
        for k in [1, 2, 3, 1000, 12345, M // d - 1, M // d]:
            for n in (k * d - 1, k * d, k * d + 1):
                if 0 <= n <= M:
                    vals.append(n)
    vals = np.array(vals + list(rng.integers(0, 1 << 32, size=200, dtype=np.uint64)), dtype=np.uint64)
    N = vals.shape[0]
    topo = Topology(level_keys=["k"], n_domains=[N], first_leaf=[np.arange(N + 1, dtype=np.uint32)])
    nodes = Nodes(leaf_start=np.arange(N + 1, dtype=np.uint32), labels=np.zeros((1, N), dtype=np.uint64),
                  taints=np.zeros(N, dtype=np.uint32), free=vals.astype(np.uint32)[None, :],
                  excl=np.full(N, -1, dtype=np.int32))
    exp_all = np.minimum(vals[None, :] // np.array(reqs, dtype=np.uint64)[:, None], 1 << 22).astype(np.uint32)
    for c0 in range(0, len(reqs), 4):  # <= 4 classes: the wave-tile device tally takes them in one pass
        rq = reqs[c0:c0 + 4]
        classes = [JobClass(pods=1 << 22, req_res=(r,)) for r in rq]
        p = Problem(topology=topo, nodes=nodes, classes=classes, job_class=np.zeros(0, dtype=np.uint32))
        got, a, cap, occ = run_both(engine, p)
        np.testing.assert_array_equal(got.cap, exp_all[c0:c0 + 4])
        np.testing.assert_array_equal(cap, exp_all[c0:c0 + 4])
        C, L = len(rq), N
        dcap = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
        engine.tally_device(dcap.data_ptr(), dcap[-1].data_ptr(), L, 0)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dcap[:C].cpu().numpy().astype(np.uint32), exp_all[c0:c0 + 4])


@pytest.mark.parametrize("cfg", [4, 5])
def test_double_buffered_wave_tally(monkeypatch, cfg):
    """The tally's double-buffered wave kernel (several tiles per wave, the next
    tile's rows in flight while one is evaluated): the default one-tile-per-wave
    kernel covers snapshots up to ~6k tiles, so this path is forced here
    (test hook tally_one=0): the tally and the placement must equal the
    oracle's."""
    import torch
    monkeypatch.setenv("JSP_TEST_HOOKS", "tally_one=0")
    e = Engine(0)
    try:
        p = synth.CONFIGS[cfg]()
        got, a, cap, occ = run_both(e, p)
        assert_same(got, a, cap, occ)
        C, L = len(p.classes), p.topology.n_leaves
        if C <= 4:
            dcap = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
            e.tally_device(dcap.data_ptr(), dcap[-1].data_ptr(), L, 0)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(dcap[:C].cpu().numpy().astype(np.uint32), cap)
            np.testing.assert_array_equal(dcap[C].cpu().numpy().astype(np.uint32), occ)
    finally:
        e.close()


def test_expand_records_three_launch(engine):
    """The three-launch path's long runs as records expanded by the grid
    (16 records per wave, straddling waves unevenly on ragged problems):
    each configuration places as the oracle does."""
    engine.set_fused(False)
    try:
        probs = [synth.CONFIGS[cfg]() for cfg in (1, 2, 4, 5)]
        probs += [synth.random_problem(7000 + s, max_nodes=100_000, max_jobs=20_000) for s in range(6)]
        for p in probs:
            got, a, cap, occ = run_both(engine, p)
            assert got.fused == 0
            assert_same(got, a, cap, occ)
    finally:
        engine.set_fused(True)


def test_patch_then_place(engine):
    p = synth.config2()
    engine.load(p)
    rows = np.array([0, 15 * 500 + 3, 14999], dtype=np.uint32)
    taints = np.array([1, 1, 0], dtype=np.uint32)
    engine.patch_rows(rows, taints=taints)
    got = engine.place(p.job_class, want_tally=True)
    p.nodes.taints[rows] = taints
    a, cap, occ = O.place_c(p)
    np.testing.assert_array_equal(got.assign, a)
    np.testing.assert_array_equal(got.cap, cap)


def test_sharded_tally_allreduce_parity(engine):
    """The multi-GPU protocol on one device: domain-aligned shards tally into
    zero-initialised buffers, the buffers are summed (what the RCCL all-reduce
    does), and every shard's assignment equals the unsharded one."""
    import torch
    p = synth.config5()
    a_ref, cap_ref, occ_ref = O.place_c(p)
    world = 3
    L, C = p.topology.n_leaves, len(p.classes)
    cap_sum = torch.zeros((C, L), dtype=torch.int32, device="cuda")
    occ_sum = torch.zeros(L, dtype=torch.int32, device="cuda")
    engines = [Engine(0) for _ in range(world)]
    try:
        for r, e in enumerate(engines):
            e.upload_topology(p.topology)
            e.upload_snapshot(shard_problem(p, r, world))
            e.upload_classes(p.classes)
            cap = torch.zeros((C, L), dtype=torch.int32, device="cuda")
            occ = torch.zeros(L, dtype=torch.int32, device="cuda")
            e.tally_device(cap.data_ptr(), occ.data_ptr(), L, torch.cuda.current_stream().cuda_stream)
            cap_sum += cap
            occ_sum += occ
        torch.cuda.synchronize()
        np.testing.assert_array_equal(cap_sum.cpu().numpy().astype(np.uint32), cap_ref)
        np.testing.assert_array_equal(occ_sum.cpu().numpy().astype(np.uint32), occ_ref)
        from jobset_amd.snapshot import job_runs
        rc, rl = job_runs(p.job_class)
        rct = torch.from_numpy(rc.astype(np.int32)).cuda()
        rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
        for e in engines:
            out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
            e.assign_device(cap_sum.data_ptr(), occ_sum.data_ptr(), L, rct.data_ptr(), rlt.data_ptr(), rc.shape[0],
                            p.n_jobs, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), a_ref)
    finally:
        for e in engines:
            e.close()


def test_place_device_matches_host_api(engine):
    import torch
    p = synth.config3()
    engine.load(p)
    from jobset_amd.snapshot import job_runs
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.full((p.n_jobs,), -7, dtype=torch.int32, device="cuda")
    engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), O.place_c(p)[0])


def test_resolve_and_audit(engine):
    """Batched A5/A9: leader row -> domain at the job's level, and follower
    nodeSelector domains audited against it (validatePodPlacements)."""
    p = synth.config5()
    engine.load(p)
    leaf_of_row = p.nodes.leaf_of_row()
    rows = np.array([0, 17, 16383, -1, 2048, 5000], dtype=np.int32)
    levels = np.array([1, 0, 1, 1, 0, 1], dtype=np.uint32)
    got = engine.resolve_leader_domains(rows, levels)
    zone_of_leaf = p.topology.parent_of_leaf(0)
    exp = []
    for r, k in zip(rows, levels):
        if r < 0:
            exp.append(-1)
        else:
            leaf = leaf_of_row[r]
            exp.append(int(leaf) if k == 1 else int(zone_of_leaf[leaf]))
    np.testing.assert_array_equal(got, exp)
    # followers per job: job0 3 matching; job1 none; job2 one wrong; job3 leader
    # unknown; job4 none; job5 one matching + two wrong
    off = np.array([0, 3, 3, 5, 6, 6, 9], dtype=np.uint32)
    fd = np.array([exp[0], exp[0], exp[0], 999, exp[2], 0, exp[5], exp[5] + 1, -1], dtype=np.int32)
    bad = engine.audit_placements(rows, levels, off, fd)
    np.testing.assert_array_equal(bad, [0, 0, 1, 0xFFFFFFFF, 0, 2])


def test_error_paths(engine):
    e = Engine(0)
    try:
        with pytest.raises(JspError) as ei:
            e.place(np.zeros(1, dtype=np.uint32))
        assert ei.value.code == JSP_ESTATE
        topo, nodes = _tiny()
        e.upload_topology(topo)
        with pytest.raises(JspError) as ei:
            e.upload_classes([JobClass(pods=0)])
        assert ei.value.code == JSP_EINVAL
        bad = Topology(level_keys=["a", "b"], n_domains=[2, 3],
                       first_leaf=[np.array([0, 2, 3], dtype=np.uint32), np.arange(4, dtype=np.uint32)])
        bad.first_leaf[0] = np.array([0, 1, 3], dtype=np.uint32)
        e.upload_topology(bad)  # 1 and 3 are level-1 boundaries: nested, accepted
        with pytest.raises(JspError) as ei:  # non-monotone coarse level
            e.upload_topology(Topology(level_keys=["a", "b"], n_domains=[3, 3],
                                       first_leaf=[np.array([0, 2, 1, 3], dtype=np.uint32),
                                                   np.arange(4, dtype=np.uint32)]))
        assert ei.value.code == JSP_EINVAL
        with pytest.raises(JspError) as ei:  # level 0 boundary 2 is not a level-1 boundary
            e.upload_topology(Topology(level_keys=["a", "b"], n_domains=[2, 2],
                                       first_leaf=[np.array([0, 1, 4], dtype=np.uint32),
                                                   np.array([0, 2, 4], dtype=np.uint32)]))
        assert ei.value.code == JSP_EINVAL
        with pytest.raises(JspError) as ei:
            e.upload_topology(Topology(level_keys=["a"], n_domains=[2_000_000],
                                       first_leaf=[np.arange(2_000_001, dtype=np.uint32)]))
        assert ei.value.code == JSP_ERANGE
    finally:
        e.close()


def test_webhook_consults_engine_identically(engine):
    """A5 rewired: with the cache bound to the engine, follower nodeSelector
    values come from the resident snapshot (jsp_resolve_leader_domains) and
    the mutation is identical to the reference's Node-Get path; the same for
    the PodReconciler audit (A9)."""
    from jobset_amd import host
    p = synth.config5()
    engine.load(p)
    topo = p.topology
    leaf_of_row = p.nodes.leaf_of_row()
    zone_of_leaf = topo.parent_of_leaf(0)
    names = [f"node-{r:05d}" for r in range(p.nodes.n_nodes)]
    keys = topo.level_keys
    plain, bound = host.Cache(), host.Cache()
    for r in range(0, p.nodes.n_nodes, 97):
        lf = int(leaf_of_row[r])
        plain.add_node({"metadata": {"name": names[r], "labels": {
            keys[0]: topo.domain_values[0][int(zone_of_leaf[lf])], keys[1]: topo.domain_values[1][lf]}}})
    bound.bind_engine(engine, {n: i for i, n in enumerate(names)}, keys, topo.domain_values)
    muts = []
    for j, r in enumerate(range(0, p.nodes.n_nodes, 97 * 7)):
        level_key = keys[j % 2]
        js, rj = f"js{j}", "w"
        key = host.jobHashKey("default", f"{js}-{rj}-0")
        lab = {"jobset.sigs.k8s.io/jobset-name": js, "jobset.sigs.k8s.io/replicatedjob-name": rj,
               "jobset.sigs.k8s.io/job-index": "0", "jobset.sigs.k8s.io/job-key": key}
        ann = {**lab, "alpha.jobset.sigs.k8s.io/exclusive-topology": level_key}
        own = [{"uid": f"u{j}", "kind": "Job", "controller": True}]
        leader = {"metadata": {"name": f"{js}-{rj}-0-0-abcde", "namespace": "default", "labels": lab,
                               "annotations": {**ann, "batch.kubernetes.io/job-completion-index": "0"},
                               "ownerReferences": own}, "spec": {"nodeName": names[r]}}
        follower = {"metadata": {"name": f"{js}-{rj}-0-1-fghij", "namespace": "default", "labels": lab,
                                 "annotations": {**ann, "batch.kubernetes.io/job-completion-index": "1"},
                                 "ownerReferences": own}, "spec": {}}
        for c in (plain, bound):
            c.add_pod(leader)
        a, ea = plain.Default(follower)
        b, eb = bound.Default(follower)
        assert ea is None and eb is None and a == b
        muts.append(a["spec"]["nodeSelector"])
        for c in (plain, bound):
            c.add_pod(a)
        assert plain.Reconcile("default", leader["metadata"]["name"]) == bound.Reconcile(
            "default", leader["metadata"]["name"]) is None
    assert len({tuple(m.items()) for m in muts}) > 1
    sb, sp = bound.stats(), plain.stats()
    assert sb["nodeGets"] == 0 and sb["engineCalls"] > 0 and sp["nodeGets"] > 0


def test_host_placer_equals_place(engine):
    """The pre-bound host-API call the bench times returns the oracle's
    assignment, repeatedly (completion words are tagged per launch)."""
    from jobset_amd.snapshot import job_runs
    for cfg in (1, 2, 3, 5):
        p = synth.CONFIGS[cfg]()
        engine.load(p)
        call = engine.host_placer(*job_runs(p.job_class))
        a = O.place_c(p)[0]
        for _ in range(30):
            st = call()
            np.testing.assert_array_equal(call.assign, a)
            assert st.placed == int((a >= 0).sum())


def test_lookback_timeout_is_reported(engine, monkeypatch):
    """A compaction launch whose look-back gives up must not return a silently
    wrong assign[]: jsp_place raises, and on the device path jsp_engine_check
    (or the next call) does. The hook lookback_spins=0 makes every wait a timeout."""
    import torch
    from jobset_amd.native import JSP_EHIP
    from jobset_amd.snapshot import job_runs
    p = synth.config4()
    p.classes = [p.classes[0]]
    p.job_class = np.zeros(30_000, dtype=np.uint32)
    # read at snapshot upload; svc_entries=1: a resident compaction service
    # answers through its look-back too (the per-job entry form, A/B)
    monkeypatch.setenv("JSP_TEST_HOOKS", "lookback_spins=0,svc_entries=1")
    engine.load(p)
    with pytest.raises(JspError) as ei:
        for _ in range(5):  # ~1000 tiles: some tile always finds a predecessor unpublished
            engine.place(p.job_class)
    assert ei.value.code == JSP_EHIP and "look-back" in str(ei.value)
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    with pytest.raises(JspError) as ei:
        for _ in range(5):
            engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), s)
            engine.check()
    assert ei.value.code == JSP_EHIP
    monkeypatch.delenv("JSP_TEST_HOOKS")
    engine.check()  # nothing new since the last report
    engine.load(p)
    got = engine.place(p.job_class, want_tally=True)
    a, cap, occ = O.place_c(p)
    assert_same(got, a, cap, occ)


@pytest.mark.parametrize("jobs", [0, 1, 39_000])
def test_compaction_ticket_interleaved_with_fused(engine, jobs):
    """Both single-launch kernels draw tiles from one ticket (oversubscribed
    grids, spare workgroups exit) and the fused one counts finished tiles on a
    second: their bases must stay right across interleaved launches of both
    shapes and snapshot re-uploads."""
    p = synth.config4()
    p.classes = [p.classes[0]]
    p.job_class = np.zeros(jobs, dtype=np.uint32)
    q = synth.config5()
    a, cap, occ = O.place_c(p)
    aq = O.place_c(q)[0]
    engine.load(p)
    for _ in range(3):
        got = engine.place(p.job_class, want_tally=True)
        assert got.fused == 2  # tallies requested: the launch path
        assert_same(got, a, cap, occ)
    engine.load(q)
    for _ in range(3):
        np.testing.assert_array_equal(engine.place(q.job_class).assign, aq)
    engine.load(p)
    for _ in range(2):
        np.testing.assert_array_equal(engine.place(p.job_class).assign, a)


def test_patch_after_device_place_is_ordered(engine):
    """jsp_snapshot_patch (engine stream) right after jsp_place_device on the
    caller's stream must not overwrite rows the placement is still reading: the
    engine orders the streams. Then the device placement on the caller's
    stream sees the patch."""
    import torch
    from jobset_amd.snapshot import job_runs
    p = synth.config2()
    engine.load(p)
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    side = torch.cuda.Stream()
    outs = [torch.empty(p.n_jobs, dtype=torch.int32, device="cuda") for _ in range(2)]
    a0 = O.place_c(p)[0]
    rows = np.arange(0, 15 * 40, 15, dtype=np.uint32)  # first node of racks 0..39
    engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, outs[0].data_ptr(), side.cuda_stream)
    engine.patch_rows(rows, taints=np.ones(rows.shape[0], dtype=np.uint32))
    engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, outs[1].data_ptr(), side.cuda_stream)
    engine.check()
    np.testing.assert_array_equal(outs[0].cpu().numpy(), a0)
    p.nodes.taints[rows] = 1
    np.testing.assert_array_equal(outs[1].cpu().numpy(), O.place_c(p)[0])


def test_tally_width_bound_is_erange(engine):
    """Per-leaf capacities are u32 sums of min(pods, fit) over the leaf's rows:
    classes whose pods x rows-per-leaf could reach 2^32 are refused."""
    from jobset_amd.native import JSP_ERANGE
    topo = Topology(level_keys=["k"], n_domains=[1], first_leaf=[np.arange(2, dtype=np.uint32)])
    N = 2048
    nodes = Nodes(leaf_start=np.array([0, N], dtype=np.uint32), labels=np.zeros((1, N), dtype=np.uint64),
                  taints=np.zeros(N, dtype=np.uint32), free=np.full((1, N), 1 << 31, dtype=np.uint32),
                  excl=np.full(N, -1, dtype=np.int32))
    engine.upload_topology(topo)
    engine.upload_snapshot(nodes)
    with pytest.raises(JspError) as ei:
        engine.upload_classes([JobClass(pods=1 << 21)])  # 2^21 x 2048 rows = 2^32
    assert ei.value.code == JSP_ERANGE
    engine.upload_classes([JobClass(pods=(1 << 21) - 1)])
    got = engine.place(np.zeros(1, dtype=np.uint32), want_tally=True)
    assert got.cap[0, 0] == ((1 << 21) - 1) * N and got.assign.tolist() == [0]


def _loaded_hip_runtime():
    """ctypes handle on the HIP runtime this process already uses (torch's
    bundled libamdhip64, which libjsplace.so binds to): found in
    /proc/self/maps, so no second runtime is loaded."""
    import ctypes
    for line in open("/proc/self/maps"):
        path = line.split()[-1]
        if "libamdhip64.so" in path and os.path.exists(path):
            return ctypes.CDLL(path)
    raise RuntimeError("libamdhip64 is not loaded")


def test_caller_stream_destroyed_between_calls(engine):
    """A caller's stream is used only inside the call it was given to: after
    the caller synchronises and destroys it, later calls (host API, device
    path on another stream, jsp_engine_check) never touch it (ADVICE r2:
    enter_stream kept the handle and recorded events on it)."""
    import ctypes

    import torch
    from jobset_amd.snapshot import job_runs
    hip = _loaded_hip_runtime()
    p = synth.config5()
    engine.load(p)
    a = O.place_c(p)[0]
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    for it in range(3):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        out = torch.full((p.n_jobs,), -7, dtype=torch.int32, device="cuda")
        engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), s.value)
        engine.check()  # waits on the engine's own event, not on the stream
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0
        np.testing.assert_array_equal(out.cpu().numpy(), a)
        # later calls: a patch (engine stream), the host API, the device path on torch's stream
        engine.patch_rows(np.array([it], dtype=np.uint32), taints=p.nodes.taints[it:it + 1])
        np.testing.assert_array_equal(engine.place(p.job_class).assign, a)
        out2 = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
        engine.place_device(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out2.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
        engine.check()
        np.testing.assert_array_equal(out2.cpu().numpy(), a)
        engine.sync()


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_device_timed_entry_points(engine, cfg):
    """jspb_tally_device_timed / jspb_place_device_timed (the bench's kernel-time
    legs): back-to-back steps timed by events on their own dispatches, warm
    and behind the library's cache scrub; the buffers they leave hold the
    oracle's answer."""
    import torch
    from jobset_amd.snapshot import job_runs
    p = synth.CONFIGS[cfg]()
    engine.set_fused(True)
    engine.load(p)
    C, L = len(p.classes), p.topology.n_leaves
    a, cap, occ = O.place_c(p)
    t = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
    med, mean = engine.tally_device_timed(t.data_ptr(), t[-1].data_ptr(), L, 50)
    assert 0.0 < med <= 2000.0 and 0.0 < mean <= 2000.0
    scrub = torch.zeros(64 << 20, dtype=torch.int32, device="cuda")  # 256 MiB
    cmed, _ = engine.tally_device_timed(t.data_ptr(), t[-1].data_ptr(), L, 5, scrub.data_ptr(), scrub.numel() * 4)
    assert cmed > 0.0
    engine.check()
    got = t.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got[:C], cap)
    np.testing.assert_array_equal(got[C], occ)
    rc, rl = job_runs(p.job_class)
    rct = torch.from_numpy(rc.astype(np.int32)).cuda()
    rlt = torch.from_numpy(rl.astype(np.int32)).cuda()
    out = torch.full((p.n_jobs,), -7, dtype=torch.int32, device="cuda")
    pmed, pmean = engine.place_device_timed(rct.data_ptr(), rlt.data_ptr(), rc.shape[0], p.n_jobs, out.data_ptr(), 20)
    assert 0.0 < pmed and 0.0 < pmean
    engine.check()
    np.testing.assert_array_equal(out.cpu().numpy(), a)
    with pytest.raises(JspError) as ei:
        engine.tally_device_timed(t.data_ptr(), t[-1].data_ptr(), L, 0)
    assert ei.value.code == JSP_EINVAL


def _one_level(p: Problem, level: int, max_classes: int, runs_sorted: bool, seed: int) -> Problem:
    import dataclasses
    rng = np.random.default_rng(seed)
    C = min(len(p.classes), max_classes)
    classes = [dataclasses.replace(c, level=level) for c in p.classes[:C]]
    jc = (p.job_class % C).astype(np.uint32)
    if runs_sorted:  # a few long runs (replicated jobs of one template each)
        jc = np.sort(jc, kind="stable")
        if rng.random() < 0.5:
            jc = jc[::-1].copy()
    return dataclasses.replace(p, classes=classes, job_class=jc)


@pytest.mark.parametrize("seed", range(24))
def test_folded_feasibility_and_level_walk(engine, seed):
    """The three-launch step with every class at one level: the wave tally
    folds the leaf classes' feasibility into its tiles (no feasibility
    launch) and the level walker assigns in one wave. Leaf level with <= 4
    classes takes both, an upper level only the walker, more runs than the
    walker takes the block walker: bit-exact with the oracle throughout."""
    base = synth.random_problem(seed, max_nodes=30_000, max_leaves=3000, max_jobs=3000)
    K = base.topology.n_levels
    engine.set_fused(False)
    try:
        for level, maxc, sorted_runs in ((K - 1, 4, True), (K - 1, 4, False), (0, 6, True), (K - 1, 16, True)):
            p = _one_level(base, level, maxc, sorted_runs, seed)
            engine.load(p)
            got = engine.place(p.job_class, want_tally=True)
            a, cap, occ = O.place_c(p)
            assert_same(got, a, cap, occ)
            assert got.fused == 0
    finally:
        engine.set_fused(True)


@pytest.mark.parametrize("seed", range(12))
def test_level_walk_one_launch_job_counts(engine, seed):
    """The level walk with its expansion in the same launch (expander
    workgroups wait for the walker's record count): J = 0, 1, a few, about
    the domain count and well past it (every run's tail unplaceable), empty
    leading runs, bit-exact."""
    import dataclasses
    base = _one_level(synth.random_problem(seed, max_nodes=30_000, max_leaves=3000, max_jobs=3000),
                      0, 4, True, seed)
    K = base.topology.n_levels
    base = dataclasses.replace(base, classes=[dataclasses.replace(c, level=K - 1) for c in base.classes])
    engine.set_fused(False)
    try:
        engine.load(base)
        D = base.topology.n_domains[K - 1]
        C = len(base.classes)
        for J in (0, 1, 7, D, 3 * D + 5):
            jc = np.sort(np.arange(J, dtype=np.uint32) % C, kind="stable")
            p = dataclasses.replace(base, job_class=jc)
            got = engine.place(p.job_class, want_tally=True)
            a, cap, occ = O.place_c(p)
            assert_same(got, a, cap, occ)
            assert got.fused == 0
    finally:
        engine.set_fused(True)


def test_folded_feasibility_after_patches(engine):
    """cfg4 (1M nodes, 4 leaf classes, 4 runs) placed repeatedly while rows
    change: every tally rewrites each leaf's bit exactly (no stale bit from
    the previous step survives the fold)."""
    p = synth.config4()
    engine.set_fused(False)
    try:
        engine.load(p)
        rng = np.random.default_rng(44)
        for step in range(4):
            got = engine.place(p.job_class)
            np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
            rows = np.sort(rng.choice(p.nodes.n_nodes, size=20_000, replace=False)).astype(np.uint32)
            if step % 2 == 0:
                free = np.zeros((p.nodes.free.shape[0], rows.shape[0]), dtype=np.uint32)  # racks become infeasible
            else:
                free = rng.integers(0, 200_000, size=(p.nodes.free.shape[0], rows.shape[0])).astype(np.uint32)
            engine.patch_rows(rows, free=free)
            p.nodes.free[:, rows] = free
        np.testing.assert_array_equal(engine.place(p.job_class).assign, O.place_c(p)[0])
    finally:
        engine.set_fused(True)


def _expect_reported_or_exact(engine, p, calls, word):
    """Place `calls` times: every call either raises JSP_EHIP naming `word`
    or returns the oracle's answer -- never a stale assign[] with success.
    Returns how many calls raised."""
    from jobset_amd.native import JSP_EHIP
    a = O.place_c(p)[0]
    errors = 0
    for _ in range(calls):
        try:
            got = engine.place(p.job_class)
        except JspError as ex:
            assert ex.code == JSP_EHIP and word in str(ex), str(ex)
            errors += 1
            continue
        np.testing.assert_array_equal(got.assign, a)
    return errors


def test_level_expand_timeout_is_reported(monkeypatch):
    """The one-launch level walk's expanders wait (bounded) for the walker's
    record count. One that gives up must fail the call, never leave a stale
    assign[]: with the hook wait_us=0 every expander that starts before the
    walker has published gives up at once."""
    monkeypatch.setenv("JSP_TEST_HOOKS", "wait_us=0")
    e = Engine(0)
    try:
        e.set_fused(False)
        p = synth.config4()
        e.load(p)
        errors = _expect_reported_or_exact(e, p, 6, "expanders")
        assert errors >= 1
        monkeypatch.delenv("JSP_TEST_HOOKS")
        e.load(p)  # hooks are read again at upload: the default wait
        assert _expect_reported_or_exact(e, p, 3, "expanders") == 0
    finally:
        e.close()


def test_pipe_walk_timeout_is_reported(monkeypatch):
    """The pipelined batch walk (many short leaf-level runs) waits for the
    earlier batches' progress words. A wait that gives up (hook pipe_spins=0:
    the first wait) fails the call on the launch path and the three-launch
    path alike; the default limit answers bit-exactly."""
    errors = 0
    for seed in range(4):
        base = synth.random_problem(seed, max_nodes=30_000, max_leaves=3000, max_jobs=3000)
        p = _one_level(base, base.topology.n_levels - 1, 4, False, seed)
        monkeypatch.setenv("JSP_TEST_HOOKS", "pipe_spins=0")
        e = Engine(0)
        try:
            e.set_service(False)
            for fused in (True, False):
                e.set_fused(fused)
                e.load(p)
                errors += _expect_reported_or_exact(e, p, 4, "pipelined")
            monkeypatch.delenv("JSP_TEST_HOOKS")
            e.load(p)
            assert _expect_reported_or_exact(e, p, 2, "pipelined") == 0
        finally:
            e.close()
    assert errors >= 1


def _device_runs(p):
    import torch
    from jobset_amd.snapshot import job_runs
    rc, rl = job_runs(p.job_class)
    return (torch.from_numpy(rc.astype(np.int32)).cuda(), torch.from_numpy(rl.astype(np.int32)).cuda(),
            int(rc.shape[0]))


@pytest.mark.parametrize("cfg", [3, 5])
def test_host_walk_device_paths(engine, cfg):
    """ABI v7 shapes 7 and 8: every shape the GPU level walker does not take
    walks on the host -- after the GPU's tally and feasibility (shape 7: the
    launch path with tallies requested, jsp_tally_device + jsp_assign_device,
    the sharded harness's halves), or over the split tiles' lines of a
    one-request launch (shape 8: the launch path without tallies and
    jsp_place_device on a caller's stream, device run list in and device
    assign[] out through pinned staging). Repeated calls reuse the staging;
    bit-exact against the oracle each time."""
    import torch
    p = synth.CONFIGS[cfg]()
    engine.load(p)
    a, cap, occ = O.place_c(p)
    got = engine.place(p.job_class, want_tally=True)
    assert_same(got, a, cap, occ)
    if cfg == 5:
        assert got.fused == 7
    # no tallies wanted, service off: the split tiles launched once (shape 8)
    engine.set_service(False)
    try:
        for _ in range(3):
            got = engine.place(p.job_class)
            # (below 256 jobs the GPU walk costs less: cfg3's 64 stay on the fused launch)
            assert got.fused == (8 if p.n_jobs >= 256 else 1)
            np.testing.assert_array_equal(got.assign, a)
    finally:
        engine.set_service(True)
    rct, rlt, nr = _device_runs(p)
    s = torch.cuda.current_stream().cuda_stream
    outs = [torch.full((p.n_jobs,), -7, dtype=torch.int32, device="cuda") for _ in range(3)]
    for i in range(9):  # back to back, three output buffers in turn
        engine.place_device(rct.data_ptr(), rlt.data_ptr(), nr, p.n_jobs, outs[i % 3].data_ptr(), s)
    engine.check()
    for o in outs:
        np.testing.assert_array_equal(o.cpu().numpy(), a)
    L = p.topology.n_leaves
    capd = torch.zeros((len(p.classes) + 1, L), dtype=torch.int32, device="cuda")
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    engine.tally_device(capd.data_ptr(), capd[-1].data_ptr(), L, s)
    engine.assign_device(capd.data_ptr(), capd[-1].data_ptr(), L, rct.data_ptr(), rlt.data_ptr(), nr, p.n_jobs,
                         out.data_ptr(), s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), a)
    np.testing.assert_array_equal(capd[:-1].cpu().numpy().astype(np.uint32), cap)
    # a patch after a device-path call is ordered after it (the walk's staging included)
    r = np.array([int(p.nodes.leaf_start[int(a[0])])], dtype=np.uint32) if a[0] >= 0 else np.array([0], np.uint32)
    t = np.array([p.nodes.taints[r[0]] | (1 << 31)], dtype=np.uint32)
    engine.place_device(rct.data_ptr(), rlt.data_ptr(), nr, p.n_jobs, out.data_ptr(), s)
    engine.patch_rows(r, taints=t)
    p.nodes.taints[r] = t
    engine.place_device(rct.data_ptr(), rlt.data_ptr(), nr, p.n_jobs, outs[0].data_ptr(), s)
    engine.check()
    np.testing.assert_array_equal(out.cpu().numpy(), a)
    np.testing.assert_array_equal(outs[0].cpu().numpy(), O.place_c(p)[0])


@pytest.mark.parametrize("seed", range(16))
def test_host_walk_random_multilevel(engine, seed):
    """Random 1-4 level snapshots with many short runs (interleaved classes
    at several levels): the host walk after the GPU feasibility, through the
    host API and the device path, equals the oracle and the GPU walkers
    (JSP_FUSED_OFF keeps the walk on the GPU)."""
    import torch
    p = synth.random_problem(9100 + seed, max_nodes=30_000, max_levels=4, max_leaves=2000, max_jobs=2500)
    engine.load(p)
    engine.set_service(False)  # the launch path: shape 8 (>= 256 jobs, split geometry), 7, 1 or 0
    try:
        got = engine.place(p.job_class)
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
    finally:
        engine.set_service(True)
    a, cap, occ = O.place_c(p)
    got = engine.place(p.job_class, want_tally=True)
    assert_same(got, a, cap, occ)
    rct, rlt, nr = _device_runs(p)
    out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    engine.place_device(rct.data_ptr(), rlt.data_ptr(), nr, p.n_jobs, out.data_ptr(), s)
    engine.check()
    np.testing.assert_array_equal(out[:p.n_jobs].cpu().numpy(), a)
    engine.set_fused(False)
    try:
        got0 = engine.place(p.job_class, want_tally=True)
        assert got0.fused == 0
        assert_same(got0, a, cap, occ)
    finally:
        engine.set_fused(True)


def test_walk_copy_timeout_is_reported(engine, monkeypatch):
    """The device paths' assign[] copy is queued before the host walks and
    waits (bounded) for the walk's release; with the hook wait_us=0 every
    such wait gives up: the device path reports JSP_EHIP (engine check or the
    next call), never a silent stale assign[]. Without the hook, bit-exact."""
    import torch
    from jobset_amd.native import JSP_EHIP
    p = synth.config5()
    monkeypatch.setenv("JSP_TEST_HOOKS", "wait_us=0")
    engine.load(p)
    rct, rlt, nr = _device_runs(p)
    out = torch.empty(p.n_jobs, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    with pytest.raises(JspError) as ei:
        for _ in range(5):
            engine.place_device(rct.data_ptr(), rlt.data_ptr(), nr, p.n_jobs, out.data_ptr(), s)
            engine.check()
    assert ei.value.code == JSP_EHIP and "copy timed out" in str(ei.value)
    monkeypatch.delenv("JSP_TEST_HOOKS")
    engine.check()
    engine.load(p)
    engine.place_device(rct.data_ptr(), rlt.data_ptr(), nr, p.n_jobs, out.data_ptr(), s)
    engine.check()
    np.testing.assert_array_equal(out.cpu().numpy(), O.place_c(p)[0])
