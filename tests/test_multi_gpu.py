"""The device-set engine behind the C ABI (jsp_engine_create_multi,
SURVEY.md §8b/§8e): one handle, the node rows sharded by whole level-0
domains, per-shard tallies SUM-combined, the assignment on the first device.
On this one-GPU pool the shard ids repeat ({0, 0, 0}), so the shards are
combined by the on-device add instead of the RCCL all-reduce (which only a
set of distinct devices takes); the sharding, the per-shard tallies, the
combine and the replicated walk are the same code. Everything is bit-exact
against the unsharded oracle (integer sums)."""
import numpy as np
import pytest

from jobset_amd import synth
from jobset_amd.engine import Engine
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def multi():
    e = Engine(devices=[0, 0, 0])
    yield e
    e.close()


def test_device_set_shape(multi):
    assert multi.shards() == (3, 1)


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_device_set_configs(multi, cfg):
    p = synth.CONFIGS[cfg]()
    multi.load(p)
    a, cap, occ = O.place_c(p)
    for _ in range(2):  # repeated placements: the shard tallies rewrite their columns only
        got = multi.place(p.job_class, want_tally=True)
        assert got.fused == 6
        np.testing.assert_array_equal(got.assign, a)
        np.testing.assert_array_equal(got.cap, cap)
        np.testing.assert_array_equal(got.occ, occ)
        assert got.placed == int((a >= 0).sum())
    got = multi.place(p.job_class)  # without tallies
    np.testing.assert_array_equal(got.assign, a)


@pytest.mark.parametrize("seed", range(16))
def test_device_set_random(multi, seed):
    """Ragged random snapshots (1-3 levels, empty leaves, occupancy, up to 16
    classes): some shards may be empty."""
    p = synth.random_problem(seed, max_nodes=20_000, max_leaves=400)
    multi.load(p)
    got = multi.place(p.job_class, want_tally=True)
    a, cap, occ = O.place_c(p)
    np.testing.assert_array_equal(got.assign, a)
    np.testing.assert_array_equal(got.cap, cap)
    np.testing.assert_array_equal(got.occ, occ)


def test_device_set_patch(multi):
    """Row patches are routed to the shard that holds each row."""
    p = synth.config5()
    multi.load(p)
    rng = np.random.default_rng(9)
    for _ in range(5):
        rows = np.sort(rng.choice(p.nodes.n_nodes, size=300, replace=False)).astype(np.uint32)
        taints = (rng.integers(0, 2, size=300) << rng.integers(0, 4, size=300)).astype(np.uint32)
        free = rng.integers(0, 200_000, size=(p.nodes.free.shape[0], 300)).astype(np.uint32)
        multi.patch_rows(rows, taints=taints, free=free)
        p.nodes.taints[rows] = taints
        p.nodes.free[:, rows] = free
        np.testing.assert_array_equal(multi.place(p.job_class).assign, O.place_c(p)[0])


def test_device_set_resolve_and_audit(multi):
    """A5 / A9 batches on global rows: each row's shard answers."""
    p = synth.config5()
    multi.load(p)
    single = Engine(0)
    try:
        single.load(p)
        rows = np.array([0, 17, 16383, -1, 2048, 5000, 9000, 12345, 99999], dtype=np.int32)
        levels = np.array([1, 0, 1, 1, 0, 1, 0, 1, 1], dtype=np.uint32)
        got = multi.resolve_leader_domains(rows, levels)
        np.testing.assert_array_equal(got, single.resolve_leader_domains(rows, levels))
        off = np.array([0, 2, 2, 4, 5, 5, 7, 8, 9, 9], dtype=np.uint32)
        fd = np.array([got[0], got[0] + 1, 3, got[2], 4, got[5], got[5], got[6], 7], dtype=np.int32)
        np.testing.assert_array_equal(multi.audit_placements(rows, levels, off, fd),
                                      single.audit_placements(rows, levels, off, fd))
    finally:
        single.close()


def test_device_set_device_path_is_refused(multi):
    from jobset_amd.native import JSP_ESTATE, JspError
    p = synth.config2()
    multi.load(p)
    with pytest.raises(JspError) as ei:
        multi.tally_device(0, 0, p.topology.n_leaves, None)
    assert ei.value.code == JSP_ESTATE


@pytest.mark.parametrize("ids", [[0], [0, 0], [0, 0, 0, 0, 0]])
def test_device_set_sizes(ids):
    """1, 2 and 5 shards give the same placement (cfg4: 1M nodes)."""
    p = synth.config4()
    a = O.place_c(p)[0]
    e = Engine(devices=ids)
    try:
        e.load(p)
        np.testing.assert_array_equal(e.place(p.job_class).assign, a)
        assert e.shards() == (len(ids), 1)
    finally:
        e.close()


def test_device_set_rejects_bad_leaf_start():
    """leaf_start is validated whole before any shard slices the caller's
    columns: non-monotone, or an interior offset past N, is
    JSP_EINVAL -- never a wrapped slice or a read past a column."""
    import dataclasses

    from jobset_amd.native import JSP_EINVAL, JspError
    p = synth.config2()
    e = Engine(devices=[0, 0])
    try:
        e.upload_topology(p.topology)
        for bad in ("swap", "past_n"):
            ls = p.nodes.leaf_start.copy()
            if bad == "swap":
                ls[5], ls[6] = ls[6], ls[5]
            else:
                ls[500] = p.nodes.n_nodes + 1000
            with pytest.raises(JspError) as ei:
                e.upload_snapshot(dataclasses.replace(p.nodes, leaf_start=ls))
            assert ei.value.code == JSP_EINVAL
        e.load(p)  # a good snapshot still loads and places
        np.testing.assert_array_equal(e.place(p.job_class).assign, O.place_c(p)[0])
    finally:
        e.close()


def test_device_set_on_one_device_needs_no_rccl(monkeypatch):
    """Repeated ids combine on the device: with the RCCL loader pointed at a
    library that does not exist, the set still builds and places."""
    monkeypatch.setenv("JSP_RCCL_LIB", "/nonexistent/librccl_missing.so")
    p = synth.config5()
    e = Engine(devices=[0, 0])
    try:
        e.load(p)
        got = e.place(p.job_class)
        assert got.fused == 6 and e.shards() == (2, 1)
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
    finally:
        e.close()


def _gpus():
    from jobset_amd import native
    return native.device_count()


@pytest.mark.skipif(_gpus() < 2, reason="needs two GPUs (the RCCL path between distinct devices)")
def test_device_set_distinct_devices_without_rccl_fails_cleanly(monkeypatch):
    from jobset_amd.native import JSP_EHIP, JspError
    monkeypatch.setenv("JSP_RCCL_LIB", "/nonexistent/librccl_missing.so")
    with pytest.raises(JspError) as ei:
        Engine(devices=[0, 1])
    assert ei.value.code == JSP_EHIP and "RCCL" in str(ei.value)


@pytest.mark.skipif(_gpus() < 2, reason="needs two GPUs (the RCCL path between distinct devices)")
@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_device_set_distinct_devices(cfg):
    """The RCCL all-reduce between distinct devices (ncclCommInitAll in this
    process), shards on every visible GPU: bit-exact with the oracle."""
    n = min(_gpus(), 8)
    p = synth.CONFIGS[cfg]()
    a, cap, occ = O.place_c(p)
    e = Engine(devices=list(range(n)))
    try:
        assert e.shards() == (n, n)
        e.load(p)
        for _ in range(2):
            got = e.place(p.job_class, want_tally=True)
            assert got.fused == 6
            np.testing.assert_array_equal(got.assign, a)
            np.testing.assert_array_equal(got.cap, cap)
            np.testing.assert_array_equal(got.occ, occ)
    finally:
        e.close()


def test_device_set_keeps_the_callers_device():
    """A device-set engine walks its devices inside each call and hands the
    calling thread back its current device (a torch rank's NCCL barrier after
    the bench's device-set leg depends on it). On one GPU the ids are {0, 0};
    with more, the set is listed last device first."""
    import torch
    n = torch.cuda.device_count()
    ids = list(range(n))[::-1] if n > 1 else [0, 0]
    torch.cuda.set_device(0)
    p = synth.config4() if n > 1 else synth.config5()
    with Engine(devices=ids) as ds:
        assert torch.cuda.current_device() == 0
        ds.load(p)
        assert torch.cuda.current_device() == 0
        got = ds.place(p.job_class)
        assert torch.cuda.current_device() == 0
        np.testing.assert_array_equal(got.assign, O.place_c(p)[0])
    assert torch.cuda.current_device() == 0
