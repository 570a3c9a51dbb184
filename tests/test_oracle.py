"""CPU tests of the parity oracle (test infrastructure): the C restatement
against the independent pure-Python restatement on ragged random snapshots,
the invariants of SURVEY.md §8c on every config, the committed fixtures, and
the tally/assign split the multi-GPU path uses."""
import hashlib
import json
import os

import numpy as np
import pytest

from jobset_amd import synth
from jobset_amd.snapshot import shard_problem
from oracle import oracle as O

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "placements.json")))


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("seed", range(60))
def test_c_matches_pure_python(seed):
    p = synth.random_problem(seed, max_nodes=600)
    a, cap, occ = O.place_c(p)
    b, cap2, occ2 = O.place_py(p)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(cap, cap2)
    np.testing.assert_array_equal(occ, occ2)
    O.check_invariants(p, a, cap, occ)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_fixtures(cfg):
    p = synth.CONFIGS[cfg]()
    a, cap, occ = O.place_c(p)
    f = FIX[str(cfg)]
    assert (p.nodes.n_nodes, p.topology.n_leaves, p.n_jobs) == (f["nodes"], f["leaves"], f["jobs"])
    assert digest(a.astype(np.int32)) == f["assign_sha256"]
    assert digest(cap.astype(np.uint32)) == f["cap_sha256"]
    assert digest(occ.astype(np.uint32)) == f["occ_sha256"]
    if "assign" in f:
        assert a.tolist() == f["assign"]
    if cfg != 4:
        O.check_invariants(p, a, cap, occ)


def test_config_shapes():
    """SURVEY.md §8d restatements of BASELINE.json configs."""
    p1 = synth.config1()
    assert (p1.nodes.n_nodes, p1.topology.n_leaves, p1.n_jobs, p1.classes[0].pods) == (12, 4, 3, 3)
    assert p1.job_names == ["default/exclusive-placement-workers-0", "default/exclusive-placement-workers-1",
                            "default/exclusive-placement-workers-2"]
    p2 = synth.config2()
    assert (p2.nodes.n_nodes, p2.topology.n_leaves, p2.n_jobs, p2.classes[0].pods) == (15000, 1000, 990, 15)
    assert int((p2.nodes.taints != 0).sum()) == 10
    p3 = synth.config3()
    assert (p3.nodes.n_nodes, p3.n_jobs, p3.classes[0].pods, len(p3.classes)) == (40960, 64, 4096, 2)
    p5 = synth.config5()
    assert p5.topology.n_domains == [8, 1024] and p5.n_jobs == 500
    assert int(sum(p5.classes[c].level == 0 for c in p5.job_class)) == 4


def test_generator_is_deterministic():
    a, b = synth.config2(trial=3), synth.config2(trial=3)
    np.testing.assert_array_equal(a.nodes.labels, b.nodes.labels)
    np.testing.assert_array_equal(a.nodes.taints, b.nodes.taints)
    assert not np.array_equal(a.nodes.taints, synth.config2(trial=4).nodes.taints)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_tallies_sum_to_full(world):
    """Domain-aligned shards: concatenating per-shard tallies gives the full
    tally, and assigning from it gives the unsharded assignment."""
    p = synth.config5()
    a, cap, occ = O.place_c(p)
    cap_s = np.zeros_like(cap)
    occ_s = np.zeros_like(occ)
    for r in range(world):
        sh = shard_problem(p, r, world)
        c, o = O.tally_nodes(p.topology.n_leaves, sh, p.classes)
        cap_s[:, sh.leaf_begin:sh.leaf_begin + sh.n_leaves] += c
        occ_s[sh.leaf_begin:sh.leaf_begin + sh.n_leaves] += o
    np.testing.assert_array_equal(cap_s, cap)
    np.testing.assert_array_equal(occ_s, occ)
    np.testing.assert_array_equal(O.assign_from_tallies(p, cap_s, occ_s), a)


def test_invariant_checker_catches_violations():
    p = synth.config3()
    a, cap, occ = O.place_c(p)
    bad = a.copy()
    bad[1] = bad[0]
    with pytest.raises(AssertionError):
        O.check_invariants(p, bad, cap, occ)
    bad = a.copy()
    bad[-1] = -1
    with pytest.raises(AssertionError):
        O.check_invariants(p, bad, cap, occ)


@pytest.mark.parametrize("threads", [1, 2, 3])
def test_fast_cpu_evaluator_bit_exact(threads):
    """oracle/cpu_fast.c (the bench's CPU baseline) equals cpu_ref.c on ragged
    random snapshots (1-4 levels, empty leaves, W/R 1..4) and configs 1, 2, 3, 5,
    at any thread count."""
    fc = O.FastCPU(threads)
    try:
        problems = [synth.random_problem(s, max_nodes=3000) for s in range(25)]
        problems += [synth.random_problem(5000 + s, max_nodes=20_000, max_levels=4, max_leaves=1500, max_jobs=1200)
                     for s in range(3)]
        problems += [synth.CONFIGS[c]() for c in (1, 2, 3, 5)]
        for p in problems:
            fc.prepare(p)
            for _ in range(2):  # the pool and buffers are reused across runs
                a, cap, occ, placed = fc.run(want_tally=True)
                a2, cap2, occ2 = O.place_c(p)
                np.testing.assert_array_equal(cap, cap2)
                np.testing.assert_array_equal(occ, occ2)
                np.testing.assert_array_equal(a, a2)
                assert placed == int((a2 >= 0).sum())
    finally:
        fc.close()
