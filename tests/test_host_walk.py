"""CPU tests of the split service's host walk (jobset_amd/csrc/jsp_walk.cc)
and of the slot format the resident tiles hand it (jsp_internal.h SplitArgs).

The tiles' output is restated here in numpy from the oracle's tallies --
per (row block, class group) tile: the ballots of its leaves' `cap >= pods`
for leaf-level classes, the partial sums of min(cap, pods) per upper-level
domain (one record per domain, at the leaf that ends it inside the tile) for
upper classes, the occupancy ballots for group 0 -- and the host walk must
then reproduce oracle/cpu_ref.c's assign[] bit for bit. The GPU tests
(test_service_gpu.py) run the same walk on the kernel's real slots."""
import ctypes

import numpy as np
import pytest

from jobset_amd import native, synth
from oracle import oracle as O

SPLIT_RECS = 64                 # jsp_internal.h kSplitRecs
SEQ = 7                         # the request number the emulated tiles tag their answer with


def line_words(cpg, nw):
    """jsp_internal.h split_line_words: 2 entries per (class slot, wave), whole lines."""
    return (2 * (cpg + 1) * nw + 7) & ~7


def tile_words(cpg, nw):
    """jsp_internal.h split_tile_words: the lines, then nw x 64 records per class slot."""
    return line_words(cpg, nw) + nw * SPLIT_RECS * cpg


def rec_tag(seq):
    """jsp_internal.h split_rec_tag."""
    return seq % 16383 + 1


def put_word(slots, entry, word, seq=SEQ):
    """A ballot as the two tagged halves at a tile's line entry."""
    slots[entry] = (seq << 32) | (word & 0xFFFFFFFF)
    slots[entry + 1] = (seq << 32) | (word >> 32)
CHUNK_ROWS, MAX_BLK_LEAVES = 1024, 256


def blocks_of(leaf_start):
    """The engine's tally row blocks (jsp_snapshot_upload): whole leaves,
    <= 1020 rows (one 1024-row chunk minus alignment) and <= 256 leaves."""
    target = CHUNK_ROWS - 4
    L = len(leaf_start) - 1
    blk, rows, leaves = [0], 0, 0
    for l in range(L):
        r = int(leaf_start[l + 1] - leaf_start[l])
        if leaves > 0 and (rows + r > target or leaves == MAX_BLK_LEAVES):
            blk.append(l)
            rows, leaves = 0, 0
        rows += r
        leaves += 1
    if L > 0:
        blk.append(L)
    return blk[:-1], blk[1:]


def split_groups(C, nb):
    """jsp_engine.cc split_groups (no override)."""
    g = 1
    if C > 2:
        g = max(1, min(min(4, (C + 1) // 2), max(1, 128 // max(nb, 1))))
    while g > 1 and nb * g > 255:
        g -= 1
    return g


def ancestor(topo, leaf, level):
    """Domain at `level` of a leaf (first_leaf ranges)."""
    return int(np.searchsorted(topo.first_leaf[level], leaf, side="right") - 1)


def emulate_tiles(p, cap, occ):
    """The split service's tiles (place_split_service_kernel split_emit), in
    numpy: per tile, its tagged lines (ballots or record counts, occupancy)
    and its upper classes' tagged records."""
    topo = p.topology
    K = topo.n_levels
    C = len(p.classes)
    b0, b1 = blocks_of(p.nodes.leaf_start)
    nb = len(b0)
    groups = split_groups(C, nb)
    cpg = (C + groups - 1) // groups
    nw = min((max([1] + [b1[b] - b0[b] for b in range(nb)]) + 63) // 64, 4)  # jsp_walk split_waves
    nlw = line_words(cpg, nw)
    tw = tile_words(cpg, nw)
    slots = np.zeros(nb * groups * tw, dtype=np.uint64)
    for b in range(nb):
        l0, l1 = b0[b], b1[b]
        nl = l1 - l0
        for g in range(groups):
            t = b * groups + g
            base_t = t * tw
            for e in range(0, nlw, 2):  # every line entry is written, tagged
                put_word(slots, base_t + e, 0)
            for j in range(cpg):
                c = g * cpg + j
                if c >= C:
                    break
                jc = p.classes[c]
                capc = cap[c, l0:l1].astype(np.int64)
                if jc.level + 1 == K:
                    ok = capc >= jc.pods
                    for w in range(nw):
                        word = 0
                        for i in range(64):
                            li = 64 * w + i
                            if li < nl and ok[li]:
                                word |= 1 << i
                        put_word(slots, base_t + 2 * (j * nw + w), word)
                else:
                    fl = topo.first_leaf[jc.level]
                    incl = np.cumsum(np.minimum(capc, jc.pods))
                    recs = [[] for _ in range(4)]
                    for li in range(nl):
                        leaf = l0 + li
                        d = ancestor(topo, leaf, jc.level)
                        beg, end = int(fl[d]), int(fl[d + 1])
                        if li == nl - 1 or leaf + 1 == end:
                            first = max(beg, l0) - l0
                            part = int(incl[li] - (incl[first - 1] if first > 0 else 0))
                            recs[li // 64].append((rec_tag(SEQ) << 50) | (d << 30) | part)
                    for w in range(nw):
                        slots[base_t + 2 * (j * nw + w)] = (SEQ << 32) | len(recs[w])
                        rb = base_t + nlw + (j * nw + w) * SPLIT_RECS
                        for i, r in enumerate(recs[w]):
                            slots[rb + i] = r
            if g == 0:
                for w in range(nw):
                    word = 0
                    for i in range(64):
                        li = 64 * w + i
                        if li < nl and occ[l0 + li] != 0:
                            word |= 1 << i
                    put_word(slots, base_t + 2 * (cpg * nw + w), word)
    return slots, (b0, b1), groups, cpg


def host_walk(p, slots, blocks, groups, cpg):
    lib = native.lib()
    f = lib.jspi_walk_test
    f.restype = ctypes.c_int
    topo = p.topology
    K = topo.n_levels
    D = np.array(topo.n_domains + [0] * (4 - K), dtype=np.uint32)
    fls = [np.ascontiguousarray(topo.first_leaf[k], dtype=np.uint32) for k in range(K)]
    flp = (ctypes.c_void_p * 4)(*([a.ctypes.data for a in fls] + [None] * (4 - K)))
    lv = np.array([c.level for c in p.classes], dtype=np.uint32)
    pods = np.array([c.pods for c in p.classes], dtype=np.uint32)
    b0 = np.array(blocks[0], dtype=np.uint32)
    b1 = np.array(blocks[1], dtype=np.uint32)
    from jobset_amd.snapshot import job_runs
    rc, rl = job_runs(p.job_class)
    rc = np.ascontiguousarray(rc, dtype=np.uint32)
    rl = np.ascontiguousarray(rl, dtype=np.uint32)
    assign = np.full(max(p.n_jobs, 1), -7, dtype=np.int32)
    placed = f(ctypes.c_uint32(K), D.ctypes.data_as(ctypes.c_void_p), flp, ctypes.c_uint32(len(p.classes)),
               lv.ctypes.data_as(ctypes.c_void_p), pods.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(len(b0)),
               b0.ctypes.data_as(ctypes.c_void_p), b1.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(groups),
               ctypes.c_uint32(cpg), slots.ctypes.data_as(ctypes.c_void_p), rc.ctypes.data_as(ctypes.c_void_p),
               rl.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(rc.shape[0]),
               assign.ctypes.data_as(ctypes.c_void_p))
    return assign[:p.n_jobs], placed


def check(p):
    a, cap, occ = O.place_c(p)
    slots, blocks, groups, cpg = emulate_tiles(p, cap, occ)
    got, placed = host_walk(p, slots, blocks, groups, cpg)
    np.testing.assert_array_equal(got, a)
    assert placed == int((a >= 0).sum())


@pytest.mark.parametrize("cfg", [1, 2, 3, 5])
def test_host_walk_configs(cfg):
    check(synth.CONFIGS[cfg]())


@pytest.mark.parametrize("seed", range(40))
def test_host_walk_random(seed):
    """Ragged random snapshots: 1-3 nested levels, empty leaves, up to 16
    classes at any level, occupancy, interleaved and run-ordered jobs."""
    check(synth.random_problem(seed, max_nodes=3000, max_leaves=150))


@pytest.mark.parametrize("seed", range(8))
def test_host_walk_deep_levels(seed):
    """Four nested levels (taking a domain takes ancestors at every level above
    and descendant ranges below)."""
    check(synth.random_problem(5000 + seed, max_nodes=6000, max_levels=4, max_leaves=400, max_jobs=500))


def test_host_walk_many_blocks():
    """Several hundred leaves over many row blocks: records of one upper
    domain arrive from several tiles and are summed."""
    p = synth.random_problem(77, max_nodes=40_000, max_levels=2, max_leaves=600)
    check(p)
