"""Deterministic synthetic cluster snapshots for BASELINE.json configs 1-5.

The reference has no multi-node fixture, fake scheduler or node simulator
(SURVEY.md §4 "How multi-node is tested without a cluster: it isn't"), so the
engine brings its own seeded generator. Random draws come from
a counter-based SplitMix64: draw(seed, stream, i) = mix64(seed*G + stream*H +
(i+1)*G), so every column is generated vectorised and identically on any host.

Config seeds follow SURVEY.md §8d: seed = config_index * 1000 + trial.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from .snapshot import JobClass, Nodes, Problem, Topology, default_domain_value

_G = 0x9E3779B97F4A7C15
_H = 0xD1B54A32D192ED03
_M64 = (1 << 64) - 1

RACK_KEY = "topology.kubernetes.io/rack"
ZONE_KEY = "topology.kubernetes.io/zone"
NODEPOOL_KEY = "cloud.google.com/gke-nodepool"   # examples/simple/exclusive-placement.yaml:6

# resources (R = 3): cpu millicores, memory MiB, GPUs
RES_NAMES = ("cpu", "memory", "amd.com/gpu")
NODE_CPU_M = 192_000
NODE_MEM_MIB = 1_536_000
NODE_GPU = 8


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def draws(seed: int, stream: int, n: int) -> np.ndarray:
    base = (seed * _G + stream * _H) & _M64
    i = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix64(np.uint64(base) + i * np.uint64(_G))


def uniform_int(seed: int, stream: int, n: int, lo: int, hi: int) -> np.ndarray:
    """Integers uniform in [lo, hi] (inclusive), int64."""
    u = (draws(seed, stream, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return lo + np.floor(u * (hi - lo + 1)).astype(np.int64)


def bernoulli(seed: int, stream: int, n: int, p: float) -> np.ndarray:
    u = (draws(seed, stream, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return u < p


def permutation(seed: int, stream: int, n: int) -> np.ndarray:
    return np.argsort(draws(seed, stream, n), kind="stable")


def random_label_bits(seed: int, stream: int, n: int, lo_bit: int, hi_bit: int) -> np.ndarray:
    """1-3 random bits in [lo_bit, hi_bit] per row (SURVEY.md §8d value distribution)."""
    cnt = uniform_int(seed, stream, n, 1, 3)
    out = np.zeros(n, dtype=np.uint64)
    for t in range(3):
        b = uniform_int(seed, stream + 1 + t, n, lo_bit, hi_bit).astype(np.uint64)
        out |= np.where(cnt > t, np.uint64(1) << b, np.uint64(0))
    return out


def _flat_topology(key: str, leaf_sizes: np.ndarray) -> Tuple[Topology, np.ndarray]:
    L = int(leaf_sizes.shape[0])
    topo = Topology(level_keys=[key], n_domains=[L],
                    first_leaf=[np.arange(L + 1, dtype=np.uint32)])
    leaf_start = np.zeros(L + 1, dtype=np.uint32)
    np.cumsum(leaf_sizes, out=leaf_start[1:])
    return topo, leaf_start


def _full_free(N: int) -> np.ndarray:
    free = np.empty((3, N), dtype=np.uint32)
    free[0] = NODE_CPU_M
    free[1] = NODE_MEM_MIB
    free[2] = NODE_GPU
    return free


def _job_names(ns: str, jobset: str, rjobs: List[Tuple[str, int]]) -> List[str]:
    # GenJobName (pkg/util/placement/placement.go:14-16), global order
    # (globalJobIndex, pkg/controllers/jobset_controller.go:1056-1065).
    return [f"{ns}/{jobset}-{rj}-{i}" for rj, n in rjobs for i in range(n)]


# ---------------------------------------------------------------- config 1
def config1(trial: int = 0) -> Problem:
    """examples/simple/exclusive-placement.yaml: JobSet "exclusive-placement",
    1 replicatedJob "workers" x 3 replicas, parallelism 3, topology key
    cloud.google.com/gke-nodepool; 4 node pools x 3 nodes."""
    seed = 1 * 1000 + trial
    topo, leaf_start = _flat_topology(NODEPOOL_KEY, np.full(4, 3, dtype=np.int64))
    topo.domain_values = [[f"pool-{i}" for i in range(4)]]
    N = 12
    labels = np.zeros((1, N), dtype=np.uint64)
    labels[0] = random_label_bits(seed, 10, N, 8, 63) | np.uint64(1)  # bit 0: kubernetes.io/os=linux
    nodes = Nodes(leaf_start=leaf_start, labels=labels, taints=np.zeros(N, dtype=np.uint32),
                  free=_full_free(N), excl=np.full(N, -1, dtype=np.int32),
                  node_names=[f"gke-pool-{i // 3}-node-{i % 3}" for i in range(N)])
    # busybox "sleep" containers request nothing.
    cls = JobClass(req_labels=(1,), level=0, pods=3, req_res=(0, 0, 0))
    return Problem(topology=topo, nodes=nodes, classes=[cls],
                   job_class=np.zeros(3, dtype=np.uint32), name="cfg1-exclusive-placement-yaml",
                   job_names=_job_names("default", "exclusive-placement", [("workers", 3)]))


# ---------------------------------------------------------------- config 2
def config2(trial: int = 0) -> Problem:
    """15k nodes / 1k racks, full-JobSet failure recovery (post-delete
    snapshot). 990 jobs x 15 pods, one pod per node (8 GPUs each); 10 racks
    carry one node tainted node.kubernetes.io/unreachable:NoSchedule."""
    seed = 2 * 1000 + trial
    D, per = 1000, 15
    N = D * per
    topo, leaf_start = _flat_topology(RACK_KEY, np.full(D, per, dtype=np.int64))
    labels = np.zeros((1, N), dtype=np.uint64)
    labels[0] = random_label_bits(seed, 10, N, 8, 63) | np.uint64(1)  # bit 0: instance-type=mi355x
    taints = np.zeros(N, dtype=np.uint32)
    bad_racks = permutation(seed, 20, D)[:10]
    bad_slot = uniform_int(seed, 21, 10, 0, per - 1)
    taints[bad_racks * per + bad_slot] = 1                            # bit 0: unreachable:NoSchedule
    nodes = Nodes(leaf_start=leaf_start, labels=labels, taints=taints, free=_full_free(N),
                  excl=np.full(N, -1, dtype=np.int32))
    cls = JobClass(req_labels=(1,), level=0, pods=per, req_res=(96_000, 1_024_000, 8))
    J = 990
    return Problem(topology=topo, nodes=nodes, classes=[cls], job_class=np.zeros(J, dtype=np.uint32),
                   name="cfg2-15k-nodes-1k-racks-recovery",
                   job_names=_job_names("default", "llm-train", [("workers", J)]),
                   meta={"bad_racks": np.sort(bad_racks)})


# ---------------------------------------------------------------- config 3
def config3(trial: int = 0) -> Problem:
    """64 replicated jobs x 4096 pods, 8 pods/node (1 GPU each), 80 racks x 512
    nodes; 16 racks tainted dedicated=x:NoSchedule, tolerated by the 32 jobs of
    the first replicatedJob only (C = 2); 2 racks have one node with 1 GPU busy."""
    seed = 3 * 1000 + trial
    D, per = 80, 512
    N = D * per
    topo, leaf_start = _flat_topology(RACK_KEY, np.full(D, per, dtype=np.int64))
    labels = np.zeros((1, N), dtype=np.uint64)
    labels[0] = random_label_bits(seed, 10, N, 8, 63) | np.uint64(1)
    taints = np.zeros(N, dtype=np.uint32)
    perm = permutation(seed, 20, D)
    tainted = perm[:16]
    for r in tainted:
        taints[r * per:(r + 1) * per] |= 2                               # bit 1: dedicated=x:NoSchedule
    free = _full_free(N)
    short = perm[16:18]
    free[2, short * per + uniform_int(seed, 22, 2, 0, per - 1)] = NODE_GPU - 1
    nodes = Nodes(leaf_start=leaf_start, labels=labels, taints=taints, free=free,
                  excl=np.full(N, -1, dtype=np.int32))
    pod = (16_000, 128_000, 1)
    c0 = JobClass(req_labels=(1,), tolerated_taints=2, level=0, pods=4096, req_res=pod)
    c1 = JobClass(req_labels=(1,), tolerated_taints=0, level=0, pods=4096, req_res=pod)
    jc = np.array([0] * 32 + [1] * 32, dtype=np.uint32)
    return Problem(topology=topo, nodes=nodes, classes=[c0, c1], job_class=jc,
                   name="cfg3-64x4k-rack-exclusive-taints",
                   job_names=_job_names("default", "pretrain", [("tolerant", 32), ("workers", 32)]),
                   meta={"tainted": np.sort(tainted), "short": np.sort(short)})


# ---------------------------------------------------------------- config 4
def config4(trial: int = 0, n_nodes: int = 1 << 20, n_domains: int = 50_000,
            jobs: Tuple[int, int, int, int] = (16_000, 12_000, 4_000, 8_000)) -> Problem:
    """1M nodes / 50k domains (20-21 nodes each), 40,000 jobs x 16 pods, C = 4
    label/taint classes. 5 % of nodes carry random taints, free resources are
    uniform in [0, capacity], labels are 1-3 random bits plus rack-uniform
    accelerator / reservation labels, 2 % of racks are covered by other
    tenants' exclusive jobs."""
    seed = 4 * 1000 + trial
    D, N = n_domains, n_nodes
    base, extra = divmod(N, D)
    sizes = np.full(D, base, dtype=np.int64)
    sizes[:extra] += 1
    topo, leaf_start = _flat_topology(RACK_KEY, sizes)
    rack_of = np.repeat(np.arange(D), sizes)
    accel = np.where(bernoulli(seed, 30, D, 0.9), np.uint64(1), np.uint64(2))  # bit0 mi355x, bit1 mi300x
    reserved = np.where(bernoulli(seed, 31, D, 0.05), np.uint64(4), np.uint64(0))  # bit2 pool=reserved
    labels = np.zeros((1, N), dtype=np.uint64)
    labels[0] = random_label_bits(seed, 10, N, 8, 63) | accel[rack_of] | reserved[rack_of]
    tmask = uniform_int(seed, 40, N, 1, 255).astype(np.uint32)
    taints = np.where(bernoulli(seed, 41, N, 0.05), tmask, 0).astype(np.uint32)
    free = np.empty((3, N), dtype=np.uint32)
    free[0] = uniform_int(seed, 50, N, 0, NODE_CPU_M)
    free[1] = uniform_int(seed, 51, N, 0, NODE_MEM_MIB)
    free[2] = uniform_int(seed, 52, N, 0, NODE_GPU)
    owned = bernoulli(seed, 60, D, 0.02)
    owner = np.where(owned, 1_000_000 + np.arange(D), -1).astype(np.int32)
    nodes = Nodes(leaf_start=leaf_start, labels=labels, taints=taints, free=free, excl=owner[rack_of])
    classes = [
        JobClass(req_labels=(1,), level=0, pods=16, req_res=(24_000, 200_000, 2)),
        JobClass(req_labels=(1,), forbid_labels=(4,), tolerated_taints=0x0F, level=0, pods=16,
                 req_res=(8_000, 64_000, 4)),
        JobClass(req_labels=(2,), level=0, pods=16, req_res=(16_000, 128_000, 1)),
        JobClass(tolerated_taints=0xFF, level=0, pods=16, req_res=(8_000, 32_000, 0)),
    ]
    jc = np.concatenate([np.full(n, c, dtype=np.uint32) for c, n in enumerate(jobs)])
    return Problem(topology=topo, nodes=nodes, classes=classes, job_class=jc,
                   name="cfg4-1M-nodes-50k-domains")


# ---------------------------------------------------------------- config 5
def config5(trial: int = 0) -> Problem:
    """Kueue-style burst: 8 zones x 128 racks x 16 nodes (K = 2). 500 JobSets
    arrive in one batch, ordered by (creationTimestamp, namespace, name): 496
    rack-exclusive (1 job x 16 pods) and 4 zone-exclusive (1 job x 2048 pods),
    one pod per node, C = 8 classes from tenant tolerations/selectors."""
    seed = 5 * 1000 + trial
    Z, RZ, per = 8, 128, 16
    D = Z * RZ
    N = D * per
    fl0 = (np.arange(Z + 1) * RZ).astype(np.uint32)
    topo = Topology(level_keys=[ZONE_KEY, RACK_KEY], n_domains=[Z, D],
                    first_leaf=[fl0, np.arange(D + 1, dtype=np.uint32)])
    topo.domain_values = [[f"zone-{z}" for z in range(Z)],
                          [f"zone-{r // RZ}-rack-{r % RZ:03d}" for r in range(D)]]
    leaf_start = (np.arange(D + 1) * per).astype(np.uint32)
    labels = np.zeros((1, N), dtype=np.uint64)
    labels[0] = random_label_bits(seed, 10, N, 8, 63) | np.uint64(1)
    # 3 % of nodes carry one of 4 taints
    taints = np.where(bernoulli(seed, 40, N, 0.03),
                      np.uint32(1) << uniform_int(seed, 41, N, 0, 3).astype(np.uint32), 0).astype(np.uint32)
    free = _full_free(N)
    busy = bernoulli(seed, 50, N, 0.004)
    free[2, busy] = uniform_int(seed, 51, int(busy.sum()), 0, NODE_GPU - 1).astype(np.uint32)
    excl = np.full(N, -1, dtype=np.int32)
    for i, r in enumerate(permutation(seed, 60, D)[:2]):        # racks held by earlier tenants
        excl[r * per:(r + 1) * per] = 2_000_000 + i
    nodes = Nodes(leaf_start=leaf_start, labels=labels, taints=taints, free=free, excl=excl)
    full = (96_000, 1_024_000, 8)
    classes = [JobClass(req_labels=(1,), tolerated_taints=tol, level=1, pods=per, req_res=full)
               for tol in (0x0, 0x1, 0x3, 0x7, 0xF, 0x2)]
    classes += [JobClass(req_labels=(1,), tolerated_taints=0xF, level=0, pods=RZ * per, req_res=full),
                JobClass(req_labels=(1,), tolerated_taints=0x3, level=0, pods=RZ * per, req_res=full)]
    # JobSet order: creation timestamps are seeded; zone JobSets land at 4 positions.
    order = permutation(seed, 70, 500)
    zone_js = set(order[:4].tolist())
    rack_cls = uniform_int(seed, 71, 500, 0, 5)
    jc, names = [], []
    for i in range(500):
        if i in zone_js:
            jc.append(6 + (len([z for z in zone_js if z < i]) % 2))
            names.append(f"tenant-{i:03d}/zone-train-{i:03d}-workers-0")
        else:
            jc.append(int(rack_cls[i]))
            names.append(f"tenant-{i:03d}/rack-train-{i:03d}-workers-0")
    return Problem(topology=topo, nodes=nodes, classes=classes, job_class=np.array(jc, dtype=np.uint32),
                   name="cfg5-kueue-burst-zone-rack", job_names=names)


CONFIGS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5}


# ---------------------------------------------------------------- property-test cases
def random_problem(seed: int, max_nodes: int = 4000, max_levels: int = 3,
                   max_classes: int = 16, max_jobs: Optional[int] = None, max_leaves: int = 200) -> Problem:
    """Ragged random snapshot for parity sweeps: 1-3 nested levels, empty and
    1-node leaves, W and R in 1..4, up to 16 classes, random occupancy and job
    orders (long same-class runs and fully interleaved ones)."""
    s = 9 * 1000 + seed
    u = lambda stream, lo, hi: int(uniform_int(s, stream, 1, lo, hi)[0])  # noqa: E731
    K = u(1, 1, max_levels)
    W = u(2, 1, 4)
    R = u(3, 1, 4)
    # leaves and their sizes (0..max per leaf; ~10 % empty)
    L = u(4, 1, max_leaves)
    mx = max(1, min(64, max_nodes // L))
    sizes = uniform_int(s, 5, L, 0, mx)
    sizes = np.where(bernoulli(s, 6, L, 0.1), 0, sizes)
    if sizes.sum() == 0:
        sizes[0] = 1
    N = int(sizes.sum())
    # nested levels: level K-1 = leaves; each coarser level groups contiguous runs
    first_leaf: List[np.ndarray] = [None] * K  # type: ignore
    first_leaf[K - 1] = np.arange(L + 1, dtype=np.uint32)
    for k in range(K - 2, -1, -1):
        fine = first_leaf[k + 1]
        Dn = fine.shape[0] - 1
        keep = bernoulli(s, 7 + k, Dn - 1, 0.3)
        b = [0] + [i + 1 for i in range(Dn - 1) if keep[i]] + [Dn]
        first_leaf[k] = fine[np.array(b)].astype(np.uint32)
    topo = Topology(level_keys=[f"example.com/level-{k}" for k in range(K)],
                    n_domains=[int(f.shape[0] - 1) for f in first_leaf], first_leaf=first_leaf)
    leaf_start = np.zeros(L + 1, dtype=np.uint32)
    np.cumsum(sizes, out=leaf_start[1:])
    labels = np.zeros((W, N), dtype=np.uint64)
    for w in range(W):
        labels[w] = draws(s, 20 + w, N) & draws(s, 30 + w, N) | draws(s, 40 + w, N)  # ~62 % density
    taints = np.where(bernoulli(s, 50, N, 0.15), uniform_int(s, 51, N, 0, 0xFFFF), 0).astype(np.uint32)
    caps = [uniform_int(s, 60 + r, 1, 1, 5000)[0] for r in range(R)]
    free = np.stack([uniform_int(s, 70 + r, N, 0, int(caps[r])) for r in range(R)]).astype(np.uint32)
    # occupancy: whole domains at random levels covered by foreign exclusive jobs
    excl = np.full(N, -1, dtype=np.int32)
    node_leaf = np.repeat(np.arange(L), sizes)
    n_own = u(80, 0, 4)
    for i in range(n_own):
        k = u(81 + 2 * i, 0, K - 1)
        d = u(82 + 2 * i, 0, topo.n_domains[k] - 1)
        a, bnd = int(first_leaf[k][d]), int(first_leaf[k][d + 1])
        excl[(node_leaf >= a) & (node_leaf < bnd)] = 500 + i
    nodes = Nodes(leaf_start=leaf_start, labels=labels, taints=taints, free=free, excl=excl)
    C = u(90, 1, max_classes)
    classes = []
    for c in range(C):
        cs = 100 + 20 * c
        req = [int(draws(s, cs + w, 1)[0] & draws(s, cs + 4 + w, 1)[0] & draws(s, cs + 8 + w, 1)[0])
               if bernoulli(s, cs + 12 + w, 1, 0.5)[0] else 0 for w in range(W)]
        fb = [int(draws(s, cs + 13 + w, 1)[0] & draws(s, cs + 17 + w, 1)[0] & draws(s, cs + 1, 1)[0] &
                  draws(s, cs + 2, 1)[0]) & ~req[w] & ((1 << 64) - 1) if bernoulli(s, cs + 9, 1, 0.3)[0] else 0
              for w in range(W)]
        rr = [int(uniform_int(s, cs + 10 + r, 1, 0, max(1, caps[r] // 3))[0]) if bernoulli(s, cs + 14, 1, 0.8)[0]
              else 0 for r in range(R)]
        classes.append(JobClass(req_labels=tuple(req), forbid_labels=tuple(fb),
                                tolerated_taints=int(uniform_int(s, cs + 15, 1, 0, 0xFFFF)[0]),
                                level=u(cs + 16, 0, K - 1), pods=u(cs + 18, 1, 3 * mx),
                                req_res=tuple(rr)))
    J = u(95, 0, max_jobs if max_jobs is not None else 2 * L + 5)
    if bernoulli(s, 96, 1, 0.5)[0]:
        jc = uniform_int(s, 97, J, 0, C - 1)                   # interleaved classes
    else:
        jc = np.sort(uniform_int(s, 97, J, 0, C - 1))          # replicated-job runs
    return Problem(topology=topo, nodes=nodes, classes=classes, job_class=jc.astype(np.uint32),
                   name=f"random-{seed}")


def domain_values_for(topo: Topology) -> List[List[str]]:
    if topo.domain_values is not None:
        return topo.domain_values
    return [[default_domain_value(k, d) for d in range(n)] for k, n in zip(topo.level_keys, topo.n_domains)]
