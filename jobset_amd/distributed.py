"""Multi-GPU placement: the node dimension sharded over ranks.

One process per GPU. Every rank holds a domain-aligned shard of the node rows
(whole level-0 domains, hence whole domains at every level:
snapshot.shard_problem) and the full, replicated domain hierarchy. A step:

  1. tally_kernel on the local rows -> per-(class, leaf) capacities and
     per-leaf occupancy for the local leaf columns (zero elsewhere);
  2. one SUM all-reduce of the [C+1, L] int32 tallies over RCCL (xGMI);
  3. every rank runs the identical deterministic feasibility + assignment
     kernels on the reduced tallies, so no second exchange is needed.

Integer sums make the result bit-exact for any world size (tests/ check it
against the unsharded oracle, on the GPU with shards on one device and on
CPU with gloo, world size 2).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from .snapshot import Problem, job_runs, shard_problem


def barrier(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_tallies(local, reduced, group=None) -> None:
    """reduced <- SUM over ranks of local ([C+1, L] int32; row C = occupancy).
    `local` is left untouched so the next step's tally can rewrite only the
    local columns."""
    import torch.distributed as dist
    reduced.copy_(local)
    dist.all_reduce(reduced, op=dist.ReduceOp.SUM, group=group)


class ShardedPlacement:
    """Device-resident placement of one Problem over `world` ranks."""

    def __init__(self, engine, p: Problem, rank: int, world: int, stream: Optional[int] = None, group=None):
        import torch
        self.engine, self.p, self.rank, self.world, self.group = engine, p, rank, world, group
        self.stream = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self.nodes = shard_problem(p, rank, world) if world > 1 else p.nodes
        engine.upload_topology(p.topology)
        engine.upload_snapshot(self.nodes)
        engine.upload_classes(p.classes)
        C, L = len(p.classes), p.topology.n_leaves
        self.C, self.L = C, L
        self.local = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
        self.reduced = torch.zeros((C + 1, L), dtype=torch.int32, device="cuda")
        rc, rl = job_runs(p.job_class)
        self.n_runs = int(rc.shape[0])
        self.rc = torch.from_numpy(rc.astype(np.int32)).cuda()
        self.rl = torch.from_numpy(rl.astype(np.int32)).cuda()
        self.out = torch.empty(max(p.n_jobs, 1), dtype=torch.int32, device="cuda")
        self._ev = []

    def step(self, time_allreduce: bool = False) -> None:
        import torch
        J = self.p.n_jobs
        if self.world == 1:
            self.engine.place_device(self.rc.data_ptr(), self.rl.data_ptr(), self.n_runs, J, self.out.data_ptr(),
                                     self.stream)
            return
        L = self.L
        self.engine.tally_device(self.local.data_ptr(), self.local[self.C].data_ptr(), L, self.stream)
        if time_allreduce:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            reduce_tallies(self.local, self.reduced, self.group)
            b.record()
            self._ev.append((a, b))
        else:
            reduce_tallies(self.local, self.reduced, self.group)
        self.engine.assign_device(self.reduced.data_ptr(), self.reduced[self.C].data_ptr(), L, self.rc.data_ptr(),
                                  self.rl.data_ptr(), self.n_runs, J, self.out.data_ptr(), self.stream)

    def assign(self) -> np.ndarray:
        return self.out[:self.p.n_jobs].cpu().numpy()

    def placed(self) -> int:
        return int((self.assign() >= 0).sum())

    def allreduce_us(self) -> Optional[float]:
        if self.world == 1:
            return None
        import torch
        if not self._ev:
            for _ in range(20):
                self.step(time_allreduce=True)
            torch.cuda.synchronize()
        us = [a.elapsed_time(b) * 1e3 for a, b in self._ev]
        self._ev = []
        return round(float(np.median(us)), 2)

    def shard_tally_bytes(self) -> int:
        n = self.nodes
        row = 8 * n.n_label_words + 4 + 4 * n.n_res + 4
        return n.n_nodes * row + 4 * (n.n_leaves + 1) + 4 * (self.C + 1) * n.n_leaves


def sharded_assign_reference(p: Problem, rank: int, world: int, tally_fn: Callable, assign_fn: Callable,
                             group=None) -> np.ndarray:
    """The same three-step protocol on CPU tensors (gloo): `tally_fn(shard)`
    returns the shard's ([C, n_leaves], [n_leaves]) tallies, `assign_fn(cap,
    occ)` the assignment from full tallies. Used by the world-size-2 gloo
    tests of the N > 1 path."""
    import torch
    C, L = len(p.classes), p.topology.n_leaves
    shard = shard_problem(p, rank, world)
    cap, occ = tally_fn(shard)
    local = torch.zeros((C + 1, L), dtype=torch.int32)
    b, e = shard.leaf_begin, shard.leaf_begin + shard.n_leaves
    local[:C, b:e] = torch.from_numpy(np.asarray(cap, dtype=np.int64).astype(np.int32))
    local[C, b:e] = torch.from_numpy(np.asarray(occ, dtype=np.int64).astype(np.int32))
    reduced = torch.empty_like(local)
    reduce_tallies(local, reduced, group)
    red = reduced.numpy().astype(np.uint32)
    return assign_fn(red[:C], red[C])
