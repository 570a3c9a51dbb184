"""The N > 1 path on CPU: world size 2 over gloo. Each rank tallies its
domain-aligned shard (oracle tally as the stand-in for tally_kernel, which
needs a GPU), the ranks SUM-all-reduce the [C+1, L] tallies exactly as
jobset_amd/distributed.py does, and every rank must produce the unsharded
assignment."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, cfg, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jobset_amd import synth
        from jobset_amd.distributed import sharded_assign_reference
        from oracle import oracle as O
        p = synth.CONFIGS[cfg]()
        a = sharded_assign_reference(
            p, rank, world,
            tally_fn=lambda shard: O.tally_nodes(p.topology.n_leaves, shard, p.classes),
            assign_fn=lambda cap, occ: O.assign_from_tallies(p, cap, occ))
        q.put((rank, a.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [3, 5])
def test_world2_gloo_sharded_placement(cfg):
    from jobset_amd import synth
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    want = O.place_c(synth.CONFIGS[cfg]())[0].tolist()
    assert res[0] == want and res[1] == want
