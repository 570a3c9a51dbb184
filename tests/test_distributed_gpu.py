"""The N > 1 sharded step itself on the GPU: two processes on cuda:0, each a
rank of a world of 2 (gloo collectives over the device tensors), run
ShardedPlacement.step -- jsp_tally_device on the rank's domain-aligned shard
-> SUM all-reduce of the [C+1, L] tallies -> jsp_assign_device on the reduced
tallies (jobset_amd/distributed.py). Every rank's assign[] and reduced
tallies must equal the unsharded oracle's, bit for bit (SURVEY.md §8e:
integer sums make the result independent of the shard count). cfg4 is the
1M-node scale-out snapshot, cfg5 the two-level (zone, rack) one."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, cfg, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jobset_amd import native, synth
        from jobset_amd.distributed import ShardedPlacement
        from jobset_amd.engine import Engine
        p = synth.CONFIGS[cfg]()
        eng = Engine(0)
        try:
            sp = ShardedPlacement(eng, p, rank, world)
            for _ in range(3):  # repeated steps: the local tallies are rewritten in place
                sp.step()
            torch.cuda.synchronize()
            eng.check()
            red = sp.reduced.cpu().numpy().astype(np.uint32)
            q.put((rank, sp.assign().tolist(), red[:sp.C].tolist(), red[sp.C].tolist(),
                   sp.nodes.leaf_begin, sp.nodes.n_leaves, native.LIB_PATH))
        finally:
            eng.close()
    except Exception as ex:  # noqa: BLE001 -- reported to the parent
        q.put((rank, repr(ex), None, None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [4, 5])
def test_world2_sharded_step_on_gpu(cfg):
    from jobset_amd import native, synth
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = {}
    for _ in procs:
        r = q.get(timeout=240)
        res[r[0]] = r
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = synth.CONFIGS[cfg]()
    a, cap, occ = O.place_c(p)
    shards = []
    for rank in (0, 1):
        _, got, rcap, rocc, lb, nl, lib_path = res[rank]
        assert isinstance(got, list), got
        assert os.path.samefile(lib_path, native.LIB_PATH)  # the in-tree HIP library ran
        np.testing.assert_array_equal(np.array(got, dtype=np.int32), a)
        np.testing.assert_array_equal(np.array(rcap, dtype=np.uint32), cap)
        np.testing.assert_array_equal(np.array(rocc, dtype=np.uint32), occ)
        shards.append((lb, nl))
    # the two shards are disjoint, domain-aligned and cover every leaf
    (b0, n0), (b1, n1) = sorted(shards)
    assert b0 == 0 and b0 + n0 == b1 and b1 + n1 == p.topology.n_leaves and n0 > 0 and n1 > 0
