"""Multi-rank path on CPU (gloo, world_size 2): sharding and the one result gather."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    from kelpie_amd import distributed as kd
    r, w, _ = kd.init_from_env(backend="gloo")
    items = list(range(11))
    mine = kd.shard(items, r, w)
    recs = np.array([[float(i), i * 2.0, 0, 0, 0] for i in mine]).reshape(-1, kd.RECORD)
    allr = kd.gather_records(recs, device="cpu")
    mx = kd.max_over_ranks(float(r + 1), device="cpu")
    kd.barrier()
    q.put((r, mine, allr[:, 0].tolist(), mx))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_shard_and_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    assert out[0][1] + out[1][1] == list(range(11))  # disjoint, complete shards
    for r, mine, gathered, mx in out:
        assert gathered == [float(i) for i in range(11)]  # rank order, padded counts trimmed
        assert mx == 2.0


def test_shard_single_rank():
    from kelpie_amd import distributed as kd
    assert kd.shard([1, 2, 3], 0, 1) == [1, 2, 3]
    recs = np.zeros((2, kd.RECORD))
    assert kd.gather_records(recs).shape == (2, kd.RECORD)
