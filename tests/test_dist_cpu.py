"""The multi-GPU path's collectives and sharding (az_amd.dist, used by bench.py) over gloo,
world size 2, on CPU: weight broadcast, MAX-elapsed / SUM-counter reduction, and the shard
seeds that make a game's record independent of the number of ranks."""
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
    import torch.distributed as dist
    from az_amd import dist as azdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = np.arange(1000, dtype=np.float32) * 0.5 if rank == 0 else None
        got = azdist.broadcast_weights(dist, blob, 1000)
        elapsed, cnt = azdist.reduce_counters(dist, 1.0 + rank, [10 + rank, 100 * (rank + 1)])
        q.put((rank, float(got.sum()), elapsed, cnt, azdist.shard(rank, 2048)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_reduce_shard():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = float((np.arange(1000, dtype=np.float32) * 0.5).sum())
    for rank, s, elapsed, cnt, sh in res:
        assert s == want                       # rank 0's weights everywhere
        assert elapsed == 2.0                  # slowest rank
        assert cnt == [21, 300]                # summed positions / evaluations
        assert sh["first_game"] == 2048 * rank and sh["noise_seed"] == 42 + 2048 * rank
    # rank 1's first game has the seed game 2048 would have on a single GPU (stride 1)
    from az_amd import dist as azdist
    one = azdist.shard(0, 4096)
    assert res[1][4]["noise_seed"] == one["noise_seed"] + 2048 * one["noise_seed_stride"]
