"""Multi-GPU plumbing of the self-play path: one process per GPU,
games sharded by contiguous global id ranges, no collective in the inner loop.

  shard(rank, games_per_rank)      -> global game ids and the seeds that make every game's
                                      record independent of the rank count
  Dist                              -> the engine's own RCCL communicator (az_dist_*, csrc/dist.hip):
                                      weights broadcast straight into the nets' device buffers,
                                      counter reductions, barriers -- the product path
  broadcast_weights / reduce_counters -> the same two collectives over a torch.distributed group
                                      (gloo on CPU tensors: the rank-logic tests without a GPU)
"""
import ctypes

import numpy as np

NOISE_SEED = 42     # ParallelMCTS setDeterministicMode seed (parallel_mcts.cpp:1268)


def shard(rank, games_per_rank, noise_seed=NOISE_SEED, eval_seed=0):
    """Game ids [rank*G, (rank+1)*G) of this rank and the per-slot seeds: game id g draws noise
    from mt19937(noise_seed + g) and the random evaluator from mt19937(eval_seed + g), so a game
    plays the same whatever the number of ranks."""
    g0 = rank * games_per_rank
    return {"first_game": g0, "games": games_per_rank, "noise_seed": noise_seed + g0, "noise_seed_stride": 1,
            "eval_seed": eval_seed + g0}


def shard_range(rank, world, total_games, noise_seed=NOISE_SEED, eval_seed=0):
    """Contiguous split of `total_games` global game ids over `world` ranks (the first
    total % world ranks take one more), with shard()'s seeds: BASELINE.json C3's "2048 games,
    sharded 1/2/4/8" is shard_range(rank, N, 2048)."""
    base, extra = divmod(int(total_games), int(world))
    g0 = rank * base + min(rank, extra)
    n = base + (1 if rank < extra else 0)
    return {"first_game": g0, "games": n, "noise_seed": noise_seed + g0, "noise_seed_stride": 1,
            "eval_seed": eval_seed + g0}


def broadcast_weights(dist, blob, n_params, device="cpu"):
    """Rank 0's fp32 blob (numpy, or None elsewhere) to every rank; returns the numpy blob."""
    import torch
    t = torch.empty(n_params, dtype=torch.float32, device=device)
    if dist.get_rank() == 0:
        t.copy_(torch.from_numpy(np.ascontiguousarray(blob, np.float32)))
    dist.broadcast(t, src=0)
    return t.cpu().numpy()


def reduce_counters(dist, elapsed, counters, device="cpu"):
    """MAX of the timed region over ranks (the slowest rank bounds the job) and SUM of the
    counters (positions, evaluations, ...)."""
    import torch
    x = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(v) for v in counters], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(x.item()), [int(v) for v in c.tolist()]


class Dist:
    """The engine's RCCL communicator over the ranks' engines (include/az_engine.h az_dist_*).
    Rank 0 makes the id (unique_id()); every rank passes the same id.  Collectives wait with a
    deadline (timeout_s): a dead rank makes the others raise AzError, not hang."""

    def __init__(self, engine, rank, world, uid, timeout_s=600.0):
        from ._lib import AZ_DIST_ID_BYTES, check, lib
        if len(uid) != AZ_DIST_ID_BYTES:
            raise ValueError(f"dist id must be {AZ_DIST_ID_BYTES} bytes")
        buf = (ctypes.c_ubyte * AZ_DIST_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        check(lib().az_dist_init(engine.h, int(rank), int(world), buf, int(timeout_s * 1000), ctypes.byref(h)))
        self.h, self.rank, self.world = h, int(rank), int(world)

    @staticmethod
    def unique_id():
        from ._lib import AZ_DIST_ID_BYTES, check, lib
        buf = (ctypes.c_ubyte * AZ_DIST_ID_BYTES)()
        check(lib().az_dist_unique_id(buf))
        return bytes(buf)

    def barrier(self):
        from ._lib import check, lib
        check(lib().az_dist_barrier(self.h))

    def allreduce(self, values, op="sum"):
        """SUM ("sum") or MAX ("max") over the ranks of a list of numbers (float64)."""
        from ._lib import AZ_DIST_MAX, AZ_DIST_SUM, check, lib
        x = np.ascontiguousarray(values, np.float64).reshape(-1)
        out = np.empty_like(x)
        dp = ctypes.POINTER(ctypes.c_double)
        check(lib().az_counters_allreduce(self.h, x.ctypes.data_as(dp), out.ctypes.data_as(dp), x.size,
                                          AZ_DIST_SUM if op == "sum" else AZ_DIST_MAX))
        return out.tolist()

    def broadcast_weights(self, net, root=0):
        """Rank root's weights into `net` on every rank, device to device (az_net_broadcast_weights)."""
        from ._lib import check, lib
        check(lib().az_net_broadcast_weights(self.h, net.h, int(root)))

    def close(self):
        from ._lib import lib
        if self.h:
            lib().az_dist_destroy(self.h)
            self.h = None
