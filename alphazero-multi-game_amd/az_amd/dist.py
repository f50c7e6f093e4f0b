"""Multi-GPU plumbing of the self-play path: one process per GPU,
games sharded by contiguous global id ranges, no collective in the inner loop.  RCCL (backend
"nccl") on the GPU box; the same functions run over gloo on CPU tensors in the tests.

  shard(rank, games_per_rank)      -> global game ids and the seeds that make every game's
                                      record independent of the rank count
  broadcast_weights(...)            -> rank 0's weight blob on every rank (one broadcast)
  reduce_counters(...)              -> (max elapsed, summed counters) for the bench line
"""
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
